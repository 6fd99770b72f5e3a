echo "== tests"; timeout -k 10 600 python3 -m pytest tests -x -q -m gpu 2>&1 | tail -3 || exit 1
echo "== bench tail"; timeout -k 10 300 python3 bench.py --steps 64 --no-cpu-baseline --no-fast --no-profile 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-220 || exit 1
echo "== bench no tail"; VSIM_TAIL=0 timeout -k 10 300 python3 bench.py --steps 64 --no-cpu-baseline --no-fast --no-profile 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-220
