VSIM_LN_DBG=1 timeout -k 10 200 python3 tools/ln_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== tests"; timeout -k 10 600 python3 -m pytest tests -x -q -m gpu 2>&1 | tail -3 || exit 1
echo "== bench"; timeout -k 10 300 python3 bench.py --steps 64 --no-cpu-baseline --no-fast --no-profile 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200
