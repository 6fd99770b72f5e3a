echo "== tests"; timeout -k 10 600 python3 -m pytest tests -x -q -m gpu 2>&1 | tail -3 || exit 1
echo "== gemv"; timeout -k 10 100 python3 tools/gemv_bench.py --iters 30 --modes exact --no-check 2>&1 | grep -v amdgpu.ids || exit 1
echo "== split"; timeout -k 10 300 python3 bench.py --steps 64 --no-cpu-baseline --no-fast --no-profile 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
echo "== single"; VSIM_SPLIT=0 timeout -k 10 300 python3 bench.py --steps 64 --no-cpu-baseline --no-fast --no-profile 2>&1 | grep -v amdgpu.ids | tail -1
