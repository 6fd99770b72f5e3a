timeout -k 10 60 ./tools/fp8_probe || exit 1
echo "== check"; timeout -k 10 100 python3 tools/gemv_bench.py --iters 30 --modes exact 2>&1 | grep -v amdgpu.ids || exit 1
echo "== check64"; VSIM_CHAIN_ROWS=64 timeout -k 10 100 python3 tools/gemv_bench.py --iters 30 --modes exact 2>&1 | grep -v amdgpu.ids || exit 1
echo "== tests"; timeout -k 10 600 python3 -m pytest tests -x -q -m gpu 2>&1 | tail -5
