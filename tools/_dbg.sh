timeout -k 10 100 python3 tools/gemv_bench.py --iters 30 --modes exact 2>&1 | grep -v amdgpu.ids || exit 1
for v in 8 5; do echo "== DBG $v"; VSIM_CHAIN_DBG=$v timeout -k 10 100 python3 tools/gemv_bench.py --iters 30 --modes exact --no-check 2>&1 | grep -v amdgpu.ids || exit 1; done
