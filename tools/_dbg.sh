timeout -k 10 100 python3 tools/gemv_bench.py --iters 30 --modes exact 2>&1 | grep -v amdgpu.ids || exit 1
