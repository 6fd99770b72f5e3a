set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_fast.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fast_tests.log 2>&1 || { tail -30 gpurun_out/fast_tests.log; exit 1; }
tail -2 gpurun_out/fast_tests.log
for ln in 1 0 1 0; do echo "== LN fused $ln"; VSIM_FAST_LN=$ln timeout -k 10 300 python3 bench.py --mode fast --no-cpu-baseline --no-profile 2>&1 | tail -1 | cut -c90-150 || exit 1; done
