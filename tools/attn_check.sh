# prompt attention: GPU tests touching it, then the microbench (output hash must stay 7959fb14e410)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or prefill or codegen or gptj or prompt" > gpurun_out/attn_check_tests.log 2>&1 || { tail -30 gpurun_out/attn_check_tests.log; exit 1; }
tail -2 gpurun_out/attn_check_tests.log
timeout -k 10 120 python3 tools/attn_bench.py && timeout -k 10 120 python3 tools/attn_bench.py
