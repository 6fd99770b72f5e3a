# long-prompt GEMM: op tests, prompt parity, determinism, codegen-16B prefill bench + kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or quant or attn_prefill" > $o/g256_ops.log 2>&1 || { tail -30 $o/g256_ops.log; exit 1; }
tail -1 $o/g256_ops.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_prefill.py tests/test_gpu_model.py -m gpu -x -q -s --timeout 300 --timeout-method thread -k "prompt or prefill or poison" > $o/g256_prefill.log 2>&1 || { tail -30 $o/g256_prefill.log; exit 1; }
grep -E "cos|passed|failed" $o/g256_prefill.log | tail -12
timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 > $o/bench_prefill_g256.log 2>&1 || { tail -5 $o/bench_prefill_g256.log; exit 1; }
tail -1 $o/bench_prefill_g256.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof_prefill_g256 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config codegen-16B --prefill 2048 --steps 2 > $GRAFT_REPO_ROOT/$o/prof_prefill_g256.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$o/prof_prefill_g256.log; exit 1; }
head -12 $GRAFT_REPO_ROOT/$o/prof_prefill_g256/run_kernel_stats.csv | cut -d, -f1-4
