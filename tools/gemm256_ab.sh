# N=288 fast prompt vs oracle: new GEMM vs the in-LDS-dequant one (A/B lib), then the prefill bench
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill.py -m gpu -q -s --timeout 300 --timeout-method thread -k "fast_prompt_vs_oracle" > $o/g256_new.log 2>&1
grep -E "cos" $o/g256_new.log
VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/oldgemm.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill.py -m gpu -q -s --timeout 300 --timeout-method thread -k "fast_prompt_vs_oracle" > $o/g256_old.log 2>&1
grep -E "cos" $o/g256_old.log
timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 > $o/bench_prefill_g256.log 2>&1 || { tail -5 $o/bench_prefill_g256.log; exit 1; }
tail -1 $o/bench_prefill_g256.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof_prefill_g256 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config codegen-16B --prefill 2048 --steps 2 > $GRAFT_REPO_ROOT/$o/prof_prefill_g256.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$o/prof_prefill_g256.log; exit 1; }
head -12 $GRAFT_REPO_ROOT/$o/prof_prefill_g256/run_kernel_stats.csv | cut -d, -f1-4
