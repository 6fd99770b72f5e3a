# in-launch LayerNorm of the layer tail: decode parity suites, then the default bench + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullwidth.py tests/test_gpu_pipeline.py tests/test_gpu_prefill.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/tailln_tests.log 2>&1 || { tail -40 $o/tailln_tests.log; exit 1; }
tail -3 $o/tailln_tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $o/bench_tailln.log 2>&1 || { tail -5 $o/bench_tailln.log; exit 1; }
tail -1 $o/bench_tailln.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof_tailln -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-fast --no-profile --steps 64 > $GRAFT_REPO_ROOT/$o/prof_tailln.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$o/prof_tailln.log; exit 1; }
find $GRAFT_REPO_ROOT/$o/prof_tailln -name "*kernel_stats.csv" | head -1 | xargs head -8 | cut -d, -f1-4
