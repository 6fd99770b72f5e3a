set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1 || exit 1
timeout -k 10 600 python3 bench.py > $o/bench_final.log 2>&1 || { tail -5 $o/bench_final.log; exit 1; }
tail -1 $o/bench_final.log | cut -c1-260
