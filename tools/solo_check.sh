# exact decode change: model/fullwidth/pipeline parity, default bench + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullwidth.py tests/test_gpu_pipeline.py tests/test_gpu_prefill.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/solo_tests.log 2>&1 || { tail -30 $o/solo_tests.log; exit 1; }
tail -1 $o/solo_tests.log
bash tools/bench_prof.sh solo
