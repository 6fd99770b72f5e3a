set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread > $o/pipe_tests.log 2>&1 || { tail -40 $o/pipe_tests.log; exit 1; }
tail -8 $o/pipe_tests.log
timeout -k 10 300 python3 bench.py --config gpt-neoxt-20b --pipeline --steps 64 --warmup 4 --no-cpu-baseline > $o/pipe1.log 2>&1 || { tail -20 $o/pipe1.log; exit 1; }
tail -1 $o/pipe1.log | cut -c1-400
timeout -k 10 300 python3 bench.py --config gpt-neoxt-20b --steps 64 --warmup 4 --no-cpu-baseline --no-fast --no-profile > $o/single20b.log 2>&1 || { tail -20 $o/single20b.log; exit 1; }
tail -1 $o/single20b.log | cut -c1-400
