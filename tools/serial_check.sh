# serial-residual fused decode: model tests + bloom-560m full width + bloom-560m bench
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullwidth.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bloom or serial or graph_replay or generate" > $o/serial_tests.log 2>&1 || { tail -40 $o/serial_tests.log; exit 1; }
tail -3 $o/serial_tests.log
timeout -k 10 300 python3 bench.py --config bloom-560m --steps 128 --warmup 8 --no-cpu-baseline > $o/bench_bloom.log 2>&1 || { tail -5 $o/bench_bloom.log; exit 1; }
tail -1 $o/bench_bloom.log | cut -c1-400
