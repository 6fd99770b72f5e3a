set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_prefill.py -s > gpurun_out/t_prefill.log 2>&1; rc=$?; grep -E "PASS|FAIL|cos" gpurun_out/t_prefill.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config codegen-16B --prefill 2048 --steps 3 --prefill-exact > gpurun_out/bench_prefill_exact.log 2>&1; rc=$?; tail -1 gpurun_out/bench_prefill_exact.log; exit $rc
