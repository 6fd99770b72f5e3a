set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ops.py -k "prompt_gemm or q4_in_lds or gemm_f16 or gelu_epilogue or rope_join" -s > gpurun_out/t_q4gemm.log 2>&1
rc=$?; grep -E "PASS|FAIL|max \|y|Error|error" gpurun_out/t_q4gemm.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gemm_bench_q4.log 2>&1; rc=$?; cat gpurun_out/gemm_bench_q4.log; [ $rc -ne 0 ] && exit $rc
REPS=20 timeout -k 10 300 python -u tools/gemm_race.py > gpurun_out/gemm_race_q4.log 2>&1; rc=$?; tail -3 gpurun_out/gemm_race_q4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config codegen-16B --prefill 2048 --steps 3 > gpurun_out/bench_prefill_q4.log 2>&1; rc=$?; tail -1 gpurun_out/bench_prefill_q4.log | cut -c1-600; exit $rc
