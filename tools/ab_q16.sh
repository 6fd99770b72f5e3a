set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or prefill or codegen or gptj" > gpurun_out/q16_tests.log 2>&1
tail -3 gpurun_out/q16_tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 2>/dev/null | tail -1 > gpurun_out/q16_new_$i.json; cat gpurun_out/q16_new_$i.json
  VSIM_LIB=vsim_amd/_build/var/noq16.so timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 2>/dev/null | tail -1 > gpurun_out/q16_old_$i.json; cat gpurun_out/q16_old_$i.json
done
