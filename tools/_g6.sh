set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/fast_prefill_distribution.py --prompts 12 --out gpurun_out/r03_fast_prefill_e2e_distribution.json > gpurun_out/fpd.log 2>&1; rc=$?; tail -2 gpurun_out/fpd.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config codegen-16B --prefill 2048 --steps 3 --prefill-exact > gpurun_out/bench_prefill_exact.log 2>&1; rc=$?; tail -1 gpurun_out/bench_prefill_exact.log; exit $rc
