# stream-K prompt GEMM: GEMM / prefill tests, the race screen, then prefill A/B against VSIM_STREAMK=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or prefill or prompt or codegen or gptj" > gpurun_out/sk_tests.log 2>&1 || { tail -30 gpurun_out/sk_tests.log; exit 1; }
tail -2 gpurun_out/sk_tests.log
REPS=20 timeout -k 10 300 python3 tools/gemm_race.py > gpurun_out/sk_race.log 2>&1 || { tail -20 gpurun_out/sk_race.log; exit 2; }
tail -8 gpurun_out/sk_race.log
GEMM_IMG=0 timeout -k 10 200 python3 tools/gemm_bench.py || exit 3
GEMM_IMG=0 VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/nosk.so timeout -k 10 200 python3 tools/gemm_bench.py || exit 3
for i in 1 2; do
  echo "== sk"; timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 2>/dev/null | tail -1 | cut -c1-200 || exit 4
  echo "== nosk"; VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/nosk.so timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 2>/dev/null | tail -1 | cut -c1-200 || exit 4
done
