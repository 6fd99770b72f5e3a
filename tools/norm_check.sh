# prompt LayerNorm: op test + prefill tests, then prefill A/B against VSIM_NORM_WAVE=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "norm or prefill or prompt" > gpurun_out/norm_tests.log 2>&1 || { tail -30 gpurun_out/norm_tests.log; exit 1; }
tail -2 gpurun_out/norm_tests.log
for i in 1 2; do
  echo "== wave"; timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 2>/dev/null | tail -1 | cut -c1-200 || exit 4
  echo "== nonw"; VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/nonw.so timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 2>/dev/null | tail -1 | cut -c1-200 || exit 4
done
