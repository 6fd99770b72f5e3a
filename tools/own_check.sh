# solo consumer's own block: exact-path tests, then the default bench A/B against VSIM_SOLO_OWN=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gemv or fullwidth or fulldepth or solo or exact or lm_head or decode" > gpurun_out/own_tests.log 2>&1 || { tail -30 gpurun_out/own_tests.log; exit 1; }
tail -2 gpurun_out/own_tests.log
B="--no-cpu-baseline --no-pipeline-20b --no-fast"
for i in 1 2; do
  echo "== own"; timeout -k 10 300 python3 bench.py $B 2>/dev/null | tail -1 | cut -c1-160 || exit 4
  echo "== noown"; VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/noown.so timeout -k 10 300 python3 bench.py $B 2>/dev/null | tail -1 | cut -c1-160 || exit 4
done
