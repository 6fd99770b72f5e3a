#!/bin/bash
# r05 A/B of library builds: VARIANTS="name ..." (vsim_amd/_build/var/NAME.so; "product" = the in-tree
# library; "VAR=VAL" = the in-tree library with that environment variable), PARITY=1 runs the
# full-width parity tests on the product first (PARITY_ENV="VAR=VAL" for them); 248-token bench
# lines, two alternating rounds, per-kernel event times.
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
tag=${1:-v1}
if [ "${PARITY:-1}" = 1 ]; then
  env ${PARITY_ENV:-VSIM_NONE=0} timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    "$root/tests/test_gpu_fullwidth.py" > "$out/r05_${tag}_parity.log" 2>&1
  rc=$?; echo "[parity] exit=$rc"; tail -3 "$out/r05_${tag}_parity.log" | cut -c1-300; [ "$rc" -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for v in ${VARIANTS:-product}; do
    lib=""; ev="VSIM_NONE=0"
    case $v in product) ;; *=*) ev=$v ;; *) lib=$root/vsim_amd/_build/var/$v.so ;; esac
    env VSIM_LIB=$lib "$ev" timeout -k 10 200 python3 "$root/bench.py" --no-cpu-baseline --no-pipeline-20b --no-fast \
      --no-other-configs --no-prefill-companion ${BENCH_ARGS:-} > "$out/r05_${tag}_bench_${v}_${rep}.log" 2>&1
    rc=$?; [ "$rc" -ne 0 ] && { echo "[bench $v] exit=$rc"; tail -5 "$out/r05_${tag}_bench_${v}_${rep}.log"; exit $rc; }
    python3 - "$out/r05_${tag}_bench_${v}_${rep}.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk = {k["kernel"].split(" (")[0] + (" lm" if "lm_head" in k["kernel"] else ""): k["avg_us"] for k in d["roofline"]["per_kernel"]}
print(f"{sys.argv[2]:10s} {d['value']:.1f} tok/s {d['ms_per_step']:.4f} ms", pk)
PY
  done
done
exit 0
