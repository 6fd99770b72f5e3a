#!/bin/bash
# r05 experiment batch (barrier-free chain GEMVs).  Env: PARITY="t:s" (full-width parity of the four
# configs with VSIM_TAIL_NB=t VSIM_SOLO_NB=s first), STAMPS="t:s ..." (tools/nb_stamps.py on the
# nbstamps variant build), BENCH="t:s ..." (248-token bench lines, two alternating rounds).
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
tag=$1
if [ -n "${PARITY:-}" ]; then
  VSIM_TAIL_NB=${PARITY%:*} VSIM_SOLO_NB=${PARITY#*:} timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 \
    --timeout-method thread -m gpu "$root/tests/test_gpu_fullwidth.py" > "$out/r05_${tag}_parity.log" 2>&1
  rc=$?; echo "[parity $PARITY] exit=$rc"; tail -3 "$out/r05_${tag}_parity.log" | cut -c1-300; [ "$rc" -ne 0 ] && exit $rc
fi
for v in ${STAMPS:-}; do
  VSIM_LIB=$root/vsim_amd/_build/var/nbstamps.so VSIM_TAIL_NB=${v%:*} VSIM_SOLO_NB=${v#*:} timeout -k 10 120 \
    python3 "$root/tools/nb_stamps.py" 64 > "$out/r05_${tag}_stamps_${v/:/}.txt" 2>&1
  rc=$?; echo "[stamps $v] exit=$rc"; cat "$out/r05_${tag}_stamps_${v/:/}.txt"; [ "$rc" -ne 0 ] && exit $rc
done
for rep in 1 2; do
  for v in ${BENCH:-}; do
    t=${v%:*}; so=${v#*:}
    VSIM_TAIL_NB=$t VSIM_SOLO_NB=$so timeout -k 10 200 python3 "$root/bench.py" --no-cpu-baseline --no-pipeline-20b \
      --no-fast --no-other-configs > "$out/r05_${tag}_bench_$t${so}_$rep.log" 2>&1
    rc=$?; [ "$rc" -ne 0 ] && { echo "[bench $v] exit=$rc"; tail -5 "$out/r05_${tag}_bench_$t${so}_$rep.log"; exit $rc; }
    python3 - "$out/r05_${tag}_bench_$t${so}_$rep.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk = {k["kernel"].split(" (")[0] + (" lm" if "lm_head" in k["kernel"] else ""): k["avg_us"] for k in d["roofline"]["per_kernel"]}
print(f"tail:solo={sys.argv[2]} {d['value']:.1f} tok/s {d['ms_per_step']:.4f} ms", pk)
PY
  done
done
exit 0
