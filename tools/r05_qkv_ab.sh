#!/bin/bash
# r05: Q, K, V in the layer tail (VSIM_TAIL_QKV=1, default) vs in the solo batch (=0): full-width
# parity of the four configs first, then 248-token bench lines alternating, per-kernel event times.
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
tag=${1:-q1}
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    "$root/tests/test_gpu_fullwidth.py" > "$out/r05_${tag}_parity.log" 2>&1
  rc=$?; echo "[parity] exit=$rc"; tail -3 "$out/r05_${tag}_parity.log" | cut -c1-300; [ "$rc" -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for v in ${VARIANTS:-0 1}; do
    VSIM_TAIL_QKV=$v timeout -k 10 200 python3 "$root/bench.py" --no-cpu-baseline --no-pipeline-20b --no-fast \
      --no-other-configs > "$out/r05_${tag}_bench_${v}_${rep}.log" 2>&1
    rc=$?; [ "$rc" -ne 0 ] && { echo "[bench $v] exit=$rc"; tail -5 "$out/r05_${tag}_bench_${v}_${rep}.log"; exit $rc; }
    python3 - "$out/r05_${tag}_bench_${v}_${rep}.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk = {k["kernel"].split(" (")[0] + (" lm" if "lm_head" in k["kernel"] else ""): k["avg_us"] for k in d["roofline"]["per_kernel"]}
print(f"qkv_in_tail={sys.argv[2]} {d['value']:.1f} tok/s {d['ms_per_step']:.4f} ms", pk)
PY
  done
done
exit 0
