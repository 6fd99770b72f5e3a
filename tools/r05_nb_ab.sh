#!/bin/bash
# r05: barrier-free chain GEMVs in the exact decode (VSIM_TAIL_NB bit 0: the tail's fc_out tiles,
# bit 1: its out-projection tiles; VSIM_SOLO_NB=1: k_gemv_solo).  Parity first (GPT-J-6B and
# bloom-560m full width, 300 steps, every NB path on), then 248-token bench lines alternating the
# variants, with the per-kernel event times.
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
tag=${1:-nb}
VSIM_TAIL_NB=3 VSIM_SOLO_NB=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  "$root/tests/test_gpu_fullwidth.py" -k "gpt-j or bloom" > "$out/r05_${tag}_parity.log" 2>&1
rc=$?; echo "[parity] exit=$rc"; tail -3 "$out/r05_${tag}_parity.log" | cut -c1-300
[ "$rc" -ne 0 ] && exit $rc
for v in 0:0 3:0 0:1 3:1 0:0 3:0 0:1 3:1; do
  t=${v%:*}; so=${v#*:}
  VSIM_TAIL_NB=$t VSIM_SOLO_NB=$so timeout -k 10 200 python3 "$root/bench.py" --no-cpu-baseline --no-pipeline-20b \
    --no-fast --no-other-configs > "$out/r05_${tag}_bench_$t$so.log" 2>&1
  rc=$?; [ "$rc" -ne 0 ] && { echo "[bench $v] exit=$rc"; tail -5 "$out/r05_${tag}_bench_$t$so.log"; exit $rc; }
  python3 - "$out/r05_${tag}_bench_$t$so.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk = {k["kernel"].split(" (")[0] + (" lm" if "lm_head" in k["kernel"] else ""): k["avg_us"] for k in d["roofline"]["per_kernel"]}
print(f"tail:solo={sys.argv[2]} {d['value']:.1f} tok/s {d['ms_per_step']:.4f} ms", pk)
PY
done
exit 0
