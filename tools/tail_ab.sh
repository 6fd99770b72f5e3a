#!/bin/bash
# tools/tail_ab.sh [VARIANT...] — decode A/B in one call: the consumer-loop probe (tools/cons_lat3,
# when built), then for each round and variant a 128-token bench line with per-kernel event
# times.  "product" is the in-tree library; any other name is vsim_amd/_build/var/NAME.so
# (tools/build_variant.sh); NAME+bidx also sets VSIM_TAIL_BLOCKIDX=1 (builds that read it).
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
[ -n "${CONS_LAT:-}" ] && [ -x "$root/tools/cons_lat3" ] && { timeout -k 10 120 "$root/tools/cons_lat3" | tee "$out/r04_cons_lat3.txt" || exit 1; }
vars=${*:-product}
for i in 1 2; do
  for v in $vars; do
    unset VSIM_TAIL_BLOCKIDX VSIM_LIB
    name=${v%+bidx}
    [ "$name" != "$v" ] && export VSIM_TAIL_BLOCKIDX=1
    [ "$name" != product ] && export VSIM_LIB=$root/vsim_amd/_build/var/$name.so
    timeout -k 10 300 python3 "$root/bench.py" --no-cpu-baseline --no-pipeline-20b --no-fast --steps ${STEPS:-128} > "$out/tail_ab_$v$i.log" 2>&1 || exit 2
    python3 -c "
import json
d=json.loads([l for l in open('$out/tail_ab_$v$i.log') if l.startswith('{')][-1])
print('$v', d['value'], [(k['kernel'].split()[0], k['avg_us']) for k in d['roofline']['per_kernel']])"
  done
done
