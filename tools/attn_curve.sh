#!/bin/bash
# tools/attn_curve.sh — exact attention kernel time vs decode position (VSIM_TAIL=0 puts the
# attention in its own launch, k_attn_decode); prints the per-token mean every 16 positions.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
rm -rf gpurun_out/prof_notail
VSIM_TAIL=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_notail -o run --output-format csv -- \
  python3 bench.py --steps 248 --warmup 8 --no-cpu-baseline --no-pipeline-20b --no-fast --no-profile > gpurun_out/notail.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_notail/**/run_kernel_trace.csv', recursive=True)
rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r['Start_Timestamp']))
att = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if 'k_attn_decode' in r['Kernel_Name']]
per = [sum(att[i * 28:(i + 1) * 28]) / 28 for i in range(len(att) // 28)]
print(len(per), [round(x, 1) for x in per[::16]])
PY
