#!/bin/bash
# tools/r06_round.sh — r06's measurement pass on the commit being measured: tools/gpu_round.sh r06
# (FETCH_SIZE passes, the default bench line with every companion, prefill and bloom lines, rocprof
# kernel summaries of exact / fast decode and the codegen-16B prompt, the bloom CPU baseline), then
# the files bench.py cites installed under profiles/ with this round's names, and the pythia-12b and
# GPT-NeoXT-20B 248-token lines.  Every GPU step has its own time limit (in gpu_round.sh too).
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"
bash "$root/tools/gpu_round.sh" r06 || exit $?
for m in exact fast prefill; do
  f=$(find "$out/prof_${m}_r06" -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$out/r06_${m}_kernel_stats.csv"
done
cd /tmp && export TMPDIR=/tmp
for cfg in pythia-12b gpt-neoxt-20b; do
  timeout -k 10 400 python3 "$root/bench.py" --config $cfg --no-cpu-baseline --no-pipeline-20b --no-fast --no-other-configs \
    --no-prefill-companion > "$out/r06_bench_$cfg.log" 2>&1 || { echo "[r06_round] $cfg exit=$?"; exit 1; }
  tail -1 "$out/r06_bench_$cfg.log" | cut -c1-160
done
echo "[r06_round] done"
