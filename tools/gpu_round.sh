#!/bin/bash
# tools/gpu_round.sh TAG — the round's measurement pass on one GPU box: the default bench line
# (exact value + fast companion + CPU baseline) after FETCH_SIZE passes (HBM traffic) of both
# decode modes, rocprofv3 kernel summaries of exact decode, fast decode and the codegen-16B
# prefill, and the bloom-560m CPU-path baseline on this box's host.  Every GPU step has its own time limit; a fatal exit ends the script.
set -u
tag=${1:-r01}
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/gpurun_out
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
fatal() { local rc=$1; echo "[gpu_round] $2 exit=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
# FETCH_SIZE passes first, installed as this round's profiles/<tag>_pmc_fetch_*.csv on this box,
# so the bench line below reports traffic measured on the same commit in the same call
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc_exact_$tag" -o run --output-format csv -- \
  python3 "$root/bench.py" --steps 8 --warmup 2 --no-cpu-baseline --no-pipeline-20b --no-profile --no-fast --no-other-configs --no-prefill-companion > "$out/pmc_exact_$tag.log" 2>&1
fatal $? pmc_exact
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc_fast_$tag" -o run --output-format csv -- \
  python3 "$root/bench.py" --mode fast --steps 8 --warmup 2 --no-cpu-baseline --no-pipeline-20b --no-profile > "$out/pmc_fast_$tag.log" 2>&1
fatal $? pmc_fast
for m in exact fast; do
  f=$(find "$out/pmc_${m}_$tag" -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$root/profiles/${tag}_pmc_fetch_$m.csv" && cp "$f" "$out/${tag}_pmc_fetch_$m.csv"
done
timeout -k 10 400 python3 "$root/bench.py" > "$out/bench_default_$tag.log" 2>&1
fatal $? bench; tail -1 "$out/bench_default_$tag.log"
timeout -k 10 300 python3 "$root/bench.py" --config codegen-16B --prefill 2048 --steps 3 > "$out/bench_prefill_$tag.log" 2>&1
fatal $? prefill; tail -1 "$out/bench_prefill_$tag.log"
timeout -k 10 300 python3 "$root/bench.py" --config bloom-560m --steps 128 --no-cpu-baseline > "$out/bench_bloom_$tag.log" 2>&1
fatal $? bloom; tail -1 "$out/bench_bloom_$tag.log" | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/prof_exact_$tag" -o run --output-format csv -- \
  python3 "$root/bench.py" --steps 64 --warmup 4 --no-cpu-baseline --no-pipeline-20b --no-fast --no-profile --no-other-configs --no-prefill-companion > "$out/prof_exact_$tag.log" 2>&1
fatal $? prof_exact
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/prof_fast_$tag" -o run --output-format csv -- \
  python3 "$root/bench.py" --mode fast --steps 64 --warmup 4 --no-cpu-baseline --no-pipeline-20b --no-profile > "$out/prof_fast_$tag.log" 2>&1
fatal $? prof_fast
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/prof_prefill_$tag" -o run --output-format csv -- \
  python3 "$root/bench.py" --config codegen-16B --prefill 2048 --steps 2 > "$out/prof_prefill_$tag.log" 2>&1
fatal $? prof_prefill
timeout -k 10 300 python3 "$root/tools/cpu_bloom_baseline.py" --out "$out/${tag}_cpu_bloom560m_gpubox.json" > "$out/cpu_bloom_$tag.log" 2>&1
fatal $? cpu_bloom; tail -1 "$out/cpu_bloom_$tag.log" | cut -c1-300
echo "[gpu_round] done"
