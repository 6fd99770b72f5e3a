#!/bin/bash
# Kernel-time summary and HBM-traffic counters of the exact-mode bench (run on the GPU box):
#   gpurun -- bash tools/profile_round.sh r01
# then copy gpurun_out/prof_<tag>/run_kernel_stats.csv and the counter CSV under profiles/.
set -e
tag=${1:-r01}
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/prof_$tag" -o run --output-format csv -- \
  python3 "$root/bench.py" --steps 32 --warmup 4 --no-cpu-baseline --no-fast > "$out/prof_$tag.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc_$tag" -o run --output-format csv -- \
  python3 "$root/bench.py" --steps 8 --warmup 2 --no-cpu-baseline --no-profile --no-fast > "$out/pmc_$tag.log" 2>&1
echo done
