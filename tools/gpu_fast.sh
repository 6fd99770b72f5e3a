#!/bin/bash
# tools/gpu_fast.sh — one gpurun call for the fast-mode decode step: its tests, a fast-mode
# bench line and a rocprofv3 kernel summary (each GPU step under its own time limit).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fast.py -s \
  > gpurun_out/fast_tests.log 2>&1
rc=$?; echo "[gpu_fast] tests exit=$rc"; grep -E "passed|failed|^(tiny|small)|\[\(" gpurun_out/fast_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --mode fast --steps 64 --warmup 4 --no-cpu-baseline --no-pipeline-20b ${BENCH_ARGS:-} > gpurun_out/bench_fast.log 2>&1
rc=$?; echo "[gpu_fast] bench exit=$rc"; tail -1 gpurun_out/bench_fast.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fast -o run --output-format csv -- \
  python3 bench.py --mode fast --steps 32 --warmup 4 --no-cpu-baseline --no-pipeline-20b --no-profile ${BENCH_ARGS:-} > gpurun_out/prof_fast.log 2>&1
rc=$?; echo "[gpu_fast] rocprof exit=$rc"
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_fast/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/prof_fast/run_kernel_stats.csv"):
    for r in list(csv.DictReader(open(f)))[:10]:
        print(f"{r['Name'][:58]:58s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.2f}%")
    break
PY
