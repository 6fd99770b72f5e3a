#!/bin/bash
# tools/gpu_check.sh — one gpurun call: GPU tests, smoke, short bench, rocprof summary.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
STEPS=${STEPS:-64}
stop_if_fatal() {  # $1 = exit code, $2 = step name ; test failures (1) are not fatal
  local rc=$1
  echo "[gpu_check] $2 exit=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[gpu_check] fatal exit in $2, stopping"; exit "$rc"; fi
}
echo "[gpu_check] host: $(nproc) cpus, $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)"
rocm-smi --showproductname 2>/dev/null | head -8 || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
stop_if_fatal $? pytest_gpu
tail -30 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
stop_if_fatal $? smoke
cat gpurun_out/smoke.log | tail -3
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 4 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
stop_if_fatal $? bench
tail -3 gpurun_out/bench.log
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline --no-pipeline-20b --no-profile ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  stop_if_fatal $? rocprof
  find gpurun_out/prof -name "*stats*" | head
fi
echo "[gpu_check] done"
