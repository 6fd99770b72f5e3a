#!/bin/bash
# tools/r04_probe.sh [suite] — round 4 GPU pass: the op tests of the exact prompt path first (or
# the whole -m gpu suite with "suite"), the prompt tests, then a kernel-stats profile of the
# codegen-16B exact-mode prompt (and its bench line).  A test failure (exit 1) still lets the
# profile run; any other non-zero exit ends the script.
set -u
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/gpurun_out
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
if [ -x "$root/tools/chain_lat" ]; then
  timeout -k 10 60 "$root/tools/chain_lat" > "$out/r04_chain_lat.txt" 2>&1
  rc=$?; echo "[probe] chain_lat exit=$rc"; cat "$out/r04_chain_lat.txt"
  if [ "$rc" -ne 0 ]; then exit "$rc"; fi
fi
if [ "${1:-}" = suite ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread --durations 15 -m gpu \
    "$root/tests" > "$out/r04_suite.log" 2>&1
  rc=$?; echo "[probe] gpu suite exit=$rc"; tail -4 "$out/r04_suite.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
  REPS=20 RACE_SHAPES=6144x6144x2048,4096x16384x2048,6144x24576x2048 timeout -k 10 300 python3 "$root/tools/gemm_race.py" \
    > "$out/r04_race.log" 2>&1
  rc3=$?; echo "[probe] race screen exit=$rc3"; tail -3 "$out/r04_race.log"
  if [ "$rc3" -ne 0 ]; then exit "$rc3"; fi
  for i in 1 2; do
    timeout -k 10 300 python3 "$root/bench.py" --config codegen-16B --prefill 2048 --steps 3 > "$out/r04_pf_$i.log" 2>&1 || exit 4
    echo "[probe] prefill $(grep -o '"ms_per_prompt": [0-9.]*' "$out/r04_pf_$i.log" | head -1)"
  done
  timeout -k 10 300 python3 "$root/bench.py" --no-cpu-baseline --no-pipeline-20b > "$out/r04_bench.log" 2>&1
  rc3=$?; echo "[probe] bench exit=$rc3"; tail -1 "$out/r04_bench.log" | cut -c1-300
  if [ "$rc3" -ne 0 ]; then exit "$rc3"; fi
else
  timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -s \
    "$root/tests/test_gpu_ops.py" -k "exact or prompt_gemm or kq" > "$out/r04_exact_ops.log" 2>&1
  rc=$?; echo "[probe] exact op tests exit=$rc"; tail -3 "$out/r04_exact_ops.log"
  if [ "$rc" -ne 0 ]; then exit "$rc"; fi
  timeout -k 10 700 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -s \
    "$root/tests/test_gpu_prefill.py" > "$out/r04_prefill_tests.log" 2>&1
  rc=$?; echo "[probe] prefill tests exit=$rc"; tail -3 "$out/r04_prefill_tests.log"
fi
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_pf_exact" -o run --output-format csv -- \
  python3 "$root/bench.py" --config codegen-16B --prefill 2048 --prefill-exact --steps 1 > "$out/prof_pf_exact.log" 2>&1
rc2=$?; echo "[probe] exact prefill profile exit=$rc2"; grep -o '"exact_mode": {[^}]*}' "$out/prof_pf_exact.log"
exit $(( rc > rc2 ? rc : rc2 ))
