#!/bin/bash
# decode variant batch: full-width parity (GPT-J-6B, bloom-560m) per variant library, then the
# alternating decode A/B (tools/tail_ab.sh).  usage: r04_batch2.sh VARIANT...
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  unset VSIM_LIB; [ $v != product ] && export VSIM_LIB=$root/vsim_amd/_build/var/$v.so
  timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    "$root/tests/test_gpu_fullwidth.py" -k "${PARITY_K:-gpt-j or bloom}" > "$out/r04_par_$v.log" 2>&1
  rc=$?; echo "[$v] parity exit=$rc $(grep -E 'passed|failed' "$out/r04_par_$v.log" | tail -1)"
  [ "$rc" -gt 1 ] && exit $rc
done
unset VSIM_LIB
bash "$root/tools/tail_ab.sh" "$@"
