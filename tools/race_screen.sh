#!/bin/bash
# tools/race_screen.sh — r06 race screen (tools/variants/mk_race_screen.py): the full-width
# bit-exact decode tests and the argmax test on the build whose hand-off producers are delayed
# (vsim_amd/_build/var/rsdelay.so: must pass), then the full-width tests on the same build with
# the r05 key-row barrier removed (rsnobar.so: must fail).  Writes gpurun_out/r06_race_screen.txt.
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
rep=$out/r06_race_screen.txt
{
  echo "race screen: $(date -u)  commit $(cat "$root/.git_head" 2>/dev/null || echo '?')"
  echo "[1] delayed producers (rsdelay.so): test_gpu_fullwidth.py + test_argmax_numpy_conventions, expected PASS"
} > "$rep"
VSIM_LIB=$root/vsim_amd/_build/var/rsdelay.so timeout -k 10 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread -m gpu \
  "$root/tests/test_gpu_fullwidth.py" "$root/tests/test_gpu_ops.py::test_argmax_numpy_conventions" -p no:cacheprovider > "$out/r06_rs_delay.log" 2>&1
rc=$?
tail -3 "$out/r06_rs_delay.log" >> "$rep"; echo "exit=$rc" >> "$rep"
[ "$rc" -gt 1 ] && { cat "$rep"; exit $rc; }
echo "[2] delayed producers + the key-row barrier removed (rsnobar.so): test_gpu_fullwidth.py gpt-j-6B, expected FAIL" >> "$rep"
VSIM_LIB=$root/vsim_amd/_build/var/rsnobar.so timeout -k 10 600 python3 -u -m pytest -q --timeout 400 --timeout-method thread -m gpu \
  "$root/tests/test_gpu_fullwidth.py::test_full_width_decode_bit_exact[gpt-j-6B-300]" -p no:cacheprovider > "$out/r06_rs_nobar.log" 2>&1
rc2=$?
grep -E "Failed:|decode step|passed|failed" "$out/r06_rs_nobar.log" | head -5 >> "$rep"; echo "exit=$rc2" >> "$rep"
cat "$rep"
[ "$rc2" -gt 1 ] && exit $rc2
exit 0
