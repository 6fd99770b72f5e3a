#!/bin/bash
# bloom-560m full-width decode (the fused tail without fc_out tiles) on the product library and
# on the no-steal variant of the head-claim protocol
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 "$root/tools/cons_lat2" | tee "$out/r04_cons_lat2.txt" || exit 1
for v in product nosteal; do
  unset VSIM_LIB; [ $v = nosteal ] && export VSIM_LIB=$root/vsim_amd/_build/var/nosteal.so
  timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    "$root/tests/test_gpu_fullwidth.py" -k "bloom or gpt-j" > "$out/r04_bloom_$v.log" 2>&1
  rc=$?; echo "[$v] exit=$rc"; grep -E "passed|failed|Failed" "$out/r04_bloom_$v.log" | tail -3 | cut -c1-250
  [ "$rc" -gt 1 ] && exit $rc
done
python3 -c "
import sys; sys.path.insert(0, '$root')
from vsim_amd import hip; print('spin timeouts', hip.spin_timeouts())"
exit 0
