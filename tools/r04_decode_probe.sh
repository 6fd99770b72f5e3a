#!/bin/bash
# tools/r04_decode_probe.sh — consumer-loop cycles per add (tools/cons_lat), the decode-path GPU
# tests, then the default bench line (exact decode with the per-kernel event times)
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 "$root/tools/cons_lat" | tee "$out/r04_cons_lat.txt" || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  "$root/tests/test_gpu_fullwidth.py" "$root/tests/test_gpu_fulldepth.py" "$root/tests/test_gpu_model.py" \
  "$root/tests/test_graph_dropin.py" "$root/tests/test_gpu_pipeline.py" > "$out/r04_decode_tests.log" 2>&1
rc=$?; echo "[probe] decode tests exit=$rc"; tail -3 "$out/r04_decode_tests.log"
[ "$rc" -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 "$root/bench.py" --no-cpu-baseline --no-pipeline-20b --no-fast --steps 128 > "$out/r04_dec_$i.log" 2>&1 || exit 2
  python3 -c "
import json
d=json.loads([l for l in open('$out/r04_dec_$i.log') if l.startswith('{')][-1])
print(d['value'], [(k['kernel'].split()[0], k['avg_us']) for k in d['roofline']['per_kernel']])"
done
