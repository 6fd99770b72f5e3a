#!/bin/bash
# r04: tile-order A/B (GEMM microbench and the codegen-16B prompt, in process), then the GEMM and
# prompt parity tests and the full-width decode tests on the product library.
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
GEMM_IMG=0 GEMM_ORDERS=4,0 timeout -k 10 180 python3 "$root/tools/gemm_bench.py" > "$out/r04_tile_order_gemm.txt" 2>&1 || exit 1
grep "tile order" "$out/r04_tile_order_gemm.txt"
timeout -k 10 300 python3 "$root/tools/prefill_order_ab.py" 4,0 3 3 > "$out/r04_tile_order_prefill.txt" 2>&1 || exit 2
grep "tile order" "$out/r04_tile_order_prefill.txt" | tail -2
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$root/tests/test_gpu_ops.py" \
  "$root/tests/test_gpu_prefill.py" "$root/tests/test_gpu_fullwidth.py" > "$out/r04_batch3_tests.log" 2>&1
rc=$?; tail -3 "$out/r04_batch3_tests.log"; exit $rc
