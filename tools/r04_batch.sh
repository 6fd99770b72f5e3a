#!/bin/bash
# round-4 experiment batch: full-width decode parity (GPT-J-6B, bloom-560m) of each decode
# variant library, then the decode A/B (tools/tail_ab.sh), then the exact prompt on the product
# library and on the scalar-VALU build of k_gemm_exact (gx_scalar)
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
VARS="product burst burst6 r03tail"
for v in $VARS; do
  unset VSIM_LIB; [ $v != product ] && export VSIM_LIB=$root/vsim_amd/_build/var/$v.so
  timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    "$root/tests/test_gpu_fullwidth.py" -k "gpt-j or bloom" > "$out/r04_par_$v.log" 2>&1
  rc=$?; echo "[$v] parity exit=$rc $(grep -E 'passed|failed' "$out/r04_par_$v.log" | tail -1)"
  [ "$rc" -gt 1 ] && exit $rc
done
unset VSIM_LIB
bash "$root/tools/tail_ab.sh" $VARS || exit $?
for v in product gx_scalar; do
  unset VSIM_LIB; [ $v != product ] && export VSIM_LIB=$root/vsim_amd/_build/var/$v.so
  timeout -k 10 300 python3 "$root/bench.py" --config codegen-16B --prefill 2048 --prefill-exact --steps 1 > "$out/r04_pfx_$v.log" 2>&1 || exit 3
  echo "$v $(grep -o '"exact_mode": {"ms_per_prompt": [0-9.]*' "$out/r04_pfx_$v.log")"
done
for i in 1 2; do
  for v in product skold; do
    unset VSIM_LIB; [ $v != product ] && export VSIM_LIB=$root/vsim_amd/_build/var/$v.so
    timeout -k 10 300 python3 "$root/bench.py" --config codegen-16B --prefill 2048 --steps 3 > "$out/r04_pf_$v$i.log" 2>&1 || exit 4
    echo "prefill $v $(grep -o '"ms_per_prompt": [0-9.]*' "$out/r04_pf_$v$i.log" | head -1)"
  done
done
