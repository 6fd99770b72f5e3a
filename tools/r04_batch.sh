#!/bin/bash
# round-4 experiment batch: decode tail variants (tools/tail_ab.sh), then the exact prompt on the
# product library and on the scalar-VALU build of k_gemm_exact (gx_scalar)
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
bash "$root/tools/tail_ab.sh" product burst r03tail || exit $?
for v in product gx_scalar; do
  unset VSIM_LIB; [ $v != product ] && export VSIM_LIB=$root/vsim_amd/_build/var/$v.so
  timeout -k 10 300 python3 "$root/bench.py" --config codegen-16B --prefill 2048 --prefill-exact --steps 1 > "$out/r04_pfx_$v.log" 2>&1 || exit 3
  echo "$v $(grep -o '"exact_mode": {"ms_per_prompt": [0-9.]*' "$out/r04_pfx_$v.log")"
done
