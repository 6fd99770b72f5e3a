#!/bin/bash
# tools/pmc_prefill_gemm.sh — SQ counter passes (one rocprofv3 run per counter set) and a
# kernel-stats pass over the long-prompt GEMM microbench at the codegen-16B shapes (N = 2048,
# the model's register-dequant kernel k_gemm_q4r only: GEMM_IMG=0), then the summary.
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
export GEMM_IMG=0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  -d "$out/pmc_gemm1" -o run --output-format csv -- python3 "$root/tools/gemm_bench.py" > "$out/pmc_gemm1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA \
  -d "$out/pmc_gemm2" -o run --output-format csv -- python3 "$root/tools/gemm_bench.py" > "$out/pmc_gemm2.log" 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$out/pmc_gemm_stats" -o run --output-format csv -- python3 "$root/tools/gemm_bench.py" > "$out/pmc_gemm_stats.log" 2>&1 || exit 3
python3 "$root/tools/pmc_summary.py" "$out/pmc_gemm1" "$out/pmc_gemm2" k_gemm_q4r > "$out/r04_pmc_sq_prefill_gemm_summary.txt"
cat "$out/r04_pmc_sq_prefill_gemm_summary.txt"
