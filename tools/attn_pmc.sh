# SQ counters of the prompt attention (tools/attn_bench.py), one rocprofv3 pass per counter set
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d $R/gpurun_out/attn_pmc1 -o run --output-format csv -- python3 $R/tools/attn_bench.py > $R/gpurun_out/attn_pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/attn_pmc2 -o run --output-format csv -- python3 $R/tools/attn_bench.py > $R/gpurun_out/attn_pmc2.log 2>&1 || exit 2

timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/attn_stats -o run --output-format csv -- python3 $R/tools/attn_bench.py > $R/gpurun_out/attn_stats.log 2>&1 || exit 3
echo stats done
