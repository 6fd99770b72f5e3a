cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python3 $R/tools/gemv_bench.py --iters 5 --modes exact --no-check > $R/gpurun_out/pmc_sq.log 2>&1
echo rc=$?
