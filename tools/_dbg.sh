set -o pipefail
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pf -o pf -- python3 $GRAFT_REPO_ROOT/bench.py --config codegen-16B --prefill 2048 > $GRAFT_REPO_ROOT/gpurun_out/pf.log 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/pf -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -14
