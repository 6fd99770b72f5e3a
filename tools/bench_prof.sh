# default bench line + a rocprofv3 kernel-stats pass (csv) of a shorter bench run
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
tag=${1:-x}
mkdir -p $o
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pipeline-20b ${BENCH_ARGS} > $o/bench_$tag.log 2>&1 || { tail -5 $o/bench_$tag.log; exit 1; }
tail -1 $o/bench_$tag.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-pipeline-20b --no-fast --no-profile --steps 64 ${BENCH_ARGS} > $GRAFT_REPO_ROOT/$o/prof_$tag.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$o/prof_$tag.log; exit 1; }
find $GRAFT_REPO_ROOT/$o/prof_$tag -name "*kernel_stats.csv" | head -1 | xargs head -8 | cut -d, -f1-4
