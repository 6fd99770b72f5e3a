# codegen-16B N=2048 prefill: bench line twice, then a rocprofv3 kernel-stats pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 $R/bench.py --config codegen-16B --prefill 2048 --steps 3 2>/dev/null | tail -1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_prefill -o run --output-format csv -- \
  python3 $R/bench.py --config codegen-16B --prefill 2048 --steps 2 > $R/gpurun_out/prof_prefill.log 2>&1 || exit 2
echo prof done
