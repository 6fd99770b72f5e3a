#!/bin/bash
# tools/ab_check.sh TAG [VARIANT...] — parity of the decode path at full width on the main
# build, then the default bench line of the main build and of each A/B variant
# (vsim_amd/_build/var/VARIANT.so, tools/variant.sh), per-kernel times side by side.
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
tag=${1:-ab}; shift
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullwidth.py tests/test_gpu_model.py -x -q --timeout 400 --timeout-method thread > $o/ab_tests_$tag.log 2>&1 || { tail -30 $o/ab_tests_$tag.log; exit 1; }
tail -2 $o/ab_tests_$tag.log
show() {
  tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac']); [print('  %-52s %8.3f us %7.1f GB/s' % (k['kernel'], k['avg_us'], k['GBps'])) for k in r['per_kernel']]"
}
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-pipeline-20b --no-fast > $o/ab_bench_${tag}_main.log 2>&1 || { tail -20 $o/ab_bench_${tag}_main.log; exit 1; }
echo "== main"; show $o/ab_bench_${tag}_main.log
for v in "$@"; do
  VSIM_LIB=vsim_amd/_build/var/$v.so timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-pipeline-20b --no-fast > $o/ab_bench_${tag}_$v.log 2>&1 || { tail -20 $o/ab_bench_${tag}_$v.log; exit 1; }
  echo "== $v"; show $o/ab_bench_${tag}_$v.log
done
