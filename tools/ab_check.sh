#!/bin/bash
# tools/ab_check.sh TAG — parity of the decode path at full width + the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
tag=${1:-ab}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullwidth.py tests/test_gpu_model.py -x -q --timeout 400 --timeout-method thread > $o/ab_tests_$tag.log 2>&1 || { tail -30 $o/ab_tests_$tag.log; exit 1; }
tail -2 $o/ab_tests_$tag.log
timeout -k 10 600 python3 bench.py --no-cpu-baseline > $o/ab_bench_$tag.log 2>&1 || { tail -20 $o/ab_bench_$tag.log; exit 1; }
tail -1 $o/ab_bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step']); [print('  %-45s %8.3f us %6.1f GB/s' % (k['kernel'], k['avg_us'], k['GBps'])) for k in r['per_kernel']]; print('fast', d.get('fast_mode',{}).get('value'))"
