# bench lines of the other decode configs (exact + fast companion), one file
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
mkdir -p $o
: > $o/bench_other_configs.jsonl
for c in pythia-12b gpt-neoxt-20b bloom-560m; do
  timeout -k 10 400 python3 bench.py --config $c --steps 128 --no-cpu-baseline > $o/bench_$c.log 2>&1 || { tail -3 $o/bench_$c.log; exit 1; }
  tail -1 $o/bench_$c.log >> $o/bench_other_configs.jsonl
  python3 -c "
import json; d=json.loads(open('$o/bench_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], (d.get('fast_mode') or {}).get('value'))"
done
