set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
: > $o/other.jsonl
for c in pythia-12b gpt-neoxt-20b bloom-560m; do for md in exact fast; do
timeout -k 10 400 python3 bench.py --config $c --mode $md --no-cpu-baseline --no-fast --steps 128 > $o/oc.log 2>&1 || { tail -5 $o/oc.log; exit 1; }
tail -1 $o/oc.log >> $o/other.jsonl; tail -1 $o/oc.log | cut -c1-140
done; done
