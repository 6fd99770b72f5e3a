set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
run() { for t in 1 2 3 4 5; do env $1 timeout -k 10 120 python3 tools/prefill_ab.py $2 --out $o/n$t.npz > $o/n$t.log 2>&1 || { tail -5 $o/n$t.log; return 1; }; done
echo "== $1 $2"; for t in 2 3 4 5; do python3 tools/prefill_ab.py --compare $o/n1.npz $o/n$t.npz | cut -c1-60; done; }
run "X=1" "--config small-neox --n2 8"
run "X=1" "--config small-neox --file --n2 16"
run "X=1" "--config small-gptj --n2 12"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
timeout -k 10 300 python3 bench.py --config codegen-16B --prefill 2048 --steps 3 2>&1 | tail -1 | cut -c1-200
