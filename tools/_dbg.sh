set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
for t in 1 2 3 4; do VSIM_PF_ACT=0 timeout -k 10 120 python3 tools/prefill_ab.py --file --config small-gptj --n2 8 --out $o/b$t.npz > $o/b$t.log 2>&1 || { tail -5 $o/b$t.log; exit 1; }; done
for t in 2 3 4; do python3 tools/prefill_ab.py --compare $o/b1.npz $o/b$t.npz | cut -c1-70; done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
