set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_fast.py -x -q --timeout 120 --timeout-method thread > $o/fast_tests.log 2>&1 || { tail -30 $o/fast_tests.log; exit 1; }
tail -1 $o/fast_tests.log
for c in gpt-j-6B pythia-12b gpt-neoxt-20b; do
VSIM_LIB=vsim_amd/_build/var/base.so timeout -k 10 200 python3 tools/fast_ab.py --config $c --steps 300 --out $o/fa.npz > $o/fa.log 2>&1 || { tail -5 $o/fa.log; exit 1; }
timeout -k 10 200 python3 tools/fast_ab.py --config $c --steps 300 --out $o/fb.npz > $o/fb.log 2>&1 || { tail -5 $o/fb.log; exit 1; }
python3 tools/fast_ab.py --compare $o/fa.npz $o/fb.npz
done
for lib in vsim_amd/_build/var/base.so vsim_amd/_build/libvsim_hip.so vsim_amd/_build/var/base.so vsim_amd/_build/libvsim_hip.so; do echo "== $lib"; VSIM_LIB=$lib timeout -k 10 300 python3 bench.py --mode fast --no-cpu-baseline --no-profile 2>&1 | tail -1 | cut -c90-150 || exit 1; done
