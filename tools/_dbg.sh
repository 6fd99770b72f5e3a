set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "prefill" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
VSIM_LIB=vsim_amd/_build/var/base.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "prefill_deterministic" > gpurun_out/pt0.log 2>&1; tail -3 gpurun_out/pt0.log
