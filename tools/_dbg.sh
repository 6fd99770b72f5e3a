set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k layer_kernel > gpurun_out/lk.log 2>&1 || { tail -30 gpurun_out/lk.log; exit 1; }
tail -2 gpurun_out/lk.log
