set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "bloom_fast" > gpurun_out/bt.log 2>&1 || { tail -20 gpurun_out/bt.log; exit 1; }
tail -1 gpurun_out/bt.log
