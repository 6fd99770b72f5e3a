set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_model.py::test_stage_step_needs_fresh_begin_after_eval tests/test_gpu_pipeline.py tests/test_gpu_fulldepth.py > gpurun_out/t_fulldepth.log 2>&1
rc=$?; tail -15 gpurun_out/t_fulldepth.log; exit $rc
