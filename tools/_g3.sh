set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_graph_dropin.py tests/test_dropin.py > gpurun_out/t_graph.log 2>&1
rc=$?; tail -20 gpurun_out/t_graph.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/graph_speed.py --layers 4 --out gpurun_out/graph_speed_4l.json > gpurun_out/graph_speed.log 2>&1
rc=$?; tail -8 gpurun_out/graph_speed.log; exit $rc
