set -u
for v in 1 2; do echo "== variant $v"; VSIM_LIB=$PWD/tools/_ab$v/libvsim_hip.so timeout -k 10 300 python -u tools/gemm_bench.py 2>&1 | grep q4; done
