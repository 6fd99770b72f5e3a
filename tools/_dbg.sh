for v in 0 1 2 4 5 6 7; do echo "== DBG $v"; VSIM_CHAIN_DBG=$v timeout -k 10 100 python3 tools/gemv_bench.py --iters 30 --modes exact --no-check 2>&1 | grep -E "qkvo|fc_out" || exit 1; done
