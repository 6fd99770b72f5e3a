for d in 10 12; do
echo "== dbg $d"; VSIM_CHAIN_DBG=$d VSIM_CHAIN_ROWS=64 timeout -k 10 100 python3 tools/gemv_bench.py --iters 30 --modes exact --no-check 2>&1 | grep -v amdgpu.ids || exit 1
done
