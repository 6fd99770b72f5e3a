set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/attn_check.sh || exit 1
echo "== nostag"; VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/nostag.so timeout -k 10 120 python3 tools/attn_bench.py || exit 1
echo "== stag"; timeout -k 10 120 python3 tools/attn_bench.py || exit 1
echo "== nostag"; VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/nostag.so timeout -k 10 120 python3 tools/attn_bench.py
