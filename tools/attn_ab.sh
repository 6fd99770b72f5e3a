# attention A/B: tools/attn_bench.py on the default library and each variant library given
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 tools/attn_bench.py || exit 1
for v in "$@"; do
  echo "== $v"
  VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/$v.so timeout -k 10 120 python3 tools/attn_bench.py || exit 1
done
echo "== default again"
timeout -k 10 120 python3 tools/attn_bench.py
