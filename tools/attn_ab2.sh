# prompt attention A/B: the tests and the microbench on the default library, alternating with variant $1
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/attn_check.sh || exit 1
for i in 1 2; do
  echo "== $1"; VSIM_LIB=$GRAFT_REPO_ROOT/vsim_amd/_build/var/$1.so timeout -k 10 120 python3 tools/attn_bench.py || exit 1
  echo "== default"; timeout -k 10 120 python3 tools/attn_bench.py || exit 1
done
