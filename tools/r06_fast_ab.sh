#!/bin/bash
# r06 late: fast-mode A/B of library builds (VARIANTS: vsim_amd/_build/var/NAME.so, "product" = in-tree):
# the fast GPU tests on the product, bit-identity of every variant's fast decode against the first
# (tools/fast_ab.py, GPT-J-6B and GPT-NeoXT-20B widths, 4 layers), then fast-mode 248-token bench lines.
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
tag=${1:-fa}
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$root/tests/test_gpu_fast.py" \
  > "$out/r06_${tag}_fast_tests.log" 2>&1; rc=$?; echo "[fast tests] exit=$rc"; tail -2 "$out/r06_${tag}_fast_tests.log"
[ "$rc" -ne 0 ] && exit $rc
V=${VARIANTS:-tpw1 product}
for c in gpt-j-6B gpt-neoxt-20b; do
  first=""
  for v in $V; do
    lib=""; [ "$v" != product ] && lib=$root/vsim_amd/_build/var/$v.so
    env VSIM_LIB=$lib timeout -k 10 200 python3 "$root/tools/fast_ab.py" --config $c --out "$out/fa_${c}_$v.npz" > /dev/null 2>&1 \
      || { echo "[fast_ab $c $v] failed"; exit 1; }
    if [ -z "$first" ]; then first=$v; else
      echo -n "$c $first vs $v: "; python3 "$root/tools/fast_ab.py" --compare "$out/fa_${c}_$first.npz" "$out/fa_${c}_$v.npz"
    fi
  done
done
for rep in 1 2; do
  for v in $V; do
    lib=""; [ "$v" != product ] && lib=$root/vsim_amd/_build/var/$v.so
    env VSIM_LIB=$lib timeout -k 10 200 python3 "$root/bench.py" --mode fast --no-cpu-baseline --no-pipeline-20b --no-fast \
      --no-other-configs --no-prefill-companion > "$out/r06_${tag}_bench_${v}_${rep}.log" 2>&1
    rc=$?; [ "$rc" -ne 0 ] && { echo "[bench $v] exit=$rc"; tail -5 "$out/r06_${tag}_bench_${v}_${rep}.log"; exit $rc; }
    python3 - "$out/r06_${tag}_bench_${v}_${rep}.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk = {k["kernel"].split(" (")[0] + (" lm" if "lm_head" in k["kernel"] else ""): k["avg_us"] for k in d["roofline"]["per_kernel"]}
print(f"{sys.argv[2]:10s} {d['value']:.1f} tok/s {d['ms_per_step']:.4f} ms", pk)
PY
  done
done
exit 0
