#!/bin/bash
# r06 late: A/B of the wide configs (pythia-12b, GPT-NeoXT-20B: the heads at the end of the GEMV
# launch, k_gemv_solo_heads) -- PARITY=1 first runs the full-width decode parity tests on the
# product; then CONFIGS x VARIANTS bench lines, two alternating rounds.
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
tag=${1:-w1}
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    "$root/tests/test_gpu_fullwidth.py" > "$out/r06_${tag}_parity.log" 2>&1
  rc=$?; echo "[parity] exit=$rc"; tail -3 "$out/r06_${tag}_parity.log" | cut -c1-300; [ "$rc" -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for c in ${CONFIGS:-pythia-12b gpt-neoxt-20b}; do
    for v in ${VARIANTS:-prev product}; do
      lib=""; [ "$v" != product ] && lib=$root/vsim_amd/_build/var/$v.so
      env VSIM_LIB=$lib timeout -k 10 300 python3 "$root/bench.py" --config "$c" --steps ${STEPS:-120} --no-cpu-baseline \
        --no-pipeline-20b --no-fast --no-other-configs --no-prefill-companion > "$out/r06_${tag}_${c}_${v}_${rep}.log" 2>&1
      rc=$?; [ "$rc" -ne 0 ] && { echo "[bench $c $v] exit=$rc"; tail -5 "$out/r06_${tag}_${c}_${v}_${rep}.log"; exit $rc; }
      python3 - "$out/r06_${tag}_${c}_${v}_${rep}.log" "$c $v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk = {k["kernel"].split(" (")[0] + (" lm" if "lm_head" in k["kernel"] else ""): k["avg_us"] for k in d["roofline"]["per_kernel"]}
print(f"{sys.argv[2]:26s} {d['value']:.1f} tok/s {d['ms_per_step']:.4f} ms", pk)
PY
    done
  done
done
exit 0
