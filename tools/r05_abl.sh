#!/bin/bash
# r05: timing-only ablations of the barrier-free fc_out tiles (VSIM_TAIL_NB=1): variant builds
# vsim_amd/_build/var/abl_<name>.so given as arguments ("product" = the product library)
set -u
root=$(cd "$(dirname "$0")/.." && pwd); out=$root/gpurun_out; mkdir -p "$out"; cd /tmp && export TMPDIR=/tmp
tag=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    lib=$root/vsim_amd/_build/var/abl_$v.so; [ "$v" = product ] && lib=$root/vsim_amd/_build/libvsim_hip.so
    nb=1; [ "$v" = base ] && { nb=0; lib=$root/vsim_amd/_build/libvsim_hip.so; }
    VSIM_LIB=$lib VSIM_TAIL_NB=$nb timeout -k 10 200 python3 "$root/bench.py" --no-cpu-baseline --no-pipeline-20b \
      --no-fast --no-other-configs > "$out/r05_${tag}_${v}_${rep}.log" 2>&1
    rc=$?; [ "$rc" -ne 0 ] && { echo "[$v] exit=$rc"; tail -5 "$out/r05_${tag}_${v}_${rep}.log"; exit $rc; }
    python3 - "$out/r05_${tag}_${v}_${rep}.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk = {k["kernel"].split(" (")[0] + (" lm" if "lm_head" in k["kernel"] else ""): k["avg_us"] for k in d["roofline"]["per_kernel"]}
print(f"{sys.argv[2]:<10} {d['value']:.1f} tok/s", pk)
PY
  done
done
exit 0
