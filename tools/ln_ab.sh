# k_ln_quant shape A/B: the default bench's per-kernel event timing for each variant library
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
mkdir -p $o
for v in default t1024s8 t256s8 t512s16 t512s4 t1024s16; do
  lib=$GRAFT_REPO_ROOT/vsim_amd/_build/var/$v.so
  [ $v = default ] && lib=$GRAFT_REPO_ROOT/vsim_amd/_build/libvsim_hip.so
  VSIM_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-fast --steps 128 > $o/ln_$v.log 2>&1 || { tail -3 $o/ln_$v.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$o/ln_$v.log').read().strip().splitlines()[-1])
k={x['kernel']:x['avg_us'] for x in d['roofline']['per_kernel']}
print('$v', d['value'], k.get('k_ln_quant'))"
done
