#!/bin/bash
# tools/variant.sh NAME SRC "FLAGS" [ALT] — an A/B build of the library with one source
# compiled with extra flags (or replaced by the file ALT): vsim_amd/_build/var/NAME.so (select
# with VSIM_LIB=... for a run).
set -e
cd "$(dirname "$0")/../vsim_amd"
name=$1; src=$2; flags=$3; alt=${4:-csrc/$2}
mkdir -p _build/var
objs=""
extra=""
case $(basename $src) in gemm_f16.hip|gemv_chain.hip) extra=-fno-slp-vectorize;; esac  # (the Makefile's per-file flags)
for o in _build/*.o; do
  b=$(basename $o .o)
  if [ "$b" = "$(basename $src)" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include $extra $flags -c $alt -o _build/var/$name.o
    objs="$objs _build/var/$name.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _build/var/$name.so $objs
echo "built _build/var/$name.so"
