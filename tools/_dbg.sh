set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in vsim_amd/_build/libvsim_hip.so vsim_amd/_build/var/u8o2.so vsim_amd/_build/var/u4o3.so vsim_amd/_build/var/u8o3.so vsim_amd/_build/libvsim_hip.so; do echo "== $lib"; VSIM_LIB=$lib timeout -k 10 300 python3 bench.py --mode fast --no-cpu-baseline --no-profile 2>&1 | tail -1 | cut -c90-150 || exit 1; done
