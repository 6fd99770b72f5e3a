#!/bin/bash
# tools/build_variant.sh NAME FILE 'SED-EXPR' [FILE 'SED-EXPR' ...] — an A/B build of the library:
# copies vsim_amd/ to a scratch tree, applies each sed expression to its csrc file (an expression
# '@REV' instead replaces the file by its version at git revision REV, '=PATH' by the file at
# PATH), builds it and
# installs vsim_amd/_build/var/NAME.so (gitignored; it travels to the GPU box, where
# VSIM_LIB=vsim_amd/_build/var/NAME.so selects it).  The product sources are not touched.
set -eu
root=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
tmp=$(mktemp -d /tmp/vsim_var.XXXXXX)
cp -r "$root/vsim_amd" "$tmp/vsim_amd"
ln -s "$root/include" "$tmp/include"
rm -rf "$tmp/vsim_amd/_build"
while [ $# -ge 2 ]; do
  f=csrc/$1; [ -f "$tmp/vsim_amd/$1" ] && f=$1  # (vsim_amd/Makefile and the like by their own name)
  case $2 in
    @*) git -C "$root" show "${2#@}:vsim_amd/$f" > "$tmp/vsim_amd/$f" ;;
    =*) cp "${2#=}" "$tmp/vsim_amd/$f" ;;
    *) sed -i -e "$2" "$tmp/vsim_amd/$f" ;;
  esac
  grep -q . "$tmp/vsim_amd/$f"
  shift 2
done
make -C "$tmp/vsim_amd" -j8 _build/libvsim_hip.so > "$tmp/build.log" 2>&1 || { tail -20 "$tmp/build.log"; exit 1; }
mkdir -p "$root/vsim_amd/_build/var"
cp "$tmp/vsim_amd/_build/libvsim_hip.so" "$root/vsim_amd/_build/var/$name.so"
rm -rf "$tmp"
echo "built vsim_amd/_build/var/$name.so"
