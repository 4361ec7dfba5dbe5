#!/bin/bash
# Build an A/B variant of the native library: this tree with some files taken from another
# commit, linked as kvedge_amd/<name> (load it with KVEDGE_LIB=<name>).
#   bash tools/ab_build.sh _C_ab.so <commit> csrc/kernels/stem12.hip [more files...]
set -e
name=$1; rev=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
work=/tmp/kv_ab_tree
rm -rf "$work"; mkdir -p "$work"
tar -C "$root" --exclude=./.git --exclude=./build --exclude=./gpurun_out --exclude='*.so' -cf - . | tar -C "$work" -xf -
for f in "$@"; do git -C "$root" show "$rev:$f" > "$work/$f"; done
(cd "$work" && python -m kvedge_amd._build > /tmp/kv_ab_build.log 2>&1)
cp "$work/kvedge_amd/_C.so" "$root/kvedge_amd/$name"
echo "built kvedge_amd/$name ($rev: $*)"
