#!/bin/bash
# Build a variant of p64_amd/libp64gpu.so into abtest/ (development aid):
#   tools/ablib.sh <name> <variant.hip> <replaces> [-- extra hipcc flags]
# <replaces> is the kernel unit the variant stands in for (k_search, k_block,
# k_aux or p64gpu_abi); every other object comes from the current tree's build.
# The variant is compiled next to the real sources so its includes resolve.
set -e
name=$1 src=$2 rep=$3; shift 3
[ "$1" = "--" ] && shift
mkdir -p abtest
cp "$src" p64_amd/csrc/_ab_tmp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" \
  -c p64_amd/csrc/_ab_tmp.hip -o abtest/$name.o
rm -f p64_amd/csrc/_ab_tmp.hip
objs=""
for u in k_search k_block k_aux p64gpu_abi; do
  [ "$u" = "$rep" ] && objs="$objs abtest/$name.o" || objs="$objs p64_amd/csrc/$u.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o abtest/lib_$name.so $objs \
  p64_amd/csrc/synth.o p64_amd/csrc/p64stream.o p64_amd/csrc/p64seq.o p64_amd/csrc/p64prog.o p64_amd/csrc/p64vlc.o
rm -f abtest/$name.o
echo abtest/lib_$name.so
