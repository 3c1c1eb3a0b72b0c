#!/bin/bash
# Build a variant of p64_amd/libp64gpu.so into abtest/ (development aid):
#   tools/ablib.sh <name> [<p64gpu.hip source>] [-- extra hipcc flags]
# The other objects come from the current tree's build.
set -e
name=$1; shift
src=p64_amd/csrc/p64gpu.hip
if [ $# -gt 0 ] && [ "$1" != "--" ]; then src=$1; shift; fi
[ "$1" = "--" ] && shift
mkdir -p abtest
cp "$src" p64_amd/csrc/_ab_tmp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" \
  -c p64_amd/csrc/_ab_tmp.hip -o abtest/$name.o
rm -f p64_amd/csrc/_ab_tmp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o abtest/lib_$name.so abtest/$name.o \
  p64_amd/csrc/synth.o p64_amd/csrc/p64stream.o p64_amd/csrc/p64seq.o p64_amd/csrc/p64prog.o p64_amd/csrc/p64vlc.o
rm -f abtest/$name.o
echo abtest/lib_$name.so
