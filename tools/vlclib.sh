#!/bin/bash
# Build a variant of the library with p64vlc.hip compiled under extra flags
# into abtest/ (development aid): tools/vlclib.sh <name> [hipcc flags...]
set -e
name=$1; shift
mkdir -p abtest
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" \
  -c p64_amd/csrc/p64vlc.hip -o abtest/$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o abtest/lib_$name.so p64_amd/csrc/k_search.o \
  p64_amd/csrc/k_block.o p64_amd/csrc/k_aux.o p64_amd/csrc/p64gpu_abi.o p64_amd/csrc/synth.o \
  p64_amd/csrc/p64stream.o p64_amd/csrc/p64seq.o p64_amd/csrc/p64prog.o abtest/$name.o
rm -f abtest/$name.o
echo abtest/lib_$name.so
