# Top-level build.  `make` builds the product library and the CPU oracle;
# `make ref` additionally builds the reference harness from /root/reference
# (test infrastructure, see oracle/Makefile).
#
#   p64_amd/libp64gpu.so   HIP kernels (gfx950) + C ABI (include/p64gpu.h)
#   p64_amd/p64gpu_enc     C host encoder driver over the C ABI
#   oracle/liboracle.so    CPU restatement used as the parity checker

HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
CXX     ?= g++
ARCH    ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
LIB     := p64_amd/libp64gpu.so

all: $(LIB) p64_amd/p64gpu oracle

p64_amd/csrc/synth.o: p64_amd/csrc/synth.c include/p64gpu.h
	$(CC) -O2 -fPIC -Wall -c $< -o $@

KERNEL_DEPS := include/p64gpu.h p64_amd/csrc/common.h p64_amd/csrc/launch.h
GPU_OBJS := p64_amd/csrc/k_search.o p64_amd/csrc/k_block.o p64_amd/csrc/k_aux.o p64_amd/csrc/p64gpu_abi.o

p64_amd/csrc/k_aux.o: p64_amd/csrc/k_aux.hip $(KERNEL_DEPS) p64_amd/csrc/synth_impl.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

p64_amd/csrc/%.o: p64_amd/csrc/%.hip $(KERNEL_DEPS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

p64_amd/csrc/p64stream.o: p64_amd/csrc/p64stream.c include/p64stream.h include/p64gpu.h
	$(CC) -O2 -fPIC -Wall -Wextra -c $< -o $@

p64_amd/csrc/p64seq.o: p64_amd/csrc/p64seq.c include/p64seq.h include/p64stream.h include/p64gpu.h \
                       include/p64prog.h
	$(CC) -O2 -fPIC -Wall -Wextra -c $< -o $@

p64_amd/csrc/p64prog.o: p64_amd/csrc/p64prog.c include/p64prog.h include/p64gpu.h
	$(CC) -O2 -fPIC -Wall -Wextra -c $< -o $@

p64_amd/csrc/p64vlc.o: p64_amd/csrc/p64vlc.hip include/p64gpu.h include/p64stream.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(GPU_OBJS) p64_amd/csrc/synth.o p64_amd/csrc/p64stream.o p64_amd/csrc/p64seq.o \
        p64_amd/csrc/p64prog.o p64_amd/csrc/p64vlc.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^

p64_amd/p64gpu: p64_amd/host/p64gpu_cli.c $(LIB) include/p64gpu.h include/p64stream.h include/p64seq.h
	$(CC) -O2 -Wall -Wextra -o $@ $< -Lp64_amd -lp64gpu -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

# ISA listing of the kernels for inspection (not part of the build)
asm: p64_amd/csrc/k_search.hip p64_amd/csrc/k_block.hip
	mkdir -p build
	for k in k_search k_block; do \
	  $(HIPCC) $(HIPFLAGS) -S --cuda-device-only -o build/$$k.s p64_amd/csrc/$$k.hip || exit 1; done

clean:
	rm -f p64_amd/csrc/*.o $(LIB) p64_amd/p64gpu_enc
	$(MAKE) -C oracle clean

.PHONY: all oracle ref asm clean

# bounds-checked entropy coder (diagnostic aid, tools/vlc_fault_probe.py):
# the same library with k_vlc_blk's stores range-tested (P64_VLC_CHECK)
vlccheck: abtest/lib_vlccheck.so
abtest/lib_vlccheck.so: p64_amd/csrc/p64vlc.hip $(GPU_OBJS) p64_amd/csrc/synth.o p64_amd/csrc/p64stream.o \
                        p64_amd/csrc/p64seq.o p64_amd/csrc/p64prog.o
	mkdir -p abtest
	$(HIPCC) $(HIPFLAGS) -DP64_VLC_CHECK -c $< -o abtest/p64vlc_check.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(GPU_OBJS) p64_amd/csrc/synth.o p64_amd/csrc/p64stream.o \
	  p64_amd/csrc/p64seq.o p64_amd/csrc/p64prog.o abtest/p64vlc_check.o

# the same checked build with the round-5 status memset (hipMemsetAsync) instead
# of the zeroing kernel: the A/B of tools/vlc_fault_probe.py stage E
vlcmemset: abtest/lib_vlcmemset.so
abtest/lib_vlcmemset.so: p64_amd/csrc/p64vlc.hip $(GPU_OBJS) p64_amd/csrc/synth.o p64_amd/csrc/p64stream.o \
                         p64_amd/csrc/p64seq.o p64_amd/csrc/p64prog.o
	mkdir -p abtest
	$(HIPCC) $(HIPFLAGS) -DP64_VLC_CHECK -DVLC_STATUS_MEMSET -c $< -o abtest/p64vlc_memset.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(GPU_OBJS) p64_amd/csrc/synth.o p64_amd/csrc/p64stream.o \
	  p64_amd/csrc/p64seq.o p64_amd/csrc/p64prog.o abtest/p64vlc_memset.o
