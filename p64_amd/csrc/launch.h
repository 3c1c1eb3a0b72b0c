// launch.h -- host-side launchers of the kernel families, one per kernel
// translation unit, called by the C ABI (p64gpu_abi.hip).  Shapes and
// pointers are validated by the caller (check_geometry, alignment, the 2 GiB
// launch split); a launcher only computes its grid and launches.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/p64gpu.h"

namespace p64k {

// k_search.hip -- one wavefront per macroblock.  mode: 0 intra picture,
// 1 TSS, 2 FULL.  grid = macroblocks (or mb_list entries when mb_list != NULL).
hipError_t encode_fused(int mode, unsigned grid, const p64gpu_encode_args &a, const int32_t *mb_list,
                        hipStream_t st);
// ME records of every macroblock of nframes luma planes (mode 1 TSS, 2 FULL)
hipError_t motion(int mode, int w, int h, int nframes, int64_t stride, const uint8_t *ref_y,
                  const uint8_t *cur_y, int sl, p64_me_rec *out, bool stats, hipStream_t st);

// k_block.hip -- one lane per 8x8 block, 10 macroblocks per wave.  Every
// buffer of one launch lies within 2 GiB (32-bit buffer offsets).
// vlc_len: VLC_LEN_WORDS dwords, the code-length table of
// p64gpu_vlc_len_table_ (vlc_count.h; read only when a.vlc_bits is given)
hipError_t intra_mbg(const p64gpu_encode_args &a, const uint32_t *vlc_len, hipStream_t st);
hipError_t inter_mbg(const p64gpu_encode_args &a, p64_me_rec *me, const uint32_t *vlc_len, hipStream_t st);
hipError_t recon_mbg(int w, int h, int nframes, int64_t stride, const uint8_t *ref, uint8_t *recon,
                     const int16_t *coef, const p64_mb_rec *mb, const uint8_t *quant_mb,
                     const uint8_t *coded_mask, hipStream_t st);
hipError_t recon_pk(int w, int h, int nframes, int64_t stride, const uint8_t *ref, uint8_t *recon,
                    const int16_t *levels, uint32_t nlev, const uint32_t *index, const p64_mb_rec *mb,
                    const uint8_t *quant_mb, const uint8_t *coded_mask, hipStream_t st);

// k_aux.hip -- reference block routines one thread per block; synthetic input;
// the clock probe
hipError_t block_op(int op, const int32_t *in, int32_t *out, int64_t nblocks, int dcq, int acq,
                    hipStream_t st);
hipError_t synth(int content, int w, int h, uint32_t seed0, int nseeds, int frame0, int nslots, int64_t stride,
                 uint8_t *out, hipStream_t st);
// clock probe: clock_waves() waves (8 per SIMD), each spinning `ticks` of the
// 100 MHz counter; out [clock_waves()][2] = (shader ticks, real-time ticks)
unsigned clock_waves();
hipError_t clock(uint32_t ticks, uint32_t *out, hipStream_t st);

}  // namespace p64k
