// vlc_count.h -- the coded bits of one 8x8 block's levels, for the encoders'
// vlc_bits output (k_block.hip) and the entropy coder's count pass
// (p64vlc.hip): EncodeAC / CBPEncodeAC codec.c:96-205 incl. EOB, and an intra
// block's 8-bit DC (EncodeDC codec.c:343).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace p64k {

// Code lengths by (run, |level|), escapes folded in: byte
// min(run, 27) * 17 + min(|level|, 16) = the TCOEFF code length + 1 (sign)
// for runs < 27 and levels < 16 that have a code, else 20 (ESCAPE 6 + run 6 +
// level 8).  Built on the host from the entropy coder's own tables
// (p64gpu_vlc_len_table_, p64vlc.hip); FIRST01 (2 bits with its sign) and EOB
// (2) are constants there, checked against the tables.
constexpr int VLC_LEN_RUNS = 28, VLC_LEN_LEVELS = 17, VLC_LEN_WORDS = (VLC_LEN_RUNS * VLC_LEN_LEVELS + 3) / 4;
struct VlcLenTab {
  uint32_t w[VLC_LEN_WORDS];  // 476 bytes
};

// the positions holding a nonzero level of one zigzag level pair as mask
// bits (lo, hi): v_pk_min_u16 against 1 (a nonzero int16 is >= 1 as u16;
// the inline constant's high half taken from its low half) and v_dot2
// (lo + 2 hi)
__device__ __forceinline__ uint32_t nz2(uint32_t pair) {
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(r) : "v"(pair));
  typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, r), (u16x2_t){1, 2}, 0u, false);
}

// bits of one transmitted block from its 64 levels in scan order (lvs)
// and its nonzero positions (m0: 0..31, m1: 32..63).  cbpt: a type with CBP
// (the first coefficient may take FIRST01, no DC of its own); else an intra
// block (its DC as 8 bits, the AC codes from position 1).  The loop visits
// the nonzero positions only, two per step and without branches: both
// levels and both lengths are read together, so each step waits for two
// LDS round trips, not four.
template <typename L>  // int16 levels, or an int8 copy of levels that fit it
__device__ __forceinline__ int block_vlc_bits(const uint8_t *len, const L *lvs, uint32_t m0, uint32_t m1, bool cbpt) {
  int bits = cbpt ? 2 : 10;  // EOB (+ the intra DC)
  if (!cbpt) m0 &= ~1u;
  uint64_t m = ((uint64_t)m1 << 32) | m0;
  int last = cbpt ? -1 : 0;
  bool first = cbpt;
  while (m) {
    // (cttz of a nonzero 64-bit value: two v_ffbl + v_min, no branch; of
    // zero it is never used)
    const int p1 = (int)__builtin_ctzll(m);
    m &= m - 1u;
    const bool two = m != 0;
    const int p2 = two ? (int)__builtin_ctzll(m | (1ull << 63)) : p1;
    m &= m - 1u;
    const int l1 = lvs[p1], l2 = lvs[p2];
    const int a1 = l1 < 0 ? -l1 : l1, a2 = l2 < 0 ? -l2 : l2;
    const int r1 = p1 - last - 1, r2 = p2 - p1 - 1;
    last = p2;
    const int n1 = len[__mul24(min(r1, VLC_LEN_RUNS - 1), VLC_LEN_LEVELS) + min(a1, VLC_LEN_LEVELS - 1)];
    const int n2 = len[__mul24(min(r2, VLC_LEN_RUNS - 1), VLC_LEN_LEVELS) + min(a2, VLC_LEN_LEVELS - 1)];
    bits += ((first && r1 == 0 && a1 == 1) ? 2 : n1) + (two ? n2 : 0);
    first = false;
  }
  return bits;
}

// the table into a wave's LDS copy
__device__ __forceinline__ void load_vlc_len(const VlcLenTab &vt, uint32_t *dst, int lane) {
  dst[lane] = vt.w[lane];
  if (lane < VLC_LEN_WORDS - 64) dst[lane + 64] = vt.w[lane + 64];
}
// the same from the device copy (p64gpu_vlc_len_dev_: the table is not a
// kernel argument)
__device__ __forceinline__ void load_vlc_len(const uint32_t *vt, uint32_t *dst, int lane) {
  dst[lane] = vt[lane];
  if (lane < VLC_LEN_WORDS - 64) dst[lane + 64] = vt[lane + 64];
}

}  // namespace p64k
