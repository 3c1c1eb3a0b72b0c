// k_block.hip -- the block-layout kernels: one LANE per 8x8 block, the whole
// block in registers, a wave = 10 consecutive macroblocks (lane 6m + b).
//
//   k_intra_mbg  intra pictures: ChenDct, CCITTFlatQuantize, zigzag, ICCITT-
//                FlatQuantize, ChenIDct, reconstruction (p64.c:823-1013)
//   k_inter_mbg  inter pictures after k_motion: MTYPE decision from the ME
//                record, prediction + loop filter (io.c:142-496), residual
//                ChenDct, quantisers, CBP (p64.c:887-908), IQ/IDCT, recon
//   k_recon_mbg  decoder reconstruction (DecompressMDU p64.c:1179 +
//                DecodeSaveMDU p64.c:971)
//
// No LDS exchange between the transform passes; levels leave through a
// per-wave LDS staging area as whole 1-KB stores; every load and store is a
// buffer access whose out-of-range offset replaces a branch.

#include <type_traits>

#include "common.h"
#include "launch.h"
#include "quant_int.h"
#include "vlc_count.h"

namespace {

// ---------------------------------------------------------------------------
// Block layout: one LANE per 8x8 block, the whole block in 64 VGPRs.  For the
// two HBM-bound paths (intra pictures, decoder reconstruction) this removes
// every lane exchange: the Chen column and row passes, the zigzag (a register
// renaming) and the quantisers run in registers, with no LDS and no barrier,
// and no lane idles (the row layout of k_encode leaves 16 of 64 lanes idle).
// Thread t of a launch maps to picture t / (6 nmb) and, inside the picture,
// first the luma blocks in raster order of the 8x8 block grid, then the U and
// the V blocks in raster order: a wave's 64 lanes read and write 64 adjacent
// 8-byte row segments (512 contiguous bytes per row instruction), and each
// lane writes its block's 128 bytes of levels as whole cache lines.

constexpr ZigZag k_zz = make_zigzag();  // compile-time copy for register renaming
typedef short s16x2 __attribute__((ext_vector_type(2)));  // an int16 pair in one VGPR

// The forward quantiser from the raw row-pass output (quant_int.h: final /8,
// BoundDct, CCITT(Flat)Quantize, bound, as one clamp, one 24-bit multiply-add
// and one shift; tests/test_quant_int.py checks every q and value).  The
// binary32 form it replaces (quantise in common.h) spent two conversions per
// coefficient.
struct QIntTab {
  p64_qint ac[32], dc[32];  // AC (intra and inter), inter DC; by q
};
constexpr QIntTab make_qint_tab() {
  QIntTab t{};
  for (int q = 1; q < 32; q++) {
    t.ac[q] = p64_qint_make(q, 0);
    t.dc[q] = p64_qint_make(q, 1);
  }
  return t;
}
__constant__ QIntTab c_qint = make_qint_tab();
// The quantiser on an int16 pair when D = 16q is a power of two (q = 1, 2, 4,
// 8, 16: the table's multiplier is 1, level = (vc + C) >> s): clamp (two
// v_pk min/max against per-half bounds), the sign-selected addend by v_bfi
// under v_pk_ashrrev 15, v_pk_add, v_pk_ashrrev s -- four to six
// instructions per two levels instead of four to five per level.
template <bool CLAMP>
__device__ __forceinline__ uint32_t qlevel_pk2(uint32_t x, uint32_t lo2, uint32_t hi2, uint32_t cp2, uint32_t cn2,
                                               int s) {
  if (CLAMP) {
    asm("v_pk_min_i16 %0, %1, %2" : "=v"(x) : "v"(x), "v"(hi2));
    asm("v_pk_max_i16 %0, %1, %2" : "=v"(x) : "v"(x), "v"(lo2));
  }
  const s16x2 v = __builtin_bit_cast(s16x2, x);
  const uint32_t m = __builtin_bit_cast(uint32_t, (s16x2)(v >> (s16x2){15, 15}));
  uint32_t c;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(c) : "v"(m), "v"(cn2), "v"(cp2));
  const s16x2 r = (s16x2)(v + __builtin_bit_cast(s16x2, c)) >> (s16x2){(short)s, (short)s};
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t pk16u(int lo, int hi) { return (uint32_t)(lo & 0xffff) | ((uint32_t)hi << 16); }
// CLAMP false: the caller knows |v| <= t.vhi (tests/test_intra_dct_bound.py)
template <bool CLAMP = true>
__device__ __forceinline__ int qlevel_int(int v, const p64_qint &t) {
  // the clamp as one v_med3_i32 (4 clocks; hipcc's v_max + v_min are 4 each;
  // intra 42.0 -> 41.1 us A/B x2)
  int vc = v;
  if (CLAMP) asm("v_med3_i32 %0, %1, %2, %3" : "=v"(vc) : "v"(v), "v"(t.vlo), "v"(t.vhi));
  return (__mul24(vc, t.m) + (vc < 0 ? t.cn : t.cp)) >> t.s;
}

// keeps the machine scheduler from interleaving the 8 lines of a pass (it
// would trade registers for ILP the block layout does not need: other waves
// hide latency)
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
// orders a wave's LDS accesses across a lane exchange at the IR level (a
// wave's LDS operations complete in order; the fence only stops the compiler
// from moving them across the exchange)
#define WAVE_FENCE() __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront")

// A wave issues its loads at raised priority, so a freshly launched wave gets
// its requests out ahead of the older waves' arithmetic
#define PRIO_HIGH() __builtin_amdgcn_s_setprio(3)
#define PRIO_LOW() __builtin_amdgcn_s_setprio(0)

struct BlkPos {
  int fi;     // picture in the launch
  int mb;     // raster macroblock
  int b;      // block c = 0..5 of the MB (p64.c:77-79)
  int plane;  // 0 Y, 1 U, 2 V
  int x, y;   // block origin in its plane
};
// MB-grouped block layout: wave w takes macroblocks 10w .. 10w+9 of the
// launch, lane 6m + b block b of its m-th MB (lanes 60..63 repeat lane 59).
// A wave's levels are then 7,680 contiguous bytes and its pixel rows and
// records contiguous runs per plane: its HBM traffic is a few long runs
// instead of 64 blocks scattered over a block row.  (MBS_PER_WAVE: common.h)
// Workgroups map to MB runs XCD-aware (xcd_remap): neighbouring groups share
// the 128-B lines at their edges, and the groups of one XCD (one L2) take one
// contiguous run, so a shared line is fetched once per XCD rather than per
// group (intra/inter/decode launches 0.3-0.6 us faster, tools/trace_libs.sh).
__device__ __forceinline__ BlkPos blk_pos_mb(unsigned gmb, int b, int w, int h, const BlkDiv &k) {
  const int mbw = w >> 4;
  BlkPos p;
  p.fi = (int)mdiv(gmb, k.mn, k.sn);
  p.mb = (int)(gmb - (unsigned)p.fi * (unsigned)(mbw * (h >> 4)));
  const int mby = (int)mdiv((unsigned)p.mb, k.mw, k.sw), mbx = p.mb - mby * mbw;
  p.b = b;
  p.plane = b < 4 ? 0 : b - 3;
  p.x = b < 4 ? 16 * mbx + 8 * (b & 1) : 8 * mbx;
  p.y = b < 4 ? 16 * mby + 8 * (b >> 1) : 8 * mby;
  return p;
}
// ChenDct (chendct.c:97-206) on a register block given as its 8 packed pixel
// rows (or the residual rows - prow), both passes in packed 16-bit
// arithmetic: the column pass (fwd_col_pk, below) leaves each row as four (column 2j, 2j+1) int16 pairs -- its
// outputs stay within +-5,800 for pixel or +-255 residual input -- and the
// row pass runs the butterfly of fwd8 on pairs: v_pk_add/sub/ashr for the
// sums, and every product pair C_a x + C_b y as ONE v_dot2_i32_i16 with the
// constant pair as its literal (the two products and their sum exact in
// 32 bits, the same ms9 rounding after).  Row-pass intermediates stay below
// 2^15: sums <= 11,600, u = d + r <= 14,000.  Half the registers of the
// scalar form between the passes.
__device__ __forceinline__ s16x2 pk16(int lo, int hi) {  // two values that fit int16
  return __builtin_bit_cast(s16x2, (uint32_t)(lo & 0xffff) | ((uint32_t)hi << 16));
}
__device__ __forceinline__ int dot2(s16x2 a, short ca, short cb) {
  // VOP3P with the constant pair in an SGPR and an inline-0 accumulator: the
  // builtin becomes v_mov 0 + v_dot2c (6 clocks per wave instead of 4)
  const uint32_t c = (uint32_t)(uint16_t)ca | ((uint32_t)(uint16_t)cb << 16);
  int r;
  asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "s"(c));
  return r;
}
// the same with a VGPR accumulator (acc + C_a x + C_b y in one instruction)
__device__ __forceinline__ int dot2acc(s16x2 a, short ca, short cb, int acc) {
  const uint32_t c = (uint32_t)(uint16_t)ca | ((uint32_t)(uint16_t)cb << 16);
  int r;
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(c), "v"(acc));
  return r;
}
// (ms9(A), ms9(B)) as one int16 pair when A = 2a, B = 2b are given with halved
// constants: floor(a / 512) = floor(A / 256) = A >> 8, whose low 16 bits are
// bytes 1 and 2 of A -- one v_perm instead of two shifts and a v_bfi.  The
// constants of the forward column pass (4 C_k; the odd part's C_k1D16..C7D16,
// all even) and C1D4 halve exactly, so the halved products are the same
// rationals.
__device__ __forceinline__ s16x2 pk_ms8(int A, int B) {
  return __builtin_bit_cast(s16x2, __builtin_amdgcn_perm((uint32_t)B, (uint32_t)A, 0x06050201u));
}
static_assert(C1D4 % 2 == 0 && C1D16 % 2 == 0 && C3D16 % 2 == 0 && C5D16 % 2 == 0 && C7D16 % 2 == 0,
              "halved constants");
// row pass of one row given as (x0,x1), (x2,x3), (x4,x5), (x6,x7)
__device__ __forceinline__ void fwd_row_pk(const s16x2 p[4], int o[8]) {
  const s16x2 s01 = (p[0] + p[3].yx) >> 1, s23 = (p[1] + p[2].yx) >> 1;  // (s0,s1) (s2,s3)
  const s16x2 d01 = (p[0] - p[3].yx) >> 1, d23 = (p[1] - p[2].yx) >> 1;  // (d0,d1) (d2,d3)
  const s16x2 e01 = s01 + s23.yx, e32 = s01 - s23.yx;                    // (e0,e1) (e3,e2)
  o[0] = ms9(dot2(e01, C1D4, C1D4));
  o[4] = ms9(dot2(e01, C1D4, -C1D4));
  o[2] = ms9(dot2(e32, C1D8, C3D8));   // C3D8 e2 + C1D8 e3
  o[6] = ms9(dot2(e32, C3D8, -C1D8));  // C3D8 e3 - C1D8 e2
  const s16x2 q = __builtin_shufflevector(d01, d23, 1, 2);   // (d1, d2)
  const s16x2 dd = __builtin_shufflevector(d23, d01, 1, 2);  // (d3, d0)
  const s16x2 rr = pk_ms8(dot2(q, C1D4 / 2, -C1D4 / 2), dot2(q, C1D4 / 2, C1D4 / 2));  // (r0, r1)
  const s16x2 u03 = dd + rr, u12 = dd - rr;                   // (u0,u3) (u1,u2)
  o[1] = ms9(dot2(u03, C7D16, C1D16));
  o[7] = ms9(dot2(u03, -C1D16, C7D16));
  o[3] = ms9(dot2(u12, -C5D16, C3D16));
  o[5] = ms9(dot2(u12, C3D16, C5D16));
}
// column pass of one column given as its packed row pairs (x0,x1), (x2,x3),
// (x4,x5), (x6,x7): fwd8<N, 4> (chendct.c:120-159) with the pairs of butterfly
// terms packed the way fwd_row_pk packs them -- no >>1, the <<2 input scale
// folded into the dot-product constants (<= 4 x 502 = 2,008, int16) except
// for d0, d3, which are added to products and shift themselves.  Pixel or
// residual input (|x| <= 255): sums <= 1,020, u = 4d + r <= 2,462, every
// intermediate inside int16; the products and their sums exact in 32 bits.
// The same row pass with its outputs as natural int16 pairs (o0,o1) (o2,o3)
// (o4,o5) (o6,o7) (|o| <= 8,187 x ... < 2^15 for 8-bit input, BoundDct's
// range): pk_ms8 for the pairs whose constants halve, one shift for o2 and o6
// (C1D8 is odd) joined to the halved o3 / o7 by one v_perm.
__device__ __forceinline__ void fwd_row_pk2(const s16x2 p[4], uint32_t P[4]) {
  const s16x2 s01 = (p[0] + p[3].yx) >> 1, s23 = (p[1] + p[2].yx) >> 1;
  const s16x2 d01 = (p[0] - p[3].yx) >> 1, d23 = (p[1] - p[2].yx) >> 1;
  const s16x2 e01 = s01 + s23.yx, e32 = s01 - s23.yx;
  const int A0 = dot2(e01, C1D4 / 2, C1D4 / 2), A4 = dot2(e01, C1D4 / 2, -C1D4 / 2);
  const int o2 = ms9(dot2(e32, C1D8, C3D8)), o6 = ms9(dot2(e32, C3D8, -C1D8));
  const s16x2 q = __builtin_shufflevector(d01, d23, 1, 2);
  const s16x2 dd = __builtin_shufflevector(d23, d01, 1, 2);
  const s16x2 rr = pk_ms8(dot2(q, C1D4 / 2, -C1D4 / 2), dot2(q, C1D4 / 2, C1D4 / 2));
  const s16x2 u03 = dd + rr, u12 = dd - rr;
  const int A1 = dot2(u03, C7D16 / 2, C1D16 / 2), A7 = dot2(u03, -C1D16 / 2, C7D16 / 2);
  const int A3 = dot2(u12, -C5D16 / 2, C3D16 / 2), A5 = dot2(u12, C3D16 / 2, C5D16 / 2);
  P[0] = __builtin_bit_cast(uint32_t, pk_ms8(A0, A1));
  P[2] = __builtin_bit_cast(uint32_t, pk_ms8(A4, A5));
  P[1] = __builtin_amdgcn_perm((uint32_t)A3, (uint32_t)o2, 0x06050100u);
  P[3] = __builtin_amdgcn_perm((uint32_t)A7, (uint32_t)o6, 0x06050100u);
}
// The outputs are left as 2 x the pre-shift sums (halved constants, A above):
// the caller packs two columns' outputs with pk_ms8.
__device__ __forceinline__ void fwd_col_pk(const s16x2 p[4], int o[8]) {
  const s16x2 s01 = p[0] + p[3].yx, s23 = p[1] + p[2].yx;  // (s0,s1) (s2,s3)
  const s16x2 d01 = p[0] - p[3].yx, d23 = p[1] - p[2].yx;  // (d0,d1) (d2,d3)
  const s16x2 e01 = s01 + s23.yx, e32 = s01 - s23.yx;      // (e0,e1) (e3,e2)
  o[0] = dot2(e01, 2 * C1D4, 2 * C1D4);
  o[4] = dot2(e01, 2 * C1D4, -2 * C1D4);
  o[2] = dot2(e32, 2 * C1D8, 2 * C3D8);   // (4 C3D8 e2 + 4 C1D8 e3) / 2
  o[6] = dot2(e32, 2 * C3D8, -2 * C1D8);  // (4 C3D8 e3 - 4 C1D8 e2) / 2
  const s16x2 q = __builtin_shufflevector(d01, d23, 1, 2);  // (d1, d2)
  const s16x2 rr = pk_ms8(dot2(q, 2 * C1D4, -2 * C1D4), dot2(q, 2 * C1D4, 2 * C1D4));  // (r0, r1)
  const s16x2 dd = __builtin_shufflevector(d23, d01, 1, 2) << 2;  // (4 d3, 4 d0)
  const s16x2 u03 = dd + rr, u12 = dd - rr;  // (u0,u3) (u1,u2)
  o[1] = dot2(u03, C7D16 / 2, C1D16 / 2);
  o[7] = dot2(u03, -C1D16 / 2, C7D16 / 2);
  o[3] = dot2(u12, -C5D16 / 2, C3D16 / 2);
  o[5] = dot2(u12, C3D16 / 2, C5D16 / 2);
}
// byte b of w0 and of w1 zero-extended into the two int16 halves
__device__ __forceinline__ s16x2 byte_pair(uint32_t w1, uint32_t w0, int b) {
  return __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(w1, w0, 0x0c000c00u | ((uint32_t)(4 + b) << 16) | (uint32_t)b));
}
// (the final rounding dct_final(v) reads the sign of v = X >> 9; hipcc then
// takes it from X itself and keeps all 64 pre-shift sums alive next to the
// shifted coefficients until quantisation -- 64 extra VGPRs.  The opaque copy
// ends X's life at the shift.)
// RES: the input is the residual rows - prow (both packed pixel rows)
// column pass: p[row][column pair]
template <bool RES = false>
__device__ __forceinline__ void fdct_cols_pk(const uint2 rows[8], s16x2 p[8][4], const uint2 *prow = nullptr) {
#pragma unroll
  for (int c = 0; c < 8; c += 2) {
    s16x2 x[4], y[4];  // columns c and c + 1 as row pairs
    int o[8], u[8];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t w0 = c < 4 ? rows[2 * j].x : rows[2 * j].y, w1 = c < 4 ? rows[2 * j + 1].x : rows[2 * j + 1].y;
      x[j] = byte_pair(w1, w0, c & 3);
      y[j] = byte_pair(w1, w0, (c + 1) & 3);
      if (RES) {
        const uint32_t q0 = c < 4 ? prow[2 * j].x : prow[2 * j].y, q1 = c < 4 ? prow[2 * j + 1].x : prow[2 * j + 1].y;
        x[j] -= byte_pair(q1, q0, c & 3);
        y[j] -= byte_pair(q1, q0, (c + 1) & 3);
      }
    }
    fwd_col_pk(x, o);
    fwd_col_pk(y, u);
#pragma unroll
    for (int k = 0; k < 8; k++) p[k][c >> 1] = pk_ms8(o[k], u[k]);
    SCHED_FENCE();
  }
}
template <bool RES = false>
__device__ __forceinline__ void fdct_block_pk(const uint2 rows[8], int v[64], const uint2 *prow = nullptr) {
  s16x2 p[8][4];  // [row][column pair]
  fdct_cols_pk<RES>(rows, p, prow);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    fwd_row_pk(p[r], v + 8 * r);
#pragma unroll
    for (int k = 0; k < 8; k++) v[8 * r + k] = opaque(v[8 * r + k]);
    SCHED_FENCE();
  }
}

// 8 IDCT row outputs o (before the final rounding) -> BoundIDct(idct_final(o))
// as 8 packed bytes.  For o < 0 idct_final(o) <= 0 and (o + 8) >> 4 <= 0 alike,
// so after the clamp to 0..255 the final rounding's sign term drops out:
// clamp((o + 8) >> 4).  The clamp + pack is v_cvt_pk_i16_i32 (saturating) +
// v_sat_pk_u8_i16 per pair and one v_perm per 4 pixels (inline asm: hipcc's
// own clamp+pack fusion is the miscompiled v_ashr_pk_u8_i32 form, see pack8).
__device__ __forceinline__ uint32_t sat4(const int x[4]) {
  uint32_t p01, p23, s01, s23;
  asm("v_cvt_pk_i16_i32 %0, %1, %2" : "=v"(p01) : "v"(x[0]), "v"(x[1]));
  asm("v_cvt_pk_i16_i32 %0, %1, %2" : "=v"(p23) : "v"(x[2]), "v"(x[3]));
  asm("v_sat_pk_u8_i16 %0, %1" : "=v"(s01) : "v"(p01));
  asm("v_sat_pk_u8_i16 %0, %1" : "=v"(s23) : "v"(p23));
  return __builtin_amdgcn_perm(s23, s01, 0x05040100u);
}
// The same from o8 = o + 8 (the +8 folded into the row pass): the pairs
// saturated to int16 first (v_cvt_pk_i16_i32), then >> 4 in packed 16-bit
// arithmetic and v_sat_pk_u8_i16: 16 instructions a row instead of 26.  The
// saturation changes nothing: o8 > 32,767 gives >= 2,047 and o8 < -32,768
// gives <= -2,048 either way, both clamped to 255 / 0 after.
__device__ __forceinline__ uint32_t sat4_shr4(const int x[4]) {
  uint32_t p01, p23, s01, s23;
  asm("v_cvt_pk_i16_i32 %0, %1, %2" : "=v"(p01) : "v"(x[0]), "v"(x[1]));
  asm("v_cvt_pk_i16_i32 %0, %1, %2" : "=v"(p23) : "v"(x[2]), "v"(x[3]));
  const s16x2 h01 = __builtin_bit_cast(s16x2, p01) >> (s16x2){4, 4};
  const s16x2 h23 = __builtin_bit_cast(s16x2, p23) >> (s16x2){4, 4};
  asm("v_sat_pk_u8_i16 %0, %1" : "=v"(s01) : "v"(h01));
  asm("v_sat_pk_u8_i16 %0, %1" : "=v"(s23) : "v"(h23));
  return __builtin_amdgcn_perm(s23, s01, 0x05040100u);
}
__device__ __forceinline__ uint2 final_clamp_pack8_o8(const int o8[8]) {
  return make_uint2(sat4_shr4(o8), sat4_shr4(o8 + 4));
}
// ICCITTFlatQuantize + ChenIDct + BoundIDctMatrix of an intra block from its
// levels (natural order in v; the DC dequantised as DC x 8): the dequantiser
// runs on natural level pairs (x_k, x_k') of a column in packed 16-bit
// arithmetic (dequantise_pk; |value| <= 7,905) and the column pass takes
// every product pair C_a x_k + C_b x_k' as one v_dot2_i32_i16 on those pairs
// (the <<2 input scale folded into the constants, <= 2,008: products and sums
// exact in 32 bits); row pass and final stage as idct_block_rec
__device__ __forceinline__ uint32_t pk2(int lo, int hi) { return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u); }
// the column pass of that from natural level pairs: pair(e, e') returns the
// levels of natural positions e (low half) and e' (high half) packed; q2/qq
// packed per lane (0 for a block without coefficients); dcfix: the DC is
// the intra DC (dequantised as dc8 = DC x 8)
// ChenIDct column pass of column c from its dequantised natural pairs
// (x_c, x_4c) (x_1c, x_7c) (x_5c, x_3c) (x_2c, x_6c) -- x_rc = row r
__device__ __forceinline__ void idct_col8(uint32_t p04, uint32_t p17, uint32_t p53, uint32_t p26, int o[8]) {
  const s16x2 a04 = __builtin_bit_cast(s16x2, p04), a17 = __builtin_bit_cast(s16x2, p17);
  const s16x2 a53 = __builtin_bit_cast(s16x2, p53), a26 = __builtin_bit_cast(s16x2, p26);
  const int p0 = ms9(dot2(a17, 4 * C7D16, -4 * C1D16)), p3 = ms9(dot2(a17, 4 * C1D16, 4 * C7D16));
  const int p1 = ms9(dot2(a53, 4 * C3D16, -4 * C5D16)), p2 = ms9(dot2(a53, 4 * C5D16, 4 * C3D16));
  const int q0 = ms9(dot2(a04, 4 * C1D4, 4 * C1D4)), q1 = ms9(dot2(a04, 4 * C1D4, -4 * C1D4));
  const int q2_ = ms9(dot2(a26, 4 * C3D8, -4 * C1D8)), q3 = ms9(dot2(a26, 4 * C1D8, 4 * C3D8));
  const int e0 = q0 + q3, e1 = q1 + q2_, e2 = q1 - q2_, e3 = q0 - q3;
  const int f0 = p0 + p1, f1 = p0 - p1, f2 = p3 - p2, f3 = p3 + p2;
  const int g1 = ms9(kmul<true>(C1D4, f2 - f1)), g2 = ms9(kmul<true>(C1D4, f2 + f1));
  o[0] = e0 + f3;
  o[1] = e1 + g2;
  o[2] = e2 + g1;
  o[3] = e3 + f0;
  o[4] = e3 - f0;
  o[5] = e2 - g1;
  o[6] = e1 - g2;
  o[7] = e0 - f3;
}
__device__ __forceinline__ void idct_col_pairs(int c, uint32_t p04, uint32_t p17, uint32_t p53, uint32_t p26,
                                               int v[64]) {
  int o[8];
  idct_col8(p04, p17, p53, p26, o);
#pragma unroll
  for (int k = 0; k < 8; k++) v[8 * k + c] = o[k];
}
template <class PairFn>
__device__ __forceinline__ void iq_idct_cols(PairFn pair, uint32_t q2, uint32_t qq, bool dcfix, int dc8,
                                             int v[64]) {
#pragma unroll
  for (int c = 0; c < 8; c++) {
    uint32_t p04 = dequantise_pk(pair(c, 32 + c), q2, qq);
    if (c == 0) p04 = dcfix ? __builtin_amdgcn_perm(p04, (uint32_t)dc8, 0x07060100u) : p04;  // (DC x 8, x4)
    idct_col_pairs(c, p04, dequantise_pk(pair(8 + c, 56 + c), q2, qq), dequantise_pk(pair(40 + c, 24 + c), q2, qq),
                   dequantise_pk(pair(16 + c, 48 + c), q2, qq), v);
    SCHED_FENCE();
  }
}
// levels (ints, natural order) in v -> reconstructed rows of an intra block.
// The row pass takes its product pairs by v_dot2 too: in an intra picture
// the dequantised inputs are bounded by the quantiser (|AC| <= 1,023 + q <=
// 1,054, DC <= 254 x 8 = 2,032), which bounds the column-pass outputs by
// 25,062 (every sign pattern at those magnitudes) < 2^15; a decoder or an
// inter residual may exceed that (up to 167,072), so only here.
// The final rounding's +8 rides in the accumulators of q0 and q1 (8 x 512:
// ms9(x + 4,096) = ms9(x) + 8, and every output is e_i +- f with e_i built
// from q0 or q1), then final_clamp_pack8_o8.
// The intra column pass two columns at a time on packed int16 pairs: the
// quantiser's bounds keep every intermediate of the pass (and its outputs,
// above) within int16 (q and p sums <= 25,062, f2 -+ f1 <= 4 x 4,958), so
// each product pair is one v_dot2 with halved constants and two columns'
// ms9 results pack by pk_ms8, the butterflies run as v_pk_add/sub_i16, and
// g = ms9(C1D4 x) = (181 x) >> 8 per half.  Columns (A, B) = (0, 4), (1, 7),
// (5, 3), (2, 6): out[k] = (x_kA, x_kB) is the row pass's input pair as it
// stands (a04, a17, a53, a26 of row k).
__device__ __forceinline__ void idct_col_pair_pk(const uint32_t a[4], const uint32_t b[4], s16x2 out[8]) {
  // a/b: column A's/B's dequantised natural pairs (x0,x4) (x1,x7) (x5,x3) (x2,x6)
  auto d = [](uint32_t x) { return __builtin_bit_cast(s16x2, x); };
  const s16x2 P0 = pk_ms8(dot2(d(a[1]), 2 * C7D16, -2 * C1D16), dot2(d(b[1]), 2 * C7D16, -2 * C1D16));
  const s16x2 P3 = pk_ms8(dot2(d(a[1]), 2 * C1D16, 2 * C7D16), dot2(d(b[1]), 2 * C1D16, 2 * C7D16));
  const s16x2 P1 = pk_ms8(dot2(d(a[2]), 2 * C3D16, -2 * C5D16), dot2(d(b[2]), 2 * C3D16, -2 * C5D16));
  const s16x2 P2 = pk_ms8(dot2(d(a[2]), 2 * C5D16, 2 * C3D16), dot2(d(b[2]), 2 * C5D16, 2 * C3D16));
  const s16x2 Q0 = pk_ms8(dot2(d(a[0]), 2 * C1D4, 2 * C1D4), dot2(d(b[0]), 2 * C1D4, 2 * C1D4));
  const s16x2 Q1 = pk_ms8(dot2(d(a[0]), 2 * C1D4, -2 * C1D4), dot2(d(b[0]), 2 * C1D4, -2 * C1D4));
  const s16x2 Q2 = pk_ms8(dot2(d(a[3]), 2 * C3D8, -2 * C1D8), dot2(d(b[3]), 2 * C3D8, -2 * C1D8));
  const s16x2 Q3 = pk_ms8(dot2(d(a[3]), 2 * C1D8, 2 * C3D8), dot2(d(b[3]), 2 * C1D8, 2 * C3D8));
  const s16x2 E0 = Q0 + Q3, E1 = Q1 + Q2, E2 = Q1 - Q2, E3 = Q0 - Q3;
  const s16x2 F0 = P0 + P1, F1 = P0 - P1, F2 = P3 - P2, F3 = P3 + P2;
  const s16x2 Dm = F2 - F1, Dp = F2 + F1;
  const s16x2 G1 = pk_ms8(dot2(Dm, C1D4 / 2, 0), dot2(Dm, 0, C1D4 / 2));
  const s16x2 G2 = pk_ms8(dot2(Dp, C1D4 / 2, 0), dot2(Dp, 0, C1D4 / 2));
  out[0] = E0 + F3;
  out[1] = E1 + G2;
  out[2] = E2 + G1;
  out[3] = E3 + F0;
  out[4] = E3 - F0;
  out[5] = E2 - G1;
  out[6] = E1 - G2;
  out[7] = E0 - F3;
}
// pair(e, f): the levels of natural positions e (low half) and f (high half)
// packed; dc: the DC level
template <class PairFn>
__device__ __forceinline__ void iq_idct_intra_rec_pairs(PairFn pair, int dc, int q, uint2 rec[8]) {
  const uint32_t q2 = 0x20002u * (uint32_t)q, qq = 0x10001u * (uint32_t)(q - (int)!(q & 1));
  const int dc8 = dc * 8;
  // the column's dequantised natural pairs (x0,x4) (x1,x7) (x5,x3) (x2,x6)
  auto col = [&](int c, uint32_t o[4]) {
    o[0] = dequantise_pk(pair(c, 32 + c), q2, qq);
    if (c == 0) o[0] = __builtin_amdgcn_perm(o[0], (uint32_t)dc8, 0x07060100u);  // (DC x 8, x4)
    o[1] = dequantise_pk(pair(8 + c, 56 + c), q2, qq);
    o[2] = dequantise_pk(pair(40 + c, 24 + c), q2, qq);
    o[3] = dequantise_pk(pair(16 + c, 48 + c), q2, qq);
  };
  s16x2 cp[4][8];  // [column pair (0,4) (1,7) (5,3) (2,6)][row]
  {
    constexpr int CA[4] = {0, 1, 5, 2}, CB[4] = {4, 7, 3, 6};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      uint32_t a[4], b[4];
      col(CA[i], a);
      col(CB[i], b);
      idct_col_pair_pk(a, b, cp[i]);
      SCHED_FENCE();
    }
  }
  const int r8 = opaque(8 << 9);  // one VGPR for every row (not rematerialised per use)
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const s16x2 a04 = cp[0][r], a17 = cp[1][r], a53 = cp[2][r], a26 = cp[3][r];
    const int p0 = ms9(dot2(a17, C7D16, -C1D16)), p3 = ms9(dot2(a17, C1D16, C7D16));
    const int p1 = ms9(dot2(a53, C3D16, -C5D16)), p2 = ms9(dot2(a53, C5D16, C3D16));
    const int q0 = ms9(dot2acc(a04, C1D4, C1D4, r8)), q1 = ms9(dot2acc(a04, C1D4, -C1D4, r8));
    const int q2_ = ms9(dot2(a26, C3D8, -C1D8)), q3 = ms9(dot2(a26, C1D8, C3D8));
    const int e0 = q0 + q3, e1 = q1 + q2_, e2 = q1 - q2_, e3 = q0 - q3;
    const int f0 = p0 + p1, f1 = p0 - p1, f2 = p3 - p2, f3 = p3 + p2;
    const int g1 = ms9(kmul<true>(C1D4, f2 - f1)), g2 = ms9(kmul<true>(C1D4, f2 + f1));
    const int o8[8] = {e0 + f3, e1 + g2, e2 + g1, e3 + f0, e3 - f0, e2 - g1, e1 - g2, e0 - f3};
    rec[r] = final_clamp_pack8_o8(o8);
    SCHED_FENCE();
  }
}
__device__ __forceinline__ void iq_idct_intra_rec(int v[64], int q, uint2 rec[8]) {
  iq_idct_intra_rec_pairs([&](int e, int f) { return pk2(v[e], v[f]); }, v[0], q, rec);
}
// the levels of natural positions e (low half) and f (high half) of the
// natural int16 level pairs L[r][j] = (x_r,2j, x_r,2j+1) as one pair
__device__ __forceinline__ uint32_t lvl_pair(const uint32_t L[8][4], int e, int f) {
  const uint32_t sel = (uint32_t)(2 * (e & 1)) | ((uint32_t)(2 * (e & 1) + 1) << 8) |
                       ((uint32_t)(4 + 2 * (f & 1)) << 16) | ((uint32_t)(5 + 2 * (f & 1)) << 24);
  return __builtin_amdgcn_perm(L[f >> 3][(f & 7) >> 1], L[e >> 3][(e & 7) >> 1], sel);
}

// intra picture (p64.c:635, 770-771: every MB is MTYPE 0, CBP 0x3f), block
// layout: load -> ChenDct -> BoundDct + CCITTFlatQuantize + FlatBound ->
// zigzag store -> ICCITTFlatQuantize -> ChenIDct -> BoundIDct -> recon.
// Levels leave through LDS: a lane's block is 128 bytes of levels, and 64
// lanes storing their own 16-byte pieces touch 64 cache lines per store
// instruction (measured: the level stores alone took 44 us of the 63 us a
// load/store-only version of the intra kernel needed).  Each wave writes its
// 64 blocks' levels to its own LDS slot, then store instruction k writes
// blocks 8k..8k+7 with 8 lanes per block: whole 128-byte lines.
constexpr int LVL_STRIDE = 144;  // bytes per lane: 128 + 16 pad, conflict-free ds_write_b128
constexpr int LVL_WAVE = 64 * LVL_STRIDE;
__device__ __forceinline__ void put_levels(uint8_t *lds, int lane, int k, uint4 v) {
  *reinterpret_cast<uint4 *>(lds + lane * LVL_STRIDE + k * 16) = v;
}

// ---------------------------------------------------------------------------
// Coded-bit counts for the entropy coder (p64gpu_encode_args.vlc_bits): a
// transmitted block's bits counted from the zigzag levels the kernel has just
// staged in LDS (vlc_count.h), so the entropy coder needs no count pass over
// the levels (p64vlc.hip).
using p64k::VlcLenTab;
using p64k::nz2;
using p64k::block_vlc_bits;
using p64k::load_vlc_len;
using p64k::VLC_LEN_WORDS;
// one uint16 per block into vlc_bits[gmb][1 + b] (slot 0: the entropy coder's)
__device__ __forceinline__ void store_vlc_bits(const p64gpu_encode_args &a, unsigned nmbs, bool valid, unsigned gmb,
                                               int b, int bits) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.vlc_bits, (short)0, (int)(nmbs * 16u), BUF_RSRC_W3);
  __builtin_amdgcn_raw_buffer_store_b16((uint16_t)bits, r, valid ? (gmb * 8u + 1u + (unsigned)b) * 2u : BUF_OOB, 0,
                                        0);
}

struct IntraFetch {
  BlkPos p;
  uint2 rows[8];  // the block's pixels
  int q;          // UseQuant
};
// QMB: a per-MB UseQuant array is given (else a.quant, uniform, no load)
template <bool QMB>
__device__ __forceinline__ IntraFetch intra_fetch_at(const p64gpu_encode_args &a, const BlkPos &pos) {
  const int w = a.width, h = a.height, nmb = (w >> 4) * (h >> 4);
  IntraFetch f;
  f.p = pos;
  const int pw = f.p.plane ? w >> 1 : w;
  // buffer loads: 32-bit offsets (a launch covers < 2 GiB of pictures), no
  // 64-bit address arithmetic per row
  const __amdgpu_buffer_rsrc_t cur = __builtin_amdgcn_make_buffer_rsrc(
      (void *)a.cur, (short)0, (int)((int64_t)a.nframes * a.frame_stride), BUF_RSRC_W3);
  const uint32_t o = (uint32_t)((int64_t)f.p.fi * a.frame_stride) +
                     (uint32_t)(plane_offset(f.p.plane, w, h) + mul24(f.p.y, pw) + f.p.x);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(cur, o + (uint32_t)mul24(k, pw), 0, 0);
    f.rows[k] = make_uint2(v[0], v[1]);
  }
  f.q = QMB ? a.quant_mb[f.p.fi * nmb + f.p.mb] : a.quant;
  return f;
}
// A block's outputs between its computation and its stores
struct IntraOut {
  uint2 rec[8];     // reconstructed rows
  uint32_t rec_off; // byte offset of the block's first row from a.recon
  int pw;           // its plane's width
};
// one block: ChenDct, quantise + zigzag into the LDS staging, dequantise,
// ChenIDct, reconstruction into `out`
template <bool CLAMP, bool POW2 = false>
__device__ __forceinline__ void intra_block(const p64gpu_encode_args &a, const IntraFetch &f, uint8_t *lds,
                                            int lane, IntraOut &out, uint32_t nzm[2] = nullptr) {
  const int w = a.width, h = a.height;
  const BlkPos &p = f.p;
  const int q = f.q;
  const p64_qint qt = c_qint.ac[q];
  out.pw = p.plane ? w >> 1 : w;
  out.rec_off = (uint32_t)((int64_t)p.fi * a.frame_stride) + (uint32_t)plane_offset(p.plane, w, h) +
                (uint32_t)mul24(p.y, out.pw) + (uint32_t)p.x;
  if (POW2) {  // a uniform q with 16q a power of two: level pairs from the packed row pass (qlevel_pk2)
    uint32_t L[8][4];
    int l0;
    {
      s16x2 pc[8][4];
      fdct_cols_pk(f.rows, pc);
      const uint32_t lo2 = pk16u(qt.vlo, qt.vlo), hi2 = pk16u(qt.vhi, qt.vhi);
      const uint32_t cp2 = pk16u(qt.cp, qt.cp), cn2 = pk16u(qt.cn, qt.cn);
#pragma unroll
      for (int r = 0; r < 8; r++) {
        uint32_t P[4];
        fwd_row_pk2(pc[r], P);
#pragma unroll
        for (int j = 0; j < 4; j++) L[r][j] = qlevel_pk2<CLAMP>(P[j], lo2, hi2, cp2, cn2, qt.s);
        if (r == 0) {  // intra DC: ((DC +- 4) / 8) in 1..254 of the bounded DC (transform.c:321-325)
          l0 = clampi(dct_final(min(dct_final((int)(int16_t)(P[0] & 0xffffu)), 2047)), 1, 254);
          L[0][0] = (L[0][0] & 0xffff0000u) | (uint32_t)l0;
        }
        SCHED_FENCE();
      }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t pk[4];
#pragma unroll
      for (int j = 0; j < 4; j++) pk[j] = lvl_pair(L, k_zz.inv[8 * k + 2 * j], k_zz.inv[8 * k + 2 * j + 1]);
      if (nzm)
#pragma unroll
        for (int j = 0; j < 4; j++) nzm[k >> 2] |= nz2(pk[j]) << (2 * (4 * (k & 3) + j));
      put_levels(lds, lane, k, make_uint4(pk[0], pk[1], pk[2], pk[3]));
      SCHED_FENCE();
    }
    iq_idct_intra_rec_pairs([&](int e, int f) { return lvl_pair(L, e, f); }, l0, q, out.rec);
    return;
  }
  int v[64];
  fdct_block_pk(f.rows, v);
  // in scan order: quantise (BoundDct + CCITTFlatQuantize + FlatBound), pack
  // the level pair; 16 bytes of levels at a time into the wave's LDS staging.
  // From q = 5 on the level bound lies beyond BoundDct's and an 8-bit block's
  // AC never reaches BoundDct's (|v| <= 8,163.5 < 8,187, proved in
  // tests/test_intra_dct_bound.py): CLAMP false then (a kernel of its own,
  // chosen by the host for a uniform UseQuant >= 5)
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int l2[2];
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const int e = k_zz.inv[8 * k + 2 * j + i];
        // intra DC: ((DC +- 4) / 8) in 1..254 of the bounded DC (transform.c:321-325)
        l2[i] = e == 0 ? clampi(dct_final(min(dct_final(v[0]), 2047)), 1, 254) : qlevel_int<CLAMP>(v[e], qt);
        v[e] = l2[i];  // dequantised in pairs by iq_idct_intra_rec
      }
      pk[j] = __builtin_amdgcn_perm((uint32_t)l2[1], (uint32_t)l2[0], 0x05040100u);
      if (nzm) nzm[k >> 2] |= nz2(pk[j]) << (2 * (4 * (k & 3) + j));
    }
    put_levels(lds, lane, k, make_uint4(pk[0], pk[1], pk[2], pk[3]));
    SCHED_FENCE();
  }
  iq_idct_intra_rec(v, q, out.rec);  // ICCITTFlatQuantize + ChenIDct + BoundIDctMatrix
}
// the stores of an MB-grouped wave (k_intra_mbg, k_inter_mbg), all buffer
// stores with out-of-range offsets instead of branches: the wave's levels run
// (nvalid MBs x 768 bytes at coef + gmb0 x 768) from the LDS staging, the
// lane's 8 reconstructed rows (rec_off, plane width pw), and from the record
// lanes (rl) the MB record dword and the LastIntra byte of MB gmb
// (block form: the wave's blocks g0 .. g0 + nblk - 1 of the launch, 128 bytes
// of levels each, from lane b's staging; block b only if bit b of keep is set)
__device__ __forceinline__ void blk_store_levels(const p64gpu_encode_args &a, const uint8_t *lds, int lane,
                                                 unsigned nmbs, unsigned g0, uint32_t nblk,
                                                 uint64_t keep = ~0ull) {
  const __amdgpu_buffer_rsrc_t coef =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.coef, (short)0, (int)(nmbs * 768u), BUF_RSRC_W3);
  const uint32_t nbytes = nblk * 128u;
  WAVE_FENCE();  // the staging writes (put_levels, every lane) before these reads
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t ob = 1024u * k + 16u * lane;
    const uint4 v = *reinterpret_cast<const uint4 *>(lds + (ob >> 7) * LVL_STRIDE + (ob & 127));
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 d;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
    const bool st = ob < nbytes && ((keep >> (ob >> 7)) & 1u);
    __builtin_amdgcn_raw_buffer_store_b128(d, coef, st ? g0 * 128u + ob : BUF_OOB, 0, 0);
  }
  __builtin_amdgcn_wave_barrier();
  WAVE_FENCE();  // these reads before the staging is reused (idct_coded_blocks' slots)
}
__device__ __forceinline__ void mbg_store_levels(const p64gpu_encode_args &a, const uint8_t *lds, int lane,
                                                 unsigned nmbs, unsigned gmb0, uint32_t nvalid,
                                                 uint64_t keep = ~0ull) {
  blk_store_levels(a, lds, lane, nmbs, 6u * gmb0, 6u * nvalid, keep);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t recon_rsrc(const p64gpu_encode_args &a, const BlkDiv &kd,
                                                             unsigned nmbs) {
  const int nfr = (int)mdiv(nmbs, kd.mn, kd.sn);
  return __builtin_amdgcn_make_buffer_rsrc((void *)a.recon, (short)0, (int)(nfr * a.frame_stride), BUF_RSRC_W3);
}
// the rows (rec_off out of range: none) and the record of an MB-grouped wave,
// with the MB's nonzero-block mask nzm (bit 5-b: block b has a nonzero level)
// when the caller asked for it (a.nzmask)
__device__ __forceinline__ void mbg_store_rows(const p64gpu_encode_args &a, const BlkDiv &kd, unsigned nmbs,
                                               uint32_t rec_off, int pw, const uint2 rows[8], bool rl,
                                               unsigned gmb, uint32_t mbw, uint8_t li, uint32_t nzm) {
  const __amdgpu_buffer_rsrc_t rec = recon_rsrc(a, kd, nmbs);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 d;
    d[0] = rows[k].x;
    d[1] = rows[k].y;
    __builtin_amdgcn_raw_buffer_store_b64(d, rec, rec_off + (uint32_t)mul24(k, pw), 0, 0);
  }
  const __amdgpu_buffer_rsrc_t mbr =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.mb, (short)0, (int)(nmbs * 4u), BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t lir =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.last_intra, (short)0, (int)nmbs, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t nzr =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.nzmask, (short)0, a.nzmask ? (int)nmbs : 0, BUF_RSRC_W3);
  __builtin_amdgcn_raw_buffer_store_b32(mbw, mbr, rl ? 4u * gmb : BUF_OOB, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(li, lir, rl ? gmb : BUF_OOB, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)nzm, nzr, rl ? gmb : BUF_OOB, 0, 0);
}
// intra picture, block layout over all 64 lanes: wave w takes the launch's
// blocks 64 w .. 64 w + 63 in MB-major order (blk_pos_mb of block g: MB g / 6,
// block g % 6), so an MB may straddle two waves -- nothing in an intra block
// looks at its MB's other blocks; levels leave as one contiguous 8-KB run per
// wave.  (Ten whole MBs per wave, as the inter kernel needs for its CBP
// ballots, leave lanes 60..63 idle: 6.25% more waves.)
template <bool QMB, bool CLAMP, bool POW2 = false, bool BITS = false>
__global__ __launch_bounds__(64 * MBG_WAVES) void k_intra_mbg(p64gpu_encode_args a, BlkDiv kd, unsigned nmbs,
                                                                 const uint32_t *vt) {
  __shared__ __align__(16) uint8_t lvl[MBG_WAVES * LVL_WAVE];
  __shared__ uint32_t vlen[BITS ? MBG_WAVES * VLC_LEN_WORDS : 1];
  const int lane = threadIdx.x & 63;
  uint8_t *lds = lvl + (threadIdx.x >> 6) * LVL_WAVE;
  const unsigned nblk = 6u * nmbs;
  const unsigned g0 = (xcd_remap(blockIdx.x, gridDim.x) * MBG_WAVES + (threadIdx.x >> 6)) * 64u;
  if (g0 >= nblk) return;  // whole wave
  PRIO_HIGH();
  const unsigned g = min(g0 + (unsigned)lane, nblk - 1);  // tail lanes repeat the last block
  const unsigned gmb = __umulhi(g, 0xAAAAAAABu) >> 2;      // g / 6
  const int b = (int)(g - 6u * gmb);
  const IntraFetch f = intra_fetch_at<QMB>(a, blk_pos_mb(gmb, b, a.width, a.height, kd));
  PRIO_LOW();
  IntraOut o;
  uint32_t nzm[2] = {0u, 0u};
  intra_block<CLAMP, POW2>(a, f, lds, lane, o, BITS ? nzm : nullptr);
  if (BITS) {  // every intra block is transmitted: DC + AC codes + EOB
    uint32_t *vl = vlen + (threadIdx.x >> 6) * VLC_LEN_WORDS;
    load_vlc_len(vt, vl, lane);
    WAVE_FENCE();
    const int bb = block_vlc_bits(reinterpret_cast<const uint8_t *>(vl),
                                  reinterpret_cast<const int16_t *>(lds + lane * LVL_STRIDE), nzm[0], nzm[1], false);
    store_vlc_bits(a, nmbs, g0 + (unsigned)lane < nblk, gmb, b, bb);
  }
  // the MB's record and LastIntra (p64.c:909-910: MTYPE 0, CBP 0x3f, LastIntra
  // reset) from the lane of its block 0; every intra block has a nonzero level
  // (the DC, 1..254)
  const bool rl = b == 0 && g0 + (unsigned)lane < nblk;
  blk_store_levels(a, lds, lane, nmbs, g0, min(64u, nblk - g0));
  mbg_store_rows(a, kd, nmbs, o.rec_off, o.pw, o.rec, rl, gmb, 0x3f00u, 0, 0x3fu);
}
// The source of an 8x8 prediction at (x, y) of a plane (any byte alignment):
// three aligned dwords per row (the third only matters when the row is
// misaligned)
struct PredSrc {
  uint32_t d[8][3];
  int sh;
};
// the horizontal taps of the H.261 loop filter ([1 2 1], edge columns x4) of
// a row as four packed 16-bit pairs (hz_2i, hz_2i+1), each tap sum one byte
// dot product of the packed source row, biased by 2 in its accumulator (the
// vertical pass's +8 rounding, spread over its weights 1 + 2 + 1 or 4): at
// most 4 x 255 + 2 = 1,022
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void hz_row_pk(const PredSrc &p, int r, u16x2 hz[4]) {
  const uint32_t lo = align4(p.d[r][1], p.d[r][0], p.sh), hi = align4(p.d[r][2], p.d[r][1], p.sh);
  const uint32_t mid = align4(hi, lo, 2);  // pixels 2..5
  const uint32_t w[8] = {__builtin_amdgcn_udot4(lo, 0x00000004u, 2u, false),
                         __builtin_amdgcn_udot4(lo, 0x00010201u, 2u, false),
                         __builtin_amdgcn_udot4(lo, 0x01020100u, 2u, false),
                         __builtin_amdgcn_udot4(mid, 0x00010201u, 2u, false),
                         __builtin_amdgcn_udot4(mid, 0x01020100u, 2u, false),
                         __builtin_amdgcn_udot4(hi, 0x00010201u, 2u, false),
                         __builtin_amdgcn_udot4(hi, 0x01020100u, 2u, false),
                         __builtin_amdgcn_udot4(hi, 0x04000000u, 2u, false)};
#pragma unroll
  for (int i = 0; i < 4; i++) hz[i] = __builtin_bit_cast(u16x2, (w[2 * i + 1] << 16) | w[2 * i]);
}
// pred_rows' loop filter in packed 16-bit arithmetic: the vertical
// [1 2 1] + 8 >> 4 of the tap pairs (at most 4 x 1,022 = 4,088; the +8 is in
// the taps' bias) as v_pk_ operations, half the registers of the unpacked
// rows: edge rows (4 hz + 8) >> 4 = hz' >> 2
__device__ __forceinline__ void pred_rows_filter_pk(const PredSrc &P, uint2 prow[8]) {
  u16x2 hp[4], hc[4], hn[4];
  hz_row_pk(P, 0, hc);
  hz_row_pk(P, 1, hn);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    uint32_t t[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      u16x2 v;
      if (r == 0 || r == 7) {
        v = hc[i] >> (u16x2){2, 2};
      } else {  // 2 hc + hp as one v_pk_mad_u16 (hipcc: a shift and an add)
        u16x2 m;
        asm("v_pk_mad_u16 %0, %1, 2, %2 op_sel_hi:[1,0,1]" : "=v"(m) : "v"(hc[i]), "v"(hp[i]));
        v = (u16x2)(m + hn[i]) >> (u16x2){4, 4};
      }
      t[i] = __builtin_bit_cast(uint32_t, v);
    }
    prow[r] = make_uint2(__builtin_amdgcn_perm(t[1], t[0], 0x06040200u), __builtin_amdgcn_perm(t[3], t[2], 0x06040200u));
#pragma unroll
    for (int i = 0; i < 4; i++) {
      hp[i] = hc[i];
      hc[i] = hn[i];
    }
    if (r + 2 < 8) hz_row_pk(P, r + 2, hn);
  }
}
// decoder reconstruction (DecompressMDU p64.c:1179-1237 + DecodeSaveMDU
// p64.c:971-1013), block layout: a lane loads its MB's record, then its
// block's levels and prediction source (rec_stage_b), forms the prediction,
// and the wave's coded blocks go through idct_coded_blocks (below).  Every
// load is a buffer load: where a block needs no levels
// (uncoded) or no prediction (intra MB) its offset is out of range, which
// reads zeros without touching memory -- no branch around any load, so the
// wait counts stay exact and only the algorithmic bytes move.
// MBs whose coded_mask is 0 are left alone.  Motion vectors are clamped so a
// block's source stays inside its plane: a conforming stream never needs it
// (H.261 vectors point inside the picture; the reader rejects others) and a
// corrupt one cannot make the kernel read outside the picture.
// One launch covers at most 2 GiB of levels and of pictures (the host splits
// larger batches), so every offset fits the 32-bit buffer range.

struct RecBufs {
  __amdgpu_buffer_rsrc_t ref, coef, mb, q, mask;
};
struct RecStageA {  // the block and its MB's record
  BlkPos p;
  uint32_t m;  // p64_mb_rec as one dword
  int q, coded;
};
struct RecStageB {  // what the block's reconstruction reads
  uint32_t lq[8][4];  // zigzag levels, 8 x 16 bytes (zeros if not coded)
  PredSrc pred;       // prediction source (zeros if intra)
  bool ck, inter, filter;
};
// does block p.b of the MB carry levels (MTYPE with TCOEFF, CBP bit; p64.c:1200)
__device__ __forceinline__ bool rec_block_coded(const RecStageA &A) {
  const int mt = (int)(int8_t)(A.m & 0xff);
  const int cbp = mt_cbp(mt) ? (int)((A.m >> 8) & 0x3f) : 0x3f;
  return A.coded && mt_tcoeff(mt) && ((cbp >> (5 - A.p.b)) & 1);
}
// LEVELS: load the block's levels into S.lq (else the caller fills them)
template <bool LEVELS = true>
__device__ __forceinline__ RecStageB rec_stage_b(const RecBufs &B, int w, int h, int64_t stride,
                                                 const RecStageA &A) {
  const int nmb = (w >> 4) * (h >> 4);
  const BlkPos &p = A.p;
  const int mt = (int)(int8_t)(A.m & 0xff);
  RecStageB S;
  S.ck = rec_block_coded(A);
  S.inter = A.coded && !mt_intra(mt);
  S.filter = mt_filter(mt);
  const int pw = p.plane ? w >> 1 : w, ph = p.plane ? h >> 1 : h;
  int dx = 0, dy = 0;
  if (mt_mf(mt)) {  // chroma MV/2 with C truncation (io.c:268-270)
    const int mvx = (int)(int8_t)((A.m >> 16) & 0xff), mvy = (int)(int8_t)(A.m >> 24);
    dx = p.plane ? mvx / 2 : mvx;
    dy = p.plane ? mvy / 2 : mvy;
  }
  const int sx = clampi(p.x + dx, 0, pw - 8), sy = clampi(p.y + dy, 0, ph - 8);
  S.pred.sh = sx & 3;
  const uint32_t po = S.inter ? (uint32_t)((int64_t)p.fi * stride) + (uint32_t)plane_offset(p.plane, w, h) +
                                    (uint32_t)(mul24(sy, pw) + (sx & ~3))
                              : BUF_OOB;
  // rows 0..6 as 12-byte loads (the third dword matters only when the row is
  // misaligned; otherwise it is the start of the next row, inside the
  // buffer); row 7 takes its third dword only when misaligned (then it lies
  // inside the row: sx <= pw - 9) -- an aligned last row at the end of the
  // buffer would reach past it
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(B.ref, po + (uint32_t)mul24(k, pw), 0, 0);
    S.pred.d[k][0] = v[0];
    S.pred.d[k][1] = v[1];
    S.pred.d[k][2] = v[2];
  }
  {
    const uint32_t o7 = po + (uint32_t)mul24(7, pw);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(B.ref, o7, 0, 0);
    S.pred.d[7][0] = v[0];
    S.pred.d[7][1] = v[1];
    S.pred.d[7][2] = __builtin_amdgcn_raw_buffer_load_b32(B.ref, S.pred.sh ? o7 + 8 : BUF_OOB, 0, 0);
  }
  // the levels after the prediction source: the prediction is formed first,
  // and wait counts are in issue order
  if (LEVELS) {
    const uint32_t co = S.ck ? (uint32_t)(((p.fi * nmb + p.mb) * 6 + p.b) * 128) : BUF_OOB;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(B.coef, co + 16 * k, 0, 0);
      S.lq[k][0] = v[0];
      S.lq[k][1] = v[1];
      S.lq[k][2] = v[2];
      S.lq[k][3] = v[3];
    }
  }
  return S;
}
// one reconstructed row: residual v[0..7] (after idct_final) + prediction
// row pr (packed bytes), clamped to 0..255 (BoundIDctMatrix), packed -- in
// 16-bit pairs: v_cvt_pk_i16_i32 (saturating), the prediction bytes widened by
// v_perm, v_pk_add_i16 with clamp, v_sat_pk_u8_i16.  Saturating the residual
// to +-32767 first changes nothing: the prediction is 0..255.
__device__ __forceinline__ uint2 recon_row(const int v[8], uint2 pr) {
  uint32_t o2[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint32_t rp, sum, sat;
    asm("v_cvt_pk_i16_i32 %0, %1, %2" : "=v"(rp) : "v"(v[2 * j]), "v"(v[2 * j + 1]));
    const uint32_t pd = j < 2 ? pr.x : pr.y;
    const uint32_t pp = __builtin_amdgcn_perm(0u, pd, (j & 1) ? 0x0c030c02u : 0x0c010c00u);
    asm("v_pk_add_i16 %0, %1, %2 clamp" : "=v"(sum) : "v"(pp), "v"(rp));
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(sat) : "v"(sum));
    o2[j] = sat;
  }
  return make_uint2(__builtin_amdgcn_perm(o2[1], o2[0], 0x05040100u), __builtin_amdgcn_perm(o2[3], o2[2], 0x05040100u));
}
__device__ __forceinline__ void pred_rows(const PredSrc &P, bool filter, uint2 prow[8]);
// IQ + ChenIDct + reconstruction over a wave's CODED blocks only (decoder
// and k_inter_mbg).  A wave holds 60 blocks, typically a quarter of them with
// levels (1.5 of 6 per MB on the bench stream), but a one-lane-per-block
// transform costs the wave the same whatever that count.  Here the coded
// blocks are ranked (ballot + mbcnt) and go through the transform 64/LPB at
// a time with LPB lanes per block: each pass, the coded lanes of rank
// NS p .. NS p + NS - 1 put their raw natural level pairs (per column) and
// prediction rows into the wave's LDS slots; lane LPB j + g dequantises and
// runs the column pass of columns g, g + LPB, ... of slot j, then the row
// pass and the reconstruction of rows g, g + LPB, ..., written back over the
// slot's prediction rows, which the block's own lane then reads back into
// prow.  ceil(n/NS) passes of 8/LPB columns and rows per lane instead of
// eight of each per lane; the caller stores every block (reconstruction or
// prediction) with its wave-wide row stores.  All exchanges stay inside one wave: a
// wave's LDS operations complete in order, so no barrier; the wavefront-scope
// fences only keep the compiler from moving LDS accesses across an exchange.
//   ck       this lane's block carries levels
//   np       its raw levels as natural column pairs: np[c] = (x0c,x4c) (x1c,x7c)
//            (x5c,x3c) (x2c,x6c), x_rc = level of row r, column c
//   q, intra UseQuant and the intra-DC rule (DC x 8, transform.c:371)
//   prow     in: prediction rows (zeros for intra); out: the reconstruction
//            if ck (else unchanged)
// Four lanes per block: a pass takes 16 blocks, lane 4j+g columns (rows) g,
// g+4 of slot j (eight lanes per block, 8 blocks a pass, measured 1.7 us
// slower in the decoder).  Slot: 64 row-major values, 16 prediction dwords,
// header; its stride (84 = 20 mod 64) keeps the row-major writes of the
// column pass free of bank conflicts.
constexpr int LPB = 4, RSLOT = 84, RSLOT_PRED = 64, RSLOT_HDR = 80;
constexpr int RSLOTS_BYTES = 4 * RSLOT * (64 / LPB);
static_assert(RSLOTS_BYTES <= LVL_WAVE, "k_inter_mbg's slots live in its level staging");
// The row pass writes the reconstructed rows back into the slot and each
// coded lane reads its block's rows into prow: the caller then stores every
// block of the wave with the same wave-wide row stores (contiguous 8-byte row
// pieces of adjacent blocks).  Stores from the pass itself (one block row per
// lane, scattered) cost the decoder 34.3 vs 28.6 us and +14 MB of HBM writes
// per launch, k_inter_mbg ~1.5 us.
__device__ __forceinline__ void idct_coded_blocks(bool ck, const uint32_t np[8][4], int q, bool intra,
                                                  uint2 prow[8], uint32_t *slots, int lane) {
  constexpr int NS = 64 / LPB, CPL = 8 / LPB, RS = RSLOT;
  const uint64_t cm = __builtin_amdgcn_ballot_w64(ck);
  const int n = __builtin_popcountll(cm);
  const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
  const int j = lane / LPB, g = lane % LPB;  // this lane's slot, first column (row)
  uint32_t *const mine = slots + RS * j;
  for (int pass = 0; pass < n; pass += NS) {  // uniform
    WAVE_FENCE();
    if (ck && rank >= pass && rank < pass + NS) {
      uint32_t *const s = slots + RS * (rank - pass);
#pragma unroll
      for (int cc = 0; cc < 8; cc++) *(uint4 *)(s + 4 * cc) = make_uint4(np[cc][0], np[cc][1], np[cc][2], np[cc][3]);
#pragma unroll
      for (int k = 0; k < 8; k += 2)
        *(uint4 *)(s + RSLOT_PRED + 2 * k) = make_uint4(prow[k].x, prow[k].y, prow[k + 1].x, prow[k + 1].y);
      *(uint4 *)(s + RSLOT_HDR) = make_uint4((uint32_t)q | (intra ? 0x100u : 0u), 0u, 0u, 0u);
    }
    WAVE_FENCE();
    {  // column pass: columns g + LPB i of slot j, written back row-major in place
      uint4 lv[CPL];
#pragma unroll
      for (int i = 0; i < CPL; i++) lv[i] = *(const uint4 *)(mine + 4 * (g + LPB * i));
      const uint32_t hx = mine[RSLOT_HDR];  // q | intra << 8
      const int qj = (int)(hx & 0xff);
      const uint32_t q2 = 0x20002u * (uint32_t)qj, qq = 0x10001u * (uint32_t)(qj - (int)!(qj & 1));
      WAVE_FENCE();  // every column read before the first write
#pragma unroll
      for (int i = 0; i < CPL; i++) {
        uint32_t p04 = dequantise_pk(lv[i].x, q2, qq);
        if (i == 0 && g == 0 && (hx & 0x100u))  // intra DC: DC x 8
          p04 = __builtin_amdgcn_perm(p04, (uint32_t)((int)(int16_t)(lv[i].x & 0xffff) * 8), 0x07060100u);
        int o[8];
        idct_col8(p04, dequantise_pk(lv[i].y, q2, qq), dequantise_pk(lv[i].z, q2, qq),
                  dequantise_pk(lv[i].w, q2, qq), o);
#pragma unroll
        for (int k = 0; k < 8; k++) mine[8 * k + g + LPB * i] = (uint32_t)o[k];
        SCHED_FENCE();
      }
    }
    WAVE_FENCE();
#pragma unroll
    for (int i = 0; i < CPL; i++) {  // row pass of row g + LPB i of slot j, + prediction, BoundIDctMatrix, store
      const int r = g + LPB * i;
      const uint4 x0 = *(const uint4 *)(mine + 8 * r), x1 = *(const uint4 *)(mine + 8 * r + 4);
      const uint2 pr = *(const uint2 *)(mine + RSLOT_PRED + 2 * r);
      const int x[8] = {(int)x0.x, (int)x0.y, (int)x0.z, (int)x0.w, (int)x1.x, (int)x1.y, (int)x1.z, (int)x1.w};
      int o[8];
      inv8<true>(x, o);
#pragma unroll
      for (int k = 0; k < 8; k++) o[k] = idct_final(o[k]);
      const uint2 rr = recon_row(o, pr);
      *(uint2 *)(mine + RSLOT_PRED + 2 * r) = rr;  // (this lane's own row: read above)
      SCHED_FENCE();
    }
    WAVE_FENCE();  // the pass's coded lanes take their reconstructed rows back
    if (ck && rank >= pass && rank < pass + NS) {
      const uint32_t *const s = slots + RS * (rank - pass);
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        const uint4 t = *(const uint4 *)(s + RSLOT_PRED + 2 * k);
        prow[k] = make_uint2(t.x, t.y);
        prow[k + 1] = make_uint2(t.z, t.w);
      }
    }
  }
  WAVE_FENCE();
}
// IQ (ICCITTQuantize transform.c:400) + ChenIDct + reconstruction of one
// inter-coded block in its own lane, no LDS: the packed column pass of the
// intra path (idct_col_pair_pk on dequantised natural column pairs) -- exact
// when every dequantised value is within +-1,291, the largest box whose every
// intermediate of that pass stays inside int16
// (tests/test_intra_dct_bound.py) -- then the row pass on those pairs by
// v_dot2 (32-bit sums), idct_final and the prediction (recon_row), as
// idct_coded_blocks computes them.  np: the block's raw natural column pairs
// (x0c,x4c) (x1c,x7c) (x5c,x3c) (x2c,x6c); prow: prediction in,
// reconstruction out.
__device__ __forceinline__ void iq_idct_inter_rec(const uint32_t np[8][4], int q, uint2 prow[8]) {
  const uint32_t q2 = 0x20002u * (uint32_t)q, qq = 0x10001u * (uint32_t)(q - (int)!(q & 1));
  s16x2 cp[4][8];  // [column pair (0,4) (1,7) (5,3) (2,6)][row]
  {
    constexpr int CA[4] = {0, 1, 5, 2}, CB[4] = {4, 7, 3, 6};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      uint32_t a[4], b[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        a[k] = dequantise_pk(np[CA[i]][k], q2, qq);
        b[k] = dequantise_pk(np[CB[i]][k], q2, qq);
      }
      idct_col_pair_pk(a, b, cp[i]);
      SCHED_FENCE();
    }
  }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const s16x2 a04 = cp[0][r], a17 = cp[1][r], a53 = cp[2][r], a26 = cp[3][r];
    const int p0 = ms9(dot2(a17, C7D16, -C1D16)), p3 = ms9(dot2(a17, C1D16, C7D16));
    const int p1 = ms9(dot2(a53, C3D16, -C5D16)), p2 = ms9(dot2(a53, C5D16, C3D16));
    const int q0 = ms9(dot2(a04, C1D4, C1D4)), q1 = ms9(dot2(a04, C1D4, -C1D4));
    const int q2_ = ms9(dot2(a26, C3D8, -C1D8)), q3 = ms9(dot2(a26, C1D8, C3D8));
    const int e0 = q0 + q3, e1 = q1 + q2_, e2 = q1 - q2_, e3 = q0 - q3;
    const int f0 = p0 + p1, f1 = p0 - p1, f2 = p3 - p2, f3 = p3 + p2;
    const int g1 = ms9(kmul<true>(C1D4, f2 - f1)), g2 = ms9(kmul<true>(C1D4, f2 + f1));
    int o[8] = {e0 + f3, e1 + g2, e2 + g1, e3 + f0, e3 - f0, e2 - g1, e1 - g2, e0 - f3};
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = idct_final(o[k]);
    prow[r] = recon_row(o, prow[r]);
    SCHED_FENCE();
  }
}
// the largest level magnitude, squared, whose dequantised value (2|l| + 1) q
// stays within the +-1,291 of iq_idct_inter_rec's packed column pass, by q
struct InterIdctLim {
  int l2[32];
};
constexpr InterIdctLim make_inter_idct_lim() {
  InterIdctLim t{};
  for (int q = 1; q < 32; q++) {
    int l = 0;
    while ((2 * (l + 1) + 1) * q <= 1291) l++;
    t.l2[q] = l * l;
  }
  return t;
}
__constant__ InterIdctLim c_idct_lim = make_inter_idct_lim();
#ifndef INTER_DIRECT_MIN
#define INTER_DIRECT_MIN 32  // coded blocks in a wave from which each lane runs its own IQ/IDCT
#endif

// the decoder's reconstruction through idct_coded_blocks (DIRECT: or, in a
// wave of many small-level inter blocks, one block per lane in registers)
template <bool DIRECT = false>
__device__ __forceinline__ void rec_wave_compact(int w, int h, int64_t stride, __amdgpu_buffer_rsrc_t rec,
                                                 const RecStageA &A, const RecStageB &S, uint32_t *slots,
                                                 int lane) {
  const BlkPos &p = A.p;
  uint2 prow[8];
  pred_rows(S.pred, S.filter && S.inter, prow);  // zeros for intra (source not loaded)
  const int pw = p.plane ? w >> 1 : w;
  const uint32_t ro = (uint32_t)((int64_t)p.fi * stride) + (uint32_t)plane_offset(p.plane, w, h) +
                      (uint32_t)(mul24(p.y, pw) + p.x);
  // natural column pairs straight from the packed zigzag words (one v_perm each)
  auto pair = [&](int e, int f) {
    const int s1 = k_zz.pos[e], s2 = k_zz.pos[f];
    const uint32_t sel = ((s1 & 1) ? 0x0302u : 0x0100u) | (((s2 & 1) ? 0x0706u : 0x0504u) << 16);
    return __builtin_amdgcn_perm(S.lq[s2 >> 3][(s2 >> 1) & 3], S.lq[s1 >> 3][(s1 >> 1) & 3], sel);
  };
  uint32_t np[8][4];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    np[c][0] = pair(c, 32 + c);
    np[c][1] = pair(8 + c, 56 + c);
    np[c][2] = pair(40 + c, 24 + c);
    np[c][3] = pair(16 + c, 48 + c);
  }
  // a wave with many coded blocks (SURVEY.md 8(d)'s stream: ~50 of 64) runs
  // one block per lane in registers when every coded block is an inter one
  // whose levels keep the packed column pass exact (sum l^2 <= the limit
  // squared bounds max |l|), as k_inter_mbg does; else the LDS pass
  int ss = 0;
#pragma unroll
  for (int c = 0; c < (DIRECT ? 8 : 0); c++)
#pragma unroll
    for (int j = 0; j < 4; j++)
      ss = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, np[c][j]), __builtin_bit_cast(s16x2, np[c][j]), ss, false);
  const int nck = __popcll(__ballot(S.ck));
  const bool lane_ok = !S.ck || (S.inter && ss <= c_idct_lim.l2[A.q & 31]);
  if (DIRECT && nck >= INTER_DIRECT_MIN && uni(__all(lane_ok))) {
    if (S.ck) iq_idct_inter_rec(np, A.q, prow);
  } else {
    idct_coded_blocks(S.ck, np, A.q, !S.inter, prow, slots, lane);
  }
  {  // every block of a coded MB, wave-wide: the reconstruction (coded blocks,
     // read back from the pass) or the prediction (uncoded blocks)
    const uint32_t uo = A.coded ? ro : BUF_OOB;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int k = 0; k < 8; k++) {
      u32x2 d;
      d[0] = prow[k].x;
      d[1] = prow[k].y;
      __builtin_amdgcn_raw_buffer_store_b64(d, rec, uo + (uint32_t)mul24(k, pw), 0, 0);
    }
  }
}
// occupancy target of k_inter_mbg and k_recon_mbg: at least 4 waves per
// SIMD (<= 128 VGPRs).  Both run one-wave workgroups: a wave's slot and its
// LDS free as soon as it ends (with the priority raised first, -1.5 us for
// the decoder and -1 us for k_inter_mbg); k_intra_mbg keeps four (MBG_WAVES).
#define OCC4 __attribute__((amdgpu_waves_per_eu(4)))
// decoder reconstruction, block layout over all 64 lanes (as k_intra_mbg: wave
// w takes blocks 64 w .. 64 w + 63, an MB may straddle two waves), one block
// per lane: each lane loads its MB's record, then its levels and
// prediction; coded blocks go through idct_coded_blocks, then every block
// stores its rows (reconstruction or prediction) wave-wide.  87 VGPRs: 5 waves per SIMD, which hide each other's two
// dependent load latencies (eight lanes per block: 80 VGPRs, 6 waves, but two
// passes per wave instead of one and 1.7 us slower; a persistent
// variant with the next block's loads in flight needed 237 VGPRs, 2 waves,
// and was slower).  Lanes past the batch get coded = 0:
// every load and store of theirs is out of range.
__global__ __launch_bounds__(64) OCC4 void k_recon_mbg(int w, int h, int64_t stride, const uint8_t *refp,
                                                           uint8_t *recp, const int16_t *coef,
                                                           const p64_mb_rec *mbr, const uint8_t *quant_mb,
                                                           const uint8_t *coded_mask, BlkDiv kd, unsigned nmbs) {
  const int lane = threadIdx.x & 63;
  const unsigned nblk = 6u * nmbs;
  const unsigned g0 = xcd_remap(blockIdx.x, gridDim.x) * 64u;  // the wave's first block
  if (g0 >= nblk) return;  // whole wave
  PRIO_HIGH();
  const int nmb = (w >> 4) * (h >> 4), nfr = (int)mdiv(nmbs, kd.mn, kd.sn);
  RecBufs B;
  B.ref = __builtin_amdgcn_make_buffer_rsrc((void *)refp, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  B.coef = __builtin_amdgcn_make_buffer_rsrc((void *)coef, (short)0, nfr * nmb * 768, BUF_RSRC_W3);
  B.mb = __builtin_amdgcn_make_buffer_rsrc((void *)mbr, (short)0, nfr * nmb * 4, BUF_RSRC_W3);
  B.q = __builtin_amdgcn_make_buffer_rsrc((void *)quant_mb, (short)0, nfr * nmb, BUF_RSRC_W3);
  B.mask = __builtin_amdgcn_make_buffer_rsrc((void *)coded_mask, (short)0, nfr * nmb, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t rec =
      __builtin_amdgcn_make_buffer_rsrc((void *)recp, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  const bool valid = g0 + (unsigned)lane < nblk;
  const unsigned g = min(g0 + (unsigned)lane, nblk - 1);
  const unsigned gmb = __umulhi(g, 0xAAAAAAABu) >> 2;  // g / 6
  RecStageA A;
  A.p = blk_pos_mb(gmb, (int)(g - 6u * gmb), w, h, kd);
  A.m = __builtin_amdgcn_raw_buffer_load_b32(B.mb, 4 * gmb, 0, 0);
  A.q = __builtin_amdgcn_raw_buffer_load_b8(B.q, gmb, 0, 0);
  A.coded = __builtin_amdgcn_raw_buffer_load_b8(B.mask, valid ? gmb : BUF_OOB, 0, 0);
  const RecStageB S = rec_stage_b(B, w, h, stride, A);
  PRIO_LOW();
  __shared__ uint32_t slots[RSLOT * (64 / LPB)];
  rec_wave_compact(w, h, stride, rec, A, S, slots, lane);
}

// Decoder reconstruction from PACKED levels (p64gpu_decode_recon_packed, ABI
// v3): the transmitted blocks' levels contiguous in raster order, and per
// group of 64 consecutive blocks of the batch (a wave, as k_recon_mbg's: an
// MB and a group may straddle two pictures) its first transmitted block's
// index and its transmitted-block mask, {start, 0, mask lo, mask hi}
// (p64s_pack_levels).  The wave reads its group's entry with one scalar load
// while its records are in flight; the prediction source's loads go out as
// soon as the record is in, then the level loads from start + (the lane's
// rank among the set bits) -- they need no record (in k_recon_mbg a lane
// learns from its record whether, and so where, to load).  Measured: levels
// issued before the prediction source 35.6-35.8 us, after it 34.9 (HBM 0.497,
// A/B in one lease, r06ar).  (Round 6's first form gave each picture
// ceil(6 nmb / 64) groups of its own: 2.4% more waves at CIF, the last of
// each picture 8/64 full.)
typedef unsigned su4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(64) OCC4 void k_recon_pk(int w, int h, int64_t stride, const uint8_t *refp,
                                                          uint8_t *recp, const int16_t *levels, uint32_t nlev,
                                                          const uint32_t *index, const p64_mb_rec *mbr,
                                                          const uint8_t *quant_mb, const uint8_t *coded_mask,
                                                          BlkDiv kd, unsigned nmbs) {
  const int lane = threadIdx.x & 63;
  const unsigned nblk = 6u * nmbs;
  const unsigned wv = xcd_remap(blockIdx.x, gridDim.x);  // the wave's group
  const unsigned g0 = wv * 64u;                           // its first block
  if (g0 >= nblk) return;  // whole wave
  PRIO_HIGH();
  const int nmb = (w >> 4) * (h >> 4), nfr = (int)mdiv(nmbs, kd.mn, kd.sn);
  RecBufs B;
  B.ref = __builtin_amdgcn_make_buffer_rsrc((void *)refp, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  B.coef = __builtin_amdgcn_make_buffer_rsrc((void *)levels, (short)0, (int)(nlev * 128u), BUF_RSRC_W3);
  B.mb = __builtin_amdgcn_make_buffer_rsrc((void *)mbr, (short)0, nfr * nmb * 4, BUF_RSRC_W3);
  B.q = __builtin_amdgcn_make_buffer_rsrc((void *)quant_mb, (short)0, nfr * nmb, BUF_RSRC_W3);
  B.mask = __builtin_amdgcn_make_buffer_rsrc((void *)coded_mask, (short)0, nfr * nmb, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t rec =
      __builtin_amdgcn_make_buffer_rsrc((void *)recp, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  const bool valid = g0 + (unsigned)lane < nblk;
  const unsigned g = min(g0 + (unsigned)lane, nblk - 1);
  const unsigned gmb = __umulhi(g, 0xAAAAAAABu) >> 2;  // g / 6
  RecStageA A;
  A.p = blk_pos_mb(gmb, (int)(g - 6u * gmb), w, h, kd);
  A.m = __builtin_amdgcn_raw_buffer_load_b32(B.mb, 4 * gmb, 0, 0);
  A.q = __builtin_amdgcn_raw_buffer_load_b8(B.q, gmb, 0, 0);
  A.coded = __builtin_amdgcn_raw_buffer_load_b8(B.mask, valid ? gmb : BUF_OOB, 0, 0);
  // the group's entry by a scalar load issued now and waited for only after
  // the prediction source's loads are out (rec_stage_b waits for the record
  // alone), then the level loads
  su4 ix;
  asm volatile("s_load_dwordx4 %0, %1, %2" : "=s"(ix) : "s"(index), "s"(16u * wv));
  RecStageB S = rec_stage_b<false>(B, w, h, stride, A);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(ix));
  const uint64_t msk = (uint64_t)ix.z | ((uint64_t)ix.w << 32);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(msk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)msk, 0u));
  const uint32_t lo = ((msk >> lane) & 1) && valid ? (ix.x + rank) * 128u : BUF_OOB;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(B.coef, lo + 16 * k, 0, 0);
    S.lq[k][0] = v[0];
    S.lq[k][1] = v[1];
    S.lq[k][2] = v[2];
    S.lq[k][3] = v[3];
  }
  PRIO_LOW();
  __shared__ uint32_t slots[RSLOT * (64 / LPB)];
  rec_wave_compact<false>(w, h, stride, rec, A, S, slots, lane);  // (DIRECT: 119 VGPRs, 4 waves: 39.6 vs 36.1 us, r06f)
}

// ---------------------------------------------------------------------------
// inter picture, second stage of the split encoder: k_motion writes every
// MB's ME record, then this block-layout kernel does the rest of
// ReadCompressMDU / CompressMDU (p64.c:734-1013) with one lane per 8x8 block
// (10 MBs per wave, lane = 6m + b, as k_intra_mbg): MTYPE decision from the
// ME record, prediction (MC, loop filter), ChenDct of the residual,
// quantisation, the CBP decision across the MB's six lanes (wave ballots),
// zigzag levels through the LDS staging, dequantisation, ChenIDct and the
// reconstruction.  The fused one-wave-per-MB k_encode spends 40% of its time
// in this half with 48 of 64 lanes busy on LDS-exchanged row passes; here
// every lane holds its block in registers.
__device__ __forceinline__ void pred_rows(const PredSrc &P, bool filter, uint2 prow[8]);
struct InterMe {  // the fields of p64_me_rec the decision needs
  int mx, my, sad, sad0, var, varor;
};
// prediction of the lane's block for MTYPE mt / vector (mvx, mvy), packed rows
__device__ __forceinline__ void inter_pred(const RecBufs &B, int w, int h, int64_t stride, const BlkPos &p,
                                           int mt, int mvx, int mvy, uint2 prow[8]) {
  RecStageA A;
  A.p = p;
  A.m = (uint32_t)(mt & 0xff) | ((uint32_t)(mvx & 0xff) << 16) | ((uint32_t)(mvy & 0xff) << 24);
  A.q = 0;
  A.coded = 1;
  const RecStageB S = rec_stage_b<false>(B, w, h, stride, A);  // source OOB (zeros) if intra
  PRIO_LOW();  // the loads are out: the loop filter at normal priority
  pred_rows(S.pred, S.filter, prow);
}
// the prediction as packed rows (all zero when the source was not loaded),
// the H.261 loop filter in packed 16-bit arithmetic (pred_rows_filter_pk;
// k_inter_mbg -0.45 us and the step -1.5 us against the unpacked adds,
// A/B x2 in round 4)
__device__ __forceinline__ void pred_rows(const PredSrc &P, bool filter, uint2 prow[8]) {
  if (filter) {
    pred_rows_filter_pk(P, prow);
  } else {  // the source rows as they are
#pragma unroll
    for (int r = 0; r < 8; r++)
      prow[r] = make_uint2(align4(P.d[r][1], P.d[r][0], P.sh), align4(P.d[r][2], P.d[r][1], P.sh));
  }
}
// OVR: an -o MTYPE override array is given.  Without one every MTYPE the
// decision can return (0, 2, 5, 8: decide_mtype) carries coefficients, so
// the level mask for MC-only types (4, 7) is left out.
// POW2: a uniform q whose D = 16q is a power of two (qlevel_pk2)
template <bool QMB, bool OVR, bool POW2 = false, bool BITS = false>
__global__ __launch_bounds__(64) OCC4 void k_inter_mbg(p64gpu_encode_args a, BlkDiv kd, unsigned nmbs,
                                                             p64_me_rec *me, const uint32_t *vt) {
  __shared__ __align__(16) uint8_t lds[LVL_WAVE];
  __shared__ uint32_t vlen[BITS ? VLC_LEN_WORDS : 1];
  const int lane = threadIdx.x;
  const unsigned gmb0 = xcd_remap(blockIdx.x, gridDim.x) * MBS_PER_WAVE;
  if (gmb0 >= nmbs) return;  // whole wave
  PRIO_HIGH();  // first: a fresh wave's loads go out before the older waves' arithmetic
  const int w = a.width, h = a.height, nfr = (int)mdiv(nmbs, kd.mn, kd.sn);
  const int64_t stride = a.frame_stride;
  RecBufs B;
  B.ref = __builtin_amdgcn_make_buffer_rsrc((void *)a.ref, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  const int l = min(lane, 6 * MBS_PER_WAVE - 1), b = l % 6;
  const unsigned gmb = min(gmb0 + (unsigned)(l / 6), nmbs - 1);  // tail lanes repeat the last MB
  const BlkPos pos = blk_pos_mb(gmb, b, w, h, kd);
  // the ME record, LastIntra and override first: the prediction loads wait
  // on them (wait counts are in issue order), the current rows only later
  const __amdgpu_buffer_rsrc_t mer =
      __builtin_amdgcn_make_buffer_rsrc((void *)me, (short)0, (int)(nmbs * sizeof(p64_me_rec)), BUF_RSRC_W3);
  const uint32_t mo = gmb * (uint32_t)sizeof(p64_me_rec);
  InterMe m;
  const auto r0 = __builtin_amdgcn_raw_buffer_load_b128(mer, mo, 0, 0);  // mx my sad sad0
  m.mx = (int)r0[0];
  m.my = (int)r0[1];
  m.sad = (int)r0[2];
  m.sad0 = (int)r0[3];
  // LastIntra and the -o override by buffer loads (an absent override array
  // reads as out of range: no branch around a load)
  const __amdgpu_buffer_rsrc_t lir =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.last_intra, (short)0, (int)nmbs, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t ovr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)a.mtype_override, (short)0, a.mtype_override ? (int)nmbs : 0, BUF_RSRC_W3);
  const int li = __builtin_amdgcn_raw_buffer_load_b8(lir, gmb, 0, 0);
  const int ov = OVR ? (int)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(ovr, gmb, 0, 0) : -1;
  const IntraFetch f = intra_fetch_at<QMB>(a, pos);  // current rows, q
  const int mvx = m.mx, mvy = m.my;
  // the source at the ME vector (luma MV, chroma MV/2, as an MC type reads
  // it): the prediction of every MC type, and on the luma lanes the block the
  // decision statistics are taken on (round 6: moved here from k_motion,
  // which no longer computes them for this path)
  RecStageA A1;
  A1.p = pos;
  A1.m = 5u | ((uint32_t)(mvx & 0xff) << 16) | ((uint32_t)(mvy & 0xff) << 24);
  A1.q = 0;
  A1.coded = 1;
  const RecStageB S1 = rec_stage_b<false>(B, w, h, stride, A1);
  // and the zero-vector source where the MB may turn out a non-MC inter type
  // (2, 3) with a vector other than (0,0): the decision's inter test needs
  // only the two SADs (decide_inter), the override is known too -- so these
  // loads go out at the same level as the ones above instead of after the
  // statistics (29% of the waves on SURVEY.md 8(d)'s content have such an MB)
  const bool cand0 = (mvx | mvy) != 0 && li <= 131 && (ov >= 0 ? ov == 2 || ov == 3 : decide_inter(m.sad, m.sad0));
  RecStageB S0;
  const bool any0 = uni(__any(cand0));
  if (any0) {
    RecStageA A0;
    A0.p = pos;
    A0.m = 2u;
    A0.q = 0;
    A0.coded = cand0 ? 1 : 0;  // (others: out of range, no traffic)
    S0 = rec_stage_b<false>(B, w, h, stride, A0);
  }
  PRIO_LOW();  // the loads are out
  // VAR, VAROR, MWOR at the chosen vector (me.c:229-245 == 313-329): per luma
  // lane the sums over its 8x8 quadrant by byte dot products, sum (r-c)^2 =
  // r.r - 2 r.c + c.c (exact in u32; c.c first: the current rows arrive
  // before the source), then every lane adds its MB's four luma lanes
  // (6m..6m+3) from one LDS exchange (the level staging, not in use yet)
  uint32_t rr = 0, rc = 0, cc = 0, rs = 0;
#pragma unroll
  for (int r = 0; r < 8; r++)
    cc = __builtin_amdgcn_udot4(f.rows[r].y, f.rows[r].y, __builtin_amdgcn_udot4(f.rows[r].x, f.rows[r].x, cc, false),
                                false);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const uint32_t w0 = align4(S1.pred.d[r][1], S1.pred.d[r][0], S1.pred.sh);
    const uint32_t w1 = align4(S1.pred.d[r][2], S1.pred.d[r][1], S1.pred.sh);
    rr = __builtin_amdgcn_udot4(w1, w1, __builtin_amdgcn_udot4(w0, w0, rr, false), false);
    rc = __builtin_amdgcn_udot4(w1, f.rows[r].y, __builtin_amdgcn_udot4(w0, f.rows[r].x, rc, false), false);
    rs = sad4(w1, 0u, sad4(w0, 0u, rs));
  }
  uint32_t e2 = rr + cc - 2 * rc, tr = 0, te = 0, ts = 0;
  {
    uint8_t *x = lds + lane * 16;
    *reinterpret_cast<uint4 *>(x) = make_uint4(e2, rr, rs, 0u);
    WAVE_FENCE();
    const uint8_t *g0 = lds + (l - b) * 16;  // the MB's lane 0 (tail lanes 60..63 copy lane 59)
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint4 v = *reinterpret_cast<const uint4 *>(g0 + 16 * i);
      te += v.x;
      tr += v.y;
      ts += v.z;
    }
    WAVE_FENCE();  // (the staging is written again later)
  }
  const int var = (int)(te / 256u);
  const uint32_t rs_mb = ts;
  const int varor = (int)(tr / 256u) - (int)(rs_mb / 256u) * (int)(rs_mb / 256u);

  // MTYPE (p64.c:734-772): the decision, the -o override, the intra refresh
  MeOut mo_;
  mo_.mx = m.mx;
  mo_.my = m.my;
  mo_.sad = m.sad;
  mo_.sad0 = m.sad0;
  mo_.var = var;
  mo_.varor = varor;
  mo_.mwor = (int)rs_mb;
  int mt = decide_mtype(mo_);
  if (ov >= 0) mt = ov;
  if (li > 131) mt = 0;
  // the prediction: MC types from the source already loaded; the non-MC
  // inter types (2, 3) from the zero vector, loaded now where the ME vector
  // is not (0,0); intra none
  uint2 prow[8];
  {
    // (need0 implies cand0: a non-MC inter type comes from the inter test or
    // the override, and a refreshed MB is intra)
    const bool need0 = !mt_intra(mt) && !mt_mf(mt) && (mvx | mvy) != 0;
    PredSrc P = S1.pred;
    if (any0 && need0) P = S0.pred;
    pred_rows(P, mt_filter(mt), prow);
    if (mt_intra(mt)) {
#pragma unroll
      for (int r = 0; r < 8; r++) prow[r] = make_uint2(0u, 0u);
    }
  }
  // the statistics into the ME record (p64_me_rec var, varor, mwor)
  {
    const bool rl0 = b == 0 && lane < 6 * MBS_PER_WAVE && gmb0 + (unsigned)(l / 6) < nmbs;
    typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
    u32x3 st;
    st[0] = (uint32_t)var;
    st[1] = (uint32_t)varor;
    st[2] = rs_mb;
    __builtin_amdgcn_raw_buffer_store_b96(st, mer, rl0 ? mo + 16 : BUF_OOB, 0, 0);
  }

  const bool intra = mt_intra(mt), tc = mt_tcoeff(mt);
  const int q = f.q;
  const p64_qint qt = c_qint.ac[q], qd = c_qint.dc[q];
  // levels & tcm: 0 when the MB type carries no coefficients (through an
  // opaque mask: as a select hipcc branches around every quantisation)
  const uint32_t tcm = OVR ? (uint32_t)opaque(tc ? -1 : 0) : ~0u;
  // ChenDct of the residual, each row quantised right after its row pass and
  // kept as natural int16 level pairs L[r][j] = (x_r,2j, x_r,2j+1): 32
  // registers instead of 64 ints for the levels
  // BoundDct's clamp of the quantiser cannot act from q = 5 on (the level
  // bound then lies beyond it) when every AC |v| <= 8,187: for a residual
  // block |v| <= 1.9227 sum|r| + 8.56 (affine bound over this kernel's
  // butterfly, tests/test_intra_dct_bound.py), so sum|r| <= 4,253 suffices
  // (the DC's own bound, >= 10,235 from q = 5, is then far away too); an intra
  // MB's block is 8-bit pixels, 8,163.5 at most.  sum|r| is 16 v_sad_u8 of the
  // current rows against the prediction; where the whole wave qualifies (on
  // natural content nearly always) the quantiser runs without its v_med3.
  uint32_t sar = 0;
#pragma unroll
  for (int r = 0; r < 8; r++) sar = sad4(f.rows[r].y, prow[r].y, sad4(f.rows[r].x, prow[r].x, sar));
  const bool no_clamp = uni(__all(q >= 5 && (intra || sar <= 4253u)));
  uint32_t L[8][4];
  {
    s16x2 p[8][4];
    fdct_cols_pk<true>(f.rows, p, prow);
    auto rows = [&](auto clamp) {
      constexpr bool CL = decltype(clamp)::value;
      if (POW2) {  // level pairs straight from the packed row pass
        const uint32_t lo_ac = pk16u(qt.vlo, qt.vlo), hi_ac = pk16u(qt.vhi, qt.vhi);
        const uint32_t cp2 = pk16u(qt.cp, qt.cp), cn2 = pk16u(qt.cn, qt.cn);
#pragma unroll
        for (int r = 0; r < 8; r++) {
          uint32_t P[4];
          fwd_row_pk2(p[r], P);
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const bool dcp = r == 0 && j == 0;  // (DC, o1): the DC's own bounds in the low half
            L[r][j] = qlevel_pk2<CL>(P[j], dcp ? pk16u(qd.vlo, qt.vlo) : lo_ac, dcp ? pk16u(qd.vhi, qt.vhi) : hi_ac,
                                     cp2, cn2, qt.s);
          }
          if (r == 0) {  // intra DC: (DC +- 4) / 8 in 1..254 of the bounded DC (transform.c:321-325)
            const int dc = (int)(int16_t)(P[0] & 0xffffu);
            const int l0 = clampi(dct_final(min(dct_final(dc), 2047)), 1, 254);
            L[0][0] = intra ? (L[0][0] & 0xffff0000u) | (uint32_t)l0 : L[0][0];
          }
          SCHED_FENCE();
        }
        return;
      }
#pragma unroll
      for (int r = 0; r < 8; r++) {
        int o[8];
        fwd_row_pk(p[r], o);
#pragma unroll
        for (int k = 0; k < 8; k++) o[k] = opaque(o[k]);
        int l[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
          if (r == 0 && k == 0)  // DC: intra (DC +- 4) / 8 in 1..254, inter as AC with DC bounds
            l[k] = intra ? clampi(dct_final(min(dct_final(o[0]), 2047)), 1, 254) : qlevel_int<CL>(o[0], qd);
          else
            l[k] = qlevel_int<CL>(o[k], qt);
        }
#pragma unroll
        for (int j = 0; j < 4; j++) L[r][j] = pk2(l[2 * j], l[2 * j + 1]);
        SCHED_FENCE();
      }
    };
    if (no_clamp)
      rows(std::false_type{});
    else
      rows(std::true_type{});
  }
  // natural positions e (low half) and f (high half) as one pair
  auto lpair = [&](int e, int f) {
    const uint32_t sel = (uint32_t)(2 * (e & 1)) | ((uint32_t)(2 * (e & 1) + 1) << 8) |
                         ((uint32_t)(4 + 2 * (f & 1)) << 16) | ((uint32_t)(5 + 2 * (f & 1)) << 24);
    return __builtin_amdgcn_perm(L[f >> 3][(f & 7) >> 1], L[e >> 3][(e & 7) >> 1], sel);
  };
  // in scan order into the LDS staging (levels of a block whose MB type
  // carries no coefficients are 0); sum of l^2 for the CBP decision:
  // sum|l| > 1 <=> sum l^2 > 1 and sum|l| > 0 <=> sum l^2 > 0 for integers
  int ss = 0;
  uint32_t nzm[2] = {0u, 0u};  // (BITS) the nonzero scan positions
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      pk[j] = lpair(k_zz.inv[8 * k + 2 * j], k_zz.inv[8 * k + 2 * j + 1]);
      if (OVR) pk[j] &= tcm;
      ss = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, pk[j]), __builtin_bit_cast(s16x2, pk[j]), ss, false);
      if (BITS) nzm[k >> 2] |= nz2(pk[j]) << (2 * (4 * (k & 3) + j));
    }
    put_levels(lds, lane, k, make_uint4(pk[0], pk[1], pk[2], pk[3]));
    SCHED_FENCE();
  }
  // CBP (p64.c:887-908): block coded if sum|l| > 1; none such -> the first
  // block with a nonzero level; no nonzero level at all -> MC without
  // coefficients (MTYPE 4 / 7), vector kept, CBP 0x3f
  const int sh = 6 * (l / 6);
  const uint64_t nz = __ballot(ss > 0);  // blocks with a nonzero level
  const uint32_t big = (uint32_t)(__ballot(ss > 1) >> sh) & 63u, any = (uint32_t)(nz >> sh) & 63u;
  int cbp = 0x3f;
  bool repred = false;  // 2/3 -> 4 switches from the zero vector to the ME vector
  if (mt_cbp(mt)) {
    if (any == 0) {
      repred = !mt_mf(mt);
      mt = mt_filter(mt) ? 7 : 4;
    } else {
      const uint32_t sel = big ? big : (any & (0u - any));  // lane-bit b = block b
      cbp = (int)(__builtin_bitreverse32(sel) >> 26);           // block b -> bit 5 - b
    }
  }
  const bool ck = mt_tcoeff(mt) && ((cbp >> (5 - b)) & 1);
  if (BITS) {  // the transmitted block's coded bits, from its staged levels (before the slots reuse them)
    load_vlc_len(vt, vlen, lane);
    WAVE_FENCE();
    const int bb = ck ? block_vlc_bits(reinterpret_cast<const uint8_t *>(vlen),
                                       reinterpret_cast<const int16_t *>(lds + lane * LVL_STRIDE), nzm[0], nzm[1],
                                       mt_cbp(mt))
                      : 0;
    store_vlc_bits(a, nmbs, lane < 6 * MBS_PER_WAVE && gmb0 + (unsigned)(l / 6) < nmbs, gmb, b, bb);
  }
  // the levels as natural column pairs (unmasked: only coded blocks, whose MB
  // type carries coefficients, use them)
  uint32_t np[8][4];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    np[c][0] = lpair(c, 32 + c);
    np[c][1] = lpair(8 + c, 56 + c);
    np[c][2] = lpair(40 + c, 24 + c);
    np[c][3] = lpair(16 + c, 48 + c);
  }
  // the levels leave first: the staging then holds idct_coded_blocks' slots
  const uint32_t nvalid = min((unsigned)MBS_PER_WAVE, nmbs - gmb0);
  // only blocks with a nonzero level are written (include/p64gpu.h): three
  // quarters of the inter blocks have none (k_inter_mbg 49.1 -> 42.9 us, A/B x3)
  mbg_store_levels(a, lds, lane, nmbs, gmb0, nvalid, nz);
  const int pw = pos.plane ? w >> 1 : w;
  const uint32_t ro = (uint32_t)((int64_t)pos.fi * stride) + (uint32_t)plane_offset(pos.plane, w, h) +
                      (uint32_t)mul24(pos.y, pw) + (uint32_t)pos.x;
  // IQ + ChenIDct + reconstruction of the coded blocks, into their prow: a
  // wave with many coded blocks (SURVEY.md 8(d)'s content: 46 of 60 on
  // average) runs one block per lane in registers when every coded block is
  // an inter one whose levels keep the packed column pass exact (sum l^2 <=
  // the limit squared bounds max |l|); else the coded-block pass through LDS
  const int nck = __popcll(__ballot(ck));
  const bool lane_ok = !ck || (!intra && ss <= c_idct_lim.l2[q]);
  if (nck >= INTER_DIRECT_MIN && uni(__all(lane_ok))) {
    if (ck) iq_idct_inter_rec(np, q, prow);
  } else {
    idct_coded_blocks(ck, np, q, intra, prow, (uint32_t *)lds, lane);
  }
  // no levels at all in the MB: the reconstruction is the new prediction
  if (repred) inter_pred(B, w, h, stride, pos, mt, mvx, mvy, prow);
  // p64.c:909-910: the record (transmitted vector only for MC types) and LastIntra
  const bool rl = b == 0 && lane < 6 * MBS_PER_WAVE && gmb0 + (unsigned)(l / 6) < nmbs;
  const uint32_t mbw = (uint32_t)(mt & 0xff) | ((uint32_t)(cbp & 0xff) << 8) |
                       (mt_mf(mt) ? ((uint32_t)(mvx & 0xff) << 16) | ((uint32_t)(mvy & 0xff) << 24) : 0u);
  // every block: the reconstruction (coded) or the prediction (uncoded); the
  // MB's nonzero-block mask (block b -> bit 5 - b, as the CBP)
  mbg_store_rows(a, kd, nmbs, ro, pw, prow, rl, gmb, mbw,
                 mt_intra(mt) ? (uint8_t)0 : (uint8_t)(li + 1), __builtin_bitreverse32(any) >> 26);
}

}  // namespace

namespace p64k {

static unsigned mbg_workgroups(unsigned nmbs, unsigned per = MBG_WAVES) {
  const unsigned waves = (nmbs + MBS_PER_WAVE - 1) / MBS_PER_WAVE;
  return (waves + per - 1) / per;
}

// the instance of k_intra_mbg for the call's options: <QMB, CLAMP, POW2, BITS>
template <bool BITS>
static void intra_launch(const p64gpu_encode_args &a, const uint32_t *vt, dim3 grid, dim3 block, BlkDiv kd,
                         unsigned nm, hipStream_t st) {
  const bool pow2 = !a.quant_mb && (a.quant & (a.quant - 1)) == 0 && make_qint_tab().ac[a.quant].m == 1;
  if (a.quant_mb)
    hipLaunchKernelGGL((k_intra_mbg<true, true, false, BITS>), grid, block, 0, st, a, kd, nm, vt);
  else if (a.quant >= 5 && pow2)  // no BoundDct clamp can act (intra_block), packed quantiser
    hipLaunchKernelGGL((k_intra_mbg<false, false, true, BITS>), grid, block, 0, st, a, kd, nm, vt);
  else if (a.quant >= 5)
    hipLaunchKernelGGL((k_intra_mbg<false, false, false, BITS>), grid, block, 0, st, a, kd, nm, vt);
  else if (pow2)
    hipLaunchKernelGGL((k_intra_mbg<false, true, true, BITS>), grid, block, 0, st, a, kd, nm, vt);
  else
    hipLaunchKernelGGL((k_intra_mbg<false, true, false, BITS>), grid, block, 0, st, a, kd, nm, vt);
}

hipError_t intra_mbg(const p64gpu_encode_args &a, const uint32_t *vlc_len, hipStream_t st) {
  const unsigned nm = (unsigned)((int64_t)a.nframes * (a.width / 16) * (a.height / 16));
  const unsigned waves = (6u * nm + 63u) / 64u;  // 64 blocks a wave
  const dim3 grid((waves + MBG_WAVES - 1) / MBG_WAVES), block(64 * MBG_WAVES);
  const BlkDiv kd = blk_div(a.width, a.height);
  if (a.vlc_bits)  // vlc_len: the count's table in device memory (p64gpu_vlc_len_dev_)
    intra_launch<true>(a, vlc_len, grid, block, kd, nm, st);
  else
    intra_launch<false>(a, nullptr, grid, block, kd, nm, st);
  return hipGetLastError();
}

template <bool BITS>
static void inter_launch(const p64gpu_encode_args &a, p64_me_rec *me, const uint32_t *vt, dim3 grid,
                         dim3 block, BlkDiv kd, unsigned nm, hipStream_t st) {
  const bool ovr = a.mtype_override != nullptr;
  // a uniform q with D = 16q a power of two: the packed quantiser (multiplier 1)
  const bool pow2 = !a.quant_mb && (a.quant & (a.quant - 1)) == 0 && make_qint_tab().ac[a.quant].m == 1 &&
                    make_qint_tab().dc[a.quant].m == 1;
  if (a.quant_mb && ovr)
    hipLaunchKernelGGL((k_inter_mbg<true, true, false, BITS>), grid, block, 0, st, a, kd, nm, me, vt);
  else if (a.quant_mb)
    hipLaunchKernelGGL((k_inter_mbg<true, false, false, BITS>), grid, block, 0, st, a, kd, nm, me, vt);
  else if (ovr && pow2)
    hipLaunchKernelGGL((k_inter_mbg<false, true, true, BITS>), grid, block, 0, st, a, kd, nm, me, vt);
  else if (ovr)
    hipLaunchKernelGGL((k_inter_mbg<false, true, false, BITS>), grid, block, 0, st, a, kd, nm, me, vt);
  else if (pow2)
    hipLaunchKernelGGL((k_inter_mbg<false, false, true, BITS>), grid, block, 0, st, a, kd, nm, me, vt);
  else
    hipLaunchKernelGGL((k_inter_mbg<false, false, false, BITS>), grid, block, 0, st, a, kd, nm, me, vt);
}

hipError_t inter_mbg(const p64gpu_encode_args &a, p64_me_rec *me, const uint32_t *vlc_len, hipStream_t st) {
  const unsigned nm = (unsigned)((int64_t)a.nframes * (a.width / 16) * (a.height / 16));
  const dim3 grid(mbg_workgroups(nm, 1)), block(64);
  const BlkDiv kd = blk_div(a.width, a.height);
  if (a.vlc_bits)
    inter_launch<true>(a, me, vlc_len, grid, block, kd, nm, st);
  else
    inter_launch<false>(a, me, nullptr, grid, block, kd, nm, st);
  return hipGetLastError();
}

hipError_t recon_mbg(int w, int h, int nframes, int64_t stride, const uint8_t *ref, uint8_t *recon,
                     const int16_t *coef, const p64_mb_rec *mb, const uint8_t *quant_mb,
                     const uint8_t *coded_mask, hipStream_t st) {
  const unsigned nm = (unsigned)((int64_t)nframes * (w / 16) * (h / 16));
  hipLaunchKernelGGL(k_recon_mbg, dim3((6u * nm + 63u) / 64u), dim3(64), 0, st, w, h, stride, ref, recon,
                     coef, mb, quant_mb, coded_mask, blk_div(w, h), nm);
  return hipGetLastError();
}

hipError_t recon_pk(int w, int h, int nframes, int64_t stride, const uint8_t *ref, uint8_t *recon,
                    const int16_t *levels, uint32_t nlev, const uint32_t *index, const p64_mb_rec *mb,
                    const uint8_t *quant_mb, const uint8_t *coded_mask, hipStream_t st) {
  const unsigned nm = (unsigned)((int64_t)nframes * (w / 16) * (h / 16));
  hipLaunchKernelGGL(k_recon_pk, dim3((6u * nm + 63u) / 64u), dim3(64), 0, st, w, h, stride, ref, recon, levels,
                     nlev, index, mb, quant_mb, coded_mask, blk_div(w, h), nm);
  return hipGetLastError();
}

}  // namespace p64k
