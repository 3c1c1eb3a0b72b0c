// common.h -- device-side building blocks shared by the kernel families of
// libp64gpu (MI355X / gfx950): MTYPE predicates, the Chen DCT butterflies
// (chendct.c:97-375), the H.261 quantisers (transform.c:271-451), wave
// reductions by DPP, the magic-number divisions that map a launch index to
// (picture, macroblock, block), and the MTYPE decision (p64.c:734-756).
// Everything here is inline device code or a host-side constant helper; each
// kernel translation unit (k_search.hip, k_block.hip, k_aux.hip) includes it.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/p64gpu.h"

// phase labels of the search kernels: no code; the development tools
// (tools/me_stamps.py, tools/me_variants.py, tools/section_census.py) rewrite
// them in a copy of the source into timestamps or ISA markers
#define SECTION(name)

namespace {

// ---------------------------------------------------------------------------
// coding-control tables (p64.c:217-222) as predicates on MTYPE 0..9

__host__ __device__ constexpr bool mt_intra(int m) { return m < 2; }
__host__ __device__ constexpr bool mt_cbp(int m) {
  return m == 2 || m == 3 || m == 5 || m == 6 || m == 8 || m == 9;
}
__host__ __device__ constexpr bool mt_mf(int m) { return m >= 4; }
__host__ __device__ constexpr bool mt_filter(int m) { return m >= 7; }
__host__ __device__ constexpr bool mt_tcoeff(int m) { return m != 4 && m != 7; }

// zigzag scan position of natural index n (transform.c:67-75), generated
struct ZigZag {
  uint8_t pos[64];  // natural index -> scan position
  uint8_t inv[64];  // scan position -> natural index
};
constexpr ZigZag make_zigzag() {
  ZigZag z{};
  int k = 0;
  for (int s = 0; s < 15; s++) {
    int lo = s < 8 ? 0 : s - 7, hi = s < 8 ? s : 7;
    if (s & 1)
      for (int r = lo; r <= hi; r++) z.pos[8 * r + s - r] = (uint8_t)k++;
    else
      for (int r = hi; r >= lo; r--) z.pos[8 * r + s - r] = (uint8_t)k++;
  }
  for (int n = 0; n < 64; n++) z.inv[z.pos[n]] = (uint8_t)n;
  return z;
}
__constant__ ZigZag c_zz = make_zigzag();

// ---------------------------------------------------------------------------
// Chen integer DCT of one 8-point line (chendct.c:97-375).
// NARROW = operands proven < 2^23 (fused kernels): full-rate v_mul_i32_i24;
// otherwise (block-op API, arbitrary int32) the 32-bit multiply.

constexpr int C1D4 = 362, C1D8 = 473, C3D8 = 196, C1D16 = 502, C3D16 = 426,
              C5D16 = 284, C7D16 = 100;

template <bool NARROW>
__device__ __forceinline__ int kmul(int c, int v) {
  return NARROW ? __mul24(c, v) : c * v;
}
__device__ __forceinline__ int ms9(int v) { return v >> 9; }  // MSCALE, arithmetic

// 24-bit constant products as the instructions themselves: hipcc turns some
// __mul24 of the forward column pass (sums of sums of bytes, <<2) into the
// quarter-rate v_mul_lo_u32, having lost the operand range on the way
template <int C>
__device__ __forceinline__ int mul_c(int v) {
  int r;
  asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "i"(C), "v"(v));
  return r;
}
template <int C>
__device__ __forceinline__ int mad_c(int v, int acc) {  // C v + acc
  int r;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(v), "s"(C), "v"(acc));
  return r;
}

// forward butterfly on scaled sums s[k] and differences d[k] (chendct.c:135-159).
// S: the scale the caller left out of s and d (the column pass's <<2,
// chendct.c:120-133): every s and the d[1], d[2] terms only meet constant
// multiplies, so S folds into the constants (same bits mod 2^32); d[0] and
// d[3] are added to products, so they take the shift themselves
template <bool N, int S = 1>
__device__ __forceinline__ void fwd8(const int s[4], const int d[4], int o[8]) {
  static_assert(S == 1 || S == 4, "scale");
  constexpr int L = S == 4 ? 2 : 0;
  const int e0 = s[0] + s[3], e1 = s[1] + s[2], e2 = s[1] - s[2], e3 = s[0] - s[3];
  const int d0 = d[0] << L, d3 = d[3] << L;
  if (N) {  // operands proven < 2^23 (callers: pixels or residuals)
    o[0] = ms9(mul_c<S * C1D4>(e0 + e1));
    o[4] = ms9(mul_c<S * C1D4>(e0 - e1));
    o[2] = ms9(mad_c<S * C3D8>(e2, mul_c<S * C1D8>(e3)));
    o[6] = ms9(mad_c<S * C3D8>(e3, mul_c<-S * C1D8>(e2)));
    const int r0 = ms9(mul_c<S * C1D4>(d[1] - d[2])), r1 = ms9(mul_c<S * C1D4>(d[1] + d[2]));
    const int u0 = d3 + r0, u1 = d3 - r0, u2 = d0 - r1, u3 = d0 + r1;
    o[1] = ms9(mad_c<C7D16>(u0, mul_c<C1D16>(u3)));
    o[3] = ms9(mad_c<C3D16>(u2, mul_c<-C5D16>(u1)));
    o[5] = ms9(mad_c<C3D16>(u1, mul_c<C5D16>(u2)));
    o[7] = ms9(mad_c<C7D16>(u3, mul_c<-C1D16>(u0)));
    return;
  }
  o[0] = ms9(kmul<N>(S * C1D4, e0 + e1));
  o[4] = ms9(kmul<N>(S * C1D4, e0 - e1));
  o[2] = ms9(kmul<N>(S * C3D8, e2) + kmul<N>(S * C1D8, e3));
  o[6] = ms9(kmul<N>(S * C3D8, e3) - kmul<N>(S * C1D8, e2));
  const int r0 = ms9(kmul<N>(S * C1D4, d[1] - d[2])), r1 = ms9(kmul<N>(S * C1D4, d[1] + d[2]));
  const int u0 = d3 + r0, u1 = d3 - r0, u2 = d0 - r1, u3 = d0 + r1;
  o[1] = ms9(kmul<N>(C7D16, u0) + kmul<N>(C1D16, u3));
  o[3] = ms9(kmul<N>(C3D16, u2) - kmul<N>(C5D16, u1));
  o[5] = ms9(kmul<N>(C3D16, u1) + kmul<N>(C5D16, u2));
  o[7] = ms9(kmul<N>(C7D16, u3) - kmul<N>(C1D16, u0));
}

// column pass: sums/differences scaled <<2 (chendct.c:120-133), the scale
// folded into fwd8
template <bool N>
__device__ __forceinline__ void fwd_col(const int x[8], int o[8]) {
  int s[4], d[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    s[k] = x[k] + x[7 - k];
    d[k] = x[k] - x[7 - k];
  }
  fwd8<N, 4>(s, d, o);
}
// row pass: sums/differences >>1 (chendct.c:167-174)
template <bool N>
__device__ __forceinline__ void fwd_row(const int x[8], int o[8]) {
  int s[4], d[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    s[k] = (x[k] + x[7 - k]) >> 1;
    d[k] = (x[k] - x[7 - k]) >> 1;
  }
  fwd8<N>(s, d, o);
}

// inverse butterfly (chendct.c:254-303 == 320-365).  S scales the inputs: the
// column pass takes them <<2 (chendct.c:235-243); every input only meets a
// constant multiply, so the shift folds into the constants (same bits mod 2^32)
template <bool N, int S = 1>
__device__ __forceinline__ void inv8(const int x[8], int o[8]) {
  const int p0 = ms9(kmul<N>(S * C7D16, x[1]) - kmul<N>(S * C1D16, x[7]));
  const int p1 = ms9(kmul<N>(S * C3D16, x[5]) - kmul<N>(S * C5D16, x[3]));
  const int p2 = ms9(kmul<N>(S * C3D16, x[3]) + kmul<N>(S * C5D16, x[5]));
  const int p3 = ms9(kmul<N>(S * C1D16, x[1]) + kmul<N>(S * C7D16, x[7]));
  const int q0 = ms9(kmul<N>(S * C1D4, x[0] + x[4])), q1 = ms9(kmul<N>(S * C1D4, x[0] - x[4]));
  const int q2 = ms9(kmul<N>(S * C3D8, x[2]) - kmul<N>(S * C1D8, x[6]));
  const int q3 = ms9(kmul<N>(S * C1D8, x[2]) + kmul<N>(S * C3D8, x[6]));
  const int e0 = q0 + q3, e1 = q1 + q2, e2 = q1 - q2, e3 = q0 - q3;
  const int f0 = p0 + p1, f1 = p0 - p1, f2 = p3 - p2, f3 = p3 + p2;
  const int g1 = ms9(kmul<N>(C1D4, f2 - f1)), g2 = ms9(kmul<N>(C1D4, f2 + f1));
  o[0] = e0 + f3;
  o[1] = e1 + g2;
  o[2] = e2 + g1;
  o[3] = e3 + f0;
  o[4] = e3 - f0;
  o[5] = e2 - g1;
  o[6] = e1 - g2;
  o[7] = e0 - f3;
}

// (v < 0 ? v - h : v + h) / 2h with C truncation == (v + h - [v < 0]) >> k for
// h = 2^(k-1): one add3 and two shifts instead of a select and a signed divide
// (v >= 0: floor((v+h)/2^k); v < 0: ceil((v-h)/2^k) = floor((v+h-1)/2^k))
__device__ __forceinline__ int dct_final(int v) { return (v + 4 + (v >> 31)) >> 3; }   // chendct.c:204
__device__ __forceinline__ int idct_final(int v) { return (v + 8 + (v >> 31)) >> 4; }  // chendct.c:373
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }
// Per-lane row offsets on the 24-bit multiplier: both factors are below 2^23
// (pictures are at most 4096 x 4096, check_geometry) and the product below
// 2^25; a plain int product of two vector values is the quarter-rate v_mul_lo.
__device__ __forceinline__ int mul24(int a, int b) { return __mul24(a, b); }
// byte offset of plane 0/1/2 in a 4:2:0 picture (selects of uniform values)
__device__ __forceinline__ int plane_offset(int plane, int w, int h) {
  const int wh = w * h;
  return plane == 0 ? 0 : (plane == 1 ? wh : wh + (wh >> 2));
}

// ---------------------------------------------------------------------------
// quantisers (transform.c:271-451, non-VERSION_1_0)

// Truncating c / 2q.  In the fused kernels |c| <= 2048 (BoundDctMatrix plus
// the +-1 of even q): there (int)(c * r) in binary32, r = 1/(2q) rounded and
// then raised one ulp, equals C's c / (2q) for every q = 1..31 (|c| <= 4096:
// tests/test_quant_recip.py checks it exhaustively); the block-op path
// handles arbitrary int32 with a true division.
struct QuantRecip {
  float r[32];
};
constexpr QuantRecip make_quant_recip() {
  QuantRecip t{};
  for (int q = 1; q < 32; q++)
    t.r[q] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, 1.0f / (float)(2 * q)) + 1u);
  return t;
}
__constant__ QuantRecip c_qrecip = make_quant_recip();

// H.261 level: odd q -> c/(2q); even q -> (c + sign(c))/(2q), sign(0) = -1
// (transform.c:283-306, 339-347)
__device__ __forceinline__ int qlevel(int c, int q) {
  if (!(q & 1)) c += c > 0 ? 1 : -1;
  return c / (2 * q);
}
// intra DC (transform.c:321-325): (DC +- dcq/2) / dcq, sign by DC > 0
__device__ __forceinline__ int qdc_intra(int c, int dcq) {
  return c > 0 ? (c + dcq / 2) / dcq : (c - dcq / 2) / dcq;
}
// reconstruction level (transform.c:376-389, 436-448)
template <bool NARROW>
__device__ __forceinline__ int rlevel(int l, int q) {
  if (l == 0) return 0;
  const int sg = l > 0 ? 1 : -1;
  int v = kmul<NARROW>(2 * l + sg, q);
  if (!(q & 1)) v -= sg;
  return v;
}


// ---------------------------------------------------------------------------
// wave helpers

// Wave reductions without the LDS crossbar: DPP folds each 16-lane row
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then the four
// row results are combined in scalar registers.  The result is wave-uniform.
// (CTRL: full permutations only -- quad_perm, row_half_mirror, row_mirror --
// so every lane has a source and bound_ctrl changes nothing; with it the
// compiler needs no zeroed destination first: one v_mov fewer per use that
// is not fused into its consumer)
template <int CTRL>
__device__ __forceinline__ unsigned dpp(unsigned v) {
  static_assert((CTRL >= 0 && CTRL <= 0xFF) || CTRL == 0x140 || CTRL == 0x141, "full permutations only");
  return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}
// after the row folds every lane of a row holds the row's result; row_bcast:15
// (rows 1 and 3 take lane 15 of rows 0 and 2) and row_bcast:31 (rows 2 and 3
// take lane 31) finish the wave in lane 63 -- one v_readlane instead of four
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp_rows(unsigned old, unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ unsigned wave_min(unsigned v) {
  v = min(v, dpp<0xB1>(v));
  v = min(v, dpp<0x4E>(v));
  v = min(v, dpp<0x141>(v));
  v = min(v, dpp<0x140>(v));
  v = min(v, dpp_rows<0x142, 0xa>(0xFFFFFFFFu, v));
  v = min(v, dpp_rows<0x143, 0xc>(0xFFFFFFFFu, v));
  return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ int wave_sum(int v) {
  unsigned u = (unsigned)v;
  u += dpp<0xB1>(u);
  u += dpp<0x4E>(u);
  u += dpp<0x141>(u);
  u += dpp<0x140>(u);
  u += dpp_rows<0x142, 0xa>(0u, u);
  u += dpp_rows<0x143, 0xc>(0u, u);
  return __builtin_amdgcn_readlane((int)u, 63);
}
// a value the compiler cannot see through (nor hoist out of a loop)
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
// wave-uniform by construction (results of wave reductions); saying so lets
// hipcc use scalar registers and scalar branches for everything that follows
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// LDS pointer in the LDS address space: stores through it cannot alias global
// memory, so later uniform global loads stay scalar (s_load)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ lds_u32 *as_lds(uint32_t *p) { return (lds_u32 *)p; }
__device__ __forceinline__ uint32_t sad4(uint32_t a, uint32_t b, uint32_t acc) {
  return __builtin_amdgcn_sad_u8(a, b, acc);
}
__device__ __forceinline__ uint32_t align4(uint32_t hi, uint32_t lo, int shift) {
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)shift);
}
// value of lane-1 / lane+1 inside the 16-lane DPP row (row_shr:1 / row_shl:1)
// (bound_ctrl: a lane without a source reads 0, so `x + from_prev_lane(v)`
// fuses into one v_add_u32_dpp)
__device__ __forceinline__ int from_prev_lane(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ int from_next_lane(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x101, 0xf, 0xf, true);
}

// workgroup id -> macroblock id, bijective, so that ids sharing an XCD
// (blockIdx % 8 under round-robin dispatch) get contiguous macroblocks and
// neighbouring search windows meet in the same L2 (speed only, never
// correctness: cdna_hip_programming.md T1)
__device__ __forceinline__ unsigned xcd_remap(unsigned bid, unsigned n) {
  const unsigned q = n >> 3, r = n & 7, x = bid & 7, k = bid >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// macroblock index -> (picture, MB, MB column, MB row) without integer
// division (a runtime divide is ~25 scalar instructions): q = umulhi(n, m) >> s
// with s = floor(log2 d) - 1 and m = floor(2^(32+s)/d) + 1 < 2^32 is exact for
// n < 2^30 and 2 <= d <= 65536, since the excess n (m - 2^(32+s)/d) / 2^(32+s)
// stays below 1/d.  check_geometry keeps n < 2^30.
struct MbDiv {
  uint32_t mn, sn, mw, sw;  // magic and shift for nmb and for mbw
};
static inline MbDiv mb_div(int w, int h) {
  auto magic = [](uint32_t d, uint32_t &m, uint32_t &s) {
    s = 31 - (uint32_t)__builtin_clz(d);
    s = s ? s - 1 : 0;
    m = (uint32_t)((((uint64_t)1) << (32 + s)) / d + 1);
  };
  MbDiv k;
  magic((uint32_t)((w >> 4) * (h >> 4)), k.mn, k.sn);
  magic((uint32_t)(w >> 4), k.mw, k.sw);
  return k;
}
struct MbPos {
  int fi, mb, mbx, mby;
};
__device__ __forceinline__ MbPos mb_pos(unsigned gid, int nmb, int mbw, const MbDiv &k) {
  MbPos p;
  p.fi = (int)(__umulhi(gid, k.mn) >> k.sn);
  p.mb = (int)(gid - (unsigned)p.fi * (unsigned)nmb);
  p.mby = (int)(__umulhi((unsigned)p.mb, k.mw) >> k.sw);
  p.mbx = p.mb - p.mby * mbw;
  return p;
}
struct Picture {  // one planar 4:2:0 picture
  const uint8_t *y, *u, *v;
};
__device__ __forceinline__ Picture picture_at(const uint8_t *base, int w, int h) {
  Picture p;
  p.y = base;
  p.u = base + (size_t)w * h;
  p.v = p.u + (size_t)(w / 2) * (h / 2);
  return p;
}
struct MeOut {
  int mx, my, sad, sad0, var, varor, mwor;
};
// MTYPE decision (p64.c:734-756).  xv = sad0/256 and yv = sad/256 are exact
// in binary64, so xv < 1, xv < 3 and yv > xv*0.5 are integer tests; yv >
// xv/1.1 is 11 sad > 10 sad0 unless the two are equal (the double quotient's
// error, < 2e-11, cannot cross a gap of 1/11 otherwise), and on equality the
// rounded quotient decides, computed as written.
// the inter-without-MC test of the decision (p64.c:745-753): from the two
// SADs alone, so a caller can act on it before VAR / VAROR are known
__device__ __forceinline__ bool decide_inter(int sad, int sad0) {
  bool inter = sad0 < 256 || (sad0 < 768 && 2 * sad > sad0);
  if (!inter) {
    const int t = 11 * sad - 10 * sad0;
    inter = t != 0 ? t > 0 : (double)sad / 256 > ((double)sad0 / 256) / 1.1;
  }
  return inter;
}
__device__ __forceinline__ int decide_mtype(const MeOut &m) {
  if (m.var < 64 || m.varor > m.var) {
    if (decide_inter(m.sad, m.sad0)) return 2;
    return m.var < 6 ? 5 : 8;  // VAR < D_FILTERTHRESHOLD (6.0)
  }
  return 0;
}

// ---------------------------------------------------------------------------
// prediction (io.c:142-496), row layout: lane (b, r) computes row r of block b.
// The 8 source bytes of the row arrive packed in (lo, hi).

__device__ __forceinline__ void unpack8(uint32_t lo, uint32_t hi, int v[8]) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    v[k] = (lo >> (8 * k)) & 255;
    v[4 + k] = (hi >> (8 * k)) & 255;
  }
}
// Values are taken through an empty asm (opaque) first: on ROCm 7.2 hipcc fuses
// "(x >> 4) clamped to 0..255, packed" into gfx950's v_ashr_pk_u8_i32 and then
// ORs the packed pair into a dword whose upper half it assumes is zero, which
// corrupted byte 3 on the hardware (tools/repro_ashr_pk.hip); the barrier keeps
// the clamp and the pack as separate instructions.
__device__ __forceinline__ uint2 pack8(const int in[8]) {
  int v[8];
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = opaque(in[k]);
  uint2 q;
  q.x = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
  q.y = (uint32_t)v[4] | ((uint32_t)v[5] << 8) | ((uint32_t)v[6] << 16) | ((uint32_t)v[7] << 24);
  return q;
}
// compensated block geometry (MoveTo io.c:719-747): luma MV, chroma MV/2 with
// C truncation (io.c:268-270), zero vector for non-MC types
struct BlockGeom {
  int plane;  // 0 Y, 1 U, 2 V
  int x, y;   // block origin in its plane
};
__device__ __forceinline__ BlockGeom block_geom(int b, int mbx, int mby) {
  BlockGeom g;
  if (b < 4) {
    g.plane = 0;
    g.x = 16 * mbx + 8 * (b & 1);
    g.y = 16 * mby + 8 * (b >> 1);
  } else {
    g.plane = b - 3;
    g.x = 8 * mbx;
    g.y = 8 * mby;
  }
  return g;
}
// BoundDctMatrix + CCITT(Flat)Quantize + (Flat)BoundQuantizeMatrix of one raw
// coefficient (transform.c:271-350, 460-537), branch-free.  lo/hi: the lane's
// BoundDct range (DC: no lower bound, <= 2047; AC: +-1023).  The even-q step
// c + sign(c) (sign(0) = -1, transform.c:285) is folded into one fma: with
// s = copysign(rqe, c), rqe = rq for even q and 0 for odd q, fma(c, rq, s) is
// the one rounding of the exact (c + sign c) * rq that the reference division
// truncates (c_qrecip: trunc of that product == C's c / 2q; for c = 0 both
// give 0).  INTRA selects the flat DC quantiser (dc: lane holds the DC).
// TIGHT: the caller's AC bounds are already +-quant_bound(q), which makes the
// +-127 level clamp redundant (quant_bound).
template <bool INTRA, bool TIGHT = false>
__device__ __forceinline__ int quantise(int raw, int lo, int hi, bool dc, float rq, float rqe) {
  int v;  // clamp to [lo, hi] (per-lane bounds: one v_med3 instead of max + min)
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(v) : "v"(dct_final(raw)), "v"(lo), "v"(hi));
  const float x = (float)v;
  int l = (int)__builtin_fmaf(x, rq, __builtin_copysignf(rqe, x));
  if (!TIGHT) l = clampi(l, -127, 127);
  if (INTRA) l = dc ? clampi(dct_final(v), 1, 254) : l;  // (DC +- 4) / 8, transform.c:321-325
  return l;
}
// ICCITT(Flat)Quantize of one level (transform.c:359-451), branch-free: with
// sg = sign(l) (0 for l = 0) the reconstruction (2l + sg) q, minus sg for even
// q, is l * q2 + sg * qq with q2 = 2q and qq = q - [q even]; 0 stays 0.  An
// uncoded block passes q2 = qq = 0 (uniform per block).  Intra DC: DC * 8.
// The quantiser l(c) = trunc((c + [q even] sign c) / 2q) is odd and monotone,
// l(256q - 1 - e) = 127 and l(256q - e) = 128 (e = [q even]): clamping c to
// +-min(1023, 256q - 1 - e) before it gives exactly clamp(l(clamp(c, +-1023)),
// +-127), with one v_med3 instead of two.
__device__ __forceinline__ int quant_bound(int q) { return min(1023, 256 * q - 1 - (int)!(q & 1)); }
// MED3: sign(l) as one v_med3 (clampi compiles to two compares + two selects
// on a 32-bit l; on int16 levels straight from memory the compares take the
// half-word by SDWA for free, so the decoder keeps clampi)
template <bool INTRA, bool MED3 = false>
__device__ __forceinline__ int dequantise(int l, bool dc, int q2, int qq) {
  int sg, v;
  if (MED3) {  // the 24-bit multiplies spelled out: behind the asm sign hipcc
               // loses the operand ranges and falls back to v_mad_u64_u32
    asm("v_med3_i32 %0, %1, -1, 1" : "=v"(sg) : "v"(l));
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(v) : "v"(sg), "v"(qq));
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(v) : "v"(l), "v"(q2), "v"(v));
  } else {
    sg = clampi(l, -1, 1);
    v = __mul24(l, q2) + __mul24(sg, qq);
  }
  if (INTRA) v = dc ? l * 8 : v;
  return v;
}

// dequantise for two int16 levels at once (decoder): packed 16-bit
// arithmetic is exact for |level| <= 528 (|l q2 + sg qq| <= 528 * 62 + 31 <
// 2^15); H.261 levels are at most 127 in magnitude (escape: 8-bit signed) and
// the intra DC, at most 254, is handled by the caller.  q2/qq packed pairs.
__device__ __forceinline__ uint32_t dequantise_pk(uint32_t l, uint32_t q2, uint32_t qq) {
  uint32_t sg, m, r;
  asm("v_pk_min_i16 %0, %1, %2" : "=v"(sg) : "v"(l), "s"(0x00010001u));
  asm("v_pk_max_i16 %0, %1, %2" : "=v"(sg) : "v"(sg), "s"(0xffffffffu));
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(m) : "v"(l), "v"(q2));  // q2, qq per lane (per MB)
  asm("v_pk_mad_i16 %0, %1, %2, %3" : "=v"(r) : "v"(sg), "v"(qq), "v"(m));
  return r;
}
struct BlkDiv {
  uint32_t mp, sp;  // picture: 6 nmb blocks
  uint32_t mb, sb;  // luma block row: w/8 blocks
  uint32_t mw, sw;  // MB row: w/16 MBs
  uint32_t mn, sn;  // picture: nmb MBs
};
static inline void magic_div(uint32_t d, uint32_t &m, uint32_t &s) {
  s = 31 - (uint32_t)__builtin_clz(d);
  s = s ? s - 1 : 0;
  m = (uint32_t)((((uint64_t)1) << (32 + s)) / d + 1);
}
static inline BlkDiv blk_div(int w, int h) {
  BlkDiv k;
  magic_div((uint32_t)(6 * (w >> 4) * (h >> 4)), k.mp, k.sp);
  magic_div((uint32_t)(w >> 3), k.mb, k.sb);
  magic_div((uint32_t)(w >> 4), k.mw, k.sw);
  magic_div((uint32_t)((w >> 4) * (h >> 4)), k.mn, k.sn);
  return k;
}
__device__ __forceinline__ unsigned mdiv(unsigned n, uint32_t m, uint32_t s) { return __umulhi(n, m) >> s; }

// dword 3 of a raw buffer resource on gfx9-family parts (CDNA): 32-bit data format
constexpr int BUF_RSRC_W3 = 0x00020000;
constexpr uint32_t BUF_OOB = 0x80000000u;  // >= every buffer's num_records: loads 0, stores dropped

// MB-grouped block layout (k_block.hip): a wave takes 10 consecutive
// macroblocks, lane 6m + b block b of its m-th MB (lanes 60..63 idle)
constexpr int MBS_PER_WAVE = 10;
// waves per workgroup of k_intra_mbg (each wave is independent; one-wave
// groups cost it 3 us)
constexpr unsigned MBG_WAVES = 4u;

}  // namespace
