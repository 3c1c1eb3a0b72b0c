// p64gpu.hip -- MI355X (gfx950) kernels and C ABI for the PVRG-P64 macroblock
// encode hot path.  See include/p64gpu.h for the interface and DESIGN.md for
// the data layout and rooflines.
//
// Execution model: one 64-lane wavefront (one workgroup) per macroblock.
//   * the 16x16 current luma block and a 46x48-byte window of the previous
//     reconstruction around it are staged in LDS with 16-byte loads;
//   * FULL search: lane = (dx, dy-half), 15 candidates per lane; a lower bound
//     on every candidate's SAD from 4x4 sub-block averages (v_lerp_u8 map, four
//     v_sad_u8 per candidate) prunes all but a handful, which get full SADs;
//     low-contrast blocks, where nothing prunes, take the dense exhaustive pass
//     (window rows slid past current rows held in SGPRs).  The argmin is one
//     wave-wide min over packed (SAD, scan-order) keys, reproducing FastBME's
//     first-minimum rule;
//   * TSS: lane = (candidate, row pair); four dependent steps of 8 candidates;
//   * encode: "row" layout lane = (block, row) for the prediction, the loop
//     filter (vertical taps exchanged with DPP) and the Chen row/column passes;
//     "element" layout lane = coefficient for quantisation, zigzag, CBP (wave
//     ballots) and dequantisation; the layouts exchange through LDS.
// All arithmetic is integer except the MTYPE decision, which is evaluated in
// IEEE binary64 exactly as p64.c:745-756 writes it.  Products whose operands
// are provably below 2^23 use the full-rate 24-bit multiplier.

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "../../include/p64gpu.h"

#define SYNTH_FN __host__ __device__ static inline
#include "synth_impl.h"

namespace {

// development aid: -DP64_SECTIONS marks kernel phases in the ISA listing
// (tools/section_census.py counts instructions per phase)
#if defined(P64_TIMING)
// -DP64_TIMING: each SECTION() stores the wave's s_memtime offset from its
// start into a per-wave slot of g_phase_buf (tools/phase_times.py)
__device__ uint32_t *g_phase_buf;
__shared__ uint64_t g_tm_t0;
__shared__ uint32_t g_tm_gid;
__device__ __forceinline__ void p64_stamp(int k) {
  const uint64_t now = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && g_phase_buf && g_tm_gid < gridDim.x)  // (kernels without TIMING_BEGIN)
    g_phase_buf[(size_t)g_tm_gid * 32 + k] = (uint32_t)(now - g_tm_t0);
}
#define SECTION(name) p64_stamp(__COUNTER__)
#define TIMING_BEGIN(gid)                                      \
  do {                                                         \
    if (threadIdx.x == 0) {                                    \
      g_tm_t0 = __builtin_amdgcn_s_memtime();                  \
      g_tm_gid = (gid);                                        \
    }                                                          \
    __syncthreads();                                           \
  } while (0)
#define TIMING_END() p64_stamp(31)
#elif defined(P64_SECTIONS)
#define SECTION(name) asm volatile(";## " name)
#else
#define SECTION(name)
#endif
#ifndef TIMING_BEGIN
#define TIMING_BEGIN(gid)
#define TIMING_END()
#endif

// ---------------------------------------------------------------------------
// error reporting

thread_local char g_err[512];

int fail(int status, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return status;
}

#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess)                                                    \
      return fail(P64GPU_E_HIP, "%s: %s", #expr, hipGetErrorString(e_));     \
  } while (0)

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

// forward butterfly on scaled sums s[k] and differences d[k] (chendct.c:135-159)
template <bool N>
__device__ __forceinline__ void fwd8(const int s[4], const int d[4], int o[8]) {
  const int e0 = s[0] + s[3], e1 = s[1] + s[2], e2 = s[1] - s[2], e3 = s[0] - s[3];
  o[0] = ms9(kmul<N>(C1D4, e0 + e1));
  o[4] = ms9(kmul<N>(C1D4, e0 - e1));
  o[2] = ms9(kmul<N>(C3D8, e2) + kmul<N>(C1D8, e3));
  o[6] = ms9(kmul<N>(C3D8, e3) - kmul<N>(C1D8, e2));
  const int r0 = ms9(kmul<N>(C1D4, d[1] - d[2])), r1 = ms9(kmul<N>(C1D4, d[1] + d[2]));
  const int u0 = d[3] + r0, u1 = d[3] - r0, u2 = d[0] - r1, u3 = d[0] + r1;
  o[1] = ms9(kmul<N>(C7D16, u0) + kmul<N>(C1D16, u3));
  o[3] = ms9(kmul<N>(C3D16, u2) - kmul<N>(C5D16, u1));
  o[5] = ms9(kmul<N>(C3D16, u1) + kmul<N>(C5D16, u2));
  o[7] = ms9(kmul<N>(C7D16, u3) - kmul<N>(C1D16, u0));
}

// column pass: sums/differences scaled <<2 (chendct.c:120-133)
template <bool N>
__device__ __forceinline__ void fwd_col(const int x[8], int o[8]) {
  int s[4], d[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    s[k] = (x[k] + x[7 - k]) << 2;
    d[k] = (x[k] - x[7 - k]) << 2;
  }
  fwd8<N>(s, d, o);
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
template <int CTRL>
__device__ __forceinline__ unsigned dpp(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
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

// ---------------------------------------------------------------------------
// per-macroblock LDS image

constexpr int WIN_ROWS = 46;   // y0-15 .. y0+30 (TSS reaches dy=+15)
constexpr int WIN_BYTES = 48;  // x0-16 .. x0+31 (16-byte aligned loads)
constexpr int WIN_WORDS = WIN_BYTES / 4;
constexpr int WIN_OY = 15, WIN_OX = 16;  // window coordinates of (x0, y0)
constexpr int BLK_STRIDE = 72, ROW_STRIDE = 9;  // padded DCT scratch

constexpr int LB_MAP_WORDS = 4 * 42 * 12 / 4;  // FULL search lower-bound map (me_full)
constexpr int SURV_LIST_MAX = 256;             // FULL search survivor list (me_full)

// (the union comes first: LDS offset 0 keeps the map's row offsets within the
// 8-bit dword offsets of ds_read2_b32)
struct __align__(16) MbLds {
  union {  // the transform scratch is free while the FULL search runs
    struct {
      int blk[6 * BLK_STRIDE];  // row/column exchange for DCT/IDCT
      int16_t zz[6 * 64];       // zigzagged levels for the store
    };
    uint32_t map[LB_MAP_WORDS];   // lower-bound map (phase planes)
    uint32_t list[SURV_LIST_MAX];  // survivor list (after the map is dead)
  };
  uint32_t win[WIN_ROWS * WIN_WORDS];  // previous reconstruction, luma
  uint32_t cur[64];                    // current 16x16 luma
  uint32_t cpred[2 * 16];              // chroma prediction sources, 2 x 8x8 bytes
};

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

// The search window (zero outside the picture: such candidates are never
// valid, me.c:212/292) and the current luma block, fetched into registers
// (LumaFetch) one macroblock ahead of its use, then stored to LDS (put_luma).
constexpr int WIN_SEGS = WIN_ROWS * 3, WIN_NIT = (WIN_SEGS + 63) / 64;  // 16-byte segments
struct LumaFetch {
  uint4 v[WIN_NIT];
  uint32_t c;
};
__device__ __forceinline__ LumaFetch fetch_luma(const uint8_t *ref_y, const uint8_t *cur_y, int w,
                                                int h, int x0, int y0, int lane) {
  // interior macroblocks (the whole window inside the picture) skip the
  // per-segment bounds test
  const bool inside = y0 >= WIN_OY && y0 - WIN_OY + WIN_ROWS <= h && x0 >= WIN_OX &&
                      x0 - WIN_OX + WIN_BYTES <= w;
  LumaFetch f;
#pragma unroll
  for (int i = 0; i < WIN_NIT; i++) {
    const int t = lane + 64 * i, row = t / 3, seg = t - row * 3;
    const int gy = y0 - WIN_OY + row, gx = x0 - WIN_OX + seg * 16;
    f.v[i] = make_uint4(0, 0, 0, 0);
    if (t < WIN_SEGS && (inside || (gy >= 0 && gy < h && gx >= 0 && gx < w)))
      f.v[i] = *reinterpret_cast<const uint4 *>(ref_y + (uint32_t)(mul24(gy, w) + gx));
  }
  f.c = *reinterpret_cast<const uint32_t *>(cur_y + (uint32_t)(mul24(y0 + (lane >> 2), w) + x0 + 4 * (lane & 3)));
  return f;
}
__device__ __forceinline__ void put_luma(MbLds &L, const LumaFetch &f, int lane) {
#pragma unroll
  for (int i = 0; i < WIN_NIT; i++) {
    const int t = lane + 64 * i;
    if (t < WIN_SEGS) reinterpret_cast<uint4 *>(L.win)[t] = f.v[i];
  }
  L.cur[lane] = f.c;
}

struct MeOut {
  int mx, my, sad, sad0, var, varor, mwor;
};

// SAD of the zero vector (OMV, me.c:203/271): one dword per lane
__device__ __forceinline__ int sad_zero(const MbLds &L, int lane) {
  const uint32_t r = L.win[(WIN_OY + (lane >> 2)) * WIN_WORDS + WIN_OX / 4 + (lane & 3)];
  return wave_sum((int)sad4(r, L.cur[lane], 0));
}

// FastBME (me.c:187-227) over [-sl/2, sl/2)^2, exact, pruned by a lower bound
// on the SAD built from 4x4 sub-block averages (the GPU form of ComputeError's
// early exit, me.c:122-170: work on candidates that cannot win is skipped, the
// answer is unchanged).
//
//  1. m(x, y) = nested floor average of the 4x4 pixels at (x, y), four levels of
//     v_lerp_u8 (bytewise (a+b)>>1): m = sum/16 - e with e in [0, 2] (each level
//     adds at most 1/2).  For a candidate and the current block, per 4x4
//     sub-block |sum_c - sum_r| >= 16 |m_c - m_r| - 32, so
//         SAD >= LB = 16 S - 512,  S = sum over the 16 sub-blocks |m_c - m_r|
//     (S: four v_sad_u8 per candidate against the current block's 16 averages).
//  2. c* = the valid candidate with the least S (first in scan order); its full
//     SAD and SAD(0,0) bound the answer: T = min(SAD(c*), SAD(0,0)).
//  3. a candidate with LB > T, i.e. S > (T + 512) / 16, can neither win nor tie;
//     the survivors (a handful on natural content) get their full SAD: 4, 8 or
//     16 lanes per candidate for up to 32 of them, one per lane up to
//     ME_LIST_MAX, every candidate densely beyond (flat content, where nothing
//     prunes).
//  4. the winner is the least (SAD, scan order) key among c*, the survivors and
//     (0,0), which wins ties because FastBME evaluates it first (me.c:203, 220).
// The result is identical to the exhaustive search for every input.
//
// Lane layout of the bound: lane = (dy half, dx index), 15 candidates
// dy = -15 + 15*half + d, d = 0..14, of the column dx = dxi - 15.  Keys are
// SUM << 10 | ord, ord = 1 + (dx+15)*32 + (dy+15): FastBME's dx-major scan order
// (ord 0 is reserved for the zero vector).
#ifndef ME_LIST_MAX
#define ME_LIST_MAX 256
#endif
static_assert(ME_LIST_MAX <= SURV_LIST_MAX, "survivor list size");
constexpr uint32_t ME_INVALID = 1u << 19;
#ifndef ME_LOW_CONTRAST
#define ME_LOW_CONTRAST 12
#endif  // above any real SAD (<= 65280) or S
constexpr int KEY_SHIFT = 10;
constexpr unsigned KEY_ORD = (1u << KEY_SHIFT) - 1;
// lower-bound map: 4 phase planes (x mod 4) x MAP_ROWS rows x MAP_ROW_BYTES
// bytes; plane p, row y, byte k holds m(4k + p, y) in window coordinates
constexpr int MAP_ROWS = 42, MAP_ROW_BYTES = 12, MAP_PLANE_BYTES = MAP_ROWS * MAP_ROW_BYTES;
static_assert(4 * MAP_PLANE_BYTES == 4 * LB_MAP_WORDS, "map size");

// rows [R0, R1) of the current block against window rows [I0, I1) of the lane
template <int R0, int R1, int I0, int I1>
__device__ __forceinline__ void full_rows(const uint32_t *wrow, int sh, const uint32_t *cs,
                                          uint32_t *acc) {
#pragma unroll
  for (int i = I0; i < I1; i++) {
    const uint32_t *p = wrow + i * WIN_WORDS;
    const uint32_t a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3], a4 = p[4];
    const uint32_t r0 = align4(a1, a0, sh), r1 = align4(a2, a1, sh);
    const uint32_t r2 = align4(a3, a2, sh), r3 = align4(a4, a3, sh);
#pragma unroll
    for (int r = R0; r < R1; r++) {
      const int d = i - r;
      if (d >= 0 && d < 15) {
        uint32_t a = acc[d];
        a = sad4(r0, cs[4 * r + 0], a);
        a = sad4(r1, cs[4 * r + 1], a);
        a = sad4(r2, cs[4 * r + 2], a);
        a = sad4(r3, cs[4 * r + 3], a);
        acc[d] = a;
      }
    }
    // keep the scheduler from hoisting later rows' loads: occupancy, not
    // single-wave latency, hides LDS latency here
    __builtin_amdgcn_sched_barrier(0);
  }
}

// current-block rows R0..R0+7 as wave-uniform dwords, read straight from
// global memory into SGPRs with scalar loads (no vector instructions, no
// VGPRs).  Inline asm: the compiler turns these loads into vector loads when it
// cannot prove that no store of the kernel clobbers them (the current picture
// is never written by this kernel).  The wait is inside the same statement, so
// no use can be scheduled ahead of it.
typedef unsigned su4 __attribute__((ext_vector_type(4)));
template <int R0>
__device__ __forceinline__ void load_cur_rows8(const uint8_t *cur_blk, int w, uint32_t *cs) {
  su4 v0, v1, v2, v3, v4, v5, v6, v7;
  const int o = R0 * w;
  asm volatile(
      "s_load_dwordx4 %0, %8, %9\n"
      "s_load_dwordx4 %1, %8, %10\n"
      "s_load_dwordx4 %2, %8, %11\n"
      "s_load_dwordx4 %3, %8, %12\n"
      "s_load_dwordx4 %4, %8, %13\n"
      "s_load_dwordx4 %5, %8, %14\n"
      "s_load_dwordx4 %6, %8, %15\n"
      "s_load_dwordx4 %7, %8, %16\n"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(v0), "=&s"(v1), "=&s"(v2), "=&s"(v3), "=&s"(v4), "=&s"(v5), "=&s"(v6), "=&s"(v7)
      : "s"(cur_blk), "s"(o), "s"(o + w), "s"(o + 2 * w), "s"(o + 3 * w), "s"(o + 4 * w),
        "s"(o + 5 * w), "s"(o + 6 * w), "s"(o + 7 * w));
  const su4 v[8] = {v0, v1, v2, v3, v4, v5, v6, v7};
#pragma unroll
  for (int r = 0; r < 8; r++) {
    cs[4 * (R0 + r) + 0] = v[r].x;
    cs[4 * (R0 + r) + 1] = v[r].y;
    cs[4 * (R0 + r) + 2] = v[r].z;
    cs[4 * (R0 + r) + 3] = v[r].w;
  }
}

__device__ __forceinline__ uint32_t lerp4(uint32_t a, uint32_t b) {  // bytewise (a+b)>>1
  return __builtin_amdgcn_lerp(a, b, 0u);
}
// value of lane+1 across the whole wave (DPP wave_shl:1; lane 63 reads 0)
__device__ __forceinline__ uint32_t from_next_lane_wave(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, true);
}

// 1. the map over the window (rows 0..41, x 1..42 used) into L.map.  Lane =
// (chunk c of 9 map rows, natural dword n = x/4); vertical levels on the window
// dwords, horizontal levels with the neighbour dword from lane + 1, the four
// bytes of a natural dword scattered to the four phase planes.
__device__ __forceinline__ void build_lb_map(MbLds &L, int lane) {
  const int c = lane / 12, n = lane - 12 * c;
  const bool act = lane < 60;
  const int y0 = 9 * min(c, 4);
  uint32_t v1[11];
#pragma unroll
  for (int t = 0; t < 11; t++) {
    const int ya = min(y0 + t, WIN_ROWS - 1), yb = min(y0 + t + 1, WIN_ROWS - 1);
    v1[t] = lerp4(L.win[ya * WIN_WORDS + n], L.win[yb * WIN_WORDS + n]);
  }
  uint8_t *mp = reinterpret_cast<uint8_t *>(L.map) + n;
#pragma unroll
  for (int t = 0; t < 9; t++) {
    const uint32_t v = lerp4(v1[t], v1[t + 2]);  // rows y..y+3
    const uint32_t h1 = lerp4(v, align4(from_next_lane_wave(v), v, 1));
    const uint32_t h2 = lerp4(h1, align4(from_next_lane_wave(h1), h1, 2));
    const int y = y0 + t;
    if (act && y < MAP_ROWS) {  // bytes 0/2 and, after one shift, 1/3 (ds_write_b8[_d16_hi])
      uint8_t *q = mp + y * MAP_ROW_BYTES;
      const uint32_t h2s = h2 >> 8;
      q[0] = (uint8_t)h2;
      q[2 * MAP_PLANE_BYTES] = (uint8_t)(h2 >> 16);
      q[MAP_PLANE_BYTES] = (uint8_t)h2s;
      q[3 * MAP_PLANE_BYTES] = (uint8_t)(h2s >> 16);
    }
  }
}

// the current block's 16 sub-block averages (same nesting as the map), row j
// of sub-blocks as one wave-uniform dword cm[j] (byte i = sub-block (i, j));
// returns their range (max - min)
__device__ __forceinline__ int cur_lb_map(MbLds &L, int lane, uint32_t cm[4]) {
  unsigned lo = 255, hi = 0;
  if (lane < 16) {
    const int i = lane & 3, j = lane >> 2;
    const uint32_t *r = L.cur + 16 * j + i;
    const uint32_t v = lerp4(lerp4(r[0], r[4]), lerp4(r[8], r[12]));
    const uint32_t h1 = lerp4(v, v >> 8);
    const uint32_t h2 = lerp4(h1, h1 >> 16);
    reinterpret_cast<uint8_t *>(L.cpred)[lane] = (uint8_t)h2;
    lo = hi = h2 & 255u;
  }
  // min and max over DPP row 0 (lanes 0..15)
  lo = min(lo, dpp<0xB1>(lo));
  hi = max(hi, dpp<0xB1>(hi));
  lo = min(lo, dpp<0x4E>(lo));
  hi = max(hi, dpp<0x4E>(hi));
  lo = min(lo, dpp<0x141>(lo));
  hi = max(hi, dpp<0x141>(hi));
  lo = min(lo, dpp<0x140>(lo));
  hi = max(hi, dpp<0x140>(hi));
  const int range = __builtin_amdgcn_readlane((int)(hi - lo), 0);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; j++) cm[j] = (uint32_t)uni((int)L.cpred[j]);
  return range;
}

__device__ __forceinline__ void ord_pos(unsigned ord, int &cdx, int &cdy) {  // ord >= 1
  cdx = (int)((ord - 1) >> 5) - 15;
  cdy = (int)((ord - 1) & 31) - 15;
}

// full SADs of the n <= 32 listed candidates (ords in L.list), 4*RG lanes per
// candidate: lane (slot, rg, d) sums dword d of rows rg, rg+RG, ...; returns the
// least key
template <int RG>
__device__ __forceinline__ unsigned finish_groups(const MbLds &L, int n, int lane) {
  constexpr int G = 4 * RG, PER = 64 / G, NR = 16 / RG;
  const int d = lane & 3, rg = (lane >> 2) & (RG - 1), slot = lane / G;
  uint32_t cw[NR];
#pragma unroll
  for (int t = 0; t < NR; t++) cw[t] = L.cur[4 * (rg + RG * t) + d];
  unsigned bk = 0xFFFFFFFFu;
  for (int c0 = 0; c0 < n; c0 += PER) {
    const int j = c0 + slot;
    const unsigned ord = j < n ? L.list[j] : 1u;
    int cdx, cdy;
    ord_pos(ord, cdx, cdy);
    const int cb = WIN_OX + cdx, csh = cb & 3;
    const uint32_t *p0 = L.win + (WIN_OY + cdy + rg) * WIN_WORDS + (cb >> 2) + d;
    uint32_t a = 0;
#pragma unroll
    for (int t = 0; t < NR; t++) {
      const uint32_t *p = p0 + RG * t * WIN_WORDS;
      a = sad4(align4(p[1], p[0], csh), cw[t], a);
    }
    a += dpp<0xB1>(a);  // the group's lanes: quad, then 8, then 16
    a += dpp<0x4E>(a);
    if (RG >= 2) a += dpp<0x141>(a);
    if (RG >= 4) a += dpp<0x140>(a);
    if (j < n) bk = min(bk, (a << KEY_SHIFT) | ord);
  }
  return wave_min(bk);
}

// full SADs of the listed candidates (keys with the ord in the low bits), one
// per lane; returns the least key
__device__ __forceinline__ unsigned finish_list(const MbLds &L, int n, int lane) {
  unsigned bk = 0xFFFFFFFFu;
  for (int c0 = 0; c0 < n; c0 += 64) {
    if (c0 + lane < n) {
      const unsigned ord = L.list[c0 + lane] & KEY_ORD;
      int cdx, cdy;
      ord_pos(ord, cdx, cdy);
      const int cb = WIN_OX + cdx, csh = cb & 3;
      const uint32_t *p0 = L.win + (WIN_OY + cdy) * WIN_WORDS + (cb >> 2);
      uint32_t a = 0;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const uint32_t *p = p0 + r * WIN_WORDS;
        const uint32_t a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3], a4 = p[4];
        // LDS broadcast, re-read per chunk (opaque index: not hoisted out of
        // the loop into live registers)
        const uint4 c = reinterpret_cast<const uint4 *>(L.cur)[opaque(r)];
        a = sad4(align4(a1, a0, csh), c.x, a);
        a = sad4(align4(a2, a1, csh), c.y, a);
        a = sad4(align4(a3, a2, csh), c.z, a);
        a = sad4(align4(a4, a3, csh), c.w, a);
      }
      bk = min(bk, (a << KEY_SHIFT) | ord);
    }
  }
  return wave_min(bk);
}

#ifdef P64_ME_STATS
// development aid (tools/me_paths.py): which survivor path each macroblock took
__device__ unsigned long long g_me_stats[48];
__device__ __forceinline__ void me_stats_count(int lane, int nsurv, int range) {
  // range of the current block's 16 sub-block averages, against the path
  const int bucket = min(range >> 2, 15);
  if (lane == 0) {
    atomicAdd(&g_me_stats[8 + 2 * bucket + (nsurv > ME_LIST_MAX ? 1 : 0)], 1ull);
    atomicAdd(&g_me_stats[0], 1ull);
    atomicAdd(&g_me_stats[1], (unsigned long long)nsurv);
    atomicAdd(&g_me_stats[nsurv <= 4 ? 2 : nsurv <= 8 ? 3 : nsurv <= 32 ? 4 : nsurv <= ME_LIST_MAX ? 5 : 6], 1ull);
  }
}
#endif

__device__ __forceinline__ void me_full(MbLds &L, const uint8_t *cur_blk, int w, int h, int x0,
                                        int y0, int sl, int lane, int sad0, int &mx, int &my,
                                        int &best) {
  const int half = lane >> 5, dxi = lane & 31;
  const bool lane_ok = dxi < 30;
  const int colb = (lane_ok ? dxi : 29) + 1;  // window byte column of dx = dxi-15

  // Validity (me.c:206-212: range and `< W-16`) is folded into the sums: an
  // invalid candidate starts at ME_INVALID, so it never survives and never wins.
  const int hl = sl >> 1;
  const int dx = dxi - 15, px = x0 + dx;
  const bool col_ok = lane_ok && dx >= -hl && dx < hl && px >= 0 && px < w - 16;
  // valid dy: [max(-hl, -y0), min(hl, h-16-y0)), i.e. d in [dlo, dhi) for this half
  const int dlo = max(-hl, -y0) + 15 - 15 * half, dhi = min(hl, h - 16 - y0) + 15 - 15 * half;
  const bool all_rows = dlo <= 0 && dhi >= 15;
  const bool interior = uni(__all(!lane_ok || (col_ok && all_rows)));
  auto init = [&](uint32_t *a) {
    if (interior) {  // one select for all
      const uint32_t v = lane_ok ? 0u : ME_INVALID;
#pragma unroll
      for (int d = 0; d < 15; d++) a[d] = v;
    } else {
#pragma unroll
      for (int d = 0; d < 15; d++) a[d] = (col_ok && d >= dlo && d < dhi) ? 0u : ME_INVALID;
    }
  };
  const unsigned base = ((unsigned)dxi << 5) + (unsigned)(15 * half) + 1u;  // ord of d = 0

  SECTION("cur_map");
  uint32_t cm[4];
  const int range = uni(cur_lb_map(L, lane, cm));
  unsigned bk = 0xFFFFFFFFu, ckey = 0xFFFFFFFFu, Ts = 0, pk = 0;
  uint32_t acc[15];
  lds_u32 *list = as_lds(L.list);  // aliases the map once the map is dead
  int nsurv = 1000;
  // Low-contrast blocks (sub-block averages within a few levels) prune almost
  // nothing: they go to the dense search straight away (speed only, the result
  // is the same; tools/me_paths.py measured 98% dense below 12, none above 15).
  if (range >= ME_LOW_CONTRAST) {
    // 1. lower bounds S
    SECTION("lb_map");
    build_lb_map(L, lane);
    __syncthreads();
    SECTION("lb_pass");
    init(acc);
    {
      const int xq = colb >> 2;
      const uint32_t *mrow =
          L.map + ((colb & 3) * MAP_PLANE_BYTES + 15 * half * MAP_ROW_BYTES) / 4 + (xq >> 2);
      const int msh = xq & 3;
#pragma unroll
      for (int i = 0; i < 27; i++) {
        const uint32_t *q = mrow + i * (MAP_ROW_BYTES / 4);
        const uint32_t m4 = align4(q[1], q[0], msh);
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int d = i - 4 * j;
          if (d >= 0 && d < 15) acc[d] = sad4(m4, cm[j], acc[d]);
        }
      }
    }

    // 2. c* and its full SAD
    SECTION("cstar");
    {  // least (S, d) of the lane as S << 4 | d, then its key S << 10 | ord
      unsigned m = 0xFFFFFFFFu;
#pragma unroll
      for (int d = 0; d < 15; d++) m = min(m, (acc[d] << 4) | (unsigned)d);
      pk = m == 0xFFFFFFFFu ? m : ((m >> 4) << KEY_SHIFT) + base + (m & 15u);
    }
    pk = uni((int)wave_min(pk));
    if ((pk >> KEY_SHIFT) < ME_INVALID) {  // else nothing is valid
      int cdx, cdy;
      ord_pos(pk & KEY_ORD, cdx, cdy);
      const int cb = WIN_OX + cdx + 4 * (lane & 3);
      const uint32_t *p = L.win + (WIN_OY + cdy + (lane >> 2)) * WIN_WORDS + (cb >> 2);
      const uint32_t s = sad4(align4(p[1], p[0], cb & 3), L.cur[lane], 0u);
      ckey = (pk & KEY_ORD) | ((unsigned)uni(wave_sum((int)s)) << KEY_SHIFT);
    }
    const unsigned T = min(ckey >> KEY_SHIFT, (unsigned)sad0);
    Ts = (T + 512u) >> 4;  // survivors: S <= Ts

    SECTION("survivors");
    // 3. survivors: their ords compacted into L.list with ballot + mbcnt (the
    // first ME_LIST_MAX of them), counted on the way
    nsurv = 0;
#pragma unroll
    for (int d = 0; d < 15; d++) {
      const bool sv = acc[d] <= Ts;
      const uint64_t bl = __ballot(sv);
      if (bl) {
        const int idx = nsurv + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
        if (sv && idx < ME_LIST_MAX) list[idx] = base + d;
        nsurv += __popcll(bl);
      }
    }
    nsurv = uni(nsurv);
  }
#ifdef P64_ME_STATS
  me_stats_count(lane, nsurv, range);
#endif

  SECTION("finish");
  if (nsurv <= ME_LIST_MAX) {
    __syncthreads();
    // nothing to finish when c* (whose key is known) is the only survivor
    if (nsurv == 0 || (nsurv == 1 && (unsigned)uni((int)list[0]) == (pk & KEY_ORD)))
      ;
    else if (nsurv <= 4)
      bk = finish_groups<4>(L, nsurv, lane);
    else if (nsurv <= 8)
      bk = finish_groups<2>(L, nsurv, lane);
    else if (nsurv <= 32)
      bk = finish_groups<1>(L, nsurv, lane);
    else
      bk = finish_list(L, nsurv, lane);
  } else {  // little pruned: every candidate densely, rows in two chunks
    const uint32_t *wrow = L.win + (15 * half) * WIN_WORDS + (colb >> 2);
    const int sh = colb & 3;
    uint32_t cs[64];
    init(acc);
    load_cur_rows8<0>(cur_blk, w, cs);
    full_rows<0, 8, 0, 22>(wrow, sh, cs, acc);
    load_cur_rows8<8>(cur_blk, w, cs);
    full_rows<8, 16, 8, 30>(wrow, sh, cs, acc);
#pragma unroll
    for (int d = 0; d < 15; d++) bk = min(bk, (acc[d] << KEY_SHIFT) + base + d);
    bk = wave_min(bk);
  }

  // 4. winner
  SECTION("winner");
  bk = min(min(bk, ckey), (unsigned)sad0 << KEY_SHIFT);
  const unsigned ord = bk & KEY_ORD;
  best = (int)(bk >> KEY_SHIFT);
  if (ord == 0) {
    mx = my = 0;
  } else {
    ord_pos(ord, mx, my);
  }
}

// StepBME (me.c:255-311): steps 8,4,2,1, 8 neighbours each in (diry, dirx)
// raster order, strict '<' against the running best.
__device__ __forceinline__ void me_tss(const MbLds &L, int w, int h, int x0, int y0, int lane,
                                       int sad0, int &mx, int &my, int &best) {
  const int k = lane >> 3, rg = lane & 7;
  const int kk = k < 4 ? k : k + 1;  // skip the centre of the 3x3
  const int dirx = kk % 3 - 1, diry = kk / 3 - 1;
  uint32_t c[8];
#pragma unroll
  for (int j = 0; j < 8; j++) c[j] = L.cur[8 * rg + j];  // rows 2rg, 2rg+1
  int bx = 0, by = 0;
  unsigned bsad = (unsigned)sad0;
#pragma unroll
  for (int step = 8; step >= 1; step >>= 1) {
    const int dx = bx + dirx * step, dy = by + diry * step;
    const int px = x0 + dx, py = y0 + dy;
    const bool ok = px >= 0 && px < w - 16 && py >= 0 && py < h - 16 && dx >= -15 &&
                    dx <= 15 && dy >= -15 && dy <= 15;
    uint32_t s = 0;
    if (ok) {
      const int colb = WIN_OX + dx, sh = colb & 3;
      const uint32_t *p = L.win + (WIN_OY + dy + 2 * rg) * WIN_WORDS + (colb >> 2);
#pragma unroll
      for (int rr = 0; rr < 2; rr++) {
        const uint32_t *q = p + rr * WIN_WORDS;
        const uint32_t a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3], a4 = q[4];
        s = sad4(align4(a1, a0, sh), c[4 * rr + 0], s);
        s = sad4(align4(a2, a1, sh), c[4 * rr + 1], s);
        s = sad4(align4(a3, a2, sh), c[4 * rr + 2], s);
        s = sad4(align4(a4, a3, sh), c[4 * rr + 3], s);
      }
    }
    s += dpp<0xB1>(s);   // sum over the lane's group of 8
    s += dpp<0x4E>(s);
    s += dpp<0x141>(s);
    // the first least SAD in neighbour order: min of (SAD << 3 | k) over the
    // wave (every lane of a group holds its group's key)
    const unsigned key = ok ? (s << 3) | (unsigned)k : 0xFFFFFFFFu;
    const unsigned m = wave_min(key);
    if ((m >> 3) < bsad) {
      bsad = m >> 3;
      const int j = (int)(m & 7u), jj = j < 4 ? j : j + 1;
      bx += (jj % 3 - 1) * step;
      by += (jj / 3 - 1) * step;
    }
  }
  mx = bx;
  my = by;
  best = (int)bsad;
}

// decision statistics on the chosen block (me.c:229-245 == 313-329), with the
// byte dot product: sum (r-c)^2 = r.r - 2 r.c + c.c, all exact in u32
__device__ __forceinline__ void me_stats(const MbLds &L, int lane, MeOut &o) {
  const int colb = WIN_OX + o.mx + 4 * (lane & 3);
  const uint32_t *p = L.win + (WIN_OY + o.my + (lane >> 2)) * WIN_WORDS + (colb >> 2);
  const uint32_t rw = align4(p[1], p[0], colb & 3), cw = L.cur[lane];
  const unsigned rr = __builtin_amdgcn_udot4(rw, rw, 0u, false);
  const unsigned rc = __builtin_amdgcn_udot4(rw, cw, 0u, false);
  const unsigned cc = __builtin_amdgcn_udot4(cw, cw, 0u, false);
  const int var = wave_sum((int)(rr + cc - 2 * rc));
  const int sq = wave_sum((int)rr);
  const int sum = wave_sum((int)sad4(rw, 0u, 0u));
  o.var = var / 256;
  o.varor = sq / 256 - (sum / 256) * (sum / 256);
  o.mwor = sum;
}


template <int MODE>  // 1 = TSS, 2 = FULL
__device__ __forceinline__ MeOut motion_estimate(MbLds &L, const uint8_t *cur_y, int w, int h,
                                                 int x0, int y0, int sl, int lane) {
  MeOut o;
  o.sad0 = uni(sad_zero(L, lane));
  if (MODE == 2)
    me_full(L, cur_y + (size_t)y0 * w + x0, w, h, x0, y0, sl, lane, o.sad0, o.mx, o.my, o.sad);
  else
    me_tss(L, w, h, x0, y0, lane, o.sad0, o.mx, o.my, o.sad);
  o.mx = uni(o.mx);
  o.my = uni(o.my);
  o.sad = uni(o.sad);
  me_stats(L, lane, o);
  o.var = uni(o.var);
  o.varor = uni(o.varor);
  o.mwor = uni(o.mwor);
  return o;
}

// MTYPE decision (p64.c:734-756).  xv = sad0/256 and yv = sad/256 are exact
// in binary64, so xv < 1, xv < 3 and yv > xv*0.5 are integer tests; yv >
// xv/1.1 is 11 sad > 10 sad0 unless the two are equal (the double quotient's
// error, < 2e-11, cannot cross a gap of 1/11 otherwise), and on equality the
// rounded quotient decides, computed as written.
__device__ __forceinline__ int decide_mtype(const MeOut &m) {
  if (m.var < 64 || m.varor > m.var) {
    bool inter = m.sad0 < 256 || (m.sad0 < 768 && 2 * m.sad > m.sad0);
    if (!inter) {
      const int t = 11 * m.sad - 10 * m.sad0;
      inter = t != 0 ? t > 0 : (double)m.sad / 256 > ((double)m.sad0 / 256) / 1.1;
    }
    if (inter) return 2;
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

// MUST run on all 64 lanes (DPP): the vertical taps of the H.261 loop filter
// (LoadFilterMatrix io.c:323-372) come from lanes r-1 / r+1 of the same block.
__device__ __forceinline__ void pred_from_row(uint32_t lo, uint32_t hi, bool filter, int r,
                                              int p[8]) {
  int s[8];
  unpack8(lo, hi, s);
  if (!filter) {
#pragma unroll
    for (int k = 0; k < 8; k++) p[k] = s[k];
    return;
  }
  // hz[k] = s[k-1] + 2 s[k] + s[k+1] as sums of neighbour pairs (two-source
  // adds issue at twice the rate of the three-source forms)
  int a[7], hz[8];
#pragma unroll
  for (int k = 0; k < 7; k++) a[k] = opaque(s[k] + s[k + 1]);
  hz[0] = s[0] << 2;
#pragma unroll
  for (int k = 1; k < 7; k++) hz[k] = a[k - 1] + a[k];
  hz[7] = s[7] << 2;
  const bool edge = r == 0 || r == 7;  // rows 0 and 7 are not filtered vertically
#pragma unroll
  for (int k = 0; k < 8; k++) {
    // reference: v = (up + 2hz + dn) >> 2 (edge rows: v = hz), then
    // (v & 2) ? (v >> 2) + 1 : v >> 2 == (v + 2) >> 2 for v >= 0; and
    // ((t >> 2) + 2) >> 2 == (t + 8) >> 4 for t >= 0 (t mod 4 never borrows)
    // (opaque: two DPP-fused adds instead of two DPP moves and a v_add3)
    const int h2 = opaque(hz[k] << 1);
    const int t = opaque(h2 + from_prev_lane(hz[k])) + from_next_lane(hz[k]);
    p[k] = ((edge ? h2 << 1 : t) + 8) >> 4;
  }
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

// stage the two 8x8 chroma prediction sources of this MB at the compensated
// origin (one byte pair per lane)
__device__ __forceinline__ void stage_chroma(MbLds &L, const Picture &ref, int w, int mbx, int mby,
                                             int mt, int mvx, int mvy, int lane) {
  const int cw = w >> 1;
  const bool mf = mt_mf(mt);
  const int ox = 8 * mbx + (mf ? mvx / 2 : 0), oy = 8 * mby + (mf ? mvy / 2 : 0);
  const int pl = lane >> 5, row = (lane >> 2) & 7, c2 = (lane & 3) * 2;
  const uint8_t *src = (pl ? ref.v : ref.u) + (uint32_t)(mul24(oy + row, cw) + ox + c2);
  const uint32_t v = (uint32_t)src[0] | ((uint32_t)src[1] << 8);
  reinterpret_cast<uint16_t *>(L.cpred)[pl * 32 + row * 4 + (c2 >> 1)] = (uint16_t)v;
}

// prediction row for the encoder: luma from the LDS search window, chroma from
// the staged sources.  All 64 lanes execute (lanes b >= 6 compute garbage).
__device__ __forceinline__ void predict_row(const MbLds &L, int b, int r, int mt, int mvx, int mvy,
                                            int p[8]) {
  const bool mf = mt_mf(mt);
  uint32_t lo, hi;
  if (b < 4) {
    const int col = WIN_OX + 8 * (b & 1) + (mf ? mvx : 0);
    const int row = WIN_OY + 8 * (b >> 1) + (mf ? mvy : 0) + r;
    const uint32_t *q = L.win + row * WIN_WORDS + (col >> 2);
    const uint32_t a0 = q[0], a1 = q[1], a2 = q[2];
    lo = align4(a1, a0, col & 3);
    hi = align4(a2, a1, col & 3);
  } else {
    const uint32_t *q = L.cpred + (b - 4) * 16 + r * 2;
    lo = q[0];
    hi = q[1];
  }
  pred_from_row(lo, hi, mt_filter(mt), r, p);
}

// prediction row straight from global memory (decoder)
__device__ __forceinline__ void predict_row_glb(const Picture &ref, int w, int b, int mbx, int mby,
                                                int r, int mt, int mvx, int mvy, int p[8]) {
  const bool mf = mt_mf(mt);
  const BlockGeom g = block_geom(b, mbx, mby);
  const int pw = g.plane ? w / 2 : w;
  const uint8_t *pl = g.plane == 0 ? ref.y : (g.plane == 1 ? ref.u : ref.v);
  const int dx = mf ? (g.plane ? mvx / 2 : mvx) : 0, dy = mf ? (g.plane ? mvy / 2 : mvy) : 0;
  const uint8_t *src = pl + mul24(g.y + dy + r, pw) + g.x + dx;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    lo |= (uint32_t)src[k] << (8 * k);
    hi |= (uint32_t)src[4 + k] << (8 * k);
  }
  pred_from_row(lo, hi, mt_filter(mt), r, p);
}

// ---------------------------------------------------------------------------
// transforms through the LDS scratch.  All 64 lanes compute the row/column
// passes (lanes 48..63 shadow block 5, b is clamped); only lanes < 48 (act)
// store, so no two lanes write one LDS word.

// rows res[8] of block b -> forward 2-D transform -> raw (pre-/8) coefficients
// left in L.blk in natural order
__device__ __forceinline__ void forward_2d(MbLds &L, bool act, int b, int r, const int res[8]) {
  int *B = L.blk + b * BLK_STRIDE;
  if (act) {
#pragma unroll
    for (int k = 0; k < 8; k++) B[r * ROW_STRIDE + k] = res[k];
  }
  __syncthreads();
  {  // column pass, lane owns column c = r
    int x[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = B[k * ROW_STRIDE + r];
    fwd_col<true>(x, o);
    if (act) {
#pragma unroll
      for (int k = 0; k < 8; k++) B[k * ROW_STRIDE + r] = o[k];
    }
  }
  __syncthreads();
  {
    int x[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = B[r * ROW_STRIDE + k];
    fwd_row<true>(x, o);
    if (act) {
#pragma unroll
      for (int k = 0; k < 8; k++) B[r * ROW_STRIDE + k] = o[k];
    }
  }
  __syncthreads();
}

// dequantised blocks in L.blk (natural order) -> inverse 2-D transform -> row r
// of block b's residual
__device__ __forceinline__ void inverse_2d(MbLds &L, bool act, int b, int r, int res[8]) {
  int *B = L.blk + b * BLK_STRIDE;
  {  // column pass: inputs <<2, folded into the constants
    int x[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = B[k * ROW_STRIDE + r];
    inv8<true, 4>(x, o);
    if (act) {
#pragma unroll
      for (int k = 0; k < 8; k++) B[k * ROW_STRIDE + r] = o[k];
    }
  }
  __syncthreads();
  int x[8], o[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = B[r * ROW_STRIDE + k];
  inv8<true>(x, o);
#pragma unroll
  for (int k = 0; k < 8; k++) res[k] = idct_final(o[k]);
}

// element layout: lane e holds natural coefficient e of each block k
__device__ __forceinline__ int blk_at(const MbLds &L, int k, int e) {
  return L.blk[k * BLK_STRIDE + (e >> 3) * ROW_STRIDE + (e & 7)];
}
__device__ __forceinline__ void blk_put(MbLds &L, int k, int e, int v) {
  L.blk[k * BLK_STRIDE + (e >> 3) * ROW_STRIDE + (e & 7)] = v;
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

// CBP decision from the six blocks' levels (p64.c:887-908), with wave ballots:
// sum|level| > 1 <=> two or more nonzero levels, or one of magnitude > 1.
struct CbpOut {
  int cbp;       // CBP bits, block c -> bit 5-c
  bool nothing;  // no block has any nonzero level
};
__device__ __forceinline__ CbpOut cbp_decide(const int lev[6]) {
  int cbp = 0, pmask = 0;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const uint64_t nz = __ballot(lev[k] != 0);
    const uint64_t big = __ballot(lev[k] > 1 || lev[k] < -1);
    if (nz && !pmask) pmask = 1 << (5 - k);
    if (big || __popcll(nz) >= 2) cbp |= 1 << (5 - k);
  }
  CbpOut o;
  o.nothing = pmask == 0;
  o.cbp = cbp ? cbp : pmask;
  return o;
}

// ---------------------------------------------------------------------------
// the fused encode kernel: ME -> decision -> prediction -> DCT -> quant ->
// zigzag -> CBP -> IQ -> IDCT -> reconstruction, one wave per macroblock.
// MODE: 0 intra picture, 1 TSS, 2 FULL.

// per-macroblock inputs, all loads in flight before the first use
struct MbFetch {
  LumaFetch luma;  // MODE != 0: search window and current luma
  uint2 crow;      // the lane's row of its block in the current picture
  int li, q, ov;   // LastIntra, UseQuant and the -o MTYPE override of the MB
};
template <int MODE>
__device__ __forceinline__ MbFetch fetch_mb(const p64gpu_encode_args &a, const uint8_t *cur_all,
                                            unsigned gid, const MbDiv &kd, int lane) {
  const int w = a.width, h = a.height, mbw = w >> 4, nmb = mbw * (h >> 4);
  const MbPos ps = mb_pos(gid, nmb, mbw, kd);
  const int fi = ps.fi, mb = ps.mb, mbx = ps.mbx, mby = ps.mby;
  const Picture cur = picture_at(cur_all + (size_t)fi * a.frame_stride, w, h);
  const int b = min(lane >> 3, 5), r = lane & 7;
  const BlockGeom g = block_geom(b, mbx, mby);
  const int pw = g.plane ? w >> 1 : w;
  const uint8_t *cplane = g.plane == 0 ? cur.y : (g.plane == 1 ? cur.u : cur.v);
  MbFetch f;
  f.crow = *reinterpret_cast<const uint2 *>(cplane + (uint32_t)(mul24(g.y + r, pw) + g.x));
  const size_t gmb = (size_t)fi * nmb + mb;
  f.li = a.last_intra[gmb];
  f.q = a.quant_mb ? a.quant_mb[gmb] : a.quant;
  f.ov = a.mtype_override ? a.mtype_override[gmb] : -1;
  if (MODE != 0)
    f.luma = fetch_luma(a.ref + (size_t)fi * a.frame_stride, cur.y, w, h, 16 * mbx, 16 * mby, lane);
  return f;
}

// one macroblock, its luma already in L (MODE != 0)
template <int MODE>
__device__ __forceinline__ void encode_mb(const p64gpu_encode_args &a, const uint8_t *cur_all,
                                          MbLds &L, int lane, unsigned gid, const MbDiv &kd,
                                          const MbFetch &f) {
  const uint2 crow = f.crow;
  const int w = a.width, h = a.height, mbw = w >> 4, nmb = mbw * (h >> 4);
  const MbPos ps = mb_pos(gid, nmb, mbw, kd);
  const int fi = ps.fi, mb = ps.mb, mbx = ps.mbx, mby = ps.mby, x0 = 16 * mbx, y0 = 16 * mby;
  const size_t gmb = (size_t)fi * nmb + mb;
  const Picture cur = picture_at(cur_all + (size_t)fi * a.frame_stride, w, h);
  const Picture ref = picture_at(a.ref + (size_t)fi * a.frame_stride, w, h);
  uint8_t *rec = a.recon + (size_t)fi * a.frame_stride;

  // row layout coordinates (lanes 48..63 shadow block 5, masked on stores)
  const int b = min(lane >> 3, 5), r = lane & 7;
  const bool act = lane < 48;
  const BlockGeom g = block_geom(b, mbx, mby);
  const int pw = g.plane ? w >> 1 : w;

  int mt = 0, mvx = 0, mvy = 0;
  if (MODE != 0) {
    __syncthreads();
    SECTION("e_me");
    const MeOut me = motion_estimate<MODE>(L, cur.y, w, h, x0, y0, a.search_limit, lane);
    if (a.me && lane == 0) {
      p64_me_rec o;
      o.mx = me.mx;
      o.my = me.my;
      o.sad = me.sad;
      o.sad0 = me.sad0;
      o.var = me.var;
      o.varor = me.varor;
      o.mwor = me.mwor;
      a.me[gmb] = o;
    }
    SECTION("e_decide");
    mt = decide_mtype(me);
    const int ov = uni(f.ov);
    if (ov >= 0) mt = ov;
    mvx = me.mx;
    mvy = me.my;
  }
  const int li = uni(f.li);
  if (li > 131) mt = 0;  // SEQUENCE_INTRA_THRESHOLD (p64.c:159, 772)
  mt = uni(mt);
  const int q = uni(f.q);
  const float rq = c_qrecip.r[q];
  const bool qeven = !(q & 1);
  const float rqe = qeven ? rq : 0.0f;

  SECTION("e_predict");
  int pred[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!mt_intra(mt)) {
    stage_chroma(L, ref, w, mbx, mby, mt, mvx, mvy, lane);
    __syncthreads();
    predict_row(L, b, r, mt, mvx, mvy, pred);
  }

  SECTION("e_fwd_dct");
  // ReadCompressMDU (p64.c:830-912): levels in element layout
  const int e = lane;
  const bool dc = e == 0;
  const int qlo = dc ? -0x7fffffff : -1023, qhi = dc ? 2047 : 1023;  // BoundDctMatrix
  int lev[6] = {0, 0, 0, 0, 0, 0};
  if (mt_tcoeff(mt)) {
    int res[8];
    unpack8(crow.x, crow.y, res);
#pragma unroll
    for (int k = 0; k < 8; k++) res[k] -= pred[k];
    forward_2d(L, act, b, r, res);
    SECTION("e_quant");
    if (mt_intra(mt)) {
#pragma unroll
      for (int k = 0; k < 6; k++) lev[k] = quantise<true>(blk_at(L, k, e), qlo, qhi, dc, rq, rqe);
    } else {
#pragma unroll
      for (int k = 0; k < 6; k++) lev[k] = quantise<false>(blk_at(L, k, e), qlo, qhi, dc, rq, rqe);
    }
  }
  SECTION("e_cbp");
  int cbp = 0x3f;
  if (mt_cbp(mt)) {
    const CbpOut c = cbp_decide(lev);
    cbp = uni(c.cbp);
    if (c.nothing) {  // no coefficients: MC without coefficients, ME vector kept
      const int old = mt;
      mt = uni(mt_filter(mt) ? 7 : 4);
      cbp = 0x3f;
      if (!mt_mf(old)) {  // 2/3 -> 4 switches from the zero vector to the ME vector
        __syncthreads();
        stage_chroma(L, ref, w, mbx, mby, mt, mvx, mvy, lane);
        __syncthreads();
        predict_row(L, b, r, mt, mvx, mvy, pred);
      }
    }
  }
  SECTION("e_zz_dequant");
  const int zpos = c_zz.pos[e];
  __syncthreads();  // element reads of blk are complete before it is rewritten
  const int coded = mt_tcoeff(mt) ? cbp : 0;  // block c coded <=> bit 5-c
  const bool intra = mt_intra(mt);
#pragma unroll
  for (int k = 0; k < 6; k++) {
    L.zz[k * 64 + zpos] = (int16_t)lev[k];
    const bool ck = (coded >> (5 - k)) & 1;
    const int q2 = ck ? 2 * q : 0, qq = ck ? q - (int)qeven : 0;
    blk_put(L, k, e, intra ? dequantise<true>(lev[k], dc, q2, qq) : dequantise<false>(lev[k], dc, q2, qq));
  }
  __syncthreads();
  if (lane < 48)
    reinterpret_cast<uint4 *>(a.coef + gmb * 384)[lane] = reinterpret_cast<const uint4 *>(L.zz)[lane];

  SECTION("e_inverse");
  // reconstruction (p64.c:945-959, 971-1013)
  int res[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (coded) inverse_2d(L, act, b, r, res);
  if (act) {
#pragma unroll
    for (int k = 0; k < 8; k++) res[k] = clampi(res[k] + pred[k], 0, 255);  // pred = 0 if intra
    *reinterpret_cast<uint2 *>(rec + (uint32_t)(plane_offset(g.plane, w, h) + mul24(g.y + r, pw) + g.x)) =
        pack8(res);
  }
  SECTION("e_mbrec");
  if (lane == 0) {
    p64_mb_rec o;
    o.mtype = (int8_t)mt;
    o.cbp = (int8_t)cbp;
    o.mvx = (int8_t)(mt_mf(mt) ? mvx : 0);
    o.mvy = (int8_t)(mt_mf(mt) ? mvy : 0);
    a.mb[gmb] = o;
    a.last_intra[gmb] = mt_intra(mt) ? 0 : (uint8_t)(li + 1);
  }
}

#ifndef ENCODE_WAVES_PER_SIMD
#define ENCODE_WAVES_PER_SIMD 1
#endif
template <int MODE>
__global__ __launch_bounds__(64, ENCODE_WAVES_PER_SIMD) void k_encode(p64gpu_encode_args a, const int32_t *mb_list,
                                                                      MbDiv kd) {
  __shared__ MbLds L;
  const int lane = threadIdx.x;
  unsigned gid;
  if (mb_list) {  // one picture, listed macroblocks only (p64gpu_encode_mb_list)
    const int mb = mb_list[blockIdx.x];
    if (mb < 0 || mb >= (a.width >> 4) * (a.height >> 4)) return;  // whole workgroup
    gid = (unsigned)mb;
  } else {
    gid = xcd_remap(blockIdx.x, gridDim.x);
  }
  TIMING_BEGIN(gid);
  const MbFetch f = fetch_mb<MODE>(a, a.cur, gid, kd, lane);
  if (MODE != 0) put_luma(L, f.luma, lane);
  SECTION("fetched");
  encode_mb<MODE>(a, a.cur, L, lane, gid, kd, f);
  TIMING_END();
}

// ME only (MotionEstimation me.c:340-363 over a batch of luma planes)
template <int MODE>
__global__ __launch_bounds__(64, ENCODE_WAVES_PER_SIMD) void k_motion(int w, int h, int64_t stride, const uint8_t *ref_y,
                                               const uint8_t *cur_y, int sl, p64_me_rec *out,
                                               MbDiv kd) {
  __shared__ MbLds L;
  const int lane = threadIdx.x;
  const int mbw = w >> 4, nmb = mbw * (h >> 4);
  const unsigned gid = xcd_remap(blockIdx.x, gridDim.x);
  TIMING_BEGIN(gid);
  const MbPos ps = mb_pos(gid, nmb, mbw, kd);
  const int fi = ps.fi, x0 = 16 * ps.mbx, y0 = 16 * ps.mby;
  put_luma(L, fetch_luma(ref_y + (size_t)fi * stride, cur_y + (size_t)fi * stride, w, h, x0, y0, lane),
           lane);
  __syncthreads();
  SECTION("m_fetched");
  const MeOut me = motion_estimate<MODE>(L, cur_y + (size_t)fi * stride, w, h, x0, y0, sl, lane);
  SECTION("m_me_done");
  if (lane == 0) {
    p64_me_rec o;
    o.mx = me.mx;
    o.my = me.my;
    o.sad = me.sad;
    o.sad0 = me.sad0;
    o.var = me.var;
    o.varor = me.varor;
    o.mwor = me.mwor;
    out[gid] = o;
  }
  TIMING_END();
}

// decoder-side reconstruction of coded macroblocks (DecompressMDU p64.c:1179 +
// DecodeSaveMDU p64.c:971)
__global__ __launch_bounds__(64) void k_decode_recon(int w, int h, int64_t stride,
                                                     const uint8_t *refp, uint8_t *recp,
                                                     const int16_t *coef, const p64_mb_rec *mbr,
                                                     const uint8_t *quant_mb,
                                                     const uint8_t *coded_mask, MbDiv kd) {
  __shared__ MbLds L;
  const int lane = threadIdx.x;
  const int mbw = w >> 4, nmb = mbw * (h >> 4);
  const unsigned gid = xcd_remap(blockIdx.x, gridDim.x);
  const MbPos ps = mb_pos(gid, nmb, mbw, kd);
  const int fi = ps.fi, mb = ps.mb, mbx = ps.mbx, mby = ps.mby;
  const size_t gmb = (size_t)fi * nmb + mb;
  if (!coded_mask[gmb]) return;  // whole workgroup exits together
  const Picture ref = picture_at(refp + (size_t)fi * stride, w, h);
  uint8_t *rec = recp + (size_t)fi * stride;
  const p64_mb_rec m = mbr[gmb];
  const int mt = uni(m.mtype), q = uni(quant_mb[gmb]);
  const int cbp = uni(mt_cbp(mt) ? m.cbp : 0x3f);  // p64.c:1200
  const int b = min(lane >> 3, 5), r = lane & 7;
  const bool act = lane < 48;
  const BlockGeom g = block_geom(b, mbx, mby);
  const int pw = g.plane ? w / 2 : w;
  const int e = lane, zpos = c_zz.pos[e];
  const bool dc = e == 0, qeven = !(q & 1), intra = mt_intra(mt);
  const int coded = mt_tcoeff(mt) ? cbp : 0;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const bool ck = (coded >> (5 - k)) & 1;
    const int lev = ck ? coef[gmb * 384 + k * 64 + zpos] : 0;  // IZigzagMatrix
    const int q2 = ck ? 2 * q : 0, qq = ck ? q - (int)qeven : 0;
    blk_put(L, k, e, intra ? dequantise<true>(lev, dc, q2, qq) : dequantise<false>(lev, dc, q2, qq));
  }
  int pred[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!mt_intra(mt)) predict_row_glb(ref, w, b, mbx, mby, r, mt, m.mvx, m.mvy, pred);
  __syncthreads();
  int res[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (coded) inverse_2d(L, act, b, r, res);
  if (act) {
#pragma unroll
    for (int k = 0; k < 8; k++) res[k] = clampi(res[k] + pred[k], 0, 255);
    *reinterpret_cast<uint2 *>(rec + (uint32_t)(plane_offset(g.plane, w, h) + mul24(g.y + r, pw) + g.x)) =
        pack8(res);
  }
}

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

// keeps the machine scheduler from interleaving the 8 lines of a pass (it
// would trade registers for ILP the block layout does not need: other waves
// hide latency; -DNO_SCHED_FENCE to compare)
#ifdef NO_SCHED_FENCE
#define SCHED_FENCE()
#else
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

// A wave issues its loads at raised priority (-DNO_SETPRIO: not), so a freshly
// launched wave gets its requests out ahead of the older waves' arithmetic
#if !defined(NO_SETPRIO)
#define PRIO_HIGH() __builtin_amdgcn_s_setprio(3)
#define PRIO_LOW() __builtin_amdgcn_s_setprio(0)
#else
#define PRIO_HIGH()
#define PRIO_LOW()
#endif
#if defined(SETPRIO_ST)  // and its stores
#define PRIO_ST() __builtin_amdgcn_s_setprio(3)
#else
#define PRIO_ST()
#endif
// occupancy hint for the block-layout kernels (-DBLK_WAVES=n: at least n waves
// per SIMD, i.e. at most 512/n VGPRs)
#if defined(BLK_WAVES) && BLK_WAVES > 0
#define BLK_OCC __attribute__((amdgpu_waves_per_eu(BLK_WAVES)))
#else
#define BLK_OCC
#endif

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

struct BlkPos {
  int fi;     // picture in the launch
  int mb;     // raster macroblock
  int b;      // block c = 0..5 of the MB (p64.c:77-79)
  int plane;  // 0 Y, 1 U, 2 V
  int x, y;   // block origin in its plane
};
__device__ __forceinline__ BlkPos blk_pos(unsigned t, int w, int h, const BlkDiv &k) {
  const int mbw = w >> 4, nmb = mbw * (h >> 4), bw = w >> 3;
  BlkPos p;
  p.fi = (int)mdiv(t, k.mp, k.sp);
  int i = (int)(t - (unsigned)p.fi * (unsigned)(6 * nmb));
  if (i < 4 * nmb) {  // luma block (bx, by)
    const int by = (int)mdiv((unsigned)i, k.mb, k.sb), bx = i - by * bw;
    p.plane = 0;
    p.x = 8 * bx;
    p.y = 8 * by;
    p.mb = (by >> 1) * mbw + (bx >> 1);
    p.b = ((by & 1) << 1) | (bx & 1);
  } else {
    i -= 4 * nmb;
    const int pl = i >= nmb;
    i -= pl ? nmb : 0;
    const int mby = (int)mdiv((unsigned)i, k.mw, k.sw), mbx = i - mby * mbw;
    p.plane = 1 + pl;
    p.x = 8 * mbx;
    p.y = 8 * mby;
    p.mb = i;
    p.b = 4 + pl;
  }
  return p;
}
// MB-grouped block layout: wave w takes macroblocks 10w .. 10w+9 of the
// launch, lane 6m + b block b of its m-th MB (lanes 60..63 repeat lane 59).
// A wave's levels are then 7,680 contiguous bytes and its pixel rows and
// records contiguous runs per plane: its HBM traffic is a few long runs
// instead of 64 blocks scattered over a block row.
constexpr int MBS_PER_WAVE = 10;
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

// 64 reconstructed values (already in 0..255) -> 8 row stores
__device__ __forceinline__ void store_block(uint8_t *dst, int pw, const int v[64]) {
#pragma unroll
  for (int k = 0; k < 8; k++) *reinterpret_cast<uint2 *>(dst + (uint32_t)mul24(k, pw)) = pack8(v + 8 * k);
}

// ChenDct (chendct.c:97-206) on a register block given as its 8 packed pixel
// rows (or the residual rows - prow), the row pass in packed 16-bit
// arithmetic: the column pass (scalar) leaves each row as four (column 2j, 2j+1) int16 pairs -- its
// outputs stay within +-5,800 for pixel or +-255 residual input -- and the
// row pass runs the butterfly of fwd8 on pairs: v_pk_add/sub/ashr for the
// sums, and every product pair C_a x + C_b y as ONE v_dot2_i32_i16 with the
// constant pair as its literal (the two products and their sum exact in
// 32 bits, the same ms9 rounding after).  Row-pass intermediates stay below
// 2^15: sums <= 11,600, u = d + r <= 14,000.  Half the registers of the
// scalar form between the passes.
typedef short s16x2 __attribute__((ext_vector_type(2)));
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
  const int r1 = ms9(dot2(q, C1D4, C1D4)), r0 = ms9(dot2(q, C1D4, -C1D4));
  const s16x2 dd = __builtin_shufflevector(d23, d01, 1, 2);  // (d3, d0)
  const s16x2 rr = pk16(r0, r1);
  const s16x2 u03 = dd + rr, u12 = dd - rr;                   // (u0,u3) (u1,u2)
  o[1] = ms9(dot2(u03, C7D16, C1D16));
  o[7] = ms9(dot2(u03, -C1D16, C7D16));
  o[3] = ms9(dot2(u12, -C5D16, C3D16));
  o[5] = ms9(dot2(u12, C3D16, C5D16));
}
// (the final rounding dct_final(v) reads the sign of v = X >> 9; hipcc then
// takes it from X itself and keeps all 64 pre-shift sums alive next to the
// shifted coefficients until quantisation -- 64 extra VGPRs.  The opaque copy
// ends X's life at the shift.)
// RES: the input is the residual rows - prow (both packed pixel rows)
template <bool RES = false>
__device__ __forceinline__ void fdct_block_pk(const uint2 rows[8], int v[64], const uint2 *prow = nullptr) {
  s16x2 p[8][4];  // [row][column pair]
#pragma unroll
  for (int c = 0; c < 8; c += 2) {
    int x[8], y[8], o[8], u[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t wd = c < 4 ? rows[k].x : rows[k].y;
      x[k] = (int)((wd >> (8 * (c & 3))) & 255);
      y[k] = (int)((wd >> (8 * ((c + 1) & 3))) & 255);
      if (RES) {
        const uint32_t pd = c < 4 ? prow[k].x : prow[k].y;
        x[k] -= (int)((pd >> (8 * (c & 3))) & 255);
        y[k] -= (int)((pd >> (8 * ((c + 1) & 3))) & 255);
      }
    }
    fwd_col<true>(x, o);
    fwd_col<true>(y, u);
#pragma unroll
    for (int k = 0; k < 8; k++) p[k][c >> 1] = pk16(o[k], u[k]);
    SCHED_FENCE();
  }
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
__device__ __forceinline__ uint2 final_clamp_pack8(const int o[8]) {
  int x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = (o[k] + 8) >> 4;
  return make_uint2(sat4(x), sat4(x + 4));
}
// ChenIDct (chendct.c:217-375) on a register block: column pass (inputs <<2,
// folded into the constants), row pass, final rounding
__device__ __forceinline__ void idct_block(int v[64]) {
#pragma unroll
  for (int c = 0; c < 8; c++) {
    int x[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = v[8 * k + c];
    inv8<true, 4>(x, o);
#pragma unroll
    for (int k = 0; k < 8; k++) v[8 * k + c] = o[k];
    SCHED_FENCE();
  }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    int o[8];
    inv8<true>(v + 8 * r, o);
#pragma unroll
    for (int k = 0; k < 8; k++) v[8 * r + k] = idct_final(o[k]);
    SCHED_FENCE();
  }
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
template <class PairFn>
__device__ __forceinline__ void iq_idct_cols(PairFn pair, uint32_t q2, uint32_t qq, bool dcfix, int dc8,
                                             int v[64]) {
#pragma unroll
  for (int c = 0; c < 8; c++) {
    uint32_t p04 = dequantise_pk(pair(c, 32 + c), q2, qq);
    if (c == 0) p04 = dcfix ? __builtin_amdgcn_perm(p04, (uint32_t)dc8, 0x07060100u) : p04;  // (DC x 8, x4)
    const s16x2 a04 = __builtin_bit_cast(s16x2, p04);
    const s16x2 a17 = __builtin_bit_cast(s16x2, dequantise_pk(pair(8 + c, 56 + c), q2, qq));
    const s16x2 a53 = __builtin_bit_cast(s16x2, dequantise_pk(pair(40 + c, 24 + c), q2, qq));
    const s16x2 a26 = __builtin_bit_cast(s16x2, dequantise_pk(pair(16 + c, 48 + c), q2, qq));
    const int p0 = ms9(dot2(a17, 4 * C7D16, -4 * C1D16)), p3 = ms9(dot2(a17, 4 * C1D16, 4 * C7D16));
    const int p1 = ms9(dot2(a53, 4 * C3D16, -4 * C5D16)), p2 = ms9(dot2(a53, 4 * C5D16, 4 * C3D16));
    const int q0 = ms9(dot2(a04, 4 * C1D4, 4 * C1D4)), q1 = ms9(dot2(a04, 4 * C1D4, -4 * C1D4));
    const int q2_ = ms9(dot2(a26, 4 * C3D8, -4 * C1D8)), q3 = ms9(dot2(a26, 4 * C1D8, 4 * C3D8));
    const int e0 = q0 + q3, e1 = q1 + q2_, e2 = q1 - q2_, e3 = q0 - q3;
    const int f0 = p0 + p1, f1 = p0 - p1, f2 = p3 - p2, f3 = p3 + p2;
    const int g1 = ms9(kmul<true>(C1D4, f2 - f1)), g2 = ms9(kmul<true>(C1D4, f2 + f1));
    v[c] = e0 + f3;
    v[8 + c] = e1 + g2;
    v[16 + c] = e2 + g1;
    v[24 + c] = e3 + f0;
    v[32 + c] = e3 - f0;
    v[40 + c] = e2 - g1;
    v[48 + c] = e1 - g2;
    v[56 + c] = e0 - f3;
    SCHED_FENCE();
  }
}
// row pass + idct_final (the residual, to be added to a prediction)
__device__ __forceinline__ void idct_rows(int v[64]) {
#pragma unroll
  for (int r = 0; r < 8; r++) {
    int o[8];
    inv8<true>(v + 8 * r, o);
#pragma unroll
    for (int k = 0; k < 8; k++) v[8 * r + k] = idct_final(o[k]);
    SCHED_FENCE();
  }
}
// levels (ints, natural order) in v -> reconstructed rows of an intra block.
// The row pass takes its product pairs by v_dot2 too: in an intra picture
// the dequantised inputs are bounded by the quantiser (|AC| <= 1,023 + q <=
// 1,054, DC <= 254 x 8 = 2,032), which bounds the column-pass outputs by
// 25,062 (every sign pattern at those magnitudes) < 2^15; a decoder or an
// inter residual may exceed that (up to 167,072), so only here.
__device__ __forceinline__ void iq_idct_intra_rec(int v[64], int q, uint2 rec[8]) {
  const uint32_t q2 = 0x20002u * (uint32_t)q, qq = 0x10001u * (uint32_t)(q - (int)!(q & 1));
  iq_idct_cols([&](int e, int f) { return pk2(v[e], v[f]); }, q2, qq, true, v[0] * 8, v);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int *x = v + 8 * r;
    const s16x2 a04 = __builtin_bit_cast(s16x2, pk2(x[0], x[4])), a17 = __builtin_bit_cast(s16x2, pk2(x[1], x[7]));
    const s16x2 a53 = __builtin_bit_cast(s16x2, pk2(x[5], x[3])), a26 = __builtin_bit_cast(s16x2, pk2(x[2], x[6]));
    const int p0 = ms9(dot2(a17, C7D16, -C1D16)), p3 = ms9(dot2(a17, C1D16, C7D16));
    const int p1 = ms9(dot2(a53, C3D16, -C5D16)), p2 = ms9(dot2(a53, C5D16, C3D16));
    const int q0 = ms9(dot2(a04, C1D4, C1D4)), q1 = ms9(dot2(a04, C1D4, -C1D4));
    const int q2_ = ms9(dot2(a26, C3D8, -C1D8)), q3 = ms9(dot2(a26, C1D8, C3D8));
    const int e0 = q0 + q3, e1 = q1 + q2_, e2 = q1 - q2_, e3 = q0 - q3;
    const int f0 = p0 + p1, f1 = p0 - p1, f2 = p3 - p2, f3 = p3 + p2;
    const int g1 = ms9(kmul<true>(C1D4, f2 - f1)), g2 = ms9(kmul<true>(C1D4, f2 + f1));
    const int o[8] = {e0 + f3, e1 + g2, e2 + g1, e3 + f0, e3 - f0, e2 - g1, e1 - g2, e0 - f3};
    rec[r] = final_clamp_pack8(o);
    SCHED_FENCE();
  }
}

// intra picture (p64.c:635, 770-771: every MB is MTYPE 0, CBP 0x3f), block
// layout: load -> ChenDct -> BoundDct + CCITTFlatQuantize + FlatBound ->
// zigzag store -> ICCITTFlatQuantize -> ChenIDct -> BoundIDct -> recon.
// Persistent: a lane walks blocks t, t + stride, ... and issues the loads of
// its next block before transforming the current one, so every wave keeps
// HBM reads in flight under its own VALU work (without it the waves of a round
// load, compute and store in lock step and the memory system idles while they
// compute).
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


// dword 3 of a raw buffer resource on gfx9-family parts (CDNA): 32-bit data format
constexpr int BUF_RSRC_W3 = 0x00020000;
constexpr uint32_t BUF_OOB = 0x80000000u;  // >= every buffer's num_records: loads 0, stores dropped

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
#if defined(PROBE_NOLOAD)
  for (int k = 0; k < 8; k++) f.rows[k] = make_uint2(pos.x * 0x01010101u + k, pos.y * 0x03050709u ^ pos.fi);
#endif
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
__device__ __forceinline__ void intra_block(const p64gpu_encode_args &a, const IntraFetch &f, uint8_t *lds,
                                            int lane, IntraOut &out) {
  const int w = a.width, h = a.height;
  const BlkPos &p = f.p;
  const int q = f.q;
  // c_qrecip.r[q] computed in place (no dependent table load in the loop)
  const float rq = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, 1.0f / (float)(2 * q)) + 1u);
  const float rqe = (q & 1) ? 0.0f : rq;
  const int qb = quant_bound(q);
  int v[64];
  fdct_block_pk(f.rows, v);
  // in scan order: quantise (BoundDct + CCITTFlatQuantize + FlatBound), pack
  // the level pair; 16 bytes of levels at a time into the wave's LDS staging
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int l2[2];
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const int e = k_zz.inv[8 * k + 2 * j + i];
        const bool dc = e == 0;
        l2[i] = quantise<true, true>(v[e], dc ? -0x7fffffff : -qb, dc ? 2047 : qb, dc, rq, rqe);
        v[e] = l2[i];  // dequantised in pairs by iq_idct_intra_rec
      }
      pk[j] = __builtin_amdgcn_perm((uint32_t)l2[1], (uint32_t)l2[0], 0x05040100u);
    }
    put_levels(lds, lane, k, make_uint4(pk[0], pk[1], pk[2], pk[3]));
    SCHED_FENCE();
  }
  iq_idct_intra_rec(v, q, out.rec);  // ICCITTFlatQuantize + ChenIDct + BoundIDctMatrix
  out.pw = p.plane ? w >> 1 : w;
  out.rec_off = (uint32_t)((int64_t)p.fi * a.frame_stride) + (uint32_t)plane_offset(p.plane, w, h) +
                (uint32_t)mul24(p.y, out.pw) + (uint32_t)p.x;
}
// the stores of an MB-grouped wave (k_intra_mbg, k_inter_mbg), all buffer
// stores with out-of-range offsets instead of branches: the wave's levels run
// (nvalid MBs x 768 bytes at coef + gmb0 x 768) from the LDS staging, the
// lane's 8 reconstructed rows (rec_off, plane width pw), and from the record
// lanes (rl) the MB record dword and the LastIntra byte of MB gmb
__device__ __forceinline__ void mbg_store(const p64gpu_encode_args &a, const uint8_t *lds, int lane,
                                          unsigned nmbs, unsigned gmb0, uint32_t nvalid, uint32_t rec_off,
                                          int pw, const uint2 rows[8], bool rl, unsigned gmb, uint32_t mbw,
                                          uint8_t li) {
  const int nfr = (int)(nmbs / (unsigned)((a.width >> 4) * (a.height >> 4)));
  const __amdgpu_buffer_rsrc_t coef =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.coef, (short)0, (int)(nmbs * 768u), BUF_RSRC_W3);
  const uint32_t nbytes = nvalid * 768u;
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
#if defined(PROBE_NOCOEF)  // development probes: drop one output stream (the work stays)
    __builtin_amdgcn_raw_buffer_store_b128(d, coef, BUF_OOB, 0, 0);
#else
    __builtin_amdgcn_raw_buffer_store_b128(d, coef, ob < nbytes ? gmb0 * 768u + ob : BUF_OOB, 0, 0);
#endif
  }
  __builtin_amdgcn_wave_barrier();
  const __amdgpu_buffer_rsrc_t rec =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.recon, (short)0, (int)(nfr * a.frame_stride), BUF_RSRC_W3);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 d;
    d[0] = rows[k].x;
    d[1] = rows[k].y;
#if defined(PROBE_NOREC)
    __builtin_amdgcn_raw_buffer_store_b64(d, rec, BUF_OOB, 0, 0);
#else
    __builtin_amdgcn_raw_buffer_store_b64(d, rec, rec_off + (uint32_t)mul24(k, pw), 0, 0);
#endif
  }
  const __amdgpu_buffer_rsrc_t mbr =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.mb, (short)0, (int)(nmbs * 4u), BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t lir =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.last_intra, (short)0, (int)nmbs, BUF_RSRC_W3);
  __builtin_amdgcn_raw_buffer_store_b32(mbw, mbr, rl ? 4u * gmb : BUF_OOB, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(li, lir, rl ? gmb : BUF_OOB, 0, 0);
}

// intra picture, MB-grouped block layout (blk_pos_mb): one wave = 10 MBs, a
// lane per block; levels leave as one contiguous 7,680-byte run per wave
template <bool QMB>
__global__ __launch_bounds__(256) BLK_OCC void k_intra_mbg(p64gpu_encode_args a, BlkDiv kd, unsigned nmbs) {
  __shared__ __align__(16) uint8_t lvl[4 * LVL_WAVE];
  const int lane = threadIdx.x & 63;
  uint8_t *lds = lvl + (threadIdx.x >> 6) * LVL_WAVE;
  const unsigned gmb0 = (blockIdx.x * 4u + (threadIdx.x >> 6)) * MBS_PER_WAVE;
  if (gmb0 >= nmbs) return;  // whole wave
  PRIO_HIGH();
  const int l = min(lane, 6 * MBS_PER_WAVE - 1);
  const unsigned gmb = min(gmb0 + (unsigned)(l / 6), nmbs - 1);  // tail lanes repeat the last MB
  const IntraFetch f = intra_fetch_at<QMB>(a, blk_pos_mb(gmb, l % 6, a.width, a.height, kd));
  PRIO_LOW();
  IntraOut o;
  const uint32_t nvalid = min((unsigned)MBS_PER_WAVE, nmbs - gmb0);
  intra_block(a, f, lds, lane, o);
  PRIO_ST();
  // the MB's record and LastIntra (p64.c:909-910: MTYPE 0, CBP 0x3f, LastIntra
  // reset) from lane b = 0 of each MB
  const bool rl = l % 6 == 0 && lane < 6 * MBS_PER_WAVE && gmb0 + (unsigned)(l / 6) < nmbs;
  mbg_store(a, lds, lane, nmbs, gmb0, nvalid, o.rec_off, o.pw, o.rec, rl, gmb, 0x3f00u, 0);
}

// The source of an 8x8 prediction at (x, y) of a plane (any byte alignment):
// three aligned dwords per row (the third only matters when the row is
// misaligned)
struct PredSrc {
  uint32_t d[8][3];
  int sh;
};
__device__ __forceinline__ void pred_row(const PredSrc &p, int r, int s[8]) {
  unpack8(align4(p.d[r][1], p.d[r][0], p.sh), align4(p.d[r][2], p.d[r][1], p.sh), s);
}
// horizontal taps of the H.261 loop filter: [1 2 1], edge columns x4
__device__ __forceinline__ void hz_row(const PredSrc &p, int r, int hz[8]) {
  int s[8];
  pred_row(p, r, s);
  hz[0] = s[0] << 2;
#pragma unroll
  for (int k = 1; k < 7; k++) hz[k] = s[k - 1] + 2 * s[k] + s[k + 1];
  hz[7] = s[7] << 2;
}
// v += prediction, row by row (the loop filter LoadFilterMatrix io.c:323-372
// when `filter`: separable [1 2 1], rows 0/7 not filtered vertically, one
// rounding (t + 8) >> 4 as in pred_from_row); three rows of taps live at once
__device__ __forceinline__ void add_pred(const PredSrc &p, bool filter, int v[64]) {
  if (filter) {
    int hp[8], hc[8], hn[8];
    hz_row(p, 0, hc);
    hz_row(p, 1, hn);
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++)
        v[8 * r + k] += (r == 0 || r == 7) ? ((hc[k] << 2) + 8) >> 4 : (hp[k] + 2 * hc[k] + hn[k] + 8) >> 4;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        hp[k] = hc[k];
        hc[k] = hn[k];
      }
      if (r + 2 < 8) hz_row(p, r + 2, hn);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      int s8[8];
      pred_row(p, r, s8);
#pragma unroll
      for (int k = 0; k < 8; k++) v[8 * r + k] += s8[k];
    }
  }
}

// decoder reconstruction (DecompressMDU p64.c:1179-1237 + DecodeSaveMDU
// p64.c:971-1013), block layout, persistent, as a two-stage load pipeline:
// while block i is transformed, the levels and prediction source of block
// i+1 (whose record arrived during block i-1) and the record of block i+2 are
// in flight.  Every load is a buffer load: where a block needs no levels
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
__device__ __forceinline__ RecStageA rec_stage_a(const RecBufs &B, int w, int h, const BlkDiv &kd,
                                                 unsigned t) {
  const int nmb = (w >> 4) * (h >> 4);
  RecStageA A;
  A.p = blk_pos(t, w, h, kd);
  const int gmb = A.p.fi * nmb + A.p.mb;
  A.m = __builtin_amdgcn_raw_buffer_load_b32(B.mb, 4 * gmb, 0, 0);
  A.q = __builtin_amdgcn_raw_buffer_load_b8(B.q, gmb, 0, 0);
  A.coded = __builtin_amdgcn_raw_buffer_load_b8(B.mask, gmb, 0, 0);
  return A;
}
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
  // the third dword only when the row is misaligned (then it lies inside the
  // row: sx <= pw - 9); an aligned row at the plane's end would reach past it
  const uint32_t po3 = S.pred.sh ? po + 8 : BUF_OOB;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(B.ref, po + (uint32_t)mul24(k, pw), 0, 0);
    S.pred.d[k][0] = v[0];
    S.pred.d[k][1] = v[1];
    S.pred.d[k][2] = __builtin_amdgcn_raw_buffer_load_b32(B.ref, po3 + (uint32_t)mul24(k, pw), 0, 0);
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
__device__ __forceinline__ void rec_block(int w, int h, int64_t stride, __amdgpu_buffer_rsrc_t rec,
                                          const RecStageA &A, const RecStageB &S) {
  const BlkPos &p = A.p;
  int v[64];
  if (S.ck) {  // IZigzagMatrix + ICCITT(Flat)Quantize straight from the packed levels
    const int q = A.q;
    const uint32_t q2 = 0x20002u * (uint32_t)q, qq = 0x10001u * (uint32_t)(q - (int)!(q & 1));
#pragma unroll
    for (int k = 0; k < 8; k++) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t d = dequantise_pk(S.lq[k][j], q2, qq);
#pragma unroll
        for (int i = 0; i < 2; i++) v[k_zz.inv[8 * k + 2 * j + i]] = i ? (int)d >> 16 : (int)(int16_t)(d & 0xffff);
      }
    }
    if (!S.inter) v[0] = (int)(int16_t)(S.lq[0][0] & 0xffff) * 8;  // intra DC
    idct_block(v);
  } else {
#pragma unroll
    for (int e = 0; e < 64; e++) v[e] = 0;
  }
  if (S.inter) add_pred(S.pred, S.filter, v);
#pragma unroll
  for (int e = 0; e < 64; e++) v[e] = clampi(v[e], 0, 255);  // BoundIDctMatrix
  PRIO_ST();
  // buffer stores, out of range (dropped) for MBs that are not coded: no
  // branch around the stores either
  const int pw = p.plane ? w >> 1 : w;
  const uint32_t ro = A.coded ? (uint32_t)((int64_t)p.fi * stride) + (uint32_t)plane_offset(p.plane, w, h) +
                                    (uint32_t)(mul24(p.y, pw) + p.x)
                              : BUF_OOB;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint2 r = pack8(v + 8 * k);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 d;
    d[0] = r.x;
    d[1] = r.y;
    __builtin_amdgcn_raw_buffer_store_b64(d, rec, ro + (uint32_t)mul24(k, pw), 0, 0);
  }
}
__global__ __launch_bounds__(256) BLK_OCC void k_recon_blk(int w, int h, int64_t stride, const uint8_t *refp,
                                                           uint8_t *recp, const int16_t *coef,
                                                           const p64_mb_rec *mbr, const uint8_t *quant_mb,
                                                           const uint8_t *coded_mask, BlkDiv kd,
                                                           unsigned total, unsigned gstride) {
  unsigned t = blockIdx.x * 256u + threadIdx.x;
  if (t >= total) return;
  const int nmb = (w >> 4) * (h >> 4), nfr = (int)(total / (unsigned)(6 * nmb));
  RecBufs B;
  B.ref = __builtin_amdgcn_make_buffer_rsrc((void *)refp, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  B.coef = __builtin_amdgcn_make_buffer_rsrc((void *)coef, (short)0, nfr * nmb * 768, BUF_RSRC_W3);
  B.mb = __builtin_amdgcn_make_buffer_rsrc((void *)mbr, (short)0, nfr * nmb * 4, BUF_RSRC_W3);
  B.q = __builtin_amdgcn_make_buffer_rsrc((void *)quant_mb, (short)0, nfr * nmb, BUF_RSRC_W3);
  B.mask = __builtin_amdgcn_make_buffer_rsrc((void *)coded_mask, (short)0, nfr * nmb, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t rec =
      __builtin_amdgcn_make_buffer_rsrc((void *)recp, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  const unsigned last = total - 1;
  RecStageA A0 = rec_stage_a(B, w, h, kd, t);
  RecStageA A1 = rec_stage_a(B, w, h, kd, min(t + gstride, last));
  RecStageB S0 = rec_stage_b(B, w, h, stride, A0);
  // drain the pipeline fill: entering the loop with nothing pending keeps
  // hipcc's wait counts inside it exact
  __builtin_amdgcn_s_waitcnt(0);
  // unrolled by two so the stage-B registers alternate between S0 and S1
  // instead of being copied (and waited for) at the back-edge
  for (;;) {  // every lane reaches t >= total: no lane is left behind
    const RecStageA A2 = rec_stage_a(B, w, h, kd, min(t + 2 * gstride, last));  // block i+2
    const RecStageB S1 = rec_stage_b(B, w, h, stride, A1);                      // block i+1
    rec_block(w, h, stride, rec, A0, S0);
    if (t + gstride >= total) break;
    const RecStageA A3 = rec_stage_a(B, w, h, kd, min(t + 3 * gstride, last));  // block i+3
    S0 = rec_stage_b(B, w, h, stride, A2);                                      // block i+2
    rec_block(w, h, stride, rec, A1, S1);
    if (t + 2 * gstride >= total) break;
    A0 = A2;
    A1 = A3;
    t += 2 * gstride;
  }
}

// pred_rows (below) + dequantise + ChenIDct + reconstruction for the
// non-persistent decoder: the prediction is formed first and kept as 8 packed
// rows (16 registers instead of the 24-dword source), the dequantisation and
// IDCT run unconditionally (an uncoded block's levels were read as zeros and
// give a zero residual), so the register peak is the IDCT's
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
__device__ __forceinline__ void rec_block_pk(int w, int h, int64_t stride, __amdgpu_buffer_rsrc_t rec,
                                             const RecStageA &A, const RecStageB &S) {
  const BlkPos &p = A.p;
  uint2 prow[8];
  pred_rows(S.pred, S.filter && S.inter, prow);  // zeros for intra (source not loaded)
  int v[64];
  const int q = A.q;
  const uint32_t q2 = 0x20002u * (uint32_t)q, qq = 0x10001u * (uint32_t)(q - (int)!(q & 1));
  // natural level pairs straight from the packed zigzag words (one v_perm each)
  auto pair = [&](int e, int f) {
    const int s1 = k_zz.pos[e], s2 = k_zz.pos[f];
    const uint32_t sel = ((s1 & 1) ? 0x0302u : 0x0100u) | (((s2 & 1) ? 0x0706u : 0x0504u) << 16);
    return __builtin_amdgcn_perm(S.lq[s2 >> 3][(s2 >> 1) & 3], S.lq[s1 >> 3][(s1 >> 1) & 3], sel);
  };
  iq_idct_cols(pair, q2, qq, !S.inter, (int)(int16_t)(S.lq[0][0] & 0xffff) * 8, v);
  idct_rows(v);
  PRIO_ST();
  const int pw = p.plane ? w >> 1 : w;
  const uint32_t ro = A.coded ? (uint32_t)((int64_t)p.fi * stride) + (uint32_t)plane_offset(p.plane, w, h) +
                                    (uint32_t)(mul24(p.y, pw) + p.x)
                              : BUF_OOB;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint2 r = recon_row(v + 8 * k, prow[k]);  // + prediction, BoundIDctMatrix
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 d;
    d[0] = r.x;
    d[1] = r.y;
    __builtin_amdgcn_raw_buffer_store_b64(d, rec, ro + (uint32_t)mul24(k, pw), 0, 0);
  }
}
#ifndef INTER_WAVES
#define INTER_WAVES 4
#endif
#define INTER_OCC __attribute__((amdgpu_waves_per_eu(INTER_WAVES)))
#ifndef RECON_WAVES
#define RECON_WAVES 3
#endif
#define RECON_OCC __attribute__((amdgpu_waves_per_eu(RECON_WAVES)))
// decoder reconstruction, MB-grouped block layout (blk_pos_mb), one block per
// lane and no loop: 10 MBs per wave, each lane loads its MB's record, then its
// levels and prediction, reconstructs and stores.  Without the persistent
// kernel's in-flight registers it fits 3 waves per SIMD (139 VGPRs), and those
// waves hide each other's two dependent load latencies (measured faster than
// k_recon_blk, whose 237 VGPRs allow 2).  Lanes past the batch (and lanes
// 60..63) get coded = 0: every load and store of theirs is out of range.
__global__ __launch_bounds__(256) RECON_OCC void k_recon_mbg(int w, int h, int64_t stride, const uint8_t *refp,
                                                           uint8_t *recp, const int16_t *coef,
                                                           const p64_mb_rec *mbr, const uint8_t *quant_mb,
                                                           const uint8_t *coded_mask, BlkDiv kd, unsigned nmbs) {
  const int lane = threadIdx.x & 63;
  const unsigned gmb0 = (blockIdx.x * 4u + (threadIdx.x >> 6)) * MBS_PER_WAVE;
  if (gmb0 >= nmbs) return;  // whole wave
  const int nmb = (w >> 4) * (h >> 4), nfr = (int)(nmbs / (unsigned)nmb);
  RecBufs B;
  B.ref = __builtin_amdgcn_make_buffer_rsrc((void *)refp, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  B.coef = __builtin_amdgcn_make_buffer_rsrc((void *)coef, (short)0, nfr * nmb * 768, BUF_RSRC_W3);
  B.mb = __builtin_amdgcn_make_buffer_rsrc((void *)mbr, (short)0, nfr * nmb * 4, BUF_RSRC_W3);
  B.q = __builtin_amdgcn_make_buffer_rsrc((void *)quant_mb, (short)0, nfr * nmb, BUF_RSRC_W3);
  B.mask = __builtin_amdgcn_make_buffer_rsrc((void *)coded_mask, (short)0, nfr * nmb, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t rec =
      __builtin_amdgcn_make_buffer_rsrc((void *)recp, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  PRIO_HIGH();
  const int l = min(lane, 6 * MBS_PER_WAVE - 1);
  const unsigned g = gmb0 + (unsigned)(l / 6);
  const bool valid = lane < 6 * MBS_PER_WAVE && g < nmbs;
  const unsigned gmb = min(g, nmbs - 1);
  RecStageA A;
  A.p = blk_pos_mb(gmb, l % 6, w, h, kd);
  A.m = __builtin_amdgcn_raw_buffer_load_b32(B.mb, 4 * gmb, 0, 0);
  A.q = __builtin_amdgcn_raw_buffer_load_b8(B.q, gmb, 0, 0);
  A.coded = __builtin_amdgcn_raw_buffer_load_b8(B.mask, valid ? gmb : BUF_OOB, 0, 0);
  const RecStageB S = rec_stage_b(B, w, h, stride, A);
  PRIO_LOW();
  rec_block_pk(w, h, stride, rec, A, S);
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
// the prediction as packed rows (all zero when the source was not loaded)
__device__ __forceinline__ void pred_rows(const PredSrc &P, bool filter, uint2 prow[8]) {
  if (filter) {  // add_pred's loop filter, one packed row at a time
    int hp[8], hc[8], hn[8];
    hz_row(P, 0, hc);
    hz_row(P, 1, hn);
#pragma unroll
    for (int r = 0; r < 8; r++) {
      int o[8];
#pragma unroll
      for (int k = 0; k < 8; k++)
        o[k] = (r == 0 || r == 7) ? ((hc[k] << 2) + 8) >> 4 : (hp[k] + 2 * hc[k] + hn[k] + 8) >> 4;
      prow[r] = pack8(o);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        hp[k] = hc[k];
        hc[k] = hn[k];
      }
      if (r + 2 < 8) hz_row(P, r + 2, hn);
    }
  } else {  // the source rows as they are
#pragma unroll
    for (int r = 0; r < 8; r++)
      prow[r] = make_uint2(align4(P.d[r][1], P.d[r][0], P.sh), align4(P.d[r][2], P.d[r][1], P.sh));
  }
}
template <bool QMB>
__global__ __launch_bounds__(256) INTER_OCC void k_inter_mbg(p64gpu_encode_args a, BlkDiv kd, unsigned nmbs,
                                                             const p64_me_rec *me) {
  __shared__ __align__(16) uint8_t lvl[4 * LVL_WAVE];
  const int lane = threadIdx.x & 63;
  uint8_t *lds = lvl + (threadIdx.x >> 6) * LVL_WAVE;
  const unsigned gmb0 = (blockIdx.x * 4u + (threadIdx.x >> 6)) * MBS_PER_WAVE;
  if (gmb0 >= nmbs) return;  // whole wave
  const int w = a.width, h = a.height, nmb = (w >> 4) * (h >> 4), nfr = (int)(nmbs / (unsigned)nmb);
  const int64_t stride = a.frame_stride;
  RecBufs B;
  B.ref = __builtin_amdgcn_make_buffer_rsrc((void *)a.ref, (short)0, (int)(nfr * stride), BUF_RSRC_W3);
  PRIO_HIGH();
  const int l = min(lane, 6 * MBS_PER_WAVE - 1), b = l % 6;
  const unsigned gmb = min(gmb0 + (unsigned)(l / 6), nmbs - 1);  // tail lanes repeat the last MB
  const BlkPos pos = blk_pos_mb(gmb, b, w, h, kd);
  // the ME record, LastIntra and override first: the prediction loads wait
  // on them (wait counts are in issue order), the current rows only later
  const __amdgpu_buffer_rsrc_t mer =
      __builtin_amdgcn_make_buffer_rsrc((void *)me, (short)0, (int)(nmbs * sizeof(p64_me_rec)), BUF_RSRC_W3);
  const uint32_t mo = gmb * (uint32_t)sizeof(p64_me_rec);
  InterMe m;
  m.mx = (int)__builtin_amdgcn_raw_buffer_load_b32(mer, mo + 0, 0, 0);
  m.my = (int)__builtin_amdgcn_raw_buffer_load_b32(mer, mo + 4, 0, 0);
  m.sad = (int)__builtin_amdgcn_raw_buffer_load_b32(mer, mo + 8, 0, 0);
  m.sad0 = (int)__builtin_amdgcn_raw_buffer_load_b32(mer, mo + 12, 0, 0);
  m.var = (int)__builtin_amdgcn_raw_buffer_load_b32(mer, mo + 16, 0, 0);
  m.varor = (int)__builtin_amdgcn_raw_buffer_load_b32(mer, mo + 20, 0, 0);
  // LastIntra and the -o override by buffer loads (an absent override array
  // reads as out of range: no branch around a load)
  const __amdgpu_buffer_rsrc_t lir =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.last_intra, (short)0, (int)nmbs, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t ovr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)a.mtype_override, (short)0, a.mtype_override ? (int)nmbs : 0, BUF_RSRC_W3);
  const int li = __builtin_amdgcn_raw_buffer_load_b8(lir, gmb, 0, 0);
  const int ovl = (int)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(ovr, a.mtype_override ? gmb : BUF_OOB, 0, 0);
  const int ov = a.mtype_override ? ovl : -1;
  const IntraFetch f = intra_fetch_at<QMB>(a, pos);  // current rows, q

  // MTYPE (p64.c:734-772): the decision, the -o override, the intra refresh
  MeOut mo_;
  mo_.mx = m.mx;
  mo_.my = m.my;
  mo_.sad = m.sad;
  mo_.sad0 = m.sad0;
  mo_.var = m.var;
  mo_.varor = m.varor;
  mo_.mwor = 0;
  int mt = decide_mtype(mo_);
  if (ov >= 0) mt = ov;
  if (li > 131) mt = 0;
  const int mvx = m.mx, mvy = m.my;
  uint2 prow[8];
  inter_pred(B, w, h, stride, pos, mt, mvx, mvy, prow);  // (drops the priority)

  const bool intra = mt_intra(mt), tc = mt_tcoeff(mt);
  const int q = f.q;
  const float rq = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, 1.0f / (float)(2 * q)) + 1u);
  const float rqe = (q & 1) ? 0.0f : rq;
  const int qe = (int)!(q & 1), qbr = 256 * q - 1 - qe, qb = min(1023, qbr);
  // levels & tcm: 0 when the MB type carries no coefficients (through an
  // opaque mask: as a select hipcc branches around every quantisation)
  const int tcm = opaque(tc ? -1 : 0);
  int v[64];
  fdct_block_pk<true>(f.rows, v, prow);
  // quantise in scan order into the LDS staging (levels of a block whose MB
  // type carries no coefficients are 0); Σ l^2 for the CBP decision:
  // Σ|l| > 1 <=> Σ l^2 > 1 and Σ|l| > 0 <=> Σ l^2 > 0 for integers
  int ss = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int l2[2];
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const int e = k_zz.inv[8 * k + 2 * j + i];
        if (e == 0) {  // DC: intra (DC +- 4) / 8 in 1..254, inter as AC with DC bounds
          const int c = dct_final(v[0]);
          int vi;
          asm("v_med3_i32 %0, %1, %2, %3" : "=v"(vi) : "v"(c), "v"(-qbr), "v"(min(2047, qbr)));
          const float x = (float)vi;
          const int li_ = (int)__builtin_fmaf(x, rq, __builtin_copysignf(rqe, x));
          const int ld = clampi(dct_final(min(c, 2047)), 1, 254);
          l2[i] = intra ? ld : li_;
        } else {
          l2[i] = quantise<false, true>(v[e], -qb, qb, false, rq, rqe);
        }
        l2[i] &= tcm;
      }
      pk[j] = __builtin_amdgcn_perm((uint32_t)l2[1], (uint32_t)l2[0], 0x05040100u);
      ss = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, pk[j]), __builtin_bit_cast(s16x2, pk[j]), ss, false);
      v[k_zz.inv[8 * k + 2 * j]] = l2[0];
      v[k_zz.inv[8 * k + 2 * j + 1]] = l2[1];
    }
    put_levels(lds, lane, k, make_uint4(pk[0], pk[1], pk[2], pk[3]));
    SCHED_FENCE();
  }
  // CBP (p64.c:887-908): block coded if Σ|l| > 1; none such -> the first
  // block with a nonzero level; no nonzero level at all -> MC without
  // coefficients (MTYPE 4 / 7), vector kept, CBP 0x3f
  const int sh = 6 * (l / 6);
  const uint32_t big = (uint32_t)(__ballot(ss > 1) >> sh) & 63u, any = (uint32_t)(__ballot(ss > 0) >> sh) & 63u;
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
  const uint32_t q2 = ck ? 0x20002u * (uint32_t)q : 0u, qq = ck ? 0x10001u * (uint32_t)(q - qe) : 0u;
  // IQ in level pairs + ChenIDct (all-zero levels / q2 = qq = 0 give zero)
  iq_idct_cols([&](int e, int f) { return pk2(v[e], v[f]); }, q2, qq, intra, v[0] * 8, v);
  idct_rows(v);
#pragma unroll
  for (int k = 0; k < 8; k++) prow[k] = recon_row(v + 8 * k, prow[k]);  // now the reconstructed rows
  // no levels at all in the MB: the reconstruction is the new prediction
  // (late, so its registers do not overlap the block's)
  if (repred) inter_pred(B, w, h, stride, pos, mt, mvx, mvy, prow);
  const uint32_t nvalid = min((unsigned)MBS_PER_WAVE, nmbs - gmb0);
  const int pw = pos.plane ? w >> 1 : w;
  const uint32_t ro = (uint32_t)((int64_t)pos.fi * stride) + (uint32_t)plane_offset(pos.plane, w, h) +
                      (uint32_t)mul24(pos.y, pw) + (uint32_t)pos.x;
  // p64.c:909-910: the record (transmitted vector only for MC types) and LastIntra
  const bool rl = b == 0 && lane < 6 * MBS_PER_WAVE && gmb0 + (unsigned)(l / 6) < nmbs;
  const uint32_t mbw = (uint32_t)(mt & 0xff) | ((uint32_t)(cbp & 0xff) << 8) |
                       (mt_mf(mt) ? ((uint32_t)(mvx & 0xff) << 16) | ((uint32_t)(mvy & 0xff) << 24) : 0u);
  mbg_store(a, lds, lane, nmbs, gmb0, nvalid, ro, pw, prow, rl, gmb, mbw,
            mt_intra(mt) ? (uint8_t)0 : (uint8_t)(li + 1));
}

// batched 8x8 block operations (one thread per block; shares the device
// functions of the fused kernels, full 32-bit arithmetic for arbitrary input)
__global__ void k_block_op(int op, const int32_t *in, int32_t *out, int64_t nblocks, int dcq,
                           int acq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nblocks) return;
  int m[64], t[64];
  const int32_t *src = in + i * 64;
  int32_t *dst = out + i * 64;
  for (int n = 0; n < 64; n++) m[n] = src[n];
  switch (op) {
    case P64GPU_OP_DCT: {
      int x[8], o[8];
      for (int c = 0; c < 8; c++) {
        for (int k = 0; k < 8; k++) x[k] = m[8 * k + c];
        fwd_col<false>(x, o);
        for (int k = 0; k < 8; k++) t[8 * k + c] = o[k];
      }
      for (int rr = 0; rr < 8; rr++) {
        for (int k = 0; k < 8; k++) x[k] = t[8 * rr + k];
        fwd_row<false>(x, o);
        for (int k = 0; k < 8; k++) m[8 * rr + k] = dct_final(o[k]);
      }
      break;
    }
    case P64GPU_OP_IDCT: {
      int x[8], o[8];
      for (int c = 0; c < 8; c++) {
        for (int k = 0; k < 8; k++) x[k] = m[8 * k + c] << 2;
        inv8<false>(x, o);
        for (int k = 0; k < 8; k++) t[8 * k + c] = o[k];
      }
      for (int rr = 0; rr < 8; rr++) {
        for (int k = 0; k < 8; k++) x[k] = t[8 * rr + k];
        inv8<false>(x, o);
        for (int k = 0; k < 8; k++) m[8 * rr + k] = idct_final(o[k]);
      }
      break;
    }
    case P64GPU_OP_QUANT_INTRA:
      m[0] = qdc_intra(m[0], dcq);
      for (int n = 1; n < 64; n++) m[n] = qlevel(m[n], acq);
      break;
    case P64GPU_OP_QUANT_INTER:
      m[0] = qlevel(m[0], dcq);
      for (int n = 1; n < 64; n++) m[n] = qlevel(m[n], acq);
      break;
    case P64GPU_OP_IQUANT_INTRA:
      m[0] = m[0] * dcq;
      for (int n = 1; n < 64; n++) m[n] = rlevel<false>(m[n], acq);
      break;
    case P64GPU_OP_IQUANT_INTER:
      m[0] = rlevel<false>(m[0], dcq);
      for (int n = 1; n < 64; n++) m[n] = rlevel<false>(m[n], acq);
      break;
    case P64GPU_OP_BOUND_DCT:
      m[0] = min(m[0], 2047);
      for (int n = 1; n < 64; n++) m[n] = clampi(m[n], -1023, 1023);
      break;
    case P64GPU_OP_BOUND_IDCT:
      for (int n = 0; n < 64; n++) m[n] = clampi(m[n], 0, 255);
      break;
    case P64GPU_OP_BOUND_QFLAT:
      m[0] = clampi(m[0], 1, 254);
      for (int n = 1; n < 64; n++) m[n] = clampi(m[n], -127, 127);
      break;
    case P64GPU_OP_BOUND_QUANT:
      for (int n = 0; n < 64; n++) m[n] = clampi(m[n], -127, 127);
      break;
    case P64GPU_OP_ZIGZAG:
      for (int n = 0; n < 64; n++) t[c_zz.pos[n]] = m[n];
      for (int n = 0; n < 64; n++) m[n] = t[n];
      break;
    case P64GPU_OP_IZIGZAG:
      for (int n = 0; n < 64; n++) t[n] = m[c_zz.pos[n]];
      for (int n = 0; n < 64; n++) m[n] = t[n];
      break;
    default:
      break;
  }
  for (int n = 0; n < 64; n++) dst[n] = m[n];
}

// deterministic synthetic pictures on the device (same bytes as synth.c):
// picture (t, s) = stream seed0+s, frame frame0+t, at out + (t*nseeds+s)*stride
__global__ __launch_bounds__(256) void k_synth(int w, int h, uint32_t seed0, int nseeds,
                                               int frame0, int64_t stride, uint8_t *out) {
  const int pic = blockIdx.y;
  const int t = pic / nseeds, sidx = pic - t * nseeds;
  const uint32_t seed = seed0 + (uint32_t)sidx;
  const int frame = frame0 + t;
  uint8_t *y = out + (size_t)pic * stride;
  uint8_t *u = y + (size_t)w * h, *v = u + (size_t)(w / 2) * (h / 2);
  const int nl = w * h, nc = (w / 2) * (h / 2);
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < nl + nc; k += gridDim.x * blockDim.x) {
    if (k < nl) {
      y[k] = p64s_luma(seed, frame, k % w, k / w);
    } else {
      const int c = k - nl;
      p64s_chroma(seed, frame, c % (w / 2), c / (w / 2), &u[c], &v[c]);
    }
  }
}

// ---------------------------------------------------------------------------
// host-side validation

int check_geometry(int w, int h, int nframes, int64_t stride, bool luma_only = false) {
  if (w < 32 || h < 32 || w > 4096 || h > 4096 || (w & 15) || (h & 15))
    return fail(P64GPU_E_INVALID, "picture %dx%d: need multiples of 16 in 32..4096", w, h);
  if (nframes < 1) return fail(P64GPU_E_INVALID, "nframes %d < 1", nframes);
  const int64_t need = luma_only ? (int64_t)w * h : (int64_t)w * h * 3 / 2;
  if (stride < need || (stride & 15))
    return fail(P64GPU_E_INVALID, "frame_stride %lld: need >= %lld and a multiple of 16",
                (long long)stride, (long long)need);
  const int64_t blocks = (int64_t)nframes * (w / 16) * (h / 16);
  if (blocks >= (1LL << 30)) return fail(P64GPU_E_INVALID, "too many macroblocks in one call");
  return P64GPU_OK;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// Workgroups of 256 for a persistent block-layout kernel: as many as are
// resident at once (occupancy x CUs of the current device), at most one per
// 256 blocks.
int persistent_grid(const void *kernel, int64_t blocks, unsigned *wg) {
  static int cus[64], nb_cache[64][4];
  static const void *kern_cache[64][4];
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return fail(P64GPU_E_INVALID, "device %d", dev);
  if (!cus[dev]) HIP_TRY(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
  int nb = 0;
  for (int i = 0; i < 4; i++)
    if (kern_cache[dev][i] == kernel) nb = nb_cache[dev][i];
  if (!nb) {
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 256, 0));
    if (nb < 1) nb = 1;
    for (int i = 0; i < 4; i++)
      if (!kern_cache[dev][i]) {
        kern_cache[dev][i] = kernel;
        nb_cache[dev][i] = nb;
        break;
      }
  }
  const int64_t need = (blocks + 255) / 256, have = (int64_t)nb * cus[dev];
  *wg = (unsigned)(need < have ? need : have);
  return P64GPU_OK;
}

// P64GPU_MB_LAYOUT=1 (read once): intra pictures and decoder reconstruction
// take the one-wave-per-MB kernels (k_encode<0>, k_decode_recon) instead of
// the block-layout ones -- an A/B and cross-check switch, same results
bool mb_layout_forced() {
  static const bool forced = [] {
    const char *e = getenv("P64GPU_MB_LAYOUT");
    return e && *e && *e != '0';
  }();
  return forced;
}
// P64GPU_FUSED=1: inter pictures through the fused one-wave-per-MB k_encode
// instead of k_motion + k_inter_mbg (kept for A/B measurements and as the
// path of mb-list encodes)
bool fused_forced() {
  static const bool on = [] {
    const char *e = getenv("P64GPU_FUSED");
    return e && *e && *e != '0';
  }();
  return on;
}
// device scratch for the ME records of the split inter encoder when the
// caller does not ask for them (args.me == NULL): grown outside stream
// capture only (NULL during a capture that would need a larger one: the
// caller then takes the fused kernel), one per process and device
static std::mutex g_me_mu;
static p64_me_rec *g_me_buf = nullptr;
static size_t g_me_cap = 0;
static int g_me_dev = -1;
static p64_me_rec *me_scratch(size_t n, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_me_mu);
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (g_me_buf && g_me_dev == dev && n <= g_me_cap) return g_me_buf;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  if (g_me_buf && g_me_dev != dev) return nullptr;  // first device keeps it
  if (g_me_buf) {
    if (hipDeviceSynchronize() != hipSuccess) return nullptr;  // in-flight users of the old one
    (void)hipFree(g_me_buf);
    g_me_buf = nullptr;
    g_me_cap = 0;
  }
  void *p = nullptr;
  if (hipMalloc(&p, n * sizeof(p64_me_rec)) != hipSuccess) return nullptr;
  g_me_buf = static_cast<p64_me_rec *>(p);
  g_me_cap = n;
  g_me_dev = dev;
  return g_me_buf;
}

// pictures per launch of the block-layout kernels: every buffer of a launch
// within the 2 GiB of a 32-bit buffer offset (per = the larger of a picture's
// bytes and its levels' bytes).  P64GPU_CHUNK_BYTES lowers the limit (tests
// exercise the split launches with it); read on every call.
int pictures_per_launch(int64_t per) {
  int64_t lim = ((int64_t)1 << 31) - 1;
  const char *e = getenv("P64GPU_CHUNK_BYTES");
  if (e && *e) {
    const long long v = atoll(e);
    if (v > 0 && v < lim) lim = v;
  }
  const int64_t n = lim / per;
  return n < 1 ? 1 : (int)n;
}
// P64GPU_RECON_PERSISTENT=1: the persistent pipelined decoder k_recon_blk
// instead of k_recon_mbg (kept for A/B measurements)
bool recon_persistent() {
  static const bool on = [] {
    const char *e = getenv("P64GPU_RECON_PERSISTENT");
    return e && *e && *e != '0';
  }();
  return on;
}

}  // namespace

// ===========================================================================
// C ABI

extern "C" {

int p64gpu_abi_version(void) { return P64GPU_ABI_VERSION; }

const char *p64gpu_strerror(int s) {
  switch (s) {
    case P64GPU_OK: return "ok";
    case P64GPU_E_INVALID: return "invalid argument";
    case P64GPU_E_NODEVICE: return "no HIP device";
    case P64GPU_E_HIP: return "HIP runtime error";
    case P64GPU_E_NOMEM: return "out of memory";
    case P64GPU_E_STREAM: return "bitstream error";
    default: return "unknown status";
  }
}

const char *p64gpu_last_error(void) { return g_err; }

// error reporting for the host C parts of the library (p64stream.c)
int p64gpu_fail_(int status, const char *msg) { return fail(status, "%s", msg); }

int p64gpu_device_count(int *count) {
  if (!count) return fail(P64GPU_E_INVALID, "count is NULL");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return P64GPU_OK;
}

int p64gpu_set_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(P64GPU_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return fail(P64GPU_E_INVALID, "device %d of %d", device, n);
  HIP_TRY(hipSetDevice(device));
  return P64GPU_OK;
}

int p64gpu_synchronize(void *stream) {
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_alloc(void **ptr, size_t bytes) {
  if (!ptr) return fail(P64GPU_E_INVALID, "ptr is NULL");
  *ptr = nullptr;
  if (hipMalloc(ptr, bytes ? bytes : 1) != hipSuccess)
    return fail(P64GPU_E_NOMEM, "hipMalloc(%zu) failed", bytes);
  return P64GPU_OK;
}

int p64gpu_free(void *ptr) {
  if (ptr) HIP_TRY(hipFree(ptr));
  return P64GPU_OK;
}

int p64gpu_copy_to_device(void *dst, const void *src, size_t bytes, void *stream) {
  if ((!dst || !src) && bytes) return fail(P64GPU_E_INVALID, "NULL copy operand");
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_copy_to_host(void *dst, const void *src, size_t bytes, void *stream) {
  if ((!dst || !src) && bytes) return fail(P64GPU_E_INVALID, "NULL copy operand");
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_copy_on_device(void *dst, const void *src, size_t bytes, void *stream) {
  if ((!dst || !src) && bytes) return fail(P64GPU_E_INVALID, "NULL copy operand");
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_block_op(int op, const int32_t *in, int32_t *out, int64_t nblocks, int dcq, int acq,
                    void *stream) {
  if (op < 0 || op >= P64GPU_OP_COUNT) return fail(P64GPU_E_INVALID, "block op %d", op);
  if (nblocks < 0) return fail(P64GPU_E_INVALID, "nblocks %lld", (long long)nblocks);
  if (nblocks == 0) return P64GPU_OK;
  if (!in || !out) return fail(P64GPU_E_INVALID, "NULL block buffer");
  const bool q = op >= P64GPU_OP_QUANT_INTRA && op <= P64GPU_OP_IQUANT_INTER;
  if (q && (dcq < 1 || acq < 1 || dcq > 255 || acq > 31))
    return fail(P64GPU_E_INVALID, "quantiser steps dcq=%d acq=%d", dcq, acq);
  const int threads = 64;
  const int64_t grid = (nblocks + threads - 1) / threads;
  if (grid > 0x7fffffffLL) return fail(P64GPU_E_INVALID, "nblocks too large");
  hipLaunchKernelGGL(k_block_op, dim3((unsigned)grid), dim3(threads), 0, (hipStream_t)stream, op,
                     in, out, nblocks, dcq, acq);
  HIP_TRY(hipGetLastError());
  return P64GPU_OK;
}

int p64gpu_motion_estimation(int w, int h, int nframes, int64_t stride, const uint8_t *ref_y,
                             const uint8_t *cur_y, int mode, int sl, p64_me_rec *out,
                             void *stream) {
  int s = check_geometry(w, h, nframes, stride, true);
  if (s) return s;
  if (!ref_y || !cur_y || !out) return fail(P64GPU_E_INVALID, "NULL buffer");
  if (!aligned16(ref_y) || !aligned16(cur_y)) return fail(P64GPU_E_INVALID, "planes must be 16-byte aligned");
  if (mode != P64GPU_ME_TSS && mode != P64GPU_ME_FULL) return fail(P64GPU_E_INVALID, "me mode %d", mode);
  if (sl < 1 || sl > 31) return fail(P64GPU_E_INVALID, "search_limit %d not in 1..31", sl);
  const unsigned grid = (unsigned)((int64_t)nframes * (w / 16) * (h / 16));
  hipStream_t st = (hipStream_t)stream;
  if (mode == P64GPU_ME_FULL)
    hipLaunchKernelGGL(k_motion<2>, dim3(grid), dim3(64), 0, st, w, h, stride, ref_y, cur_y, sl, out,
                       mb_div(w, h));
  else
    hipLaunchKernelGGL(k_motion<1>, dim3(grid), dim3(64), 0, st, w, h, stride, ref_y, cur_y, sl, out,
                       mb_div(w, h));
  HIP_TRY(hipGetLastError());
  return P64GPU_OK;
}

static int encode_launch(const p64gpu_encode_args *a, const int32_t *mb_list, int count,
                         void *stream);

int p64gpu_encode_frames(const p64gpu_encode_args *a, void *stream) {
  return encode_launch(a, nullptr, 0, stream);
}

int p64gpu_encode_mb_list(const p64gpu_encode_args *a, const int32_t *mb_list, int count,
                          void *stream) {
  if (!a) return fail(P64GPU_E_INVALID, "args is NULL");
  if (a->nframes != 1) return fail(P64GPU_E_INVALID, "mb list needs nframes = 1");
  if (!mb_list || count < 0 || count > (a->width / 16) * (a->height / 16))
    return fail(P64GPU_E_INVALID, "mb list %p count %d", (const void *)mb_list, count);
  if (count == 0) return P64GPU_OK;
  return encode_launch(a, mb_list, count, stream);
}

static int encode_launch(const p64gpu_encode_args *a, const int32_t *mb_list, int count,
                         void *stream) {
  if (!a) return fail(P64GPU_E_INVALID, "args is NULL");
  int s = check_geometry(a->width, a->height, a->nframes, a->frame_stride);
  if (s) return s;
  if (!a->cur || !a->recon || !a->last_intra || !a->coef || !a->mb)
    return fail(P64GPU_E_INVALID, "NULL required buffer");
  if (!a->intra && !a->ref) return fail(P64GPU_E_INVALID, "inter picture needs ref");
  if (!aligned16(a->cur) || !aligned16(a->recon) || !aligned16(a->coef) ||
      (!a->intra && !aligned16(a->ref)))
    return fail(P64GPU_E_INVALID, "cur/ref/recon/coef must be 16-byte aligned");
  if (a->quant < 1 || a->quant > 31) return fail(P64GPU_E_INVALID, "quant %d not in 1..31", a->quant);
  if (a->me_mode != P64GPU_ME_TSS && a->me_mode != P64GPU_ME_FULL)
    return fail(P64GPU_E_INVALID, "me mode %d", a->me_mode);
  if (a->search_limit < 1 || a->search_limit > 31)
    return fail(P64GPU_E_INVALID, "search_limit %d not in 1..31", a->search_limit);
  if (a->reserved != 0) return fail(P64GPU_E_INVALID, "reserved must be 0");
  const unsigned grid =
      mb_list ? (unsigned)count : (unsigned)((int64_t)a->nframes * (a->width / 16) * (a->height / 16));
  hipStream_t st = (hipStream_t)stream;
  const MbDiv kd = mb_div(a->width, a->height);
  const int64_t blocks = 6 * (int64_t)grid;
  if (a->intra && !mb_list && blocks < (1LL << 30) && !mb_layout_forced()) {
    // pictures per launch: pictures and levels of a launch within 2 GiB
    const int nmb = (a->width / 16) * (a->height / 16);
    const int64_t per = (int64_t)nmb * 768 > a->frame_stride ? (int64_t)nmb * 768 : a->frame_stride;
    const int chunk = pictures_per_launch(per);
    for (int f0 = 0; f0 < a->nframes; f0 += chunk) {
      p64gpu_encode_args c = *a;
      c.nframes = a->nframes - f0 < chunk ? a->nframes - f0 : chunk;
      const size_t m0 = (size_t)f0 * nmb;
      c.cur = a->cur + (size_t)f0 * a->frame_stride;
      c.recon = a->recon + (size_t)f0 * a->frame_stride;
      c.last_intra = a->last_intra + m0;
      c.quant_mb = a->quant_mb ? a->quant_mb + m0 : nullptr;
      c.coef = a->coef + m0 * 384;
      c.mb = a->mb + m0;
      const int64_t nm = (int64_t)c.nframes * nmb, waves = (nm + MBS_PER_WAVE - 1) / MBS_PER_WAVE;
      if (c.quant_mb)
        hipLaunchKernelGGL(k_intra_mbg<true>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, c,
                           blk_div(a->width, a->height), (unsigned)nm);
      else
        hipLaunchKernelGGL(k_intra_mbg<false>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, c,
                           blk_div(a->width, a->height), (unsigned)nm);
      HIP_TRY(hipGetLastError());
    }
    return P64GPU_OK;
  } else if (!a->intra && !mb_list && blocks < (1LL << 30) && !mb_layout_forced() && !fused_forced()) {
    // split encoder: ME for the whole batch, then the block-layout rest
    const int nmb = (a->width / 16) * (a->height / 16);
    p64_me_rec *me = a->me ? a->me : me_scratch((size_t)a->nframes * nmb, st);
    if (me) {
      const int mode = a->me_mode == P64GPU_ME_FULL ? 2 : 1;
      if (mode == 2)
        hipLaunchKernelGGL(k_motion<2>, dim3(grid), dim3(64), 0, st, a->width, a->height, a->frame_stride,
                           a->ref, a->cur, a->search_limit, me, kd);
      else
        hipLaunchKernelGGL(k_motion<1>, dim3(grid), dim3(64), 0, st, a->width, a->height, a->frame_stride,
                           a->ref, a->cur, a->search_limit, me, kd);
      HIP_TRY(hipGetLastError());
      const int64_t per = (int64_t)nmb * 768 > a->frame_stride ? (int64_t)nmb * 768 : a->frame_stride;
      const int chunk = pictures_per_launch(per);
      for (int f0 = 0; f0 < a->nframes; f0 += chunk) {
        p64gpu_encode_args c = *a;
        c.nframes = a->nframes - f0 < chunk ? a->nframes - f0 : chunk;
        const size_t m0 = (size_t)f0 * nmb;
        c.cur = a->cur + (size_t)f0 * a->frame_stride;
        c.ref = a->ref + (size_t)f0 * a->frame_stride;
        c.recon = a->recon + (size_t)f0 * a->frame_stride;
        c.last_intra = a->last_intra + m0;
        c.quant_mb = a->quant_mb ? a->quant_mb + m0 : nullptr;
        c.mtype_override = a->mtype_override ? a->mtype_override + m0 : nullptr;
        c.coef = a->coef + m0 * 384;
        c.mb = a->mb + m0;
        c.me = nullptr;
        const int64_t nm = (int64_t)c.nframes * nmb, waves = (nm + MBS_PER_WAVE - 1) / MBS_PER_WAVE;
        if (c.quant_mb)
          hipLaunchKernelGGL(k_inter_mbg<true>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, c,
                             blk_div(a->width, a->height), (unsigned)nm, me + m0);
        else
          hipLaunchKernelGGL(k_inter_mbg<false>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, c,
                             blk_div(a->width, a->height), (unsigned)nm, me + m0);
        HIP_TRY(hipGetLastError());
      }
      return P64GPU_OK;
    }
  }
  if (a->intra)
    hipLaunchKernelGGL(k_encode<0>, dim3(grid), dim3(64), 0, st, *a, mb_list, kd);
  else if (a->me_mode == P64GPU_ME_FULL)
    hipLaunchKernelGGL(k_encode<2>, dim3(grid), dim3(64), 0, st, *a, mb_list, kd);
  else
    hipLaunchKernelGGL(k_encode<1>, dim3(grid), dim3(64), 0, st, *a, mb_list, kd);
  HIP_TRY(hipGetLastError());
  return P64GPU_OK;
}

int p64gpu_decode_recon(int w, int h, int nframes, int64_t stride, const uint8_t *ref,
                        uint8_t *recon, const int16_t *coef, const p64_mb_rec *mb,
                        const uint8_t *quant_mb, const uint8_t *coded_mask, void *stream) {
  int s = check_geometry(w, h, nframes, stride);
  if (s) return s;
  if (!ref || !recon || !coef || !mb || !quant_mb || !coded_mask)
    return fail(P64GPU_E_INVALID, "NULL buffer");
  if (!aligned16(ref) || !aligned16(recon) || !aligned16(coef) || ((uintptr_t)mb & 3))
    return fail(P64GPU_E_INVALID, "ref/recon/coef must be 16-byte aligned, mb 4-byte aligned");
  const int nmb = (w / 16) * (h / 16);
  const unsigned grid = (unsigned)((int64_t)nframes * nmb);
  if (!mb_layout_forced()) {
    // pictures per launch: every buffer of a launch within the 2 GiB range
    // of the block kernels' 32-bit buffer offsets
    const int64_t per = (int64_t)nmb * 768 > stride ? (int64_t)nmb * 768 : stride;
    const int chunk = pictures_per_launch(per);
    for (int f0 = 0; f0 < nframes; f0 += chunk) {
      const int nf = nframes - f0 < chunk ? nframes - f0 : chunk;
      const int64_t blocks = (int64_t)nf * nmb * 6;
      const size_t m0 = (size_t)f0 * nmb;
      if (recon_persistent()) {
        unsigned wg;
        int s2 = persistent_grid((const void *)k_recon_blk, blocks, &wg);
        if (s2) return s2;
        hipLaunchKernelGGL(k_recon_blk, dim3(wg), dim3(256), 0, (hipStream_t)stream, w, h, stride,
                           ref + (size_t)f0 * stride, recon + (size_t)f0 * stride, coef + m0 * 384,
                           mb + m0, quant_mb + m0, coded_mask + m0, blk_div(w, h), (unsigned)blocks,
                           wg * 256u);
      } else {
        const unsigned nmbs = (unsigned)((int64_t)nf * nmb);
        const unsigned waves = (nmbs + MBS_PER_WAVE - 1) / MBS_PER_WAVE;
        hipLaunchKernelGGL(k_recon_mbg, dim3((waves + 3) / 4), dim3(256), 0, (hipStream_t)stream, w, h,
                           stride, ref + (size_t)f0 * stride, recon + (size_t)f0 * stride, coef + m0 * 384,
                           mb + m0, quant_mb + m0, coded_mask + m0, blk_div(w, h), nmbs);
      }
      HIP_TRY(hipGetLastError());
    }
    return P64GPU_OK;
  }
  hipLaunchKernelGGL(k_decode_recon, dim3(grid), dim3(64), 0, (hipStream_t)stream, w, h, stride,
                       ref, recon, coef, mb, quant_mb, coded_mask, mb_div(w, h));
  HIP_TRY(hipGetLastError());
  return P64GPU_OK;
}

int p64gpu_synth_frames(int w, int h, uint32_t seed0, int nseeds, int frame0, int nslots,
                        int64_t stride, uint8_t *out, void *stream) {
  int s = check_geometry(w, h, 1, stride);
  if (s) return s;
  if (!out || nseeds < 1 || nslots < 1 || frame0 < 0 || (int64_t)nseeds * nslots > 65535)
    return fail(P64GPU_E_INVALID, "synth: out=%p nseeds=%d nslots=%d frame0=%d", (void *)out,
                nseeds, nslots, frame0);
  hipLaunchKernelGGL(k_synth, dim3(64, (unsigned)(nseeds * nslots)), dim3(256), 0,
                     (hipStream_t)stream, w, h, seed0, nseeds, frame0, stride, out);
  HIP_TRY(hipGetLastError());
  return P64GPU_OK;
}

// ---- host-buffer encoder context ------------------------------------------

struct p64gpu_encoder {
  int device, w, h, nmb, me_mode, sl;
  size_t pic;
  uint8_t *d_cur, *d_rec[2], *d_li;
  int8_t *d_ov;
  int16_t *d_coef;
  p64_mb_rec *d_mb;
  p64_me_rec *d_me;
  int cur_ref;  // index of the buffer holding the previous reconstruction
  hipStream_t stream;
};

static void enc_free(p64gpu_encoder *e) {
  if (!e) return;
  (void)hipFree(e->d_cur);
  (void)hipFree(e->d_rec[0]);
  (void)hipFree(e->d_rec[1]);
  (void)hipFree(e->d_li);
  (void)hipFree(e->d_ov);
  (void)hipFree(e->d_coef);
  (void)hipFree(e->d_mb);
  (void)hipFree(e->d_me);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  free(e);
}

int p64gpu_encoder_open(int device, int w, int h, int me_mode, int sl, p64gpu_encoder **out) {
  if (!out) return fail(P64GPU_E_INVALID, "out is NULL");
  *out = nullptr;
  int s = check_geometry(w, h, 1, (int64_t)w * h * 3 / 2);
  if (s) return s;
  if (me_mode != P64GPU_ME_TSS && me_mode != P64GPU_ME_FULL)
    return fail(P64GPU_E_INVALID, "me mode %d", me_mode);
  if (sl < 1 || sl > 31) return fail(P64GPU_E_INVALID, "search_limit %d", sl);
  s = p64gpu_set_device(device);
  if (s) return s;
  p64gpu_encoder *e = (p64gpu_encoder *)calloc(1, sizeof *e);
  if (!e) return fail(P64GPU_E_NOMEM, "host allocation");
  e->device = device;
  e->w = w;
  e->h = h;
  e->nmb = (w / 16) * (h / 16);
  e->me_mode = me_mode;
  e->sl = sl;
  e->pic = (size_t)w * h * 3 / 2;
  bool ok = hipMalloc(&e->d_cur, e->pic) == hipSuccess &&
            hipMalloc(&e->d_rec[0], e->pic) == hipSuccess &&
            hipMalloc(&e->d_rec[1], e->pic) == hipSuccess &&
            hipMalloc(&e->d_li, e->nmb) == hipSuccess &&
            hipMalloc(&e->d_ov, e->nmb) == hipSuccess &&
            hipMalloc(&e->d_coef, (size_t)e->nmb * 384 * sizeof(int16_t)) == hipSuccess &&
            hipMalloc(&e->d_mb, (size_t)e->nmb * sizeof(p64_mb_rec)) == hipSuccess &&
            hipMalloc(&e->d_me, (size_t)e->nmb * sizeof(p64_me_rec)) == hipSuccess &&
            hipStreamCreate(&e->stream) == hipSuccess;
  if (!ok) {
    enc_free(e);
    return fail(P64GPU_E_NOMEM, "device allocation for %dx%d encoder", w, h);
  }
  (void)hipMemset(e->d_rec[0], 0, e->pic);  // InitFS/ClearFS (p64.c:533-536)
  (void)hipMemset(e->d_rec[1], 0, e->pic);
  (void)hipMemset(e->d_li, 0, e->nmb);
  *out = e;
  return P64GPU_OK;
}

int p64gpu_encoder_frame(p64gpu_encoder *e, const uint8_t *picture, int intra, int quant,
                         const int8_t *mtype_override, int16_t *coef, p64_mb_rec *mb,
                         p64_me_rec *me, uint8_t *recon) {
  if (!e || !picture || !coef || !mb) return fail(P64GPU_E_INVALID, "NULL argument");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipMemcpyAsync(e->d_cur, picture, e->pic, hipMemcpyHostToDevice, e->stream));
  if (intra) HIP_TRY(hipMemsetAsync(e->d_li, 0, e->nmb, e->stream));
  if (mtype_override)
    HIP_TRY(hipMemcpyAsync(e->d_ov, mtype_override, e->nmb, hipMemcpyHostToDevice, e->stream));
  p64gpu_encode_args a;
  memset(&a, 0, sizeof a);
  a.width = e->w;
  a.height = e->h;
  a.nframes = 1;
  a.intra = intra ? 1 : 0;
  a.quant = quant;
  a.me_mode = e->me_mode;
  a.search_limit = e->sl;
  a.frame_stride = (int64_t)e->pic;
  a.cur = e->d_cur;
  a.ref = e->d_rec[e->cur_ref];
  a.recon = e->d_rec[e->cur_ref ^ 1];
  a.last_intra = e->d_li;
  a.mtype_override = mtype_override ? e->d_ov : nullptr;
  a.coef = e->d_coef;
  a.mb = e->d_mb;
  a.me = e->d_me;
  int s = p64gpu_encode_frames(&a, e->stream);
  if (s) return s;
  HIP_TRY(hipMemcpyAsync(coef, e->d_coef, (size_t)e->nmb * 384 * sizeof(int16_t),
                         hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(mb, e->d_mb, (size_t)e->nmb * sizeof(p64_mb_rec), hipMemcpyDeviceToHost,
                         e->stream));
  if (me && !intra)
    HIP_TRY(hipMemcpyAsync(me, e->d_me, (size_t)e->nmb * sizeof(p64_me_rec),
                           hipMemcpyDeviceToHost, e->stream));
  if (recon)
    HIP_TRY(hipMemcpyAsync(recon, a.recon, e->pic, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->cur_ref ^= 1;  // SwapFS(CFS, OFS), p64.c:661
  return P64GPU_OK;
}

void p64gpu_encoder_close(p64gpu_encoder *e) { enc_free(e); }

#ifdef P64_TIMING
int p64gpu_dbg_phase_buffer(uint32_t *dev_buf) {  // [grid][32] uint32, zeroed by the caller
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_buf), &dev_buf, sizeof dev_buf));
  return 0;
}
#endif
#ifdef P64_ME_STATS
int p64gpu_dbg_stats(unsigned long long *out, int reset) {  // out[48]
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_me_stats), sizeof(g_me_stats)));
  if (reset) {
    static const unsigned long long z[48] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_me_stats), z, sizeof(z)));
  }
  return 0;
}
#endif

}  // extern "C"
