// k_search.hip -- the macroblock-layout kernels: one 64-lane wavefront per
// macroblock (MotionEstimation me.c:340 and the fused per-MB encode).
//
//   * the 16x16 current luma block and a 46x48-byte window of the previous
//     reconstruction around it are staged in LDS with 16-byte loads;
//   * FULL search (FastBME me.c:187): lane = (dx, dy group), 15 candidates per
//     lane (4 for search limits up to 15); a lower bound on every candidate's SAD from 4x4 sub-block averages
//     (v_lerp_u8 map, four v_sad_u8 per candidate) prunes all but a handful,
//     which get full SADs; low-contrast blocks, where nothing prunes, take the
//     dense exhaustive pass.  The argmin is one wave-wide min over packed
//     (SAD, scan-order) keys, reproducing FastBME's first-minimum rule;
//   * TSS (StepBME me.c:255): lane = (candidate, row pair), four dependent
//     steps of 8 candidates;
//   * k_encode (per-MB lists of rate control and -o): "row" layout lane =
//     (block, row) for the prediction, the loop filter (vertical taps by DPP)
//     and the Chen passes; "element" layout lane = coefficient for
//     quantisation, zigzag, CBP (wave ballots) and dequantisation.
// k_motion alone is the first half of an inter picture; k_block.hip's
// k_inter_mbg does the rest from its records.

#include "common.h"
#include "launch.h"

namespace {

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

// The search reads its macroblock's window, current block and lower-bound map
// through these views (Sx) and a geometry G -- dwords per window row, bytes
// per map plane row and plane -- rather than one fixed LDS struct, so that
// images with wider windows (several macroblocks sharing one window and map:
// measured as a 4-MB tile per workgroup) reuse the same code.
constexpr int MAP_ROWS = 42;
template <int WS_, int MAP_ROW_>
struct Geo {
  static constexpr int WS = WS_, MAP_ROW = MAP_ROW_, MAP_PLANE = MAP_ROWS * MAP_ROW_;
};
using Geo1 = Geo<WIN_WORDS, 12>;  // MbLds: one macroblock per wave
struct Sx {
  const uint32_t *win;  // the MB's 46 x 48-byte window: row r at win + r * G::WS
  uint32_t *cur;        // current 16x16 luma, 64 dwords
  uint32_t *cpred;      // 16 bytes of scratch
  uint32_t *list;       // survivor list (SURV_LIST_MAX)
  uint32_t *map;        // the MB's origin in the lower-bound map
};
__device__ __forceinline__ Sx sx_of(MbLds &L) { return Sx{L.win, L.cur, L.cpred, L.list, L.map}; }

// Wave-level LDS ordering: every search step below syncs within its wave only
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The search window and the current luma block, fetched into registers
// (LumaFetch) one macroblock ahead of its use, then stored to LDS (put_luma).
// Buffer loads over the luma plane, no bounds test: segments above or below
// the picture read zeros (offset out of range), segments left or right of it
// the neighbouring rows' pixels -- neither is part of any valid candidate
// (me.c:212/292) or of the prediction of a valid vector.
constexpr int WIN_SEGS = WIN_ROWS * 3, WIN_NIT = (WIN_SEGS + 63) / 64;  // 16-byte segments
struct LumaFetch {
  uint4 v[WIN_NIT];
  uint32_t c;
};
// window rows [R0, R0 + NR) (the SL <= 15 search reads rows 8..38 only)
template <int R0 = 0, int NR = WIN_ROWS>
__device__ __forceinline__ LumaFetch fetch_luma(const uint8_t *ref_y, const uint8_t *cur_y, int w,
                                                int h, int x0, int y0, int lane) {
  constexpr int SEGS = NR * 3, NIT = (SEGS + 63) / 64;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)ref_y, (short)0, w * h, BUF_RSRC_W3);
  const int base = (y0 - WIN_OY + R0) * w + x0 - WIN_OX;  // (negative above the picture: out of range)
  LumaFetch f;
  // the current block first: k_motion builds its sub-block map while the
  // window is still in flight (wait counts are in issue order)
  f.c = *reinterpret_cast<const uint32_t *>(cur_y + (uint32_t)(mul24(y0 + (lane >> 2), w) + x0 + 4 * (lane & 3)));
#pragma unroll
  for (int i = 0; i < NIT; i++) {
    const int t = lane + 64 * i, row = t / 3, seg = t - row * 3;
    const uint32_t off = (64 * i + 63 < SEGS || t < SEGS) ? (uint32_t)(base + mul24(row, w) + 16 * seg) : BUF_OOB;
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
    f.v[i] = make_uint4(v[0], v[1], v[2], v[3]);
  }
  return f;
}
template <int R0 = 0, int NR = WIN_ROWS>
__device__ __forceinline__ void put_win(MbLds &L, const LumaFetch &f, int lane) {
  constexpr int SEGS = NR * 3, NIT = (SEGS + 63) / 64;
#pragma unroll
  for (int i = 0; i < NIT; i++) {
    const int t = lane + 64 * i;
    if (64 * i + 63 < SEGS || t < SEGS) reinterpret_cast<uint4 *>(L.win)[3 * R0 + t] = f.v[i];
  }
}
template <int R0 = 0, int NR = WIN_ROWS>
__device__ __forceinline__ void put_luma(MbLds &L, const LumaFetch &f, int lane) {
  put_win<R0, NR>(L, f, lane);
  L.cur[lane] = f.c;
}
// the rows the SL <= 15 search reads: its candidates' rows 8..36 (dy in
// [-7, 7)), the dense pass's up to 38
constexpr int WIN15_R0 = 8, WIN15_NR = 31;

// SAD of the zero vector (OMV, me.c:203/271): one dword per lane
template <class G>
__device__ __forceinline__ int sad_zero(const Sx &S, int lane) {
  const uint32_t r = S.win[(WIN_OY + (lane >> 2)) * G::WS + WIN_OX / 4 + (lane & 3)];
  return wave_sum((int)sad4(r, S.cur[lane], 0));
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
// Lane layout (MeLayout below): lane = (dy group q, dx index), ND candidates
// dy = D0 + ND*q + d, d = 0..ND-1, of the column dx = dxi + D0 (SL 31: two
// groups of 15, dx from -15; SL <= 15: four groups of 4, dx from -7).  Keys are
// SUM << 10 | ord, ord = 1 + (dx+15)*32 + (dy+15): FastBME's dx-major scan order
// (ord 0 is reserved for the zero vector).
constexpr int ME_LIST_MAX = 256;
#ifndef ME_GROUPS_MAX
#define ME_GROUPS_MAX 16  // survivors finished by 4-lane groups; more: finish_halves
#endif
static_assert(ME_LIST_MAX <= SURV_LIST_MAX, "survivor list size");
constexpr uint32_t ME_INVALID = 1u << 19;
constexpr int ME_LOW_CONTRAST = 12;
constexpr int ME_NOISE_SAD0 = 24 * 256;  // mean |difference| 24 at (0,0)
constexpr int KEY_SHIFT = 10;
constexpr unsigned KEY_ORD = (1u << KEY_SHIFT) - 1;
// lower-bound map: 4 phase planes (x mod 4) x MAP_ROWS rows x MAP_ROW_BYTES
// bytes; plane p, row y, byte k holds m(4k + p, y) in window coordinates
constexpr int MAP_ROW_BYTES = Geo1::MAP_ROW, MAP_PLANE_BYTES = Geo1::MAP_PLANE;
static_assert(4 * MAP_PLANE_BYTES == 4 * LB_MAP_WORDS, "map size");

// rows [R0, R1) of the current block against window rows [I0, I1) of the
// lane, candidate d = i - r of ND
template <class G, int ND, int R0, int R1, int I0, int I1>
__device__ __forceinline__ void full_rows(const lds_u32 *wrow, int sh, const uint32_t *cs,
                                          uint32_t *acc) {
#pragma unroll
  for (int i = I0; i < I1; i++) {
    const lds_u32 *p = wrow + i * G::WS;
    const uint32_t a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3], a4 = p[4];
    const uint32_t r0 = align4(a1, a0, sh), r1 = align4(a2, a1, sh);
    const uint32_t r2 = align4(a3, a2, sh), r3 = align4(a4, a3, sh);
#pragma unroll
    for (int r = R0; r < R1; r++) {
      const int d = i - r;
      if (d >= 0 && d < ND) {
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
// RB, RPC: first map row and rows per chunk (5 chunks): rows RB .. RB+5*RPC-1
// (the SL 31 layout reads rows 0..41, the SL <= 15 one rows 8..35)
template <int RB = 0, int RPC = 9>
__device__ __forceinline__ void build_lb_map(const Sx &S, int lane) {
  const int c = lane / 12, n = lane - 12 * c;
  const bool act = lane < 60;
  const int y0 = RB + RPC * min(c, 4);
  uint32_t v1[RPC + 2];
#pragma unroll
  for (int t = 0; t < RPC + 2; t++) {
    const int ya = min(y0 + t, WIN_ROWS - 1), yb = min(y0 + t + 1, WIN_ROWS - 1);
    v1[t] = lerp4(S.win[ya * WIN_WORDS + n], S.win[yb * WIN_WORDS + n]);
  }
  // the byte scatter to the planes in 16-bit pieces: lanes n and n ^ 1 swap
  // their dwords (one DPP move), the even lane then holds planes 0 and 1 of
  // map bytes n, n + 1, the odd lane planes 2 and 3 (one v_perm with a
  // per-lane selector), written by two ds_write_b16 (lo / d16_hi) instead of
  // four ds_write_b8: the map build is the largest LDS user of the search
  const bool odd = n & 1;
  const uint32_t psel = odd ? 0x03070206u : 0x05010400u;  // [x.b2 h.b2 x.b3 h.b3] : [h.b0 x.b0 h.b1 x.b1]
  uint8_t *mp = reinterpret_cast<uint8_t *>(S.map) + (n & ~1) + (odd ? 2 * MAP_PLANE_BYTES : 0);
#pragma unroll
  for (int t = 0; t < RPC; t++) {
    const uint32_t v = lerp4(v1[t], v1[t + 2]);  // rows y..y+3
    const uint32_t h1 = lerp4(v, align4(from_next_lane_wave(v), v, 1));
    const uint32_t h2 = lerp4(h1, align4(from_next_lane_wave(h1), h1, 2));
    const uint32_t x = dpp<0xB1>(h2);  // the neighbour's (quad_perm [1,0,3,2])
    const uint32_t pr = __builtin_amdgcn_perm(x, h2, psel);
    const int y = y0 + t;
    if (act && y < MAP_ROWS) {
      uint16_t *q = reinterpret_cast<uint16_t *>(mp + y * MAP_ROW_BYTES);
      q[0] = (uint16_t)pr;
      q[MAP_PLANE_BYTES / 2] = (uint16_t)(pr >> 16);
    }
  }
}

// the current block's 16 sub-block averages (same nesting as the map), row j
// of sub-blocks as one wave-uniform dword cm[j] (byte i = sub-block (i, j),
// also left as bytes 0..15 of L.cpred); returns their range (max - min)
__device__ __forceinline__ int cur_lb_map(const Sx &S, int lane, uint32_t cm[4]) {
  if (lane < 16) {
    const int i = lane & 3, j = lane >> 2;
    const uint32_t *r = S.cur + 16 * j + i;
    const uint32_t v = lerp4(lerp4(r[0], r[4]), lerp4(r[8], r[12]));
    const uint32_t h1 = lerp4(v, v >> 8);
    const uint32_t h2 = lerp4(h1, h1 >> 16);
    reinterpret_cast<uint8_t *>(S.cpred)[lane] = (uint8_t)h2;
  }
  wsync();
#pragma unroll
  for (int j = 0; j < 4; j++) cm[j] = (uint32_t)uni((int)S.cpred[j]);
  // their range from the wave-uniform dwords: scalar byte extracts, min and
  // max (the scalar unit, not the VALU the search is bound by; asm, as the
  // compiler otherwise picks v_min3/v_max3 over SGPR operands)
  auto smin = [](unsigned a, unsigned b) {
    unsigned r;
    asm("s_min_u32 %0, %1, %2" : "=s"(r) : "s"(a), "s"(b));
    return r;
  };
  auto smax = [](unsigned a, unsigned b) {
    unsigned r;
    asm("s_max_u32 %0, %1, %2" : "=s"(r) : "s"(a), "s"(b));
    return r;
  };
  unsigned lo = cm[0] & 255u, hi = lo;
#pragma unroll
  for (int k = 1; k < 16; k++) {
    const unsigned b = (cm[k >> 2] >> (8 * (k & 3))) & 255u;
    lo = smin(lo, b);
    hi = smax(hi, b);
  }
  return (int)(hi - lo);
}

// SAD(0,0) (OMV, me.c:203/271) and, in the same wave reduction, the current
// block's high-frequency energy E = sum |pixel - its 4x4 sub-block average|
// (both < 2^16: one 32-bit sum carries the two)
template <class G>
__device__ __forceinline__ void sad_zero_hf(const Sx &S, int lane, int &sad0, int &ehf) {
  const uint32_t r = S.win[(WIN_OY + (lane >> 2)) * G::WS + WIN_OX / 4 + (lane & 3)];
  const uint32_t c = S.cur[lane];
  const uint32_t m = reinterpret_cast<const uint8_t *>(S.cpred)[4 * (lane >> 4) + (lane & 3)];
  const uint32_t m4 = __builtin_amdgcn_perm(0u, m, 0x00000000u);  // m in every byte (not the quarter-rate v_mul_lo)
  const int t = wave_sum((int)(sad4(r, c, 0u) | (sad4(c, m4, 0u) << 16)));
  sad0 = t & 0xffff;
  ehf = (int)((unsigned)t >> 16);
}

// every byte of the window equal: then every valid candidate block equals the
// zero-vector block, all SADs equal SAD(0,0) and (0,0) wins (it wins ties)
template <class G, int R0 = 0, int NR = WIN_ROWS>  // window rows [R0, R0 + NR)
__device__ __forceinline__ bool window_constant(const Sx &S, int lane) {
  const uint32_t v = (S.win[R0 * G::WS] & 255u) * 0x01010101u;
  bool diff = false;
#pragma unroll
  for (int k = 0; k < (NR * WIN_WORDS + 63) / 64; k++) {
    const int t = lane + 64 * k, row = t / WIN_WORDS;
    if (t < NR * WIN_WORDS) diff |= S.win[(R0 + row) * G::WS + t - row * WIN_WORDS] != v;
  }
  return !__any(diff);
}

// an LDS pointer whose whole address is one opaque register: constant row
// offsets from it then fit the 8-bit dword offsets of ds_read2 (the compiler
// otherwise keeps the struct offset as an immediate and adds per row pair)
__device__ __forceinline__ const lds_u32 *lds_base(const uint32_t *p) {
  uint32_t a = (uint32_t)(uintptr_t)as_lds(const_cast<uint32_t *>(p));
  asm volatile("" : "+v"(a));
  return (const lds_u32 *)(uintptr_t)a;
}

__device__ __forceinline__ void ord_pos(unsigned ord, int &cdx, int &cdy) {  // ord >= 1
  cdx = (int)((ord - 1) >> 5) - 15;
  cdy = (int)((ord - 1) & 31) - 15;
}

// full SADs of the n <= 32 listed candidates (ords in S.list), 4*RG lanes per
// candidate: lane (slot, rg, d) sums dword d of rows rg, rg+RG, ...; returns the
// least key
template <class G, int RG>
__device__ __forceinline__ unsigned finish_groups(const Sx &S, int n, int lane) {
  constexpr int GL = 4 * RG, PER = 64 / GL, NR = 16 / RG;  // lanes per candidate
  const int d = lane & 3, rg = (lane >> 2) & (RG - 1), slot = lane / GL;
  uint32_t cw[NR];
#pragma unroll
  for (int t = 0; t < NR; t++) cw[t] = S.cur[4 * (rg + RG * t) + d];
  unsigned bk = 0xFFFFFFFFu;
  for (int c0 = 0; c0 < n; c0 += PER) {
    const int j = c0 + slot;
    const unsigned ord = j < n ? S.list[j] & KEY_ORD : 1u;
    int cdx, cdy;
    ord_pos(ord, cdx, cdy);
    const int cb = WIN_OX + cdx, csh = cb & 3;
    const lds_u32 *p0 = lds_base(S.win + (WIN_OY + cdy + rg) * G::WS + (cb >> 2) + d);
    uint32_t a = 0;
#pragma unroll
    for (int t = 0; t < NR; t++) {
      const lds_u32 *p = p0 + RG * t * G::WS;
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

// Two-stage finishing of many survivors (more than 8; SURVEY.md 8(d)'s
// content leaves ~46 at the median, smooth texture under N(0,4) noise): the
// first stage computes, one candidate per lane, the exact SAD of rows 0..7
// only (the current rows 0..7 wave-uniform in SGPRs, no LDS broadcast) and
// adds the lower bound of rows 8..15 from the sub-block averages, 16 Sbot -
// 256 (Sbot: the candidate's terms of sub-block rows 2 and 3, carried in its
// list entry's high half); a candidate whose
//     LB2 = SAD(rows 0..7) + 16 Sbot - 256 > T
// can neither win nor tie (LB2 <= SAD, per sub-block as in me_full's bound).
// The few left (c* excluded: its key is known) are compacted in place with
// their half SAD and finished over rows 8..15 by lane groups.  Half the
// window reads and SADs of one-per-lane finishing; the result is unchanged.
// tools/me_sim.py-style model on the survey content: 46 -> 1 at the median.
template <class G, int RG>
__device__ __forceinline__ unsigned finish_bottom(const Sx &S, int n, int lane) {
  constexpr int GL = 4 * RG, PER = 64 / GL, NR = 8 / RG;  // lanes per candidate, rows per lane
  const int d = lane & 3, rg = (lane >> 2) & (RG - 1), slot = lane / GL;
  uint32_t cw[NR];
#pragma unroll
  for (int t = 0; t < NR; t++) cw[t] = S.cur[4 * (8 + rg + RG * t) + d];
  unsigned bk = 0xFFFFFFFFu;
  for (int c0 = 0; c0 < n; c0 += PER) {
    const int j = c0 + slot;
    const unsigned e = j < n ? S.list[j] : 1u;
    const unsigned ord = e & KEY_ORD;
    int cdx, cdy;
    ord_pos(ord, cdx, cdy);
    const int cb = WIN_OX + cdx, csh = cb & 3;
    const lds_u32 *p0 = lds_base(S.win + (WIN_OY + cdy + 8 + rg) * G::WS + (cb >> 2) + d);
    uint32_t a = 0;
#pragma unroll
    for (int t = 0; t < NR; t++) {
      const lds_u32 *p = p0 + RG * t * G::WS;
      a = sad4(align4(p[1], p[0], csh), cw[t], a);
    }
    a += dpp<0xB1>(a);
    a += dpp<0x4E>(a);
    if (RG >= 2) a += dpp<0x141>(a);
    if (RG >= 4) a += dpp<0x140>(a);
    a += e >> KEY_SHIFT;  // + the SAD of rows 0..7
    if (j < n) bk = min(bk, (a << KEY_SHIFT) | ord);
  }
  return wave_min(bk);
}
template <class G>
__device__ __forceinline__ unsigned finish_halves(const Sx &S, const uint8_t *cur_blk, int w, int n, unsigned T,
                                                  unsigned cstar_ord, int lane) {
  lds_u32 *list = as_lds(S.list);
  uint32_t cs[64];
  load_cur_rows8<0>(cur_blk, w, cs);  // rows 0..7 as wave-uniform dwords (SGPRs)
  int n2 = 0;
  for (int c0 = 0; c0 < n; c0 += 64) {  // uniform
    const bool act = c0 + lane < n;
    const unsigned e = act ? (unsigned)list[c0 + lane] : 1u;
    const unsigned ord = e & KEY_ORD;
    int cdx, cdy;
    ord_pos(ord, cdx, cdy);
    const int cb = WIN_OX + cdx, csh = cb & 3;
    const lds_u32 *p0 = lds_base(S.win + (WIN_OY + cdy) * G::WS + (cb >> 2));
    uint32_t a = 0;
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const lds_u32 *p = p0 + r * G::WS;
      const uint32_t a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3], a4 = p[4];
      a = sad4(align4(a1, a0, csh), cs[4 * r + 0], a);
      a = sad4(align4(a2, a1, csh), cs[4 * r + 1], a);
      a = sad4(align4(a3, a2, csh), cs[4 * r + 2], a);
      a = sad4(align4(a4, a3, csh), cs[4 * r + 3], a);
    }
    const int lb2 = (int)a + 16 * (int)(e >> 16) - 256;  // (Sbot in the entry's high half)
    const bool sv = act && ord != cstar_ord && lb2 <= (int)T;
    const uint64_t bl = __ballot(sv);
    // compacted in place: every entry of this chunk was read above, and the
    // write index never reaches the next chunk
    const int idx = n2 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
    if (sv) list[idx] = ord | (a << KEY_SHIFT);
    n2 += __popcll(bl);
  }
  n2 = uni(n2);
  if (n2 == 0) return 0xFFFFFFFFu;
  wsync();
  if (n2 <= 4) return finish_bottom<G, 4>(S, n2, lane);
  if (n2 <= 8) return finish_bottom<G, 2>(S, n2, lane);
  return finish_bottom<G, 1>(S, n2, lane);
}

// Candidate layouts of the FULL search: lane = (dy group q, dx lane dxi),
// ND vertically consecutive candidates per lane.  Search limits up to 15
// (the reference's default, me.c:62) span dx, dy in [-7, 7): 14 dx lanes x
// 4 groups x 4 dy; up to 31 span [-15, 15): 30 dx lanes x 2 groups x 15 dy.
template <int DXL_, int NDX_, int ND_, int D0_>
struct MeLayout {
  static constexpr int DXL = DXL_, NDX = NDX_, ND = ND_, D0 = D0_;  // D0: dx of dxi 0, dy of (q 0, d 0)
  static_assert(64 % DXL == 0 && NDX <= DXL && ND <= 15, "layout");
};
using MeLay31 = MeLayout<32, 30, 15, -15>;
using MeLay15 = MeLayout<16, 14, 4, -7>;

// A lane's candidates and their validity: the search's set-up, which needs
// only the MB's position (k_motion computes it before its window arrives).
struct MeSetup {
  int dx, colb, dy0;
  bool lane_ok, col_ok, interior;
  uint32_t inv;
  unsigned base;
};
template <class LY>
__device__ __forceinline__ MeSetup me_setup(int w, int h, int x0, int y0, int sl, int lane) {
  constexpr int ND = LY::ND;
  MeSetup u;
  const int q = lane / LY::DXL, dxi = lane % LY::DXL;
  u.lane_ok = dxi < LY::NDX;
  u.dx = (u.lane_ok ? dxi : LY::NDX - 1) + LY::D0;  // (idle lanes repeat the last column)
  u.colb = u.dx + WIN_OX;                           // window byte column of dx
  u.dy0 = LY::D0 + ND * q;                          // dy of the lane's d = 0
  // Validity (me.c:206-212: range and `< W-16`) is folded into the sums: an
  // invalid candidate starts at ME_INVALID, so it never survives and never wins.
  const int hl = sl >> 1;
  // interior: every lane's every candidate valid -- from the MB's position and
  // the limit alone (scalar: the extreme columns and the extreme dy of the
  // first and last groups decide it)
  constexpr int NQ = 64 / LY::DXL;  // dy groups
  u.interior = -hl <= LY::D0 && LY::D0 + LY::NDX - 1 < hl && x0 + LY::D0 >= 0 && x0 + LY::D0 + LY::NDX - 1 < w - 16 &&
               max(-hl, -y0) <= LY::D0 && min(hl, h - 16 - y0) >= LY::D0 + ND * NQ;
  // the sums start at 0; invalid candidates are marked afterwards (bit 19 of a
  // sum < 2^17): interior macroblocks only mask the two idle lanes, the others
  // OR in the lane's invalid rows, ~valid [dlo, dhi) (or every row)
  u.inv = 0;
  u.col_ok = u.lane_ok;
  if (!u.interior) {
    const int px = x0 + u.dx;
    u.col_ok = u.lane_ok && u.dx >= -hl && u.dx < hl && px >= 0 && px < w - 16;
    // valid dy: [max(-hl, -y0), min(hl, h-16-y0)), i.e. d in [dlo, dhi) for this group
    const int dlo = max(-hl, -y0) - u.dy0, dhi = min(hl, h - 16 - y0) - u.dy0;
    const int lo = min(max(dlo, 0), ND), hi = min(max(dhi, 0), ND);
    u.inv = ~((u.col_ok && hi > lo) ? (1u << hi) - (1u << lo) : 0u);
  }
  u.base = ((unsigned)(u.dx + 15) << 5) + (unsigned)(u.dy0 + 15) + 1u;  // ord of d = 0
  return u;
}
// the current block's sub-block averages and their range (cur_lb_map) and the
// search's set-up, when the caller made them before the window arrived
// (k_motion)
struct CurMap {
  uint32_t cm[4];
  int range;
  MeSetup su;
};
template <class G, class LY, bool PRE = false>
__device__ __forceinline__ void me_full(const Sx &S, const uint8_t *cur_blk, int w, int h, int x0,
                                        int y0, int sl, int lane, int &sad0_out, int &mx, int &my,
                                        int &best, const CurMap &pre = CurMap{}) {
  constexpr int ND = LY::ND;
  const MeSetup su = PRE ? pre.su : me_setup<LY>(w, h, x0, y0, sl, lane);
  const int colb = su.colb, dy0 = su.dy0;
  const bool lane_ok = su.lane_ok, interior = su.interior;
  const uint32_t inv = su.inv;
  auto mark_invalid = [&](uint32_t *a) {
    if (!interior) {
#pragma unroll
      for (int d = 0; d < ND; d++) a[d] |= ((inv >> d) & 1u) << 19;
    }
  };
  static_assert(ME_INVALID == 1u << 19, "invalid mark");
  const unsigned base = su.base;

  SECTION("cur_map");
  uint32_t cm[4];
  int range;
  if (PRE) {
#pragma unroll
    for (int j = 0; j < 4; j++) cm[j] = pre.cm[j];
    range = pre.range;
  } else {
    range = uni(cur_lb_map(S, lane, cm));
  }
  int sad0, ehf;
  sad_zero_hf<G>(S, lane, sad0, ehf);
  sad0 = uni(sad0);
  sad0_out = sad0;
  unsigned bk = 0xFFFFFFFFu, ckey = 0xFFFFFFFFu, Ts = 0, pk = 0, T = 0;
  uint32_t acc[ND], accb[ND], sb[ND];  // bound sums of sub-block rows 0-1 and 2-3 (Sbot), and S
  lds_u32 *list = as_lds(S.list);  // (one-MB image: aliases the map once the map is dead)
  int nsurv = 1000;
  // Low-contrast blocks (sub-block averages within a few levels) prune almost
  // nothing: they go to the dense search straight away (speed only, the result
  // is the same; tools/me_paths.py measured 98% dense below 12, none above 15).
  // So do noise-like blocks: a large SAD(0,0) at least half of which the
  // current block's own high-frequency energy E (what the 4x4 averages
  // cannot see) could account for: the bound then prunes nothing anywhere
  // (tools/noise_rule.py: every uniform-noise block, no synthetic or 15-px
  // pan one)
  bool lb_path = range >= ME_LOW_CONTRAST;
  if (sad0 > ME_NOISE_SAD0 && 2 * uni(ehf) > sad0) lb_path = false;
  if (lb_path) {
    // 1. lower bounds S
    SECTION("lb_map");
    if (ND < 15)
      build_lb_map<8, 6>(S, lane);
    else
      build_lb_map(S, lane);
    wsync();
    SECTION("lb_pass");
#pragma unroll
    for (int d = 0; d < ND; d++) acc[d] = accb[d] = 0;
    {
      const int xq = colb >> 2;
      const uint32_t *mrow = S.map + ((colb & 3) * G::MAP_PLANE + (dy0 + WIN_OY) * G::MAP_ROW) / 4 + (xq >> 2);
      const int msh = xq & 3;
#pragma unroll
      for (int i = 0; i < ND + 12; i++) {
        const uint32_t *mq = mrow + i * (G::MAP_ROW / 4);
        const uint32_t m4 = align4(mq[1], mq[0], msh);
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int d = i - 4 * j;
          // sub-block rows 0, 1 into acc, rows 2, 3 (Sbot, finish_halves) into accb
          if (d >= 0 && d < ND) {
            if (j < 2)
              acc[d] = sad4(m4, cm[j], acc[d]);
            else
              accb[d] = sad4(m4, cm[j], accb[d]);
          }
        }
      }
    }
#pragma unroll
    for (int d = 0; d < ND; d++) {  // S
      sb[d] = acc[d] + accb[d];
    }
    mark_invalid(sb);

    // 2. c* and its full SAD
    SECTION("cstar");
    {  // least (S, d) of the lane as S << 4 | d, then its key S << 10 | ord
      unsigned m = 0xFFFFFFFFu;
#pragma unroll
      for (int d = 0; d < ND; d++) m = min(m, (sb[d] << 4) | (unsigned)d);
      if (!lane_ok) m = ME_INVALID << 4;
      pk = m == 0xFFFFFFFFu ? m : ((m >> 4) << KEY_SHIFT) + base + (m & 15u);
    }
    pk = uni((int)wave_min(pk));
    if ((pk >> KEY_SHIFT) < ME_INVALID) {  // else nothing is valid
      int cdx, cdy;
      ord_pos(pk & KEY_ORD, cdx, cdy);
      const int cb = WIN_OX + cdx + 4 * (lane & 3);
      const uint32_t *p = S.win + (WIN_OY + cdy + (lane >> 2)) * G::WS + (cb >> 2);
      const uint32_t s = sad4(align4(p[1], p[0], cb & 3), S.cur[lane], 0u);
      ckey = (pk & KEY_ORD) | ((unsigned)uni(wave_sum((int)s)) << KEY_SHIFT);
    }
    T = min(ckey >> KEY_SHIFT, (unsigned)sad0);
    Ts = (T + 512u) >> 4;  // survivors: S <= Ts

    SECTION("survivors");
    // 3. survivors: their ords compacted into L.list with ballot + mbcnt (the
    // first ME_LIST_MAX of them), counted on the way
    nsurv = 0;
    if (lane_ok) {  // (the idle lanes sit out: their sums are not masked)
#pragma unroll
    for (int d = 0; d < ND; d++) {
      const bool sv = sb[d] <= Ts;
      const uint64_t bl = __ballot(sv);
      if (bl) {
        const int idx = nsurv + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
        // the entry: ord | Sbot << 16 (finish_halves; acc's high half is
        // Sbot).  Past ME_LIST_MAX entries the dense pass takes over and the
        // list is not read: the index is clamped rather than tested -- only
        // once the list may reach its end (a scalar test: the clamp's VALU
        // is one of ~8 per candidate row here)
        const uint32_t e = (accb[d] << 16) | (base + d);
        if (nsurv <= ME_LIST_MAX - 64) {
          if (sv) list[idx] = e;
        } else {
          if (sv) list[min(idx, ME_LIST_MAX - 1)] = e;
        }
        nsurv += __popcll(bl);
      }
    }
    }
    nsurv = uni(nsurv);
  }

  SECTION("finish");
  if (nsurv <= ME_LIST_MAX) {
    wsync();
    // nothing to finish when c* (whose key is known) is the only survivor
    if (nsurv == 0 || (nsurv == 1 && ((unsigned)uni((int)list[0]) & KEY_ORD) == (pk & KEY_ORD)))
      ;
    else if (nsurv <= 4)
      bk = finish_groups<G, 4>(S, nsurv, lane);
    else if (nsurv <= 8)
      bk = finish_groups<G, 2>(S, nsurv, lane);
    else if (nsurv <= ME_GROUPS_MAX)
      bk = finish_groups<G, 1>(S, nsurv, lane);
    else
      bk = finish_halves<G>(S, cur_blk, w, nsurv, T, pk & KEY_ORD, lane);
  } else if (range < 4 && uni(ND < 15 ? window_constant<G, WIN15_R0, WIN15_NR>(S, lane)
                                       : window_constant<G>(S, lane))) {
    bk = 0xFFFFFFFFu;  // constant window (checked for nearly flat blocks): (0,0), below
  } else {  // little pruned: every candidate densely, the current rows in SGPRs
    const lds_u32 *wrow = lds_base(S.win + (dy0 + WIN_OY) * G::WS + (colb >> 2));
    const int sh = colb & 3;
    uint32_t cs[64];
#pragma unroll
    for (int d = 0; d < ND; d++) acc[d] = 0;
    // (in two chunks of 8 rows: all 16 in SGPRs raise the kernel's SGPR
    // count past 80 and cost every macroblock a wave slot per SIMD)
    load_cur_rows8<0>(cur_blk, w, cs);
    full_rows<G, ND, 0, 8, 0, ND + 7>(wrow, sh, cs, acc);
    load_cur_rows8<8>(cur_blk, w, cs);
    full_rows<G, ND, 8, 16, 8, ND + 15>(wrow, sh, cs, acc);
    mark_invalid(acc);
#pragma unroll
    for (int d = 0; d < ND; d++) bk = min(bk, (acc[d] << KEY_SHIFT) + base + d);
    if (!lane_ok) bk = 0xFFFFFFFFu;
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
template <class G>
__device__ __forceinline__ void me_tss(const Sx &S, int w, int h, int x0, int y0, int lane,
                                       int sad0, int &mx, int &my, int &best) {
  const int k = lane >> 3, rg = lane & 7;
  const int kk = k < 4 ? k : k + 1;  // skip the centre of the 3x3
  const int dirx = kk % 3 - 1, diry = kk / 3 - 1;
  uint32_t c[8];
#pragma unroll
  for (int j = 0; j < 8; j++) c[j] = S.cur[8 * rg + j];  // rows 2rg, 2rg+1
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
      const uint32_t *p = S.win + (WIN_OY + dy + 2 * rg) * G::WS + (colb >> 2);
#pragma unroll
      for (int rr = 0; rr < 2; rr++) {
        const uint32_t *q = p + rr * G::WS;
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
template <class G>
__device__ __forceinline__ void me_stats(const Sx &S, int lane, MeOut &o) {
  const int colb = WIN_OX + o.mx + 4 * (lane & 3);
  const uint32_t *p = S.win + (WIN_OY + o.my + (lane >> 2)) * G::WS + (colb >> 2);
  const uint32_t rw = align4(p[1], p[0], colb & 3), cw = S.cur[lane];
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


// stats: the decision statistics too (me_stats); the split encoder's
// k_inter_mbg computes them itself from its prediction source (round 6), so
// its k_motion launch leaves them out (uniform)
template <class G, int MODE, bool PRE = false>  // MODE 1 = TSS, 2 = FULL
__device__ __forceinline__ MeOut motion_estimate(const Sx &S, const uint8_t *cur_y, int w, int h,
                                                 int x0, int y0, int sl, int lane, const CurMap &pre = CurMap{},
                                                 bool stats = true) {
  MeOut o;
  if (MODE == 2) {
    if (sl <= 15)  // (uniform: one search limit per launch)
      me_full<G, MeLay15, PRE>(S, cur_y + (size_t)y0 * w + x0, w, h, x0, y0, sl, lane, o.sad0, o.mx, o.my,
                               o.sad, pre);
    else
      me_full<G, MeLay31, PRE>(S, cur_y + (size_t)y0 * w + x0, w, h, x0, y0, sl, lane, o.sad0, o.mx, o.my,
                               o.sad, pre);
  } else {
    o.sad0 = uni(sad_zero<G>(S, lane));
    me_tss<G>(S, w, h, x0, y0, lane, o.sad0, o.mx, o.my, o.sad);
  }
  o.mx = uni(o.mx);
  o.my = uni(o.my);
  o.sad = uni(o.sad);
  o.var = o.varor = o.mwor = 0;
  if (stats) {
    me_stats<G>(S, lane, o);
    o.var = uni(o.var);
    o.varor = uni(o.varor);
    o.mwor = uni(o.mwor);
  }
  return o;
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
    const MeOut me = motion_estimate<Geo1, MODE>(sx_of(L), cur.y, w, h, x0, y0, a.search_limit, lane);
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
  if (a.nzmask) {  // block k has a nonzero level -> bit 5 - k
    uint32_t nzm = 0;
#pragma unroll
    for (int k = 0; k < 6; k++) nzm |= __ballot(lev[k] != 0) ? 1u << (5 - k) : 0u;
    if (lane == 0) a.nzmask[gmb] = (uint8_t)nzm;
  }
}

template <int MODE>
__global__ __launch_bounds__(64, 1) void k_encode(p64gpu_encode_args a, const int32_t *mb_list,
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
  const MbFetch f = fetch_mb<MODE>(a, a.cur, gid, kd, lane);
  if (MODE != 0) put_luma(L, f.luma, lane);
  SECTION("fetched");
  encode_mb<MODE>(a, a.cur, L, lane, gid, kd, f);
}

// ME only (MotionEstimation me.c:340-363 over a batch of luma planes).
// stats = 0 (the split encoder, whose k_inter_mbg computes VAR / VAROR /
// MWOR from the prediction source it loads anyway): those fields are not
// written here
template <int MODE>
__global__ __launch_bounds__(64, 1) void k_motion(int w, int h, int64_t stride, const uint8_t *ref_y,
                                               const uint8_t *cur_y, int sl, p64_me_rec *out,
                                               MbDiv kd, int stats) {
  __shared__ MbLds L;
  const int lane = threadIdx.x;
  const int mbw = w >> 4, nmb = mbw * (h >> 4);
  const unsigned gid = xcd_remap(blockIdx.x, gridDim.x);
  const MbPos ps = mb_pos(gid, nmb, mbw, kd);
  const int fi = ps.fi, x0 = 16 * ps.mbx, y0 = 16 * ps.mby;
  // FULL: the current block's sub-block map (cur_lb_map) while the window is
  // in flight, then the window
  CurMap cmap;
  auto cur_first = [&](const LumaFetch &f) {
    L.cur[lane] = f.c;
    if (MODE == 2) {
      wsync();
      cmap.range = uni(cur_lb_map(sx_of(L), lane, cmap.cm));
    }
  };
  if (MODE == 2 && sl <= 15) {  // (the SL <= 15 layout reads window rows 8..38 only)
    const LumaFetch f = fetch_luma<WIN15_R0, WIN15_NR>(ref_y + (size_t)fi * stride, cur_y + (size_t)fi * stride,
                                                       w, h, x0, y0, lane);
    cmap.su = me_setup<MeLay15>(w, h, x0, y0, sl, lane);
    cur_first(f);
    put_win<WIN15_R0, WIN15_NR>(L, f, lane);
  } else {
    const LumaFetch f = fetch_luma(ref_y + (size_t)fi * stride, cur_y + (size_t)fi * stride, w, h, x0, y0, lane);
    if (MODE == 2) cmap.su = me_setup<MeLay31>(w, h, x0, y0, sl, lane);
    cur_first(f);
    put_win(L, f, lane);
  }
  __syncthreads();
  SECTION("m_fetched");
  const MeOut me = motion_estimate<Geo1, MODE, MODE == 2>(sx_of(L), cur_y + (size_t)fi * stride, w, h, x0, y0,
                                                          sl, lane, cmap, stats != 0);
  SECTION("m_me_done");
  if (lane == 0) {
    if (stats) {
      p64_me_rec o;
      o.mx = me.mx;
      o.my = me.my;
      o.sad = me.sad;
      o.sad0 = me.sad0;
      o.var = me.var;
      o.varor = me.varor;
      o.mwor = me.mwor;
      out[gid] = o;
    } else {
      *reinterpret_cast<int4 *>(&out[gid].mx) = make_int4(me.mx, me.my, me.sad, me.sad0);
    }
  }
}


}  // namespace

namespace p64k {

hipError_t encode_fused(int mode, unsigned grid, const p64gpu_encode_args &a, const int32_t *mb_list,
                        hipStream_t st) {
  const MbDiv kd = mb_div(a.width, a.height);
  if (mode == 0)
    hipLaunchKernelGGL(k_encode<0>, dim3(grid), dim3(64), 0, st, a, mb_list, kd);
  else if (mode == 2)
    hipLaunchKernelGGL(k_encode<2>, dim3(grid), dim3(64), 0, st, a, mb_list, kd);
  else
    hipLaunchKernelGGL(k_encode<1>, dim3(grid), dim3(64), 0, st, a, mb_list, kd);
  return hipGetLastError();
}

hipError_t motion(int mode, int w, int h, int nframes, int64_t stride, const uint8_t *ref_y,
                  const uint8_t *cur_y, int sl, p64_me_rec *out, bool stats, hipStream_t st) {
  const unsigned grid = (unsigned)((int64_t)nframes * (w / 16) * (h / 16));
  if (mode == 2)
    hipLaunchKernelGGL(k_motion<2>, dim3(grid), dim3(64), 0, st, w, h, stride, ref_y, cur_y, sl, out,
                       mb_div(w, h), (int)stats);
  else
    hipLaunchKernelGGL(k_motion<1>, dim3(grid), dim3(64), 0, st, w, h, stride, ref_y, cur_y, sl, out,
                       mb_div(w, h), (int)stats);
  return hipGetLastError();
}

}  // namespace p64k
