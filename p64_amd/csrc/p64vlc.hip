// p64vlc.hip -- H.261 entropy coding of GPU records on the GPU (gfx950).
//
// The same bits as the host writer (p64stream.c; the reference's WriteMBHeader
// marker.c:288, EncodeDC/EncodeAC/CBPEncodeAC codec.c:96-352, WriteGOBHeader
// marker.c:171, WritePictureHeader marker.c:103), in one launch per batch of
// pictures (k_vlc_blk, below): one lane per 8x8 block, a wave per ten
// macroblocks in stream order; each wave counts its bits (or takes the
// encoder's counts), finds where they start by a decoupled look-back over the
// waves before it in its picture, and writes them.
// A picture starts at bit `phase` of its first byte so that it continues the
// sequence's bitstream exactly (pictures are not byte aligned in H.261).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>

#include "../../include/p64gpu.h"
#include "../../include/p64stream.h"
#include "vlc_count.h"

extern "C" int p64s_vlc_tables_(uint32_t *t);
extern "C" int p64gpu_fail_(int status, const char *msg);
extern "C" int64_t p64gpu_chunk_bytes_(void);
extern "C" int p64gpu_vlc_len_table_(uint32_t *out);

namespace {

// A bounds-checked build (-DP64_VLC_CHECK, `make vlccheck`; a diagnostic aid,
// not the product): every global store and status access of k_vlc_blk tests
// its index against the buffer it was given and, out of range, sets bit
// `site` of g_vlc_err instead of touching memory.
#ifdef P64_VLC_CHECK
__device__ uint32_t g_vlc_err;
#define VLC_OK(c, site) ((c) ? true : (atomicOr(&g_vlc_err, 1u << (site)), false))
#else
#define VLC_OK(c, site) true
#endif

constexpr int T_MTYPE = 0, T_MVD = 10, T_CBP = 42, T_TC = 106, T_EOB = 538, T_ESC = 539,
              T_FIRST01 = 540, T_N = 541;
struct VlcTables {
  uint32_t t[T_N];  // code | len << 16
};

struct VlcArgs {
  int width, height, nframes, format, ngob, nmb;
  const p64_mb_rec *mb;
  const int16_t *coef;
  const uint8_t *gquant;
  const uint8_t *mquant;
  const int32_t *tr;
  const uint8_t *phase;
  uint32_t *out;  // [nframes][out_words]
  int64_t out_words;
  uint32_t *bits;     // [nframes]
  uint32_t *status;   // [nframes][workgroups][2] uint64 (look-back word, tail), zeroed before the launch
  uint16_t *blk_bits; // [nframes][nmb][8], raster order: [1 + b] block b's bits
  int64_t *seq_bits;  // NULL or [nframes]: the sequences' running bit counts (phase = & 7; updated)
  uint32_t *max_bits; // NULL or [1]: the longest valid picture's bits (zeroed by k_vlc_zero)
};

__device__ __forceinline__ bool mt_quant(int m) { return m == 1 || m == 3 || m == 6 || m == 9; }
__device__ __forceinline__ bool mt_cbp(int m) { return m == 2 || m == 3 || m == 5 || m == 6 || m == 8 || m == 9; }
__device__ __forceinline__ bool mt_mf(int m) { return m >= 4; }
__device__ __forceinline__ bool mt_tc(int m) { return m != 4 && m != 7; }

__device__ __forceinline__ int raster(int format, int g, int m) {
  return format == P64S_QCIF ? (3 * g + m / 11) * 11 + m % 11
                             : ((g >> 1) * 3 + m / 11) * 22 + (g & 1) * 11 + m % 11;
}

// one code: value in the low `len` bits
struct Code {
  uint32_t v;
  int len;
};
__device__ __forceinline__ Code tab(const VlcTables &T, int i) {
  const uint32_t e = T.t[i];
  return Code{e & 0xffffu, (int)(e >> 16)};
}

// the macroblock header (WriteMBHeader marker.c:288-357): up to six codes in
// order MBA, MTYPE, [MQUANT], [MVDH, MVDV], [CBP]; absent ones have len 0
struct Header {
  Code c[6];
  int bits;
  bool bad;
};
// r: the MB's record, rp: the previous MB's (the MVD predictor; MDUs 0, 11
// and 22 reset it, marker.c:311-327), mq: its MQUANT, m: its MDU
__device__ __forceinline__ Header header_codes(const VlcTables &T, p64_mb_rec r, p64_mb_rec rp, int mq, int m) {
  Header h;
  const int mt = r.mtype;
  h.bad = mt < 0 || mt > 9 || (mt_cbp(mt) && (r.cbp < 1 || r.cbp > 63));
#pragma unroll
  for (int i = 0; i < 6; i++) h.c[i] = Code{0u, 0};
  h.bits = 0;
  if (h.bad) return h;
  h.c[0] = Code{1u, 1};  // MBA = 1: every MDU is coded (p64.c:922)
  h.c[1] = tab(T, T_MTYPE + mt);
  if (mt_quant(mt)) h.c[2] = Code{(uint32_t)(mq & 31), 5};
  if (mt_mf(mt)) {
    int dh = r.mvx, dv = r.mvy;
    if (m != 0 && m != 11 && m != 22) {
      if (rp.mtype >= 4 && rp.mtype <= 9) {  // differential to the previous MC macroblock
        dh -= rp.mvx;
        dv -= rp.mvy;
        dh += dh < -16 ? 32 : (dh > 15 ? -32 : 0);
        dv += dv < -16 ? 32 : (dv > 15 ? -32 : 0);
      }
    }
    h.c[3] = tab(T, T_MVD + (dh & 31));
    h.c[4] = tab(T, T_MVD + (dv & 31));
  }
  if (mt_cbp(mt)) h.c[5] = tab(T, T_CBP + r.cbp);
#pragma unroll
  for (int i = 0; i < 6; i++) h.bits += h.c[i].len;
  return h;
}

// wave64 inclusive prefix sum in DPP steps (row_shr 1/2/4/8 inside each
// 16-lane row, then row_bcast 15 / 31 across rows): six VALU adds, no LDS
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false); // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false); // row_bcast:31
  return x;
}
__device__ __forceinline__ int wave_sum_i(int v) {
  return __builtin_amdgcn_readlane(wave_incl_scan(v), 63);
}
__device__ __forceinline__ int wave_excl_scan(int v, int) { return wave_incl_scan(v) - v; }
__device__ __forceinline__ int wave_max_i(int x) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) x = max(x, __shfl_xor(x, d));
  return x;
}
// the wave's LDS writes done and visible to its lanes
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef VLC_WAVES_N
#define VLC_WAVES_N 4
#endif
constexpr int VLC_WAVES = VLC_WAVES_N;  // waves per workgroup
constexpr int VLC_MBS = 10;   // macroblocks per wave: lane 6m + b codes block b of MB m

// raster macroblock k -> stream position j = 33 g + m (GOB g, MDU m; the
// inverse of raster(): GOBs of 11 x 3 MBs, two per GOB row except in QCIF)
__device__ __forceinline__ int stream_pos(int format, int k) {
  const int mbw = format == P64S_QCIF ? 11 : 22;
  const int mby = k / mbw, mbx = k - mby * mbw;
  const int g = format == P64S_QCIF ? mby / 3 : (mby / 3) * 2 + mbx / 11;
  return 33 * g + (mby % 3) * 11 + mbx % 11;
}

// The bit writer of one lane: a segment of the picture's bits starting at
// bit `pos`, MSB first, big-endian bytes in little-endian words (one bswap
// per word), every word ORed into memory -- for the rare wave whose bits
// exceed its LDS copy (k_vlc_blk zeroed its words first).  The range's
// first and last words, when a neighbouring workgroup shares them (s0, s1;
// -1 if not shared), go to two LDS words instead (sh[0], sh[1]): memory
// holds only words no other workgroup touches, and the shared ones reach it
// through the tail hand-over, as in the LDS path.
struct BitWriter {
  uint64_t acc;  // the pending bits, right-aligned
  int nacc;      // how many (< 32 between appends)
  int64_t w;     // picture word the pending bits start in
  uint32_t *out;
  int64_t s0 = -1, s1 = -1;  // the shared words
  uint32_t *sh = nullptr;    // their LDS stand-ins
  int64_t wlo = 0, whi = 0;  // (P64_VLC_CHECK: the workgroup's words)
  __device__ __forceinline__ void start(uint32_t *o, int64_t pos) {
    out = o;
    w = pos >> 5;
    nacc = (int)(pos & 31);  // the bits before the segment, as zeros
    acc = 0;
  }
  __device__ __forceinline__ void word(uint32_t v) {
    if (w == s0 || w == s1 || VLC_OK(w >= wlo && w <= whi, 2))
      atomicOr(w == s0 ? sh : (w == s1 ? sh + 1 : out + w), __builtin_bswap32(v));
  }
  __device__ __forceinline__ void put(uint32_t v, int n) {  // n <= 32
    acc = (acc << n) | v;
    nacc += n;
    if (nacc >= 32) {
      word((uint32_t)(acc >> (nacc - 32)));
      w++;
      nacc -= 32;
    }
  }
  __device__ __forceinline__ void finish() {  // the last, partial word
    if (nacc > 0) word((uint32_t)(acc << (32 - nacc)));
  }
};

// The same writer into a wave's LDS copy of its bits: words w0 ..
// w0 + VLC_EMIT_WORDS - 1 of the picture (the others dropped), all ORed (the
// copy was zeroed), stored afterwards
constexpr int VLC_EMIT_WORDS = 256;  // LDS words of a wave's bits per pass
struct LdsBitWriter {
  uint64_t acc;
  int nacc;
  int w;  // word index in the copy
  uint32_t *buf;
  int64_t w0;
  __device__ __forceinline__ void start(uint32_t *b, int64_t pos) {
    buf = b;
    w = (int)((pos >> 5) - w0);
    nacc = (int)(pos & 31);
    acc = 0;
  }
  __device__ __forceinline__ void put(uint32_t v, int n) {
    acc = (acc << n) | v;
    nacc += n;
    if (nacc >= 32) {
      if ((unsigned)w < (unsigned)VLC_EMIT_WORDS) atomicOr(buf + w, __builtin_bswap32((uint32_t)(acc >> (nacc - 32))));
      w++;
      nacc -= 32;
    }
  }
  __device__ __forceinline__ void finish() {
    if (nacc > 0 && (unsigned)w < (unsigned)VLC_EMIT_WORDS)
      atomicOr(buf + w, __builtin_bswap32((uint32_t)(acc << (32 - nacc))));
  }
};

// The block's codes from its bit 0 into the lane's scratch (VLC_SCR words in
// registers, left-aligned, MSB first), counting them: the one pass of VLC_ONE
// (the count and the codes together; the emission then copies the words to
// the lane's start).  The words shift through r[0..VLC_SCR-1] as they
// complete (r[0] the newest, static register indices: no LDS spent on it);
// a block of more than 32 VLC_SCR bits is coded again at the emission.
// (Measured, tools/vlc_time.py: 6 words 42.7 us, 5: 50.4, 7: 45.1, 8: 44.0;
// the same scratch in LDS, 8 words: 45.7 -- one workgroup less per CU.)
#ifndef VLC_SCR_N
#define VLC_SCR_N 6
#endif
constexpr int VLC_SCR = VLC_SCR_N;  // scratch words per lane (192 bits)
struct RegScrWriter {
  uint64_t acc = 0;
  int nacc = 0, nw = 0, bits = 0;
  uint32_t r[VLC_SCR];
  __device__ __forceinline__ void push(uint32_t x) {
#pragma unroll
    for (int k = VLC_SCR - 1; k > 0; k--) r[k] = r[k - 1];
    r[0] = x;
    nw++;
  }
  __device__ __forceinline__ void put(uint32_t v, int n) {
    acc = (acc << n) | v;
    nacc += n;
    bits += n;
    if (nacc >= 32) {
      push((uint32_t)(acc >> (nacc - 32)));
      nacc -= 32;
    }
  }
  __device__ __forceinline__ void finish() {
    if (nacc > 0) push((uint32_t)(acc << (32 - nacc)));
  }
};

// the scan positions of a block holding a nonzero level, as two 32-bit masks
// (bit p of m0: position p; of m1: position 32 + p) from its 32 packed level
// pairs: v_pk_min_u16 against 1 (a nonzero int16 is >= 1 as u16), v_dot2
// (low + 2 high) and v_lshl_or -- three VALU per pair
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void nz_masks(const uint32_t lv[32], uint32_t &m0, uint32_t &m1) {
  m0 = m1 = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    const u16x2_t v = __builtin_bit_cast(u16x2_t, lv[i]);
    const u16x2_t r = __builtin_elementwise_min(v, (u16x2_t){1, 1});
    const uint32_t b = __builtin_amdgcn_udot2(r, (u16x2_t){1, 2}, 0u, false);
    if (i < 16)
      m0 |= b << (2 * i);
    else
      m1 |= b << (2 * (i - 16));
  }
}

// the codes of one block's levels (EncodeAC codec.c:96 / CBPEncodeAC
// codec.c:141) into the writer, scan positions from 1 for intra blocks (the
// DC is coded alone: the caller leaves bit 0 out of m0), EOB included; a
// CBP-type block without a level writes nothing (codec.c:151; never a
// transmitted block).  Visits the nonzero positions only (m0/m1, lowest
// first), two per step: both levels and both table entries are read
// together, the codes chosen by selects (FIRST01, the TCOEFF table, ESCAPE).
__device__ __forceinline__ void code_of(const VlcTables &T, uint32_t e, bool first, int run, int l, uint32_t &v,
                                        int &n) {
  const int al = l < 0 ? -l : l;
  const uint32_t sg = (uint32_t)(l < 0);
  const Code f = tab(T, T_FIRST01), esc = tab(T, T_ESC);
  const int elen = (run < 27 && al < 16) ? (int)(e >> 16) : 0;
  v = (esc.v << 14) | ((uint32_t)run << 8) | ((uint32_t)l & 0xffu);
  n = esc.len + 14;
  if (elen) {
    v = ((e & 0xffffu) << 1) | sg;
    n = elen + 1;
  }
  if (first && run == 0 && al == 1) {
    v = (f.v << 1) | sg;
    n = f.len + 1;
  }
}
template <typename L, class W>  // L: the level copy, int8 in LDS (the common case) or the int16 levels themselves
__device__ __forceinline__ void block_codes(const VlcTables &T, const L *lvs, uint32_t m0, uint32_t m1, bool cbpt,
                                            W &bw) {
  if (cbpt && !(m0 | m1)) return;
  int last = cbpt ? -1 : 0;
  bool first = cbpt;
  // the two 32-position halves one after the other (32-bit find-first-set
  // and clear: three VALU per position instead of seven on the 64-bit mask)
  auto half = [&](uint32_t mh, int pb) {
    while (mh) {
      const int p1 = pb + (int)__builtin_ctz(mh);
      mh &= mh - 1u;
      const bool two = mh != 0;
      const int p2 = two ? pb + (int)__builtin_ctz(mh) : p1;
      mh &= mh - 1u;
      const int l1 = (int)lvs[p1], l2 = (int)lvs[p2];
      const int r1 = p1 - last - 1, r2 = p2 - p1 - 1;
      last = p2;
      const int a1 = l1 < 0 ? -l1 : l1, a2 = l2 < 0 ? -l2 : l2;
      const uint32_t e1 = T.t[T_TC + min(r1, 26) * 16 + min(a1, 15)];
      const uint32_t e2 = T.t[T_TC + min(r2, 26) * 16 + min(a2, 15)];
      uint32_t v;
      int n;
      code_of(T, e1, first, r1, l1, v, n);
      bw.put(v, n);
      if (two) {
        code_of(T, e2, false, r2, l2, v, n);
        bw.put(v, n);
      }
      first = false;
    }
  };
  half(m0, 0);
  half(m1, 32);
  const Code eob = tab(T, T_EOB);
  bw.put(eob.v, eob.len);
}

// Lane-per-block entropy coding: a wave takes 10 macroblocks consecutive in
// stream order (GOB by GOB), lane 6m + b block b of the m-th, lane b = 0 also
// the MB header (and the GOB / picture header before MDU 0 / GOB 0), so the
// lanes' bits follow each other in lane order.  Every lane runs its own
// block's scan serially (no cross-lane step per code), from an LDS copy of
// the block's levels.
//   VLC_COUNT: the blocks' bits into blk_bits[1..6] (p64gpu_vlc_block_bits_)
//   VLC_ONE / VLC_GIVEN: the picture's bits in one pass -- the blocks' bits
//     counted (VLC_ONE) or read from blk_bits (VLC_GIVEN, the encoder's
//     counts), the workgroup's total (four waves: 40 MBs, one contiguous
//     range of the picture), its start by a decoupled look-back over the
//     workgroups before it, then the codes.  Each wave writes its codes into
//     an LDS copy (ORs of the lanes' words) while wave 0's look-back reads
//     are in flight; the copies are then stored word per thread, shifted to
//     the waves' starts and ORed together where two waves share a word.  The
//     range's first and last words are shared with the neighbouring
//     workgroups: the last one is handed to the next workgroup through its
//     status word ("tail"), which ORs it into its first word and stores that
//     -- no word of the picture is written twice, nothing needs zeroing, and
//     the only waits are on earlier workgroups' totals and the previous one's
//     tail.  Forward progress: a workgroup waits only on lower-numbered ones
//     of its picture (same blockIdx.y), which the dispatcher (each XCD in
//     order over its round-robin share) started before it, so the oldest
//     unfinished workgroup is always resident and never waits.
// The levels' LDS copy is int8 (64 + 16 pad bytes per lane); H.261 levels fit
// it.  A wave with a coded level outside -128..127 (which the reference's
// quantiser never makes, but the ABI takes) reads the int16 levels from
// memory instead: the codes stay the host writer's for every int16 value.
#ifndef VLC_STAGE_N
#define VLC_STAGE_N 64  // bytes of LDS per lane for its levels (80, 16 of them padding: one workgroup less per CU)
#endif
constexpr int VLC_STAGE = VLC_STAGE_N;
enum { VLC_COUNT = 0, VLC_ONE = 1, VLC_GIVEN = 2 };
// status words, two per workgroup of a picture (zeroed before the launch):
// [0] the look-back word: flag (bits 62-63: 1 = the workgroup's own total,
//     2 = its end, i.e. the total of every workgroup up to it + the phase),
//     bit 32 = an invalid record (own / up to it), bits 0-31 the value;
// [1] the tail: bit 63 set once published, bits 0-31 the range's last word
constexpr uint64_t ST_AGG = 1ull << 62, ST_INCL = 2ull << 62, ST_BAD = 1ull << 32;
__device__ __forceinline__ uint64_t st_load(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_store(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t st_wait(const uint64_t *p) {  // until nonzero (wave-uniform)
  for (;;) {
    const uint64_t v = st_load(p);
    const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
    if (u) return u;
    __builtin_amdgcn_s_sleep(1);
  }
}
// the look-back's status words of a launch, zeroed (k_vlc_blk's precondition)
__global__ __launch_bounds__(256) void k_vlc_zero(uint4 *p, unsigned n, uint32_t *max_bits) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) p[i] = make_uint4(0u, 0u, 0u, 0u);
  if (max_bits && i == 0) *max_bits = 0u;
}

// the code tables live in device memory (d_tabs: uploaded once per device,
// vlc_tables_on_device), not in the kernel arguments: 2.6 KB of by-value
// tables made every launch's argument block that large (round 6)
struct DevTabs {
  VlcTables t;
  p64k::VlcLenTab l;
};
__device__ DevTabs d_tabs;
template <int MODE>
__global__ __launch_bounds__(64 * VLC_WAVES) void k_vlc_blk(VlcArgs a) {
  const VlcTables &Tg = d_tabs.t;
  const p64k::VlcLenTab &Lg = d_tabs.l;
  constexpr bool EMIT = MODE != VLC_COUNT, COUNT = MODE != VLC_GIVEN;
  __shared__ VlcTables T;  // per-lane table lookups from LDS, loaded once per workgroup
  __shared__ uint32_t vlen[COUNT && MODE != VLC_ONE ? p64k::VLC_LEN_WORDS : 1];  // the count's code lengths (vlc_count.h)
  if (COUNT && MODE != VLC_ONE && threadIdx.x < 64) p64k::load_vlc_len(Lg, vlen, threadIdx.x);
  __shared__ __align__(16) uint8_t stage[VLC_WAVES * 64 * VLC_STAGE];  // each lane's levels, scan order
  __shared__ __align__(16) uint32_t wbits[EMIT ? VLC_WAVES * VLC_EMIT_WORDS : 4];
  constexpr bool ONEPASS = MODE == VLC_ONE;  // the count pass writes the codes (RegScrWriter)
  RegScrWriter sw;
  for (int i = threadIdx.x; i < T_N; i += 64 * VLC_WAVES) T.t[i] = Tg.t[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fi = blockIdx.y;
  const int wi = blockIdx.x * VLC_WAVES + wv;  // the wave's index in its picture
  const int mb0 = wi * VLC_MBS;                // its first stream position
  if (!EMIT && mb0 >= a.nmb) return;  // whole wave (the coder's keep to the barriers: no bits)
  const int l = min(lane, 6 * VLC_MBS - 1), b = l % 6;
  const int j = min(mb0 + l / 6, a.nmb - 1);  // stream position (tail lanes repeat the last)
  const int g = j / 33, m = j - g * 33, k = raster(a.format, g, m);
  const bool act = lane < 6 * VLC_MBS && mb0 + l / 6 < a.nmb;
  const size_t base = (size_t)fi * a.nmb;
  const p64_mb_rec r = a.mb[base + k];
  const p64_mb_rec rp = a.mb[base + (m % 11 ? k - 1 : k)];  // MVD predictor (same GOB row)
  const int mq = a.mquant ? (int)a.mquant[base + k] : 0;
  const int mt = r.mtype;
  const bool valid = mt >= 0 && mt <= 9;
  const bool cbpt = valid && mt_cbp(mt);
  const int cbp = cbpt ? r.cbp : 0x3f;
  const bool coded = act && valid && mt_tc(mt) && ((cbp >> (5 - b)) & 1);
  // the levels of the coded blocks only (an inter picture's uncoded blocks
  // hold nothing the coder reads; -DVLC_LOAD_ALL: every lane's block, not
  // waiting for the record -- the round-5/6 form)
  const uint32_t co = (uint32_t)(((base + k) * 6 + b) * 128);
  uint32_t lv[32];
#pragma unroll
  for (int i = 0; i < 32; i++) lv[i] = 0u;
#ifndef VLC_LOAD_ALL
  if (coded)
#endif
  {
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.coef, (short)0, (int)((size_t)a.nframes * a.nmb * 768), 0x00020000);  // < 2 GiB (host split)
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(cr, co + 16 * i, 0, 0);
      lv[4 * i] = v[0];
      lv[4 * i + 1] = v[1];
      lv[4 * i + 2] = v[2];
      lv[4 * i + 3] = v[3];
    }
  }
  // the block's nonzero positions (the DC of an intra block is coded apart),
  // its levels as int8 in LDS for the indexed reads of the code loops, and
  // whether one of them does not fit (+128 per int16 half: a byte or not)
  uint32_t m0, m1;
  nz_masks(lv, m0, m1);
  if (!cbpt) m0 &= ~1u;
  if (!coded) m0 = m1 = 0;
  uint32_t wide = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    uint32_t x = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_t, lv[i]) + (u16x2_t){128, 128});
    if (i == 0 && !cbpt) x &= 0xffff0000u;  // (an intra DC is coded from lv[0] itself)
    wide |= x;
  }
  const bool narrow = !__any(coded && (wide & 0xff00ff00u));
  uint8_t *stl = stage + (wv * 64 + lane) * VLC_STAGE;
#pragma unroll
  for (int i = 0; i < 4; i++)
    *reinterpret_cast<uint4 *>(stl + 16 * i) = make_uint4(
        __builtin_amdgcn_perm(lv[8 * i + 1], lv[8 * i], 0x06040200u),
        __builtin_amdgcn_perm(lv[8 * i + 3], lv[8 * i + 2], 0x06040200u),
        __builtin_amdgcn_perm(lv[8 * i + 5], lv[8 * i + 4], 0x06040200u),
        __builtin_amdgcn_perm(lv[8 * i + 7], lv[8 * i + 6], 0x06040200u));
  const int8_t *lvs = reinterpret_cast<const int8_t *>(stl);
  const int16_t *lvg = reinterpret_cast<const int16_t *>(a.coef) + ((base + k) * 6 + b) * 64;
  uint16_t *bk = a.blk_bits + (base + k) * 8;
  int bb = 0;  // the block's bits (an intra block's DC included)
  if (ONEPASS) {
    if (coded) {
      if (!cbpt) {  // EncodeDC codec.c:343-352
        const int dc0 = (int)(int16_t)(lv[0] & 0xffffu);
        const int dc = dc0 < 1 ? 1 : (dc0 > 254 ? 254 : dc0);
        sw.put((uint32_t)(dc == 128 ? 255 : dc), 8);
      }
      if (narrow)
        block_codes(T, lvs, m0, m1, cbpt, sw);
      else
        block_codes(T, lvg, m0, m1, cbpt, sw);
      sw.finish();
      bb = sw.bits;
    }
  } else if (COUNT) {
    const uint8_t *len = reinterpret_cast<const uint8_t *>(vlen);
    if (narrow) {
      if (coded) bb = p64k::block_vlc_bits(len, lvs, m0, m1, cbpt);
    } else if (coded) {
      bb = p64k::block_vlc_bits(len, lvg, m0, m1, cbpt);
    }
  } else {
    bb = coded && VLC_OK(a.blk_bits != nullptr, 7) ? (int)bk[1 + b] : 0;
  }
  if (!EMIT) {
    if (act && VLC_OK(a.blk_bits != nullptr && fi < a.nframes && k < a.nmb, 6)) bk[1 + b] = (uint16_t)bb;
    return;
  }
  // the lane's bits: the headers (b = 0: picture header before MDU 0 of GOB 0,
  // GOB header before MDU 0, the MB header), then its block
  // (the header codes stay in registers for the emission: the workgroup's
  // LDS, not its registers, sets the occupancy)
  const Header hd = header_codes(T, r, rp, mq, m);
  const int hbits = act && b == 0 ? (j == 0 ? 32 + (a.format == P64S_NTSC ? 9 : 0) : 0) + (m == 0 ? 26 : 0) + hd.bits : 0;
  const bool hbad = act && b == 0 && hd.bad;
  const int lbits = hbits + bb;
  const int incl = wave_incl_scan(lbits);
  const int rel = incl - lbits;  // the lane's first bit, from the wave's first
  const int tot = __builtin_amdgcn_readlane(incl, 63);
  const bool bad = __any(hbad);
  const uint32_t trv = (uint32_t)a.tr[fi] & 31u, gqv = a.gquant[(size_t)fi * a.ngob + g] & 31u;
  auto emit = [&](auto &bw, uint32_t *dst, int64_t base, bool block) {
    if (act && b == 0) {
      bw.start(dst, base + rel);
      if (j == 0) {  // WritePictureHeader marker.c:103-135
        bw.put(0x10u, 20);
        bw.put(trv, 5);
        bw.put(a.format == P64S_QCIF ? 0u : 4u, 6);
        if (a.format == P64S_NTSC) bw.put(0x18cu, 9);  // PEI 1, PSPARE 0x8c
        bw.put(0u, 1);                                   // PEI 0
      }
      if (m == 0) {  // WriteGOBHeader marker.c:171-198
        const uint32_t gn = a.format == P64S_QCIF ? 2 * g + 1 : g + 1;
        bw.put((1u << 10) | (gn << 6) | (gqv << 1), 26);
      }
#pragma unroll
      for (int i = 0; i < 6; i++)
        if (hd.c[i].len) bw.put(hd.c[i].v, hd.c[i].len);
      bw.finish();
    }
    if (coded && block) {
      bw.start(dst, base + rel + hbits);
      if (!cbpt) {  // EncodeDC codec.c:343-352
        const int dc0 = (int)(int16_t)(lv[0] & 0xffffu);
        const int dc = dc0 < 1 ? 1 : (dc0 > 254 ? 254 : dc0);
        bw.put((uint32_t)(dc == 128 ? 255 : dc), 8);
      }
      if (narrow)
        block_codes(T, lvs, m0, m1, cbpt, bw);
      else
        block_codes(T, lvg, m0, m1, cbpt, bw);
      bw.finish();
    }
  };
  // The workgroup's four waves are one contiguous range of the picture: its
  // total and invalid flag from the waves' (LDS), then wave 0 publishes the
  // total and issues the look-back's first read while every wave writes its
  // codes into its LDS copy at positions from its own start (word aligned)
  __shared__ int s_tot[VLC_WAVES], s_bad[VLC_WAVES];
  __shared__ int64_t s_first;
  if (lane == 0) {
    s_tot[wv] = tot;
    s_bad[wv] = bad;
  }
  __syncthreads();
  int wt = 0, off[VLC_WAVES];
  bool wbad = false, big = false;
#pragma unroll
  for (int v = 0; v < VLC_WAVES; v++) {
    off[v] = wt;
    wt += s_tot[v];
    wbad |= s_bad[v] != 0;
    big |= s_tot[v] > 32 * VLC_EMIT_WORDS - 32;  // (a copy holds 8,160 bits at any phase)
  }
  const int G = blockIdx.x, ng = gridDim.x;  // the workgroup's index in its picture, their number
  uint64_t *stw = reinterpret_cast<uint64_t *>(a.status) + (size_t)fi * ng * 2;
  uint64_t s = ST_INCL;
  if (wv == 0 && G > 0) {
    if (lane == 0 && VLC_OK(fi < a.nframes && G < ng, 4)) st_store(stw + 2 * G, ST_AGG | (wbad ? ST_BAD : 0) | (uint64_t)(uint32_t)wt);
    if (G - 1 - lane >= 0) s = st_load(stw + 2 * (G - 1 - lane));
  }
  uint32_t *wb = wbits + wv * VLC_EMIT_WORDS;
  if (!big) {
    reinterpret_cast<uint4 *>(wb)[lane] = make_uint4(0, 0, 0, 0);
    wave_lds_sync();
#ifndef VLC_NOEMIT  // (timing experiment only: no codes)
    if (tot > 0) {
      LdsBitWriter bw;
      bw.w0 = 0;
      // VLC_ONE: a block whose codes fit the scratch is copied from it to the
      // lane's start (word by word, shifted, ORed where lanes share a word);
      // the others are coded again here
      const bool scr = ONEPASS && bb <= 32 * VLC_SCR;
      emit(bw, wb, 0, !scr);
      if (ONEPASS && coded && scr) {
        const int p = rel + hbits, sh = p & 31, wi = p >> 5;
#pragma unroll
        for (int k = 0; k < VLC_SCR; k++) {
          const int i = sw.nw - 1 - k;  // r[k] is word i of the block
          if (i >= 0) {
            const uint32_t sv = sw.r[k];
            atomicOr(wb + wi + i, __builtin_bswap32(sv >> sh));
            if (sh) atomicOr(wb + wi + i + 1, __builtin_bswap32(sv << (32 - sh)));
          }
        }
      }
    }
#endif
  }
  // the start (wave 0): the phase for the first workgroup, else the end of the
  // previous one -- 64 workgroups at a time, lane i reading the one i places
  // back: the nearest published end and every total after it (else read again)
  if (wv == 0) {
    int64_t first = 0;
    bool bad_all = wbad;
    if (G == 0) {
      first = a.seq_bits ? (a.seq_bits[fi] & 7) : (a.phase ? a.phase[fi] : 0);
#ifdef VLC_NOSYNC  // (timing experiment only: wrong bits) no look-back
    } else if (true) {
      first = (int64_t)G * 12000;
#endif
    } else {
      for (int v = G - 1;;) {
        const uint64_t inc = __ballot((s >> 62) == 2), zero = __ballot(s == 0);
        const int p = inc ? (int)__builtin_ctzll(inc) : 64;  // the nearest end
        const uint64_t need = p == 64 ? ~0ull : (2ull << p) - 1;
        if (!(zero & need)) {
          const bool use = lane <= p;
          first += wave_sum_i(use ? (int)(uint32_t)s : 0);
          bad_all |= __any(use && (s & ST_BAD));
          if (p < 64) break;
          v -= 64;
        } else {
          __builtin_amdgcn_s_sleep(1);
        }
        s = v - lane >= 0 ? st_load(stw + 2 * (v - lane)) : ST_INCL;
      }
    }
    const int64_t endb = first + wt;
    if (lane == 0 && VLC_OK(fi < a.nframes && G < ng, 4)) {
      st_store(stw + 2 * G, ST_INCL | (bad_all ? ST_BAD : 0) | (uint64_t)(uint32_t)endb);
      if (G == ng - 1 && VLC_OK(fi < a.nframes, 5)) {
        const bool ok = !bad_all && endb + 64 <= a.out_words * 32;
        a.bits[fi] = ok ? (uint32_t)endb : 0xFFFFFFFFu;
        // the sequence continues after this picture: its bits less the phase
        // (WG 0 read seq_bits before publishing its end, which this one saw)
        if (a.seq_bits && ok) a.seq_bits[fi] = (a.seq_bits[fi] & ~(int64_t)7) + endb;
        if (a.max_bits && ok) atomicMax(a.max_bits, (uint32_t)endb);
      }
      s_first = first;
    }
  }
  __syncthreads();
  const int64_t first = s_first, endb = first + wt;
  if (endb + 64 > a.out_words * 32) return;  // (nor does any later workgroup of the picture write)
  uint32_t *out = a.out + (size_t)fi * a.out_words;
  // the words [w0, wl]; the first is shared with the previous workgroup
  // unless the range starts on a word boundary (or is the picture's start),
  // the last with the next unless it ends on one (or is the picture's end)
  const int64_t w0 = first >> 5, wl = (endb - 1) >> 5;
  const bool sh_first = G > 0 && (first & 31) != 0;
  const bool sh_last = G < ng - 1 && (endb & 31) != 0;
  uint32_t firstv = 0, lastv = 0;
  if (!big && wt > 0) {  // (the common case) the four copies shifted to their starts, word per thread
    auto word = [&](int64_t gw) {  // picture word gw of this range: the waves' bits in it
      uint32_t x = 0;
#pragma unroll
      for (int v = 0; v < VLC_WAVES; v++) {
        const int tv = s_tot[v];
        const int64_t fv = first + off[v];
        const int64_t t = gw - (fv >> 5);
        if (tv > 0 && t >= 0 && gw <= (fv + tv - 1) >> 5) {
          const uint32_t *bv = wbits + v * VLC_EMIT_WORDS;
          const int sh = (int)(fv & 31), nwr = (tv + 31) >> 5;
          const uint32_t cur = t < nwr ? __builtin_bswap32(bv[t]) : 0u;
          const uint32_t prev = t > 0 ? __builtin_bswap32(bv[t - 1]) : 0u;
          x |= __builtin_bswap32(sh ? (cur >> sh) | (prev << (32 - sh)) : cur);
        }
      }
      return x;
    };
    for (int64_t gw = w0 + threadIdx.x; gw <= wl; gw += 64 * VLC_WAVES)
      if (!(gw == w0 && sh_first) && !(gw == wl && sh_last) && VLC_OK(gw >= 0 && gw < a.out_words, 0))
        out[gw] = word(gw);
    if (wv == 0) {
      firstv = word(w0);
      lastv = word(wl);
    }
  } else if (wt > 0) {  // a wave past its copy: zero our words, OR the codes in memory
    // (never a word a neighbour shares: the previous workgroup may still be
    // ORing into it in this same path, or the next one already have; the
    // shared words collect in s_shw and leave by the hand-over below.
    // A big range spans > 8,000 bits, so w0 < wl.)
    __shared__ uint32_t s_shw[2];
    const int64_t s0 = sh_first ? w0 : -1, s1 = sh_last ? wl : -1;
    if (threadIdx.x < 2) s_shw[threadIdx.x] = 0;
    for (int64_t gw = w0 + threadIdx.x; gw <= wl; gw += 64 * VLC_WAVES)
      if (gw != s0 && gw != s1 && VLC_OK(gw >= 0 && gw < a.out_words, 1)) out[gw] = 0;
    __threadfence();
    __syncthreads();
    if (tot > 0) {
      BitWriter bw;
      bw.s0 = s0;
      bw.s1 = s1;
      bw.sh = s_shw;
      bw.wlo = w0;
      bw.whi = wl;
      emit(bw, out, first + off[wv], true);
    }
    __threadfence();
    __syncthreads();
    if (wv == 0) {  // (only read where shared: the others are in memory already)
      firstv = s_shw[0];
      lastv = s_shw[1];
    }
  }
  if (wv != 0) return;
  // the shared words (wave 0): hand the last one on, then take the previous
  // workgroup's
  if (wt == 0 || w0 == wl) {  // (one word: the previous workgroup's tail and ours)
    uint32_t v = wt > 0 ? firstv : 0u;
#ifndef VLC_NOSYNC
    if (sh_first) v |= (uint32_t)st_wait(stw + 2 * (G - 1) + 1);
#endif
    if (sh_last) {
      if (lane == 0) st_store(stw + 2 * G + 1, (1ull << 63) | v);
    } else if ((wt > 0 || sh_first) && lane == 0 && VLC_OK(w0 >= 0 && w0 < a.out_words, 3)) {
      out[w0] = v;
    }
  } else {
    if (sh_last && lane == 0) st_store(stw + 2 * G + 1, (1ull << 63) | lastv);
    if (sh_first) {
#ifdef VLC_NOSYNC
      const uint32_t pv = 0;
#else
      const uint32_t pv = (uint32_t)st_wait(stw + 2 * (G - 1) + 1);
#endif
      if (lane == 0 && VLC_OK(w0 >= 0 && w0 < a.out_words, 3)) out[w0] = firstv | pv;
    }
  }
}

// Every pointer of p64gpu_vlc_args must be memory the device can address:
// device memory, host memory pinned by hipHostMalloc / hipHostRegister (torch
// pin_memory) or managed memory.  Pinned host memory is addressed through the
// device pointer HIP reports for it (the same address for hipHostMalloc,
// measured: tools/vlc_fault_probe.py stage A); pageable host memory
// (hipMemoryTypeUnregistered), which the kernel's stores would fault on, is
// refused.  Returns the pointer to pass to the kernel, or nullptr.
template <class T>
T *device_addressable(T *p) {
  if (!p) return p;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, (const void *)p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged) return p;
  if (at.type == hipMemoryTypeHost && at.devicePointer) return reinterpret_cast<T *>(at.devicePointer);
  return nullptr;
}

thread_local VlcTables g_tab;
thread_local bool g_tab_ok = false;
thread_local p64k::VlcLenTab g_len;  // the count's code lengths (p64gpu_vlc_len_table_)
thread_local bool g_len_ok = false;

// d_tabs on the current device: uploaded by the first call on each device
// from a pinned host copy (built once from the host writer's tables) and
// synchronised, so every later launch -- on any stream, captured or not --
// finds it in place.  A first call made while its stream is capturing
// records the upload as a copy node of the graph instead (the pinned copy
// outlives every graph) and leaves the device marked not yet uploaded.
std::mutex g_tabs_mu;
DevTabs *g_tabs_host = nullptr;
uint64_t g_tabs_done = 0;  // bit d: device d has d_tabs
int vlc_tables_on_device(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev > 63) return p64gpu_fail_(P64GPU_E_HIP, "vlc: device");
  std::lock_guard<std::mutex> lk(g_tabs_mu);
  if (g_tabs_done >> dev & 1) return P64GPU_OK;
  if (!g_tabs_host) {
    DevTabs *h = nullptr;
    if (hipHostMalloc((void **)&h, sizeof(DevTabs), 0) != hipSuccess)
      return p64gpu_fail_(P64GPU_E_NOMEM, "vlc: pinned table copy");
    const int s = p64gpu_vlc_len_table_(h->l.w);  // (fills g_tab)
    if (s) return s;
    h->t = g_tab;
    g_tabs_host = h;
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return p64gpu_fail_(P64GPU_E_HIP, "vlc: capture status");
  if (hipMemcpyToSymbolAsync(HIP_SYMBOL(d_tabs), g_tabs_host, sizeof(DevTabs), 0, hipMemcpyHostToDevice, st) !=
      hipSuccess)
    return p64gpu_fail_(P64GPU_E_HIP, "vlc: table upload");
  if (cs == hipStreamCaptureStatusNone) {
    if (hipStreamSynchronize(st) != hipSuccess) return p64gpu_fail_(P64GPU_E_HIP, "vlc: table upload sync");
    g_tabs_done |= 1ull << dev;
  }
  return P64GPU_OK;
}

}  // namespace

extern "C" {

#ifdef P64_VLC_CHECK
// (bounds-checked build only) the sites k_vlc_blk found out of range since
// the last call (bit i = site i of VLC_OK), then cleared; synchronises
int p64gpu_vlc_check_errors_(uint32_t *err) {
  const uint32_t z = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(err, HIP_SYMBOL(g_vlc_err), 4) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_vlc_err), &z, 4) != hipSuccess)
    return p64gpu_fail_(P64GPU_E_HIP, "vlc check: symbol copy");
  return P64GPU_OK;
}
#endif

int64_t p64gpu_vlc_max_bytes(int width, int height) {
  const int64_t nmb = (int64_t)(width / 16) * (height / 16);
  // picture + GOB headers; per MB header <= 1+10+5+22+9 bits, 6 blocks of
  // DC 8 + 63 escapes of 20 + EOB 2; plus 8 words of slack
  return (41 + 12 * 26 + nmb * (47 + 6 * (8 + 63 * 20 + 2)) + 7) / 8 + 32;
}

int p64gpu_vlc_pictures(const p64gpu_vlc_args *x, void *stream) {
  if (!x || !x->mb || !x->coef || !x->gquant || !x->tr || !x->out || !x->bits || !x->scratch)
    return p64gpu_fail_(P64GPU_E_INVALID, "vlc: NULL argument");
  const int fmt = p64s_format_of(x->width, x->height);
  if (fmt < 0) return fmt;
  if (x->nframes < 1 || x->nframes > 65535)
    return p64gpu_fail_(P64GPU_E_INVALID, "vlc: nframes out of range");
  if (x->flags != 0) return p64gpu_fail_(P64GPU_E_INVALID, "vlc: unknown flags");
  if (x->out_stride < p64gpu_vlc_max_bytes(x->width, x->height) || (x->out_stride & 3) ||
      ((uintptr_t)x->out & 3))
    return p64gpu_fail_(P64GPU_E_INVALID, "vlc: out_stride below p64gpu_vlc_max_bytes or not 4-aligned");
  if (((uintptr_t)x->scratch & 7) || ((uintptr_t)x->coef & 15) || ((uintptr_t)x->mb & 3) ||
      ((uintptr_t)x->blk_bits & 15) || ((uintptr_t)x->seq_bits & 7) || ((uintptr_t)x->max_bits & 3))
    return p64gpu_fail_(P64GPU_E_INVALID,
                        "vlc: scratch must be 8-byte, coef and blk_bits 16-byte, mb 4-byte aligned");
  p64gpu_vlc_args y = *x;  // the pointers as the device addresses them
#define VLC_ADDR(f)                                                                                         \
  if (x->f && !(y.f = device_addressable(x->f)))                                                            \
    return p64gpu_fail_(P64GPU_E_INVALID, "vlc: " #f " is not device-addressable memory (pageable host memory?)");
  VLC_ADDR(mb) VLC_ADDR(coef) VLC_ADDR(gquant) VLC_ADDR(mquant) VLC_ADDR(tr) VLC_ADDR(phase) VLC_ADDR(out)
  VLC_ADDR(bits) VLC_ADDR(scratch) VLC_ADDR(blk_bits) VLC_ADDR(seq_bits) VLC_ADDR(max_bits)
#undef VLC_ADDR
  x = &y;
  if (!g_len_ok) {  // (fills g_tab too)
    const int s = p64gpu_vlc_len_table_(g_len.w);
    if (s) return s;
    g_len_ok = true;
  }
  {
    const int s = vlc_tables_on_device((hipStream_t)stream);
    if (s) return s;
  }
  int ngob = 0;
  p64s_geometry(fmt, nullptr, nullptr, &ngob);
  const int nmb = ngob * 33;
  // pictures per launch: the levels of one launch within the 2 GiB range of
  // the kernels' 32-bit buffer offsets (the encoder's split, p64gpu_abi.hip)
  const int64_t per = (int64_t)nmb * 768;
  const int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(x->nframes, p64gpu_chunk_bytes_() / per));
  hipStream_t st = (hipStream_t)stream;
  const int64_t out_words = x->out_stride / 4;
  for (int f0 = 0; f0 < x->nframes; f0 += chunk) {
    const int nc = std::min(chunk, x->nframes - f0);
    const size_t m0 = (size_t)f0 * nmb;
    VlcArgs a;
    a.width = x->width;
    a.height = x->height;
    a.nframes = nc;
    a.format = fmt;
    a.ngob = ngob;
    a.nmb = nmb;
    a.mb = x->mb + m0;
    a.coef = x->coef + m0 * 384;
    a.gquant = x->gquant + (size_t)f0 * ngob;
    a.mquant = x->mquant ? x->mquant + m0 : nullptr;
    a.tr = x->tr + f0;
    a.phase = x->phase ? x->phase + f0 : nullptr;
    a.out = reinterpret_cast<uint32_t *>(x->out) + (size_t)f0 * out_words;
    a.out_words = out_words;
    a.bits = x->bits + f0;
    a.seq_bits = x->seq_bits ? x->seq_bits + f0 : nullptr;
    a.max_bits = x->max_bits;
    // this chunk's [6][nc][nmb] words of the scratch
    uint32_t *scr = x->scratch + 6 * m0;
    a.status = scr;  // [nc][nwg][2] uint64: the look-back word and the tail
    const int nwg = (nmb + VLC_WAVES * VLC_MBS - 1) / (VLC_WAVES * VLC_MBS);  // workgroups per picture
    const dim3 grid((unsigned)nwg, (unsigned)nc);
    // the status words zeroed by a kernel, not hipMemsetAsync: captured in a
    // HIP graph, the memset node was seen not to complete before this
    // launch's look-back on some replays (stale status words: wrong starts,
    // invalid flags, and stores from a garbage start -- the illegal-address
    // faults of round 5's variant and of round 6's per-step fed graphs;
    // DESIGN.md 9c); kernel-to-kernel order within a stream always holds
    const unsigned nz = (unsigned)nc * (unsigned)nwg;  // uint4 per workgroup
#ifdef VLC_STATUS_MEMSET  // (the round-5 form, kept for the A/B of tools/vlc_fault_probe.py stage E)
    hipError_t me = hipMemsetAsync(scr, 0, (size_t)nz * 16, st);
    if (me == hipSuccess && f0 == 0 && x->max_bits) me = hipMemsetAsync(x->max_bits, 0, 4, st);
    if (me != hipSuccess) return p64gpu_fail_(P64GPU_E_HIP, hipGetErrorString(me));
#else
    hipLaunchKernelGGL(k_vlc_zero, dim3((nz + 255) / 256), dim3(256), 0, st, reinterpret_cast<uint4 *>(scr), nz,
                       f0 == 0 ? x->max_bits : nullptr);
#endif
    if (x->blk_bits) {  // the blocks' bits from the encoder: no count
      a.blk_bits = x->blk_bits + m0 * 8;
      hipLaunchKernelGGL(k_vlc_blk<VLC_GIVEN>, grid, dim3(64 * VLC_WAVES), 0, st, a);
    } else {
      a.blk_bits = nullptr;
      hipLaunchKernelGGL(k_vlc_blk<VLC_ONE>, grid, dim3(64 * VLC_WAVES), 0, st, a);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return p64gpu_fail_(P64GPU_E_HIP, hipGetErrorString(e));
  return P64GPU_OK;
}

// (library-internal) the count's code-length table in device memory (for the
// BITS instances of the block-layout encoders), uploaded if needed
const uint32_t *p64gpu_vlc_len_dev_(void *stream) {
  if (vlc_tables_on_device((hipStream_t)stream)) return nullptr;
  void *p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(d_tabs)) != hipSuccess) return nullptr;
  return reinterpret_cast<const DevTabs *>(p)->l.w;
}

// (library-internal) the code-length table of the block bit counts
// (vlc_count.h VlcLenTab): byte min(run, 27) * 17 + min(|level|, 16) = the
// TCOEFF code length + 1 (sign), 20 (escape) where there is no code.  The
// counting takes FIRST01 as 2 bits and EOB as 2 -- checked here against the
// tables.
int p64gpu_vlc_len_table_(uint32_t *out) {
  if (!g_tab_ok) {
    const int s = p64s_vlc_tables_(g_tab.t);
    if (s) return s;
    g_tab_ok = true;
  }
  const int lf = (int)(g_tab.t[T_FIRST01] >> 16), le = (int)(g_tab.t[T_EOB] >> 16), lx = (int)(g_tab.t[T_ESC] >> 16);
  if (lf != 1 || le != 2 || lx != 6) return p64gpu_fail_(P64GPU_E_INVALID, "vlc: unexpected table lengths");
  uint8_t *b = reinterpret_cast<uint8_t *>(out);
  for (int i = 0; i < 4 * p64k::VLC_LEN_WORDS; i++) b[i] = 0;
  for (int r = 0; r < p64k::VLC_LEN_RUNS; r++)
    for (int l = 0; l < p64k::VLC_LEN_LEVELS; l++) {
      const int len = (r < 27 && l < 16) ? (int)(g_tab.t[T_TC + r * 16 + l] >> 16) : 0;
      b[r * p64k::VLC_LEN_LEVELS + l] = (uint8_t)(len ? len + 1 : 20);
    }
  return P64GPU_OK;
}

// (library-internal) the blocks' coded bits of an encoded batch into
// blk_bits[1..6] per MB by the count pass -- for encodes that took the fused
// kernel (P64GPU_FUSED, capture without ME records), which does not count
int p64gpu_vlc_block_bits_(int width, int height, int nframes, const p64_mb_rec *mb, const int16_t *coef,
                           uint16_t *blk_bits, void *stream) {
  const int fmt = p64s_format_of(width, height);
  if (fmt < 0) return fmt;
  int s = vlc_tables_on_device((hipStream_t)stream);
  if (s) return s;
  int ngob = 0;
  p64s_geometry(fmt, nullptr, nullptr, &ngob);
  const int nmb = ngob * 33;
  const int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(nframes, p64gpu_chunk_bytes_() / ((int64_t)nmb * 768)));
  for (int f0 = 0; f0 < nframes; f0 += chunk) {
    const int nc = std::min(chunk, nframes - f0);
    const size_t m0 = (size_t)f0 * nmb;
    VlcArgs a{};
    a.width = width;
    a.height = height;
    a.nframes = nc;
    a.format = fmt;
    a.ngob = ngob;
    a.nmb = nmb;
    a.mb = mb + m0;
    a.coef = coef + m0 * 384;
    a.blk_bits = blk_bits + m0 * 8;
    const dim3 grid((unsigned)((nmb + VLC_WAVES * VLC_MBS - 1) / (VLC_WAVES * VLC_MBS)), (unsigned)nc);
    hipLaunchKernelGGL(k_vlc_blk<VLC_COUNT>, grid, dim3(64 * VLC_WAVES), 0, (hipStream_t)stream, a);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? P64GPU_OK : p64gpu_fail_(P64GPU_E_HIP, hipGetErrorString(e));
}

}  // extern "C"
