// p64vlc.hip -- H.261 entropy coding of GPU records on the GPU (gfx950).
//
// The same bits as the host writer (p64stream.c; the reference's WriteMBHeader
// marker.c:288, EncodeDC/EncodeAC/CBPEncodeAC codec.c:96-352, WriteGOBHeader
// marker.c:171, WritePictureHeader marker.c:103), in three passes per batch of
// pictures:
//   1. k_vlc_count  one wave per macroblock: code lengths -> bits per MB.  Each
//                   lane holds one zigzag level; the run before a nonzero level
//                   is the distance to the next lower set bit of the wave's
//                   nonzero ballot, so the run-length scan needs no loop.
//   2. k_vlc_scan   stream-order prefix sum of the MB sizes per picture (GOB /
//                   MDU order of Bpos io.c:757, headers included).
//   3. k_vlc_emit   one wave per macroblock again: each lane places its codes
//                   at its bit offset (wave prefix sum of lengths) with LDS
//                   atomic ORs into the MB's segment, which is then stored;
//                   only the two words shared with neighbouring segments are
//                   ORed into global memory (the scan zeroed the used words).
// A picture starts at bit `phase` of its first byte so that it continues the
// sequence's bitstream exactly (pictures are not byte aligned in H.261).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/p64gpu.h"
#include "../../include/p64stream.h"

extern "C" int p64s_vlc_tables_(uint32_t *t);
extern "C" int p64gpu_fail_(int status, const char *msg);

namespace {

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
  uint32_t *mb_bits;  // [nframes][nmb], stream order
  uint32_t *mb_off;   // [nframes][nmb], stream order
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
__device__ __forceinline__ Header header_codes(const VlcTables &T, const VlcArgs &a, int fi, int g,
                                               int m) {
  Header h;
  const size_t base = (size_t)fi * a.nmb;
  const p64_mb_rec r = a.mb[base + raster(a.format, g, m)];
  const int mt = r.mtype;
  h.bad = mt < 0 || mt > 9 || (mt_cbp(mt) && (r.cbp < 1 || r.cbp > 63));
#pragma unroll
  for (int i = 0; i < 6; i++) h.c[i] = Code{0u, 0};
  h.bits = 0;
  if (h.bad) return h;
  h.c[0] = Code{1u, 1};  // MBA = 1: every MDU is coded (p64.c:922)
  h.c[1] = tab(T, T_MTYPE + mt);
  if (mt_quant(mt)) h.c[2] = Code{a.mquant ? (uint32_t)(a.mquant[base + raster(a.format, g, m)] & 31) : 0u, 5};
  if (mt_mf(mt)) {
    int dh = r.mvx, dv = r.mvy;
    if (m != 0 && m != 11 && m != 22) {
      const p64_mb_rec p = a.mb[base + raster(a.format, g, m - 1)];
      if (p.mtype >= 4 && p.mtype <= 9) {  // differential to the previous MC macroblock
        dh -= p.mvx;
        dv -= p.mvy;
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

// the code of this lane's level in block c (EncodeAC codec.c:96 / CBPEncodeAC
// codec.c:141); len 0 for no code
__device__ __forceinline__ Code level_code(const VlcTables &T, int lane, int lev, uint64_t nz,
                                           bool cbp_block) {
  if (!((nz >> lane) & 1)) return Code{0, 0};
  const uint64_t below = nz & ((1ull << lane) - 1ull);
  const int start = cbp_block ? 0 : 1;
  const int prev = below ? 63 - __clzll(below) : start - 1;
  const int run = lane - prev - 1;
  const int al = lev < 0 ? -lev : lev;
  const bool first = cbp_block && !below;
  if (first && run == 0 && al == 1) {
    const Code f = tab(T, T_FIRST01);
    return Code{(f.v << 1) | (lev < 0), f.len + 1};
  }
  if (run < 27 && al < 16) {
    const Code e = tab(T, T_TC + run * 16 + al);
    if (e.len) return Code{(e.v << 1) | (lev < 0), e.len + 1};
  }
  const Code esc = tab(T, T_ESC);  // ESCAPE, 6-bit run, 8-bit level
  return Code{(esc.v << 14) | ((uint32_t)run << 8) | ((uint32_t)lev & 0xffu), esc.len + 14};
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

// bits of `c` at bit position `pos` of a word buffer (MSB-first bytes,
// little-endian words: bswap per word); LDS atomics in the emit kernel
__device__ __forceinline__ void put_bits(uint32_t *out, int pos, Code c) {
  if (!c.len) return;
  const int w = pos >> 5;
  const int sh = pos & 31;
  const uint64_t x = (uint64_t)c.v << (64 - c.len - sh);  // big-endian within 64 bits
  const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
  if (hi) atomicOr(out + w, __builtin_bswap32(hi));
  if (lo) atomicOr(out + w + 1, __builtin_bswap32(lo));
}

constexpr int SEG_WORDS = 256;  // >= (8192 bits) one macroblock's segment + headers
constexpr int VLC_WAVES = 4;    // waves per workgroup
constexpr int VLC_MBS = 1;      // consecutive stream-order macroblocks per wave

// one macroblock (wave-wide); EMIT places its segment's bits into seg
template <bool EMIT>
__device__ __forceinline__ int code_mb(const VlcTables &T, const VlcArgs &a, int fi, int j,
                                       int lane, uint32_t *seg, int64_t *seg_first) {
  const int g = j / 33, m = j - g * 33;
  const size_t base = (size_t)fi * a.nmb;
  const int k = raster(a.format, g, m);
  const p64_mb_rec r = a.mb[base + k];
  const Header hd = header_codes(T, a, fi, g, m);
  if (hd.bad) return -1;
  const int mt = r.mtype;
  const bool cbpt = mt_cbp(mt);
  const int cbp = cbpt ? r.cbp : 0x3f;
  // this macroblock's segment of the picture: [s0, off + bits), s0 including
  // the GOB header before MDU 0 and the picture header before GOB 0
  int64_t off = 0, s0 = 0, sbase = 0;
  if (EMIT) {
    off = a.mb_off[base + j];
    s0 = j == 0 ? (a.phase ? a.phase[fi] : 0) : (m == 0 ? off - 26 : off);
    sbase = s0 & ~(int64_t)31;  // seg[0] <-> picture word s0 >> 5
    *seg_first = s0;
    if (lane == 0) {
      if (j == 0) {  // picture header (WritePictureHeader marker.c:103-135)
        const int p0 = (int)(s0 - sbase);
        put_bits(seg, p0, Code{0x10u, 20});
        put_bits(seg, p0 + 20, Code{(uint32_t)a.tr[fi] & 31u, 5});
        put_bits(seg, p0 + 25, Code{a.format == P64S_QCIF ? 0u : 4u, 6});
        if (a.format == P64S_NTSC) put_bits(seg, p0 + 31, Code{0x18cu, 9});  // PSPARE 0x8c
      }
      if (m == 0) {  // GOB header (WriteGOBHeader marker.c:171-198)
        const uint32_t gn = a.format == P64S_QCIF ? 2 * g + 1 : g + 1;
        const uint32_t gq = a.gquant[(size_t)fi * a.ngob + g] & 31u;
        put_bits(seg, (int)(off - 26 - sbase), Code{(1u << 10) | (gn << 6) | (gq << 1), 26});
      }
      int p = (int)(off - sbase);
#pragma unroll
      for (int i = 0; i < 6; i++) {
        put_bits(seg, p, hd.c[i]);
        p += hd.c[i].len;
      }
    }
  }
  int bits = hd.bits;
  if (mt_tc(mt)) {
    int levs[6];  // all six blocks' levels in flight at once (latency, not bandwidth, binds)
#pragma unroll
    for (int c = 0; c < 6; c++) levs[c] = a.coef[(base + k) * 384 + c * 64 + lane];
#pragma unroll
    for (int c = 0; c < 6; c++) {
      if (!((cbp >> (5 - c)) & 1)) continue;
      const int lev = levs[c];
      const uint64_t nz = __ballot(lev != 0 && (cbpt || lane > 0));
      if (cbpt && !nz) continue;  // CBPEncodeAC: no level, nothing written
      const Code lc = level_code(T, lane, lev, nz, cbpt);
      const int dcbits = cbpt ? 0 : 8;
      if (EMIT) {
        const int b0 = (int)(off - sbase) + bits;
        if (!cbpt && lane == 0) {  // EncodeDC codec.c:343-352
          const int dc = lev < 1 ? 1 : (lev > 254 ? 254 : lev);
          put_bits(seg, b0, Code{(uint32_t)(dc == 128 ? 255 : dc), 8});
        }
        const int pre = wave_excl_scan(lc.len, lane);
        put_bits(seg, b0 + dcbits + pre, lc);
        const int tot = __shfl(pre + lc.len, 63);
        if (lane == 0) put_bits(seg, b0 + dcbits + tot, tab(T, T_EOB));
        bits += dcbits + tot + 2;
      } else {
        bits += dcbits + wave_sum_i(lc.len) + 2;
      }
    }
  }
  return bits;
}

template <bool EMIT>
__global__ __launch_bounds__(64 * VLC_WAVES) void k_vlc_mb(VlcArgs a, VlcTables Tg) {
  __shared__ VlcTables T;  // per-lane table lookups from LDS, loaded once per workgroup
  __shared__ uint32_t segs[VLC_WAVES][SEG_WORDS + 2];
  for (int i = threadIdx.x; i < T_N; i += 64 * VLC_WAVES) T.t[i] = Tg.t[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fi = blockIdx.y;
  const int j0 = (blockIdx.x * VLC_WAVES + wv) * VLC_MBS;
  uint32_t *seg = segs[wv];
  const size_t base = (size_t)fi * a.nmb;
  if (EMIT && a.bits[fi] == 0xFFFFFFFFu) return;  // invalid record or no room: nothing written
  uint32_t *out = a.out + (size_t)fi * a.out_words;
  for (int j = j0; j < min(j0 + VLC_MBS, a.nmb); j++) {
    if (EMIT)
      for (int i = lane; i < SEG_WORDS + 2; i += 64) seg[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    int64_t s0 = 0;
    const int bits = code_mb<EMIT>(T, a, fi, j, lane, seg, &s0);
    if (!EMIT) {
      if (lane == 0) a.mb_bits[base + j] = bits < 0 ? 0x80000000u : (uint32_t)bits;
      continue;
    }
    // copy the segment out: words strictly inside it are this wave's alone; the
    // first and last word are shared with the neighbouring segments
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int64_t w0 = s0 >> 5, w1 = ((int64_t)a.mb_off[base + j] + bits - 1) >> 5;
    for (int64_t w = w0 + lane; w <= w1; w += 64) {
      const uint32_t v = seg[w - w0];
      if (w == w0 || w == w1)
        atomicOr(out + w, v);
      else
        out[w] = v;
    }
  }
}

// stream-order offsets per picture (one wave per picture: each lane sums a
// run of MBs, a wave scan combines them); bits[fi] = total incl. the phase,
// or 0xFFFFFFFF if a record was invalid.  Zeroes the words the picture uses.
__global__ __launch_bounds__(64) void k_vlc_scan(VlcArgs a) {
  const int fi = blockIdx.x, lane = threadIdx.x;
  const size_t base = (size_t)fi * a.nmb;
  const int per = (a.nmb + 63) / 64, j0 = lane * per, j1 = min(j0 + per, a.nmb);
  int sum = 0, bad = 0;
  for (int j = j0; j < j1; j++) {
    const uint32_t b = a.mb_bits[base + j];
    bad |= (b >> 31) & 1;
    sum += (int)(b & 0x7fffffffu) + (j % 33 == 0 ? 26 : 0);  // GOB header before MDU 0
  }
  const int head = (a.phase ? a.phase[fi] : 0) + 32 + (a.format == P64S_NTSC ? 9 : 0);
  int64_t off = head + wave_excl_scan(sum, lane);
  for (int j = j0; j < j1; j++) {
    if (j % 33 == 0) off += 26;
    a.mb_off[base + j] = (uint32_t)off;
    off += a.mb_bits[base + j] & 0x7fffffffu;
  }
  const int64_t total = __shfl(off, 63);
  bad = __any(bad);
  const bool fits = total + 64 <= a.out_words * 32;
  if (lane == 0) a.bits[fi] = (bad || !fits) ? 0xFFFFFFFFu : (uint32_t)total;
  if (fits) {
    uint32_t *out = a.out + (size_t)fi * a.out_words;
    for (int64_t w = lane; w <= (total >> 5) + 1; w += 64) out[w] = 0;
  }
}

thread_local VlcTables g_tab;
thread_local bool g_tab_ok = false;

}  // namespace

extern "C" {

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
  if (x->out_stride < p64gpu_vlc_max_bytes(x->width, x->height) || (x->out_stride & 3) ||
      ((uintptr_t)x->out & 3))
    return p64gpu_fail_(P64GPU_E_INVALID, "vlc: out_stride below p64gpu_vlc_max_bytes or not 4-aligned");
  if (!g_tab_ok) {
    const int s = p64s_vlc_tables_(g_tab.t);
    if (s) return s;
    g_tab_ok = true;
  }
  VlcArgs a;
  a.width = x->width;
  a.height = x->height;
  a.nframes = x->nframes;
  a.format = fmt;
  p64s_geometry(fmt, nullptr, nullptr, &a.ngob);
  a.nmb = a.ngob * 33;
  a.mb = x->mb;
  a.coef = x->coef;
  a.gquant = x->gquant;
  a.mquant = x->mquant;
  a.tr = x->tr;
  a.phase = x->phase;
  a.out = reinterpret_cast<uint32_t *>(x->out);
  a.out_words = x->out_stride / 4;
  a.bits = x->bits;
  a.mb_bits = x->scratch;
  a.mb_off = x->scratch + (size_t)x->nframes * a.nmb;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((a.nmb + VLC_WAVES * VLC_MBS - 1) / (VLC_WAVES * VLC_MBS)),
                  (unsigned)a.nframes);
  hipLaunchKernelGGL(k_vlc_mb<false>, grid, dim3(64 * VLC_WAVES), 0, st, a, g_tab);
  hipLaunchKernelGGL(k_vlc_scan, dim3((unsigned)a.nframes), dim3(64), 0, st, a);
  hipLaunchKernelGGL(k_vlc_mb<true>, grid, dim3(64 * VLC_WAVES), 0, st, a, g_tab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return p64gpu_fail_(P64GPU_E_HIP, hipGetErrorString(e));
  return P64GPU_OK;
}

}  // extern "C"
