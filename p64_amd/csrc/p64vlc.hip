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
//                   at its absolute bit offset (wave prefix sum of lengths) with
//                   32-bit atomic ORs into a zeroed, byte-ordered buffer.
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

// the macroblock header codes (WriteMBHeader marker.c:288-357), in order;
// returns the count (<= 6): MBA, MTYPE, [MQUANT], [MVDH, MVDV], [CBP]
__device__ int header_codes(const VlcTables &T, const VlcArgs &a, int fi, int g, int m, Code *c,
                            bool *bad) {
  const size_t base = (size_t)fi * a.nmb;
  const int k = raster(a.format, g, m);
  const p64_mb_rec r = a.mb[base + k];
  const int mt = r.mtype;
  int n = 0;
  if (mt < 0 || mt > 9 || (mt_cbp(mt) && (r.cbp < 1 || r.cbp > 63))) {
    *bad = true;
    return 0;
  }
  c[n++] = Code{1u, 1};  // MBA = 1: every MDU is coded (p64.c:922)
  c[n++] = tab(T, T_MTYPE + mt);
  if (mt_quant(mt)) c[n++] = Code{a.mquant ? (uint32_t)(a.mquant[base + k] & 31) : 0u, 5};
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
    c[n++] = tab(T, T_MVD + (dh & 31));
    c[n++] = tab(T, T_MVD + (dv & 31));
  }
  if (mt_cbp(mt)) c[n++] = tab(T, T_CBP + r.cbp);
  return n;
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

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s);
  return v;
}
__device__ __forceinline__ int wave_excl_scan(int v, int lane) {
  int x = v;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const int y = __shfl_up(x, s);
    if (lane >= s) x += y;
  }
  return x - v;
}

// bits of `c` at absolute bit position `pos` of the picture's buffer (MSB-first
// bytes, little-endian words: bswap per word)
__device__ __forceinline__ void put_bits(uint32_t *out, int64_t pos, Code c) {
  if (!c.len) return;
  const int64_t w = pos >> 5;
  const int sh = (int)(pos & 31);
  const uint64_t x = (uint64_t)c.v << (64 - c.len - sh);  // big-endian within 64 bits
  const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
  if (hi) atomicOr(out + w, __builtin_bswap32(hi));
  if (lo) atomicOr(out + w + 1, __builtin_bswap32(lo));
}

template <bool EMIT>
__global__ __launch_bounds__(64) void k_vlc_mb(VlcArgs a, VlcTables T) {
  const int lane = threadIdx.x;
  const int fi = blockIdx.y, j = blockIdx.x;  // j = g*33 + m, stream order
  const int g = j / 33, m = j - g * 33;
  const size_t base = (size_t)fi * a.nmb;
  const int k = raster(a.format, g, m);
  const p64_mb_rec r = a.mb[base + k];
  Code hc[6];
  bool bad = false;
  const int nh = header_codes(T, a, fi, g, m, hc, &bad);
  if (bad) {
    if (!EMIT && lane == 0) a.mb_bits[base + j] = 0x80000000u;
    return;
  }
  int hbits = 0;
  for (int i = 0; i < nh; i++) hbits += hc[i].len;
  const int mt = r.mtype;
  const bool cbpt = mt_cbp(mt);
  const int cbp = cbpt ? r.cbp : 0x3f;
  int64_t pos = 0;
  if (EMIT) {
    pos = a.mb_off[base + j];
    uint32_t *out = a.out + (size_t)fi * a.out_words;
    if (lane == 0) {
      if (j == 0) {  // picture header (WritePictureHeader marker.c:103-135)
        const int64_t p0 = a.phase ? a.phase[fi] : 0;
        put_bits(out, p0, Code{0x10u, 20});
        put_bits(out, p0 + 20, Code{(uint32_t)a.tr[fi] & 31u, 5});
        put_bits(out, p0 + 25, Code{a.format == P64S_QCIF ? 0u : 4u, 6});
        if (a.format == P64S_NTSC) put_bits(out, p0 + 31, Code{0x18cu, 9});  // PSPARE 0x8c
      }
      if (m == 0) {  // GOB header (WriteGOBHeader marker.c:171-198)
        const uint32_t gn = a.format == P64S_QCIF ? 2 * g + 1 : g + 1;
        const uint32_t gq = a.gquant[(size_t)fi * a.ngob + g] & 31u;
        put_bits(out, pos - 26, Code{(1u << 10) | (gn << 6) | (gq << 1), 26});
      }
      int64_t p = pos;
      for (int i = 0; i < nh; i++) {
        put_bits(out, p, hc[i]);
        p += hc[i].len;
      }
    }
  }
  int bits = hbits;
  if (mt_tc(mt)) {
    for (int c = 0; c < 6; c++) {
      if (!((cbp >> (5 - c)) & 1)) continue;
      const int lev = a.coef[(base + k) * 384 + c * 64 + lane];
      const uint64_t nz = __ballot(lev != 0 && (cbpt || lane > 0));
      if (cbpt && !nz) continue;  // CBPEncodeAC: no level, nothing written
      const Code lc = level_code(T, lane, lev, nz, cbpt);
      const int dcbits = cbpt ? 0 : 8;
      if (EMIT) {
        uint32_t *out = a.out + (size_t)fi * a.out_words;
        const int64_t b0 = pos + bits;
        if (!cbpt && lane == 0) {  // EncodeDC codec.c:343-352
          int dc = lev < 1 ? 1 : (lev > 254 ? 254 : lev);
          put_bits(out, b0, Code{(uint32_t)(dc == 128 ? 255 : dc), 8});
        }
        const int off = wave_excl_scan(lc.len, lane);
        put_bits(out, b0 + dcbits + off, lc);
        const int tot = __shfl(off + lc.len, 63);
        if (lane == 0) put_bits(out, b0 + dcbits + tot, tab(T, T_EOB));
        bits += dcbits + tot + 2;
      } else {
        bits += dcbits + wave_sum_i(lc.len) + 2;
      }
    }
  }
  if (!EMIT && lane == 0) a.mb_bits[base + j] = (uint32_t)bits;
}

// stream-order offsets per picture; bits[fi] = total incl. the phase, or
// 0xFFFFFFFF if a record was invalid
__global__ void k_vlc_scan(VlcArgs a) {
  const int fi = blockIdx.x * blockDim.x + threadIdx.x;
  if (fi >= a.nframes) return;
  const size_t base = (size_t)fi * a.nmb;
  int64_t off = (a.phase ? a.phase[fi] : 0) + 32 + (a.format == P64S_NTSC ? 9 : 0);
  bool bad = false;
  for (int g = 0; g < a.ngob; g++) {
    off += 26;
    for (int m = 0; m < 33; m++) {
      const uint32_t b = a.mb_bits[base + g * 33 + m];
      bad |= (b & 0x80000000u) != 0;
      a.mb_off[base + g * 33 + m] = (uint32_t)off;
      off += b & 0x7fffffffu;
    }
  }
  a.bits[fi] = (bad || off > a.out_words * 32 - 64) ? 0xFFFFFFFFu : (uint32_t)off;
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
  hipError_t e = hipMemsetAsync(x->out, 0, (size_t)x->nframes * x->out_stride, st);
  if (e != hipSuccess) return p64gpu_fail_(P64GPU_E_HIP, hipGetErrorString(e));
  const dim3 grid((unsigned)a.nmb, (unsigned)a.nframes);
  hipLaunchKernelGGL(k_vlc_mb<false>, grid, dim3(64), 0, st, a, g_tab);
  hipLaunchKernelGGL(k_vlc_scan, dim3((unsigned)((a.nframes + 63) / 64)), dim3(64), 0, st, a);
  hipLaunchKernelGGL(k_vlc_mb<true>, grid, dim3(64), 0, st, a, g_tab);
  e = hipGetLastError();
  if (e != hipSuccess) return p64gpu_fail_(P64GPU_E_HIP, hipGetErrorString(e));
  return P64GPU_OK;
}

}  // extern "C"
