// k_aux.hip -- batched reference block routines (one thread per 8x8 block,
// full 32-bit arithmetic for arbitrary int32 input: the p64gpu_block_op API)
// and the device generator of the synthetic pictures.

#include "common.h"
#include "launch.h"

#define SYNTH_FN __host__ __device__ static inline
#include "synth_impl.h"

namespace {

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

// the SURVEY.md 8(d) content (synth_impl.h p64v_*), same layout as k_synth;
// a chroma sample recomputes its four luma samples (same bytes as synth.c,
// which averages the stored luma plane)
__global__ __launch_bounds__(256) void k_synth_survey(int w, int h, uint32_t seed0, int nseeds, int frame0,
                                                      int64_t stride, uint8_t *out) {
  const int pic = blockIdx.y;
  const int t = pic / nseeds, sidx = pic - t * nseeds;
  const uint32_t seed = seed0 + (uint32_t)sidx;
  const int frame = frame0 + t;
  uint8_t *y = out + (size_t)pic * stride;
  uint8_t *u = y + (size_t)w * h, *v = u + (size_t)(w / 2) * (h / 2);
  const int nl = w * h, nc = (w / 2) * (h / 2);
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < nl + nc; k += gridDim.x * blockDim.x) {
    if (k < nl) {
      y[k] = p64v_luma(seed, frame, k % w, k / w);
    } else {
      const int c = k - nl, i = c % (w / 2), j = c / (w / 2);
      const int a4 = p64v_luma(seed, frame, 2 * i, 2 * j) + p64v_luma(seed, frame, 2 * i + 1, 2 * j) +
                     p64v_luma(seed, frame, 2 * i, 2 * j + 1) + p64v_luma(seed, frame, 2 * i + 1, 2 * j + 1);
      p64v_chroma_of(a4, &u[c], &v[c]);
    }
  }
}

// Clock probe and spin-up (measurement aid, bench.py): every wave issues
// chains of v_sad_u8 -- k_motion's dominant instruction -- until `ticks` of
// the 100 MHz real-time counter have passed, then records how many shader
// clock ticks (s_memtime) and real-time ticks the span took: the clock the
// chip held over the span is their ratio x 100 MHz.  A short probe right
// after a timed region reads the clock the workload left the chip at (the
// chip ramps its clocks over tens of ms of load, and this dense v_sad_u8
// load itself holds a lower clock than the search kernels do).
// out: [waves][2] (shader ticks, real-time ticks), vector stores only.
__global__ __launch_bounds__(256) void k_clock(uint32_t ticks, uint32_t *out) {
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  uint32_t a0 = threadIdx.x * 0x01010101u, a1 = a0 ^ 0x5a5a5a5au, a2 = a0 + 0x10203040u, a3 = ~a0;
  const uint32_t b = blockIdx.x * 0x9e3779b1u;
  uint64_t r = r0;
  while ((uint32_t)(r - r0) < ticks) {  // uniform: a scalar loop
#pragma unroll
    for (int i = 0; i < 32; i++) {  // four independent chains
      a0 = sad4(a0, b, a0);
      a1 = sad4(a1, b, a1);
      a2 = sad4(a2, b, a2);
      a3 = sad4(a3, b, a3);
    }
    r = __builtin_amdgcn_s_memrealtime();
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const unsigned wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    out[2 * wave] = (uint32_t)(c1 - c0);
    // the chains' results decide nothing but must not be optimised away: a
    // real-time count of 0 is impossible, so the OR below never changes it
    out[2 * wave + 1] = (uint32_t)(r - r0) | ((a0 ^ a1 ^ a2 ^ a3) == 0x7fffffffu && r == r0 ? 1u : 0u);
  }
}

}  // namespace

namespace p64k {

unsigned clock_waves() { return 2048u * 4u; }

hipError_t clock(uint32_t ticks, uint32_t *out, hipStream_t st) {
  hipLaunchKernelGGL(k_clock, dim3(2048), dim3(256), 0, st, ticks, out);
  return hipGetLastError();
}


hipError_t block_op(int op, const int32_t *in, int32_t *out, int64_t nblocks, int dcq, int acq,
                    hipStream_t st) {
  const int threads = 64;
  const int64_t grid = (nblocks + threads - 1) / threads;
  hipLaunchKernelGGL(k_block_op, dim3((unsigned)grid), dim3(threads), 0, st, op, in, out, nblocks, dcq, acq);
  return hipGetLastError();
}

hipError_t synth(int content, int w, int h, uint32_t seed0, int nseeds, int frame0, int nslots, int64_t stride,
                 uint8_t *out, hipStream_t st) {
  if (content == P64_SYNTH_SURVEY)
    hipLaunchKernelGGL(k_synth_survey, dim3(64, (unsigned)(nseeds * nslots)), dim3(256), 0, st, w, h, seed0,
                       nseeds, frame0, stride, out);
  else
    hipLaunchKernelGGL(k_synth, dim3(64, (unsigned)(nseeds * nslots)), dim3(256), 0, st, w, h, seed0, nseeds,
                       frame0, stride, out);
  return hipGetLastError();
}

}  // namespace p64k
