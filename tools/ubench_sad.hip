// Microbenchmark + semantics probe: v_sad_u8 vs v_qsad_pk_u16_u8 (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

__global__ void k_sem(const uint64_t* a, const uint32_t* b, const uint64_t* c, uint64_t* o, uint32_t* o2) {
  int i = threadIdx.x;
  o[i] = __builtin_amdgcn_qsad_pk_u16_u8(a[i], b[i], c[i]);
  o2[i] = __builtin_amdgcn_sad_u8((uint32_t)a[i], b[i], (uint32_t)c[i]);
}

template <int KIND>
__global__ __launch_bounds__(256) void k_rate(uint32_t seed, int iters, uint32_t* out) {
  // operands live in registers; the loop body is nothing but the SAD
  // instructions (8 independent accumulator chains, SGPR current operand)
  uint32_t s0 = __builtin_amdgcn_readfirstlane(seed * 7 + blockIdx.x);
  uint32_t s1 = __builtin_amdgcn_readfirstlane(seed * 13 + 1);
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = (threadIdx.x + 37 * k) * 0x01010101u ^ (k * 0x1f2e3d4c);
  if (KIND == 0) {
    uint32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int u = 0; u < 8; u++)
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = __builtin_amdgcn_sad_u8(r[(u + k) & 7], (k & 1) ? s1 : s0, a[k]);
      asm volatile("" : "+v"(r[0]), "+v"(r[3]));
    }
    uint32_t t = 0;
    for (int k = 0; k < 8; k++) t += a[k];
    out[blockIdx.x * 256 + threadIdx.x] = t;
  } else {
    uint64_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t q[8];
#pragma unroll
    for (int k = 0; k < 8; k++) q[k] = ((uint64_t)r[(k + 1) & 7] << 32) | r[k];
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int u = 0; u < 8; u++)
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = __builtin_amdgcn_qsad_pk_u16_u8(q[(u + k) & 7], (k & 1) ? s1 : s0, a[k]);
      asm volatile("" : "+v"(q[0]), "+v"(q[3]));
    }
    uint64_t t = 0;
    for (int k = 0; k < 8; k++) t += a[k];
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)t ^ (uint32_t)(t >> 32);
  }
}

static int sad4(uint32_t a, uint32_t b) {
  int s = 0;
  for (int k = 0; k < 4; k++) s += abs((int)((a >> 8 * k) & 255) - (int)((b >> 8 * k) & 255));
  return s;
}

int main() {
  // semantics
  const int n = 256;
  std::vector<uint64_t> a(n), c(n), o(n);
  std::vector<uint32_t> b(n), o2(n);
  srand(1);
  for (int i = 0; i < n; i++) {
    a[i] = ((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 2) ^ rand();
    b[i] = (uint32_t)rand() * 2654435761u;
    c[i] = (i < 128) ? ((uint64_t)(rand() & 0x3fff) * 0x0001000100010001ull) : 0xfff0fff0fff0fff0ull;
  }
  uint64_t *da, *dc, *dout; uint32_t *db, *do2;
  hipMalloc(&da, n * 8); hipMalloc(&dc, n * 8); hipMalloc(&dout, n * 8); hipMalloc(&db, n * 4); hipMalloc(&do2, n * 4);
  hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dc, c.data(), n * 8, hipMemcpyHostToDevice);
  k_sem<<<1, n>>>(da, db, dc, dout, do2);
  hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(o2.data(), do2, n * 4, hipMemcpyDeviceToHost);
  int bad_lo = 0, bad_sat = 0, bad_wrap = 0, bad_sad = 0;
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < 4; j++) {
      uint32_t win = (uint32_t)(a[i] >> (8 * j));
      int s = sad4(win, b[i]);
      int acc = (int)((c[i] >> (16 * j)) & 0xffff);
      int got = (int)((o[i] >> (16 * j)) & 0xffff);
      int wrap = (acc + s) & 0xffff, sat = std::min(acc + s, 65535);
      if (got != wrap) bad_wrap++;
      if (got != sat) bad_sat++;
      if (i < 128 && got != acc + s) bad_lo++;
    }
    if (o2[i] != (uint32_t)(sad4((uint32_t)a[i], b[i]) + (uint32_t)c[i])) bad_sad++;
  }
  printf("qsad semantics (offsets 0..3 of S0, 16-bit acc): mismatches no-overflow=%d wrap=%d saturate=%d; sad_u8 mismatches=%d\n",
         bad_lo, bad_wrap, bad_sat, bad_sad);
  // rate
  uint32_t* dres; hipMalloc(&dres, 256 * 4096 * 4);
  int blocks = 256 * 16, iters = 2000;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int kind = 0; kind < 2; kind++) {
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      if (kind == 0) k_rate<0><<<blocks, 256>>>(1, iters, dres); else k_rate<1><<<blocks, 256>>>(1, iters, dres);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double winstr = (double)blocks * 4 * iters * 64;  // wave-instructions (4 waves/block, 64 per iter)
      double bad_per = kind == 0 ? 4 : 16;
      printf("%s: %.3f ms  %.3f Twave-instr/s  %.1f T byte-AD/s\n", kind == 0 ? "v_sad_u8" : "v_qsad_pk_u16_u8",
             ms, winstr / ms / 1e9, winstr * 64 * bad_per / ms / 1e9);
    }
  }
  return 0;
}
