// Does gfx950 serve byte-unaligned ds_read_b32 correctly, and at what rate?
// Variant U: 4 unaligned ds_read_b32 per row; variant A: 5 aligned + 4 v_alignbyte.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
typedef uint32_t __attribute__((aligned(1))) u32u;

template <int V>
__global__ __launch_bounds__(256) void k(const uint32_t* win_g, int iters, uint32_t* out, uint32_t* probe) {
  __shared__ uint32_t win[4][48 * 12 + 16];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int t = lane; t < 48 * 12; t += 64) win[wv][t] = win_g[t];
  __syncthreads();
  const int colb = (lane % 30) + 1, sh = colb & 3;
  const uint8_t* wb = (const uint8_t*)win[wv];
  uint32_t c0 = __builtin_amdgcn_readfirstlane(win_g[5]), c1 = __builtin_amdgcn_readfirstlane(win_g[6]);
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 30; i++) {
      uint32_t r0, r1, r2, r3;
      if (V == 0) {
        const uint8_t* p = wb + (i + (it & 7)) * 48 + colb;
        r0 = *(const u32u*)(p); r1 = *(const u32u*)(p + 4); r2 = *(const u32u*)(p + 8); r3 = *(const u32u*)(p + 12);
      } else {
        const uint32_t* p = win[wv] + (i + (it & 7)) * 12 + (colb >> 2);
        uint32_t a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3], a4 = p[4];
        r0 = __builtin_amdgcn_alignbyte(a1, a0, sh); r1 = __builtin_amdgcn_alignbyte(a2, a1, sh);
        r2 = __builtin_amdgcn_alignbyte(a3, a2, sh); r3 = __builtin_amdgcn_alignbyte(a4, a3, sh);
      }
      if (it == 0 && i == 0 && blockIdx.x == 0 && wv == 0) {
        probe[lane * 4 + 0] = r0; probe[lane * 4 + 1] = r1; probe[lane * 4 + 2] = r2; probe[lane * 4 + 3] = r3;
      }
#pragma unroll
      for (int r = 0; r < 8; r++) {
        acc = __builtin_amdgcn_sad_u8(r0, c0 + r, acc);
        acc = __builtin_amdgcn_sad_u8(r1, c1 + r, acc);
        acc = __builtin_amdgcn_sad_u8(r2, c0 ^ r, acc);
        acc = __builtin_amdgcn_sad_u8(r3, c1 ^ r, acc);
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  uint32_t h[48 * 12];
  for (int i = 0; i < 48 * 12; i++) h[i] = i * 2654435761u;
  uint32_t *d, *o, *pr;
  (void)hipMalloc(&d, sizeof h); (void)hipMalloc(&o, 4096 * 256 * 4); (void)hipMalloc(&pr, 64 * 4 * 4);
  (void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  const uint8_t* hb = (const uint8_t*)h;
  for (int v = 0; v < 2; v++) {
    float best = 1e9;
    for (int rep = 0; rep < 4; rep++) {
      hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      if (v == 0) k<0><<<4096, 256>>>(d, 40, o, pr); else k<1><<<4096, 256>>>(d, 40, o, pr);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    uint32_t p[256];
    (void)hipMemcpy(p, pr, sizeof p, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int lane = 0; lane < 64; lane++) {
      int colb = (lane % 30) + 1;
      for (int k2 = 0; k2 < 4; k2++) {
        uint32_t e; memcpy(&e, hb + colb + 4 * k2, 4);
        if (p[lane * 4 + k2] != e) bad++;
      }
    }
    printf("%s: %.3f ms, %d/256 probe words wrong\n", v == 0 ? "unaligned ds_read_b32" : "aligned + alignbyte", best, bad);
  }
  return 0;
}
