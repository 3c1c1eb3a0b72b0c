// Repro: clamp((x +- 8) / 16, 0, 255) of 8 values packed into two dwords.
// hipcc (ROCm 7.2, gfx950) selects v_ashr_pk_u8_i32 for byte pairs and then
// v_or3_b32 with the other bytes; compare against the host result.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const int* in, uint2* out) {
  int t = threadIdx.x;
  int v[8];
  for (int k = 0; k < 8; k++) {
    int x = in[t * 8 + k];
    x = (x < 0 ? x - 8 : x + 8) / 16;
    v[k] = min(max(x, 0), 255);
  }
  uint2 q;
  q.x = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
  q.y = (uint32_t)v[4] | ((uint32_t)v[5] << 8) | ((uint32_t)v[6] << 16) | ((uint32_t)v[7] << 24);
  out[t] = q;
}
int main() {
  const int n = 256;
  int h[n * 8];
  for (int i = 0; i < n * 8; i++) h[i] = (int)((i * 2654435761u) % 6000) - 1000;
  int* d; uint2* o; uint2 r[n];
  (void)hipMalloc(&d, sizeof h); (void)hipMalloc(&o, sizeof r);
  (void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  k<<<1, n>>>(d, o);
  (void)hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int t = 0; t < n; t++) {
    uint32_t e[2] = {0, 0};
    for (int k = 0; k < 8; k++) {
      int x = h[t * 8 + k];
      x = (x < 0 ? x - 8 : x + 8) / 16;
      x = x < 0 ? 0 : (x > 255 ? 255 : x);
      e[k / 4] |= (uint32_t)x << (8 * (k % 4));
    }
    if (e[0] != r[t].x || e[1] != r[t].y) {
      if (bad < 4) printf("lane %d: got %08x %08x want %08x %08x\n", t, r[t].x, r[t].y, e[0], e[1]);
      bad++;
    }
  }
  printf("ashr_pk repro: %d of %d lanes wrong\n", bad, n);
  return 0;
}
