// Probe: v_lerp_u8 (__builtin_amdgcn_lerp) with a zero rounding operand is the
// bytewise floor average (a+b)>>1 (the lower-bound map of the FULL search relies on it).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t* a, const uint32_t* b, uint32_t* o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = __builtin_amdgcn_lerp(a[i], b[i], 0u);
}
int main() {
  const int n = 1 << 20;
  static uint32_t a[n], b[n], o[n];
  uint32_t *da, *db, *dout;
  if (hipMalloc(&da, n * 4) || hipMalloc(&db, n * 4) || hipMalloc(&dout, n * 4)) return 2;
  uint32_t s = 12345;
  for (int i = 0; i < n; i++) { s = s * 1664525u + 1013904223u; a[i] = s; s = s * 1664525u + 1013904223u; b[i] = s; }
  a[0] = 0xFFFFFFFF; b[0] = 0xFFFFFFFF; a[1] = 0x01FF00FE; b[1] = 0x00FE01FF;
  if (hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice) || hipMemcpy(db, b, n * 4, hipMemcpyHostToDevice)) return 2;
  k<<<n / 256, 256>>>(da, db, dout, n);
  if (hipMemcpy(o, dout, n * 4, hipMemcpyDeviceToHost)) return 2;
  long bad = 0;
  for (int i = 0; i < n; i++) {
    uint32_t e = 0;
    for (int k2 = 0; k2 < 4; k2++) e |= ((((a[i] >> (8 * k2)) & 255) + ((b[i] >> (8 * k2)) & 255)) >> 1) << (8 * k2);
    if (e != o[i]) { if (bad < 5) printf("mismatch %08x %08x -> %08x want %08x\n", a[i], b[i], o[i], e); bad++; }
  }
  printf("lerp floor-average check: %ld mismatches of %d\n", bad, n);
  return bad != 0;
}
