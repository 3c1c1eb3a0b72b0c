// HBM calibration for the intra/decode rooflines (development aid, gfx950):
// achievable bandwidth of streaming 16-B-per-lane reads, writes and mixes in
// the read:write ratios of the HBM-bound kernels (intra 1:3, decode ~3:2),
// and of 8-B-per-lane rows (the block-layout pixel rows).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// R uint4 reads and W uint4 writes per "unit"; grid-stride over units
template <int R, int W, int WIDTH>
__global__ __launch_bounds__(256) void k_mix(const uint4* __restrict__ in, uint4* __restrict__ out,
                                             size_t units, uint32_t salt) {
  const size_t n = (size_t)gridDim.x * blockDim.x;
  for (size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += n) {
    uint32_t acc = salt;
    if (WIDTH == 16) {
#pragma unroll
      for (int r = 0; r < R; r++) {
        const uint4 v = in[(size_t)r * units + u];
        acc += v.x ^ v.y ^ v.z ^ v.w;
      }
#pragma unroll
      for (int w = 0; w < W; w++) out[(size_t)w * units + u] = make_uint4(acc, acc + w, u, salt);
    } else {  // 8-byte lanes
      const uint2* in2 = reinterpret_cast<const uint2*>(in);
      uint2* out2 = reinterpret_cast<uint2*>(out);
#pragma unroll
      for (int r = 0; r < 2 * R; r++) {
        const uint2 v = in2[(size_t)r * units + u];
        acc += v.x ^ v.y;
      }
#pragma unroll
      for (int w = 0; w < 2 * W; w++) out2[(size_t)w * units + u] = make_uint2(acc + w, u);
    }
  }
}

template <int R, int W, int WIDTH>
void run(const char* name, uint4* in, uint4* out, size_t bytes_each) {
  const size_t units = bytes_each / 16 / (R > W ? R : W);
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  for (int wg_per_cu : {4, 8, 16, 0}) {
    const unsigned grid = wg_per_cu ? cus * wg_per_cu : (unsigned)((units + 255) / 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9;
    for (int rep = 0; rep < 6; rep++) {
      (void)hipEventRecord(e0);
      k_mix<R, W, WIDTH><<<grid, 256>>>(in, out, units, rep);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    const double rb = (double)units * 16 * R, wb = (double)units * 16 * W;
    printf("%-28s wg/cu %-4d %8.1f us  read %6.2f TB/s  write %6.2f TB/s  total %6.2f TB/s\n", name,
           wg_per_cu, best * 1e3, rb / best / 1e9, wb / best / 1e9, (rb + wb) / best / 1e9);
  }
}

int main() {
  const size_t bytes = (size_t)1 << 30;  // 1 GiB per stream (well past the 256 MB MALL)
  uint4 *in, *out;
  if (hipMalloc(&in, 4 * bytes) != hipSuccess || hipMalloc(&out, 4 * bytes) != hipSuccess) return 1;
  (void)hipMemset(in, 1, 4 * bytes);
  (void)hipMemset(out, 0, 4 * bytes);
  run<1, 0, 16>("read 16B/lane", in, out, bytes);
  run<0, 1, 16>("write 16B/lane", in, out, bytes);
  run<1, 1, 16>("copy 1:1 16B/lane", in, out, bytes);
  run<1, 3, 16>("1 read : 3 write 16B", in, out, bytes);
  run<3, 2, 16>("3 read : 2 write 16B", in, out, bytes);
  run<1, 1, 8>("copy 1:1 8B/lane", in, out, bytes);
  run<1, 3, 8>("1 read : 3 write 8B", in, out, bytes);
  return 0;
}
