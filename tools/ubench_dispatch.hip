// Microbenchmark: what does launching 101,376 one-wave workgroups cost on its
// own (the fused encode kernel's grid), against the same waves packed four to
// a workgroup, and against a grid-stride loop over fewer workgroups?
// Each wave does a token amount of work: 5 KB of static LDS declared, one LDS
// round trip, one 4-byte store.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int NMB = 101376;
constexpr int LDS_WORDS = 1272;  // ~5 KB per wave, as k_encode

__device__ __forceinline__ void work(const uint4 *in, uint4 *out, uint32_t *L, unsigned mb, int lane) {
  // token work: one LDS round trip, one 4-byte store per lane for lane 0 only
  L[lane] = mb + lane;
  __builtin_amdgcn_wave_barrier();
  const uint32_t v = L[(lane + 1) & 63];
  if (lane == 0) reinterpret_cast<uint32_t *>(out)[mb] = v ^ (uint32_t)(uintptr_t)in;
}

__global__ __launch_bounds__(64) void k_wave(const uint4 *in, uint4 *out) {
  __shared__ uint32_t L[LDS_WORDS];
  work(in, out, L, blockIdx.x, threadIdx.x);
}

__global__ __launch_bounds__(256) void k_wg4(const uint4 *in, uint4 *out) {
  __shared__ uint32_t L[4][LDS_WORDS];
  const int wv = threadIdx.x >> 6;
  work(in, out, L[wv], blockIdx.x * 4 + wv, threadIdx.x & 63);
}

__global__ __launch_bounds__(64) void k_loop(const uint4 *in, uint4 *out, int per) {
  __shared__ uint32_t L[LDS_WORDS];
  for (int i = 0; i < per; i++) {
    const unsigned mb = blockIdx.x + i * gridDim.x;
    if (mb < NMB) work(in, out, L, mb, threadIdx.x);
  }
}

int main() {
  uint4 *in, *out;
  CK(hipMalloc(&in, (size_t)NMB * 64 * 16));
  CK(hipMalloc(&out, (size_t)NMB * 64 * 16));
  CK(hipMemset(in, 1, (size_t)NMB * 64 * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char *name, auto launch) {
    for (int i = 0; i < 3; i++) launch();
    hipDeviceSynchronize();
    const int reps = 20;
    hipEventRecord(a);
    for (int i = 0; i < reps; i++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.1f us/launch\n", name, ms * 1e3f / reps);
  };
  run("1 wave x 101376 WGs", [&] { k_wave<<<NMB, 64>>>(in, out); });
  run("4 waves x 25344 WGs", [&] { k_wg4<<<NMB / 4, 256>>>(in, out); });
  for (int per : {2, 4, 8, 16, 32}) {
    char nm[64];
    snprintf(nm, sizeof nm, "loop %2d MB/WG (%d WGs)", per, (NMB + per - 1) / per);
    run(nm, [&] { k_loop<<<(NMB + per - 1) / per, 64>>>(in, out, per); });
  }
  return 0;
}
