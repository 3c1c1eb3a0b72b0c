"""Counted side build of k_search.hip (development aid, never shipped):
writes abtest/k_search_sadcount.hip, whose every v_sad_u8 (sad4) and
v_sad_hi_u8 (the bound pass's high halves) also adds 1
to a per-lane counter in device memory, so a launch's executed v_sad_u8
work (lane-instructions x 4 byte-absolute-differences) can be read back by
p64dbg_sadcnt_read().  Control flow is data-dependent only, so the counts are
the product kernel's.  Build with
  python tools/sad_count.py && tools/ablib.sh sadcount abtest/k_search_sadcount.hip k_search
and run tools/sad_count_run.py on the GPU box (P64GPU_LIB=abtest/lib_sadcount.so)."""
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(REPO, "p64_amd/csrc/k_search.hip")).read()
n = s.count("sad4(")
assert n > 10, n
s = s.replace("sad4(", "sad4c(")
# the bound pass's high-half SADs (v_sad_hi_u8: the same 4 byte-absolute-differences)
s = s.replace("__builtin_amdgcn_sad_hi_u8(", "sad4hic(")
s = s.replace("namespace {\n", """namespace {
// one counter per lane of the launch (grid < 131072 one-wave workgroups)
__device__ unsigned g_sadcnt[1u << 23];
__device__ __forceinline__ uint32_t sad4c(uint32_t a, uint32_t b, uint32_t acc) {
  g_sadcnt[blockIdx.x * 64u + (threadIdx.x & 63u)] += 1u;
  return __builtin_amdgcn_sad_u8(a, b, acc);
}
__device__ __forceinline__ uint32_t sad4hic(uint32_t a, uint32_t b, uint32_t acc) {
  g_sadcnt[blockIdx.x * 64u + (threadIdx.x & 63u)] += 1u;
  return __builtin_amdgcn_sad_hi_u8(a, b, acc);
}
""", 1)
s += """
extern "C" int p64dbg_sadcnt_read(unsigned *host, size_t n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sadcnt), n * 4);
}
extern "C" int p64dbg_sadcnt_clear(void) {
  void *p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_sadcnt)) != hipSuccess) return -1;
  return (int)hipMemset(p, 0, sizeof(unsigned) << 23);
}
"""
os.makedirs(os.path.join(REPO, "abtest"), exist_ok=True)
open(os.path.join(REPO, "abtest", "k_search_sadcount.hip"), "w").write(s)
print("abtest/k_search_sadcount.hip", n, "call sites")
