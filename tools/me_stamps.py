"""Per-wave timeline of k_motion<2> (development aid, never shipped): writes
abtest/k_search_stamp.hip, whose k_motion stamps s_memrealtime at wave start
(T0), once the window is in LDS (T1), after the search + statistics (T2) and
after the record store completed (T3).  Build with tools/ablib.sh mestamp
abtest/k_search_stamp.hip k_search; run tools/me_timeline.py on the GPU box."""
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(REPO, "p64_amd/csrc/k_search.hip")).read()


def sub(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)


sub("namespace {\n", """namespace {
__device__ unsigned long long g_stamp[4u << 17];
#define STAMP(k)                                                                              \\
  do {                                                                                        \\
    if (threadIdx.x == 0) g_stamp[4u * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime(); \\
  } while (0)
""")
sub("""  const MbPos ps = mb_pos(gid, nmb, mbw, kd);
  const int fi = ps.fi, x0 = 16 * ps.mbx, y0 = 16 * ps.mby;
  put_luma(L,""", """  STAMP(0);
  const MbPos ps = mb_pos(gid, nmb, mbw, kd);
  const int fi = ps.fi, x0 = 16 * ps.mbx, y0 = 16 * ps.mby;
  put_luma(L,""")
sub("""  SECTION("m_fetched");""", """  __builtin_amdgcn_s_waitcnt(0);
  STAMP(1);
  SECTION("m_fetched");""")
sub("""  SECTION("m_me_done");
  if (lane == 0) {""", """  SECTION("m_me_done");
  STAMP(2);
  if (lane == 0) {""")
sub("""    out[gid] = o;
  }
}""", """    out[gid] = o;
  }
  __builtin_amdgcn_s_waitcnt(0);
  STAMP(3);
}""")
s += """
extern "C" int p64dbg_stamps(unsigned long long *host, size_t n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamp), n * 8);
}
extern "C" int p64dbg_stamps_clear(void) {
  static unsigned long long z[4u << 17];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof z);
}
"""
open(os.path.join(REPO, "abtest", "k_search_stamp.hip"), "w").write(s)
print("abtest/k_search_stamp.hip")
