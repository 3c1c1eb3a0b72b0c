"""Per-wave timeline of the entropy coder k_vlc_blk (development aid, never
shipped): writes p64_amd/csrc/_vlc_stamp.hip, a copy of p64vlc.hip whose
waves stamp s_memrealtime (100 MHz) at eight points -- start (with the wave's
XCD in bits 56..59), levels and records arrived, tables in LDS (barrier),
blocks counted, codes in the LDS copy, start known (barrier after the
look-back), words stored, end -- into a device array read back through
p64dbg_vlc_stamps(); builds abtest/lib_vlcstamp.so from it (the other objects
from the current build; extra hipcc flags from the command line, e.g.
-DVLC_STAGE_N=64).  Run tools/vlc_timeline.py on the GPU box."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(REPO, "p64_amd/csrc/p64vlc.hip")).read()


def sub(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


sub("namespace {\n", """namespace {
__device__ unsigned long long g_vstamp[8u << 16];
#define XCC_ID_REG ((3 << 11) | 20)
#define VSTAMP(k)                                                                                  \\
  do {                                                                                             \\
    const unsigned wid_ = (blockIdx.y * gridDim.x + blockIdx.x) * VLC_WAVES + (threadIdx.x >> 6);  \\
    if ((threadIdx.x & 63) == 0 && wid_ < (1u << 16))                                              \\
      g_vstamp[8u * wid_ + (k)] = __builtin_amdgcn_s_memrealtime() |                               \\
          ((k) == 0 ? (unsigned long long)__builtin_amdgcn_s_getreg(XCC_ID_REG) << 56 : 0ull);     \\
  } while (0)
#define WAIT_ALL() __builtin_amdgcn_s_waitcnt(0)
""")
sub("""  const VlcTables &Tg = d_tabs.t;
  const p64k::VlcLenTab &Lg = d_tabs.l;
  constexpr bool EMIT""", """  if (MODE == VLC_ONE) VSTAMP(0);
  const VlcTables &Tg = d_tabs.t;
  const p64k::VlcLenTab &Lg = d_tabs.l;
  constexpr bool EMIT""")
sub("""  for (int i = threadIdx.x; i < T_N; i += 64 * VLC_WAVES) T.t[i] = Tg.t[i];
  __syncthreads();""", """  for (int i = threadIdx.x; i < T_N; i += 64 * VLC_WAVES) T.t[i] = Tg.t[i];
  __syncthreads();
  if (MODE == VLC_ONE) VSTAMP(2);""")
sub("""  const bool narrow = !__any(coded && (wide & 0xff00ff00u));""",
    """  if (MODE == VLC_ONE) {
    WAIT_ALL();
    VSTAMP(1);
  }
  const bool narrow = !__any(coded && (wide & 0xff00ff00u));""")
sub("""  if (!EMIT) {
    if (act && VLC_OK""", """  if (MODE == VLC_ONE) VSTAMP(3);
  if (!EMIT) {
    if (act && VLC_OK""")
sub("""  // the start (wave 0): the phase for the first workgroup, else the end of the""",
    """  if (MODE == VLC_ONE) VSTAMP(4);
  // the start (wave 0): the phase for the first workgroup, else the end of the""")
sub("""  const int64_t first = s_first, endb = first + wt;""", """  if (MODE == VLC_ONE) VSTAMP(5);
  const int64_t first = s_first, endb = first + wt;""")
sub("""  if (wv != 0) return;
  // the shared words (wave 0)""", """  if (MODE == VLC_ONE) {
    WAIT_ALL();
    VSTAMP(6);
    if (wv != 0) VSTAMP(7);
  }
  if (wv != 0) return;
  // the shared words (wave 0)""")
# the end of wave 0: the last statement of the kernel body
i = s.index("// Every pointer of p64gpu_vlc_args must be memory")
j = s.rindex("\n}\n", 0, i)
s = s[:j] + "\n  if (MODE == VLC_ONE) {\n    WAIT_ALL();\n    VSTAMP(7);\n  }" + s[j:]
s += """
extern "C" int p64dbg_vlc_stamps(unsigned long long *host, size_t n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vstamp), n * 8);
}
"""
src = os.path.join(REPO, "p64_amd/csrc/_vlc_stamp.hip")
open(src, "w").write(s)
try:
    os.makedirs(os.path.join(REPO, "abtest"), exist_ok=True)
    obj = os.path.join(REPO, "abtest/vlcstamp.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *sys.argv[1:], "-c",
                    src, "-o", obj], check=True)
finally:
    os.remove(src)
c = os.path.join(REPO, "p64_amd/csrc")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o",
                os.path.join(REPO, "abtest/lib_vlcstamp.so")] +
               [os.path.join(c, f) for f in ("k_search.o", "k_block.o", "k_aux.o", "p64gpu_abi.o", "synth.o",
                                             "p64stream.o", "p64seq.o", "p64prog.o")] + [obj], check=True)
os.remove(obj)
print("abtest/lib_vlcstamp.so")
