"""Timing-only variants of k_search.hip (development aid, never shipped):
writes abtest/k_search_<name>.hip with one phase of the FULL search switched
off or rerouted, for cost-by-subtraction A/B runs (tools/ablib.sh +
tools/trace_libs.sh).  Variants that drop work give WRONG vectors; they are
timing probes only.
"""
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(REPO, "p64_amd/csrc/k_search.hip")).read()
DENSE = "  } else {  // little pruned: every candidate densely, rows in two chunks"
LB = "  if (range >= ME_LOW_CONTRAST) {"
FIN = "  if (nsurv <= ME_LIST_MAX) {"
assert DENSE in src and LB in src and FIN in src

def cut(text, start, end):
    """text with the lines from the one containing `start` up to (not
    including) the one containing `end` removed"""
    a = text.index(start)
    a = text.rindex("\n", 0, a) + 1
    b = text.index(end, a)
    b = text.rindex("\n", 0, b) + 1
    return text[:a] + text[b:]


NOFIN = [(FIN, "  if (lane < 0) {"), (DENSE, "  } else if (lane < 0) {")]
variants = {
    "nodense": [(DENSE, "  } else if (lane < 0) {")],            # dense pass off
    "alldense": [(LB, "  if (range < 0) {")],                       # every MB dense
    "nolowc": [("constexpr int ME_LOW_CONTRAST = 12;", "constexpr int ME_LOW_CONTRAST = 0;")],
    "nofinish": [(FIN, "  if (lane < 0) {"), (DENSE, "  } else if (lane < 0) {")],
}
os.makedirs(os.path.join(REPO, "abtest"), exist_ok=True)
cuts = {  # (start, end) line ranges removed, on top of NOFIN
    "nofin_nomap": [("    build_lb_map(L, lane);", '    SECTION("lb_pass");')],
    "nofin_nolb": [("    {\n      const int xq = colb >> 2;", "    // 2. c* and its full SAD")],
    "nofin_nocstar": [('    SECTION("cstar");', "    const unsigned T = min(")],
    "nofin_nosurv": [("    nsurv = 0;\n#pragma unroll", "    nsurv = uni(nsurv);")],
    "nofin_nothing": [("  if (range >= ME_LOW_CONTRAST) {", '  SECTION("finish");')],
}
for name, cl in cuts.items():
    variants[name] = NOFIN + [("@cut", c) for c in cl]
for name, subs in variants.items():
    s = src
    for a, b in subs:
        if a == "@cut":
            s = cut(s, *b)
        else:
            assert a in s, (name, a)
            s = s.replace(a, b)
    open(os.path.join(REPO, "abtest", f"k_search_{name}.hip"), "w").write(s)
    print(name)

# k_motion with WPG macroblock-waves per workgroup (wave-level barriers): is
# the one-wave-workgroup launch limited by workgroup slots per CU?
for wpg in (2, 4):
    s = src.replace("namespace {\n", "namespace {\n__device__ __forceinline__ void wave_sync() {\n"
                    "  __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");\n"
                    "  __builtin_amdgcn_wave_barrier();\n"
                    "  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");\n}\n"
                    "#define __syncthreads() wave_sync()\n", 1)
    old = ("__global__ __launch_bounds__(64, 1) void k_motion(")
    assert old in s
    s = s.replace(old, f"__global__ __launch_bounds__({64 * wpg}, 1) void k_motion(")
    old = ("  __shared__ MbLds L;\n  const int lane = threadIdx.x;\n  const int mbw = w >> 4, nmb = mbw * (h >> 4);\n"
           "  const unsigned gid = xcd_remap(blockIdx.x, gridDim.x);\n")
    assert old in s
    s = s.replace(old, f"  __shared__ MbLds Ls[{wpg}];\n  MbLds &L = Ls[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];\n"
                  "  const int lane = threadIdx.x & 63;\n  const int mbw = w >> 4, nmb = mbw * (h >> 4);\n"
                  f"  const unsigned gid = xcd_remap(blockIdx.x, gridDim.x) * {wpg}u + (unsigned)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n")
    old = "  const unsigned grid = (unsigned)((int64_t)nframes * (w / 16) * (h / 16));\n  if (mode == 2)\n"
    assert old in s
    s = s.replace(old, f"  const unsigned grid = (unsigned)((int64_t)nframes * (w / 16) * (h / 16)) / {wpg};\n  if (mode == 2)\n")
    s = s.replace("hipLaunchKernelGGL(k_motion<2>, dim3(grid), dim3(64),", f"hipLaunchKernelGGL(k_motion<2>, dim3(grid), dim3({64 * wpg}),")
    s = s.replace("hipLaunchKernelGGL(k_motion<1>, dim3(grid), dim3(64),", f"hipLaunchKernelGGL(k_motion<1>, dim3(grid), dim3({64 * wpg}),")
    open(os.path.join(REPO, "abtest", f"k_search_wpg{wpg}.hip"), "w").write(s)
    print(f"wpg{wpg}")
