"""Per-wave timeline of the block-layout kernels (development aid, never
shipped): writes abtest/k_block_stamp.hip, a copy of k_block.hip whose
kernels stamp s_memrealtime (100 MHz) at wave start (T0, with the wave's XCD in
bits 56..59), once the first
loads have arrived (T1, after an s_waitcnt 0), before the stores (T2) and
once the stores have completed (T3), into a device array read back through
p64dbg_stamps().  Build with tools/ablib.sh stamp abtest/k_block_stamp.hip
k_block; run tools/blk_timeline.py on the GPU box.
"""
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(REPO, "p64_amd/csrc/k_block.hip")).read()


def sub(old, new, count=1):
    global s
    assert s.count(old) >= count, old
    s = s.replace(old, new)


sub("namespace {\n", """namespace {
__device__ unsigned long long g_stamp[4u << 16];
#define STAMP(k)                                                                 \\
  do {                                                                           \\
    if ((threadIdx.x & 63) == 0)                                                 \\
      g_stamp[4u * (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) + (k)] =                    \\
          __builtin_amdgcn_s_memrealtime() |                                                           \\
          ((k) == 0 ? (unsigned long long)__builtin_amdgcn_s_getreg(XCC_ID_REG) << 56 : 0ull);        \\
  } while (0)
#define WAIT_ALL() __builtin_amdgcn_s_waitcnt(0)
// s_getreg HW_REG_XCC_ID (gfx940+: hwreg 20, bits 3:0): the XCD the wave runs on
#define XCC_ID_REG ((3 << 11) | 20)
""")
# intra
sub("""  if (gmb0 >= nmbs) return;  // whole wave
  PRIO_HIGH();
  const int l = min(lane, 6 * MBS_PER_WAVE - 1);
  const unsigned gmb = min(gmb0 + (unsigned)(l / 6), nmbs - 1);  // tail lanes repeat the last MB
  const IntraFetch f = intra_fetch_at<QMB>(a, blk_pos_mb(gmb, l % 6, a.width, a.height, kd));
  PRIO_LOW();""", """  if (gmb0 >= nmbs) return;  // whole wave
  STAMP(0);
  PRIO_HIGH();
  const int l = min(lane, 6 * MBS_PER_WAVE - 1);
  const unsigned gmb = min(gmb0 + (unsigned)(l / 6), nmbs - 1);  // tail lanes repeat the last MB
  const IntraFetch f = intra_fetch_at<QMB>(a, blk_pos_mb(gmb, l % 6, a.width, a.height, kd));
  PRIO_LOW();
  WAIT_ALL();
  STAMP(1);""")
sub("""  mbg_store(a, kd, lds, lane, nmbs, gmb0, nvalid, o.rec_off, o.pw, o.rec, rl, gmb, 0x3f00u, 0);
}""", """  STAMP(2);
  mbg_store(a, kd, lds, lane, nmbs, gmb0, nvalid, o.rec_off, o.pw, o.rec, rl, gmb, 0x3f00u, 0);
  WAIT_ALL();
  STAMP(3);
}""")
# decoder
sub("""  const RecStageB S = rec_stage_b(B, w, h, stride, A);
  PRIO_LOW();
  rec_block_pk(w, h, stride, rec, A, S);
}""", """  const RecStageB S = rec_stage_b(B, w, h, stride, A);
  PRIO_LOW();
  WAIT_ALL();
  STAMP(1);
  rec_block_pk(w, h, stride, rec, A, S);
  STAMP(2);
  WAIT_ALL();
  STAMP(3);
}""")
sub("""  const int nmb = (w >> 4) * (h >> 4), nfr = (int)mdiv(nmbs, kd.mn, kd.sn);
  RecBufs B;""", """  STAMP(0);
  const int nmb = (w >> 4) * (h >> 4), nfr = (int)mdiv(nmbs, kd.mn, kd.sn);
  RecBufs B;""")
# inter
sub("""  const int64_t stride = a.frame_stride;
  RecBufs B;""", """  STAMP(0);
  const int64_t stride = a.frame_stride;
  RecBufs B;""")
sub("""  const IntraFetch f = intra_fetch_at<QMB>(a, pos);  // current rows, q
""", """  const IntraFetch f = intra_fetch_at<QMB>(a, pos);  // current rows, q
  WAIT_ALL();
  STAMP(1);
""")
sub("""  mbg_store(a, kd, lds, lane, nmbs, gmb0, nvalid, ro, pw, prow, rl, gmb, mbw,
            mt_intra(mt) ? (uint8_t)0 : (uint8_t)(li + 1));
}""", """  STAMP(2);
  mbg_store(a, kd, lds, lane, nmbs, gmb0, nvalid, ro, pw, prow, rl, gmb, mbw,
            mt_intra(mt) ? (uint8_t)0 : (uint8_t)(li + 1));
  WAIT_ALL();
  STAMP(3);
}""")
s += """
extern "C" int p64dbg_stamps(unsigned long long *host, size_t n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamp), n * 8);
}
extern "C" int p64dbg_stamps_clear(void) {
  static unsigned long long z[4u << 16];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof z);
}
"""
open(os.path.join(REPO, "abtest", "k_block_stamp.hip"), "w").write(s)
print("abtest/k_block_stamp.hip")
