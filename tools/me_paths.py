"""Which FULL-search path each macroblock takes on the kbench workload
(development aid; needs a library built with -DP64_ME_STATS)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import p64_amd  # noqa: E402

w, h, S = 352, 288, 256
nmb = (w // 16) * (h // 16)
pic = w * h * 3 // 2
fr = p64_amd.synth_frames_device(w, h, 1, S, 0, 6)
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
r1 = torch.zeros_like(r0)
out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                            mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                            me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"))
p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, out=out)
torch.cuda.synchronize()
lib = p64_amd.lib()
st = (ctypes.c_ulonglong * 48)()
lib.p64gpu_dbg_stats(st, 1)
for t in range(1, 6):
    p64_amd.encode_frames(fr[t].reshape(-1), r0, r1, li, width=w, height=h, intra=False,
                          me_mode=p64_amd.ME_FULL, search_limit=31, out=out)
    torch.cuda.synchronize()
    r0, r1 = r1, r0
    lib.p64gpu_dbg_stats(st, 1)
    n = st[0]
    print(f"picture {t}: MBs {n}  mean survivors {st[1]/n:.1f}  <=4 {st[2]/n:.3f}  <=8 {st[3]/n:.3f}  "
          f"<=32 {st[4]/n:.3f}  list {st[5]/n:.3f}  dense {st[6]/n:.4f}")
    if t == 5:  # sub-block-average range of the current block vs the dense path
        for b in range(16):
            a, d = st[8 + 2 * b], st[9 + 2 * b]
            if a + d:
                print(f"  range {4*b:3d}-{4*b+3:3d}{'+' if b == 15 else ' '}: MBs {a+d:7d}  dense {d/(a+d):.3f}")
