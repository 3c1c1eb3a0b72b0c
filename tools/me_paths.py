"""Which FULL-search path each macroblock takes on the kbench workload
(development aid; needs a library built with the g_dbg counters)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import p64_amd  # noqa: E402

w, h, S = 352, 288, 256
nmb = (w // 16) * (h // 16)
pic = w * h * 3 // 2
fr = p64_amd.synth_frames_device(w, h, 1, S, 0, 3)
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
r1 = torch.zeros_like(r0)
out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                            mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                            me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"))
p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, out=out)
torch.cuda.synchronize()
lib = p64_amd.lib()
st = (ctypes.c_ulonglong * 8)()
lib.p64gpu_dbg_stats(st, 1)
p64_amd.encode_frames(fr[1].reshape(-1), r0, r1, li, width=w, height=h, intra=False, me_mode=p64_amd.ME_FULL, search_limit=31,
                      out=out)
torch.cuda.synchronize()
lib.p64gpu_dbg_stats(st, 1)
n = st[0]
print(f"MBs {n}  dense {st[1]/n:.3f}  list16 {st[2]/n:.3f}  list64 {st[3]/n:.3f}  "
      f"mean survivors {st[4]/n:.1f}  second stage: MBs {st[6]/n:.3f} mean n2 {st[5]/max(st[6],1):.1f} "
      f"n2>16 {st[7]/n:.3f}")
