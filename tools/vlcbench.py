"""Times the GPU entropy coder on the bench workload's records (GPU box).
usage: python tools/vlcbench.py [survey|synth]  (rocprofv3 --kernel-trace
gives the per-kernel split: tools/vlc_prof.sh)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import p64_amd  # noqa: E402
from p64_amd import stream  # noqa: E402

w, h, S = 352, 288, 256
nmb = 396
pic = w * h * 3 // 2
content = sys.argv[1] if len(sys.argv) > 1 else "survey"
fr = p64_amd.synth_frames_device(w, h, 1, S, 0, 2, content=p64_amd.CONTENTS[content])
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
r1 = torch.zeros_like(r0)
def outbuf():
    return p64_amd.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                 mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                 me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"),
                                 vlc_bits=torch.zeros((S, nmb, 8), dtype=torch.int16, device="cuda"))


o0 = p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, out=outbuf())
o1 = p64_amd.encode_frames(fr[1].reshape(-1), r0, r1, li, width=w, height=h, intra=False, me_mode=1,
                           search_limit=31, out=outbuf())
gq = torch.full((S, 12), 8, dtype=torch.uint8, device="cuda")
tr = torch.ones(S, dtype=torch.int32, device="cuda")
for name, o, vb in (("intra", o0, None), ("inter", o1, None), ("intra_given", o0, o0.vlc_bits),
                    ("inter_given", o1, o1.vlc_bits)):
    for _ in range(3):
        stream.vlc_pictures(o.mb, o.coef, gq, tr, width=w, height=h, blk_bits=vb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 10
    for _ in range(n):
        _, bits = stream.vlc_pictures(o.mb, o.coef, gq, tr, width=w, height=h, blk_bits=vb)
    dt = (time.perf_counter() - t0) / n
    print(f"{name}: {dt * 1e6:.1f} us per call incl. sync, {S * nmb / dt / 1e6:.1f} M MB/s, "
          f"{sum(bits) / (S * nmb):.1f} bits/MB")
