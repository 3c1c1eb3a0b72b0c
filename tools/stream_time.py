"""Kernel timing on the bench's own stream (development aid): a closed-loop
FULL encode of the synth content (as bench.py's inter config), then the last
steps' encodes and decodes repeated, for a rocprofv3 kernel trace
(tools/trace_libs.sh with SCRIPT=tools/stream_time.py).  tools/kbench.py
re-codes one picture against its own reconstruction, which leaves almost no
coded blocks; the decoder's and k_inter_mbg's coded-block passes need the
real distribution (tools/coded_hist.py: ~1.44 coded blocks per MB).
  python3 tools/stream_time.py [--steps N] [--reps R]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import p64_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--seqs", type=int, default=256)
a = ap.parse_args()
w, h, S = 352, 288, a.seqs
nmb = (w // 16) * (h // 16)
pic = p64_amd.picture_bytes(w, h)
fr = p64_amd.synth_frames_device(w, h, 1, S, 0, a.steps)
rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(a.steps + 1)]
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
outs = []
for t in range(a.steps):
    o = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                              mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"), me=None)
    p64_amd.encode_frames(fr[t].reshape(-1), rec[t], rec[t + 1], li, width=w, height=h,
                          intra=(t == 0), quant=8, me_mode=p64_amd.ME_FULL, search_limit=31, out=o)
    outs.append(o)
torch.cuda.synchronize()
qmb = torch.full((S * nmb,), 8, dtype=torch.uint8, device="cuda")
mask = torch.ones_like(qmb)
dec = torch.empty_like(rec[0])
li2 = li.clone()
scratch = torch.empty_like(rec[0])
ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
# every inter picture in turn: its levels (78 MB a batch) are not in the
# 256-MB last-level cache when its launch starts, as in bench.py
ts = list(range(1, a.steps))
ev[0].record()
for _ in range(a.reps):
    for t in ts:
        p64_amd.decode_recon(rec[t], dec, outs[t].coef, outs[t].mb, qmb, mask, width=w, height=h)
ev[1].record()
for _ in range(a.reps):
    for t in ts:
        li2.copy_(li)
        p64_amd.encode_frames(fr[t].reshape(-1), rec[t], scratch, li2, width=w, height=h, intra=False,
                              quant=8, me_mode=p64_amd.ME_FULL, search_limit=31, out=outs[t])
ev[2].record()
torch.cuda.synchronize()
n = len(ts) * a.reps
print(f"decode_recon {ev[0].elapsed_time(ev[1]) / n * 1e3:.1f} us  encode (FULL) "
      f"{ev[1].elapsed_time(ev[2]) / n * 1e3:.1f} us per picture batch (events, incl. launch gaps)")
ok = torch.equal(dec, rec[ts[-1] + 1])
print("last decode == encoder reconstruction:", ok)
