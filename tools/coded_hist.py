"""Coded blocks per wave (10 MBs) of a closed-loop FULL encode of the bench's
synth content (development aid): the distribution that sets the number of
idct_coded_blocks passes in k_recon_mbg / k_inter_mbg.
  python3 tools/coded_hist.py [--steps N] [--seqs S]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import p64_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--seqs", type=int, default=256)
a = ap.parse_args()
w, h, S = 352, 288, a.seqs
nmb = (w // 16) * (h // 16)
pic = p64_amd.picture_bytes(w, h)
fr = p64_amd.synth_frames_device(w, h, 1, S, 0, a.steps)
rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
tc_t = torch.tensor([1, 1, 1, 1, 0, 1, 1, 0, 1, 1], device="cuda")
cbp_t = torch.tensor([0, 0, 1, 1, 0, 1, 1, 0, 1, 1], device="cuda")
hist = torch.zeros(61, dtype=torch.long, device="cuda")
mtypes = torch.zeros(10, dtype=torch.long, device="cuda")
per_step = []
for t in range(a.steps):
    o = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                              mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"), me=None)
    p64_amd.encode_frames(fr[t].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li, width=w, height=h,
                          intra=(t == 0), quant=8, me_mode=p64_amd.ME_FULL, search_limit=31, out=o)
    if t == 0:
        continue
    mt = o.mb[..., 0].reshape(-1).long()
    cbp = o.mb[..., 1].reshape(-1).long() & 63
    cbp = torch.where(cbp_t[mt] == 1, cbp, torch.full_like(cbp, 63))
    nblk = sum(((cbp >> b) & 1) for b in range(6)) * tc_t[mt]
    nw = nblk.numel() // 10
    per_wave = nblk[: nw * 10].reshape(nw, 10).sum(1)
    hist += torch.bincount(per_wave, minlength=61)
    per_step.append(nblk.float().mean())
    mtypes += torch.bincount(mt, minlength=10)
hist = hist.cpu().tolist()
tot = sum(hist)
passes = [0] * 9
for n, c in enumerate(hist):
    passes[(n + 7) // 8] += c
print("MTYPE share:", [round(x / mtypes.sum().item(), 3) for x in mtypes.cpu().tolist()])
print("coded blocks per MB:", round(sum(n * c for n, c in enumerate(hist)) / tot / 10, 3))
print("passes per wave share:", [round(p / tot, 3) for p in passes])
ps = torch.stack(per_step).cpu().tolist()
print("coded blocks per MB by step (means of 10):",
      [round(sum(ps[i:i + 10]) / len(ps[i:i + 10]), 2) for i in range(0, len(ps), 10)])
print("mean passes:", round(sum(i * p for i, p in enumerate(passes)) / tot, 2))
