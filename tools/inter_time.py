"""k_inter_mbg (and k_motion) on the bench workload (development aid, GPU
box): S CIF sequences of --content, an intra picture then --steps inter
pictures through p64_amd.encode_frames, closed loop; run under rocprofv3
--kernel-trace (tools/inter_prof.sh) for the per-kernel times."""
import argparse
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

import bench  # noqa: E402
import p64_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--content", default="survey")
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--streams", type=int, default=256)
a = ap.parse_args()
w, h, S = 352, 288, a.streams
nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
fr = bench.make_inputs(torch, p64_amd, a.content, w, h, 1, S, 1 + a.steps)
rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                            mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                            me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"))
for t in range(1 + a.steps):
    p64_amd.encode_frames(fr[t].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li, width=w, height=h,
                          intra=(t == 0), quant=8, me_mode=p64_amd.ME_FULL, search_limit=31, out=out)
torch.cuda.synchronize()
print("done")
