"""k_motion<2> timing per content (development aid, GPU box): S CIF sequences,
reference = the intra reconstruction of picture t-1, current = picture t, for
the bench's contents (synth, pan15, noise, flat; bench.make_inputs).  Median
of R launches by HIP events; also checks that the library's records equal
those of P64GPU_REF_LIB (if given) -- timing probes that drop work differ.
usage: [P64GPU_LIB=...] python tools/me_time.py [--reps R] [--streams S] [--search-limit SL]
"""
import argparse
import os
import statistics
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

import bench  # noqa: E402
import p64_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--contents", default="synth,pan15,noise,flat")
    ap.add_argument("--search-limit", type=int, default=31)
    a = ap.parse_args()
    w, h, S = 352, 288, a.streams
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    out = {}
    for content in a.contents.split(","):
        fr = bench.make_inputs(torch, p64_amd, content, w, h, 1, S, 4)
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        rec = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
        p64_amd.encode_frames(fr[2].reshape(-1), None, rec, li, width=w, height=h, intra=True, quant=8)
        cur = fr[3].reshape(-1)
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            me = p64_amd.MotionEstimation(rec, cur, w, h, mode=p64_amd.ME_FULL, search_limit=a.search_limit)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        out[content] = (statistics.median(ts), min(ts), me.cpu())
        print(f"{content:6s} k_motion<2> median {out[content][0]:8.1f} us  min {out[content][1]:8.1f} us",
              flush=True)
    torch.save({k: v[2] for k, v in out.items()}, os.path.join(R, "gpurun_out", "me_time_records.pt"))


if __name__ == "__main__":
    main()
