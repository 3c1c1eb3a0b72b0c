"""Per-kernel timing on the bench workload (development aid, GPU box).

Times, on S CIF sequences resident in HBM: the fused encode (FULL and TSS),
motion estimation alone (FULL and TSS), and the intra-picture encode, each as
the median of R launches bracketed by HIP events on torch's stream.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import p64_amd  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--width", type=int, default=352)
    ap.add_argument("--height", type=int, default=288)
    ap.add_argument("--skew", type=int, default=0,
                    help="bytes between the two reconstruction buffers' placements (16-aligned)")
    a = ap.parse_args()
    w, h, S = a.width, a.height, a.streams
    nmb = (w // 16) * (h // 16)
    pic = w * h * 3 // 2
    fr = p64_amd.synth_frames_device(w, h, 1, S, 0, 8)  # 8 slots: 311 MB > the 256 MB MALL
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
    if a.skew:  # the second buffer `skew` bytes into a larger allocation
        r1 = torch.zeros(S * pic + a.skew, dtype=torch.uint8, device="cuda")[a.skew:]
    else:
        r1 = torch.zeros_like(r0)
    out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"))
    p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, out=out)
    torch.cuda.synchronize()
    res = {}
    slot = [0]

    def intra():  # a different input picture batch every launch
        slot[0] = (slot[0] + 1) % 8
        p64_amd.encode_frames(fr[slot[0]].reshape(-1), None, r1, li, width=w, height=h, intra=True,
                              out=out)
    res["intra_encode"] = timed(intra, a.reps)
    for mode, name in ((p64_amd.ME_FULL, "full"), (p64_amd.ME_TSS, "tss")):
        res[f"fused_{name}"] = timed(lambda: p64_amd.encode_frames(
            fr[1].reshape(-1), r0, r1, li, width=w, height=h, intra=False, me_mode=mode,
            search_limit=31, out=out), a.reps)
        res[f"me_only_{name}"] = timed(lambda: p64_amd.MotionEstimation(
            r0, fr[1].reshape(-1), w, h, mode=mode, search_limit=31), a.reps)
    # decode-side reconstruction (config 5) of the inter picture just coded
    qmb = torch.full((S * nmb,), 8, dtype=torch.uint8, device="cuda")
    mask = torch.ones_like(qmb)
    d1 = torch.empty_like(r1)
    p64_amd.encode_frames(fr[1].reshape(-1), r0, r1, li, width=w, height=h, intra=False,
                          me_mode=p64_amd.ME_FULL, search_limit=31, out=out)
    res["decode_recon"] = timed(lambda: p64_amd.decode_recon(r0, d1, out.coef, out.mb, qmb, mask,
                                                             width=w, height=h), a.reps)
    # entropy coding of that picture batch (count, scan, emit + the bits copy)
    from p64_amd import stream as p64s
    gq = torch.full((S, nmb // 33), 8, dtype=torch.uint8, device="cuda")
    trs = torch.full((S,), 1, dtype=torch.int32, device="cuda")
    res["vlc"] = timed(lambda: p64s.vlc_pictures(out.mb, out.coef, gq, trs, width=w, height=h), a.reps)
    for k, (med, mn) in res.items():
        print(f"{k:16s} median {med:9.1f} us  min {mn:9.1f} us  {S * nmb / med * 1e6 / 1e6:8.1f} M MB/s")


if __name__ == "__main__":
    main()
