"""Closed-loop CPU simulation of exact lower bounds for the FULL search on the
macroblocks k_motion sends to its dense pass (development aid).

The bench's low-contrast sequences (seed % 8 == 7) are encoded by the oracle
(closed loop, FULL SL=31, q=8); for each MB of picture t whose nested 4x4
averages span < 12 levels (the kernel's low-contrast rule), every candidate's
exact SAD against the reconstruction of picture t-1 is computed, T =
min(SAD(c*), SAD(0,0)) with c* the least-bound candidate, and the survivors
(bound <= T) are counted for several exact bounds:
  rows     sum over the 16 rows of |row sum cur - row sum candidate|
  cols     the same over the 16 columns
  rowcol   max(rows, cols)
  s44      sum over the 16 4x4 sub-blocks of |sum cur - sum candidate|
  s22      the same over the 64 2x2 sub-blocks
  p8       the partial SAD of rows 0..7
  p8s44    p8 + the s44 terms of sub-block rows 2..3
usage: python tools/lowc_sim.py [pictures]"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "oracle"))
import oracle  # noqa: E402
import p64_amd  # noqa: E402

W, H = 352, 288
NP = int(sys.argv[1]) if len(sys.argv) > 1 else 6


def lerp(a, b):
    return (a + b) >> 1


def nested_range(C):
    v = lerp(lerp(C[0::4], C[1::4]), lerp(C[2::4], C[3::4]))
    h = lerp(lerp(v[:, 0::4], v[:, 1::4]), lerp(v[:, 2::4], v[:, 3::4]))
    return int(h.max() - h.min())


def blocksum(B, k):
    return B.reshape(16 // k, k, 16 // k, k).sum((1, 3))


stats = {k: [] for k in ("rows", "cols", "rowcol", "s44", "s22", "p8", "p8s44")}
for seed in (7, 15):
    frames = [p64_amd.synth_frame(seed, t, W, H) for t in range(NP)]
    outs = oracle.encode_sequence(frames, W, H, quant=8, me_mode=oracle.ME_FULL, search_limit=31)
    for t in range(2, NP):
        ref = outs[t - 1][3][:W * H].reshape(H, W).astype(np.int64)
        cur = frames[t][:W * H].reshape(H, W).astype(np.int64)
        for mb in range(396):
            x0, y0 = 16 * (mb % 22), 16 * (mb // 22)
            C = cur[y0:y0 + 16, x0:x0 + 16]
            if nested_range(C) >= 12:
                continue
            cands = [(dx, dy) for dx in range(-15, 15) for dy in range(-15, 15)
                     if 0 <= x0 + dx < W - 16 and 0 <= y0 + dy <= H - 16]
            sad, b = {}, {k: {} for k in stats}
            for dx, dy in cands:
                Rb = ref[y0 + dy:y0 + dy + 16, x0 + dx:x0 + dx + 16]
                sad[(dx, dy)] = int(np.abs(C - Rb).sum())
                rr = int(np.abs(C.sum(1) - Rb.sum(1)).sum())
                cc = int(np.abs(C.sum(0) - Rb.sum(0)).sum())
                b["rows"][(dx, dy)] = rr
                b["cols"][(dx, dy)] = cc
                b["rowcol"][(dx, dy)] = max(rr, cc)
                b["s44"][(dx, dy)] = int(np.abs(blocksum(C, 4) - blocksum(Rb, 4)).sum())
                b["s22"][(dx, dy)] = int(np.abs(blocksum(C, 2) - blocksum(Rb, 2)).sum())
                p8 = int(np.abs(C[:8] - Rb[:8]).sum())
                b["p8"][(dx, dy)] = p8
                b["p8s44"][(dx, dy)] = p8 + int(np.abs(blocksum(C, 4)[2:] - blocksum(Rb, 4)[2:]).sum())
            s00 = sad.get((0, 0), 1 << 30)
            for k in stats:
                bb = b[k]
                assert all(bb[c] <= sad[c] for c in cands)
                cs = min(cands, key=lambda c: (bb[c], c))
                T = min(sad[cs], s00)
                stats[k].append(sum(1 for c in cands if bb[c] <= T))
n = len(stats["rows"])
print(f"{n} low-contrast MBs")
for k, v in stats.items():
    v = np.array(v)
    print(f"{k:7s} survivors mean {v.mean():7.1f}  median {np.median(v):6.0f}  p90 {np.percentile(v, 90):6.0f}"
          f"  <=32: {np.mean(v <= 32):.2f}  <=64: {np.mean(v <= 64):.2f}  <=256: {np.mean(v <= 256):.2f}")
