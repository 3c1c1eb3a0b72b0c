"""Survivor counts of the FULL search's first bound under other bounds and
thresholds (development aid; numpy model of k_motion<2>).

For closed-loop survey pictures (reference = the oracle's reconstruction) and
every MB that takes the bound path, counts the candidates left after the
first bound for: the kernel's nested-lerp averages (16 S - 512 <= T), exact
floor averages (16 S - 240 <= T), exact 4x4 sums (S <= T); and for the
kernel's bound the thresholds T from the best full SAD among the 1, 4 or 16
lowest bounds, or the true minimum, with the half-SAD stage after it.
usage: python tools/me_bound_sim.py [--seeds N]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import me_sim  # noqa: E402
import oracle  # noqa: E402  (development aid, not product)
import p64_amd  # noqa: E402

W, H = 352, 288


def box4(P):
    c = np.cumsum(np.cumsum(np.pad(P, ((1, 0), (1, 0))), 0), 1)
    return c[4:, 4:] - c[:-4, 4:] - c[4:, :-4] + c[:-4, :-4]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=3)
    a = ap.parse_args()
    res = {}
    add = lambda k, v: res.setdefault(k, []).append(v)  # noqa: E731
    for seed in range(1, a.seeds + 1):
        fr = [p64_amd.synth_frame(seed, t, W, H, content=p64_amd.SYNTH_SURVEY) for t in range(5)]
        outs = oracle.encode_sequence(fr, W, H, quant=8, me_mode=oracle.ME_FULL, search_limit=31)
        ref = outs[3][3][:W * H].reshape(H, W).astype(np.int64)
        cur = fr[4][:W * H].reshape(H, W).astype(np.int64)
        Rn, Cn = me_sim.nested44(ref), me_sim.nested44(cur)
        Rs, Cs = box4(ref), box4(cur)
        for mb in range(0, 396, 2):
            x0, y0 = 16 * (mb % 22), 16 * (mb // 22)
            C = cur[y0:y0 + 16, x0:x0 + 16]
            cm = Cn[y0:y0 + 16:4, x0:x0 + 16:4]
            if int(cm.max() - cm.min()) < 12:
                continue
            cs = Cs[y0:y0 + 16:4, x0:x0 + 16:4]
            sad0 = int(np.abs(ref[y0:y0 + 16, x0:x0 + 16] - C).sum())
            big = 1 << 40
            SL, SF, SE, Sb, sad, half = (np.full((30, 30), big, np.int64) for _ in range(6))
            for i, dx in enumerate(range(-15, 15)):
                px = x0 + dx
                if not 0 <= px < W - 16:
                    continue
                for j, dy in enumerate(range(-15, 15)):
                    py = y0 + dy
                    if not 0 <= py < H - 16:
                        continue
                    d = np.abs(Rn[py:py + 16:4, px:px + 16:4] - cm)
                    SL[i, j], Sb[i, j] = d.sum(), d[2:].sum()
                    rs = Rs[py:py + 16:4, px:px + 16:4]
                    SF[i, j] = np.abs(rs // 16 - cs // 16).sum()
                    SE[i, j] = np.abs(rs - cs).sum()
                    ad = np.abs(ref[py:py + 16, px:px + 16] - C)
                    sad[i, j], half[i, j] = ad.sum(), ad[:8].sum()
            T = min(int(sad.flat[np.argmin(SL)]), sad0)
            add("bound lerp (16S-512)", int((16 * SL - 512 <= T).sum()))
            T2 = min(int(sad.flat[np.argmin(SF)]), sad0)
            add("bound floor avg (16S-240)", int((16 * SF - 240 <= T2).sum()))
            T3 = min(int(sad.flat[np.argmin(SE)]), sad0)
            add("bound exact 4x4 sums", int((SE <= T3).sum()))
            order = np.argsort(SL, axis=None, kind="stable")
            for name, k in (("T best of 1", 1), ("T best of 4", 4), ("T best of 16", 16), ("T optimal", None)):
                Tk = min(int(sad.min()) if k is None else int(sad.flat[order[:k]].min()), sad0)
                surv = 16 * SL - 512 <= Tk
                add(f"lerp, {name}", int(surv.sum()))
                add(f"lerp, {name}, after half SAD", int((surv & (half + 16 * Sb - 256 <= Tk)).sum()))
    for k, v in res.items():
        v = np.array(v)
        print(f"{k:40s} mean {v.mean():6.1f} median {np.median(v):4.0f} p90 {np.percentile(v, 90):4.0f} "
              f"<=16 {np.mean(v <= 16):.2f}")


if __name__ == "__main__":
    main()
