"""CPU simulation of the FULL-search pruning bounds (development aid).

For each macroblock of a few synthetic CIF pictures (the bench generator,
host side), computes every candidate's exact SAD and three lower bounds:
  p6        the partial SAD of rows 0..5 (the pre-pass this kernel used before)
  nested44  16*S - 512 over nested-lerp 4x4 averages (the kernel's bound)
  exact44   16*S - 240 over exact floor 4x4 averages
and counts the survivors (bound <= T, T = min(SAD(c*), SAD(0,0)), c* = argmin of
the bound); it also asserts bound <= SAD for every candidate.  Open loop: the
previous *source* picture stands in for the reconstruction, which makes the
best match tighter than in the closed-loop encoder (tools/me_paths.py measures
the kernel's real path mix on the bench content).  usage: python tools/lb_sim.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import p64_amd  # noqa: E402

W, H = 352, 288


def lerp(a, b):
    return (a + b) >> 1


def nested44(P):
    v1 = lerp(P[:-1], P[1:])
    v2 = lerp(v1[:-2], v1[2:])
    h1 = lerp(v2[:, :-1], v2[:, 1:])
    return lerp(h1[:, :-2], h1[:, 2:])


def exact44(P):
    c = np.zeros((P.shape[0] + 1, P.shape[1] + 1), np.int64)
    c[1:, 1:] = P.cumsum(0).cumsum(1)
    return (c[4:, 4:] - c[:-4, 4:] - c[4:, :-4] + c[:-4, :-4]) // 16


def main():
    for seed, t in ((1, 2), (2, 3), (3, 2), (4, 3), (7, 2)):
        res = {"p6": [], "nested44": [], "exact44": []}
        ref = p64_amd.synth_frame(seed, t - 1, W, H)[:W * H].reshape(H, W).astype(np.int64)
        cur = p64_amd.synth_frame(seed, t, W, H)[:W * H].reshape(H, W).astype(np.int64)
        Rn, Cn, Re, Ce = nested44(ref), nested44(cur), exact44(ref), exact44(cur)
        for mb in range(0, 396, 2):
            x0, y0 = 16 * (mb % 22), 16 * (mb // 22)
            C = cur[y0:y0 + 16, x0:x0 + 16]
            big = np.int64(1) << 40
            sad, p6, ln, le = (np.full((30, 30), big) for _ in range(4))
            cn, ce = Cn[y0:y0 + 16:4, x0:x0 + 16:4], Ce[y0:y0 + 16:4, x0:x0 + 16:4]
            for i, dx in enumerate(range(-15, 15)):
                for j, dy in enumerate(range(-15, 15)):
                    px, py = x0 + dx, y0 + dy
                    if not (0 <= px < W - 16 and 0 <= py < H - 16):
                        continue
                    d = np.abs(ref[py:py + 16, px:px + 16] - C)
                    sad[i, j], p6[i, j] = d.sum(), d[:6].sum()
                    ln[i, j] = 16 * np.abs(Rn[py:py + 16:4, px:px + 16:4] - cn).sum() - 512
                    le[i, j] = 16 * np.abs(Re[py:py + 16:4, px:px + 16:4] - ce).sum() - 240
            assert (ln <= sad).all() and (le <= sad).all()
            sad0 = np.abs(ref[y0:y0 + 16, x0:x0 + 16] - C).sum()
            for name, lb in (("p6", p6), ("nested44", ln), ("exact44", le)):
                k = np.unravel_index(np.argmin(lb), lb.shape)
                res[name].append(int((lb <= min(sad[k], sad0)).sum()))
        for name, v in res.items():
            v = np.array(v)
            print(f"seed {seed} picture {t}  {name:9s} survivors mean {v.mean():6.1f} "
                  f"median {np.median(v):5.1f} p90 {np.percentile(v, 90):6.1f}  >256 {(v > 256).mean():.3f}")


if __name__ == "__main__":
    main()
