"""CPU model of k_motion<2>'s path choice (development aid, FULL SL=31).

For macroblocks of closed-loop pictures (the reference picture is the oracle's
reconstruction of the previous picture, as in the encoder) this replays the
kernel's decisions from DESIGN.md 5 step 2 with numpy: the current block's
sub-block range (< 12: dense pass), the noise rule (SAD(0,0) > 24*256 and
2E > SAD(0,0): dense pass), the nested-lerp 4x4 bound S per candidate, c*,
T = min(SAD(c*), SAD(0,0)), the survivors S <= (T + 512) >> 4 and the
finishing path they take (<= 4, <= 8, <= 32 grouped lanes, <= 256 one per
lane, else dense).  Prints the path mix and survivor statistics per content.
usage: python tools/me_sim.py [survey|synth ...] [--seeds N] [--t T]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402  (development aid, not product)
import p64_amd  # noqa: E402

W, H = 352, 288


def lerp(a, b):
    return (a + b) >> 1


def nested44(P):
    v1 = lerp(P[:-1], P[1:])
    v2 = lerp(v1[:-2], v1[2:])
    h1 = lerp(v2[:, :-1], v2[:, 1:])
    return lerp(h1[:, :-2], h1[:, 2:])


def mb_paths(ref, cur, stats, sample=1):
    Rn, Cn = nested44(ref), nested44(cur)
    for mb in range(0, 396, sample):
        x0, y0 = 16 * (mb % 22), 16 * (mb // 22)
        C = cur[y0:y0 + 16, x0:x0 + 16]
        cm = Cn[y0:y0 + 16:4, x0:x0 + 16:4]
        rng = int(cm.max() - cm.min())
        sad0 = int(np.abs(ref[y0:y0 + 16, x0:x0 + 16] - C).sum())
        # E: sum |pixel - its sub-block average| (the kernel's average m)
        ehf = int(np.abs(C - np.repeat(np.repeat(cm, 4, 0), 4, 1)).sum())
        if rng < 12:
            stats["dense_lowc"] += 1
            continue
        if sad0 > 24 * 256 and 2 * ehf > sad0:
            stats["dense_noise"] += 1
            continue
        big = 1 << 40
        S = np.full((30, 30), big, np.int64)
        sad = np.full((30, 30), big, np.int64)
        for i, dx in enumerate(range(-15, 15)):
            px = x0 + dx
            if not 0 <= px < W - 16:
                continue
            for j, dy in enumerate(range(-15, 15)):
                py = y0 + dy
                if not 0 <= py < H - 16:
                    continue
                S[i, j] = np.abs(Rn[py:py + 16:4, px:px + 16:4] - cm).sum()
                sad[i, j] = np.abs(ref[py:py + 16, px:px + 16] - C).sum()
        k = np.unravel_index(np.argmin(S), S.shape)  # first in dx-major scan order
        T = min(int(sad[k]), sad0)
        Ts = (T + 512) >> 4
        n = int((S <= Ts).sum())
        stats["surv"].append(n)
        stats["Smin"].append(int(S[k]))
        stats["T"].append(T)
        if n <= 1:
            stats["lb_le1"] += 1
        elif n <= 4:
            stats["lb_g4"] += 1
        elif n <= 8:
            stats["lb_g2"] += 1
        elif n <= 32:
            stats["lb_g1"] += 1
        elif n <= 256:
            stats["lb_list"] += 1
        else:
            stats["dense_many"] += 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("contents", nargs="*", default=["survey", "synth"])
    ap.add_argument("--seeds", type=int, default=4)
    ap.add_argument("--t", type=int, default=4)
    ap.add_argument("--sample", type=int, default=3)
    a = ap.parse_args()
    for content in a.contents:
        stats = {k: 0 for k in ("dense_lowc", "dense_noise", "lb_le1", "lb_g4", "lb_g2", "lb_g1", "lb_list",
                                "dense_many")}
        stats.update(surv=[], Smin=[], T=[])
        for seed in range(1, a.seeds + 1):
            fr = [p64_amd.synth_frame(seed, t, W, H, content=p64_amd.CONTENTS[content]) for t in range(a.t + 1)]
            outs = oracle.encode_sequence(fr, W, H, quant=8, me_mode=oracle.ME_FULL, search_limit=31)
            ref = outs[a.t - 1][3][:W * H].reshape(H, W).astype(np.int64)
            cur = fr[a.t][:W * H].reshape(H, W).astype(np.int64)
            mb_paths(ref, cur, stats, a.sample)
        tot = sum(v for k, v in stats.items() if not isinstance(v, list))
        print(f"{content}: {tot} MBs  " + "  ".join(f"{k} {v / tot:.3f}" for k, v in stats.items()
                                                  if not isinstance(v, list)))
        s = np.array(stats["surv"])
        if s.size:
            print(f"  survivors mean {s.mean():.1f} median {np.median(s):.0f} p90 {np.percentile(s, 90):.0f}"
                  f"  T mean {np.mean(stats['T']):.0f}  S(c*) mean {np.mean(stats['Smin']):.1f}")


if __name__ == "__main__":
    main()
