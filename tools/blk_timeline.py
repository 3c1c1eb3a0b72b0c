"""Per-wave timelines of k_intra_mbg / k_inter_mbg / k_recon_mbg from the
stamp build (tools/blk_stamps.py): P64GPU_LIB=abtest/lib_stamp.so python
tools/blk_timeline.py.  Prints, per kernel, the span, the per-wave phase
durations (load = T1-T0, compute = T2-T1, store = T3-T2; us) and how many
waves are in each phase over time (10 bins), plus wave start-time quantiles
(rounds of residency)."""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

import bench  # noqa: E402
import p64_amd  # noqa: E402

L = p64_amd.lib()
L.p64dbg_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]


def grab(nw):
    buf = np.zeros(4 * nw, np.uint64)
    torch.cuda.synchronize()
    assert L.p64dbg_stamps(buf.ctypes.data, buf.size) == 0
    L.p64dbg_stamps_clear()
    t = buf.reshape(nw, 4).astype(np.int64)
    t = t[t[:, 0] > 0]
    xcd = t[:, 0] >> 56
    t[:, 0] &= (1 << 56) - 1
    t0 = t[:, 0].min()
    return np.concatenate([(t - t0) / 100.0, xcd[:, None]], axis=1)  # 100 MHz -> us; column 4 = XCD


def report(name, t):
    if os.environ.get("TL_SAVE"):  # raw per-wave rows for offline analysis
        np.save(os.path.join(os.environ["TL_SAVE"], name.replace("<", "_").replace(">", "") + ".npy"), t)
    span = t[:, 3].max()
    t = t.copy()
    ld, cp, st = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    q = lambda a: " ".join(f"{x:6.2f}" for x in np.percentile(a, [10, 50, 90]))  # noqa: E731
    print(f"== {name}: {len(t)} waves, span {span:.1f} us")
    print(f"   load    p10/50/90 {q(ld)}")
    print(f"   compute p10/50/90 {q(cp)}")
    print(f"   store   p10/50/90 {q(st)}")
    print(f"   start   quantiles {' '.join(f'{x:6.1f}' for x in np.percentile(t[:, 0], [0, 10, 25, 50, 75, 90, 100]))}")
    bins = np.linspace(0, span, 11)
    for i in range(10):
        mid = 0.5 * (bins[i] + bins[i + 1])
        a = ((t[:, 0] <= mid) & (t[:, 1] > mid)).sum()
        b = ((t[:, 1] <= mid) & (t[:, 2] > mid)).sum()
        c = ((t[:, 2] <= mid) & (t[:, 3] > mid)).sum()
        per = [int(((t[:, 0] <= mid) & (t[:, 3] > mid) & (t[:, 4] == x)).sum()) for x in range(8)]
        print(f"   t={mid:6.1f}  loading {a:5d}  computing {b:5d}  storing {c:5d}   per XCD {per}")


def main():
    w, h, S = 352, 288, 256
    if len(sys.argv) > 1 and sys.argv[1] == "motion":  # the k_motion stamp build
        nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
        fr = bench.make_inputs(torch, p64_amd, "synth", w, h, 1, S, 3)
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
        p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, quant=8)
        for _ in range(2):
            p64_amd.MotionEstimation(r0, fr[1].reshape(-1), w, h, mode=p64_amd.ME_FULL, search_limit=31)
        grab(S * nmb)
        p64_amd.MotionEstimation(r0, fr[1].reshape(-1), w, h, mode=p64_amd.ME_FULL, search_limit=31)
        report("k_motion<2>", grab(S * nmb))
        return
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    nw = (S * nmb + 9) // 10
    fr = bench.make_inputs(torch, p64_amd, "synth", w, h, 1, S, 3)
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
    r1 = torch.zeros_like(r0)
    for _ in range(3):  # warm
        p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, quant=8)
    grab(nw)
    p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, quant=8)
    report("k_intra_mbg", grab(nw + 4))
    o = p64_amd.encode_frames(fr[1].reshape(-1), r0, r1, li, width=w, height=h, intra=False, quant=8,
                              me_mode=p64_amd.ME_FULL, search_limit=31)
    report("k_inter_mbg", grab(nw + 4))
    qmb = torch.full((S * nmb,), 8, dtype=torch.uint8, device="cuda")
    d = torch.empty_like(r1)
    p64_amd.decode_recon(r0, d, o.coef, o.mb, qmb, torch.ones_like(qmb), width=w, height=h)
    report("k_recon_mbg", grab(nw + 4))


if __name__ == "__main__":
    main()
