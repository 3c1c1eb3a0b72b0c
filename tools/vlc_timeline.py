"""The entropy coder's per-wave timeline (GPU box, development aid; build
abtest/lib_vlcstamp.so with tools/vlc_stamps.py first): the bench's survey
records (256 CIF sequences, closed loop, picture 4), one timed-mode launch of
the coder (counting itself), then the eight stamps of every wave: phase
durations, wave lifetimes, when waves start, and how many are resident over
the launch.  usage: P64GPU_LIB=abtest/lib_vlcstamp.so python3 tools/vlc_timeline.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import p64_amd
    from p64_amd import stream as p64s
    w, h, S, nmb, P = 352, 288, 256, 396, 4
    pic = w * h * 3 // 2
    fr = p64_amd.synth_frames_device(w, h, 1, S, 0, P + 1, content=p64_amd.SYNTH_SURVEY)
    rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    out = p64_amd.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"))
    for t in range(P + 1):
        p64_amd.encode_frames(fr[t].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li, width=w, height=h,
                              intra=(t == 0), quant=8, me_mode=p64_amd.ME_FULL, search_limit=31, out=out)
    gq = torch.full((S, 12), 8, dtype=torch.uint8, device="cuda")
    tr = torch.full((S,), P, dtype=torch.int32, device="cuda")
    bufs = p64s.vlc_buffers(S, w, h)
    for _ in range(5):  # warm (clocks, tables)
        p64s.vlc_pictures(out.mb, out.coef, gq, tr, width=w, height=h, buffers=bufs, host_bits=False)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    p64s.vlc_pictures(out.mb, out.coef, gq, tr, width=w, height=h, buffers=bufs, host_bits=False)
    b.record()
    torch.cuda.synchronize()
    nw = S * 10 * 4
    st = np.zeros(8 * nw, np.uint64)
    L = p64_amd.lib()
    assert L.p64dbg_vlc_stamps(ctypes.c_void_p(st.ctypes.data), ctypes.c_size_t(st.size)) == 0
    st = st.reshape(nw, 8)
    xcd = (st[:, 0] >> np.uint64(56)).astype(int)
    t = (st & np.uint64((1 << 56) - 1)).astype(np.int64)
    t0 = t[:, 0].min()
    t = (t - t0) * 10  # ns (100 MHz)
    print(f"launch (events) {a.elapsed_time(b) * 1e3:.1f} us; stamped span {t[:, 7].max() / 1e3:.1f} us; "
          f"{nw} waves")
    names = ["loads", "tables+barrier", "count", "emit(LDS)", "look-back+barrier", "assembly+stores", "tail"]
    ok = (t[:, 7] > 0) & (t[:, 6] > 0)
    print(f"waves with all stamps: {ok.sum()}")
    for k, nm in enumerate(names):
        d = (t[ok, k + 1] - t[ok, k]) / 1e3
        print(f"  {nm:20s} p10 {np.percentile(d, 10):6.2f}  p50 {np.percentile(d, 50):6.2f}  "
              f"p90 {np.percentile(d, 90):6.2f}  mean {d.mean():6.2f} us")
    life = (t[ok, 7] - t[ok, 0]) / 1e3
    print(f"  lifetime             p10 {np.percentile(life, 10):6.2f}  p50 {np.percentile(life, 50):6.2f}  "
          f"p90 {np.percentile(life, 90):6.2f}  mean {life.mean():6.2f} us")
    starts = np.sort(t[:, 0]) / 1e3
    for q in (0, 10, 25, 50, 75, 90, 100):
        print(f"  wave start p{q:3d}: {np.percentile(starts, q):6.1f} us")
    span = t[:, 7].max()
    print("  resident waves (and in each phase) over the launch:")
    for f in np.linspace(0.02, 0.98, 13):
        x = f * span
        res = ((t[:, 0] <= x) & (t[:, 7] > x)).sum()
        ph = [((t[:, k] <= x) & (t[:, k + 1] > x)).sum() for k in range(7)]
        print(f"    {x / 1e3:6.1f} us: {res:5d}  " + " ".join(f"{n[:6]}={p}" for n, p in zip(names, ph)))
    print("  waves per XCD:", np.bincount(xcd, minlength=8).tolist())
    # look-back: workgroups by index within the picture
    G = (np.arange(nw) // 4) % 10
    for g in (0, 1, 5, 9):
        m = ok & (G == g) & (np.arange(nw) % 4 == 0)
        d = (t[m, 5] - t[m, 4]) / 1e3
        print(f"  look-back wave 0, workgroup {g} of its picture: p50 {np.percentile(d, 50):.2f} "
              f"p90 {np.percentile(d, 90):.2f} us")


if __name__ == "__main__":
    main()
