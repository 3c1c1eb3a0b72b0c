"""Wave timeline of the block-layout intra kernel (development aid).

Needs a library built with -DP64_TIMING: every wave of k_intra_blk stores its
start and end s_memrealtime (100 MHz), its s_memtime cycles and its hardware
id.  Prints how many waves are resident over time, the mean wave lifetime and
the shader clock the waves saw (cycles / real time)."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import p64_amd  # noqa: E402

w, h, S = 352, 288, 256
nmb = (w // 16) * (h // 16)
pic = w * h * 3 // 2
fr = p64_amd.synth_frames_device(w, h, 1, S, 0, 4)
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
rec = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                            mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"), me=None)
nw = S * nmb * 6 // 64
buf = torch.zeros(nw * 32, dtype=torch.int32, device="cuda")
lib = p64_amd.lib()
lib.p64gpu_dbg_phase_buffer(ctypes.c_void_p(buf.data_ptr()))
for t in range(4):
    buf.zero_()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    p64_amd.encode_frames(fr[t].reshape(-1), None, rec, li, width=w, height=h, intra=True, out=out)
    ev[1].record()
    torch.cuda.synchronize()
b = buf.cpu().numpy().view(np.uint32)[: nw * 8].reshape(nw, 8).astype(np.int64)
b = b[b[:, 1] > 0]
r0, r1, cyc = b[:, 0], b[:, 1], b[:, 2]
t0 = r0.min()
life = (r1 - r0) / 100.0  # us
print(f"kernel (events) {ev[0].elapsed_time(ev[1]) * 1e3:.1f} us; waves stamped {len(b)}; "
      f"span {(r1.max() - t0) / 100:.1f} us")
print(f"wave lifetime us: mean {life.mean():.2f}  p10 {np.percentile(life, 10):.2f}  "
      f"p90 {np.percentile(life, 90):.2f}")
if (b[:, 3] > 0).all():
    rl, rc = b[:, 3], b[:, 4]
    print(f"phases us (mean): loads {((rl - r0) / 100).mean():.2f}  compute {((rc - rl) / 100).mean():.2f}  "
          f"store issue {((r1 - rc) / 100).mean():.2f}")
print(f"shader clock seen by the waves: {np.median(cyc / (r1 - r0) / 10):.3f} GHz")
for us in range(0, int((r1.max() - t0) / 100) + 2, 2):
    t = t0 + us * 100
    live = ((r0 <= t) & (r1 > t)).sum()
    started = (r0 <= t).sum()
    print(f"t={us:3d} us  resident {live:6d}  started {started:6d}")
