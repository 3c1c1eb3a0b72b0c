"""Per-phase wall cycles of the fused FULL encode kernel (development aid).

Needs a library built with -DP64_TIMING (every SECTION() of k_search.hip stores
the wave's s_memtime offset).  Runs the kbench workload (256 CIF sequences,
pictures 1..3 after an intra picture) and prints, per phase, the mean cycles a
macroblock's wave spends between that SECTION and the next one it reaches:
residency time (it includes waiting for issue slots behind the SIMD's other
waves), so shares, not absolute costs, are the useful part.
"""
import ctypes
import os
import re
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import p64_amd  # noqa: E402

src = open(os.path.join(REPO, "p64_amd/csrc/k_search.hip")).read()
names = re.findall(r'^\s*SECTION\("([^"]+)"\);', src, re.M)
names = names + ["?"] * (31 - len(names)) + ["end"]
w, h, S = 352, 288, 256
nmb = (w // 16) * (h // 16)
pic = w * h * 3 // 2
fr = p64_amd.synth_frames_device(w, h, 1, S, 0, 4)
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                            mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                            me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"))
buf = torch.zeros(S * nmb * 32, dtype=torch.int32, device="cuda")
lib = p64_amd.lib()
lib.p64gpu_dbg_phase_buffer(ctypes.c_void_p(buf.data_ptr()))
p64_amd.encode_frames(fr[0].reshape(-1), None, rec[0], li, width=w, height=h, intra=True, out=out)
acc = {}
for t in (1, 2, 3):
    buf.zero_()
    p64_amd.encode_frames(fr[t].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li, width=w, height=h,
                          intra=False, me_mode=p64_amd.ME_FULL, search_limit=31, out=out)
    torch.cuda.synchronize()
    b = buf.cpu().numpy().view(np.uint32).reshape(-1, 32).astype(np.int64)
    for k in range(31):
        col = b[:, k]
        hit = col > 0
        if not hit.any():
            continue
        # the next stamp this wave reached after k
        later = np.where((b > col[:, None]) & hit[:, None], b, np.iinfo(np.int64).max).min(axis=1)
        d = np.where(hit, later - col, 0)
        acc[k] = acc.get(k, 0) + d.sum()
    first = np.where(b[:, :31] > 0, b[:, :31], np.iinfo(np.int64).max).min(axis=1)
    acc[-1] = acc.get(-1, 0) + first.sum()
tot = sum(acc.values())
n = 3 * S * nmb
print(f"{'phase':14s} {'cycles/MB':>10s} {'share':>7s}")
for k in sorted(acc, key=lambda k: -acc[k]):
    nm = "start" if k < 0 else names[k]
    print(f"{nm:14s} {acc[k] / n:10.0f} {acc[k] / tot:7.1%}")
print(f"{'total':14s} {tot / n:10.0f}")
