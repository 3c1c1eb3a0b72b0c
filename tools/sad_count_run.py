"""Executed v_sad_u8 work of k_motion on the bench workload (GPU box; counted
side build of tools/sad_count.py): P64GPU_LIB=abtest/lib_sadcount.so python
tools/sad_count_run.py [--steps K --warmup W --content C --mode full|tss].
Runs the bench's closed loop (S = 256 CIF sequences, the bench's inputs) and
prints one JSON object: per timed picture the executed lane-instructions of
v_sad_u8, the byte-absolute-differences they did (x 4) per launch and per MB,
and the mean over the timed pictures (bench.py reads it from
profiles/sad_executed.json as `executed_sad`)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

import bench  # noqa: E402
import p64_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--content", default="synth")
ap.add_argument("--mode", default="full")
ap.add_argument("--search-limit", type=int, default=31)
ap.add_argument("--streams", type=int, default=256)
a = ap.parse_args()
L = p64_amd.lib()
L.p64dbg_sadcnt_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
w, h, S = 352, 288, a.streams
nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
nslots = min(1 + a.warmup + a.steps, bench.MAX_SLOTS)
frames = bench.make_inputs(torch, p64_amd, a.content, w, h, 1, S, nslots)
rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                            mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                            me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"))
mode = p64_amd.ME_FULL if a.mode == "full" else p64_amd.ME_TSS
buf = np.zeros(S * nmb * 64, np.uint32)
per = []
for t in range(1 + a.warmup + a.steps):
    torch.cuda.synchronize()
    assert L.p64dbg_sadcnt_clear() == 0
    p64_amd.encode_frames(frames[t % nslots].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li, width=w,
                          height=h, intra=(t == 0), quant=8, me_mode=mode, search_limit=a.search_limit,
                          out=out)
    torch.cuda.synchronize()
    assert L.p64dbg_sadcnt_read(buf.ctypes.data, buf.size) == 0
    if t > a.warmup:
        per.append(int(buf.sum(dtype=np.uint64)))
mbs = S * nmb
mean = float(np.mean(per))
print(json.dumps({"workload": f"{w}x{h} {a.mode.upper()} SL={a.search_limit}, content {a.content}, "
                              f"S={S}, pictures {a.warmup + 1}..{a.warmup + a.steps}",
                  "v_sad_u8_lane_instr_per_launch": per,
                  "mean_lane_instr_per_launch": mean,
                  "byte_absdiff_per_launch": 4 * mean,
                  "byte_absdiff_per_mb": 4 * mean / mbs,
                  "exhaustive_equivalent_per_mb": (2 * (a.search_limit // 2)) ** 2 * 256
                  if a.mode == "full" else None}))
