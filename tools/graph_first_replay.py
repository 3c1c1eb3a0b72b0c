"""Probe (GPU box): host wall time of the first and later replays of one
captured graph of K intra launches (bench.py's timed region replays a graph
once, right after its capture and the spin-up of another graph)."""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch  # noqa: E402

import p64_amd  # noqa: E402

w, h, S, K = 352, 288, 256, 20
nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
frames = p64_amd.synth_frames_device(w, h, 1, S, 0, K)
rec = torch.empty(S * pic, dtype=torch.uint8, device="cuda")
li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                            mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"), me=None)


def step(t):
    p64_amd.encode_frames(frames[t].reshape(-1), None, rec, li, width=w, height=h, intra=True, out=out)


for t in range(3):
    step(t)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for t in range(K):
        step(t)
torch.cuda.synchronize()
# spin: 50 eager launches to raise the clocks
for t in range(200):
    step(t % K)
torch.cuda.synchronize()
for r in range(4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"replay {r}: wall {wall * 1e6 / K:.2f} us/step, events {e0.elapsed_time(e1) * 1e3 / K:.2f} us/step", flush=True)
