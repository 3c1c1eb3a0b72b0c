#!/usr/bin/env python3
"""Times the GPU entropy coder (k_vlc_blk) on the bench's records (GPU box;
development aid): 256 CIF sequences of survey content encoded closed loop
(FULL SL=31, q=8) to picture P, then the coder over picture P's records --
count-only (VLC_COUNT), one pass counting itself (VLC_ONE) and with the
encoder's counts (VLC_GIVEN) -- each N times back to back, bracketed by HIP
events on the launching stream.  Prints one JSON line per library.

    python3 tools/vlc_time.py [--libs a.so b.so ...] [--pictures P] [--reps N]

With --libs, each library is timed in a child process of its own (P64GPU_LIB)
and the coded bits are compared with the first library's."""
import argparse
import ctypes
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(args):
    import hashlib

    import torch

    import p64_amd
    from p64_amd import stream as p64s
    w, h, S, nmb = 352, 288, 256, 396
    pic = w * h * 3 // 2
    P = args.pictures
    fr = p64_amd.synth_frames_device(w, h, 1, S, 0, P + 1, content=p64_amd.CONTENTS[args.content])
    rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    out = p64_amd.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"),
                                vlc_bits=torch.zeros((S, nmb, 8), dtype=torch.int16, device="cuda"))
    for t in range(P + 1):
        p64_amd.encode_frames(fr[t].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li, width=w, height=h,
                              intra=(t == 0), quant=8, me_mode=p64_amd.ME_FULL, search_limit=31, out=out)
    gq = torch.full((S, 12), 8, dtype=torch.uint8, device="cuda")
    tr = torch.full((S,), P % 32, dtype=torch.int32, device="cuda")
    bufs = p64s.vlc_buffers(S, w, h)
    L = p64_amd.lib()
    cnt = torch.zeros((S, nmb, 8), dtype=torch.int16, device="cuda")
    res = {"lib": os.path.basename(p64_amd.LIB_PATH), "content": args.content, "picture": P}

    def one():
        p64s.vlc_pictures(out.mb, out.coef, gq, tr, width=w, height=h, buffers=bufs, host_bits=False)

    def given():
        p64s.vlc_pictures(out.mb, out.coef, gq, tr, width=w, height=h, buffers=bufs, host_bits=False,
                          blk_bits=out.vlc_bits)

    def count():
        p64_amd._check(L.p64gpu_vlc_block_bits_(w, h, S, ctypes.c_void_p(out.mb.data_ptr()),
                                                ctypes.c_void_p(out.coef.data_ptr()),
                                                ctypes.c_void_p(cnt.data_ptr()), p64_amd._stream(torch)))
    L.p64gpu_vlc_block_bits_.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    for name, fn in (("count", count), ("one", one), ("given", given)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(a.elapsed_time(b) * 1e3 / args.reps, 2)
        if name != "count":
            bits = bufs[1][:S].cpu().numpy()
            o = bufs[0].cpu().numpy()
            hsh = hashlib.sha256(bits.tobytes())
            for i in range(S):
                hsh.update(o[i, :(int(bits[i]) + 7) // 8].tobytes())
            res[name + "_sha"] = hsh.hexdigest()[:16]
            res["bits_per_mb"] = round(float(bits.astype("int64").sum()) / (S * nmb), 1)
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="*", default=[])
    ap.add_argument("--pictures", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--content", default="survey")
    args = ap.parse_args()
    if not args.libs:
        run(args)
        return
    ref = None
    for lib in args.libs:
        env = dict(os.environ, P64GPU_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--pictures", str(args.pictures),
                            "--reps", str(args.reps), "--content", args.content],
                           env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:], file=sys.stderr)
            raise SystemExit(f"{lib}: exit {r.returncode}")
        d = json.loads(r.stdout.strip().splitlines()[-1])
        if ref is None:
            ref = d
        d["same_bits"] = d.get("one_sha") == ref.get("one_sha") and d.get("given_sha") == ref.get("given_sha")
        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
