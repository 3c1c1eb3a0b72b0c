"""HIP-graph capture probes (development aid, GPU box): which two-stream
capture patterns torch + HIP (ROCm 7) accept, to name the cause of the
round-4 `capture_end` segfault.  One pattern per process:
    python tools/capture_probe.py <mode>
modes:
  joined      fork onto a side stream (side.wait_stream(capture stream)),
              work on both, join back (capture.wait_stream(side)) before the
              capture ends -- the legal fork/join
  unjoined    the same without the join: the side stream's work is still
              part of the capture when it ends
  external    the side stream waits on an event recorded BEFORE the capture
              began (a dependency from outside the graph)
  null_launch a library launch on the NULL stream while another stream
              captures (global capture mode)
  unforked    work on a side stream that never waited on the capture stream
  lib_side    the library's inter encode with args->me == NULL on a side
              stream forked from the capture stream and joined back (under
              capture: the fused-kernel path, no library scratch), replayed:
              results equal the eager call (split kernels, library scratch)
Prints "<mode> ok ..." or raises; a segfault shows as the process's
signal in the caller's exit status."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402


def work(x, k):
    for _ in range(k):
        x.mul_(2).add_(1)


def main(mode):
    torch.cuda.set_device(0)
    cap = torch.cuda.Stream()
    side = torch.cuda.Stream()
    a = torch.zeros(1 << 20, device="cuda")
    b = torch.zeros(1 << 20, device="cuda")
    torch.cuda.synchronize()
    if mode == "lib_side":
        import numpy as np
        import p64_amd
        w, h, S = 176, 144, 4
        nmb, pic = 99, w * h * 3 // 2
        fr = p64_amd.synth_frames_device(w, h, 1, S, 0, 2, content=p64_amd.SYNTH_SURVEY)
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
        p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True)
        li0 = li.clone()
        outs = []
        for graph in (False, True):
            r1 = torch.zeros_like(r0)
            li.copy_(li0)
            o = p64_amd.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                      mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"), me=None)
            torch.cuda.synchronize()

            def call():
                # the Python mirror passes its own ME buffer unless want_me is False and
                # me is None: go through the raw ABI with args->me == NULL
                a_ = p64_amd.EncodeArgs(width=w, height=h, nframes=S, intra=0, quant=8, me_mode=p64_amd.ME_FULL,
                                        search_limit=31, flags=0, frame_stride=pic, cur=fr[1].data_ptr(),
                                        ref=r0.data_ptr(), recon=r1.data_ptr(), last_intra=li.data_ptr(),
                                        coef=o.coef.data_ptr(), mb=o.mb.data_ptr(), me=None)
                import ctypes
                st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
                assert p64_amd.lib().p64gpu_encode_frames(ctypes.byref(a_), st) == 0
            if graph:  # forked from the capture stream onto `side`, joined back
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cap):
                    side.wait_stream(cap)
                    with torch.cuda.stream(side):
                        call()
                    cap.wait_stream(side)
                torch.cuda.synchronize()
                li.copy_(li0)
                g.replay()
            else:
                call()
            torch.cuda.synchronize()
            outs.append((o.coef.cpu(), o.mb.cpu(), r1.cpu()))
        assert all(torch.equal(x, y) for x, y in zip(*outs)), "graph replay differs from the eager call"
        print("lib_side ok", flush=True)
        return
    if mode == "null_launch":  # a library launch on the NULL stream during another stream's capture
        import ctypes
        import p64_amd
        x = torch.zeros(64 * 64, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            work(a, 1)
            rc = p64_amd.lib().p64gpu_block_op(0, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                               64, 8, 8, None)
            print(f"null_launch: block_op on the NULL stream returned {rc}: "
                  f"{p64_amd.lib().p64gpu_last_error().decode()}", flush=True)
        print("null_launch: capture ended", flush=True)
        g.replay()
        torch.cuda.synchronize()
        print("null_launch ok", flush=True)
        return
    if mode == "unforked":  # a side stream that never waited on the capture stream
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            work(a, 1)
            with torch.cuda.stream(side):
                work(b, 1)
        print("unforked: capture ended", flush=True)
        g.replay()
        torch.cuda.synchronize()
        print(f"unforked ok {float(a[0])} {float(b[0])}", flush=True)
        return
    ev_before = torch.cuda.Event()
    if mode == "external":
        with torch.cuda.stream(side):
            work(b, 1)
            ev_before.record(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        work(a, 3)
        if mode in ("joined", "unjoined"):
            side.wait_stream(cap)
            with torch.cuda.stream(side):
                work(b, 3)
            if mode == "joined":
                cap.wait_stream(side)
        elif mode == "external":
            cap.wait_event(ev_before)
            work(a, 1)
    print(f"{mode}: capture ended", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"{mode} ok {float(a[0])} {float(b[0])}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
