"""GPU parity: the HIP path (through the C ABI) against the golden fixtures and
the pinned CPU oracle, bit-exact.  Run on an MI355X with `pytest -m gpu`."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_oracle_golden import (SEQS, check_sequence_outputs, load, sequence_frames, sequence_params,
                                tie_mbs)

pytestmark = pytest.mark.gpu


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.cpu().numpy()


# ---------------------------------------------------------------------------
# block routines (chendct.c / transform.c)

def test_block_ops_golden(p64, torch_dev):
    torch = torch_dev
    z = load("blocks.npz")
    np.testing.assert_array_equal(host(p64.ChenDct(dev(torch, z["dct_in"]))), z["dct_out"])
    np.testing.assert_array_equal(host(p64.ChenIDct(dev(torch, z["idct_in"]))), z["idct_out"])
    b = dev(torch, z["bound_in"])
    np.testing.assert_array_equal(host(p64.BoundDctMatrix(b)), z["bound_dct"])
    np.testing.assert_array_equal(host(p64.BoundIDctMatrix(b)), z["bound_idct"])
    np.testing.assert_array_equal(host(p64.FlatBoundQuantizeMatrix(b)), z["bound_qflat"])
    np.testing.assert_array_equal(host(p64.BoundQuantizeMatrix(b)), z["bound_quant"])
    zz = dev(torch, z["zz_in"])
    np.testing.assert_array_equal(host(p64.ZigzagMatrix(zz)), z["zz_out"])
    np.testing.assert_array_equal(host(p64.IZigzagMatrix(zz)), z["izz_out"])
    qin = dev(torch, z["quant_in"])
    for q in range(1, 32):
        np.testing.assert_array_equal(host(p64.CCITTQuantize(qin, q, q)), z[f"inter_q{q}"])
        np.testing.assert_array_equal(host(p64.CCITTFlatQuantize(qin, 8, q)), z[f"intra_q{q}"])
        lv = dev(torch, z[f"ilev_q{q}"])
        np.testing.assert_array_equal(host(p64.ICCITTQuantize(lv, q, q)), z[f"iinter_q{q}"])
        np.testing.assert_array_equal(host(p64.ICCITTFlatQuantize(lv, 8, q)), z[f"iintra_q{q}"])


def test_block_ops_random_vs_oracle(p64, oracle_mod, torch_dev):
    torch = torch_dev
    rng = np.random.default_rng(7)
    x = rng.integers(-255, 256, (4096, 64)).astype(np.int32)
    np.testing.assert_array_equal(host(p64.ChenDct(dev(torch, x))), oracle_mod.block_apply("orc_chen_dct", x))
    y = rng.integers(-7905, 7906, (4096, 64)).astype(np.int32)
    np.testing.assert_array_equal(host(p64.ChenIDct(dev(torch, y))), oracle_mod.block_apply("orc_chen_idct", y))


def test_empty_batch(p64, torch_dev):
    torch = torch_dev
    e = torch.empty((0, 64), dtype=torch.int32, device="cuda")
    assert p64.ChenDct(e).shape == (0, 64)


# ---------------------------------------------------------------------------
# motion estimation (me.c)

@pytest.mark.parametrize("key,mode,sl", [("full31", 1, 31), ("full15", 1, 15), ("full7", 1, 7),
                                         ("tss", 0, 15)])
def test_motion_estimation_golden(p64, torch_dev, key, mode, sl):
    torch = torch_dev
    z = load("me.npz")
    w, h = int(z["width"]), int(z["height"])
    n = z["ref"].shape[0]
    # batch every case into one launch: each luma plane is its own "picture"
    ref = dev(torch, z["ref"].reshape(n, w * h))
    cur = dev(torch, z["cur"].reshape(n, w * h))
    got = host(p64.MotionEstimation(ref, cur, w, h, mode=mode, search_limit=sl, frame_stride=w * h))
    for i, name in enumerate(z["names"]):
        np.testing.assert_array_equal(got[i], z[key][i], err_msg=f"{key} case {name}")


def test_motion_estimation_random_cif_vs_oracle(p64, oracle_mod, torch_dev):
    torch = torch_dev
    w, h = 352, 288
    rng = np.random.default_rng(11)
    frames = [p64.synth_frame(s, 3, w, h) for s in (1, 2)] + \
        [rng.integers(0, 256, w * h * 3 // 2, dtype=np.uint8)]
    prevs = [p64.synth_frame(s, 2, w, h) for s in (1, 2)] + \
        [rng.integers(0, 256, w * h * 3 // 2, dtype=np.uint8)]
    cur = dev(torch, np.stack(frames))
    ref = dev(torch, np.stack(prevs))
    for mode, sl in ((1, 31), (0, 15)):
        got = host(p64.MotionEstimation(ref, cur, w, h, mode=mode, search_limit=sl))
        for i in range(len(frames)):
            exp = oracle_mod.motion_estimation(prevs[i][: w * h], frames[i][: w * h], w, h, mode, sl)
            exp = np.stack([exp[f] for f in exp.dtype.names], axis=1)
            np.testing.assert_array_equal(got[i], exp, err_msg=f"mode {mode} frame {i}")


def _adversarial_pictures(w, h):
    """Luma planes that stress the pruned full search (me_full): ties, flat and
    low-contrast blocks on both sides of the dense-path threshold, periodic
    patterns, ramps, saturated blocks, plain noise."""
    rng = np.random.default_rng(2026)
    y, x = np.mgrid[0:h, 0:w]
    out = []
    tex = rng.integers(0, 256, (h, w)).astype(np.int32)
    # periodic in x and y (exact ties at every multiple of the period)
    for px, py in ((4, 4), (8, 2), (3, 5)):
        base = rng.integers(0, 256, (py, px))
        out.append(base[y % py, x % px])
    # low contrast around the dense-path threshold (sub-block ranges ~4..24)
    for amp in (3, 6, 10, 16):
        out.append(128 + (tex * amp) // 255 - amp // 2)
    out.append((x * 255) // (w - 1))                  # ramp
    out.append(np.where((x // 16 + y // 16) % 2 == 0, 0, 255))  # saturated checkerboard
    out.append(tex)                                   # noise
    mixed = tex.copy()
    mixed[:, : w // 2] = 77
    out.append(mixed)                                 # half flat, half noise
    return [np.clip(p, 0, 255).astype(np.uint8).reshape(-1) for p in out]


@pytest.mark.parametrize("w,h", [(352, 288), (176, 144)])
def test_full_search_adversarial_vs_oracle(p64, oracle_mod, torch_dev, w, h):
    """The lower-bound pruning must never change FastBME's answer (me.c:187-246):
    each picture against a shifted-and-noised copy of itself and against an
    unrelated picture, every search limit class."""
    torch = torch_dev
    rng = np.random.default_rng(7)
    pics = _adversarial_pictures(w, h)
    refs, curs = [], []
    for p in pics:
        img = p.reshape(h, w).astype(np.int32)
        dy, dx = rng.integers(-9, 10, 2)
        shifted = np.roll(np.roll(img, dy, 0), dx, 1) + rng.integers(-2, 3, img.shape)
        refs.append(np.clip(shifted, 0, 255).astype(np.uint8).reshape(-1))
        curs.append(p)
    refs.append(pics[0])
    curs.append(pics[-1])
    cur = dev(torch, np.stack(curs))
    ref = dev(torch, np.stack(refs))
    for sl in (31, 15, 7, 2):
        got = host(p64.MotionEstimation(ref, cur, w, h, mode=1, search_limit=sl, frame_stride=w * h))
        for i in range(len(curs)):
            exp = oracle_mod.motion_estimation(refs[i], curs[i], w, h, 1, sl)
            exp = np.stack([exp[f] for f in exp.dtype.names], axis=1)
            np.testing.assert_array_equal(got[i], exp, err_msg=f"sl {sl} picture {i}")


def test_search_windows_at_picture_edges_vs_oracle(p64, oracle_mod, torch_dev):
    """The search window is fetched without bounds tests (k_search.hip
    fetch_luma): left/right of the picture it holds the neighbouring rows'
    pixels, above/below zeros.  Edge MBs whose current block equals exactly
    that wrapped or zero data (a perfect, but invalid, match at dx/dy beyond
    the picture) must still get FastBME's answer over the valid candidates
    (me.c:206-212), in every search mode."""
    torch = torch_dev
    w, h = 176, 144
    rng = np.random.default_rng(99)
    refs, curs = [], []
    for k in range(3):
        ref = rng.integers(0, 256, w * h, dtype=np.uint8)
        cur = rng.integers(0, 256, (h, w), dtype=np.uint8)
        for mby in range(h // 16):
            y0 = 16 * mby
            for x0, d in ((0, -(3 + 4 * k)), (w - 16, 5 + 3 * k)):  # left: previous rows' ends, right: next rows' starts
                for r in range(16):
                    s = (y0 + r) * w + x0 + d
                    if 0 <= s and s + 16 <= w * h:
                        cur[y0 + r, x0:x0 + 16] = ref[s:s + 16]
        cur[0:16, 16:w - 16] = 0        # top row: a zero block matches the zeros above the picture
        cur[h - 16:h, 16:w - 16] = 0    # bottom row: and below it
        refs.append(ref)
        curs.append(cur.reshape(-1))
    cur_d = dev(torch, np.stack(curs))
    ref_d = dev(torch, np.stack(refs))
    for mode, sl in ((1, 31), (1, 15), (1, 7), (0, 31), (0, 15)):
        got = host(p64.MotionEstimation(ref_d, cur_d, w, h, mode=mode, search_limit=sl, frame_stride=w * h))
        for i in range(len(curs)):
            exp = oracle_mod.motion_estimation(refs[i], curs[i], w, h, mode, sl)
            exp = np.stack([exp[f] for f in exp.dtype.names], axis=1)
            np.testing.assert_array_equal(got[i], exp, err_msg=f"mode {mode} sl {sl} picture {i}")


# ---------------------------------------------------------------------------
# whole-encoder fixtures, through the batched device API and the host context

def run_device_sequence(p64, torch, frames, w, h, *, quant, me_mode, search_limit, mtype_override):
    """Closed loop through p64gpu_encode_frames, one stream."""
    nmb = (w // 16) * (h // 16)
    pic = w * h * 3 // 2
    li = torch.zeros(nmb, dtype=torch.uint8, device="cuda")
    bufs = [torch.zeros(pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    ov = dev(torch, mtype_override) if mtype_override is not None else None
    outs = []
    for t, f in enumerate(frames):
        cur = dev(torch, f)
        ref, rec = bufs[(t + 1) % 2], bufs[t % 2]
        o = p64.encode_frames(cur, ref, rec, li, width=w, height=h, intra=(t == 0), quant=quant,
                              me_mode=me_mode, search_limit=search_limit,
                              mtype_override=(ov if t > 0 else None))
        coef = host(o.coef)[0]
        mb = host(o.mb)[0].view(p64.MB_DTYPE).reshape(nmb)
        me = host(o.me)[0].view(p64.ME_DTYPE).reshape(nmb)
        outs.append((coef, mb, me, host(rec).copy()))
    return outs


@pytest.mark.parametrize("name", SEQS)
def test_sequence_golden_device(p64, torch_dev, name):
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    frames = sequence_frames(p64, z)
    outs = run_device_sequence(p64, torch_dev, frames, w, h, **sequence_params(z))
    check_sequence_outputs(z, outs, name)


@pytest.mark.parametrize("name", ["qcif_tie_full31", "qcif_tie_tss"])
def test_mtype_tie_branch_on_device(p64, torch_dev, name):
    """k_encode reaches the binary64 tie of the MTYPE decision (decide_mtype:
    11 MV == 10 OMV with VAR < 64, p64.c:745-756) on the constructed fixture
    and takes both outcomes exactly as the reference did: MTYPE 2 where the
    rounded x/1.1 falls below y, motion compensation (8) where it does not."""
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    outs = run_device_sequence(p64, torch_dev, sequence_frames(p64, z), w, h, **sequence_params(z))
    coef, mb, me, _ = outs[1]
    got = np.stack([me[f] for f in me.dtype.names], axis=1)
    np.testing.assert_array_equal(got, z["merec"][1])
    mbs = tie_mbs(z, 1)
    assert len(mbs) >= 4
    mt = mb["mtype"].astype(int)[mbs]
    np.testing.assert_array_equal(mt, z["mb"][1][mbs, 0])
    assert 2 in mt and 8 in mt
    check_sequence_outputs(z, outs, name)


@pytest.mark.parametrize("name", ["qcif_tss", "cif_full31", "qcif_intra", "qcif_flat_tss"])
def test_sequence_golden_host_context(p64, torch_dev, name):
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    prm = sequence_params(z)
    frames = sequence_frames(p64, z)
    enc = p64.Encoder(w, h, me_mode=prm["me_mode"], search_limit=prm["search_limit"])
    outs = []
    for t, f in enumerate(frames):
        ov = prm["mtype_override"] if t > 0 else None
        coef, mb, me, recon = enc.frame(f, intra=(t == 0), quant=prm["quant"], mtype_override=ov,
                                        want_recon=True)
        outs.append((coef, mb, me, recon))
    enc.close()
    check_sequence_outputs(z, outs, name)


# ---------------------------------------------------------------------------
# batched multi-stream closed loop vs the oracle (the bench's shape, smaller)

@pytest.mark.parametrize("w,h,me_mode,sl,q", [(352, 288, 1, 31, 8), (352, 288, 0, 15, 5),
                                             (704, 576, 1, 31, 12), (176, 144, 1, 15, 3),
                                             (352, 240, 1, 31, 31)])
def test_batched_streams_vs_oracle(p64, oracle_mod, torch_dev, w, h, me_mode, sl, q):
    torch = torch_dev
    nstreams, nframes = 4, 3
    seeds = [3 + 5 * s for s in range(nstreams)]
    nmb = (w // 16) * (h // 16)
    pic = w * h * 3 // 2
    frames = np.stack([[p64.synth_frame(s, t, w, h) for s in seeds] for t in range(nframes)])
    li = torch.zeros(nstreams * nmb, dtype=torch.uint8, device="cuda")
    bufs = [torch.zeros(nstreams * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    qmb = np.full((nstreams, nmb), q, np.uint8)
    qmb[1] = np.arange(nmb) % 31 + 1  # per-MB UseQuant on one stream
    qmb_d = dev(torch, qmb)
    got = []
    for t in range(nframes):
        cur = dev(torch, frames[t])
        ref, rec = bufs[(t + 1) % 2], bufs[t % 2]
        o = p64.encode_frames(cur, ref, rec, li, width=w, height=h, intra=(t == 0), quant=q,
                              me_mode=me_mode, search_limit=sl, quant_mb=qmb_d)
        got.append((host(o.coef), host(o.mb), host(o.me), host(rec).reshape(nstreams, pic)))
    for s in range(nstreams):
        li_o = np.zeros(nmb, np.uint8)
        ref = None
        for t in range(nframes):
            coef, mb, me, recon = oracle_mod.encode_frame(
                w, h, frames[t][s], ref, li_o, intra=(t == 0), quant=q, me_mode=me_mode,
                search_limit=sl, quant_mb=qmb[s])
            ref = recon
            g = got[t]
            np.testing.assert_array_equal(g[0][s], coef, err_msg=f"coef s{s} t{t}")
            np.testing.assert_array_equal(g[1][s].view(p64.MB_DTYPE).reshape(nmb), mb,
                                          err_msg=f"mb s{s} t{t}")
            if t > 0:
                np.testing.assert_array_equal(g[2][s].view(p64.ME_DTYPE).reshape(nmb), me,
                                              err_msg=f"me s{s} t{t}")
            np.testing.assert_array_equal(g[3][s], recon, err_msg=f"recon s{s} t{t}")


def test_split_encoder_without_me_output_and_in_graph(p64, torch_dev):
    """Inter pictures without an ME-record output run k_motion into the
    library's scratch buffer: same levels, records and reconstruction as with
    the output; and the same again when the launches are captured into a HIP
    graph after one eager call (the scratch then exists outside the capture)."""
    torch = torch_dev
    w, h, S, T = 352, 288, 3, 3
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    frames = np.stack([[p64.synth_frame(11 + s, t, w, h) for s in range(S)] for t in range(T)])

    def run(want_me, graph=False):
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        bufs = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
        cur = [dev(torch, frames[t]) for t in range(T)]
        outs = [p64.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                  mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                  me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda")
                                  if want_me else None) for _ in range(T)]

        def step(t):
            p64.encode_frames(cur[t], bufs[(t + 1) % 2], bufs[t % 2], li, width=w, height=h,
                              intra=(t == 0), quant=8, me_mode=p64.ME_FULL, search_limit=31,
                              out=outs[t])
        step(0)
        if graph:
            step(1)  # eager inter call: the scratch is allocated here
            li.zero_()
            step(0)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for t in range(1, T):
                    step(t)
            g.replay()
        else:
            for t in range(1, T):
                step(t)
        torch.cuda.synchronize()
        return [(host(o.coef), host(o.mb)) for o in outs], host(bufs[(T - 1) % 2])

    ref_outs, ref_rec = run(True)
    for graph in (False, True):
        outs, rec = run(False, graph)
        for t in range(T):
            np.testing.assert_array_equal(outs[t][0], ref_outs[t][0], err_msg=f"coef t{t} graph={graph}")
            np.testing.assert_array_equal(outs[t][1], ref_outs[t][1], err_msg=f"mb t{t} graph={graph}")
        np.testing.assert_array_equal(rec, ref_rec)


@pytest.mark.parametrize("mode,sl", [(1, 31), (1, 15), (0, 15)])
def test_encode_with_given_me_records(p64, torch_dev, mode, sl):
    """P64GPU_FLAG_ME_GIVEN: the reference's own order -- MotionEstimation
    for the picture (me.c:340) as its own call, then the MDU loop reading the
    records (p64.c:734-756) -- gives the same levels, records and
    reconstructions as the encode that runs the search itself."""
    torch = torch_dev
    w, h, S, T = 352, 288, 3, 4
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    frames = [dev(torch, np.stack([p64.synth_frame(21 + s, t, w, h) for s in range(S)])).reshape(-1)
              for t in range(T)]

    def run(given):
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        bufs = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
        got = []
        for t in range(T):
            ref, rec = bufs[t % 2], bufs[(t + 1) % 2]
            o = p64.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                  mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                  me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"))
            if given and t > 0:
                o.me.copy_(p64.MotionEstimation(ref, frames[t], w, h, mode=mode, search_limit=sl))
            p64.encode_frames(frames[t], ref, rec, li, width=w, height=h, intra=(t == 0), quant=8,
                              me_mode=mode, search_limit=sl, out=o, me_given=given and t > 0)
            torch.cuda.synchronize()
            got.append((host(o.coef), host(o.mb), host(o.me) if t > 0 else None, host(rec)))
        return got

    for t, (a, b) in enumerate(zip(run(False), run(True))):
        for x, y in zip(a, b):
            if x is not None:
                np.testing.assert_array_equal(x, y, err_msg=f"picture {t}")


@pytest.mark.parametrize("mode,sl", [(1, 31), (0, 15)])
def test_encode_in_two_halves(p64, torch_dev, mode, sl):
    """P64GPU_FLAG_SEARCH_ONLY then P64GPU_FLAG_ME_GIVEN over the same
    arguments (prepare_encode's launches, as bench.py's with_vlc issues them)
    is the encode: levels, records, ME vectors and SADs, reconstruction, over
    a closed loop of 4 pictures."""
    torch = torch_dev
    w, h, S, T = 352, 288, 3, 4
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    frames = [dev(torch, np.stack([p64.synth_frame(31 + s, t, w, h) for s in range(S)])).reshape(-1)
              for t in range(T)]

    def run(halves):
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        bufs = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
        got = []
        for t in range(T):
            ref, rec = bufs[t % 2], bufs[(t + 1) % 2]
            o = p64.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                  mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                  me=torch.zeros((S, nmb, 7), dtype=torch.int32, device="cuda"))
            kw = dict(width=w, height=h, intra=(t == 0), quant=8, me_mode=mode, search_limit=sl, out=o)
            if halves and t > 0:
                p64.prepare_encode(frames[t], ref, rec, li, search_only=True, **kw)()
                p64.prepare_encode(frames[t], ref, rec, li, me_given=True, **kw)()
            else:
                p64.encode_frames(frames[t], ref, rec, li, **kw)
            torch.cuda.synchronize()
            got.append((host(o.coef), host(o.mb), host(o.me) if t > 0 else None, host(rec)))
        return got

    for t, (a, b) in enumerate(zip(run(False), run(True))):
        for x, y in zip(a, b):
            if x is not None:
                np.testing.assert_array_equal(x, y, err_msg=f"picture {t}")


def _raw_encode(p64, torch, cur, ref, recon, li, coef, mb, *, w, h, stream, me=None):
    """p64gpu_encode_frames straight through the C ABI (me = NULL unless given)."""
    import ctypes
    nframes = cur.numel() // p64.picture_bytes(w, h)
    a = p64.EncodeArgs(width=w, height=h, nframes=nframes, intra=0, quant=8, me_mode=p64.ME_FULL,
                       search_limit=31, flags=0, frame_stride=p64.picture_bytes(w, h),
                       cur=cur.data_ptr(), ref=ref.data_ptr(), recon=recon.data_ptr(),
                       last_intra=li.data_ptr(), quant_mb=None, mtype_override=None,
                       coef=coef.data_ptr(), mb=mb.data_ptr(),
                       me=(me.data_ptr() if me is not None else None))
    st = ctypes.c_void_p(stream.cuda_stream)
    assert p64.lib().p64gpu_encode_frames(ctypes.byref(a), st) == 0, p64.lib().p64gpu_last_error()


def test_library_me_scratch_per_stream_and_graph_safe(p64, torch_dev):
    """Inter encodes without an ME-record output (args.me == NULL) keep their
    records in a library scratch private to the calling stream: two batches
    encoded concurrently on two streams give their own results; a graph
    captured on a stream with a scratch takes the fused kernel (a graph never
    points at library scratch) and replays the same results after the
    scratch has grown.  ADVICE r02 (high), r03 (medium)."""
    torch = torch_dev
    w, h = 352, 288
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2

    def batch(seed, S):
        f = [dev(torch, np.stack([p64.synth_frame(seed + s, t, w, h) for s in range(S)])).reshape(-1)
             for t in range(2)]
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
        p64.encode_frames(f[0], None, r0, li, width=w, height=h, intra=True, quant=8)
        torch.cuda.synchronize()
        return f[1], r0, li

    def outputs(S):
        return (torch.empty(S * pic, dtype=torch.uint8, device="cuda"),
                torch.zeros(S * nmb, dtype=torch.uint8, device="cuda"),
                torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"))

    def expected(cur, ref, li, S):
        rec, li2, coef, mb = outputs(S)
        li2.copy_(li)
        me = torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda")
        _raw_encode(p64, torch, cur, ref, rec, li2, coef, mb, w=w, h=h,
                    stream=torch.cuda.current_stream(), me=me)
        torch.cuda.synchronize()
        return host(rec), host(coef), host(mb)

    cur_a, ref_a, li_a = batch(101, 4)
    cur_b, ref_b, li_b = batch(202, 4)
    exp_a, exp_b = expected(cur_a, ref_a, li_a, 4), expected(cur_b, ref_b, li_b, 4)

    # two streams, interleaved launches, both through the scratch
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    oa, ob = outputs(4), outputs(4)
    for _ in range(3):
        for (cur, ref, li, o, st) in ((cur_a, ref_a, li_a, oa, s1), (cur_b, ref_b, li_b, ob, s2)):
            o[1].copy_(li)
            torch.cuda.synchronize()
            with torch.cuda.stream(st):
                _raw_encode(p64, torch, cur, ref, o[0], o[1], o[2], o[3], w=w, h=h, stream=st)
    torch.cuda.synchronize()
    for o, e in ((oa, exp_a), (ob, exp_b)):
        for got, want in zip((host(o[0]), host(o[2]), host(o[3])), e):
            np.testing.assert_array_equal(got, want)

    # graph captured with the stream's scratch at 1 picture, then the scratch
    # grows (an eager 4-picture call on the same stream), then the replay
    s3 = torch.cuda.Stream()
    one = outputs(1)
    cur1, ref1 = cur_a[:pic], ref_a[:pic]
    with torch.cuda.stream(s3):
        one[1].copy_(li_a[:nmb])
        _raw_encode(p64, torch, cur1, ref1, one[0], one[1], one[2], one[3], w=w, h=h, stream=s3)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s3):
        _raw_encode(p64, torch, cur1, ref1, one[0], one[1], one[2], one[3], w=w, h=h, stream=s3)
    big = outputs(4)
    with torch.cuda.stream(s3):
        big[1].copy_(li_a)
        _raw_encode(p64, torch, cur_a, ref_a, big[0], big[1], big[2], big[3], w=w, h=h, stream=s3)
    torch.cuda.synchronize()
    for o in one:
        o.zero_()
    one[1].copy_(li_a[:nmb])
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(one[0]), exp_a[0][:pic])
    np.testing.assert_array_equal(host(one[2]), exp_a[1][:1])
    np.testing.assert_array_equal(host(one[3]), exp_a[2][:1])
    for got, want in zip((host(big[0]), host(big[2]), host(big[3])), exp_a):
        np.testing.assert_array_equal(got, want)
    del g
    torch.cuda.synchronize()
    assert p64.lib().p64gpu_release_scratch() == 0


def test_capture_fork_join_side_stream_without_me(p64, torch_dev):
    """An inter encode with args.me == NULL launched on a side stream that a
    capture forked from its stream and joined back (the two-stream pattern
    of DESIGN.md 9b): the captured call takes the fused kernel (no library
    scratch under capture), its replay equals the eager split-kernel call."""
    torch = torch_dev
    w, h, S = 176, 144, 4
    nmb, pic = 99, w * h * 3 // 2
    fr = p64.synth_frames_device(w, h, 1, S, 0, 2, content=p64.SYNTH_SURVEY)
    li0 = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
    p64.encode_frames(fr[0].reshape(-1), None, r0, li0, width=w, height=h, intra=True)
    cap, side = torch.cuda.Stream(), torch.cuda.Stream()
    res = []
    for graph in (False, True):
        rec = torch.zeros_like(r0)
        li = li0.clone()
        coef = torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda")
        mb = torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda")
        torch.cuda.synchronize()
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                side.wait_stream(cap)
                with torch.cuda.stream(side):
                    _raw_encode(p64, torch, fr[1].reshape(-1), r0, rec, li, coef, mb, w=w, h=h, stream=side)
                cap.wait_stream(side)
            torch.cuda.synchronize()
            li.copy_(li0)
            g.replay()
        else:
            _raw_encode(p64, torch, fr[1].reshape(-1), r0, rec, li, coef, mb, w=w, h=h,
                        stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        res.append((host(coef), host(mb), host(rec), host(li)))
    for a, b in zip(*res):
        np.testing.assert_array_equal(a, b)


def test_library_me_scratch_per_thread_stream(p64, torch_dev):
    """hipStreamPerThread stands for each calling thread's own stream: two
    threads encoding without an ME-record output on it, at the same time,
    get scratch buffers of their own and their own results; and so do two
    threads sharing the NULL stream (the library holds its lock until both
    kernels of a call are enqueued).  ADVICE r03 (medium)."""
    import threading
    torch = torch_dev
    w, h, S = 352, 288, 4
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2

    class Raw:  # a raw stream handle for _raw_encode
        def __init__(self, v):
            self.cuda_stream = v

    jobs = []
    for seed in (303, 404):
        f = [dev(torch, np.stack([p64.synth_frame(seed + s, t, w, h) for s in range(S)])).reshape(-1)
             for t in range(2)]
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
        p64.encode_frames(f[0], None, r0, li, width=w, height=h, intra=True, quant=8)
        jobs.append((f[1], r0, li))
    torch.cuda.synchronize()

    def outputs():
        return (torch.empty(S * pic, dtype=torch.uint8, device="cuda"),
                torch.zeros(S * nmb, dtype=torch.uint8, device="cuda"),
                torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"))

    want = []
    for cur, ref, li in jobs:
        o = outputs()
        o[1].copy_(li)
        me = torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda")
        _raw_encode(p64, torch, cur, ref, o[0], o[1], o[2], o[3], w=w, h=h,
                    stream=torch.cuda.current_stream(), me=me)
        torch.cuda.synchronize()
        want.append(tuple(host(x) for x in (o[0], o[2], o[3])))

    for handle in (2, 0):  # hipStreamPerThread, the NULL stream
        outs = [outputs() for _ in jobs]
        for (cur, ref, li), o in zip(jobs, outs):
            o[1].copy_(li)
        torch.cuda.synchronize()
        errs = []

        def work(i):
            try:
                cur, ref, li = jobs[i]
                o = outs[i]
                for _ in range(4):  # the same picture again: same results every time
                    _raw_encode(p64, torch, cur, ref, o[0], o[1], o[2], o[3], w=w, h=h,
                                stream=Raw(handle))
                    torch.cuda.synchronize()
                    o[1].copy_(li)  # LastIntra back for the next round
                    torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        torch.cuda.synchronize()
        assert not errs, errs
        for o, e in zip(outs, want):
            for got, exp in zip((host(o[0]), host(o[2]), host(o[3])), e):
                np.testing.assert_array_equal(got, exp, err_msg=f"stream handle {handle}")
    assert p64.lib().p64gpu_release_scratch() == 0


def test_split_launches_match_single_launch(p64, torch_dev, monkeypatch):
    """Batches larger than one launch's 2 GiB of 32-bit buffer offsets are cut
    into several launches (intra, inter block kernel, decoder).  A lowered
    limit (P64GPU_CHUNK_BYTES: one picture per launch) gives the same levels,
    records and reconstructions as one launch."""
    torch = torch_dev
    w, h, S = 352, 288, 3
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    frames = [dev(torch, np.stack([p64.synth_frame(31 + s, t, w, h) for s in range(S)])) for t in range(2)]

    def run():
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
        r1 = torch.zeros_like(r0)
        o0 = p64.encode_frames(frames[0], None, r0, li, width=w, height=h, intra=True, quant=5)
        o1 = p64.encode_frames(frames[1], r0, r1, li, width=w, height=h, intra=False, quant=5,
                               me_mode=p64.ME_FULL, search_limit=31)
        qmb = torch.full((S * nmb,), 5, dtype=torch.uint8, device="cuda")
        d1 = torch.zeros_like(r0)
        p64.decode_recon(r0, d1, o1.coef, o1.mb, qmb, torch.ones_like(qmb), width=w, height=h)
        torch.cuda.synchronize()
        return [host(t) for t in (o0.coef, o0.mb, r0, o1.coef, o1.mb, r1, d1, li)]

    whole = run()
    monkeypatch.setenv("P64GPU_CHUNK_BYTES", "200000")
    split = run()
    for a, b in zip(whole, split):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(whole[6], whole[5])  # decoder == encoder reconstruction


def test_packed_decode_split_launches(p64, torch_dev, monkeypatch):
    """p64gpu_decode_recon_packed over 40 QCIF pictures: its index groups run
    across picture boundaries, so a split launch (P64GPU_CHUNK_BYTES: the
    smallest split, at 32 pictures) starts on a group boundary; one launch,
    the split launches and the dense entry give the same reconstructions,
    which equal the encoder's."""
    torch = torch_dev
    w, h, S = 176, 144, 40
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    frames = [dev(torch, np.stack([p64.synth_frame(51 + s, t, w, h) for s in range(S)])) for t in range(2)]
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
    r1 = torch.zeros_like(r0)
    p64.encode_frames(frames[0], None, r0, li, width=w, height=h, intra=True, quant=6)
    o1 = p64.encode_frames(frames[1], r0, r1, li, width=w, height=h, intra=False, quant=6,
                           me_mode=p64.ME_FULL, search_limit=31)
    qmb = torch.full((S * nmb,), 6, dtype=torch.uint8, device="cuda")
    mask = torch.ones_like(qmb)
    mask[::5] = 0  # some MBs not coded: their prediction only
    lv, n, ix = p64.pack_levels_device(o1.coef, o1.mb, mask, w, h)
    assert ix.shape[0] == (S * 6 * nmb + 63) // 64
    dense = torch.zeros_like(r0)
    p64.decode_recon(r0, dense, o1.coef, o1.mb, qmb, mask, width=w, height=h)
    whole = torch.zeros_like(r0)
    p64.decode_recon_packed(r0, whole, lv, n, ix, o1.mb, qmb, mask, width=w, height=h)
    monkeypatch.setenv("P64GPU_CHUNK_BYTES", "20000")
    split = torch.zeros_like(r0)
    p64.decode_recon_packed(r0, split, lv, n, ix, o1.mb, qmb, mask, width=w, height=h)
    torch.cuda.synchronize()
    assert torch.equal(whole, dense)
    assert torch.equal(split, dense)
    full = torch.zeros_like(r0)
    p64.decode_recon_packed(r0, full, *p64.pack_levels_device(o1.coef, o1.mb, torch.ones_like(qmb), w, h),
                            o1.mb, qmb, torch.ones_like(qmb), width=w, height=h)
    torch.cuda.synchronize()
    assert torch.equal(full, r1)  # decoder == encoder reconstruction


@pytest.mark.parametrize("content,mode", [("pan15", 1), ("noise", 1), ("flat", 1), ("pan15", 0)])
def test_stress_contents_vs_oracle(p64, oracle_mod, torch_dev, content, mode):
    """The bench's stress inputs (+-15-px pans, uniform noise,
    constant planes) through the split encoder, checked picture by picture
    against the oracle; the decoder reproduces the encoder's reconstruction."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(GOLDEN), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    torch = torch_dev
    w, h, S, T = 352, 288, 2, 3
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    frames = bench.make_inputs(torch, p64, content, w, h, 5, S, T)  # [T][S][pic] on the device
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    bufs = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    got = []
    for t in range(T):
        ref, rec = bufs[(t + 1) % 2], bufs[t % 2]
        o = p64.encode_frames(frames[t].reshape(-1), ref, rec, li, width=w, height=h, intra=(t == 0),
                              quant=8, me_mode=mode, search_limit=31)
        got.append((host(o.coef), host(o.mb), host(rec).reshape(S, pic)))
        if t > 0:  # decode the inter picture from its records and levels
            qmb = torch.full((S * nmb,), 8, dtype=torch.uint8, device="cuda")
            d = torch.zeros_like(rec)
            p64.decode_recon(ref, d, o.coef, o.mb, qmb, torch.ones_like(qmb), width=w, height=h)
            assert torch.equal(d, rec), f"decoder != encoder reconstruction at t{t}"
    fr = host(frames)
    for s in range(S):
        li_o = np.zeros(nmb, np.uint8)
        ref = None
        for t in range(T):
            coef, mb, _, recon = oracle_mod.encode_frame(w, h, fr[t][s], ref, li_o, intra=(t == 0), quant=8,
                                                         me_mode=mode, search_limit=31)
            ref = recon
            np.testing.assert_array_equal(got[t][0][s], coef, err_msg=f"{content} coef s{s} t{t}")
            np.testing.assert_array_equal(got[t][1][s].view(p64.MB_DTYPE).reshape(nmb), mb,
                                          err_msg=f"{content} mb s{s} t{t}")
            np.testing.assert_array_equal(got[t][2][s], recon, err_msg=f"{content} recon s{s} t{t}")


def test_env_switches_same_bytes(torch_dev):
    """The A/B switch selects other kernels, never other
    bytes: the fused one-wave-per-MB encoder gives the default path's outputs
    exactly, for intra and inter pictures."""
    import subprocess
    import sys
    probe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "switch_probe.py")

    def digest(extra):
        env = dict(os.environ)
        env.update(extra)
        r = subprocess.run([sys.executable, probe], env=env, capture_output=True, text=True, timeout=150)
        assert r.returncode == 0, r.stderr[-2000:]
        return r.stdout.strip().splitlines()[-1]

    ref = digest({})
    for sw in ({"P64GPU_FUSED": "1"},):
        assert digest(sw) == ref, sw


def test_inter_levels_sparse_store(p64, oracle_mod, torch_dev):
    """coef contract (include/p64gpu.h): an inter picture writes exactly the
    blocks with a nonzero level; all-zero blocks keep what the buffer held.
    Sentinel-filled output vs the oracle, with and without -o overrides (MC
    types without coefficients write nothing)."""
    torch = torch_dev
    w, h, nmb = 176, 144, 99
    rng = np.random.default_rng(11)
    f0, f1 = p64.synth_frame(33, 0, w, h), p64.synth_frame(33, 1, w, h)
    _, _, _, rec0 = oracle_mod.encode_frame(w, h, f0, None, np.zeros(nmb, np.uint8), intra=True, quant=8)
    SENT = 0x5A5A
    for ov in (None, rng.integers(-1, 10, nmb).astype(np.int8)):
        for quant in (3, 8, 16):
            li_o = np.zeros(nmb, np.uint8)
            coef, mb, _, recon = oracle_mod.encode_frame(w, h, f1, rec0, li_o, intra=False, quant=quant,
                                                          me_mode=p64.ME_FULL, search_limit=31,
                                                          mtype_override=ov)
            out = p64.FrameBatchOut(coef=torch.full((1, nmb, 6, 64), SENT, dtype=torch.int16, device="cuda"),
                                    mb=torch.empty((1, nmb, 4), dtype=torch.int8, device="cuda"),
                                    me=torch.empty((1, nmb, 7), dtype=torch.int32, device="cuda"),
                                    nz=torch.full((1, nmb), 0xC0, dtype=torch.uint8, device="cuda"))
            rec_d = torch.zeros(w * h * 3 // 2, dtype=torch.uint8, device="cuda")
            p64.encode_frames(dev(torch, f1), dev(torch, rec0), rec_d, dev(torch, np.zeros(nmb, np.uint8)),
                              width=w, height=h, intra=False, quant=quant, me_mode=p64.ME_FULL,
                              search_limit=31, mtype_override=dev(torch, ov) if ov is not None else None,
                              out=out)
            got = host(out.coef)[0].reshape(-1, 64)
            want = coef.reshape(-1, 64)
            nz = want.any(axis=1)
            tag = f"q{quant} ov={ov is not None}"
            assert 0 < nz.sum() < nz.size, tag  # both kinds present
            np.testing.assert_array_equal(got[nz], want[nz], err_msg=tag)
            assert (got[~nz] == SENT).all(), tag
            # the nonzero-block mask names exactly those blocks (bit 5 - b), ABI v2
            m = host(out.nz)[0]
            np.testing.assert_array_equal(((m[:, None] >> (5 - np.arange(6))[None, :]) & 1).reshape(-1) == 1,
                                          nz, err_msg=tag)
            np.testing.assert_array_equal(host(out.mb)[0].view(p64.MB_DTYPE).reshape(nmb), mb, err_msg=tag)
            np.testing.assert_array_equal(host(rec_d), recon, err_msg=tag)


def test_intra_refresh_and_override(p64, oracle_mod, torch_dev):
    """LastIntra > 131 forces MTYPE 0 (p64.c:772); -o overrides (p64.c:761-768),
    including MC types without coefficients (4, 7) and MQUANT types."""
    torch = torch_dev
    w, h = 176, 144
    nmb = 99
    rng = np.random.default_rng(5)
    f0, f1 = p64.synth_frame(21, 0, w, h), p64.synth_frame(21, 1, w, h)
    li0 = rng.integers(120, 140, nmb).astype(np.uint8)
    ov = rng.integers(-1, 10, nmb).astype(np.int8)
    # reference picture = oracle intra recon of f0
    li_tmp = np.zeros(nmb, np.uint8)
    _, _, _, rec0 = oracle_mod.encode_frame(w, h, f0, None, li_tmp, intra=True, quant=8)
    li_o = li0.copy()
    coef, mb, me, recon = oracle_mod.encode_frame(w, h, f1, rec0, li_o, intra=False, quant=8,
                                                  me_mode=1, search_limit=31, mtype_override=ov)
    li_d = dev(torch, li0)
    rec_d = torch.zeros(w * h * 3 // 2, dtype=torch.uint8, device="cuda")
    o = p64.encode_frames(dev(torch, f1), dev(torch, rec0), rec_d, li_d, width=w, height=h,
                          intra=False, quant=8, me_mode=1, search_limit=31,
                          mtype_override=dev(torch, ov))
    np.testing.assert_array_equal(host(o.coef)[0], coef)
    np.testing.assert_array_equal(host(o.mb)[0].view(p64.MB_DTYPE).reshape(nmb), mb)
    np.testing.assert_array_equal(host(rec_d), recon)
    np.testing.assert_array_equal(host(li_d), li_o)
    assert (mb["mtype"][li0 > 131] == 0).all()


def test_decoder_recon_matches_encoder(p64, torch_dev):
    """Decode-side reconstruction of the encoder's own output reproduces the
    encoder's closed-loop reconstruction (encoder recon ==
    decoder output)."""
    torch = torch_dev
    w, h = 352, 288
    nmb = 396
    seeds = [1, 6, 7, 13]
    pic = w * h * 3 // 2
    f0 = dev(torch, np.stack([p64.synth_frame(s, 0, w, h) for s in seeds]))
    f1 = dev(torch, np.stack([p64.synth_frame(s, 1, w, h) for s in seeds]))
    li = torch.zeros(len(seeds) * nmb, dtype=torch.uint8, device="cuda")
    r0 = torch.zeros(len(seeds) * pic, dtype=torch.uint8, device="cuda")
    r1 = torch.zeros_like(r0)
    o0 = p64.encode_frames(f0, None, r0, li, width=w, height=h, intra=True, quant=6)
    o1 = p64.encode_frames(f1, r0, r1, li, width=w, height=h, intra=False, quant=6, me_mode=1,
                           search_limit=31)
    qmb = torch.full((len(seeds) * nmb,), 6, dtype=torch.uint8, device="cuda")
    mask = torch.ones_like(qmb)
    d0 = torch.zeros_like(r0)
    p64.decode_recon(d0, d0, o0.coef, o0.mb, qmb, mask, width=w, height=h)
    assert torch.equal(d0, r0)
    d1 = d0.clone()
    p64.decode_recon(d0, d1, o1.coef, o1.mb, qmb, mask, width=w, height=h)
    assert torch.equal(d1, r1)


def test_invalid_arguments_raise(p64, torch_dev):
    torch = torch_dev
    x = torch.zeros(10, dtype=torch.uint8, device="cuda")
    with pytest.raises(p64.P64GpuError):
        p64.encode_frames(x, x, x, x, width=100, height=64, intra=True)
    with pytest.raises(p64.P64GpuError):
        p64.MotionEstimation(x, x, 176, 144, mode=5)


# ---------------------------------------------------------------------------
# link-level drop-in: the reference CLI with MotionEstimation/ChenDct/ChenIDct
# served by the GPU (p64_amd/host/p64gpu_refshim.c)

REFSHIM = os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "p64gpu_ref")


@pytest.mark.parametrize("name", ["qcif_tss", "qcif_full31", "qcif_q31", "cif_full31",
                                  "qcif_flat_tss"])
def test_reference_cli_with_gpu_shim(p64, torch_dev, tmp_path, name):
    import subprocess
    if not os.access(REFSHIM, os.X_OK):
        pytest.skip("oracle/_ref/p64gpu_ref not built (needs /root/reference at build time)")
    z = load(f"seq_{name}.npz")
    w, h, n = int(z["width"]), int(z["height"]), int(z["nframes"])
    frames = sequence_frames(p64, z)
    y4m = tmp_path / "in.y4m"
    with open(y4m, "wb") as f:
        f.write(b"YUV4MPEG2 W%d H%d F30000:1001 Ip A0:0 C420jpeg\n" % (w, h))
        for fr in frames:
            f.write(b"FRAME\n" + fr.tobytes())
    env = dict(os.environ)
    if str(z["me"]) == "full":
        env["P64GPU_ME"] = "full"
    out = tmp_path / "out.p64"
    subprocess.run([REFSHIM, "-" + str(z["fmt"]), "-y4m", "-a", "0", "-b", str(n - 1), "-q",
                    str(int(z["q"])), "-i", str(int(z["sl"])), str(tmp_path / "in"), "-z", ".y4m",
                    "-s", str(out)], env=env, stdout=subprocess.DEVNULL, check=True, timeout=300)
    data = out.read_bytes()
    assert len(data) == int(z["stream_len"])
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])


def test_device_synth_matches_host(p64, torch_dev):
    """The bench's on-device inputs are the same bytes the CPU legs use (both
    contents: the survey sines are a fixed-point polynomial of integer phases,
    identical on host and device)."""
    for c in (p64.SYNTH_VNOISE, p64.SYNTH_SURVEY):
        for (w, h) in ((352, 288), (176, 144), (704, 576)):
            d = host(p64.synth_frames_device(w, h, 5, 3, 10, 2, content=c))
            for t in range(2):
                for s in range(3):
                    np.testing.assert_array_equal(d[t, s], p64.synth_frame(5 + s, 10 + t, w, h, content=c))
    # far along a sequence (texture coordinates well away from the origin)
    d = host(p64.synth_frames_device(352, 288, 200, 2, 250, 1, content=p64.SYNTH_SURVEY))
    np.testing.assert_array_equal(d[0, 1], p64.synth_frame(201, 250, 352, 288, content=p64.SYNTH_SURVEY))
    # more than 65535 pictures: the wrapper splits the slots over launches
    w, h = 176, 144
    big = p64.synth_frames_device(w, h, 3, 4096, 7, 17)
    for t, s in ((0, 0), (15, 4095), (16, 0), (16, 4095)):
        np.testing.assert_array_equal(host(big[t, s]), p64.synth_frame(3 + s, 7 + t, w, h))
    del big


# ---------------------------------------------------------------------------
# the bench's full size: 256 CIF sequences per launch, FULL SL=31, q=8

@pytest.mark.parametrize("content", ["survey", "synth"])
def test_bench_scale_properties(p64, oracle_mod, torch_dev, content):
    """At BASELINE's full size (one launch over 256 CIF pictures = 101,376 MBs,
    device-generated as in bench.py; SURVEY.md 8(d)'s content and the
    builder's synth): the decoder reconstruction of the coded output equals
    the encoder's closed-loop reconstruction for every sequence, a relaunch is
    bit-identical, the levels obey the H.261 bounds, and sampled sequences
    equal the oracle exactly -- for synth one of every seed class (1 plain,
    5 scene cut, 6 noise-free, 7 low contrast: the dense-search class) and
    the last one -- levels rebuilt through the nonzero-block mask."""
    torch = torch_dev
    w, h, S, nfr, q = 352, 288, 256, 3, 8
    if content == "synth":
        nfr = 14  # past the scene cut of seeds = 5 (mod 8) at picture 12
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    # [t][s] = synth_frame(1 + s, t, content)
    fr = p64.synth_frames_device(w, h, 1, S, 0, nfr, content=p64.CONTENTS[content])
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    recs = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(nfr)]
    outs = []
    for t in range(nfr):
        o = p64.FrameBatchOut(coef=torch.full((S, nmb, 6, 64), 0x5A5A, dtype=torch.int16, device="cuda"),
                              mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                              me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"),
                              nz=torch.empty((S, nmb), dtype=torch.uint8, device="cuda"))
        p64.encode_frames(fr[t].reshape(-1), recs[t - 1] if t else None, recs[t], li, width=w,
                          height=h, intra=(t == 0), quant=q, me_mode=p64.ME_FULL,
                          search_limit=31, out=o)
        outs.append((o.coef, o.mb, o.me, o.nz))
    qmb = torch.full((S * nmb,), q, dtype=torch.uint8, device="cuda")
    mask = torch.ones_like(qmb)
    prev = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
    sel = torch.tensor([32 >> b for b in range(6)], dtype=torch.uint8, device="cuda")
    prevp = prev.clone()
    for t in range(nfr):
        d = torch.zeros_like(prev)
        p64.decode_recon(prev, d, outs[t][0], outs[t][1], qmb, mask, width=w, height=h)
        assert torch.equal(d, recs[t]), f"decoder recon != encoder recon at picture {t}"
        prev = d
        # the packed layout (ABI v3), built on the device from the same levels
        lv, n, ix = p64.pack_levels_device(outs[t][0], outs[t][1], mask, w, h)
        dp = torch.zeros_like(prevp)
        p64.decode_recon_packed(prevp, dp, lv if n else torch.zeros((1, 64), dtype=torch.int16, device="cuda"),
                                n, ix, outs[t][1], qmb, mask, width=w, height=h)
        assert torch.equal(dp, recs[t]), f"packed decoder recon != encoder recon at picture {t}"
        prevp = dp
        coef = outs[t][0].view(S, nmb, 6, 64)
        stored = (outs[t][3][..., None] & sel) != 0  # [S, nmb, 6]: the nonzero-block mask
        lv = torch.where(stored[..., None], coef, torch.zeros_like(coef))
        assert int(lv.abs().max()) <= 254 and int(lv[:, :, :, 1:].abs().max()) <= 127
        # every block outside the mask was left alone (sentinel), every block in it is nonzero
        assert bool((coef[~stored] == 0x5A5A).all())
        assert bool((lv != 0).any(dim=3).eq(stored).all())
    # relaunch of the last picture: identical levels, records and reconstruction
    li2 = li.clone()
    li2.zero_()
    rec_again = torch.zeros_like(recs[-1])
    o = p64.encode_frames(fr[nfr - 1].reshape(-1), recs[nfr - 2], rec_again, li2, width=w, height=h,
                          intra=False, quant=q, me_mode=p64.ME_FULL, search_limit=31)
    # (o.coef starts zeroed; LastIntra differs only through the counters, all < 131 here)
    stored = ((outs[-1][3][..., None] & sel) != 0)[..., None]
    assert torch.equal(o.coef, torch.where(stored, outs[-1][0], torch.zeros_like(outs[-1][0])))
    assert torch.equal(o.mb, outs[-1][1])
    assert torch.equal(rec_again, recs[-1])
    # sampled sequences against the oracle: the whole inputbuf array rebuilt
    # through the mask, the mask, the records and the reconstruction
    checked = (0, 4, 5, 6, S - 1) if content == "synth" else (0, S - 1)
    for s in checked:
        frames_h = host(fr[:, s])
        li_o = np.zeros(nmb, np.uint8)
        ref = None
        for t in range(nfr):
            coef, mb, me, recon = oracle_mod.encode_frame(w, h, frames_h[t], ref, li_o,
                                                          intra=(t == 0), quant=q, me_mode=1,
                                                          search_limit=31)
            ref = recon
            nz = host(outs[t][3][s])
            bits = ((nz[:, None] >> (5 - np.arange(6))[None, :]) & 1) == 1
            np.testing.assert_array_equal(bits, coef.any(axis=2), err_msg=f"mask seed{s + 1} t{t}")
            got = np.where(bits[:, :, None], host(outs[t][0][s]), 0)
            np.testing.assert_array_equal(got, coef, err_msg=f"coef seed{s + 1} t{t}")
            np.testing.assert_array_equal(host(outs[t][1][s]).view(p64.MB_DTYPE).reshape(nmb), mb,
                                          err_msg=f"mb seed{s + 1} t{t}")
            np.testing.assert_array_equal(host(recs[t].view(S, pic)[s]), recon,
                                          err_msg=f"recon seed{s + 1} t{t}")


# ---------------------------------------------------------------------------
# the range proofs of the packed 16-bit arithmetic, pinned at
# their edges against the oracle: extreme levels through the decoder for every
# q, extreme residuals and pixels through the block encoders

def _edge_level_blocks(rng, n):
    """n zigzag level blocks at the H.261 extremes: all +-127 with the sign
    patterns that maximise the IDCT sums (constant, alternating, the sign of
    each 1-D cosine basis row/column), plus random +-127 and random levels."""
    pos = np.zeros(64, int)  # natural index -> scan position (transform.c:67-75)
    k = 0
    for d in range(15):
        rows = range(max(0, d - 7), min(d, 7) + 1)
        for r in (rows if d % 2 else reversed(rows)):
            pos[8 * r + d - r] = k
            k += 1
    cosv = np.cos((2 * np.arange(8)[:, None] + 1) * np.arange(8)[None, :] * np.pi / 16)  # [x, u]
    pats = [np.ones(64), -np.ones(64), np.tile([1, -1], 32), np.repeat([1, -1], 32)]
    for u in range(8):  # natural-order sign patterns: outer products of basis signs
        for v in range(0, 8, 3):
            s = np.sign(np.outer(cosv[u], cosv[v]) + 1e-9).reshape(64)
            pats += [s, -s]
    out = np.zeros((n, 64), np.int16)
    for i in range(n):
        k = i % (len(pats) + 2)
        if k < len(pats):
            nat = (127 * pats[k]).astype(np.int16)
        elif k == len(pats):
            nat = (127 * rng.choice([-1, 1], 64)).astype(np.int16)
        else:
            nat = rng.integers(-127, 128, 64).astype(np.int16)
        out[i, pos] = nat  # zigzag order
    return out


@pytest.mark.parametrize("packed", [False, True])
def test_decoder_extreme_levels_every_q_vs_oracle(p64, oracle_mod, torch_dev, packed):
    """k_recon_mbg's packed dequantiser (exact for |level| <= 528) and v_dot2
    IDCT column pass at their edges: |level| = 127 in every position with the
    IDCT's worst sign patterns, every q = 1..31, intra (DC 1..254) and inter
    types with and without the loop filter, against oracle.decode_mb
    (p64.c:1179-1237 + 971-1013).  Rounds 2-3 leave about a third of the MBs
    out of the coded mask (MBs the MBA addressing skips, p64.c:1163-1167,
    1185-1186): their pixels must stay untouched while the wave-wide row
    stores write their neighbours.  packed: the same through
    p64gpu_decode_recon_packed (ABI v3) with the levels packed by
    p64s_pack_levels (the transmitted blocks only, per-64-block index)."""
    from p64_amd import stream
    torch = torch_dev
    w, h = 176, 144
    mbw, nmb, pic = w // 16, 99, w * h * 3 // 2
    rng = np.random.default_rng(127)
    ref = rng.integers(0, 256, pic).astype(np.uint8)
    for rnd in range(4):
        recon0 = rng.integers(0, 256, pic).astype(np.uint8)
        mt = rng.integers(0, 10, nmb)
        mt[: 10] = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9]
        cbp = rng.integers(1, 64, nmb)
        cbp[rnd::5] = 63
        q = (np.arange(nmb) + 7 * rnd) % 31 + 1
        mbx, mby = np.arange(nmb) % mbw, np.arange(nmb) // mbw
        mvx = np.array([rng.integers(max(-15, -16 * x), min(15, w - 16 - 16 * x) + 1) for x in mbx])
        mvy = np.array([rng.integers(max(-15, -16 * y), min(15, h - 16 - 16 * y) + 1) for y in mby])
        mf = mt >= 4
        mvx, mvy = np.where(mf, mvx, 0), np.where(mf, mvy, 0)
        coef = _edge_level_blocks(rng, nmb * 6).reshape(nmb, 6, 64)
        intra = mt < 2
        coef[intra, :, 0] = rng.choice([1, 2, 127, 128, 253, 254], (intra.sum(), 6))
        coded = np.ones(nmb, np.uint8) if rnd < 2 else (rng.random(nmb) > 0.33).astype(np.uint8)
        exp = recon0.copy()
        for k in range(nmb):
            if coded[k]:
                oracle_mod.decode_mb(w, h, ref, exp, int(mbx[k]), int(mby[k]), int(mt[k]), int(cbp[k]),
                                     int(mvx[k]), int(mvy[k]), int(q[k]), coef[k])
        mb = np.stack([mt, cbp, mvx, mvy], 1).astype(np.int8)
        d = dev(torch, recon0)
        if packed:
            lv, ix = stream.pack_levels(stream.QCIF, mb, coded, coef)
            p64.decode_recon_packed(dev(torch, ref), d, dev(torch, lv), len(lv), dev(torch, ix.view(np.int32)),
                                    dev(torch, mb), dev(torch, q.astype(np.uint8)), dev(torch, coded),
                                    width=w, height=h)
        else:
            p64.decode_recon(dev(torch, ref), d, dev(torch, coef), dev(torch, mb),
                             dev(torch, q.astype(np.uint8)), dev(torch, coded),
                             width=w, height=h)
        np.testing.assert_array_equal(host(d), exp, err_msg=f"round {rnd}")


def _edge_pictures(w, h):
    """(cur, ref) pairs whose residuals sit at +-255 in the patterns that drive
    the forward DCT to its extremes: 1/2/4-pixel checkerboards, stripes,
    half-planes, and 0/255 pictures against their inverse."""
    y, x = np.mgrid[0:h, 0:w]
    out = []
    for pat in ((x + y) % 2, (x // 2 + y // 2) % 2, (x // 4 + y // 4) % 2, x % 2, y % 2,
                (x % 8) >= 4, (y % 8) >= 4, np.zeros((h, w), int)):
        a = (255 * np.asarray(pat, np.int64)).astype(np.uint8)
        yc, xc = np.mgrid[0:h // 2, 0:w // 2]
        ac = (255 * ((xc + yc) % 2)).astype(np.uint8)
        cur = np.concatenate([a.reshape(-1), ac.reshape(-1), (255 - ac).reshape(-1)])
        out.append((cur, 255 - cur))
    return out


@pytest.mark.parametrize("quant", [1, 2, 3, 4, 5, 8, 16, 31])
def test_inter_uniform_quant_vs_oracle(p64, oracle_mod, torch_dev, quant):
    """k_intra_mbg / k_inter_mbg at one uniform q, the case their launches specialise: q with
    D = 16q a power of two (1, 2, 4, 8, 16) quantises packed level pairs
    (qlevel_pk2), q >= 5 drops the clamp where the residual-sum bound allows,
    the others keep the scalar clamped quantiser.  Extreme +-255 residuals
    (every clamp active), a synthetic picture pair (small residuals), and the
    MTYPE overrides 0..9 (the override instance), against oracle.encode_frame."""
    torch = torch_dev
    w, h = 176, 144
    nmb = 99
    pairs = _edge_pictures(w, h)[:3] + [(p64.synth_frame(5, 3, w, h), p64.synth_frame(5, 2, w, h))]
    for i, (cur, ref) in enumerate(pairs):
        # the intra picture at the same uniform q (k_intra_mbg's packed
        # quantiser for powers of two, the clamp below q = 5)
        li = np.zeros(nmb, np.uint8)
        coef, mb, _, rec = oracle_mod.encode_frame(w, h, cur, None, li, intra=True, quant=quant)
        lid = torch.zeros(nmb, dtype=torch.uint8, device="cuda")
        rd = torch.zeros(cur.size, dtype=torch.uint8, device="cuda")
        o = p64.encode_frames(dev(torch, cur), None, rd, lid, width=w, height=h, intra=True, quant=quant)
        np.testing.assert_array_equal(host(o.coef)[0], coef, err_msg=f"intra coef q{quant} picture {i}")
        np.testing.assert_array_equal(host(rd), rec, err_msg=f"intra recon q{quant} picture {i}")
        for ov in (None, (np.arange(nmb) % 10).astype(np.int8)):
            li = np.zeros(nmb, np.uint8)
            coef, mb, me, rec = oracle_mod.encode_frame(w, h, cur, ref, li, intra=False, quant=quant,
                                                        me_mode=1, search_limit=31, mtype_override=ov)
            lid = torch.zeros(nmb, dtype=torch.uint8, device="cuda")
            rd = torch.zeros(cur.size, dtype=torch.uint8, device="cuda")
            o = p64.encode_frames(dev(torch, cur), dev(torch, ref), rd, lid, width=w, height=h,
                                  intra=False, quant=quant, me_mode=p64.ME_FULL, search_limit=31,
                                  mtype_override=(dev(torch, ov) if ov is not None else None))
            tag = f"q{quant} pair {i} override {ov is not None}"
            np.testing.assert_array_equal(host(o.coef)[0], coef, err_msg=f"coef {tag}")
            np.testing.assert_array_equal(host(o.mb)[0].view(p64.MB_DTYPE).reshape(nmb), mb, err_msg=f"mb {tag}")
            np.testing.assert_array_equal(host(rd), rec, err_msg=f"recon {tag}")


def test_block_encoders_extreme_residuals_vs_oracle(p64, oracle_mod, torch_dev):
    """k_intra_mbg / k_inter_mbg at the edges of their 16-bit range proofs
    (column outputs of a +-255 residual, row-pass intermediates < 2^15, the
    intra v_dot2 IDCT row pass bound): residuals of +-255 in checkerboard and
    stripe patterns, 0/255 intra pictures, every q = 1..31 by per-MB UseQuant,
    through MTYPE overrides 0..9, against oracle.encode_frame."""
    torch = torch_dev
    w, h = 176, 144
    nmb = 99
    q = ((np.arange(nmb) % 31) + 1).astype(np.uint8)
    for i, (cur, ref) in enumerate(_edge_pictures(w, h)):
        # intra picture of cur
        li = np.zeros(nmb, np.uint8)
        coef, mb, _, rec = oracle_mod.encode_frame(w, h, cur, None, li, intra=True, quant=8, quant_mb=q)
        lid = torch.zeros(nmb, dtype=torch.uint8, device="cuda")
        rd = torch.zeros(cur.size, dtype=torch.uint8, device="cuda")
        o = p64.encode_frames(dev(torch, cur), None, rd, lid, width=w, height=h, intra=True, quant=8,
                              quant_mb=dev(torch, q))
        np.testing.assert_array_equal(host(o.coef)[0], coef, err_msg=f"intra coef pattern {i}")
        np.testing.assert_array_equal(host(rd), rec, err_msg=f"intra recon pattern {i}")
        # inter picture cur predicted from ref, every MTYPE by override (MC
        # types take the ME vector the search finds)
        ov = (np.arange(nmb) % 10).astype(np.int8)
        li = np.zeros(nmb, np.uint8)
        coef, mb, me, rec = oracle_mod.encode_frame(w, h, cur, ref, li, intra=False, quant=8,
                                                    me_mode=1, search_limit=31, quant_mb=q,
                                                    mtype_override=ov)
        lid = torch.zeros(nmb, dtype=torch.uint8, device="cuda")
        rd = torch.zeros(cur.size, dtype=torch.uint8, device="cuda")
        o = p64.encode_frames(dev(torch, cur), dev(torch, ref), rd, lid, width=w, height=h,
                              intra=False, quant=8, me_mode=p64.ME_FULL, search_limit=31,
                              quant_mb=dev(torch, q), mtype_override=dev(torch, ov))
        np.testing.assert_array_equal(host(o.coef)[0], coef, err_msg=f"inter coef pattern {i}")
        np.testing.assert_array_equal(host(o.mb)[0].view(p64.MB_DTYPE).reshape(nmb), mb,
                                      err_msg=f"inter mb pattern {i}")
        np.testing.assert_array_equal(host(rd), rec, err_msg=f"inter recon pattern {i}")
