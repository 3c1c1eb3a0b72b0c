"""GPU end-to-end: the hot path plus the host bitstream layer against the
reference's own outputs -- .p64 bytes (stream_sha256 of the golden sequences)
and the decoded planes of short.p64 (decode.json MD5s).  Run with -m gpu."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO
from test_oracle_golden import PROG_SEQS, RATE_SEQS, SEQS, load, sequence_frames

pytestmark = pytest.mark.gpu

CLI = os.path.join(REPO, "p64_amd", "p64gpu")
PLAIN = [s for s in SEQS if not str(load(f"seq_{s}.npz")["oracle"])]  # no -o program


def write_y4m(path, frames, w, h):
    with open(path, "wb") as f:
        f.write(b"YUV4MPEG2 W%d H%d F30000:1001 Ip A0:0 C420jpeg\n" % (w, h))
        for fr in frames:
            f.write(b"FRAME\n" + fr.tobytes())


def cli_flags(z):
    """The reference CLI flags the fixture was made with (make_golden.run_sequence)."""
    n = int(z["nframes"])
    f = ["-" + str(z["fmt"]), "-y4m", "-a", "0", "-b", str(n - 1), "-i", str(int(z["sl"]))]
    if int(z["q"]):
        f += ["-q", str(int(z["q"]))]
    for key, flag in (("rate", "-r"), ("filesize", "-x")):
        if key in z.files and int(z[key]):
            f += [flag, str(int(z[key]))]
    if str(z["me"]) == "full":
        f.append("-full")
    if str(z["oracle"]):
        f.append("-o")
    return f


def cli_stdin(z):
    """-o reads the program from stdin: the interpreter programs under
    tests/golden/progs/ are the builder's own (written in the reference's
    program language, lexer.l), not the reference's test.* files."""
    prog = str(z["oracle"])
    return open(os.path.join(GOLDEN, "progs", prog), "rb") if prog else subprocess.DEVNULL


@pytest.mark.parametrize("name", PLAIN + RATE_SEQS + PROG_SEQS + ["qcif_intra"])
def test_cli_encode_byte_identical(p64, torch_dev, tmp_path, name):
    """`p64gpu -FMT -y4m -a 0 -b N-1 [-q Q] -i SL [-r R | -x X] [-full]` == the
    reference CLI's .p64 (rate control included: per-GOB GQUANT, MTYPE 4 on
    buffer overflow)."""
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    write_y4m(tmp_path / "in.y4m", sequence_frames(p64, z), w, h)
    cmd = [CLI] + cli_flags(z) + [str(tmp_path / "in"), "-z", ".y4m", "-s", str(tmp_path / "o.p64")]
    subprocess.run(cmd, check=True, stdin=cli_stdin(z), stdout=subprocess.DEVNULL, timeout=300)
    data = (tmp_path / "o.p64").read_bytes()
    assert len(data) == int(z["stream_len"])
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])


@pytest.mark.parametrize("host_vlc", [False, True])
@pytest.mark.parametrize("name", ["qcif_tss", "cif_full31", "ntsc_tss", "qcif_rate",
                                  "cif_rate_full31", "qcif_filesize", "qcif_prog_mq_rate",
                                  "qcif_orate", "qcif_prog_words"])
def test_python_encode_sequence_byte_identical(p64, torch_dev, name, host_vlc):
    from p64_amd import stream
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    g = lambda k: int(z[k]) if k in z.files else 0  # noqa: E731
    prog = str(z["oracle"])
    program = open(os.path.join(GOLDEN, "progs", prog)).read() if prog else None
    data = stream.encode_sequence(sequence_frames(p64, z), w, h, quant=g("q"),
                                  me_mode=1 if str(z["me"]) == "full" else 0,
                                  search_limit=g("sl"), rate=g("rate"), file_size_bits=g("filesize"),
                                  program=program, host_vlc=host_vlc)
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])


def test_cli_decode_short_p64_md5(p64, torch_dev, tmp_path):
    """`p64gpu -d -s short.p64 short` writes the reference's 7 x 3 component files."""
    exp = json.load(open(os.path.join(GOLDEN, "decode.json")))
    subprocess.run([CLI, "-d", "-s", os.path.join(GOLDEN, "short.p64"), str(tmp_path / "short")],
                   check=True, stdout=subprocess.DEVNULL, timeout=120)
    for name, md5 in exp.items():
        assert hashlib.md5((tmp_path / name).read_bytes()).hexdigest() == md5, name


def test_cli_decode_force_cif_md5(p64, torch_dev, tmp_path):
    """`p64gpu -d -c -s short.p64 sc`: ForceCIF (p64.c:308-310, 1071-1072)
    decodes the NTSC stream into CIF frames; the reference's 7 x 3 MD5s."""
    exp = json.load(open(os.path.join(GOLDEN, "decode_forcecif.json")))
    subprocess.run([CLI, "-d", "-c", "-s", os.path.join(GOLDEN, "short.p64"), str(tmp_path / "sc")],
                   check=True, stdout=subprocess.DEVNULL, timeout=120)
    for name, md5 in exp.items():
        assert hashlib.md5((tmp_path / name).read_bytes()).hexdigest() == md5, name


def test_cli_verbose_loud_parity_flags(p64, torch_dev, tmp_path):
    """-v prints the reference's `BufferContents: n  New Q1: q` line at every
    rate-control update (p64.c:466-470), in the same order with the same
    values; -l n and -p are accepted and leave the stream byte-identical."""
    z = load("seq_qcif_rate.npz")
    w, h = int(z["width"]), int(z["height"])
    write_y4m(tmp_path / "in.y4m", sequence_frames(p64, z), w, h)
    r = subprocess.run([CLI, "-QCIF", "-y4m", "-a", "0", "-b", "7", "-r", "30000", "-v", "-l", "1", "-p",
                        str(tmp_path / "in"), "-z", ".y4m", "-s", str(tmp_path / "o.p64")],
                       check=True, capture_output=True, text=True, timeout=300)
    got = [ln for ln in r.stdout.splitlines() if ln.startswith("BufferContents:")]
    exp = open(os.path.join(GOLDEN, "verbose_qcif_rate.txt")).read().splitlines()
    assert got == exp
    assert hashlib.sha256((tmp_path / "o.p64").read_bytes()).hexdigest() == str(z["stream_sha256"])


@pytest.mark.parametrize("packed", [True, False])
def test_python_decode_short_p64_md5(p64, torch_dev, packed):
    """short.p64 through the Python reader + GPU reconstruction, with the
    levels packed (p64gpu_decode_recon_packed, ABI v3; the CLI's path too) and
    dense (p64gpu_decode_recon): the reference's 21 plane MD5s."""
    from p64_amd import stream
    exp = json.load(open(os.path.join(GOLDEN, "decode.json")))
    frames = stream.decode_sequence(open(os.path.join(GOLDEN, "short.p64"), "rb").read(), packed=packed)
    assert len(frames) == 7
    w, h = 352, 240
    for i, f in enumerate(frames):
        for c, a in zip("YUV", (f[:w * h], f[w * h:w * h * 5 // 4], f[w * h * 5 // 4:])):
            assert hashlib.md5(a.tobytes()).hexdigest() == exp[f"short{i}.{c}"]


@pytest.mark.parametrize("name", ["qcif_tss", "qcif_full31", "qcif_q31", "qcif_flat_tss",
                                  "qcif_rate", "qcif_filesize", "qcif_prog_mq_rate", "qcif_orate"])
def test_decode_of_encoded_stream_is_encoder_recon(p64, torch_dev, tmp_path, name):
    """encode -> .p64 -> decode (y4m) reproduces the encoder's closed-loop
    reconstruction, which the fixtures hold from the reference encoder
    (including MBs forced to MTYPE 4 by a buffer overflow)."""
    z = load(f"seq_{name}.npz")
    w, h, n = int(z["width"]), int(z["height"]), int(z["nframes"])
    write_y4m(tmp_path / "in.y4m", sequence_frames(p64, z), w, h)
    enc = [CLI] + cli_flags(z) + [str(tmp_path / "in"), "-z", ".y4m", "-s", str(tmp_path / "o.p64")]
    subprocess.run(enc, check=True, stdin=cli_stdin(z), stdout=subprocess.DEVNULL, timeout=300)
    subprocess.run([CLI, "-d", "-y4m", "-s", str(tmp_path / "o.p64"), str(tmp_path / "dec")],
                   check=True, stdout=subprocess.DEVNULL, timeout=300)
    raw = (tmp_path / "dec.y4m").read_bytes()
    hdr, body = raw.split(b"\n", 1)
    assert hdr.startswith(b"YUV4MPEG2 W176 H144")
    pic = w * h * 3 // 2
    assert len(body) == n * (6 + pic)
    for t in range(n):
        c = body[t * (6 + pic):(t + 1) * (6 + pic)]
        assert c[:6] == b"FRAME\n"
        np.testing.assert_array_equal(np.frombuffer(c[6:], np.uint8), z["recon"][t], err_msg=f"t{t}")


@pytest.mark.parametrize("name", ["qcif_tss", "cif_full31"])
def test_cli_raw_component_input(p64, torch_dev, tmp_path, name):
    """Without -y4m the CLI reads <prefix><n>.Y/.U/.V per picture (MakeFileNames
    p64.c:1581); the same pictures give the reference's y4m-run stream."""
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    for t, fr in enumerate(sequence_frames(p64, z)):
        for c, (a, b) in zip("YUV", ((0, w * h), (w * h, w * h * 5 // 4), (w * h * 5 // 4, w * h * 3 // 2))):
            (tmp_path / f"raw{t}.{c}").write_bytes(fr[a:b].tobytes())
    flags = [f for f in cli_flags(z) if f != "-y4m"]
    subprocess.run([CLI] + flags + [str(tmp_path / "raw"), "-s", str(tmp_path / "o.p64")],
                   check=True, stdout=subprocess.DEVNULL, timeout=300)
    data = (tmp_path / "o.p64").read_bytes()
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])


# ---------------------------------------------------------------------------
# entropy coding on the GPU (p64gpu_vlc_pictures)

def fixture_records(z, fmt_code):
    from test_stream import gob_quant
    from p64_amd import stream
    n = int(z["nframes"])
    gq = np.stack([gob_quant(stream, fmt_code, z["usequant"][t]) for t in range(n)])
    return z["mb"].astype(np.int8), z["coef"].astype(np.int16), gq, z["usequant"].astype(np.uint8)


@pytest.mark.parametrize("name", ["qcif_tss", "qcif_q1", "qcif_intra", "cif_full31", "ntsc_tss",
                                  "qcif_rate", "qcif_prog_mq", "qcif_prog_words", "cif_scene_full31"])
def test_gpu_vlc_byte_identical(p64, torch_dev, name):
    """GPU entropy coding of the fixture's records, picture by picture at the
    stream's running bit phase, reassembled == the reference's .p64."""
    from p64_amd import stream
    torch = torch_dev
    z = load(f"seq_{name}.npz")
    w, h, n = int(z["width"]), int(z["height"]), int(z["nframes"])
    fmt = stream.format_of(w, h)
    mb, coef, gq, uq = fixture_records(z, fmt)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    asm = stream.BitAssembler()
    for t in range(n):
        out, bits = stream.vlc_pictures(d(mb[t:t + 1]), d(coef[t:t + 1]), d(gq[t:t + 1]),
                                        d(np.array([t % 32], np.int32)), width=w, height=h,
                                        phase=d(np.array([asm.phase], np.uint8)),
                                        mquant=d(uq[t:t + 1]))
        asm.append(out[0].cpu().numpy().tobytes(), bits[0])
    data = asm.end(fmt, n % 32)
    assert len(data) == int(z["stream_len"])
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])


@pytest.mark.parametrize("chunk", [None, 3 * 99 * 768])
def test_gpu_vlc_batch_matches_host_writer(p64, torch_dev, monkeypatch, chunk):
    """One launch over pictures of several sequences, each at its own phase,
    equals the host writer's bits for every picture -- also when the batch is
    split into launches of three pictures (P64GPU_CHUNK_BYTES lowers the 2 GiB
    level limit of one launch)."""
    if chunk:
        monkeypatch.setenv("P64GPU_CHUNK_BYTES", str(chunk))
    from p64_amd import stream
    torch = torch_dev
    names = ["qcif_tss", "qcif_q31", "qcif_full31", "qcif_prog_words"]
    recs, pics = [], []
    for name in names:
        z = load(f"seq_{name}.npz")
        fmt = stream.format_of(176, 144)
        mb, coef, gq, uq = fixture_records(z, fmt)
        for t in range(int(z["nframes"])):
            recs.append((mb[t], coef[t], gq[t], uq[t], t % 32))
    rng = np.random.default_rng(1)
    phases = rng.integers(0, 8, len(recs)).astype(np.uint8)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    out, bits = stream.vlc_pictures(d(np.stack([r[0] for r in recs])), d(np.stack([r[1] for r in recs])),
                                    d(np.stack([r[2] for r in recs])),
                                    d(np.array([r[4] for r in recs], np.int32)), width=176, height=144,
                                    phase=d(phases), mquant=d(np.stack([r[3] for r in recs])))
    out = out.cpu().numpy()
    for i, (mb, coef, gq, uq, tr) in enumerate(recs):
        wr = stream.Writer(stream.QCIF)
        wr.write_picture(tr, mb, coef, gq, quant_mb=uq)
        host_bits = wr.bits()
        full = wr.data()  # the complete bytes; the last partial byte is pending
        nb = (bits[i] + 7) // 8
        gpu = int.from_bytes(out[i, :nb].tobytes(), "big") >> (nb * 8 - bits[i])
        assert bits[i] - int(phases[i]) == host_bits
        assert gpu >> host_bits == 0  # the leading phase bits are zero
        assert gpu >> (host_bits - 8 * len(full)) == int.from_bytes(full, "big")


@pytest.mark.parametrize("case", ["inter_q8", "inter_q5", "inter_q31_qmb", "inter_override", "intra_q8",
                                  "intra_q3_qmb", "fused_inter"])
def test_gpu_vlc_block_bits_from_encoder(p64, torch_dev, monkeypatch, case):
    """The encoder's coded-bit counts (p64gpu_encode_args.vlc_bits, counted
    inside k_inter_mbg / k_intra_mbg from the staged levels; the fused kernel
    path through the count pass) handed to the entropy coder as blk_bits give
    the same bits as the coder's own count pass, picture for picture, and
    those equal the host writer's."""
    from p64_amd import stream
    torch = torch_dev
    if case == "fused_inter":
        monkeypatch.setenv("P64GPU_FUSED", "1")
    w, h, S = 176, 144, 6
    nmb, pic, ngob = 99, w * h * 3 // 2, 3
    rng = np.random.default_rng(abs(hash(case)) % 1000)
    fr = p64.synth_frames_device(w, h, 7, S, 0, 2, content=p64.SYNTH_SURVEY if "q8" in case else p64.SYNTH_VNOISE)
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
    r1 = torch.zeros_like(r0)
    q = int(case.split("_q")[1].split("_")[0]) if "_q" in case else 8
    qmb = (torch.from_numpy(rng.integers(1, 32, S * nmb).astype(np.uint8)).cuda() if "qmb" in case else None)
    ov = (torch.from_numpy(rng.integers(-1, 10, S * nmb).astype(np.int8)).cuda() if "override" in case else None)
    intra = case.startswith("intra")
    p64.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, quant=q)
    out = p64.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                            mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                            me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"),
                            vlc_bits=torch.full((S, nmb, 8), -1, dtype=torch.int16, device="cuda"))
    cur = fr[0] if intra else fr[1]
    p64.encode_frames(cur.reshape(-1), None if intra else r0, r1, li, width=w, height=h, intra=intra,
                      quant=q, me_mode=p64.ME_FULL, search_limit=31, quant_mb=qmb,
                      mtype_override=None if intra else ov, out=out)
    gq = torch.full((S, ngob), q, dtype=torch.uint8, device="cuda")
    mq = qmb.view(S, nmb) if qmb is not None else None
    if ov is not None:  # MQUANT types among the overrides: their MQUANT is the uniform q
        mq = torch.full((S, nmb), q, dtype=torch.uint8, device="cuda")
    tr = torch.arange(S, dtype=torch.int32, device="cuda")
    phase = torch.from_numpy(rng.integers(0, 8, S).astype(np.uint8)).cuda()
    o1, b1 = stream.vlc_pictures(out.mb, out.coef, gq, tr, width=w, height=h, phase=phase, mquant=mq)
    o1 = o1.cpu().numpy()
    o2, b2 = stream.vlc_pictures(out.mb, out.coef, gq, tr, width=w, height=h, phase=phase, mquant=mq,
                                 blk_bits=out.vlc_bits)
    assert b1 == b2
    o2 = o2.cpu().numpy()
    for i in range(S):
        nb = (b1[i] + 7) // 8
        np.testing.assert_array_equal(o1[i, :nb], o2[i, :nb], err_msg=f"{case} picture {i}")
    # the host writer's bits (the reference's, tests/test_stream.py) for the same records
    mb_h, coef_h = out.mb.cpu().numpy(), out.coef.cpu().numpy()
    for i in range(S):
        wr = stream.Writer(stream.QCIF)
        wr.write_picture(int(tr[i]), mb_h[i], coef_h[i], q, quant_mb=mq[i].cpu().numpy() if mq is not None else None)
        assert b1[i] - int(phase[i]) == wr.bits()


@pytest.mark.parametrize("name", ["qcif_intra", "qcif_full31"])
def test_gpu_vlc_levels_outside_int8(p64, torch_dev, name):
    """The coder keeps an int8 copy of the levels (p64vlc.hip VLC_STAGE): a
    picture with levels outside -128..127 (the ABI takes any int16; the
    reference's quantiser never makes them) codes from the int16 levels and
    still equals the host writer bit for bit -- the escape's 8-bit field and
    the table/escape choice by |level|, the intra DC clamp -- through both the
    coder's count pass and the emit."""
    from p64_amd import stream
    torch = torch_dev
    z = load(f"seq_{name}.npz")
    mb, coef, gq, uq = fixture_records(z, stream.format_of(176, 144))
    n = mb.shape[0]
    rng = np.random.default_rng(5)
    wide = np.array([128, -129, 200, -250, 250, 256, -256, 300, 1000, -32768, 32767], np.int16)
    coef = coef.copy()
    for t in range(0, n, 2):  # every other picture keeps its levels: both paths in one launch
        k = rng.integers(0, mb.shape[1], 12)
        coef[t, k, rng.integers(0, 6, 12), rng.integers(1, 64, 12)] = rng.choice(wide, 12)
        coef[t, k[:3], 0, 0] = [300, -5, 128]  # intra DCs clamp (1..254, 128 -> 255)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    tr = np.arange(n, dtype=np.int32) % 32
    out, bits = stream.vlc_pictures(d(mb), d(coef), d(gq), d(tr), width=176, height=144, mquant=d(uq))
    out = out.cpu().numpy()
    for t in range(n):
        wr = stream.Writer(stream.QCIF)
        wr.write_picture(int(tr[t]), mb[t], coef[t], gq[t], quant_mb=uq[t])
        full = wr.data()
        assert bits[t] == wr.bits()
        nb = (bits[t] + 7) // 8
        gpu = int.from_bytes(out[t, :nb].tobytes(), "big") >> (nb * 8 - bits[t])
        assert gpu >> (bits[t] - 8 * len(full)) == int.from_bytes(full, "big"), f"{name} picture {t}"


@pytest.mark.parametrize("given", [False, True])
def test_gpu_vlc_invalid_records(p64, torch_dev, given):
    """An invalid MB record (MTYPE outside 0..9, or a CBP type with CBP 0)
    makes its picture's bit count 0xFFFFFFFF (vlc_pictures raises), and only
    its picture's: the others of the launch equal the host writer.  A picture
    of nothing but invalid records has waves without a single bit, whose
    look-back and shared-word hand-over (p64vlc.hip) must still complete."""
    from p64_amd import stream
    torch = torch_dev
    z = load("seq_qcif_full31.npz")
    mb, coef, gq, uq = fixture_records(z, stream.format_of(176, 144))
    sel = [1, 2, 3, 4, 5]
    mb, coef, gq, uq = mb[sel].copy(), coef[sel], gq[sel], uq[sel]
    mb[1, :, 0] = 12               # every record invalid
    mb[2, 50, 0] = 10              # one
    cbpt = np.isin(mb[3, :, 0], [2, 3, 5, 6, 8, 9])
    k = int(np.flatnonzero(cbpt)[0])
    mb[3, k, 1] = 0                # a CBP type without a coded block
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    tr = np.arange(len(sel), dtype=np.int32)
    kw = {}
    if given:  # the block bits from the coder's own count of the same records
        vb = torch.zeros((len(sel), 99, 8), dtype=torch.int16, device="cuda")
        assert p64.lib().p64gpu_vlc_block_bits_(176, 144, len(sel), ctypes_ptr(d(mb)), ctypes_ptr(d(coef)),
                                                ctypes_ptr(vb), None) == 0
        kw["blk_bits"] = vb
    out, bits = stream.vlc_pictures(d(mb), d(coef), d(gq), d(tr), width=176, height=144, mquant=d(uq),
                                    host_bits=False, **kw)
    bits = [int(x) & 0xFFFFFFFF for x in bits.cpu().tolist()]
    assert bits[1] == bits[2] == bits[3] == 0xFFFFFFFF
    out = out.cpu().numpy()
    for t in (0, 4):
        wr = stream.Writer(stream.QCIF)
        wr.write_picture(int(tr[t]), mb[t], coef[t], gq[t], quant_mb=uq[t])
        assert bits[t] == wr.bits()
        full = wr.data()
        nb = (bits[t] + 7) // 8
        gpu = int.from_bytes(out[t, :nb].tobytes(), "big") >> (nb * 8 - bits[t])
        assert gpu >> (bits[t] - 8 * len(full)) == int.from_bytes(full, "big")


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


def test_gpu_vlc_graph_replay(p64, torch_dev):
    """The coder's launch (a zeroing kernel for its status words + the coder
    kernel; a captured hipMemsetAsync was seen not to order before the coder
    on replay) captured in a HIP graph and replayed
    twice gives the eager call's bits: the look-back state is reset inside
    the graph, not by the host."""
    from p64_amd import stream
    torch = torch_dev
    z = load("seq_qcif_full31.npz")
    mb, coef, gq, uq = fixture_records(z, stream.format_of(176, 144))
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    tr = d(np.arange(mb.shape[0], dtype=np.int32) % 32)
    mbd, cd, gqd, uqd = d(mb), d(coef), d(gq), d(uq)
    out0, bits0 = stream.vlc_pictures(mbd, cd, gqd, tr, width=176, height=144, mquant=uqd)
    out0 = out0.cpu().numpy()
    bufs = stream.vlc_buffers(mb.shape[0], 176, 144)
    stream.vlc_pictures(mbd, cd, gqd, tr, width=176, height=144, mquant=uqd, buffers=bufs)  # (tables)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        stream.vlc_pictures(mbd, cd, gqd, tr, width=176, height=144, mquant=uqd, buffers=bufs, host_bits=False)
    for _ in range(2):
        bufs[0].zero_()
        g.replay()
        torch.cuda.synchronize()
        bits = [int(x) & 0xFFFFFFFF for x in bufs[1][:mb.shape[0]].cpu().tolist()]
        assert bits == list(bits0)
        out = bufs[0].cpu().numpy()
        for t in range(mb.shape[0]):
            nb = (bits[t] + 7) // 8
            np.testing.assert_array_equal(out[t, :nb], out0[t, :nb])


def test_gpu_encode_with_forked_coder_graph(p64, torch_dev):
    """bench.py's with_vlc pattern: each step's encode on the capturing
    stream, its coder forked onto a side stream behind an event (beside the
    next step's encode), the bit counts stored straight into pinned host rows,
    the side stream joined at the end -- one HIP graph, replayed twice from
    the same closed-loop state.  Every step's pictures equal the host writer
    over that step's records, bit counts and bytes, on both replays."""
    from p64_amd import stream
    torch = torch_dev
    w, h, S, T = 176, 144, 6, 4
    nmb, pic = 99, 176 * 144 * 3 // 2
    fmt = stream.format_of(w, h)
    fr = p64.synth_frames_device(w, h, 7, S, 0, T + 1, content=p64.SYNTH_SURVEY)
    rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    outs = [p64.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                              mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                              me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda")) for _ in range(T)]
    p64.encode_frames(fr[0].reshape(-1), None, rec[1], li, width=w, height=h, intra=True, quant=8,
                      out=outs[0])  # picture 0 (intra), then T inter steps in the graph
    gq = torch.full((S, 3), 8, dtype=torch.uint8, device="cuda")
    trs = [torch.full((S,), 1 + k, dtype=torch.int32, device="cuda") for k in range(T)]
    vb = [stream.vlc_buffers(S, w, h) for _ in range(T)]
    host = torch.empty((T, S), dtype=torch.int32, pin_memory=True)
    stream.vlc_pictures(outs[0].mb, outs[0].coef, gq, trs[0], width=w, height=h, buffers=vb[0],
                        host_bits=False)  # (tables uploaded before the capture)
    saved = [r.clone() for r in rec] + [li.clone()]
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    ev = [torch.cuda.Event() for _ in range(T)]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        main = torch.cuda.current_stream()
        for k in range(T):
            t = 1 + k
            p64.encode_frames(fr[t].reshape(-1), rec[t % 2], rec[(t + 1) % 2], li, width=w, height=h,
                              intra=False, quant=8, me_mode=p64.ME_FULL, search_limit=31, out=outs[k])
            ev[k].record(main)
            side.wait_event(ev[k])
            with torch.cuda.stream(side):
                stream.vlc_pictures(outs[k].mb, outs[k].coef, gq, trs[k], width=w, height=h,
                                    buffers=(vb[k][0], host[k], vb[k][2]), host_bits=False)
        main.wait_stream(side)
    for rep in range(2):
        for a, b in zip(rec + [li], saved):
            a.copy_(b)
        host.zero_()
        for b in vb:
            b[0].zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        for k in range(T):
            mb, coef, data = outs[k].mb.cpu().numpy(), outs[k].coef.cpu().numpy(), vb[k][0].cpu().numpy()
            for s in range(S):
                wr = stream.Writer(fmt)
                wr.write_picture(1 + k, mb[s], coef[s], 8)
                nb, bits = wr.bits(), int(host[k, s]) & 0xFFFFFFFF
                assert bits == nb, (rep, k, s)
                full = wr.data()
                nbytes = (bits + 7) // 8
                gpu = int.from_bytes(data[s, :nbytes].tobytes(), "big") >> (nbytes * 8 - bits)
                assert gpu >> (nb - 8 * len(full)) == int.from_bytes(full, "big"), (rep, k, s)


@pytest.mark.parametrize("given", [False, True])
def test_gpu_vlc_big_path_stress(p64, torch_dev, given):
    """The coder's big path (a wave past its 8,160-bit LDS copy writes its
    words straight into memory) next to big and small neighbours, in many
    pictures per launch at every phase: dense random levels (escapes, up to
    ~5,000 bits per MB) in some 40-MB stretches, sparse ones in others.
    Every picture equals the host writer bit for bit, over repeated launches
    (the round-5 big path zeroed and ORed the words it shares with its
    neighbours in memory: a race; tests/test_vlc_protocol.py
    models the interleavings)."""
    from p64_amd import stream
    torch = torch_dev
    w, h, n, nmb, ngob = 352, 288, 48, 396, 12
    rng = np.random.default_rng(11)
    mb = np.zeros((n, nmb, 4), np.int8)
    mb[..., 1] = 0x3f
    coef = np.zeros((n, nmb, 6, 64), np.int16)
    for t in range(n):
        dense = rng.random(nmb // 20 + 1) < 0.5  # stretches of 20 raster MBs
        for k in range(nmb):
            if dense[k // 20]:
                coef[t, k] = rng.integers(-127, 128, (6, 64))
                coef[t, k, :, rng.integers(1, 64, 6)] = 0
            else:
                coef[t, k, rng.integers(0, 6, 2), rng.integers(1, 64, 2)] = rng.integers(-3, 4, 2)
            coef[t, k, :, 0] = rng.integers(1, 255, 6)
    gq = np.full((n, ngob), 1, np.uint8)
    tr = np.arange(n, dtype=np.int32) % 32
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    mbd, cd = d(mb), d(coef)
    host = []
    for t in range(n):
        wr = stream.Writer(stream.CIF)
        wr.write_picture(int(tr[t]), mb[t], coef[t], gq[t])
        host.append((wr.bits(), wr.data()))
    kw = {}
    if given:
        vb = torch.zeros((n, nmb, 8), dtype=torch.int16, device="cuda")
        assert p64.lib().p64gpu_vlc_block_bits_(w, h, n, ctypes_ptr(mbd), ctypes_ptr(cd), ctypes_ptr(vb),
                                                None) == 0
        kw["blk_bits"] = vb
    bufs = stream.vlc_buffers(n, w, h)
    for rep in range(4):
        phases = rng.integers(0, 8, n).astype(np.uint8)
        bufs[0].fill_(0xA5)  # (stale bytes: every word up to the last bit must be written)
        out, bits = stream.vlc_pictures(mbd, cd, d(gq), d(tr), width=w, height=h, phase=d(phases),
                                        buffers=bufs, **kw)
        out = out.cpu().numpy()
        for t in range(n):
            hb, full = host[t]
            assert bits[t] - int(phases[t]) == hb, (rep, t)
            nb = (bits[t] + 7) // 8
            gpu = int.from_bytes(out[t, :nb].tobytes(), "big") >> (nb * 8 - bits[t])
            assert gpu >> hb == 0, (rep, t)
            assert gpu >> (hb - 8 * len(full)) == int.from_bytes(full, "big"), (rep, t)


@pytest.mark.parametrize("given,fork", [(False, True), (True, True), (False, False)])
def test_fed_path_stitched_streams(p64, torch_dev, tmp_path, given, fork):
    """bench.py --feed root --gather coded at world 1: each step's pictures
    coded on the GPU at their sequences' bit phases (bench.CodedFeed: the
    coder forked onto the side stream beside the next step's encode, the
    output sets alternating -- or, fork=False, on the encode stream), gathered
    on the side stream, stitched on rank 0 (stitch_pieces): byte-identical to
    the host writer over the same records (p64s_write_picture) and to the
    .p64 the CLI writes for those pictures (p64.c:524-613, stream.c:142-150,
    193)."""
    import sys
    sys.path.insert(0, REPO)
    import bench
    from p64_amd import stream
    torch = torch_dev
    w, h, S, n = 352, 288, 4, 6
    nmb, pic = 396, w * h * 3 // 2
    fr = p64.synth_frames_device(w, h, 3, S, 0, n, content=p64.SYNTH_SURVEY)
    rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    outs = [p64.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                              mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                              me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"),
                              vlc_bits=(torch.empty((S, nmb, 8), dtype=torch.int16, device="cuda")
                                        if given else None)) for _ in range(2)]
    feed = bench.CodedFeed(torch, stream, 1, 0, S, w, h, 8, keep=range(S))
    assert feed.fork  # (the default)
    feed.fork = fork
    fmt = stream.format_of(w, h)
    host = [stream.Writer(fmt) for _ in range(S)]
    for t in range(n):
        out = outs[t % 2]
        feed.before_encode(t)  # (the coder of step t-2 read this set)
        out.coef.zero_()  # (inter pictures store only their nonzero blocks)
        p64.encode_frames(fr[t].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li, width=w, height=h,
                          intra=(t == 0), quant=8, me_mode=p64.ME_FULL, search_limit=31, out=out)
        feed.code(t, out)
        mb, coef = out.mb.cpu().numpy(), out.coef.cpu().numpy()
        for s in range(S):
            host[s].write_picture(t % 32, mb[s], coef[s], 8)
    feed.finish()
    got = feed.streams(fmt, n % 32)
    for s in range(S):
        data, nbits = got[s]
        assert nbits == host[s].bits(), s
        assert data == host[s].end(n % 32), s
    frames = fr.cpu().numpy()
    for s in (0, S - 1):
        write_y4m(tmp_path / f"in{s}.y4m", [frames[t, s] for t in range(n)], w, h)
        subprocess.run([CLI, "-CIF", "-y4m", "-a", "0", "-b", str(n - 1), "-q", "8", "-i", "31", "-full",
                        str(tmp_path / f"in{s}"), "-z", ".y4m", "-s", str(tmp_path / f"o{s}.p64")],
                       check=True, stdout=subprocess.DEVNULL, timeout=300)
        assert (tmp_path / f"o{s}.p64").read_bytes() == got[s][0], s


def test_gpu_vlc_bits_in_pinned_host_memory(p64, torch_dev):
    """p64gpu_vlc_args.bits in hipHostMalloc'd (pinned) host memory: the coder
    writes the bit counts there directly, eagerly and captured in a HIP graph
    replayed several times (the round-5 with_vlc variant that ended in an
    illegal-address fault wrote them into a torch pin_memory tensor;
    tools/vlc_fault_probe.py reconstructs it).  Pageable host memory is
    refused by the ABI (include/p64gpu.h), not handed to the kernel."""
    import ctypes
    from p64_amd import stream
    torch = torch_dev
    z = load("seq_qcif_full31.npz")
    mb, coef, gq, uq = fixture_records(z, stream.format_of(176, 144))
    n = mb.shape[0]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    tr = d(np.arange(n, dtype=np.int32) % 32)
    mbd, cd, gqd, uqd = d(mb), d(coef), d(gq), d(uq)
    _, want = stream.vlc_pictures(mbd, cd, gqd, tr, width=176, height=144, mquant=uqd)
    hip = None
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                hip = ctypes.CDLL(line.split()[-1])
                break
    hp = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(4 * n), 0) == 0
    try:
        host = np.frombuffer((ctypes.c_uint32 * n).from_address(hp.value), np.uint32)
        out, _, scr = stream.vlc_buffers(n, 176, 144)

        def call(bits_ptr):
            a = stream.VlcArgs(width=176, height=144, nframes=n, flags=0, mb=mbd.data_ptr(), coef=cd.data_ptr(),
                               gquant=gqd.data_ptr(), mquant=uqd.data_ptr(), tr=tr.data_ptr(), phase=None,
                               out=out.data_ptr(), out_stride=int(out.shape[1]), bits=bits_ptr,
                               scratch=scr.data_ptr(), blk_bits=None)
            return p64.lib().p64gpu_vlc_pictures(ctypes.byref(a), p64._stream(torch))

        host[:] = 0
        assert call(hp.value) == 0
        torch.cuda.synchronize()
        assert host.tolist() == list(want)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            assert call(hp.value) == 0
        for _ in range(3):
            host[:] = 0
            g.replay()
            torch.cuda.synchronize()
            assert host.tolist() == list(want)
        del g
        pageable = np.zeros(n, np.uint32)
        assert call(pageable.ctypes.data) == -1  # P64GPU_E_INVALID
        assert b"device-addressable" in p64.lib().p64gpu_last_error()
        assert not pageable.any()
    finally:
        hip.hipHostFree(hp)


@pytest.mark.parametrize("name", ["qcif_tss", "cif_full31", "qcif_q1"])
def test_gpu_vlc_seq_bits_continue_the_stream(p64, torch_dev, name):
    """p64gpu_vlc_args.seq_bits (ABI v3): each picture starts at its
    sequence's running bit count & 7 and the count advances on the device,
    call after call, with no host round trip; max_bits gets the longest
    picture.  Two copies of the fixture's sequence side by side (one starting
    5 bits into its stream), reassembled == the reference's .p64."""
    from p64_amd import stream
    torch = torch_dev
    z = load(f"seq_{name}.npz")
    w, h, n = int(z["width"]), int(z["height"]), int(z["nframes"])
    fmt = stream.format_of(w, h)
    mb, coef, gq, uq = fixture_records(z, fmt)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    seq = torch.tensor([0, 5], dtype=torch.int64, device="cuda")
    mx = torch.zeros(1, dtype=torch.int32, device="cuda")
    bufs = stream.vlc_buffers(2, w, h)
    asm = [stream.BitAssembler(), stream.BitAssembler()]
    asm[1].append(b"\xa8", 5)  # (5 bits of something before the second copy's stream)
    for t in range(n):
        two = lambda a: np.stack([a[t], a[t]])  # noqa: E731
        out, bits = stream.vlc_pictures(d(two(mb)), d(two(coef)), d(two(gq)), d(np.array([t % 32] * 2, np.int32)),
                                        width=w, height=h, mquant=d(two(uq)), buffers=bufs, seq_bits=seq,
                                        max_bits=mx)
        assert int(mx.item()) == max(bits)
        o = out.cpu().numpy()
        for i in range(2):
            asm[i].append(o[i].tobytes(), bits[i])
        assert seq.cpu().tolist() == [asm[0].nbits, asm[1].nbits]
    data = asm[0].end(fmt, n % 32)
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])
    data1 = asm[1].end(fmt, n % 32)
    assert len(data1) == len(data) + 1 or len(data1) == len(data)  # (shifted by 5 bits)
