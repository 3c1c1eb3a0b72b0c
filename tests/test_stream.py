"""H.261 bitstream layer (include/p64stream.h, p64_amd.stream) on the CPU.

Pinned by the reference's own outputs:
  * writer: the .p64 the reference CLI wrote for every golden sequence
    (stream_sha256 / stream_len in tests/golden/seq_*.npz), regenerated here
    from the fixture's per-MB records -- byte-identical;
  * reader: the reference's short.p64 (tests/golden/short.p64, a data file the
    reference ships) decoded to the 21 plane MD5s of `p64 -d -s short.p64`
    (tests/golden/decode.json); the pixel reconstruction in this CPU test is the
    oracle's (test infrastructure), the GPU test of the same stream is in
    test_gpu_stream.py.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_oracle_golden import ALL_SEQS, load

FMTS = {"QCIF": 0, "CIF": 1, "NTSC": 2}


@pytest.fixture(scope="module")
def st(p64):
    from p64_amd import stream
    return stream


def gob_quant(st, fmt, usequant):
    """GQUANT of each GOB = UseQuant of its first MDU (no MQUANT in the fixtures)."""
    _, _, ngob = st.geometry(fmt)
    first = [(3 * g) * 11 if fmt == st.QCIF else ((g >> 1) * 3) * 22 + (g & 1) * 11
             for g in range(ngob)]
    return np.asarray(usequant)[first].astype(np.uint8)


def write_fixture_stream(st, z):
    fmt = FMTS[str(z["fmt"])]
    w = st.Writer(fmt)
    n = int(z["nframes"])
    for t in range(n):
        w.write_picture(t % 32, z["mb"][t].astype(np.int8), z["coef"][t],
                        gob_quant(st, fmt, z["usequant"][t]),
                        quant_mb=z["usequant"][t].astype(np.uint8))  # MQUANT of types 1/3/6/9
    return w.end(n % 32)


@pytest.mark.parametrize("name", ALL_SEQS)
def test_writer_byte_identical_to_reference(st, name):
    z = load(f"seq_{name}.npz")
    data = write_fixture_stream(st, z)
    assert len(data) == int(z["stream_len"])
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])


def coded_block_mask(p64, mb):
    """[nmb, 6] True where WriteMDU emits the block (p64.c:929-931)."""
    mt = mb["mtype"].astype(int)
    cbp = np.where(np.asarray(p64.CBP_MTYPE)[mt] == 1, mb["cbp"].astype(int) & 63, 63)
    tc = np.asarray(p64.TCOEFF_MTYPE)[mt] == 1
    bits = (cbp[:, None] >> (5 - np.arange(6))[None, :]) & 1
    return (bits == 1) & tc[:, None]


@pytest.mark.parametrize("name", ["qcif_tss", "qcif_q31", "qcif_intra", "cif_full31", "ntsc_tss",
                                  "qcif_q1"])
def test_reader_round_trip(p64, st, name):
    z = load(f"seq_{name}.npz")
    r = st.Reader(write_fixture_stream(st, z))
    assert r.fmt == FMTS[str(z["fmt"])]
    pics = list(r)
    n = int(z["nframes"])
    assert len(pics) == n and r.end_tr == n % 32
    for t, p in enumerate(pics):
        assert p.tr == t % 32
        assert p.coded.all()
        mb = z["mb"][t].astype(np.int8)
        mt = mb[:, 0]
        np.testing.assert_array_equal(p.mb["mtype"], mt)
        mf = np.asarray(p64.MF_MTYPE)[mt] == 1
        np.testing.assert_array_equal(p.mb["mvx"], np.where(mf, mb[:, 2], 0))
        np.testing.assert_array_equal(p.mb["mvy"], np.where(mf, mb[:, 3], 0))
        cbpt = np.asarray(p64.CBP_MTYPE)[mt] == 1
        np.testing.assert_array_equal(p.mb["cbp"][cbpt], mb[cbpt, 1])
        np.testing.assert_array_equal(p.quant_mb, z["usequant"][t])
        mask = coded_block_mask(p64, p.mb)
        exp = z["coef"][t].copy()
        intra = np.asarray(p64.INTRA_MTYPE)[mt] == 1
        exp[intra, :, 0] = np.clip(exp[intra, :, 0], 1, 254)  # EncodeDC clamp, codec.c:345-346
        np.testing.assert_array_equal(p.coef[mask], exp[mask])
        assert not p.coef[~mask].any()


def random_records(p64, rng, nmb, width, height, *, mtypes=range(10)):
    mt = rng.choice(list(mtypes), nmb).astype(np.int8)
    mb = np.zeros(nmb, p64.MB_DTYPE)
    mb["mtype"] = mt
    mb["cbp"] = rng.integers(1, 64, nmb)
    # vectors keep the 16x16 source inside the picture (the reader rejects others)
    x0 = 16 * (np.arange(nmb) % (width // 16))
    y0 = 16 * (np.arange(nmb) // (width // 16))
    mb["mvx"] = np.clip(rng.integers(-15, 16, nmb), -x0, width - 16 - x0)
    mb["mvy"] = np.clip(rng.integers(-15, 16, nmb), -y0, height - 16 - y0)
    coef = np.zeros((nmb, 6, 64), np.int16)
    for k in range(nmb):
        for c in range(6):
            nz = rng.integers(1, 12)
            pos = rng.choice(64, nz, replace=False)
            # long runs, escapes (|l| > 15 or run > 26), the run-27/level-1 code
            # that collides with ESCAPE's own table value
            coef[k, c, pos] = rng.choice([-127, -40, -16, -15, -2, -1, 1, 2, 3, 15, 16, 77, 127], nz)
        if rng.random() < 0.2:
            coef[k, :, :] = 0
            coef[k, 0, 28] = 1  # run 27 after an intra DC / 28 from 0
        if p64.INTRA_MTYPE[mt[k]]:
            coef[k, :, 0] = rng.choice([1, 127, 128, 129, 254], 6)
    # a CBP block must hold a nonzero level (WriteMDU would emit nothing for it)
    nz = coef.astype(bool).any(axis=2)
    mb["cbp"] = (nz * (1 << (5 - np.arange(6)))[None, :]).sum(axis=1) & rng.integers(1, 64, nmb)
    mb["cbp"][mb["cbp"] == 0] = 32
    return mb, coef


def test_round_trip_escapes_mquant_and_mv_prediction(p64, st):
    rng = np.random.default_rng(3)
    for fmt in (st.QCIF, st.CIF, st.NTSC):
        w = st.Writer(fmt)
        nmb = w.nmb
        sent = []
        for t in range(3):
            mb, coef = random_records(p64, rng, nmb, w.width, w.height)
            qm = rng.integers(1, 32, nmb).astype(np.uint8)
            gq = rng.integers(1, 32, w.ngob).astype(np.uint8)
            w.write_picture(5 * t + 30, mb, coef, gq, quant_mb=qm)
            sent.append((mb, coef, qm, gq))
        data = w.end(12)
        r = st.Reader(data)
        pics = list(r)
        assert [p.tr for p in pics] == [30, 3, 8] and r.end_tr == 12
        for p, (mb, coef, qm, gq) in zip(pics, sent):
            mt = mb["mtype"].astype(int)
            np.testing.assert_array_equal(p.mb["mtype"], mb["mtype"])
            mf = np.asarray(p64.MF_MTYPE)[mt] == 1
            np.testing.assert_array_equal(p.mb["mvx"], np.where(mf, mb["mvx"], 0))
            np.testing.assert_array_equal(p.mb["mvy"], np.where(mf, mb["mvy"], 0))
            mask = coded_block_mask(p64, p.mb)
            np.testing.assert_array_equal(p.coef[mask], coef[mask])
            # UseQuant: MQUANT where sent, and it persists as GQuant for the
            # rest of the GOB (p64.c:1205-1208)
            gob_of = np.empty(nmb, int)
            order = []
            for g in range(w.ngob):
                for m in range(33):
                    k = ((3 * g + m // 11) * 11 + m % 11 if fmt == st.QCIF else
                         ((g >> 1) * 3 + m // 11) * 22 + (g & 1) * 11 + m % 11)
                    gob_of[k] = g
                    order.append(k)
            exp_q = np.empty(nmb, np.uint8)
            cur = None
            for i, k in enumerate(order):
                if i % 33 == 0:
                    cur = gq[gob_of[k]]
                if p64.QUANT_MTYPE[mt[k]]:
                    cur = qm[k]
                exp_q[k] = cur
            np.testing.assert_array_equal(p.quant_mb, exp_q)


def test_intra_dc_128_is_sent_as_255(p64, st):
    mb = np.zeros(99, p64.MB_DTYPE)
    mb["cbp"] = 63
    coef = np.zeros((99, 6, 64), np.int16)
    coef[:, :, 0] = 128
    w = st.Writer(st.QCIF)
    w.write_picture(0, mb, coef, 8)
    data = w.end(1)
    # picture header 32 bits, GOB header 26 bits, MBA "1", MTYPE "0001", DC
    bits = "".join(f"{b:08b}" for b in data)
    assert bits[32 + 26 + 5: 32 + 26 + 5 + 8] == "11111111"
    p = st.Reader(data).read()
    assert (p.coef[:, :, 0] == 128).all()


class Bits:
    def __init__(self):
        self.s = ""

    def put(self, n, v):
        self.s += format(v & ((1 << n) - 1), f"0{n}b")

    def code(self, bits):
        self.s += bits.replace(" ", "")

    def bytes(self):
        s = self.s + "1" * (-len(self.s) % 8)
        return bytes(int(s[i:i + 8], 2) for i in range(0, len(s), 8))


def test_reader_skipped_mbs_stuffing_and_mquant(p64, st):
    """Hand-built stream: MBA stuffing, skipped MDUs (MBA > 1 resets the MV
    predictor), MQUANT, an escaped level of -128 and a picture with no GOBs."""
    b = Bits()
    b.put(20, 0x10); b.put(5, 3); b.put(6, 0); b.put(1, 0)  # QCIF picture, TR 3
    b.put(16, 1); b.put(4, 3); b.put(5, 9); b.put(1, 0)     # GN 3 -> GOB 1, GQUANT 9
    b.code("0000 0001 111")                                   # stuffing
    b.code("0010")                                            # MBA 5 -> MDU 4
    b.code("0000 0001")                                       # MTYPE 5 (MC + coded)
    b.code("0010"); b.code("0011")                            # MVD +2, -2
    b.code("0101 1")                                          # CBP 1 (V only)
    b.code("1"); b.put(1, 1)                                  # first coef (0,1) = -1
    b.code("0000 01"); b.put(6, 3); b.put(8, 0x80)            # escape run 3 level -128
    b.code("10")                                              # EOB
    b.code("1")                                               # MBA 1 -> MDU 5
    b.code("0000 01"); b.put(5, 17)                           # MTYPE 9, MQUANT 17
    b.code("011"); b.code("1")                                # MVD -1 (predicted), 0
    b.code("0100 1")                                          # CBP 2 (U only)
    b.code("0101"); b.put(1, 0); b.code("10")                 # (2,1) +1, EOB
    b.code("0000 0000 0000 0001")                             # start code (MBA 35)
    b.put(4, 0)                                               # GN 0: next picture
    b.put(5, 4); b.put(6, 0); b.put(1, 0)                     # TR 4, no GOBs
    b.put(16, 1); b.put(4, 0)                                 # PSC again
    b.put(5, 9); b.put(6, 0); b.put(1, 0)                     # trailer TR 9
    r = st.Reader(b.bytes())
    p = r.read()
    assert p.tr == 3 and p.coded.sum() == 2
    k4, k5 = (3 + 0) * 11 + 4, (3 + 0) * 11 + 5
    assert p.coded[k4] and p.coded[k5]
    assert tuple(p.mb[k4]) == (5, 1, 2, -2) and p.quant_mb[k4] == 9
    assert p.coef[k4, 5, 0] == -1 and p.coef[k4, 5, 4] == -128 and p.coef[k4].astype(bool).sum() == 2
    assert tuple(p.mb[k5]) == (9, 2, 1, -2) and p.quant_mb[k5] == 17
    assert p.coef[k5, 4, 2] == 1 and p.coef[k5].astype(bool).sum() == 1
    p2 = r.read()
    assert p2.tr == 4 and not p2.coded.any()
    assert r.read() is None and r.end_tr == 9
    assert st.output_schedule([3, 4], 9) == [1, 5]


def test_reader_rejects_garbage(p64, st):
    with pytest.raises(p64.P64GpuError):
        st.Reader(b"\x12\x34\x56\x78\x9a")
    b = Bits()
    b.put(20, 0x10); b.put(5, 0); b.put(6, 0); b.put(1, 0)
    b.put(16, 1); b.put(4, 1); b.put(5, 8); b.put(1, 0)
    b.code("1"); b.code("0000 0000 00")                       # MBA 1, invalid MTYPE prefix
    r = st.Reader(b.bytes() + b"\x00\x00")
    with pytest.raises(p64.P64GpuError, match="bitstream"):
        r.read()


def test_reader_rejects_vectors_outside_the_picture(p64, st):
    """A vector that would fetch the 16x16 prediction from outside the picture
    (H.261 forbids it; a conforming encoder never sends it) is a stream error,
    so a hostile stream cannot steer the GPU reconstruction out of bounds."""
    for mbx, mby, mvx, mvy in ((0, 0, -1, 0), (0, 0, 0, -3), (10, 8, 1, 0), (10, 8, 0, 15),
                               (5, 4, -15, 15), (5, 4, 15, -15), (0, 8, 0, 0)):
        mb = np.zeros(99, p64.MB_DTYPE)
        mb["mtype"] = 2          # inter, zero vector, CBP: one coded level per MB
        mb["cbp"] = 32
        coef = np.zeros((99, 6, 64), np.int16)
        coef[:, 0, 0] = 1
        k = mby * 11 + mbx
        mb[k] = (4, 0, mvx, mvy)  # MC without coefficients
        w = st.Writer(st.QCIF)
        w.write_picture(0, mb, coef, 8)
        r = st.Reader(w.end(1))
        x, y = 16 * mbx + mvx, 16 * mby + mvy
        if 0 <= x <= 176 - 16 and 0 <= y <= 144 - 16:
            assert tuple(r.read().mb[k])[2:] == (mvx, mvy)
        else:
            with pytest.raises(p64.P64GpuError, match="outside the picture"):
                r.read()


def test_writer_rejects_bad_records(p64, st):
    w = st.Writer(st.QCIF)
    mb = np.zeros(99, p64.MB_DTYPE)
    coef = np.zeros((99, 6, 64), np.int16)
    mb["mtype"][7] = 2  # CBP type with CBP 0
    with pytest.raises(p64.P64GpuError):
        w.write_picture(0, mb, coef, 8)
    mb["mtype"][7] = 3  # MQUANT type without quant_mb
    mb["cbp"][7] = 5
    with pytest.raises(p64.P64GpuError):
        w.write_picture(0, mb, coef, 8)
    assert w.bits() == 0  # a rejected picture writes nothing


def test_output_schedule_matches_reference_rules(st):
    assert st.output_schedule([0, 1, 2], 3) == [1, 1, 1]
    assert st.output_schedule([0, 2, 5], 6) == [2, 3, 1]  # skipped TRs repeat the picture
    assert st.output_schedule([30, 31, 0, 1], 2) == [1, 1, 1, 1]  # TR wraps mod 32


@pytest.mark.parametrize("force_cif", [False, True])
def test_decode_short_p64_matches_reference_md5(p64, st, oracle_mod, force_cif):
    """Plain decode, and -c (ForceCIF, p64.c:1071-1072): the NTSC stream decoded
    into CIF frames, GOBs 11-12 never sent (reference MD5s of `p64 -d -c`)."""
    data = open(os.path.join(GOLDEN, "short.p64"), "rb").read()
    exp = json.load(open(os.path.join(GOLDEN, "decode_forcecif.json" if force_cif else "decode.json")))
    r = st.Reader(data, force_cif=force_cif)
    w, h = r.width, r.height
    assert (r.fmt, w, h) == ((st.CIF, 352, 288) if force_cif else (st.NTSC, 352, 240))
    prev = np.zeros(w * h * 3 // 2, np.uint8)
    pics, trs = [], []
    for p in r:
        rec = prev.copy()
        for k in np.nonzero(p.coded)[0]:
            m = p.mb[k]
            oracle_mod.decode_mb(w, h, prev, rec, int(k) % (w // 16), int(k) // (w // 16),
                                 int(m["mtype"]), int(m["cbp"]), int(m["mvx"]), int(m["mvy"]),
                                 int(p.quant_mb[k]), p.coef[k])
        pics.append(rec)
        trs.append(p.tr)
        prev = rec
    out = [pic for pic, n in zip(pics, st.output_schedule(trs, r.end_tr)) for _ in range(n)]
    assert len(out) == 7
    for i, pic in enumerate(out):
        planes = (pic[:w * h], pic[w * h:w * h * 5 // 4], pic[w * h * 5 // 4:])
        for c, a in zip("YUV", planes):
            key = f"{'sc' if force_cif else 'short'}{i}.{c}"
            assert hashlib.md5(a.tobytes()).hexdigest() == exp[key], key


def test_force_cif_refused_after_first_picture(p64, st):
    """p64s_reader_force_cif changes the geometry the caller sized its arrays
    for: once a picture has been read it is refused, before that
    it is accepted."""
    import ctypes
    data = open(os.path.join(GOLDEN, "short.p64"), "rb").read()
    r = st.Reader(data)
    assert r.read() is not None
    assert p64.lib().p64s_reader_force_cif(r._h) == -1
    assert b"already read" in p64.lib().p64gpu_last_error()
    r2 = st.Reader(data)
    assert p64.lib().p64s_reader_force_cif(r2._h) == 0
    info = st._Info()
    assert p64.lib().p64s_reader_info(r2._h, ctypes.byref(info)) == 0
    assert (info.width, info.height) == (352, 288)


def test_pack_levels_matches_restatement(p64):
    """p64s_pack_levels (the packed layout of p64gpu_decode_recon_packed) on
    the reader's output of short.p64 and on a golden sequence's records:
    exactly the blocks DecompressMDU reads (p64.c:1200-1217: MB present,
    MTYPE with coefficients, CBP bit) in raster order, and per 64-block
    group of the batch (groups straddle pictures) its first block's index
    and mask."""
    import numpy as np
    from p64_amd import stream
    from test_oracle_golden import load
    TC = np.array(p64.TCOEFF_MTYPE)
    CB = np.array(p64.CBP_MTYPE)

    def restate(mb, coded, coef, nmb):
        n = coded.size // nmb
        mt = mb["mtype"].astype(int).reshape(n, nmb)
        cbp = np.where(CB[mt] == 1, mb["cbp"].astype(int).reshape(n, nmb) & 63, 63)
        bits = (cbp[..., None] >> (5 - np.arange(6))) & 1
        tx = (bits * TC[mt][..., None] * (coded.reshape(n, nmb)[..., None] != 0)).reshape(n * 6 * nmb)
        ngr = (n * 6 * nmb + 63) // 64  # groups of 64 consecutive blocks of the batch
        pad = np.zeros(ngr * 64, np.int64)
        pad[:n * 6 * nmb] = tx
        g = pad.reshape(-1, 64)
        cnt = g.sum(1)
        m = (g.astype(np.uint64) << np.arange(64, dtype=np.uint64)).sum(1, dtype=np.uint64)
        return coef.reshape(n * 6 * nmb, 64)[tx == 1], np.cumsum(cnt) - cnt, m

    r = stream.Reader(open(os.path.join(GOLDEN, "short.p64"), "rb").read())
    pics = list(r)
    cases = [(r.fmt, np.stack([p.mb for p in pics]), np.stack([p.coded for p in pics]),
              np.stack([p.coef for p in pics]))]
    z = load("seq_cif_full31.npz")
    mbz = z["mb"].astype(np.int8).reshape(-1, 4).view(p64.MB_DTYPE).reshape(-1)
    coded = np.ones(mbz.size, np.uint8)
    coded[::7] = 0
    cases.append((stream.CIF, mbz, coded, z["coef"].astype(np.int16)))
    for fmt, mb, cd, coef in cases:
        nmb = stream.geometry(fmt)[2] * 33
        lv, ix = stream.pack_levels(fmt, mb, cd, coef)
        elv, start, m = restate(np.asarray(mb).reshape(-1), cd.reshape(-1), coef, nmb)
        np.testing.assert_array_equal(lv, elv)
        np.testing.assert_array_equal(ix[:, 0], start)
        assert not ix[:, 1].any()
        np.testing.assert_array_equal(ix[:, 2].astype(np.uint64) | (ix[:, 3].astype(np.uint64) << np.uint64(32)), m)


def test_pack_levels_device_matches_host_packer(p64, monkeypatch):
    """p64_amd.pack_levels_device (the bench's packer, torch ops -- run here
    on CPU tensors) writes the same levels and index as p64s_pack_levels, for
    QCIF and CIF batches whose groups straddle pictures."""
    import numpy as np
    import torch
    from p64_amd import stream
    monkeypatch.setattr(p64, "_torch", lambda: torch)
    rng = np.random.default_rng(1)
    for w, h in ((176, 144), (352, 288)):
        nmb, S = (w // 16) * (h // 16), 7
        mb = np.zeros((S, nmb, 4), np.int8)
        mb[..., 0] = rng.integers(0, 10, (S, nmb))
        mb[..., 1] = rng.integers(1, 64, (S, nmb))
        coef = rng.integers(-5, 5, (S, nmb, 6, 64)).astype(np.int16)
        coded = (rng.random((S, nmb)) > 0.2).astype(np.uint8)
        lv, n, ix = p64.pack_levels_device(torch.tensor(coef), torch.tensor(mb), torch.tensor(coded), w, h)
        lv2, ix2 = stream.pack_levels(stream.format_of(w, h), mb.reshape(-1, 4).view(p64.MB_DTYPE).reshape(-1),
                                      coded, coef)
        assert n == len(lv2)
        np.testing.assert_array_equal(lv.numpy(), lv2)
        np.testing.assert_array_equal(ix.numpy().view(np.uint32), ix2)
