"""Pin the CPU oracle (oracle/p64_oracle.c) to the reference's own outputs.

Golden vectors in tests/golden/ were captured from the unmodified reference
(tests/golden/make_golden.py): per-function vectors from chendct.c/transform.c/
me.c built as a shared library, and whole-encoder runs of the reference CLI with
link-time hooks.  Every comparison here is bit-exact.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN

MF = np.array([0, 0, 0, 0, 1, 1, 1, 1, 1, 1], bool)


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def test_blocks_dct_idct(oracle_mod):
    z = load("blocks.npz")
    np.testing.assert_array_equal(oracle_mod.block_apply("orc_chen_dct", z["dct_in"]), z["dct_out"])
    np.testing.assert_array_equal(oracle_mod.block_apply("orc_chen_idct", z["idct_in"]), z["idct_out"])


@pytest.mark.parametrize("q", range(1, 32))
def test_blocks_quant(oracle_mod, q):
    z = load("blocks.npz")
    qin = z["quant_in"]
    np.testing.assert_array_equal(oracle_mod.block_apply("orc_quant_inter", qin, q, q), z[f"inter_q{q}"])
    np.testing.assert_array_equal(oracle_mod.block_apply("orc_quant_intra", qin, 8, q), z[f"intra_q{q}"])
    lv = z[f"ilev_q{q}"]
    np.testing.assert_array_equal(oracle_mod.block_apply("orc_iquant_inter", lv, q, q), z[f"iinter_q{q}"])
    np.testing.assert_array_equal(oracle_mod.block_apply("orc_iquant_intra", lv, 8, q), z[f"iintra_q{q}"])


def test_blocks_bounds_zigzag(oracle_mod):
    z = load("blocks.npz")
    b = z["bound_in"]
    for fn, key in (("orc_bound_dct", "bound_dct"), ("orc_bound_idct", "bound_idct"),
                    ("orc_bound_quant_flat", "bound_qflat"), ("orc_bound_quant", "bound_quant")):
        np.testing.assert_array_equal(oracle_mod.block_apply(fn, b), z[key], err_msg=fn)
    np.testing.assert_array_equal(oracle_mod.block_apply("orc_zigzag", z["zz_in"]), z["zz_out"])
    np.testing.assert_array_equal(oracle_mod.block_apply("orc_izigzag", z["zz_in"]), z["izz_out"])


@pytest.mark.parametrize("key,mode,sl", [("full31", 1, 31), ("full15", 1, 15), ("full7", 1, 7),
                                         ("tss", 0, 15)])
def test_motion_estimation(oracle_mod, key, mode, sl):
    z = load("me.npz")
    w, h = int(z["width"]), int(z["height"])
    for i, name in enumerate(z["names"]):
        got = oracle_mod.motion_estimation(z["ref"][i], z["cur"][i], w, h, mode, sl)
        got = np.stack([got[f] for f in got.dtype.names], axis=1)
        np.testing.assert_array_equal(got, z[key][i], err_msg=f"{key} case {name}")


def test_me_two_exact_matches_dx_major(oracle_mod):
    """exact matches at (+5,-3) and (-4,+6) -> FastBME picks (-4,+6)."""
    z = load("me.npz")
    i = list(z["names"]).index("twomatch")
    w = int(z["width"])
    mb = (48 // 16) * (w // 16) + 48 // 16
    assert tuple(z["full31"][i][mb][:3]) == (-4, 6, 0)


ALL_SEQS = sorted(f[4:-4] for f in os.listdir(GOLDEN) if f.startswith("seq_") and f.endswith(".npz"))


def _rate_controlled(name):
    z = np.load(os.path.join(GOLDEN, f"seq_{name}.npz"))
    return tuple(int(z[k]) if k in z.files else 0 for k in ("rate", "filesize"))


# fixed-quantiser runs: every picture at -q; the oracle and the batched GPU API
# reproduce them directly.  Rate-controlled runs (-r/-x) choose GQUANT per GOB
# from the bits written; they pin the sequence encoder (p64seq) instead.
def _program(name):
    return str(np.load(os.path.join(GOLDEN, f"seq_{name}.npz"))["oracle"])


# -o runs other than intra_only.prog (a constant MTYPE) are driven by the
# program interpreter and pin the sequence encoder as well
INTRA_PROG = "intra_only.prog"
SEQS = [s for s in ALL_SEQS if _rate_controlled(s) == (0, 0) and _program(s) in ("", INTRA_PROG)]
RATE_SEQS = [s for s in ALL_SEQS if _rate_controlled(s) != (0, 0) and not _program(s)]
PROG_SEQS = [s for s in ALL_SEQS if _program(s) not in ("", INTRA_PROG)]


def check_sequence_outputs(z, outs, label):
    """Compare one encoded sequence with a golden reference run."""
    nf = int(z["nframes"])
    assert len(outs) == nf
    for t, (coef, mb, me, recon) in enumerate(outs):
        ref_mb = z["mb"][t]
        mt = mb["mtype"].astype(int)
        np.testing.assert_array_equal(mt, ref_mb[:, 0], err_msg=f"{label} mtype frame {t}")
        np.testing.assert_array_equal(mb["cbp"].astype(int) & 0x3f, ref_mb[:, 1] & 0x3f,
                                      err_msg=f"{label} cbp frame {t}")
        exp_mvx = np.where(MF[ref_mb[:, 0]], ref_mb[:, 2], 0)
        exp_mvy = np.where(MF[ref_mb[:, 0]], ref_mb[:, 3], 0)
        np.testing.assert_array_equal(mb["mvx"], exp_mvx, err_msg=f"{label} mvx frame {t}")
        np.testing.assert_array_equal(mb["mvy"], exp_mvy, err_msg=f"{label} mvy frame {t}")
        np.testing.assert_array_equal(coef, z["coef"][t], err_msg=f"{label} coef frame {t}")
        if t > 0:
            got = np.stack([me[f] for f in me.dtype.names], axis=1)
            np.testing.assert_array_equal(got, z["merec"][t], err_msg=f"{label} ME frame {t}")
            # ReadCompressMDU's MVDH/MVDV are the ME vector (p64.c:740-741)
            np.testing.assert_array_equal(ref_mb[:, 2], z["merec"][t][:, 0])
        digest = hashlib.sha256(np.ascontiguousarray(recon).tobytes()).hexdigest()
        assert digest == z["recon_sha256"][t], f"{label} recon frame {t}"


def sequence_params(z):
    me_mode = 1 if str(z["me"]) == "full" else 0
    ov = None
    if str(z["oracle"]) == INTRA_PROG:  # program 0 stores MTYPE 0
        ov = np.zeros(int(z["mb"].shape[1]), np.int8)
    return dict(quant=int(z["q"]), me_mode=me_mode, search_limit=int(z["sl"]), mtype_override=ov)


def sequence_frames(p64, z):
    w, h = int(z["width"]), int(z["height"])
    if int(z["seed"]) < 0:  # constructed pictures (make_golden.py make_tie_frames), kept as data
        frames = [np.ascontiguousarray(f) for f in z["frames"]]
    else:
        frames = [p64.synth_frame(int(z["seed"]), t, w, h) for t in range(int(z["nframes"]))]
    for t, f in enumerate(frames):  # pins the synthetic generator
        assert hashlib.sha256(f.tobytes()).hexdigest() == z["frames_sha256"][t]
    return frames


@pytest.mark.parametrize("name", SEQS)
def test_sequence_golden(oracle_mod, p64, name):
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    assert (z["usequant"] == int(z["q"])).all()
    frames = sequence_frames(p64, z)
    outs = oracle_mod.encode_sequence(frames, w, h, **sequence_params(z))
    check_sequence_outputs(z, outs, name)
    if "recon" in z.files:
        for t in range(int(z["nframes"])):
            np.testing.assert_array_equal(outs[t][3], z["recon"][t])


def tie_mbs(z, t):
    """Macroblocks of picture t that reach the binary64 tie of the MTYPE
    decision (p64.c:745-756): VAR < 64 or VAROR > VAR, x = OMV/256 >= 3 (so
    neither earlier inter test fires) and 11 MV == 10 OMV, where `y > x/1.1`
    is decided by the rounding of the double quotient."""
    me = z["merec"][t]
    sad, sad0, var, varor = me[:, 2], me[:, 3], me[:, 4], me[:, 5]
    return np.nonzero((11 * sad == 10 * sad0) & ((var < 64) | (varor > var)) & (sad0 >= 768))[0]


@pytest.mark.parametrize("name", ["qcif_tie_full31", "qcif_tie_tss"])
def test_mtype_tie_fixture_covers_both_outcomes(name):
    """The constructed fixture reaches the tie with both results of the double
    comparison: MTYPE 2 (y > x/1.1 true) and MC (false), as the reference chose."""
    z = load(f"seq_{name}.npz")
    mbs = tie_mbs(z, 1)
    assert len(mbs) >= 4
    got = set()
    for k in mbs:
        omv = int(z["merec"][1][k, 3])
        inter = (omv * 10 // 11) / 256 > (omv / 256) / 1.1
        assert int(z["mb"][1][k, 0]) in ((2,) if inter else (5, 8))
        got.add(inter)
    assert got == {True, False}


def test_fixture_coverage():
    """The fixture set exercises every MTYPE the encoder can choose, both searches,
    q extremes and the CBP fallbacks (SURVEY.md 8(c) fixture policy)."""
    seen = set()
    mes, qs = set(), set()
    for name in SEQS:
        z = load(f"seq_{name}.npz")
        seen |= set(np.unique(z["mb"][..., 0]).tolist())
        mes.add(str(z["me"]))
        qs.add(int(z["q"]))
    assert {0, 2, 4, 5, 7, 8} <= seen
    assert mes == {"tss", "full"}
    assert {1, 2, 31} <= qs
