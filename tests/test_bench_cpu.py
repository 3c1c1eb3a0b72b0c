"""bench.py's CPU-baseline legs (host only, no GPU): the reference encoder,
its -o intra run and its decoder, each timed as one process and as the box's
CPU share; 4CIF, which the reference cannot encode, falls back to the
clean-room port with the reason stated.  Tiny samples (a few pictures)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

HOOK = os.path.join(REPO, "oracle", "_ref", "p64hook")


@pytest.mark.skipif(not os.access(HOOK, os.X_OK), reason="oracle/_ref not built (make ref)")
def test_cpu_baseline_legs_reference():
    a = bench.parse(["--cpu-frames", "3", "--cpu-procs", "2"])
    out = bench.cpu_baselines(a, ["inter", "intra", "decode"])
    assert set(out) == {"inter", "intra", "decode"}
    for leg, r in out.items():
        assert r["kind"] == "reference", leg
        assert r["value"] > 0 and r["single_process"]["value"] > 0, leg
        assert r["cores"] >= 1 and r["unit"] == "macroblocks/s"
    assert "intra_only.prog" in out["intra"]["sample"]
    assert "p64 -d" in out["decode"]["sample"]


def test_cpu_baseline_4cif_is_the_port():
    a = bench.parse(["--config", "4cif", "--cpu-frames", "1"])
    out = bench.cpu_baselines(a, ["inter"])
    r = out["inter"]
    assert r["kind"] == "port" and r["cores"] == 1
    assert "cannot encode 4CIF" in r["sample"]


def test_level_byte_accounting():
    """coded_level_bytes: 128 bytes per transmitted block (MTYPE with
    coefficients; CBP bit for the MTYPEs that carry one, all six otherwise);
    decode_bytes adds records, prediction source and recon on top."""
    import torch
    # (mtype, cbp): intra 0 (six blocks), inter 2 with cbp 0b100001 (two),
    # MC-only 4 (none), MC+coef 5 with cbp 0x3f (six), MQUANT intra 1 (six)
    mb = torch.tensor([[0, 0x3f, 0, 0], [2, 0x21, 0, 0], [4, 0x3f, 1, 1], [5, 0x3f, 2, 0],
                       [1, 0, 0, 0]], dtype=torch.int8)
    assert bench.coded_level_bytes(torch, mb) == 128 * (6 + 2 + 0 + 6 + 6)
    n = mb.shape[0]
    inter = 3  # mtypes >= 2
    assert bench.decode_bytes(torch, mb, n) == 6 * n + 128 * 20 + 384 * inter + 384 * n
