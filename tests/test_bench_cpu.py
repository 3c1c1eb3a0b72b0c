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
