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
from test_oracle_golden import SEQS, load, sequence_frames

pytestmark = pytest.mark.gpu

CLI = os.path.join(REPO, "p64_amd", "p64gpu")
PLAIN = [s for s in SEQS if not str(load(f"seq_{s}.npz")["oracle"])]  # no -o program


def write_y4m(path, frames, w, h):
    with open(path, "wb") as f:
        f.write(b"YUV4MPEG2 W%d H%d F30000:1001 Ip A0:0 C420jpeg\n" % (w, h))
        for fr in frames:
            f.write(b"FRAME\n" + fr.tobytes())


@pytest.mark.parametrize("name", PLAIN)
def test_cli_encode_byte_identical(p64, torch_dev, tmp_path, name):
    """`p64gpu -FMT -y4m -a 0 -b N-1 -q Q -i SL [-full]` == the reference CLI's .p64."""
    z = load(f"seq_{name}.npz")
    w, h, n = int(z["width"]), int(z["height"]), int(z["nframes"])
    write_y4m(tmp_path / "in.y4m", sequence_frames(p64, z), w, h)
    cmd = [CLI, "-" + str(z["fmt"]), "-y4m", "-a", "0", "-b", str(n - 1), "-q", str(int(z["q"])),
           "-i", str(int(z["sl"])), str(tmp_path / "in"), "-z", ".y4m", "-s", str(tmp_path / "o.p64")]
    if str(z["me"]) == "full":
        cmd.append("-full")
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, timeout=300)
    data = (tmp_path / "o.p64").read_bytes()
    assert len(data) == int(z["stream_len"])
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])


@pytest.mark.parametrize("name", ["qcif_tss", "cif_full31", "ntsc_tss"])
def test_python_encode_sequence_byte_identical(p64, torch_dev, name):
    from p64_amd import stream
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    data = stream.encode_sequence(sequence_frames(p64, z), w, h, quant=int(z["q"]),
                                  me_mode=1 if str(z["me"]) == "full" else 0,
                                  search_limit=int(z["sl"]))
    assert hashlib.sha256(data).hexdigest() == str(z["stream_sha256"])


def test_cli_decode_short_p64_md5(p64, torch_dev, tmp_path):
    """`p64gpu -d -s short.p64 short` writes the reference's 7 x 3 component files."""
    exp = json.load(open(os.path.join(GOLDEN, "decode.json")))
    subprocess.run([CLI, "-d", "-s", os.path.join(GOLDEN, "short.p64"), str(tmp_path / "short")],
                   check=True, stdout=subprocess.DEVNULL, timeout=120)
    for name, md5 in exp.items():
        assert hashlib.md5((tmp_path / name).read_bytes()).hexdigest() == md5, name


def test_python_decode_short_p64_md5(p64, torch_dev):
    from p64_amd import stream
    exp = json.load(open(os.path.join(GOLDEN, "decode.json")))
    frames = stream.decode_sequence(open(os.path.join(GOLDEN, "short.p64"), "rb").read())
    assert len(frames) == 7
    w, h = 352, 240
    for i, f in enumerate(frames):
        for c, a in zip("YUV", (f[:w * h], f[w * h:w * h * 5 // 4], f[w * h * 5 // 4:])):
            assert hashlib.md5(a.tobytes()).hexdigest() == exp[f"short{i}.{c}"]


@pytest.mark.parametrize("name", ["qcif_tss", "qcif_full31", "qcif_q31", "qcif_flat_tss"])
def test_decode_of_encoded_stream_is_encoder_recon(p64, torch_dev, tmp_path, name):
    """encode -> .p64 -> decode (y4m) reproduces the encoder's closed-loop
    reconstruction, which the fixtures hold from the reference encoder."""
    z = load(f"seq_{name}.npz")
    w, h, n = int(z["width"]), int(z["height"]), int(z["nframes"])
    write_y4m(tmp_path / "in.y4m", sequence_frames(p64, z), w, h)
    enc = [CLI, "-QCIF", "-y4m", "-a", "0", "-b", str(n - 1), "-q", str(int(z["q"])), "-i",
           str(int(z["sl"])), str(tmp_path / "in"), "-z", ".y4m", "-s", str(tmp_path / "o.p64")]
    if str(z["me"]) == "full":
        enc.append("-full")
    subprocess.run(enc, check=True, stdout=subprocess.DEVNULL, timeout=300)
    subprocess.run([CLI, "-d", "-y4m", "-s", str(tmp_path / "o.p64"), str(tmp_path / "dec")],
                   check=True, stdout=subprocess.DEVNULL, timeout=300)
    raw = (tmp_path / "dec.y4m").read_bytes()
    hdr, body = raw.split(b"\n", 1)
    assert hdr.startswith(b"YUV4MPEG2 W176 H144")
    pic = w * h * 3 // 2
    chunks = body.split(b"FRAME\n")[1:]
    assert len(chunks) == n
    for t, c in enumerate(chunks):
        assert len(c) == pic
        np.testing.assert_array_equal(np.frombuffer(c, np.uint8), z["recon"][t], err_msg=f"t{t}")
