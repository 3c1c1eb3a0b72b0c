"""End-to-end CLI throughput (GPU box): p64gpu vs the reference CLI on the same
y4m (CIF, 150 pictures, FULL search SL=31 and TSS), same flags, same bytes out."""
import hashlib
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import p64_amd  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 150
w, h = 352, 288
with tempfile.TemporaryDirectory() as td:
    with open(os.path.join(td, "in.y4m"), "wb") as f:
        f.write(b"YUV4MPEG2 W352 H288 F30000:1001 Ip A0:0 C420jpeg\n")
        for t in range(N):
            f.write(b"FRAME\n" + p64_amd.synth_frame(3, t, w, h).tobytes())
    base = ["-CIF", "-y4m", "-a", "0", "-b", str(N - 1), "-q", "8", "-i", "31",
            os.path.join(td, "in"), "-z", ".y4m"]
    runs = [("p64gpu FULL (GPU VLC)", [os.path.join(REPO, "p64_amd", "p64gpu"), "-full"], {}),
            ("p64gpu FULL (host VLC)", [os.path.join(REPO, "p64_amd", "p64gpu"), "-full", "-hostvlc"], {}),
            ("reference FULL (p64hook)", [os.path.join(REPO, "oracle", "_ref", "p64hook")], {"P64REF_ME": "full"}),
            ("p64gpu TSS (GPU VLC)", [os.path.join(REPO, "p64_amd", "p64gpu")], {}),
            ("reference TSS (p64)", [os.path.join(REPO, "oracle", "_ref", "p64")], {})]
    for name, cmd, env in runs:
        if not os.access(cmd[0], os.X_OK):
            print(f"{name}: binary missing")
            continue
        out = os.path.join(td, "o.p64")
        t0 = time.perf_counter()
        subprocess.run(cmd + base + ["-s", out], env=dict(os.environ, **env), check=True,
                       stdout=subprocess.DEVNULL)
        dt = time.perf_counter() - t0
        d = open(out, "rb").read()
        print(f"{name:28s} {dt:7.3f} s  {N / dt:8.1f} pictures/s  {N * 396 / dt / 1e6:7.3f} M MB/s  "
              f"{len(d)} B  sha {hashlib.sha256(d).hexdigest()[:12]}")
