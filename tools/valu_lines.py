"""Static VALU instruction count per source line of one kernel (development aid).
usage: python3 tools/valu_lines.py KERNEL_SUBSTRING [N]  (compiles with -g)"""
import collections
import os
import re
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src_path = os.path.join(R, "p64_amd", "csrc", "k_search.hip")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-g", "-S",
                "--cuda-device-only", "-o", "/tmp/valu_lines.s", src_path], check=True,
               stderr=subprocess.DEVNULL)
text = open("/tmp/valu_lines.s").read().split("\n")
files = {}
body, on = [], False
for l in text:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
    if m:
        files[int(m.group(1))] = m.group(3)
    if re.match(r"^_Z\w*" + ".*:", l) and sys.argv[1] in l.split(":")[0]:
        on = True
    elif on and l.startswith(".Lfunc_end"):
        on = False
    if on:
        body.append(l)
src = open(src_path).read().split("\n")
cnt, cur = collections.Counter(), None
for l in body:
    m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = (int(m.group(1)), int(m.group(2)))
    elif l.strip().startswith("v_"):
        cnt[cur] += 1
print("total VALU", sum(cnt.values()))
for (f, ln), c in cnt.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 40):
    name = files.get(f, "?")
    s = src[ln - 1].strip()[:80] if name.endswith("k_search.hip") and ln else name
    print(f"{c:5d} {ln:5d} {s}")
