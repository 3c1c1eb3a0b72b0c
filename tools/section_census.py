"""Instruction census per SECTION() phase of one kernel (development aid).

Compiles a copy of k_search.hip whose SECTION() labels (no code in the
product) become ";## name" asm markers to an ISA listing and counts VALU /
SALU / LDS instructions between the markers.  Static counts: loop
bodies count once, both sides of a branch count.
usage: python tools/section_census.py [kernel-substring] [extra hipcc flags...]
"""
import collections
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
kern = sys.argv[1] if len(sys.argv) > 1 else "k_motionILi2"
out = "/tmp/p64_sections.s"
src = open(os.path.join(REPO, "p64_amd/csrc/k_search.hip")).read().replace(
    '#include "launch.h"\n', '#include "launch.h"\n#undef SECTION\n#define SECTION(name) asm volatile(";## " name)\n', 1)
tmp = os.path.join(REPO, "p64_amd/csrc/_census_tmp.hip")
open(tmp, "w").write(src)
try:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    *sys.argv[2:], "-S", "--cuda-device-only", "-o", out, tmp], check=True)
finally:
    os.remove(tmp)
s = open(out).read()
start = next(i for i in range(len(s)) if s.startswith("_Z", i) and kern in s[i:s.find(":", i)]
             and s[s.find(":", i) + 1:s.find(":", i) + 4].strip().startswith(";"))
end = s.find(".Lfunc_end", start)
sec, cnt = "prologue", collections.OrderedDict()
for line in s[start:end].splitlines():
    if ";##" in line:
        sec = line.split(";##")[1].strip()
        continue
    t = line.strip()
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    op = t.split()[0]
    c = cnt.setdefault(sec, collections.Counter())
    kind = ("sad" if op.startswith("v_sad") else "valu" if op.startswith("v_") else
            "salu" if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch"))
            else "nop" if op == "s_nop" else "lds" if op.startswith("ds_") else "other")
    c[kind] += 1
for k, v in cnt.items():
    print(f"{k:12s} " + "  ".join(f"{x} {v[x]:4d}" for x in ("valu", "sad", "salu", "lds", "nop", "other")))
