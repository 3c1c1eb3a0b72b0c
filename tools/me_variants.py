"""Timing-only variants of k_search.hip (development aid, never shipped):
writes abtest/k_search_<name>.hip with phases of the FULL search switched off,
for cost-by-subtraction runs (tools/ablib.sh builds each into a library,
tools/me_prof.sh times k_motion<2> under rocprofv3 per content).  Variants
that drop work give WRONG vectors; they are timing probes only.
  nofin        no finishing of the survivors and no dense pass
  nofin_nomap  + no bound map (the bound pass reads whatever the LDS holds)
  nofin_nolb   + no map, no bound pass, no c*, no survivor list
  fixed        the lower-bound path off entirely: window fetch, current-block
               map, SAD(0,0), statistics only
usage: python tools/me_variants.py [name ...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(REPO, "p64_amd/csrc/k_search.hip")).read()
FIN = "  if (nsurv <= ME_LIST_MAX) {"
DENSE = "  } else {  // little pruned: every candidate densely, the current rows in SGPRs"
MAP = "    if (ND < 15)\n      build_lb_map<8, 6>(S, lane);\n    else\n      build_lb_map(S, lane);\n"
LBP_START = '    SECTION("lb_pass");'
LBP_END = '    SECTION("survivors");'
LBPATH = "  bool lb_path = range >= ME_LOW_CONTRAST;"
for s_ in (FIN, DENSE, MAP, LBP_START, LBP_END, LBPATH):
    assert s_ in src, s_

NOFIN = [(FIN, "  if (lane < 0) {"), (DENSE, "  } else if (lane < 0) {")]


def cut(text, start, end):
    a = text.index(start)
    b = text.index(end, a)
    return text[:a] + "    // (cut)\n    Ts = 0; pk = 0xFFFFFFFFu; nsurv = 0;\n" + text[b:]


variants = {
    "nofin": (NOFIN, None),
    "nofin_nomap": (NOFIN + [(MAP, "")], None),
    "nofin_nolb": (NOFIN + [(MAP, "")], (LBP_START, LBP_END)),
    "fixed": (NOFIN + [(LBPATH, "  bool lb_path = false;")], None),
}
os.makedirs(os.path.join(REPO, "abtest"), exist_ok=True)
for name in sys.argv[1:] or variants:
    reps, c = variants[name]
    s = src
    for a, b in reps:
        s = s.replace(a, b)
    if c:
        s = cut(s, *c)
    p = os.path.join(REPO, "abtest", f"k_search_{name}.hip")
    open(p, "w").write(s)
    print(p)
