"""Timing-only variants of k_block.hip (development aid, never shipped):
writes abtest/k_block_<name>.hip with one phase of k_inter_mbg switched off,
for cost-by-subtraction runs (tools/ablib.sh <name> abtest/k_block_<name>.hip
k_block, then tools/inter_prof.sh).  Variants that drop work give WRONG
outputs; they are timing probes only.
  noidct   the coded blocks' IQ/IDCT pass (idct_coded_blocks) off
  nolvl    the level stores off
  norec    the reconstructed rows' stores off
usage: python tools/blk_variants.py [name ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(REPO, "p64_amd/csrc/k_block.hip")).read()
IDCT = "  idct_coded_blocks(ck, np, q, intra, prow, (uint32_t *)lds, lane);\n"
LVL = "  mbg_store_levels(a, lds, lane, nmbs, gmb0, nvalid, nz);\n"
REC = "  mbg_store_rows(a, kd, nmbs, ro, pw, prow, rl, gmb, mbw,\n"
for s_ in (IDCT, LVL, REC):
    assert src.count(s_) == 1, s_
variants = {
    "noidct": [(IDCT, "")],
    "nolvl": [(LVL, "")],
    "norec": [(REC, "  if (lane > 64) mbg_store_rows(a, kd, nmbs, ro, pw, prow, rl, gmb, mbw,\n")],
}
os.makedirs(os.path.join(REPO, "abtest"), exist_ok=True)
for name in sys.argv[1:] or variants:
    s = src
    for a, b in variants[name]:
        s = s.replace(a, b)
    p = os.path.join(REPO, "abtest", f"k_block_{name}.hip")
    open(p, "w").write(s)
    print(p)
