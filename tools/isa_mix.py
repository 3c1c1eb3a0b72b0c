"""Static instruction mix of one kernel in a gfx950 ISA listing (development aid).

    hipcc ... -S --cuda-device-only -o /tmp/k.s p64_amd/csrc/k_search.hip
    python tools/isa_mix.py /tmp/k.s k_intra_mbg [--top 40]

Counts every instruction between the kernel's symbol label and its
.Lfunc_end, grouped by opcode, and prices the VALU ones with the issue costs
measured by tools/ubench_valu.hip (clocks per wave64 instruction on one SIMD:
2 for plain VOP2/VOP1 ALU ops, 4 for VOP3-only/VOP3P/dot/mul24/med3/cvt).
The estimate ignores loops (the block kernels are fully unrolled).
"""
import re
import sys
from collections import Counter

TWO_CLK = re.compile(r"^v_(add|sub|subrev|lshlrev|lshrrev|ashrrev|and|or|xor|not|mov|fmac|mul|max|min)"
                     r"_(u32|i32|b32|f32|co_u32|nc_u32)(_e32)?$")


def cost(op):
    if not op.startswith("v_"):
        return 0
    if op.endswith("_e64") or op.startswith(("v_pk_", "v_dot", "v_mad", "v_med3", "v_cvt", "v_perm",
                                             "v_bfi", "v_bfe", "v_lshl_or", "v_add3", "v_lshl_add",
                                             "v_and_or", "v_or3", "v_mul_i32_i24", "v_mul_u32_u24",
                                             "v_mul_lo", "v_mul_hi", "v_cndmask", "v_alignbit",
                                             "v_fma_", "v_sad", "v_readlane", "v_writelane",
                                             "v_readfirstlane", "v_cmp", "v_cmpx")):
        return 4
    if TWO_CLK.match(op) or op.startswith("v_mov"):
        return 2
    return 4


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        head = ln.split(";")[0].strip()
        if head.endswith(":") and name in head and not ln.startswith((".", "\t")):
            start = i
            break
    if start is None:
        sys.exit(f"no kernel label containing {name!r}")
    label = lines[start].split(";")[0].strip()[:-1]
    ops = Counter()
    for ln in lines[start + 1:]:
        if ln.startswith(".Lfunc_end"):
            break
        s = ln.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        ops[s.split()[0]] += 1
    valu = {o: c for o, c in ops.items() if o.startswith("v_")}
    clk = sum(cost(o) * c for o, c in valu.items())
    print(f"{label}: {sum(ops.values())} instructions, {sum(valu.values())} VALU, ~{clk} VALU clk")
    for o, c in sorted(ops.items(), key=lambda x: -x[1] * max(cost(x[0]), 1))[:top]:
        print(f"  {o:32s} {c:5d}  x{cost(o)}  = {c * cost(o)}")


if __name__ == "__main__":
    main()
