"""k_intra_mbg quantises its AC coefficients without the clamp to +-(8*1023+3)
when UseQuant >= 5 (k_block.hip intra_block).  That clamp (BoundDctMatrix,
transform.c:460, folded into quant_int.h) can only act on a row-pass output
|v| > 8,187; for q >= 5 it is the only clamp (256q - 1 - [q even] > 1023), so
it may be dropped iff no 8-bit picture block reaches |v| > 8,187 at an AC
position.  Proof by affine arithmetic over the kernel's Chen butterfly
(fdct_block_pk: column pass with the <<2 folded into the constants, row pass
with >>1, every >>9 floor; chendct.c:97-206): each value is a linear form in
the 64 pixels plus an interval for the floors' rounding, and the extreme of a
linear form over [0, 255]^64 is exact.  CPU only."""
import numpy as np

C1D4, C1D8, C3D8, C1D16, C3D16, C5D16, C7D16 = 362, 473, 196, 502, 426, 284, 100


class Aff:
    def __init__(self, a, lo=0.0, hi=0.0):
        self.a, self.lo, self.hi = np.asarray(a, np.float64), lo, hi

    def __add__(self, o):
        return Aff(self.a + o.a, self.lo + o.lo, self.hi + o.hi)

    def __sub__(self, o):
        return Aff(self.a - o.a, self.lo - o.hi, self.hi - o.lo)

    def mul(self, c):
        return Aff(self.a * c, min(self.lo * c, self.hi * c), max(self.lo * c, self.hi * c))

    def floordiv(self, d):  # floor(x / d): x/d - f, f in [0, (d-1)/d]
        return Aff(self.a / d, self.lo / d - (d - 1) / d, self.hi / d)

    def range(self, pmax=255.0):
        pos = np.clip(self.a, 0, None).sum() * pmax
        neg = np.clip(self.a, None, 0).sum() * pmax
        return neg + self.lo, pos + self.hi


def ms9(x):
    return x.floordiv(512)


def dot(x, cx, y, cy):
    return x.mul(cx) + y.mul(cy)


def col_pass(x):  # fwd_col_pk on one column x[0..7] (the <<2 in the constants)
    s = [x[0] + x[7], x[1] + x[6], x[2] + x[5], x[3] + x[4]]
    d = [x[0] - x[7], x[1] - x[6], x[2] - x[5], x[3] - x[4]]
    e0, e1, e3, e2 = s[0] + s[3], s[1] + s[2], s[0] - s[3], s[1] - s[2]
    o = [None] * 8
    o[0] = ms9(dot(e0, 4 * C1D4, e1, 4 * C1D4))
    o[4] = ms9(dot(e0, 4 * C1D4, e1, -4 * C1D4))
    o[2] = ms9(dot(e3, 4 * C1D8, e2, 4 * C3D8))
    o[6] = ms9(dot(e3, 4 * C3D8, e2, -4 * C1D8))
    r1 = ms9(dot(d[1], 4 * C1D4, d[2], 4 * C1D4))
    r0 = ms9(dot(d[1], 4 * C1D4, d[2], -4 * C1D4))
    u0, u3 = d[3].mul(4) + r0, d[0].mul(4) + r1
    u1, u2 = d[3].mul(4) - r0, d[0].mul(4) - r1
    o[1] = ms9(dot(u0, C7D16, u3, C1D16))
    o[7] = ms9(dot(u0, -C1D16, u3, C7D16))
    o[3] = ms9(dot(u1, -C5D16, u2, C3D16))
    o[5] = ms9(dot(u1, C3D16, u2, C5D16))
    return o, s + d + [e0, e1, e2, e3, r0, r1, u0, u1, u2, u3]


def row_pass(p):  # fwd_row_pk on one row p[0..7] (sums and differences >>1)
    s = [(p[k] + p[7 - k]).floordiv(2) for k in range(4)]
    d = [(p[k] - p[7 - k]).floordiv(2) for k in range(4)]
    e0, e1, e3, e2 = s[0] + s[3], s[1] + s[2], s[0] - s[3], s[1] - s[2]
    o = [None] * 8
    o[0] = ms9(dot(e0, C1D4, e1, C1D4))
    o[4] = ms9(dot(e0, C1D4, e1, -C1D4))
    o[2] = ms9(dot(e3, C1D8, e2, C3D8))
    o[6] = ms9(dot(e3, C3D8, e2, -C1D8))
    r1 = ms9(dot(d[1], C1D4, d[2], C1D4))
    r0 = ms9(dot(d[1], C1D4, d[2], -C1D4))
    u0, u3 = d[3] + r0, d[0] + r1
    u1, u2 = d[3] - r0, d[0] - r1
    o[1] = ms9(dot(u0, C7D16, u3, C1D16))
    o[7] = ms9(dot(u0, -C1D16, u3, C7D16))
    o[3] = ms9(dot(u1, -C5D16, u2, C3D16))
    o[5] = ms9(dot(u1, C3D16, u2, C5D16))
    return o, s + d + [e0, e1, e2, e3, r0, r1, u0, u1, u2, u3]


def test_intra_ac_never_reaches_the_dct_bound():
    px = [[Aff(np.eye(64)[8 * r + c]) for c in range(8)] for r in range(8)]
    cols, inter = [], []
    for c in range(8):
        o, mid = col_pass([px[r][c] for r in range(8)])
        cols.append(o)
        inter += mid + o
    worst_ac, worst_16 = 0.0, 0.0
    for r in range(8):
        o, mid = row_pass([cols[c][r] for c in range(8)])
        inter += mid
        for k in range(8):
            lo, hi = o[k].range()
            if (r, k) != (0, 0):
                worst_ac = max(worst_ac, -lo, hi)
    for v in inter:  # the packed 16-bit arithmetic's intermediates
        lo, hi = v.range()
        worst_16 = max(worst_16, -lo, hi)
    assert worst_ac <= 8 * 1023 + 3, worst_ac
    assert worst_16 < 2 ** 15, worst_16
    # for the record: the margin (the clamp's bound is 8,187)
    print(f"intra AC |v| <= {worst_ac:.1f}; packed intermediates <= {worst_16:.1f}")


def test_clamp_is_inactive_from_q5():
    # 256q - 1 - [q even] >= 1023 from q = 5 on: the level bound (127) lies
    # beyond BoundDct's, so the only clamp is BoundDct's +-(8*1023+3)
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "p64_amd", "csrc"))
    for q in range(1, 32):
        qbr = 256 * q - 1 - (0 if q & 1 else 1)
        assert (qbr >= 1023) == (q >= 5)


def test_intra_idct_column_pass_fits_int16():
    """k_intra_mbg's IDCT column pass runs two columns at a time on packed
    int16 pairs (k_block.hip idct_col_pair_pk): with the dequantised intra
    inputs bounded by the quantiser (|AC| <= 1,023 + q <= 1,054, the DC x 8 in
    8..2,032, iq_idct_intra_rec) every value the pass packs -- the products'
    ms9 results P/Q, the sums E/F, the g inputs F2 -+ F1, g itself and the
    outputs -- must stay inside int16.  Interval arithmetic per input (each
    input independent: a superset of what a block can produce)."""
    ac, dc = 1054, 2032

    class I:
        def __init__(self, lo, hi):
            self.lo, self.hi = lo, hi

        def __add__(self, o):
            return I(self.lo + o.lo, self.hi + o.hi)

        def __sub__(self, o):
            return I(self.lo - o.hi, self.hi - o.lo)

        def mul(self, c):
            return I(min(self.lo * c, self.hi * c), max(self.lo * c, self.hi * c))

        def ms9(self):
            return I(self.lo // 512, self.hi // 512)

        def mag(self):
            return max(-self.lo, self.hi)

    for col0 in (True, False):  # column 0 carries the DC in row 0
        x = [I(-ac, ac) for _ in range(8)]
        if col0:
            x[0] = I(8, dc)
        d = lambda a, ca, b, cb: (a.mul(ca) + b.mul(cb)).ms9()  # noqa: E731
        P0 = d(x[1], 4 * C7D16, x[7], -4 * C1D16)
        P3 = d(x[1], 4 * C1D16, x[7], 4 * C7D16)
        P1 = d(x[5], 4 * C3D16, x[3], -4 * C5D16)
        P2 = d(x[5], 4 * C5D16, x[3], 4 * C3D16)
        Q0 = d(x[0], 4 * C1D4, x[4], 4 * C1D4)
        Q1 = d(x[0], 4 * C1D4, x[4], -4 * C1D4)
        Q2 = d(x[2], 4 * C3D8, x[6], -4 * C1D8)
        Q3 = d(x[2], 4 * C1D8, x[6], 4 * C3D8)
        E = [Q0 + Q3, Q1 + Q2, Q1 - Q2, Q0 - Q3]
        F = [P0 + P1, P0 - P1, P3 - P2, P3 + P2]
        Dm, Dp = F[2] - F[1], F[2] + F[1]
        G1, G2 = Dm.mul(C1D4).ms9(), Dp.mul(C1D4).ms9()
        O = [E[0] + F[3], E[1] + G2, E[2] + G1, E[3] + F[0], E[3] - F[0], E[2] - G1, E[1] - G2, E[0] - F[3]]
        vals = [P0, P1, P2, P3, Q0, Q1, Q2, Q3] + E + F + [Dm, Dp, G1, G2] + O
        worst = max(v.mag() for v in vals)
        assert worst < 2 ** 15, (col0, worst)


def test_inter_residual_sum_bound_keeps_the_clamp_inactive():
    """k_inter_mbg drops the quantiser's BoundDct clamp for a wave whose
    blocks all have sum|residual| <= 4,253 (q >= 5): |v| = |sum a_i r_i + err|
    <= max|a_i| sum|r| + max|err| over every AC output of the kernel's
    butterfly must stay <= 8 x 1023 + 3, and the DC within its own bound
    (>= 10,235 from q = 5 on)."""
    px = [[Aff(np.eye(64)[8 * r + c]) for c in range(8)] for r in range(8)]
    cols = [col_pass([px[r][c] for r in range(8)])[0] for c in range(8)]
    worst_ac = worst_dc = 0.0
    for r in range(8):
        o, _ = row_pass([cols[c][r] for c in range(8)])
        for k in range(8):
            a = o[k]
            v = np.abs(a.a).max() * 4253 + max(-a.lo, a.hi)
            if (r, k) == (0, 0):
                worst_dc = max(worst_dc, v)
            else:
                worst_ac = max(worst_ac, v)
    assert worst_ac <= 8 * 1023 + 3, worst_ac
    assert worst_dc <= 8 * (256 * 5 - 1) + 3, worst_dc


def test_inter_idct_column_pass_fits_int16():
    """k_inter_mbg runs its coded blocks' IQ/IDCT one block per lane with the
    intra path's packed column pass (k_block.hip iq_idct_inter_rec) when every
    dequantised value is within +-1,291 (the wave-uniform check sum l^2 <=
    c_idct_lim.l2[q], (2|l| + 1) q <= 1,291): with every input of the pass in
    that box -- an inter DC is dequantised like an AC and may be negative --
    each packed value stays inside int16, and 1,292 does not."""
    def worst(L):
        class I:
            def __init__(self, lo, hi):
                self.lo, self.hi = lo, hi

            def __add__(self, o):
                return I(self.lo + o.lo, self.hi + o.hi)

            def __sub__(self, o):
                return I(self.lo - o.hi, self.hi - o.lo)

            def mul(self, c):
                return I(min(self.lo * c, self.hi * c), max(self.lo * c, self.hi * c))

            def ms9(self):
                return I(self.lo // 512, self.hi // 512)

            def mag(self):
                return max(-self.lo, self.hi)

        x = [I(-L, L) for _ in range(8)]
        d = lambda a, ca, b, cb: (a.mul(ca) + b.mul(cb)).ms9()  # noqa: E731
        P0, P3 = d(x[1], 4 * C7D16, x[7], -4 * C1D16), d(x[1], 4 * C1D16, x[7], 4 * C7D16)
        P1, P2 = d(x[5], 4 * C3D16, x[3], -4 * C5D16), d(x[5], 4 * C5D16, x[3], 4 * C3D16)
        Q0, Q1 = d(x[0], 4 * C1D4, x[4], 4 * C1D4), d(x[0], 4 * C1D4, x[4], -4 * C1D4)
        Q2, Q3 = d(x[2], 4 * C3D8, x[6], -4 * C1D8), d(x[2], 4 * C1D8, x[6], 4 * C3D8)
        E = [Q0 + Q3, Q1 + Q2, Q1 - Q2, Q0 - Q3]
        F = [P0 + P1, P0 - P1, P3 - P2, P3 + P2]
        Dm, Dp = F[2] - F[1], F[2] + F[1]
        G1, G2 = Dm.mul(C1D4).ms9(), Dp.mul(C1D4).ms9()
        O = [E[0] + F[3], E[1] + G2, E[2] + G1, E[3] + F[0], E[3] - F[0], E[2] - G1, E[1] - G2, E[0] - F[3]]
        return max(v.mag() for v in [P0, P1, P2, P3, Q0, Q1, Q2, Q3] + E + F + [Dm, Dp, G1, G2] + O)

    assert worst(1291) < 2 ** 15
    assert worst(1292) >= 2 ** 15
    # the kernel's per-q limit: the largest |l| with (2|l| + 1) q <= 1,291
    for q in range(1, 32):
        lmax = max(l for l in range(0, 700) if (2 * l + 1) * q <= 1291)
        # every dequantised value (2|l| + 1) q - [q even] of |l| <= lmax is inside the box
        assert (2 * lmax + 1) * q <= 1291 < (2 * lmax + 3) * q
