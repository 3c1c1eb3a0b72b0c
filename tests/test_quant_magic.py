"""The fused kernels divide by 2q with a 20-bit reciprocal (p64gpu.hip
div_trunc<true>).  Check it exhaustively against C truncating division over
every step the encoder can use (q = 1..31) and every magnitude the kernel can
see (|c| <= 2048: BoundDctMatrix clips to 2047 / -1023 and even q adds +-1)."""
import numpy as np


def magic(q):
    return (1 << 20) // (2 * q) + 1


def test_reciprocal_is_exact_over_kernel_range():
    a = np.arange(0, 2049, dtype=np.int64)
    for q in range(1, 32):
        d = 2 * q
        m = magic(q)
        assert m < (1 << 24) and a.max() < (1 << 24)  # v_mul_u32_u24 operands
        assert (a * m).max() < (1 << 32)              # low 32 bits hold the product
        got = (a * m) >> 20
        np.testing.assert_array_equal(got, a // d, err_msg=f"q={q}")


def test_reciprocal_margin():
    """Document how far past the kernel's range the reciprocal stays exact."""
    for q in range(1, 32):
        d, m = 2 * q, magic(q)
        a = np.arange(0, 1 << 15, dtype=np.int64)
        bad = np.nonzero(((a * m) >> 20) != a // d)[0]
        first_bad = int(bad[0]) if bad.size else None
        assert first_bad is None or first_bad > 4096, (q, first_bad)
