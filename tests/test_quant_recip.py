"""The fused kernels divide by 2q with a binary32 reciprocal (common.h
c_qrecip: 1/(2q) rounded to float, then raised one ulp, so that exact
multiples never fall short).  Check it exhaustively against C truncating
division for every step the encoder can use (q = 1..31) and every value the
kernel can see (|c| <= 2048: BoundDctMatrix clips to 2047 / -1023 and even q
adds +-1), with margin."""
import numpy as np


def recip(q):
    r = np.float32(1.0) / np.float32(2 * q)
    return (r.view(np.uint32) + np.uint32(1)).view(np.float32)


def c_div(a, d):
    return np.sign(a) * (np.abs(a) // d)  # C: truncation toward zero


def test_reciprocal_is_exact_over_kernel_range():
    c = np.arange(-4096, 4097, dtype=np.int32)
    for q in range(1, 32):
        got = (c.astype(np.float32) * recip(q)).astype(np.int32)  # v_mul_f32, v_cvt_i32_f32
        np.testing.assert_array_equal(got, c_div(c, 2 * q), err_msg=f"q={q}")

