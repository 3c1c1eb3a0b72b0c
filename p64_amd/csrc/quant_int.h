/*
 * quant_int.h -- the H.261 forward quantiser of the block-layout kernels as
 * one integer multiply-add and one shift per coefficient (plain C; included
 * by k_block.hip, where the table is built at compile time, and by the CPU
 * test tests/test_quant_int.py, which checks it exhaustively).
 *
 * From the raw Chen row-pass output v (before the final /8) to the level:
 *   c = final /8 (chendct.c:204: (v +- 4) / 8, C truncation),
 *   c = BoundDctMatrix(c) (transform.c:460), l = CCITT(Flat)Quantize AC
 *   (transform.c:283-306 / 339-347: (c + [q even] sign c) / 2q, truncation),
 *   l = (Flat)BoundQuantizeMatrix(l) (transform.c:502-537, +-127).
 * Algebra: with e = [q even], K = 4 + 8e, D = 16q the chain is
 *   l = sign(v) floor((|v| + K) / D)  (the nested floors of /8 and /2q merge;
 *   |v| < 4 gives 0 either way), saturating where c reaches its bound; so
 *   clamping v to +-(8 cb + 3) (cb = the c bound) reproduces every clamp.
 * For v >= 0 that is floor((v + K) / D), for v < 0 ceil((v - K) / D) =
 * floor((v - K + D - 1) / D); an offset B D makes the dividend x >= 0, and
 * floor(x / D) = (x M) >> s with M = ceil(2^s / D) is exact for
 * 0 <= x <= X when X (M D - 2^s) < 2^s.  The offset's -B folds into the
 * addend: level = (vc M + C) >> s (arithmetic), C = cp or cn by sign.
 */
#ifndef P64_QUANT_INT_H
#define P64_QUANT_INT_H

#include <stdint.h>

#ifdef __cplusplus
#define QI_FN constexpr
#else
#define QI_FN static inline
#endif

typedef struct {
  int32_t vlo, vhi; /* clamp of v */
  int32_t m, s;     /* multiplier and shift */
  int32_t cp, cn;   /* addend for v >= 0 / v < 0 (offset folded in) */
} p64_qint;

/* dc_inter: the inter DC (BoundDct: <= 2047 only; level +-127) instead of AC.
 * Its lower clamp is at -min(qbr, 2047) rather than -qbr: the same levels on
 * everything a DCT of 8-bit residuals can produce (|c| <= 2040, |v| <= 16323),
 * and it keeps the dividend range within one 32-bit multiply. */
QI_FN p64_qint p64_qint_make(int q, int dc_inter) {
  const int e = (q & 1) ? 0 : 1, K = 4 + 8 * e, D = 16 * q;
  const int qbr = 256 * q - 1 - e; /* l(qbr) = 127, l(qbr + 1) = 128 */
  const int cb = dc_inter ? 2047 : 1023;
  const int clo = qbr < cb ? qbr : cb, chi = clo;
  p64_qint t = {-(8 * clo + 3), 8 * chi + 3, 0, 0, 0, 0};
  const int64_t B = (8 * (int64_t)clo + 3 + K + 1 + D - 1) / D;
  const int64_t X = t.vhi + K + B * D;
  for (int s = 1; s < 31; s++) {
    const int64_t M = (((int64_t)1 << s) + D - 1) / D;
    const int64_t eps = M * D - ((int64_t)1 << s);
    if (X * eps < ((int64_t)1 << s) && X * M < ((int64_t)1 << 31) && M < ((int64_t)1 << 23)) {
      t.m = (int32_t)M;
      t.s = s;
      t.cp = (int32_t)((K + B * D) * M - (B << s));
      t.cn = (int32_t)((D - 1 - K + B * D) * M - (B << s));
      return t;
    }
  }
  return t; /* unreachable for q = 1..31 (the test checks m != 0) */
}

#undef QI_FN
#endif
