"""The block kernels' integer quantiser (p64_amd/csrc/quant_int.h: one
v_mad_i32_i24 and one arithmetic shift per coefficient, from the raw Chen
row-pass output) against the reference's chain restated in C -- final /8
(chendct.c:204), BoundDctMatrix (transform.c:460), CCITT(Flat)Quantize
(transform.c:283-306, 339-347), (Flat)BoundQuantizeMatrix (transform.c:
502-537) -- for every q = 1..31 and every raw value the kernels can produce
(AC: |v| <= 2^15, far beyond the largest DCT output; inter DC: |v| <=
16383, beyond the |v| <= 16323 a DCT of 8-bit residuals reaches), AC and the
inter DC.  The
kernel evaluates exactly this int32 arithmetic; the harness also checks that
no intermediate leaves int32 and that the 24-bit multiply operands fit."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include <stdio.h>
#include <stdlib.h>
#include "quant_int.h"

static int trunc_div(int a, int d) { return a / d; } /* C truncation */

/* reference: raw v -> level (dc_inter: DC of an inter block) */
static int ref_level(int v, int q, int dc_inter) {
  int c = v < 0 ? (v - 4) / 8 : (v + 4) / 8;              /* chendct.c:204 */
  if (dc_inter) { if (c > 2047) c = 2047; }                /* BoundDctMatrix DC */
  else { if (c > 1023) c = 1023; if (c < -1023) c = -1023; }
  if (!(q & 1)) c = c > 0 ? c + 1 : c - 1;                 /* transform.c:285 */
  int l = trunc_div(c, 2 * q);
  if (l > 127) l = 127;
  if (l < -127) l = -127;                                  /* BoundQuantizeMatrix */
  return l;
}

int main(void) {
  long bad = 0;
  for (int dc = 0; dc < 2; dc++)
    for (int q = 1; q <= 31; q++) {
      const p64_qint t = p64_qint_make(q, dc);
      if (!t.m || t.m >= (1 << 23) || t.vhi >= (1 << 23)) { printf("no constants q=%d dc=%d\n", q, dc); return 1; }
      const int vmax = dc ? 16383 : 32768;
      for (int v = -vmax; v <= vmax; v++) {
        const int vc = v < t.vlo ? t.vlo : (v > t.vhi ? t.vhi : v);           /* v_med3_i32 */
        const long long x = (long long)vc * t.m + (vc < 0 ? t.cn : t.cp);     /* v_mad_i32_i24 */
        if (x < -2147483648LL || x > 2147483647LL) { printf("overflow q=%d v=%d\n", q, v); return 1; }
        const int l = (int)x >> t.s;                                          /* v_ashrrev_i32 */
        if (l != ref_level(v, q, dc) && bad++ < 10) printf("q=%d dc=%d v=%d got %d want %d\n", q, dc, v, l, ref_level(v, q, dc));
      }
    }
  printf("mismatches %ld\n", bad);
  return bad != 0;
}
"""


def test_integer_quantiser_exhaustive(tmp_path):
    c = tmp_path / "qint.c"
    c.write_text(SRC)
    exe = tmp_path / "qint"
    subprocess.run(["gcc", "-O2", "-Wall", "-I", os.path.join(REPO, "p64_amd", "csrc"), str(c), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "mismatches 0" in r.stdout
