/*
 * synth_impl.h -- per-pixel body of the deterministic synthetic video source.
 * Included by synth.c (host, gcc) and k_aux.hip (device generator); the
 * includer defines SYNTH_FN (`static inline` or `__host__ __device__ static
 * inline`).  Integer arithmetic only, so every includer produces the same bytes.
 */
#include <stdint.h>

SYNTH_FN uint32_t p64s_mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352dU;
  h ^= h >> 15;
  h *= 0x846ca68bU;
  h ^= h >> 16;
  return h;
}

SYNTH_FN uint32_t p64s_hash3(uint32_t a, uint32_t b, uint32_t c) {
  return p64s_mix32(a * 0x9E3779B1U ^ p64s_mix32(b * 0x85EBCA77U ^ p64s_mix32(c * 0xC2B2AE3DU + 0x27d4eb2fU)));
}

/* Bilinear value noise on a lattice of 2^lg pixels, result 0..255. */
SYNTH_FN int p64s_vnoise(uint32_t key, int32_t X, int32_t Y, int lg) {
  int32_t gx = X >> lg, gy = Y >> lg; /* arithmetic shift = floor */
  int32_t fx = X - (gx << lg), fy = Y - (gy << lg);
  int32_t n = 1 << lg;
  int32_t v00 = p64s_hash3(key, (uint32_t)gx, (uint32_t)gy) & 255;
  int32_t v10 = p64s_hash3(key, (uint32_t)(gx + 1), (uint32_t)gy) & 255;
  int32_t v01 = p64s_hash3(key, (uint32_t)gx, (uint32_t)(gy + 1)) & 255;
  int32_t v11 = p64s_hash3(key, (uint32_t)(gx + 1), (uint32_t)(gy + 1)) & 255;
  int32_t top = v00 * (n - fx) + v10 * fx;
  int32_t bot = v01 * (n - fx) + v11 * fx;
  return (top * (n - fy) + bot * fy) >> (2 * lg);
}

SYNTH_FN int p64s_texture(uint32_t key, int32_t X, int32_t Y) {
  int v = (p64s_vnoise(key, X, Y, 5) * 5 + p64s_vnoise(key ^ 0x55u, X, Y, 3) * 3) >> 3;
  v = 128 + ((v - 128) * 3) / 2; /* stretch contrast */
  v += (int)(p64s_hash3(key ^ 0xA5A5u, (uint32_t)X, (uint32_t)Y) & 15) - 8; /* detail */
  return v;
}

SYNTH_FN uint8_t p64s_clip8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

SYNTH_FN void p64s_motion(uint32_t seed, int *mvx, int *mvy) {
  *mvx = (int)(seed % 7u) - 3;
  *mvy = (int)((seed / 7u) % 5u) - 2;
}

SYNTH_FN uint32_t p64s_key(uint32_t seed, int frame) {
  uint32_t key = seed * 2654435761u + 17u;
  if ((seed & 7u) == 5u && frame >= 12) key ^= 0x5CE4Eu; /* scene cut */
  return key;
}

/* luma sample (i, j) of picture `frame` of stream `seed` */
SYNTH_FN uint8_t p64s_luma(uint32_t seed, int frame, int i, int j) {
  int mvx, mvy;
  p64s_motion(seed, &mvx, &mvy);
  uint32_t key = p64s_key(seed, frame);
  uint32_t h = p64s_hash3(key ^ 0xF00Du, (uint32_t)(i + (j << 16)), (uint32_t)frame);
  int tn = (int)(h & 7u) + (int)((h >> 3) & 7u) - 7; /* triangular +-7 */
  if ((seed & 7u) == 6u) tn = 0;
  int t = p64s_texture(key, i + mvx * frame, j + mvy * frame);
  if ((seed & 7u) == 7u) t = 128 + (t - 128) / 16;
  return p64s_clip8(t + tn / 2);
}

/* ---- SURVEY.md 8(d) content ("survey") -----------------------------------
 * luma = 128 + 50 sin(u/7) cos(v/11) + 30 sin((u+v)/23) + N(0,12) texture at
 * texture coordinates (u, v) = (x - 3t + ox, y + 2t + oy): picture t is the
 * texture translated by (+3, -2) px per picture, plus N(0,4) temporal noise,
 * clipped to 0..255; chroma from the 2x2-averaged luma of the same picture.
 * (ox, oy) is a per-seed origin, so sequences differ.  Integer only: a sine
 * is a 32-bit phase (angle = phase * 2 pi / 2^32) through a 9th-order
 * fixed-point polynomial (|error| < 1e-5), a Gaussian is a scaled sum of four
 * uniform 16-bit draws (Irwin-Hall), all in Q8 gray levels before the final
 * rounding -- every includer produces the same bytes. */

/* sin(2 pi p / 2^32) in Q15 */
SYNTH_FN int32_t p64v_sin_q15(uint32_t p) {
  const uint32_t q = p >> 30;
  int64_t x = (int64_t)(p & 0x3fffffffu); /* angle in the quadrant, Q30 of pi/2 */
  if (q & 1u) x = ((int64_t)1 << 30) - x;
  const int64_t x2 = (x * x) >> 30;
  /* sin(pi x / 2) = x (c1 - x^2 (c3 - x^2 (c5 - x^2 (c7 - x^2 c9)))), Q30 */
  int64_t s = 172272;
  s = 5026995 - ((s * x2) >> 30);
  s = 85569306 - ((s * x2) >> 30);
  s = 693598668 - ((s * x2) >> 30);
  s = 1686629713 - ((s * x2) >> 30);
  s = (s * x) >> 30;                       /* Q30, 0..1 */
  const int32_t r = (int32_t)((s + (1 << 14)) >> 15); /* Q15 */
  return q >= 2 ? -r : r;
}
/* phase of the angle k / d for d = 7, 11, 23: k * 2^32 / (2 pi d), mod 2^32 */
SYNTH_FN uint32_t p64v_phase(int32_t k, int64_t per) { return (uint32_t)((int64_t)k * per); }
/* N(0, sigma) in Q8 gray levels from a hash pair: m = sigma * 2^24 / sd,
   sd = sqrt(4 (2^32 - 1) / 12) the deviation of the four-draw sum */
SYNTH_FN int32_t p64v_gauss_q8(uint32_t h1, uint32_t h2, int32_t m) {
  const int32_t n = (int32_t)(h1 & 0xffffu) + (int32_t)(h1 >> 16) + (int32_t)(h2 & 0xffffu) +
                    (int32_t)(h2 >> 16) - 131070;
  return (int32_t)(((int64_t)n * m) >> 16);
}
SYNTH_FN void p64v_origin(uint32_t seed, int32_t *ox, int32_t *oy) {
  *ox = (int32_t)(p64s_mix32(seed * 0x9E3779B1u + 1u) & 1023u);
  *oy = (int32_t)(p64s_mix32(seed * 0x85EBCA77u + 2u) & 1023u);
}
/* luma sample (x, y) of picture t of survey stream `seed` */
SYNTH_FN uint8_t p64v_luma(uint32_t seed, int t, int x, int y) {
  int32_t ox, oy;
  p64v_origin(seed, &ox, &oy);
  const int32_t u = x - 3 * t + ox, v = y + 2 * t + oy;
  const int32_t s7 = p64v_sin_q15(p64v_phase(u, 97652182));
  const int32_t c11 = p64v_sin_q15(p64v_phase(v, 62142298) + 0x40000000u);
  const int32_t s23 = p64v_sin_q15(p64v_phase(u + v, 29720229));
  int64_t q8 = (int64_t)128 * 256 + (((int64_t)50 * s7 * c11) >> 22) + (((int64_t)30 * s23) >> 7);
  /* the texture's N(0,12): hashed at the texture coordinate (moves with it) */
  const uint32_t kt = p64s_mix32(seed * 0xC2B2AE3Du + 0x1234567u);
  q8 += p64v_gauss_q8(p64s_hash3(kt, (uint32_t)u, (uint32_t)v), p64s_hash3(kt ^ 0x5bd1e995u, (uint32_t)u, (uint32_t)v),
                      5321);
  /* the picture's N(0,4): hashed at the picture coordinate and t */
  const uint32_t kn = p64s_mix32(seed * 0x27d4eb2fu + 0x89abcdeu) ^ (uint32_t)t * 0x9E3779B1u;
  q8 += p64v_gauss_q8(p64s_hash3(kn, (uint32_t)x, (uint32_t)y), p64s_hash3(kn ^ 0x68e31da4u, (uint32_t)x, (uint32_t)y),
                      1774);
  return p64s_clip8((int)((q8 + 128) >> 8));
}
/* chroma (i, j) of U and V from the 2x2 average a of the luma (given) */
SYNTH_FN void p64v_chroma_of(int a4, uint8_t *u, uint8_t *v) {
  const int a = (a4 + 2) >> 2;
  *u = p64s_clip8(128 + (a - 128) / 2);
  *v = p64s_clip8(128 - (a - 128) / 3);
}

/* chroma samples (i, j) of U and V */
SYNTH_FN void p64s_chroma(uint32_t seed, int frame, int i, int j, uint8_t *u, uint8_t *v) {
  int mvx, mvy;
  p64s_motion(seed, &mvx, &mvy);
  uint32_t key = p64s_key(seed, frame);
  int32_t cx = (mvx * frame) >> 1, cy = (mvy * frame) >> 1;
  uint32_t h = p64s_hash3(key ^ 0xC0DEu, (uint32_t)(i + (j << 16)), (uint32_t)frame);
  int tn = (seed & 7u) == 6u ? 0 : (int)(h & 3u) - 1;
  int tu = p64s_vnoise(key ^ 0x1111u, i + cx, j + cy, 4);
  int tv = p64s_vnoise(key ^ 0x2222u, i + cx, j + cy, 4);
  *u = p64s_clip8(128 + (tu - 128) / 3 + tn);
  *v = p64s_clip8(128 + (tv - 128) / 3 - tn);
}
