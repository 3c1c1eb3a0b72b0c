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
