/*
 * synth.c -- deterministic synthetic YCbCr 4:2:0 video (integer arithmetic only).
 *
 * SURVEY.md 8(d) asks for a seeded moving texture plus noise so that motion
 * search and the MTYPE decision see realistic content.  This generator is the
 * single source of input bytes for the GPU path, the CPU baselines and the
 * golden fixtures: it is pure integer C, so every caller gets identical bytes.
 *
 * Frame f of stream `seed`: a two-octave value-noise texture with per-pixel
 * detail, translated by f*(mvx,mvy) (chroma by the floor of half that), plus
 * small temporal noise.  Seeds = 5 (mod 8) switch texture at frame 12 so intra
 * decisions appear; seeds = 6 (mod 8) carry no temporal noise, so exact matches
 * (MTYPE 5 and the CBP fallback to MTYPE 4) appear too; seeds = 7 (mod 8) are
 * low-contrast, so the zero-vector MTYPE 2 and its fallback to 4 appear.
 */
#include <stddef.h>
#include <stdint.h>

#include "../../include/p64gpu.h"

#define SYNTH_FN static inline
#include "synth_impl.h"

void p64_synth_motion(uint32_t seed, int *mvx, int *mvy) { p64s_motion(seed, mvx, mvy); }

/* SURVEY.md 8(d) content (synth_impl.h p64v_*): luma, then chroma from it */
static void survey_frame(uint32_t seed, int frame, int width, int height, uint8_t *out) {
  uint8_t *y = out, *u = out + (size_t)width * height;
  uint8_t *v = u + (size_t)(width / 2) * (height / 2);
  for (int j = 0; j < height; j++)
    for (int i = 0; i < width; i++) y[(size_t)j * width + i] = p64v_luma(seed, frame, i, j);
  for (int j = 0; j < height / 2; j++)
    for (int i = 0; i < width / 2; i++) {
      const uint8_t *p = y + (size_t)(2 * j) * width + 2 * i;
      size_t k = (size_t)j * (width / 2) + i;
      p64v_chroma_of(p[0] + p[1] + p[width] + p[width + 1], &u[k], &v[k]);
    }
}

int p64_synth_frame_content(int content, uint32_t seed, int frame, int width, int height, uint8_t *out) {
  if (!out || width < 16 || height < 16 || (width & 15) || (height & 15) || frame < 0) return P64GPU_E_INVALID;
  if (content == P64_SYNTH_VNOISE)
    p64_synth_frame(seed, frame, width, height, out);
  else if (content == P64_SYNTH_SURVEY)
    survey_frame(seed, frame, width, height, out);
  else
    return P64GPU_E_INVALID;
  return P64GPU_OK;
}

void p64_synth_frame(uint32_t seed, int frame, int width, int height, uint8_t *out) {
  uint8_t *y = out, *u = out + (size_t)width * height;
  uint8_t *v = u + (size_t)(width / 2) * (height / 2);
  for (int j = 0; j < height; j++)
    for (int i = 0; i < width; i++) y[(size_t)j * width + i] = p64s_luma(seed, frame, i, j);
  for (int j = 0; j < height / 2; j++)
    for (int i = 0; i < width / 2; i++) {
      size_t k = (size_t)j * (width / 2) + i;
      p64s_chroma(seed, frame, i, j, &u[k], &v[k]);
    }
}
