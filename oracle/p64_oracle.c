/*
 * p64_oracle.c -- TEST INFRASTRUCTURE ONLY (see p64_oracle.h).
 *
 * Clean-room restatement of the PVRG-P64 per-macroblock hot path.  Written for
 * clarity, not speed: scalar C, one function per reference routine, each
 * citing the file:line of /root/reference it restates.  Pinned against the
 * reference by tests/test_oracle_golden.py.
 */
#include "p64_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Chen integer DCT (chendct.c).  NO_MULTIPLY is forced on (chendct.c:43), so
 * every scaling is an arithmetic shift: MSCALE(x) = x >> 9 (chendct.c:53).   */

#define K_C1D4 362 /* chendct.c:57-65 */
#define K_C1D8 473
#define K_C3D8 196
#define K_C1D16 502
#define K_C3D16 426
#define K_C5D16 284
#define K_C7D16 100

static inline int32_t ms(int32_t v) { return v >> 9; }

/* 8-point forward butterfly on already-scaled sums s[k]=(x_k+x_{7-k})*scale
 * and differences d[k]=(x_k-x_{7-k})*scale, k=0..3 (chendct.c:120-159). */
static void fwd8(const int32_t s[4], const int32_t d[4], int32_t o[8]) {
  int32_t e0 = s[0] + s[3], e1 = s[1] + s[2];
  int32_t e2 = s[1] - s[2], e3 = s[0] - s[3];
  o[0] = ms(K_C1D4 * (e0 + e1));
  o[4] = ms(K_C1D4 * (e0 - e1));
  o[2] = ms(K_C3D8 * e2 + K_C1D8 * e3);
  o[6] = ms(K_C3D8 * e3 - K_C1D8 * e2);
  /* odd half: d[1],d[2] rotate by pi/4 first */
  int32_t r0 = ms(K_C1D4 * (d[1] - d[2]));
  int32_t r1 = ms(K_C1D4 * (d[1] + d[2]));
  int32_t u0 = d[3] + r0, u1 = d[3] - r0;
  int32_t u2 = d[0] - r1, u3 = d[0] + r1;
  o[1] = ms(K_C7D16 * u0 + K_C1D16 * u3);
  o[3] = ms(K_C3D16 * u2 - K_C5D16 * u1);
  o[5] = ms(K_C3D16 * u1 + K_C5D16 * u2);
  o[7] = ms(K_C7D16 * u3 - K_C1D16 * u0);
}

/* chendct.c:97-206.  Columns: sums/differences scaled <<2; rows: >>1 applied
 * to the sum/difference (not to each input); final /8 rounds half away. */
void orc_chen_dct(const int32_t *in, int32_t *out) {
  int32_t t[64], s[4], d[4], o[8];
  for (int c = 0; c < 8; c++) {
    for (int k = 0; k < 4; k++) {
      int32_t a = in[8 * k + c], b = in[8 * (7 - k) + c];
      s[k] = (a + b) << 2;
      d[k] = (a - b) << 2;
    }
    fwd8(s, d, o);
    for (int k = 0; k < 8; k++) t[8 * k + c] = o[k];
  }
  for (int r = 0; r < 8; r++) {
    for (int k = 0; k < 4; k++) {
      int32_t a = t[8 * r + k], b = t[8 * r + 7 - k];
      s[k] = (a + b) >> 1;
      d[k] = (a - b) >> 1;
    }
    fwd8(s, d, o);
    for (int k = 0; k < 8; k++) t[8 * r + k] = o[k];
  }
  for (int i = 0; i < 64; i++)
    out[i] = (t[i] < 0 ? t[i] - 4 : t[i] + 4) / 8; /* C truncation */
}

/* 8-point inverse butterfly, inputs x[0..7] already scaled
 * (chendct.c:254-303 / 320-365). */
static void inv8(const int32_t x[8], int32_t o[8]) {
  int32_t ev0 = x[0], ev1 = x[4], ev2 = x[2], ev3 = x[6];
  int32_t od0 = x[1], od1 = x[3], od2 = x[5], od3 = x[7];
  int32_t p0 = ms(K_C7D16 * od0 - K_C1D16 * od3);
  int32_t p1 = ms(K_C3D16 * od2 - K_C5D16 * od1);
  int32_t p2 = ms(K_C3D16 * od1 + K_C5D16 * od2);
  int32_t p3 = ms(K_C1D16 * od0 + K_C7D16 * od3);
  int32_t q0 = ms(K_C1D4 * (ev0 + ev1));
  int32_t q1 = ms(K_C1D4 * (ev0 - ev1));
  int32_t q2 = ms(K_C3D8 * ev2 - K_C1D8 * ev3);
  int32_t q3 = ms(K_C1D8 * ev2 + K_C3D8 * ev3);
  int32_t e0 = q0 + q3, e1 = q1 + q2, e2 = q1 - q2, e3 = q0 - q3;
  int32_t f0 = p0 + p1, f1 = p0 - p1, f2 = p3 - p2, f3 = p3 + p2;
  int32_t g1 = ms(K_C1D4 * (f2 - f1));
  int32_t g2 = ms(K_C1D4 * (f2 + f1));
  o[0] = e0 + f3;
  o[1] = e1 + g2;
  o[2] = e2 + g1;
  o[3] = e3 + f0;
  o[4] = e3 - f0;
  o[5] = e2 - g1;
  o[6] = e1 - g2;
  o[7] = e0 - f3;
}

/* chendct.c:217-375: columns with inputs <<2, rows unscaled, final /16. */
void orc_chen_idct(const int32_t *in, int32_t *out) {
  int32_t t[64], x[8], o[8];
  for (int c = 0; c < 8; c++) {
    for (int k = 0; k < 8; k++) x[k] = in[8 * k + c] << 2;
    inv8(x, o);
    for (int k = 0; k < 8; k++) t[8 * k + c] = o[k];
  }
  for (int r = 0; r < 8; r++) {
    for (int k = 0; k < 8; k++) x[k] = t[8 * r + k];
    inv8(x, o);
    for (int k = 0; k < 8; k++) t[8 * r + k] = o[k];
  }
  for (int i = 0; i < 64; i++)
    out[i] = (t[i] < 0 ? t[i] - 8 : t[i] + 8) / 16;
}

/* ------------------------------------------------------------------------ */
/* Quantisers (transform.c, non-VERSION_1_0 branch).  FastDivide
 * (transform.c:92-127) is plain C division, i.e. truncation toward zero. */

/* H.261 level for one inter/AC coefficient with step 2q (transform.c:283-306):
 * odd q: c/(2q); even q: (c + sign(c))/(2q), where sign(0) = -1. */
static int32_t qlevel(int32_t c, int q) {
  if (q & 1) return c / (2 * q);
  return (c + (c > 0 ? 1 : -1)) / (2 * q);
}

/* Intra AC rule (transform.c:339-347): the +-1 uses (c > 0), so c == 0 -> -1 as
 * well; identical to qlevel. */

void orc_quant_inter(int32_t *m, int dcq, int acq) {
  m[0] = qlevel(m[0], dcq);
  for (int i = 1; i < 64; i++) m[i] = qlevel(m[i], acq);
}

void orc_quant_intra(int32_t *m, int dcq, int acq) {
  /* transform.c:321-325: DC rounds half away with dcq/2 */
  m[0] = m[0] > 0 ? (m[0] + dcq / 2) / dcq : (m[0] - dcq / 2) / dcq;
  for (int i = 1; i < 64; i++) m[i] = qlevel(m[i], acq);
}

/* Reconstruction level for a nonzero level (transform.c:376-389, 436-448):
 * odd q: (2l +- 1) q; even q: (2l +- 1) q -+ 1; zero stays zero. */
static int32_t rlevel(int32_t l, int q) {
  if (l == 0) return 0;
  int32_t sgn = l > 0 ? 1 : -1;
  int32_t v = (2 * l + sgn) * q;
  if (!(q & 1)) v -= sgn;
  return v;
}

void orc_iquant_intra(int32_t *m, int dcq, int acq) {
  m[0] = m[0] * dcq; /* transform.c:363 */
  for (int i = 1; i < 64; i++) m[i] = rlevel(m[i], acq);
}

void orc_iquant_inter(int32_t *m, int dcq, int acq) {
  m[0] = rlevel(m[0], dcq); /* transform.c:417-429 */
  for (int i = 1; i < 64; i++) m[i] = rlevel(m[i], acq);
}

static inline int32_t clampi(int32_t v, int32_t lo, int32_t hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

void orc_bound_dct(int32_t *m) { /* transform.c:460-474: DC upper bound only */
  if (m[0] > 2047) m[0] = 2047;
  for (int i = 1; i < 64; i++) m[i] = clampi(m[i], -1023, 1023);
}
void orc_bound_idct(int32_t *m) { /* transform.c:483-494 */
  for (int i = 0; i < 64; i++) m[i] = clampi(m[i], 0, 255);
}
void orc_bound_quant_flat(int32_t *m) { /* transform.c:502-518 */
  m[0] = clampi(m[0], 1, 254);
  for (int i = 1; i < 64; i++) m[i] = clampi(m[i], -127, 127);
}
void orc_bound_quant(int32_t *m) { /* transform.c:526-537 */
  for (int i = 0; i < 64; i++) m[i] = clampi(m[i], -127, 127);
}

/* Zigzag scan position of natural (row-major) index n; the standard H.261 /
 * JPEG scan, generated rather than tabulated (matches transform.c:67-75). */
static int zz_pos[64];
static int zz_ready;
static void zz_init(void) {
  if (zz_ready) return;
  int k = 0;
  for (int s = 0; s < 15; s++) {
    int rlo = s < 8 ? 0 : s - 7, rhi = s < 8 ? s : 7;
    if (s & 1)
      for (int r = rlo; r <= rhi; r++) zz_pos[8 * r + (s - r)] = k++;
    else
      for (int r = rhi; r >= rlo; r--) zz_pos[8 * r + (s - r)] = k++;
  }
  zz_ready = 1;
}
void orc_zigzag(const int32_t *in, int32_t *out) { /* transform.c:561-568 */
  zz_init();
  for (int n = 0; n < 64; n++) out[zz_pos[n]] = in[n];
}
void orc_izigzag(const int32_t *in, int32_t *out) { /* transform.c:546-553 */
  zz_init();
  for (int n = 0; n < 64; n++) out[n] = in[zz_pos[n]];
}

/* ------------------------------------------------------------------------ */
/* Motion estimation (me.c).  ComputeError's early exit (me.c:122/133/170)
 * never changes the result: partial sums are monotone and acceptance is a
 * strict '<' against the running best, so a full SAD is equivalent. */

int orc_sad16(const uint8_t *ref, int rs, const uint8_t *cur, int cs) {
  int e = 0;
  for (int r = 0; r < 16; r++)
    for (int c = 0; c < 16; c++) e += abs((int)ref[r * rs + c] - (int)cur[r * cs + c]);
  return e;
}

/* Candidate test shared by FastBME (me.c:212-213) and StepBME (me.c:292-294):
 * note px < W-16 excludes the last legal column (and row). */
static int in_window(int px, int py, int w, int h) {
  return px >= 0 && px < w - 16 && py >= 0 && py < h - 16;
}

/* Statistics on the chosen block (me.c:229-245 == 313-329). VAROR and MWOR
 * are measured on the REFERENCE block. */
static void me_stats(const uint8_t *ref, const uint8_t *cur, int w, int x, int y,
                     orc_me_rec *r) {
  int var = 0, sq = 0, sum = 0;
  const uint8_t *b = ref + (size_t)(y + r->my) * w + x + r->mx;
  const uint8_t *c = cur + (size_t)y * w + x;
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) {
      int bv = b[i * w + j], d = bv - c[i * w + j];
      var += d * d;
      sq += bv * bv;
      sum += bv;
    }
  r->var = var / 256;
  r->varor = sq / 256 - (sum / 256) * (sum / 256);
  r->mwor = sum;
}

void orc_me_mb(const uint8_t *ref, const uint8_t *cur, int w, int h, int x,
               int y, int mode, int sl, orc_me_rec *r) {
  const uint8_t *cb = cur + (size_t)y * w + x;
  int best = orc_sad16(ref + (size_t)y * w + x, w, cb, w);
  int bx = 0, by = 0;
  r->sad0 = best;
  if (mode == ORC_ME_FULL) {
    /* FastBME me.c:206-227: dx outer, dy inner, [-sl/2, sl/2) */
    for (int dx = -sl / 2; dx < sl / 2; dx++)
      for (int dy = -sl / 2; dy < sl / 2; dy++) {
        int px = x + dx, py = y + dy;
        if (!in_window(px, py, w, h)) continue;
        int e = orc_sad16(ref + (size_t)py * w + px, w, cb, w);
        if (e < best) best = e, bx = dx, by = dy;
      }
  } else {
    /* StepBME me.c:277-311: steps 8,4,2,1 around the running best */
    int cx = x, cy = y;
    for (int step = 8; step >= 1; step /= 2) {
      for (int diry = -1; diry <= 1; diry++)
        for (int dirx = -1; dirx <= 1; dirx++) {
          if (!dirx && !diry) continue;
          int px = cx + dirx * step, py = cy + diry * step;
          int dx = px - x, dy = py - y;
          if (!in_window(px, py, w, h) || dx < -15 || dx > 15 || dy < -15 || dy > 15)
            continue;
          int e = orc_sad16(ref + (size_t)py * w + px, w, cb, w);
          if (e < best) best = e, bx = dx, by = dy;
        }
      cx = x + bx;
      cy = y + by;
    }
  }
  r->mx = bx;
  r->my = by;
  r->sad = best;
  me_stats(ref, cur, w, x, y, r);
}

void orc_motion_estimation(const uint8_t *ref, const uint8_t *cur, int w, int h,
                           int mode, int sl, orc_me_rec *recs) {
  int n = 0; /* me.c:347-361: raster order, y outer */
  for (int y = 0; y < h; y += 16)
    for (int x = 0; x < w; x += 16) orc_me_mb(ref, cur, w, h, x, y, mode, sl, &recs[n++]);
}

/* ------------------------------------------------------------------------ */
/* Prediction (io.c). */

/* io.c:323-372: H.261 loop filter on an 8x8 block.  Horizontal [1 2 1] with the
 * edge columns taken x4; vertical [1 2 1] >>2 on rows 1..6, rows 0/7 kept;
 * then a final /4 that rounds half up: (v&2) ? (v>>2)+1 : v>>2. */
void orc_load_filter(const uint8_t *src, int stride, int32_t *out) {
  int32_t hz[64];
  for (int r = 0; r < 8; r++) {
    const uint8_t *p = src + (size_t)r * stride;
    hz[8 * r] = p[0] << 2;
    for (int c = 1; c < 7; c++) hz[8 * r + c] = p[c - 1] + 2 * p[c] + p[c + 1];
    hz[8 * r + 7] = p[7] << 2;
  }
  for (int r = 0; r < 8; r++)
    for (int c = 0; c < 8; c++) {
      int32_t v = hz[8 * r + c];
      if (r > 0 && r < 7) v = (hz[8 * (r - 1) + c] + 2 * v + hz[8 * (r + 1) + c]) >> 2;
      out[8 * r + c] = (v & 2) ? (v >> 2) + 1 : (v >> 2);
    }
}

/* Coding-control tables (p64.c:217-222), indexed by MTYPE 0..9. */
static const int8_t T_QUANT[10] = {0, 1, 0, 1, 0, 0, 1, 0, 0, 1};
static const int8_t T_CBP[10] = {0, 0, 1, 1, 0, 1, 1, 0, 1, 1};
static const int8_t T_INTRA[10] = {1, 1, 0, 0, 0, 0, 0, 0, 0, 0};
static const int8_t T_MF[10] = {0, 0, 0, 0, 1, 1, 1, 1, 1, 1};
static const int8_t T_FILTER[10] = {0, 0, 0, 0, 0, 0, 0, 1, 1, 1};
static const int8_t T_TCOEFF[10] = {1, 1, 1, 1, 0, 1, 1, 0, 1, 1};

typedef struct {
  const uint8_t *plane;
  int stride;
  int bx, by; /* block origin in the plane, pixels */
} blk_at;

/* Block c of MB (mbx,mby): c=0..3 luma (h,v) = (0,0),(1,0),(0,1),(1,1), 4=U,
 * 5=V (p64.c:77-79 BlockJ/V/H; io.c:719-747 MoveTo). */
static blk_at block_origin(const uint8_t *planes, int w, int h, int mbx, int mby,
                           int c) {
  blk_at b;
  if (c < 4) {
    b.plane = planes;
    b.stride = w;
    b.bx = 16 * mbx + 8 * (c & 1);
    b.by = 16 * mby + 8 * (c >> 1);
  } else {
    b.plane = planes + (size_t)w * h + (size_t)(c - 4) * (w / 2) * (h / 2);
    b.stride = w / 2;
    b.bx = 8 * mbx;
    b.by = 8 * mby;
  }
  return b;
}

/* Prediction for block c under MTYPE mt with vector (mvx,mvy) from the
 * previous reconstruction (io.c:142-496): MTYPE 2/3 zero vector (SubOverlay),
 * MC types full-pel for luma and MV/2 (C truncation) for chroma
 * (HalfSubCompensate io.c:268-270), filter types through LoadFilterMatrix. */
static void predict(const uint8_t *ref, int w, int h, int mbx, int mby, int c,
                    int mt, int mvx, int mvy, int32_t *pred) {
  blk_at b = block_origin(ref, w, h, mbx, mby, c);
  int dx = 0, dy = 0;
  if (T_MF[mt]) {
    dx = c < 4 ? mvx : mvx / 2;
    dy = c < 4 ? mvy : mvy / 2;
  }
  const uint8_t *src = b.plane + (size_t)(b.by + dy) * b.stride + b.bx + dx;
  if (T_FILTER[mt]) {
    orc_load_filter(src, b.stride, pred);
  } else {
    for (int r = 0; r < 8; r++)
      for (int k = 0; k < 8; k++) pred[8 * r + k] = src[(size_t)r * b.stride + k];
  }
}

/* MTYPE decision, p64.c:734-773.  The comparisons are evaluated in IEEE
 * binary64 exactly as written (an integer rewrite differs). */
static int decide_mtype(const orc_me_rec *r) {
  double xv = (double)r->sad0, yv = (double)r->sad;
  xv = xv / 256;
  yv = yv / 256;
  if (r->var < 64 || r->varor > r->var) {
    if (xv < 1.0 || (xv < 3.0 && yv > xv * 0.5) || yv > xv / 1.1) return 2;
    if (r->var < 6.0) return 5;
    return 8;
  }
  return 0;
}

#define SEQ_INTRA_THRESHOLD 131 /* p64.c:159 */
#define CBP_THRESHOLD 1         /* p64.c:151 */

void orc_encode_frame(int w, int h, const uint8_t *cur, const uint8_t *ref,
                      uint8_t *recon, int intra_frame, int quant,
                      const uint8_t *quant_mb, const int8_t *mtype_override,
                      uint8_t *last_intra, int me_mode, int sl,
                      const orc_me_rec *me_in, orc_me_rec *me_out,
                      int16_t *coef, orc_mb_rec *mbrec) {
  int mbw = w / 16, mbh = h / 16, nmb = mbw * mbh;
  orc_me_rec *me = NULL;
  if (!intra_frame) {
    if (me_in) {
      me = (orc_me_rec *)me_in;
    } else {
      me = me_out ? me_out : (orc_me_rec *)malloc(sizeof(orc_me_rec) * nmb);
      orc_motion_estimation(ref, cur, w, h, me_mode, sl, me);
    }
  }
  for (int mb = 0; mb < nmb; mb++) {
    int mbx = mb % mbw, mby = mb / mbw;
    int mt = 0, mvx = 0, mvy = 0;
    if (!intra_frame) {
      mt = decide_mtype(&me[mb]);
      if (mtype_override && mtype_override[mb] >= 0) mt = mtype_override[mb];
      mvx = me[mb].mx;
      mvy = me[mb].my;
    }
    if (last_intra[mb] > SEQ_INTRA_THRESHOLD) mt = 0; /* p64.c:772-773 */
    int q = quant_mb ? quant_mb[mb] : quant;

    int32_t lev[6][64], pred[6][64];
    int cbp;
    for (;;) { /* ReadCompressMDU p64.c:830-912 */
      for (int c = 0; c < 6; c++) {
        int32_t blk[64], tmp[64];
        if (!T_TCOEFF[mt]) {
          memset(lev[c], 0, sizeof lev[c]);
          continue;
        }
        blk_at b = block_origin(cur, w, h, mbx, mby, c);
        for (int r = 0; r < 8; r++)
          for (int k = 0; k < 8; k++)
            blk[8 * r + k] = b.plane[(size_t)(b.by + r) * b.stride + b.bx + k];
        if (!T_INTRA[mt]) {
          predict(ref, w, h, mbx, mby, c, mt, mvx, mvy, pred[c]);
          for (int i = 0; i < 64; i++) blk[i] -= pred[c][i];
        }
        orc_chen_dct(blk, tmp);
        orc_bound_dct(tmp);
        if (T_INTRA[mt]) {
          orc_quant_intra(tmp, 8, q);
          orc_bound_quant_flat(tmp);
        } else {
          orc_quant_inter(tmp, q, q);
          orc_bound_quant(tmp);
        }
        orc_zigzag(tmp, lev[c]);
      }
      if (!T_CBP[mt]) {
        cbp = 0x3f;
      } else {
        int pmask = 0;
        cbp = 0;
        for (int c = 0; c < 6; c++) {
          int acc = 0;
          for (int i = 0; i < 64; i++) acc += abs(lev[c][i]);
          if (acc && !pmask) pmask = 1 << (5 - c);
          if (acc > CBP_THRESHOLD) cbp |= 1 << (5 - c);
        }
        if (!cbp) {
          if (pmask) {
            cbp = pmask;
          } else { /* nothing to code: MC without coefficients, keep the ME vector */
            mt = T_FILTER[mt] ? 7 : 4;
            continue;
          }
        }
      }
      break;
    }
    last_intra[mb] = T_INTRA[mt] ? 0 : (uint8_t)(last_intra[mb] + 1); /* p64.c:909-910 */

    /* WriteMDU recon (p64.c:945-959) + DecodeSaveMDU (p64.c:971-1013) */
    for (int c = 0; c < 6; c++) {
      int32_t res[64], tmp[64];
      if ((cbp & (1 << (5 - c))) && T_TCOEFF[mt]) {
        orc_izigzag(lev[c], tmp);
        if (T_INTRA[mt])
          orc_iquant_intra(tmp, 8, q);
        else
          orc_iquant_inter(tmp, q, q);
        orc_chen_idct(tmp, res);
      } else {
        memset(res, 0, sizeof res);
      }
      if (!T_INTRA[mt]) {
        predict(ref, w, h, mbx, mby, c, mt, mvx, mvy, pred[c]);
        for (int i = 0; i < 64; i++) res[i] += pred[c][i];
      }
      orc_bound_idct(res);
      blk_at b = block_origin(recon, w, h, mbx, mby, c);
      uint8_t *dst = (uint8_t *)b.plane;
      for (int r = 0; r < 8; r++)
        for (int k = 0; k < 8; k++)
          dst[(size_t)(b.by + r) * b.stride + b.bx + k] = (uint8_t)res[8 * r + k];
    }
    if (coef)
      for (int c = 0; c < 6; c++)
        for (int i = 0; i < 64; i++) coef[(size_t)mb * 384 + 64 * c + i] = (int16_t)lev[c][i];
    (void)T_QUANT; /* UseQuant = MQuant for QuantMType; supplied via quant_mb */
    mbrec[mb].mtype = (int8_t)mt;
    mbrec[mb].cbp = (int8_t)cbp;
    mbrec[mb].mvx = (int8_t)(T_MF[mt] ? mvx : 0);
    mbrec[mb].mvy = (int8_t)(T_MF[mt] ? mvy : 0);
  }
  if (me && !me_in && !me_out) free(me);
}

/* Decoder-side MB reconstruction: DecompressMDU (p64.c:1218-1236) +
 * DecodeSaveMDU (p64.c:971-1013).  recon already holds the picture being
 * built; ref is the previous picture (CFS). */
void orc_decode_mb(int w, int h, const uint8_t *ref, uint8_t *recon, int mbx,
                   int mby, int mt, int cbp, int mvx, int mvy, int q,
                   const int16_t *coef) {
  if (!T_CBP[mt]) cbp = 0x3f;
  for (int c = 0; c < 6; c++) {
    int32_t res[64], tmp[64], lv[64], pred[64];
    if ((cbp & (1 << (5 - c))) && T_TCOEFF[mt]) {
      for (int i = 0; i < 64; i++) lv[i] = coef[64 * c + i];
      orc_izigzag(lv, tmp);
      if (T_INTRA[mt])
        orc_iquant_intra(tmp, 8, q);
      else
        orc_iquant_inter(tmp, q, q);
      orc_chen_idct(tmp, res);
    } else {
      memset(res, 0, sizeof res);
    }
    if (!T_INTRA[mt]) {
      predict(ref, w, h, mbx, mby, c, mt, mvx, mvy, pred);
      for (int i = 0; i < 64; i++) res[i] += pred[i];
    }
    orc_bound_idct(res);
    blk_at b = block_origin(recon, w, h, mbx, mby, c);
    uint8_t *dst = (uint8_t *)b.plane;
    for (int r = 0; r < 8; r++)
      for (int k = 0; k < 8; k++)
        dst[(size_t)(b.by + r) * b.stride + b.bx + k] = (uint8_t)res[8 * r + k];
  }
}
