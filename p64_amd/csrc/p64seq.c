/*
 * p64seq.c -- sequence loop and rate control of the reference encoder over the
 * GPU hot path (include/p64seq.h).  Host C on the public C ABI only.
 *
 * Integer arithmetic follows the reference's C `int` expressions, including
 * their 32-bit wrap-around (computed in uint32_t and converted back), so the
 * bit budget and the quantiser choices match for every -r / -x / -k / -f.
 */
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/p64prog.h"
#include "../../include/p64seq.h"

int p64gpu_fail_(int status, const char *msg); /* p64gpu_abi.hip: sets last error */

static int fail(int status, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int status, const char *fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return p64gpu_fail_(status, buf);
}

/* C int arithmetic with the wrap-around the reference's expressions have */
static int32_t imul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static int32_t idiv(int32_t a, int32_t b) { return b ? a / b : 0; }

struct p64seq {
  p64seq_config c;
  int w, h, ngob, nmb;
  size_t pic;
  /* device */
  uint8_t *d_cur, *d_rec[2], *d_li, *d_q, *d_mask;
  int16_t *d_coef;
  p64_mb_rec *d_mb;
  int32_t *d_lists; /* [ngob][33] raster MB indices of each GOB */
  int cur;          /* d_rec[cur] receives this picture; d_rec[cur ^ 1] = CFS */
  /* host */
  int16_t *h_coef;
  p64_mb_rec *h_mb;
  uint8_t *h_li_old, *h_li, *h_mask, *h_q;
  int8_t *h_ov, *d_ov;
  p64_me_rec *h_me, *d_me;
  int32_t *h_lists;
  p64s_writer *wr;
  p64prog *prog; /* -o program, or NULL */
  /* device entropy coding of whole pictures (p64gpu_vlc_pictures) */
  uint8_t *d_vout, *d_vgq, *d_vphase, *h_vout;
  uint32_t *d_vbits, *d_vscratch;
  int32_t *d_vtr;
  int64_t vstride;
  /* reference state (p64.c globals) */
  int current_frame, rate, qdfact, qoffs, gquant, mquant, mtype, buffer_offset, novfl, pic_ovfl;
  int frames, finished;
  int64_t total_bits, last_bits, first_frame_bits;
  int hist[10];
};

void p64seq_default_config(p64seq_config *c) {
  memset(c, 0, sizeof *c);
  c->search_limit = 15;
  c->frame_skip = 1;
  c->frame_rate = 30000;
  c->frame_rate_div = 1001;
}

void p64seq_close(p64seq *s) {
  if (!s) return;
  p64gpu_free(s->d_cur);
  p64gpu_free(s->d_rec[0]);
  p64gpu_free(s->d_rec[1]);
  p64gpu_free(s->d_li);
  p64gpu_free(s->d_q);
  p64gpu_free(s->d_mask);
  p64gpu_free(s->d_coef);
  p64gpu_free(s->d_mb);
  p64gpu_free(s->d_lists);
  p64gpu_free(s->d_ov);
  p64gpu_free(s->d_me);
  p64gpu_free(s->d_vout);
  p64gpu_free(s->d_vgq);
  p64gpu_free(s->d_vphase);
  p64gpu_free(s->d_vbits);
  p64gpu_free(s->d_vscratch);
  p64gpu_free(s->d_vtr);
  free(s->h_vout);
  free(s->h_ov);
  free(s->h_me);
  free(s->h_coef);
  free(s->h_mb);
  free(s->h_li_old);
  free(s->h_li);
  free(s->h_mask);
  free(s->h_q);
  free(s->h_lists);
  p64s_writer_close(s->wr);
  free(s);
}

int p64seq_open(const p64seq_config *cfg, p64seq **out) {
  int st;
  if (!cfg || !out) return fail(P64GPU_E_INVALID, "p64seq_open: NULL argument");
  const p64seq_config *c = cfg;
  if (c->me_mode != P64GPU_ME_TSS && c->me_mode != P64GPU_ME_FULL)
    return fail(P64GPU_E_INVALID, "me mode %d", c->me_mode);
  if (c->search_limit < 1 || c->search_limit > 31 || c->quant < 0 || c->quant > 31 || c->rate < 0 ||
      c->file_size_bits < 0 || c->frame_skip < 1 || c->frame_rate < 1 || c->frame_rate_div < 1 ||
      c->start_frame < 0 || c->last_frame < c->start_frame)
    return fail(P64GPU_E_INVALID, "p64seq config out of range");
  p64seq *s = (p64seq *)calloc(1, sizeof *s);
  if (!s) return fail(P64GPU_E_NOMEM, "p64seq: calloc");
  s->c = *c;
  if ((st = p64s_geometry(c->format, &s->w, &s->h, &s->ngob))) {
    free(s);
    return st;
  }
  s->nmb = s->ngob * 33;
  s->pic = (size_t)s->w * s->h * 3 / 2;
  const size_t nmb = (size_t)s->nmb;
  if ((st = p64gpu_set_device(c->device))) goto bad;
  if ((st = p64gpu_alloc((void **)&s->d_cur, s->pic)) || (st = p64gpu_alloc((void **)&s->d_rec[0], s->pic)) ||
      (st = p64gpu_alloc((void **)&s->d_rec[1], s->pic)) || (st = p64gpu_alloc((void **)&s->d_li, nmb)) ||
      (st = p64gpu_alloc((void **)&s->d_q, nmb)) || (st = p64gpu_alloc((void **)&s->d_mask, nmb)) ||
      (st = p64gpu_alloc((void **)&s->d_coef, nmb * 384 * sizeof(int16_t))) ||
      (st = p64gpu_alloc((void **)&s->d_mb, nmb * sizeof(p64_mb_rec))) ||
      (st = p64gpu_alloc((void **)&s->d_lists, nmb * sizeof(int32_t))) ||
      (st = p64gpu_alloc((void **)&s->d_ov, nmb)) ||
      (st = p64gpu_alloc((void **)&s->d_me, nmb * sizeof(p64_me_rec))))
    goto bad;
  s->h_coef = (int16_t *)calloc(nmb * 384, sizeof(int16_t));
  s->h_mb = (p64_mb_rec *)calloc(nmb, sizeof(p64_mb_rec));
  s->h_li_old = (uint8_t *)calloc(nmb, 1);
  s->h_li = (uint8_t *)calloc(nmb, 1);
  s->h_mask = (uint8_t *)calloc(nmb, 1);
  s->h_q = (uint8_t *)calloc(nmb, 1);
  s->h_lists = (int32_t *)calloc(nmb, sizeof(int32_t));
  s->h_ov = (int8_t *)calloc(nmb, 1);
  s->h_me = (p64_me_rec *)calloc(nmb, sizeof(p64_me_rec));
  uint8_t *zero = (uint8_t *)calloc(s->pic, 1);
  if (!s->h_coef || !s->h_mb || !s->h_li_old || !s->h_li || !s->h_mask || !s->h_q || !s->h_lists ||
      !s->h_ov || !s->h_me || !zero) {
    free(zero);
    st = fail(P64GPU_E_NOMEM, "p64seq: host buffers");
    goto bad;
  }
  for (int g = 0; g < s->ngob; g++)
    for (int m = 0; m < 33; m++) s->h_lists[g * 33 + m] = p64s_raster_mb(c->format, g, m);
  /* InitFS + ClearFS (p64.c:531-534): both frame stores start at zero;
   * LastIntra starts at zero (calloc, p64.c:1522-1526) */
  if ((st = p64gpu_copy_to_device(s->d_rec[0], zero, s->pic, NULL)) ||
      (st = p64gpu_copy_to_device(s->d_rec[1], zero, s->pic, NULL)) ||
      (st = p64gpu_copy_to_device(s->d_li, zero, nmb, NULL)) ||
      (st = p64gpu_copy_to_device(s->d_lists, s->h_lists, nmb * sizeof(int32_t), NULL)) ||
      (st = p64gpu_synchronize(NULL))) {
    free(zero);
    goto bad;
  }
  free(zero);
  if ((st = p64s_writer_open(&s->wr))) goto bad;
  if (!c->host_vlc) {
    s->vstride = (p64gpu_vlc_max_bytes(s->w, s->h) + 3) & ~(int64_t)3;
    if ((st = p64gpu_alloc((void **)&s->d_vout, (size_t)s->vstride)) ||
        (st = p64gpu_alloc((void **)&s->d_vgq, 12)) || (st = p64gpu_alloc((void **)&s->d_vphase, 1)) ||
        (st = p64gpu_alloc((void **)&s->d_vbits, 4)) || (st = p64gpu_alloc((void **)&s->d_vtr, 4)) ||
        (st = p64gpu_alloc((void **)&s->d_vscratch, 6 * nmb * sizeof(uint32_t))))
      goto bad;
    if (!(s->h_vout = (uint8_t *)malloc((size_t)s->vstride))) {
      st = fail(P64GPU_E_NOMEM, "p64seq: host buffers");
      goto bad;
    }
  }

  /* p64EncodeSequence p64.c:566-595 */
  s->current_frame = c->start_frame;
  int rate = c->rate, iq = c->quant;
  if (c->file_size_bits)
    rate = idiv(idiv(imul(c->file_size_bits, c->frame_rate), c->frame_rate_div),
                imul(c->frame_skip, c->last_frame - c->start_frame + 1));
  if (rate) {
    s->qdfact = rate / 320;
    s->qoffs = 1;
    if (s->qdfact == 0) { /* the reference divides by QDFact (p64.c:463) */
      st = fail(P64GPU_E_INVALID, "rate %d below 320 bits/s (QDFact would be 0)", rate);
      goto bad;
    }
    if (!iq) {
      iq = 10000000 / rate;
      if (iq > 31) iq = 31;
      else if (iq < 1) iq = 1;
    }
  }
  if (!iq) iq = 8; /* DEFAULT_QUANTIZATION p64.c:145 */
  s->rate = rate;
  if (!rate) s->qdfact = s->qoffs = 1; /* p64.c:137-138 */
  s->gquant = s->mquant = iq;        /* GQuant = MQuant = InitialQuant p64.c:589 */
  s->prog = (p64prog *)c->program;
  s->cur = 0;
  *out = s;
  return 0;
bad:
  p64seq_close(s);
  return st;
}

int p64seq_more(const p64seq *s) { return s && !s->finished && s->current_frame <= s->c.last_frame; }

p64s_writer *p64seq_writer(p64seq *s) { return s ? s->wr : NULL; }

static int64_t bits_written(const p64seq *s) {
  int64_t b;
  p64s_writer_data(s->wr, NULL, &b);
  return b;
}

/* BufferContents() p64.c:233-236 at GOB g, MDU m */
static int64_t buffer_contents(const p64seq *s, int g, int m) {
  const int32_t budget = idiv(imul(imul(g * 33 + m, s->rate), s->c.frame_skip),
                              idiv(imul(s->ngob * 33, s->c.frame_rate), s->c.frame_rate_div));
  return bits_written(s) + s->buffer_offset - budget;
}

/* (int) of a double as the reference's casts do on x86 (out of range -> INT_MIN) */
static int dtoi(double v) { return (v > -2147483649.0 && v < 2147483648.0) ? (int)v : INT32_MIN; }
static int clampq(int q) { return q < 1 ? 1 : q > 31 ? 31 : q; }

/* CallOracle p64.c:489-515: the encoder state into Memory[1..14], then run
 * program v.  k = the macroblock at (CurrentGOB, CurrentMDU). */
static int call_program(p64seq *s, int v, int mtype, int k, int64_t bc) {
  double *m = p64prog_memory(s->prog);
  const p64_me_rec *e = &s->h_me[k];
  m[P64PROG_GQUANT] = s->gquant;
  m[P64PROG_MQUANT] = s->mquant;
  m[P64PROG_MQUANTENABLE] = 0; /* MQuantEnable: never set (OracleMQuantEnable is 0) */
  m[P64PROG_MTYPE] = mtype;
  m[P64PROG_BD] = e->sad0;
  m[P64PROG_DBD] = e->sad;
  m[P64PROG_VAROR] = e->varor;
  m[P64PROG_VAR] = e->var;
  m[P64PROG_MWOR] = e->mwor;
  m[P64PROG_RATE] = s->rate;
  m[P64PROG_BUFFERSIZE] = s->rate / 4;
  m[P64PROG_BUFFERCONTENTS] = (double)(int)bc;
  m[P64PROG_QDFACT] = s->qdfact;
  m[P64PROG_QOFFS] = s->qoffs;
  return p64prog_execute(s->prog, v);
}

/* ExecuteQuantization p64.c:458-481 at GOB g, MDU m: the new GQUANT (the
 * MQUANT half has no effect: OracleMQuantEnable is never set) */
static int execute_quantization(p64seq *s, int g, int m, int *gq) {
  const int64_t bc = buffer_contents(s, g, m);
  if (s->c.verbose) printf("BufferContents: %d  New Q1: %d\n", (int)bc, s->gquant);
  int q = (int)bc / s->qdfact + s->qoffs;
  if (s->prog) {
    const int st = call_program(s, 1, s->mtype, s->h_lists[g * 33 + m], bc);
    if (st) return st;
    q = dtoi(p64prog_memory(s->prog)[P64PROG_GQUANT]);
  }
  *gq = clampq(q);
  return 0;
}

/* the MTYPE decision of p64EncodeGOB p64.c:734-756 (suggested type for -o) */
static int decide(const p64_me_rec *e) {
  const double x = (double)e->sad0 / 256, y = (double)e->sad / 256;
  if (e->var < 64 || e->varor > e->var) {
    if (x < 1.0 || (x < 3.0 && y > x * 0.5) || y > x / 1.1) return 2;
    return e->var < 6.0 ? 5 : 8;
  }
  return 0;
}

static const unsigned char QUANT_MT[10] = {0, 1, 0, 1, 0, 0, 1, 0, 0, 1};

/* program 0 for macroblock k (non-first pictures): the MTYPE it stores */
static int program_mtype(p64seq *s, int k, int64_t bc, int *mt) {
  const int st = call_program(s, 0, decide(&s->h_me[k]), k, bc);
  if (st) return st;
  const int v = dtoi(p64prog_memory(s->prog)[P64PROG_MTYPE]);
  if (v < 0 || v > 9) return fail(P64GPU_E_INVALID, "program 0 chose MTYPE %d (not 0..9)", v);
  *mt = v;
  return 0;
}

static p64gpu_encode_args picture_args(p64seq *s, int intra) {
  p64gpu_encode_args a;
  memset(&a, 0, sizeof a);
  a.width = s->w;
  a.height = s->h;
  a.nframes = 1;
  a.intra = intra;
  a.quant = s->gquant;
  a.me_mode = s->c.me_mode;
  a.search_limit = s->c.search_limit;
  a.frame_stride = (int64_t)s->pic;
  a.cur = s->d_cur;
  a.ref = s->d_rec[s->cur ^ 1];
  a.recon = s->d_rec[s->cur];
  a.last_intra = s->d_li;
  a.coef = s->d_coef;
  a.mb = s->d_mb;
  return a;
}

/* device -> host copy of the records of GOB g (three runs of 11 MBs for
 * CIF/NTSC, one run of 33 for QCIF) */
static int fetch_gob(p64seq *s, int g) {
  int st;
  const int runs = s->c.format == P64S_QCIF ? 1 : 3, len = 33 / runs;
  for (int r = 0; r < runs; r++) {
    const int k = s->h_lists[g * 33 + r * len];
    if ((st = p64gpu_copy_to_host(s->h_mb + k, s->d_mb + k, len * sizeof(p64_mb_rec), NULL)) ||
        (st = p64gpu_copy_to_host(s->h_coef + (size_t)k * 384, s->d_coef + (size_t)k * 384,
                                  (size_t)len * 384 * sizeof(int16_t), NULL)))
      return st;
  }
  return p64gpu_synchronize(NULL);
}

static int fetch_all(p64seq *s) {
  int st;
  const size_t nmb = (size_t)s->nmb;
  if ((st = p64gpu_copy_to_host(s->h_mb, s->d_mb, nmb * sizeof(p64_mb_rec), NULL)) ||
      (st = p64gpu_copy_to_host(s->h_coef, s->d_coef, nmb * 384 * sizeof(int16_t), NULL)))
    return st;
  return p64gpu_synchronize(NULL);
}

/* buffer overflow (p64.c:776-783): MTYPE 4 at (0,0), no coefficients; the
 * GPU's reconstruction and LastIntra of the MB are redone after the picture */
static void overflow_mb(p64seq *s, int k) {
  s->h_mb[k].mtype = 4;
  s->h_mb[k].cbp = 0x3f;
  s->h_mb[k].mvx = s->h_mb[k].mvy = 0;
  memset(s->h_coef + (size_t)k * 384, 0, 384 * sizeof(int16_t));
  s->h_mask[k] = 1;
  s->pic_ovfl++;
}

static int write_mb(p64seq *s, int m, int k) {
  const int st = p64s_write_mb(s->wr, m, &s->h_mb[k], s->h_coef + (size_t)k * 384, s->mquant);
  if (st) return st;
  s->hist[s->h_mb[k].mtype]++;
  s->mtype = s->h_mb[k].mtype; /* the MType global after the macroblock */
  return 0;
}

static int fix_overflows(p64seq *s, const p64gpu_encode_args *a) {
  int st;
  const size_t nmb = (size_t)s->nmb;
  if (!s->pic_ovfl) return 0;
  if ((st = p64gpu_copy_to_device(s->d_mb, s->h_mb, nmb * sizeof(p64_mb_rec), NULL)) ||
      (st = p64gpu_copy_to_device(s->d_mask, s->h_mask, nmb, NULL)) ||
      (st = p64gpu_copy_to_device(s->d_q, s->h_q, nmb, NULL)) ||
      (st = p64gpu_decode_recon(s->w, s->h, 1, (int64_t)s->pic, a->ref, a->recon, s->d_coef, s->d_mb,
                                s->d_q, s->d_mask, NULL)) ||
      (st = p64gpu_copy_to_host(s->h_li, s->d_li, nmb, NULL)) || (st = p64gpu_synchronize(NULL)))
    return st;
  for (size_t k = 0; k < nmb; k++)
    if (s->h_mask[k]) s->h_li[k] = (uint8_t)(s->h_li_old[k] + 1);
  if ((st = p64gpu_copy_to_device(s->d_li, s->h_li, nmb, NULL)) || (st = p64gpu_synchronize(NULL)))
    return st;
  s->novfl += s->pic_ovfl;
  return 0;
}

/* fixed quantiser, no program: one launch for the picture, then the VLC */
static int encode_batch(p64seq *s, p64gpu_encode_args *a) {
  int st;
  if (s->d_vout) { /* GPU entropy coding: only the picture's bits cross PCIe */
    const int phase = p64s_writer_phase(s->wr);
    const int32_t tr = s->current_frame % 32;
    const uint8_t ph = (uint8_t)phase;
    uint8_t gq[12];
    uint32_t bits = 0;
    memset(gq, s->gquant, sizeof gq);
    p64gpu_vlc_args v;
    memset(&v, 0, sizeof v);
    v.width = s->w;
    v.height = s->h;
    v.nframes = 1;
    v.mb = s->d_mb;
    v.coef = s->d_coef;
    v.gquant = s->d_vgq;
    v.tr = s->d_vtr;
    v.phase = s->d_vphase;
    v.out = s->d_vout;
    v.out_stride = s->vstride;
    v.bits = s->d_vbits;
    v.scratch = s->d_vscratch;
    if ((st = p64gpu_encode_frames(a, NULL)) || (st = p64gpu_copy_to_device(s->d_vgq, gq, 12, NULL)) ||
        (st = p64gpu_copy_to_device(s->d_vtr, &tr, 4, NULL)) ||
        (st = p64gpu_copy_to_device(s->d_vphase, &ph, 1, NULL)) || (st = p64gpu_vlc_pictures(&v, NULL)) ||
        (st = p64gpu_copy_to_host(&bits, s->d_vbits, 4, NULL)) ||
        (st = p64gpu_copy_to_host(s->h_mb, s->d_mb, (size_t)s->nmb * sizeof(p64_mb_rec), NULL)) ||
        (st = p64gpu_synchronize(NULL)))
      return st;
    if (bits == 0xFFFFFFFFu) return fail(P64GPU_E_STREAM, "GPU entropy coder rejected the picture");
    if ((st = p64gpu_copy_to_host(s->h_vout, s->d_vout, (bits + 7) / 8, NULL)) ||
        (st = p64gpu_synchronize(NULL)) || (st = p64s_write_bits(s->wr, s->h_vout, bits, phase)))
      return st;
    for (int k = 0; k < s->nmb; k++) s->hist[s->h_mb[k].mtype]++;
    s->mtype = s->h_mb[s->h_lists[s->nmb - 1]].mtype;
    return 0;
  }
  if ((st = p64s_write_picture_header(s->wr, s->c.format, s->current_frame % 32))) return st;
  if ((st = p64gpu_encode_frames(a, NULL)) || (st = fetch_all(s))) return st;
  for (int g = 0; g < s->ngob; g++) {
    if ((st = p64s_write_gob_header(s->wr, g, s->gquant))) return st;
    for (int m = 0; m < 33; m++)
      if ((st = write_mb(s, m, s->h_lists[g * 33 + m]))) return st;
  }
  return 0;
}

/* rate control, no program: GOB by GOB */
static int encode_per_gob(p64seq *s, p64gpu_encode_args *a, int first) {
  int st;
  for (int g = 0; g < s->ngob; g++) {
    if (!first && (st = execute_quantization(s, g, 0, &s->gquant))) return st; /* p64.c:697-701 */
    a->quant = s->gquant;
    if ((st = p64s_write_gob_header(s->wr, g, s->gquant)) ||
        (st = p64gpu_encode_mb_list(a, s->d_lists + g * 33, 33, NULL)) || (st = fetch_gob(s, g)))
      return st;
    for (int m = 0; m < 33; m++) {
      const int k = s->h_lists[g * 33 + m];
      /* the MDU-level ExecuteQuantization (p64.c:718-728) changes nothing
       * here (it could only enable MQUANT, which the reference never does);
       * only its -v line is reproduced */
      if (s->c.verbose && m && !(m % 11) && !first)
        printf("BufferContents: %d  New Q1: %d\n", (int)buffer_contents(s, g, m), s->gquant);
      s->h_q[k] = (uint8_t)s->gquant;
      if (buffer_contents(s, g, m) > s->rate / 4) overflow_mb(s, k);
      if ((st = write_mb(s, m, k))) return st;
    }
  }
  return 0;
}

/* -o program, decisions independent of the bits written: program 0 for every
 * macroblock in stream order, then one launch with the chosen types */
static int encode_program_batch(p64seq *s, p64gpu_encode_args *a) {
  int st;
  const size_t nmb = (size_t)s->nmb;
  uint8_t gq[12];
  const int64_t bc = buffer_contents(s, 0, 0);
  for (int g = 0; g < s->ngob; g++) {
    gq[g] = (uint8_t)s->gquant;
    for (int m = 0; m < 33; m++) {
      const int k = s->h_lists[g * 33 + m];
      int mt;
      if ((st = program_mtype(s, k, bc, &mt))) return st;
      if (s->h_li_old[k] > 131) mt = 0; /* p64.c:772-773 */
      if (QUANT_MT[mt]) s->gquant = s->mquant; /* ReadCompressMDU p64.c:835-840 */
      s->h_ov[k] = (int8_t)mt;
      s->h_q[k] = (uint8_t)(QUANT_MT[mt] ? s->mquant : s->gquant);
    }
  }
  a->mtype_override = s->d_ov;
  a->quant_mb = s->d_q;
  if ((st = p64gpu_copy_to_device(s->d_ov, s->h_ov, nmb, NULL)) ||
      (st = p64gpu_copy_to_device(s->d_q, s->h_q, nmb, NULL)) || (st = p64gpu_encode_frames(a, NULL)) ||
      (st = fetch_all(s)))
    return st;
  for (int g = 0; g < s->ngob; g++) {
    if ((st = p64s_write_gob_header(s->wr, g, gq[g]))) return st;
    for (int m = 0; m < 33; m++)
      if ((st = write_mb(s, m, s->h_lists[g * 33 + m]))) return st;
  }
  return 0;
}

/* -o program whose decisions depend on the bits written (BUFFERCONTENTS, or
 * rate control with program 1 between macroblocks): macroblock by macroblock
 * in stream order, the exact order of p64EncodeGOB p64.c:692-786 */
static int encode_program_serial(p64seq *s, p64gpu_encode_args *a, int first) {
  int st;
  a->mtype_override = s->d_ov;
  a->quant_mb = s->d_q;
  for (int g = 0; g < s->ngob; g++) {
    if (s->rate && !first && (st = execute_quantization(s, g, 0, &s->gquant))) return st;
    if ((st = p64s_write_gob_header(s->wr, g, s->gquant))) return st;
    s->mtype = 0; /* p64.c:716 */
    for (int m = 0; m < 33; m++) {
      const int k = s->h_lists[g * 33 + m];
      int mt = 0, unused;
      if (s->rate && m && !(m % 11) && !first && (st = execute_quantization(s, g, m, &unused)))
        return st;
      if (!first && (st = program_mtype(s, k, buffer_contents(s, g, m), &mt))) return st;
      if (s->h_li_old[k] > 131) mt = 0;
      if (s->rate && buffer_contents(s, g, m) > s->rate / 4) {
        s->h_q[k] = (uint8_t)s->gquant;
        overflow_mb(s, k);
      } else {
        if (QUANT_MT[mt]) s->gquant = s->mquant;
        const int8_t ov = (int8_t)mt;
        const uint8_t q = (uint8_t)(QUANT_MT[mt] ? s->mquant : s->gquant);
        s->h_q[k] = q;
        if ((st = p64gpu_copy_to_device(s->d_ov + k, &ov, 1, NULL)) ||
            (st = p64gpu_copy_to_device(s->d_q + k, &q, 1, NULL)) ||
            (st = p64gpu_encode_mb_list(a, s->d_lists + g * 33 + m, 1, NULL)) ||
            (st = p64gpu_copy_to_host(s->h_mb + k, s->d_mb + k, sizeof(p64_mb_rec), NULL)) ||
            (st = p64gpu_copy_to_host(s->h_coef + (size_t)k * 384, s->d_coef + (size_t)k * 384,
                                      384 * sizeof(int16_t), NULL)) ||
            (st = p64gpu_synchronize(NULL)))
          return st;
      }
      if ((st = write_mb(s, m, k))) return st;
    }
  }
  return 0;
}

int p64seq_encode(p64seq *s, const uint8_t *picture) {
  int st;
  if (!s || !picture) return fail(P64GPU_E_INVALID, "p64seq_encode: NULL argument");
  if (!p64seq_more(s)) return fail(P64GPU_E_INVALID, "p64seq_encode past the last frame");
  const int first = s->current_frame == s->c.start_frame;
  const size_t nmb = (size_t)s->nmb;
  p64gpu_encode_args a = picture_args(s, first);
  s->pic_ovfl = 0;
  memset(s->h_mask, 0, nmb);
  if ((st = p64gpu_copy_to_device(s->d_cur, picture, s->pic, NULL))) return st;
  if ((st = p64gpu_copy_to_host(s->h_li_old, s->d_li, nmb, NULL)) || (st = p64gpu_synchronize(NULL)))
    return st;
  /* encode_batch writes (or has the GPU write) its own picture header */
  if ((s->rate || (s->prog && !first)) &&
      (st = p64s_write_picture_header(s->wr, s->c.format, s->current_frame % 32)))
    return st;

  if (s->prog && !first) { /* GlobalMC (io.c:129): the records program 0 reads */
    if ((st = p64gpu_motion_estimation(s->w, s->h, 1, (int64_t)s->pic, a.ref, s->d_cur, s->c.me_mode,
                                       s->c.search_limit, s->d_me, NULL)) ||
        (st = p64gpu_copy_to_host(s->h_me, s->d_me, nmb * sizeof(p64_me_rec), NULL)) ||
        (st = p64gpu_synchronize(NULL)))
      return st;
  }
  if (!s->prog)
    st = s->rate ? encode_per_gob(s, &a, first) : encode_batch(s, &a);
  else if (!s->rate && (first || !p64prog_reads(s->prog, 0, P64PROG_BUFFERCONTENTS)))
    st = first ? encode_batch(s, &a) : encode_program_batch(s, &a);
  else
    st = encode_program_serial(s, &a, first);
  if (st || (st = fix_overflows(s, &a))) return st;

  /* p64EncodeFrame p64.c:653-682 */
  const int64_t x = bits_written(s);
  s->last_bits = x - s->total_bits;
  s->total_bits = x;
  if (s->rate) {
    if (first) {
      s->first_frame_bits = s->total_bits;
      /* CurrentGOB = NumberGOB, CurrentMDU = 0 once the GOB loop is done */
      s->buffer_offset = (int)((s->rate / 4) / 2 - buffer_contents(s, s->ngob, 0));
    }
    s->buffer_offset -= idiv(imul(imul(s->rate, s->c.frame_skip), s->c.frame_rate_div), s->c.frame_rate);
  } else if (first) {
    s->first_frame_bits = s->total_bits;
  }
  s->cur ^= 1; /* SwapFS(CFS, OFS) p64.c:661 */
  s->frames++;
  s->current_frame += s->c.frame_skip;
  return 0;
}

int p64seq_finish(p64seq *s) {
  if (!s) return fail(P64GPU_E_INVALID, "p64seq_finish: NULL");
  if (s->finished) return fail(P64GPU_E_INVALID, "p64seq_finish called twice");
  int f = s->current_frame; /* p64.c:606-608 */
  if (f > s->c.last_frame + 1) f = s->c.last_frame + 1;
  s->finished = 1;
  return p64s_write_end(s->wr, s->c.format, f % 32);
}

int p64seq_get_stats(const p64seq *s, p64seq_stats *st) {
  if (!s || !st) return fail(P64GPU_E_INVALID, "p64seq_get_stats: NULL");
  memset(st, 0, sizeof *st);
  st->frames = s->frames;
  st->next_frame = s->current_frame;
  st->gquant = s->gquant;
  st->rate = s->rate;
  st->bits = bits_written(s);
  st->last_bits = s->last_bits;
  st->first_frame_bits = s->first_frame_bits;
  st->overflows = s->novfl;
  memcpy(st->mtype_hist, s->hist, sizeof s->hist);
  return 0;
}
