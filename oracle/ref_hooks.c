/*
 * ref_hooks.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Link-time hooks around the UNMODIFIED PVRG-P64 reference encoder, built from
 * /root/reference sources by oracle/Makefile into oracle/_ref/p64hook.  They let
 * the fixture generator (tests/golden/make_golden.py) observe the reference's
 * per-macroblock state without editing a single reference line:
 *
 *   --wrap=MotionEstimation  (caller io.c:129-133 GlobalMC -> me.c:340)
 *       P64REF_ME=full  : run the dormant brute-force FastBME (me.c:187-246)
 *                         for every MB instead of the shipped StepBME (me.c:352),
 *                         i.e. the one-line swap SURVEY.md 0.2 describes.
 *       P64REF_ME=none  : no search, zero records (CPU-baseline timing of the
 *                         reference's intra coding under `-o` with a program
 *                         that keeps every MB intra: the records are unused).
 *       otherwise       : call the real MotionEstimation (TSS, me.c:255-330).
 *       Either way, dump the Me* record arrays (me.c:49-60).
 *   --wrap=WriteMBHeader     (caller p64.c:930 WriteMDU -> marker.c:288)
 *       dump MType/CBP/MVDH/MVDV/UseQuant and inputbuf[0..5][64] exactly as
 *       ReadCompressMDU (p64.c:823-913) left them, before the header writer
 *       zeroes MVDH/MVDV for non-MC types (marker.c:335-338).
 *   --wrap=WritePictureHeader (callers p64.c:637 and p64.c:601)
 *       dump CFS->fs[0..2] = reconstruction of the previous frame
 *       (SwapFS p64.c:661 has already run).
 *
 * inputbuf is `static` in p64.c:167; oracle/Makefile globalises its symbol in
 * the reference object with objcopy.  me.c's static VAR/VAROR/MWOR (me.c:45-47)
 * are renamed refme_* and globalised the same way, so the FULL-mode loop below
 * can read FastBME's statistics.
 *
 * Dump format (little-endian int32 words), file named by P64REF_DUMP:
 *   'E' frame n  then 7*n words: MeX MeY MeVal MeOVal MeVAR MeVAROR MeMWOR
 *   'M' frame gob mdu mtype cbp mvdh mvdv usequant  then 384 words inputbuf
 *   'R' frame w h  then w*h + 2*(w/2*h/2) bytes (Y,U,V), padded to 4 bytes
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "globals.h"

extern int CurrentFrame, CurrentGOB, CurrentMDU, MType, CBP, MVDH, MVDV,
    UseQuant;
extern int inputbuf[10][64]; /* globalised by objcopy */
extern FSTORE *CFS;
extern int MeX[], MeY[], MeVal[], MeOVal[], MeVAR[], MeVAROR[], MeMWOR[];
extern int MeN, MX, MY, MV, OMV;
extern int refme_VAR, refme_VAROR, refme_MWOR; /* renamed me.c statics */
extern void FastBME(int, int, MEM *, int, int, MEM *);

void __real_MotionEstimation(MEM *, MEM *);
void __real_WriteMBHeader(void);
void __real_WritePictureHeader(void);

static FILE *dumpf;
static int dump_tried;

static FILE *dump_file(void) {
  if (!dump_tried) {
    const char *p = getenv("P64REF_DUMP");
    dump_tried = 1;
    if (p && *p) {
      dumpf = fopen(p, "wb");
      if (!dumpf) {
        fprintf(stderr, "ref_hooks: cannot open %s\n", p);
        exit(99);
      }
    }
  }
  return dumpf;
}

static void put_words(const int *w, int n) { fwrite(w, sizeof(int), n, dumpf); }

void __wrap_MotionEstimation(MEM *pmem, MEM *fmem) {
  const char *mode = getenv("P64REF_ME");
  if (mode && !strcmp(mode, "full")) {
    int x, y;
    for (MeN = 0, y = 0; y < fmem->height; y += 16)
      for (x = 0; x < fmem->width; x += 16) {
        FastBME(x, y, pmem, x, y, fmem);
        MeVAR[MeN] = refme_VAR;
        MeVAROR[MeN] = refme_VAROR;
        MeMWOR[MeN] = refme_MWOR;
        MeX[MeN] = MX;
        MeY[MeN] = MY;
        MeVal[MeN] = MV;
        MeOVal[MeN] = OMV;
        MeN++;
      }
  } else if (mode && !strcmp(mode, "none")) {
    const int n = (fmem->width / 16) * (fmem->height / 16);
    for (MeN = 0; MeN < n; MeN++)
      MeX[MeN] = MeY[MeN] = MeVal[MeN] = MeOVal[MeN] = MeVAR[MeN] = MeVAROR[MeN] = MeMWOR[MeN] = 0;
  } else {
    __real_MotionEstimation(pmem, fmem);
  }
  if (dump_file()) {
    int hdr[3] = {'E', CurrentFrame, MeN};
    put_words(hdr, 3);
    put_words(MeX, MeN);
    put_words(MeY, MeN);
    put_words(MeVal, MeN);
    put_words(MeOVal, MeN);
    put_words(MeVAR, MeN);
    put_words(MeVAROR, MeN);
    put_words(MeMWOR, MeN);
  }
}

void __wrap_WriteMBHeader(void) {
  if (dump_file()) {
    int hdr[9] = {'M', CurrentFrame, CurrentGOB, CurrentMDU, MType,
                  CBP, MVDH,         MVDV,       UseQuant};
    put_words(hdr, 9);
    put_words(&inputbuf[0][0], 6 * 64);
  }
  __real_WriteMBHeader();
}

void __wrap_WritePictureHeader(void) {
  if (dump_file() && CFS) {
    int c, w = CFS->fs[0]->mem->width, h = CFS->fs[0]->mem->height;
    int hdr[4] = {'R', CurrentFrame, w, h};
    long total = 0;
    put_words(hdr, 4);
    for (c = 0; c < 3; c++) {
      MEM *m = CFS->fs[c]->mem;
      fwrite(m->data, 1, (size_t)m->width * m->height, dumpf);
      total += (long)m->width * m->height;
    }
    while (total & 3) {
      fputc(0, dumpf);
      total++;
    }
  }
  __real_WritePictureHeader();
}

/* Flush on exit: the reference calls exit() from main (p64.c:448). */
static void close_dump(void) __attribute__((destructor));
static void close_dump(void) {
  if (dumpf) fclose(dumpf);
}
