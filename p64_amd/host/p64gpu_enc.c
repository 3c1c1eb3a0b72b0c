/*
 * p64gpu_enc.c -- C host driver over the p64gpu C ABI.
 *
 * The host loop of the reference encoder (p64EncodeSequence p64.c:524 /
 * p64EncodeFrame p64.c:622) with the per-macroblock compute replaced by
 * p64gpu_encoder_frame(): y4m input (420jpeg), first picture intra, each later
 * picture predicted from the device-resident reconstruction of the previous one.
 *
 * Output (-s FILE): per picture, a record block
 *     "P64R" int32 frame, int32 nmb, nmb x p64_mb_rec, nmb x 384 int16 levels
 * -- the MTYPE/CBP/MV and zigzagged levels the reference's WriteMDU codes
 * (p64.c:922-961).  The entropy coder (codec.c/marker.c) is the next row
 *  and is not part of this driver yet.
 *
 * Usage: p64gpu_enc [-a first] [-b last] [-q quant] [-i searchlimit]
 *                   [-full|-tss] [-d device] [-s out.rec] input.y4m
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/p64gpu.h"

static int read_y4m_header(FILE *f, int *w, int *h) {
  char line[512];
  if (!fgets(line, sizeof line, f) || strncmp(line, "YUV4MPEG2", 9)) return -1;
  *w = *h = 0;
  for (char *t = strtok(line, " \n"); t; t = strtok(NULL, " \n")) {
    if (t[0] == 'W') *w = atoi(t + 1);
    if (t[0] == 'H') *h = atoi(t + 1);
    if (t[0] == 'C' && strncmp(t, "C420", 4)) return -2; /* 4:2:0 only */
  }
  return (*w > 0 && *h > 0) ? 0 : -1;
}

static int read_frame(FILE *f, unsigned char *buf, size_t n) {
  char line[256];
  if (!fgets(line, sizeof line, f)) return 0;
  if (strncmp(line, "FRAME", 5)) return -1;
  return fread(buf, 1, n, f) == n ? 1 : -1;
}

int main(int argc, char **argv) {
  int first = 0, last = 1 << 30, quant = 8, sl = 15, mode = P64GPU_ME_TSS, device = 0;
  const char *in = NULL, *out = NULL;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "-a") && i + 1 < argc) first = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-b") && i + 1 < argc) last = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-q") && i + 1 < argc) quant = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-i") && i + 1 < argc) sl = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-d") && i + 1 < argc) device = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-s") && i + 1 < argc) out = argv[++i];
    else if (!strcmp(argv[i], "-full")) mode = P64GPU_ME_FULL;
    else if (!strcmp(argv[i], "-tss")) mode = P64GPU_ME_TSS;
    else if (argv[i][0] != '-') in = argv[i];
    else {
      fprintf(stderr, "unknown option %s\n", argv[i]);
      return 1;
    }
  }
  if (!in) {
    fprintf(stderr, "usage: %s [-a n] [-b n] [-q q] [-i sl] [-full|-tss] [-d dev] [-s out] in.y4m\n",
            argv[0]);
    return 1;
  }
  /* BoundValue semantics of the reference CLI (p64.c:341-352) */
  if (quant < 1) quant = 1;
  if (quant > 31) quant = 31;
  if (sl < 1) sl = 1;
  if (sl > 31) sl = 31;
  FILE *f = fopen(in, "rb");
  int w, h;
  if (!f || read_y4m_header(f, &w, &h)) {
    fprintf(stderr, "cannot read y4m %s\n", in);
    return 1;
  }
  size_t pic = (size_t)w * h * 3 / 2;
  int nmb = (w / 16) * (h / 16);
  unsigned char *buf = malloc(pic);
  int16_t *coef = malloc((size_t)nmb * 384 * sizeof(int16_t));
  p64_mb_rec *mb = malloc((size_t)nmb * sizeof(p64_mb_rec));
  p64gpu_encoder *enc = NULL;
  int s = p64gpu_encoder_open(device, w, h, mode, sl, &enc);
  if (s) {
    fprintf(stderr, "p64gpu_encoder_open: %s (%s)\n", p64gpu_strerror(s), p64gpu_last_error());
    return 2;
  }
  FILE *o = out ? fopen(out, "wb") : NULL;
  int hist[10] = {0}, coded = 0;
  for (int fr = 0; fr <= last; fr++) {
    int r = read_frame(f, buf, pic);
    if (r <= 0) break;
    if (fr < first) continue; /* -a seeks (p64.c:562-565) */
    s = p64gpu_encoder_frame(enc, buf, fr == first, quant, NULL, coef, mb, NULL, NULL);
    if (s) {
      fprintf(stderr, "frame %d: %s (%s)\n", fr, p64gpu_strerror(s), p64gpu_last_error());
      return 2;
    }
    for (int k = 0; k < nmb; k++) hist[mb[k].mtype]++;
    if (o) {
      int hdr[2] = {fr, nmb};
      fwrite("P64R", 1, 4, o);
      fwrite(hdr, sizeof(int), 2, o);
      fwrite(mb, sizeof(p64_mb_rec), nmb, o);
      fwrite(coef, sizeof(int16_t), (size_t)nmb * 384, o);
    }
    printf("END>Frame: %d\n", fr);
    coded++;
  }
  printf("frames %d  MTYPE histogram:", coded);
  for (int k = 0; k < 10; k++) printf(" %d", hist[k]);
  printf("\n");
  p64gpu_encoder_close(enc);
  if (o) fclose(o);
  fclose(f);
  free(buf);
  free(coef);
  free(mb);
  return 0;
}
