/*
 * p64gpu_refshim.c -- link-level drop-in of the GPU hot path into the
 * reference encoder, through the C ABI only (no HIP headers).
 *
 * This is the binding a maintainer of the reference would add: link the
 * reference objects with this file, libp64gpu.so and
 *     -Wl,--wrap=MotionEstimation -Wl,--wrap=ChenDct -Wl,--wrap=ChenIDct
 * and the unmodified p64.c/io.c call the GPU instead of me.c/chendct.c:
 *
 *   MotionEstimation(MEM *pmem, MEM *fmem)   me.c:340, called by GlobalMC
 *       io.c:129-133 once per inter picture -> p64gpu_motion_estimation on the
 *       whole luma plane; results land in the reference's own Me* arrays
 *       (me.c:49-60), which p64EncodeGOB reads (p64.c:734-742).
 *       P64GPU_ME=full selects FastBME semantics (the me.c:351 variant) with the
 *       reference's SearchLimit (-i); default is the shipped StepBME (me.c:352).
 *   ChenDct / ChenIDct (int *in, int *out)   chendct.c:97 / :217, reached
 *       through the UseDct/UseIDct pointers (p64.c:227-231) -> p64gpu_block_op.
 *       One 8x8 block per call: correct, but launch-bound; the frame-batched
 *       p64gpu_encode_frames is the fast path.
 *
 * oracle/Makefile builds oracle/_ref/p64gpu_ref this way; tests/test_gpu_parity.py
 * checks its .p64 output is byte-identical to the stock reference encoder's.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/p64gpu.h"

/* MEM, mem.h:37-42 */
typedef struct {
  int len, width, height;
  unsigned char *data;
} RefMem;

/* reference globals (me.c:49-62) */
extern int MeX[], MeY[], MeVal[], MeOVal[], MeVAR[], MeVAROR[], MeMWOR[];
extern int MeN, SearchLimit;

static void die(const char *what, int s) {
  fprintf(stderr, "p64gpu_refshim: %s: %s (%s)\n", what, p64gpu_strerror(s), p64gpu_last_error());
  exit(6); /* ERROR_UNRECOVERABLE, globals.h:110 */
}

static struct {
  int ready, w, h;
  uint8_t *d_ref, *d_cur;
  p64_me_rec *d_rec, *h_rec;
  int32_t *d_blk;
} S;

static void setup(int w, int h) {
  int s;
  if (S.ready && S.w == w && S.h == h) return;
  if (!S.ready && (s = p64gpu_set_device(0))) die("set_device", s);
  if (S.ready) {
    p64gpu_free(S.d_ref);
    p64gpu_free(S.d_cur);
    p64gpu_free(S.d_rec);
    free(S.h_rec);
  }
  size_t plane = (size_t)w * h, nmb = (size_t)(w / 16) * (h / 16);
  if ((s = p64gpu_alloc((void **)&S.d_ref, plane)) || (s = p64gpu_alloc((void **)&S.d_cur, plane)) ||
      (s = p64gpu_alloc((void **)&S.d_rec, nmb * sizeof(p64_me_rec))))
    die("alloc", s);
  if (!S.d_blk && (s = p64gpu_alloc((void **)&S.d_blk, 64 * sizeof(int32_t)))) die("alloc", s);
  S.h_rec = (p64_me_rec *)malloc(nmb * sizeof(p64_me_rec));
  S.w = w;
  S.h = h;
  S.ready = 1;
}

void __wrap_MotionEstimation(RefMem *pmem, RefMem *fmem) {
  const char *m = getenv("P64GPU_ME");
  int mode = (m && !strcmp(m, "full")) ? P64GPU_ME_FULL : P64GPU_ME_TSS;
  int w = fmem->width, h = fmem->height, s;
  setup(w, h);
  if ((s = p64gpu_copy_to_device(S.d_ref, pmem->data, (size_t)w * h, NULL)) ||
      (s = p64gpu_copy_to_device(S.d_cur, fmem->data, (size_t)w * h, NULL)) ||
      (s = p64gpu_motion_estimation(w, h, 1, (int64_t)w * h, S.d_ref, S.d_cur, mode, SearchLimit,
                                    S.d_rec, NULL)) ||
      (s = p64gpu_copy_to_host(S.h_rec, S.d_rec, (size_t)(w / 16) * (h / 16) * sizeof(p64_me_rec),
                               NULL)) ||
      (s = p64gpu_synchronize(NULL)))
    die("motion estimation", s);
  /* me.c:347-361: raster order, MeN = number of MBs */
  for (MeN = 0; MeN < (w / 16) * (h / 16); MeN++) {
    const p64_me_rec *r = &S.h_rec[MeN];
    MeX[MeN] = r->mx;
    MeY[MeN] = r->my;
    MeVal[MeN] = r->sad;
    MeOVal[MeN] = r->sad0;
    MeVAR[MeN] = r->var;
    MeVAROR[MeN] = r->varor;
    MeMWOR[MeN] = r->mwor;
  }
}

static void block_call(int op, int *in, int *out) {
  int s;
  setup(S.ready ? S.w : 176, S.ready ? S.h : 144);
  if ((s = p64gpu_copy_to_device(S.d_blk, in, 64 * sizeof(int32_t), NULL)) ||
      (s = p64gpu_block_op(op, S.d_blk, S.d_blk, 1, 8, 8, NULL)) ||
      (s = p64gpu_copy_to_host(out, S.d_blk, 64 * sizeof(int32_t), NULL)) ||
      (s = p64gpu_synchronize(NULL)))
    die("block op", s);
}

void __wrap_ChenDct(int *x, int *y) { block_call(P64GPU_OP_DCT, x, y); }
void __wrap_ChenIDct(int *x, int *y) { block_call(P64GPU_OP_IDCT, x, y); }
