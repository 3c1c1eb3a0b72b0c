/*
 * p64seq.h -- the reference encoder's sequence loop over the GPU hot path
 * (host C, part of libp64gpu.so).
 *
 *   p64seq_open / p64seq_encode / p64seq_finish
 *       p64EncodeSequence p64.c:524-616, p64EncodeFrame p64.c:622-683 and the
 *       control half of p64EncodeGOB p64.c:692-786: temporal references, the
 *       trailing picture header, and the reference's rate control (-r / -x):
 *       GQUANT per GOB from the buffer fullness (ExecuteQuantization
 *       p64.c:458-481, BufferContents p64.c:233-236) and MTYPE 4 with a zero
 *       vector for every macroblock met while the buffer overflows
 *       (p64.c:776-783), with the buffer bookkeeping after each picture
 *       (p64.c:653-679).  The per-macroblock compute runs on the GPU
 *       (p64gpu_encode_frames / p64gpu_encode_mb_list, one launch per picture,
 *       or per GOB under rate control), the VLC on the host (p64stream.h).
 *
 *   With a -o program (p64prog.h): program 0 picks each macroblock's MTYPE
 *   from the ME statistics (p64.c:761-768) and program 1 the quantiser under
 *   rate control (p64.c:469-474), called in the reference's order.  When
 *   program 0 cannot see the bits written (no BUFFERCONTENTS read, no rate
 *   control) the decisions are made for the whole picture first and the GPU
 *   codes it in one launch; otherwise macroblock by macroblock.  MTYPEs
 *   1/3/6/9 chosen by a program send MQUANT (= the initial quantiser: the
 *   reference never changes MQuant) and make it the GOB quantiser.
 */
#ifndef P64SEQ_H
#define P64SEQ_H

#include <stddef.h>
#include <stdint.h>

#include "p64gpu.h"
#include "p64stream.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int format;            /* P64S_QCIF / P64S_CIF / P64S_NTSC                  */
  int me_mode;           /* P64GPU_ME_TSS (shipped) or P64GPU_ME_FULL          */
  int search_limit;      /* -i, 1..31                                          */
  int quant;             /* -q InitialQuant 1..31, 0 = not given (default 8,
                            or 10000000/rate under rate control)              */
  int rate;              /* -r bits/s, 0 = fixed quantiser                     */
  int file_size_bits;    /* -x: rate = bits*fps/frames, 0 = off                */
  int start_frame;       /* -a                                                 */
  int last_frame;        /* -b                                                 */
  int frame_skip;        /* -k, >= 1                                           */
  int frame_rate;        /* -f numerator   (30000 = reference default)         */
  int frame_rate_div;    /* -f denominator (1001)                              */
  int device;            /* HIP device                                         */
  void *program;         /* p64prog* (-o, p64prog.h) or NULL; borrowed, must
                            outlive the encoder; its top-level settings are the
                            caller's to apply to this config                  */
  int host_vlc;          /* 1: entropy-code on the host (p64stream.h) always;
                            0 (default): pictures coded in one launch are
                            entropy-coded on the GPU (p64gpu_vlc_pictures)     */
  int verbose;           /* -v: print "BufferContents: %d  New Q1: %d" to
                            stdout at every rate-control update, as
                            ExecuteQuantization does (p64.c:466-470)           */
} p64seq_config;

typedef struct {
  int frames;            /* pictures coded                                     */
  int next_frame;        /* CurrentFrame of the next picture                   */
  int gquant;            /* GQuant after the last picture                      */
  int rate;              /* effective rate (after -x), 0 if none               */
  int64_t bits;          /* bits written so far (mwtell)                       */
  int64_t last_bits;     /* bits of the last picture (LastBits)                */
  int64_t first_frame_bits;
  int overflows;         /* NumberOvfl: MBs forced to MTYPE 4                  */
  int mtype_hist[10];    /* MTYPEs written                                     */
} p64seq_stats;

typedef struct p64seq p64seq;
/* Fills defaults the reference uses: search_limit 15, frame_skip 1, frame
 * rate 30000/1001, everything else 0. */
void p64seq_default_config(p64seq_config *cfg);
int p64seq_open(const p64seq_config *cfg, p64seq **out);
void p64seq_close(p64seq *s);
/* 1 while CurrentFrame <= LastFrame (more pictures are expected), else 0. */
int p64seq_more(const p64seq *s);
/* Codes the next picture (host Y|U|V, w*h*3/2 bytes): frame CurrentFrame,
 * intra if it is the first.  Bytes become available through
 * p64seq_writer(). */
int p64seq_encode(p64seq *s, const uint8_t *picture);
/* Writes the trailing picture header and pads the last byte (p64.c:606-610). */
int p64seq_finish(p64seq *s);
p64s_writer *p64seq_writer(p64seq *s);
int p64seq_get_stats(const p64seq *s, p64seq_stats *st);

#ifdef __cplusplus
}
#endif

#endif /* P64SEQ_H */
