/*
 * p64_oracle.h -- TEST INFRASTRUCTURE ONLY: the parity checker.
 *
 * A clean-room CPU restatement of PVRG-P64's per-macroblock encode hot path
 * (SURVEY.md 8(a) rows a1-a17).  Every function cites the reference lines it
 * restates.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library; the product (p64_amd/) never does.
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks every function here
 * against golden vectors captured from the unmodified reference (built from
 * /root/reference by oracle/Makefile into oracle/_ref/, see
 * tests/golden/make_golden.py), and against the short.p64 decode MD5s.
 */
#ifndef P64_ORACLE_H
#define P64_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Record layouts match include/p64gpu.h field for field (checked in tests). */
typedef struct {
  int32_t mx, my;   /* MeX, MeY   (me.c:56-57) */
  int32_t sad;      /* MeVal  = MV  (best SAD)     */
  int32_t sad0;     /* MeOVal = OMV (SAD at (0,0)) */
  int32_t var;      /* MeVAR   (me.c:49)  */
  int32_t varor;    /* MeVAROR (me.c:50)  */
  int32_t mwor;     /* MeMWOR  (me.c:51)  */
} orc_me_rec;

typedef struct {
  int8_t mtype; /* final MType after CBP fallback (p64.c:899-906) */
  int8_t cbp;   /* CBP as written (0x3f for non-CBP types)         */
  int8_t mvx;   /* MVDH transmitted (0 unless MFMType[mtype])      */
  int8_t mvy;   /* MVDV transmitted                                */
} orc_mb_rec;

enum { ORC_ME_TSS = 0, ORC_ME_FULL = 1 };

/* ---- block math (chendct.c, transform.c) ---- */
void orc_chen_dct(const int32_t *in, int32_t *out);  /* chendct.c:97-206  */
void orc_chen_idct(const int32_t *in, int32_t *out); /* chendct.c:217-375 */
void orc_quant_inter(int32_t *m, int dcq, int acq);  /* transform.c:271-309 */
void orc_quant_intra(int32_t *m, int dcq, int acq);  /* transform.c:317-350 */
void orc_iquant_intra(int32_t *m, int dcq, int acq); /* transform.c:359-392 */
void orc_iquant_inter(int32_t *m, int dcq, int acq); /* transform.c:400-451 */
void orc_bound_dct(int32_t *m);                      /* transform.c:460-474 */
void orc_bound_idct(int32_t *m);                     /* transform.c:483-494 */
void orc_bound_quant_flat(int32_t *m);               /* transform.c:502-518 */
void orc_bound_quant(int32_t *m);                    /* transform.c:526-537 */
void orc_zigzag(const int32_t *in, int32_t *out);    /* transform.c:561-568 */
void orc_izigzag(const int32_t *in, int32_t *out);   /* transform.c:546-553 */

/* ---- motion estimation (me.c) ---- */
int orc_sad16(const uint8_t *ref, int ref_stride, const uint8_t *cur,
              int cur_stride);                       /* me.c:92-176 (no early exit) */
void orc_me_mb(const uint8_t *ref_y, const uint8_t *cur_y, int width,
               int height, int x, int y, int mode, int search_limit,
               orc_me_rec *rec);                     /* me.c:187-330 */
void orc_motion_estimation(const uint8_t *ref_y, const uint8_t *cur_y,
                           int width, int height, int mode, int search_limit,
                           orc_me_rec *recs);        /* me.c:340-363 */

/* ---- prediction (io.c) ---- */
void orc_load_filter(const uint8_t *src, int stride, int32_t *out); /* io.c:323-372 */

/* ---- one frame of the closed-loop encoder (p64.c:622-1013) ----
 * cur/ref/recon: planar Y(w*h) U(w/2*h/2) V(w/2*h/2), stride = plane width.
 * ref = previous reconstruction (CFS), recon = new reconstruction (OFS).
 * intra_frame: 1 for the first frame of a sequence (no ME, all MTYPE 0).
 * quant: GQuant (1..31); quant_mb: NULL or per-MB UseQuant override.
 * mtype_override: NULL or per-MB MTYPE (-o interpreter, p64.c:761-768);
 *   entries < 0 mean "no override".  Ignored on intra frames, like p64.c.
 * last_intra: per-MB uint8 counters, in/out (p64.c:772, 909-910).
 * me_in: NULL -> run ME here with (me_mode, search_limit) and write me_out;
 *        else use these records (me_out may be NULL).
 * coef: [nmb][6][64] int16, zigzag order, as left by ReadCompressMDU.
 */
void orc_encode_frame(int width, int height, const uint8_t *cur,
                      const uint8_t *ref, uint8_t *recon, int intra_frame,
                      int quant, const uint8_t *quant_mb,
                      const int8_t *mtype_override, uint8_t *last_intra,
                      int me_mode, int search_limit, const orc_me_rec *me_in,
                      orc_me_rec *me_out, int16_t *coef, orc_mb_rec *mb);

/* ---- one MB's reconstruction from coded data (p64.c:1179-1237, 971-1013) ----
 * Decoder-side recon used by the decode path: coded coefficients (zigzag),
 * MTYPE/CBP/MV and quant -> writes the MB into recon (which must hold the
 * previous picture for skipped/uncoded content).  ref = previous picture. */
void orc_decode_mb(int width, int height, const uint8_t *ref, uint8_t *recon,
                   int mbx, int mby, int mtype, int cbp, int mvx, int mvy,
                   int quant, const int16_t *coef);

#ifdef __cplusplus
}
#endif
#endif
