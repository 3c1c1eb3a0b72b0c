/*
 * p64stream.h -- H.261 bitstream layer of the drop-in (host C, part of
 * libp64gpu.so; no GPU involved).
 *
 * The GPU path (p64gpu.h) stops at the coefficient boundary: per macroblock
 * MTYPE/CBP/MV records and zigzagged levels.  These entry points turn those
 * records into the reference's .p64 bytes and back:
 *
 *   p64s_write_picture   WritePictureHeader marker.c:103 + WriteGOBHeader
 *                        marker.c:171 + the MDU loop of p64EncodeGOB
 *                        p64.c:692-786 as far as it writes: WriteMDU p64.c:920
 *                        -> WriteMBHeader marker.c:288 (MBA/MTYPE/MQUANT/MVD/CBP,
 *                        with the reference's MVD predictor reset rule), EncodeDC
 *                        codec.c:343, EncodeAC codec.c:96, CBPEncodeAC codec.c:141;
 *                        VLC tables huffman.c:102-290 + ctables.h (the H.261
 *                        tables), bit order stream.c:112-190 (MSB first)
 *   p64s_write_end       the trailing picture header p64.c:608-610 and mwclose
 *                        stream.c:121 (last byte padded with ones)
 *   p64s_read_picture    p64DecodeSequence p64.c:1022 / p64DecodeGOB p64.c:1131 /
 *                        ReadMBHeader marker.c:372 / DecompressMDU p64.c:1179 up to
 *                        the levels (DecodeDC codec.c:326, DecodeAC codec.c:215,
 *                        CBPDecodeAC codec.c:258); the IQ/IDCT/prediction half runs
 *                        on the GPU (p64gpu_decode_recon)
 *
 * Every function returns 0 (or a documented positive value) on success and a
 * negative P64GPU_E_* status on failure, with the text in p64gpu_last_error().
 * Macroblock arrays are in RASTER order (mb = mby*(w/16)+mbx), the layout of
 * the GPU records; the GOB/MDU order of the bitstream (Bpos io.c:757) is
 * applied here.
 */
#ifndef P64STREAM_H
#define P64STREAM_H

#include <stddef.h>
#include <stdint.h>

#include "p64gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Picture formats the reference codes (SetCCITT p64.c:1373, PType p64.c:414-431). */
enum p64s_format { P64S_QCIF = 0, P64S_CIF = 1, P64S_NTSC = 2 };

/* Geometry of a format: 176x144 / 352x288 / 352x240 and 3 / 12 / 10 GOBs of
 * 33 MBs.  Returns P64GPU_E_INVALID for an unknown format. */
int p64s_geometry(int format, int *width, int *height, int *ngob);
/* Format of a picture size, or P64GPU_E_INVALID. */
int p64s_format_of(int width, int height);

/* ---- writer ------------------------------------------------------------- */
typedef struct p64s_writer p64s_writer;
int p64s_writer_open(p64s_writer **out);
void p64s_writer_close(p64s_writer *w);
/* One coded picture: picture header with temporal reference tr (mod 32),
 * then every GOB (header with gquant[g]) and every macroblock in GOB order.
 * mb/coef are the GPU records ([nmb], [nmb][6][64] zigzag levels before CBP
 * zeroing); quant_mb ([nmb], may be NULL if no MB has an MQUANT type 1/3/6/9)
 * gives MQUANT.  Blocks are written when their CBP bit is set and the MTYPE
 * carries coefficients, exactly as WriteMDU. */
int p64s_write_picture(p64s_writer *w, int format, int tr, const uint8_t *gquant,
                       const uint8_t *quant_mb, const p64_mb_rec *mb, const int16_t *coef);
/* The same at finer grain, for hosts that decide per GOB or per MB while
 * writing (rate control, p64.c:697-786): a picture header, then per GOB its
 * header (resets the MBA/MVD predictors) and its macroblocks in increasing MDU
 * order (MDUs skipped are absent from the stream).  mquant is used only for
 * MTYPEs 1/3/6/9.  coef = the macroblock's 6x64 zigzag levels. */
int p64s_write_picture_header(p64s_writer *w, int format, int tr);
int p64s_write_gob_header(p64s_writer *w, int gob, int gquant);
int p64s_write_mb(p64s_writer *w, int mdu, const p64_mb_rec *mb, const int16_t *coef, int mquant);
/* Appends bits coded elsewhere (p64gpu_vlc_pictures): data holds `bits` bits
 * of which the first `phase` are the writer's pending partial byte, so phase
 * must equal p64s_writer_phase(). */
int p64s_write_bits(p64s_writer *w, const uint8_t *data, int64_t bits, int phase);
int p64s_writer_phase(const p64s_writer *w);
/* Raster macroblock index of MDU m (0..32) of GOB g (Bpos, io.c:757), -1 if
 * out of range. */
int p64s_raster_mb(int format, int gob, int mdu);
/* Trailing picture header (tr = frame after the last, mod 32) and final
 * ones-padding.  The writer accepts no more pictures afterwards. */
int p64s_write_end(p64s_writer *w, int format, int tr);
/* The bytes completed so far; *bits (may be NULL) receives the total number
 * of bits written (mwtell, stream.c:201). */
const uint8_t *p64s_writer_data(const p64s_writer *w, size_t *len, int64_t *bits);
/* Drops the first n completed bytes (after the caller has stored them). */
int p64s_writer_consume(p64s_writer *w, size_t n);

/* ---- reader ------------------------------------------------------------- */
typedef struct {
  int format, width, height, ngob;
  int tr;          /* temporal reference of the picture (5 bits)            */
  int ptype;       /* PTYPE (6 bits)                                        */
  int pspare;      /* PSPARE byte, -1 if none                               */
  int coded_mbs;   /* macroblocks present in the stream for this picture    */
} p64s_picture_info;

typedef struct p64s_reader p64s_reader;
/* The reader keeps a pointer to data, which must outlive it.  Fails with
 * P64GPU_E_STREAM when the stream does not start with a picture start code. */
int p64s_reader_open(const uint8_t *data, size_t len, p64s_reader **out);
void p64s_reader_close(p64s_reader *r);
/* -c ForceCIF (p64.c:308-310, 1071-1072): decode every picture with CIF
 * geometry and GOB numbering whatever its PTYPE says (a QCIF or NTSC stream
 * lands in the CIF frame; GOBs it does not send stay as they were).  Call
 * right after p64s_reader_open: once p64s_read_picture has run it fails with
 * P64GPU_E_INVALID (the caller's arrays are sized for the old geometry). */
int p64s_reader_force_cif(p64s_reader *r);
/* Geometry of the stream (from its first picture header, or CIF when forced). */
int p64s_reader_info(const p64s_reader *r, p64s_picture_info *info);
/* Decodes the next picture's headers and levels.  Returns 1 with a picture,
 * 0 at the end of the stream (info->tr then holds the temporal reference of
 * the trailing picture header, or the last picture's tr + 1 if the stream
 * ends without one -- the two cases of p64DecodeSequence p64.c:1040-1046).
 * Outputs, raster order, all [nmb]:
 *   mb        mtype, cbp (0x3f for types without CBP), MV (0 for non-MC types)
 *   quant_mb  UseQuant of the macroblock (GQUANT or MQUANT)
 *   coded     1 if the macroblock is present in the stream, else 0 (the
 *             decoder keeps the previous picture there, p64DecodeGOB)
 *   coef      [nmb][6][64] zigzag levels; zero where a block is not coded
 * The arrays are fully written (absent MBs get zeros). */
int p64s_read_picture(p64s_reader *r, p64s_picture_info *info, p64_mb_rec *mb,
                      uint8_t *quant_mb, uint8_t *coded, int16_t *coef);

/* The packed level layout of p64gpu_decode_recon_packed (p64gpu.h) from
 * nframes pictures of p64s_read_picture output (mb, coded, coef as that
 * call writes them, pictures consecutive): the transmitted blocks' levels
 * into `levels` (room for up to nframes*nmb*6 blocks), contiguous in raster
 * order, and the per-group index (ceil(nframes*6*nmb/64) * 4 uint32: groups
 * of 64 consecutive blocks of the batch, pictures back to back).
 * Returns the number of blocks written (>= 0) or a negative status. */
int64_t p64s_pack_levels(int format, int nframes, const p64_mb_rec *mb, const uint8_t *coded,
                         const int16_t *coef, int16_t *levels, uint32_t *index);

#ifdef __cplusplus
}
#endif

#endif /* P64STREAM_H */
