/*
 * p64gpu.h -- C ABI of the MI355X-native PVRG-P64 macroblock encode hot path.
 *
 * Plain C, plain pointers and sizes; no HIP or torch types cross this header
 * (streams are passed as `void *` = hipStream_t, NULL = the default stream).
 * Every entry point returns P64GPU_OK (0) or a negative P64GPU_E_* status and
 * never calls exit(); p64gpu_last_error() gives the text of the last failure
 * on the calling thread.
 *
 * What each entry point replaces in the reference (/root/reference, PVRG-P64
 * v1.2 + maikmerten fork); INTEGRATION.md shows the host-side re-plumbing:
 *
 *   p64gpu_block_op            ChenDct chendct.c:97, ChenIDct chendct.c:217,
 *                              CCITTQuantize transform.c:271, CCITTFlatQuantize
 *                              :317, ICCITTFlatQuantize :359, ICCITTQuantize :400,
 *                              BoundDctMatrix :460, BoundIDctMatrix :483,
 *                              FlatBoundQuantizeMatrix :502, BoundQuantizeMatrix
 *                              :526, IZigzagMatrix :546, ZigzagMatrix :561
 *                              (the `vFunc *UseDct/UseIDct` plug-in, p64.c:227-231,
 *                              batched over blocks)
 *   p64gpu_motion_estimation   MotionEstimation(MEM*,MEM*) me.c:340 (TSS StepBME
 *                              me.c:255 as shipped, or brute-force FastBME me.c:187)
 *                              writing the MeX/MeY/MeVal/MeOVal/MeVAR/MeVAROR/MeMWOR
 *                              arrays (me.c:49-60) as p64_me_rec records
 *   p64gpu_encode_frames       GlobalMC io.c:129 + the per-MDU compute of
 *                              p64EncodeGOB p64.c:692-786 (MTYPE decision),
 *                              ReadCompressMDU p64.c:823, the reconstruction half
 *                              of WriteMDU p64.c:945-959 and DecodeSaveMDU p64.c:971,
 *                              for a batch of independent pictures
 *   p64gpu_encoder_*           host-buffer, state-keeping form of the above for a C
 *                              host loop: p64EncodeFrame p64.c:622 keeps CFS/OFS
 *                              (previous/new reconstruction) device resident and
 *                              swaps them (SwapFS p64.c:661)
 *   p64gpu_decode_recon        DecompressMDU p64.c:1179 (IZigzag/IQ/IDCT) +
 *                              DecodeSaveMDU p64.c:971 for decoded pictures
 *
 * Layouts.  A picture is planar 4:2:0: Y (w*h bytes) then U then V
 * ((w/2)*(h/2) bytes each), stride = plane width (MEM, mem.h:37-42).  w and h
 * are multiples of 16; batched pictures sit `frame_stride` bytes apart
 * (multiple of 16).  Macroblocks are in RASTER order mb = mby*(w/16)+mbx (the
 * index Bpos() yields in the MDU loop, io.c:757-783); GOB order is the host
 * writer's business.  Per macroblock, blocks c = 0..3 are luma
 * (h,v) = (0,0),(1,0),(0,1),(1,1), c = 4 is U, c = 5 is V (p64.c:77-79).
 * Coefficients are int16 levels in zigzag order, [mb][6][64]: the values
 * ReadCompressMDU leaves in inputbuf (p64.c:823-913), i.e. before CBP zeroing.
 * An inter picture stores only the blocks holding a nonzero level; the
 * optional nzmask output names them (bit 5-b for block b, the CBP bit order),
 * so inputbuf is exactly: block b's stored levels if its bit is set, else 64
 * zeros (p64gpu_encode_args.coef / .nzmask).
 *
 * ABI version 2 (round 5): p64gpu_encode_args.nzmask and .vlc_bits
 * (appended); the sparse inter level store of version 1's last revision, now
 * with that mask; p64gpu_vlc_args.flags (was `reserved`, must be 0),
 * .blk_bits (appended) and its scratch of 6*nframes*nmb uint32, 8-byte
 * aligned; synthetic contents (p64_synth_content).
 *
 * ABI version 3 (round 6): p64gpu_decode_recon_packed (packed levels +
 * per-group index, p64s_pack_levels in p64stream.h); p64gpu_vlc_pictures
 * accepts any device-addressable pointer (pinned host memory included) and
 * refuses pageable host memory; p64gpu_vlc_args.seq_bits / .max_bits
 * (appended).
 */
#ifndef P64GPU_H
#define P64GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define P64GPU_ABI_VERSION 3

enum p64gpu_status {
  P64GPU_OK = 0,
  P64GPU_E_INVALID = -1,  /* bad argument: shape, range, alignment or NULL */
  P64GPU_E_NODEVICE = -2, /* no usable HIP device */
  P64GPU_E_HIP = -3,      /* a HIP runtime call failed */
  P64GPU_E_NOMEM = -4,    /* device or host allocation failed */
  P64GPU_E_STREAM = -5    /* malformed or unsupported bitstream (p64stream.h) */
};

/* Motion search (me.c).  TSS is what the reference ships (me.c:352); FULL is
 * the dormant brute-force FastBME over [-sl/2, sl/2)^2 (me.c:206-208). */
enum p64gpu_me_mode { P64GPU_ME_TSS = 0, P64GPU_ME_FULL = 1 };

/* One macroblock's motion-estimation record (me.c:49-60, 353-359). */
typedef struct {
  int32_t mx, my; /* MeX, MeY: chosen vector                          */
  int32_t sad;    /* MeVal  = MV, SAD of the chosen vector             */
  int32_t sad0;   /* MeOVal = OMV, SAD of the (0,0) vector             */
  int32_t var;    /* MeVAR   = sum((ref-cur)^2)/256 at the vector      */
  int32_t varor;  /* MeVAROR = sum(ref^2)/256 - (sum(ref)/256)^2       */
  int32_t mwor;   /* MeMWOR  = sum(ref)                                */
} p64_me_rec;

/* One coded macroblock's header fields (marker.c:288 WriteMBHeader inputs). */
typedef struct {
  int8_t mtype; /* MType 0..9 after the CBP fallback (p64.c:899-906)     */
  int8_t cbp;   /* CBP (0x3f for types without CBP)                      */
  int8_t mvx;   /* MVDH transmitted: the ME vector for MC types, else 0 */
  int8_t mvy;   /* MVDV transmitted                                      */
} p64_mb_rec;

int p64gpu_abi_version(void);
const char *p64gpu_strerror(int status);
const char *p64gpu_last_error(void);

/* ---- device selection, memory and stream helpers (C hosts need no HIP
 * headers: these wrap hipGetDeviceCount/hipSetDevice/hipMalloc/hipFree/
 * hipMemcpyAsync/hipStreamSynchronize) ---- */
int p64gpu_device_count(int *count);
int p64gpu_set_device(int device);
int p64gpu_synchronize(void *stream);
int p64gpu_alloc(void **ptr, size_t bytes);
int p64gpu_free(void *ptr);
int p64gpu_copy_to_device(void *dst, const void *src, size_t bytes, void *stream);
int p64gpu_copy_to_host(void *dst, const void *src, size_t bytes, void *stream);
int p64gpu_copy_on_device(void *dst, const void *src, size_t bytes, void *stream);

/* ---- 8x8 block operations, batched (device pointers) -------------------- */
enum p64gpu_block_op {
  P64GPU_OP_DCT = 0,           /* ChenDct(in,out)                         */
  P64GPU_OP_IDCT = 1,          /* ChenIDct(in,out)                        */
  P64GPU_OP_QUANT_INTRA = 2,   /* CCITTFlatQuantize(m, dcq, acq)          */
  P64GPU_OP_QUANT_INTER = 3,   /* CCITTQuantize(m, dcq, acq)              */
  P64GPU_OP_IQUANT_INTRA = 4,  /* ICCITTFlatQuantize(m, dcq, acq)         */
  P64GPU_OP_IQUANT_INTER = 5,  /* ICCITTQuantize(m, dcq, acq)             */
  P64GPU_OP_BOUND_DCT = 6,     /* BoundDctMatrix(m)                       */
  P64GPU_OP_BOUND_IDCT = 7,    /* BoundIDctMatrix(m)                      */
  P64GPU_OP_BOUND_QFLAT = 8,   /* FlatBoundQuantizeMatrix(m)              */
  P64GPU_OP_BOUND_QUANT = 9,   /* BoundQuantizeMatrix(m)                  */
  P64GPU_OP_ZIGZAG = 10,       /* ZigzagMatrix(in,out)                    */
  P64GPU_OP_IZIGZAG = 11,      /* IZigzagMatrix(in,out)                   */
  P64GPU_OP_COUNT = 12
};
/* in/out: nblocks * 64 int32, row-major 8x8 blocks, device memory; in may
 * equal out (in-place ops).  dcq/acq are only read by the quantiser ops
 * (1..31; the intra DC step is normally 8, p64.c:874). */
int p64gpu_block_op(int op, const int32_t *in, int32_t *out, int64_t nblocks,
                    int dcq, int acq, void *stream);

/* ---- motion estimation over a batch of pictures (device pointers) ------- */
/* ref_y/cur_y: luma planes of nframes pictures, frame_stride apart.
 * out: nframes * nmb records. search_limit in 1..31 (FULL only; TSS is +-15). */
int p64gpu_motion_estimation(int width, int height, int nframes,
                             int64_t frame_stride, const uint8_t *ref_y,
                             const uint8_t *cur_y, int mode, int search_limit,
                             p64_me_rec *out, void *stream);

/* ---- the fused per-macroblock encode (device pointers) ------------------ */
/* flags: P64GPU_FLAG_ME_GIVEN -- inter pictures only: args->me already holds
 * this batch's ME records (p64gpu_motion_estimation over the same ref/cur
 * luma, mode and search limit), so the search is not run again; the rest of
 * the encode reads them.  The reference's own order: MotionEstimation() for
 * the picture first (p64.c:652, me.c:340), then the MDU loop reads MeVAR,
 * MeVAROR, MeX/MeY... (p64.c:734-756). */
/* P64GPU_FLAG_SEARCH_ONLY -- inter pictures only, with args->me: the search
 * alone (the first half of the encode), each record's mx, my, sad and sad0
 * written (its var / varor / mwor are not: the ME_GIVEN encode that follows
 * computes them itself); nothing else is read or written.  The two halves
 * in order -- SEARCH_ONLY, then ME_GIVEN over the same arguments -- are the
 * encode (the same outputs), with a point between them where the caller can
 * place stream work (bench.py's entropy coder of the previous picture runs
 * beside the second half).  Added in ABI version 3 (no layout change). */
enum { P64GPU_FLAG_ME_GIVEN = 1, P64GPU_FLAG_SEARCH_ONLY = 2 };
typedef struct {
  int32_t width, height;  /* picture size, multiples of 16, 32..4096         */
  int32_t nframes;        /* independent pictures in this launch (>= 1)      */
  int32_t intra;          /* 1: first picture of a sequence -> all MTYPE 0,
                             no ME (p64.c:635, 770-771)                      */
  int32_t quant;          /* GQuant 1..31 (UseQuant without -r)              */
  int32_t me_mode;        /* P64GPU_ME_TSS | P64GPU_ME_FULL                  */
  int32_t search_limit;   /* FULL: 1..31 (SearchLimit, me.c:62, -i flag)     */
  int32_t flags;          /* 0, P64GPU_FLAG_ME_GIVEN or _SEARCH_ONLY         */
  int64_t frame_stride;   /* bytes between pictures in cur/ref/recon        */
  const uint8_t *cur;     /* [nframes] current pictures                       */
  const uint8_t *ref;     /* [nframes] previous reconstructions (CFS);
                             unused when intra                               */
  uint8_t *recon;         /* [nframes] new reconstructions (OFS), written    */
  uint8_t *last_intra;    /* [nframes][nmb] intra-refresh counters, in/out
                             (LastIntra, p64.c:213, 772, 909-910)            */
  const uint8_t *quant_mb;      /* NULL or [nframes][nmb] UseQuant per MB    */
  const int8_t *mtype_override; /* NULL or [nframes][nmb]; < 0 = no override
                                   (-o interpreter program 0, p64.c:761-768) */
  int16_t *coef;          /* [nframes][nmb][6][64] zigzag levels, written:
                             every block of an intra picture; of an inter
                             picture every block with a nonzero level, a
                             block whose 64 levels are all zero is left as
                             it was (zero the buffer for the whole array, or
                             read it through nzmask; every block the MB
                             record's CBP and MTYPE transmit has a nonzero
                             level)                                         */
  p64_mb_rec *mb;         /* [nframes][nmb], written                         */
  p64_me_rec *me;         /* NULL or [nframes][nmb], written (inter only)    */
  uint8_t *nzmask;        /* NULL or [nframes][nmb], written: bit 5-b set iff
                             block b has a nonzero level (then its levels
                             were stored; clear: the block's levels are all
                             zero).  Intra pictures: 0x3f (the intra DC is
                             1..254)                                         */
  uint16_t *vlc_bits;     /* NULL or [nframes][nmb][8], 16-byte aligned,
                             written: entry 1 + b = the coded bits of block b
                             as the entropy coder writes it (EncodeAC /
                             CBPEncodeAC codec.c:96-205 incl. EOB, an intra
                             block's 8-bit DC), 0 if not transmitted; entry 0
                             and 7 are not written.  Hand it to
                             p64gpu_vlc_pictures as blk_bits: the coder then
                             does not count the blocks.  Not with
                             p64gpu_encode_mb_list (P64GPU_E_INVALID)        */
} p64gpu_encode_args;

/* Alignment: cur, ref, recon and coef 16 bytes; mb and me 4 bytes (the
 * kernels use 16-byte vector and dword record accesses); frame_stride a
 * multiple of 16.  Otherwise P64GPU_E_INVALID.
 * Inter pictures with args->me == NULL keep their ME records in a library
 * scratch buffer private to the (device, stream) of the call -- and to the
 * calling thread for hipStreamPerThread; see p64gpu_release_scratch.  While
 * the stream is capturing, such a call takes the fused kernel instead (a
 * graph never references library scratch). */
int p64gpu_encode_frames(const p64gpu_encode_args *args, void *stream);
/* The same for one picture (args->nframes == 1) restricted to the count
 * macroblocks listed in mb_list (device array of raster indices; entries out
 * of range are skipped).  Hosts that decide per GOB -- rate control sets
 * GQUANT from the bits written so far (p64.c:697-712) -- encode a picture GOB
 * by GOB with it; outputs of MBs not listed are left untouched. */
int p64gpu_encode_mb_list(const p64gpu_encode_args *args, const int32_t *mb_list, int count,
                          void *stream);

/* Frees the ME-record scratch buffers the library allocated for inter encodes
 * without args->me (one per device and stream; outgrown ones are kept until
 * this call, because work still in flight may reference them).  Call only
 * when no such encode is in flight. */
int p64gpu_release_scratch(void);

/* ---- decoder-side reconstruction (device pointers) ---------------------- */
/* recon must already hold the previous picture where MBs are not coded
 * (p64DecodeGOB leaves untransmitted MBs untouched); coded_mask
 * ([nmb] bytes, nonzero = MB present in the stream) selects the MBs written.
 * mb[].mtype/cbp/mvx/mvy and quant_mb (UseQuant per MB) come from the host
 * VLC decoder.  Pictures are independent within the call (nframes >= 1).
 * Levels are what H.261 syntax can carry (|AC level| <= 127, intra DC
 * 1..254): the dequantiser works in packed 16-bit arithmetic, exact for
 * |level| <= 528.  ref, recon and coef 16-byte aligned, mb 4-byte aligned. */
int p64gpu_decode_recon(int width, int height, int nframes, int64_t frame_stride,
                        const uint8_t *ref, uint8_t *recon, const int16_t *coef,
                        const p64_mb_rec *mb, const uint8_t *quant_mb,
                        const uint8_t *coded_mask, void *stream);

/* The same from PACKED levels (ABI v3): `levels` holds only the transmitted
 * blocks' 64 zigzag levels each (nlevels blocks: MB present in coded_mask,
 * MTYPE with coefficients, its CBP bit set -- what the stream carries),
 * contiguous in (picture, MB, block) raster order; `index` holds, for each
 * group of 64 consecutive blocks of the batch (the pictures' blocks back to
 * back, block = 6*(nmb*f + mb) + b; group j covers blocks 64j .. 64j+63, a
 * group may straddle two pictures; ceil(nframes*6*nmb/64) groups), four
 * uint32: the index in `levels` of the group's first transmitted block, 0,
 * and the group's 64-bit transmitted-block mask (bit i = block 64j + i), low
 * word first.  p64s_pack_levels (p64stream.h) builds
 * both from p64s_read_picture's output.  The kernel loads a group's levels
 * from its index entry without waiting for the records.
 * levels and index 16-byte aligned; nlevels < 2^24 per call. */
int p64gpu_decode_recon_packed(int width, int height, int nframes, int64_t frame_stride,
                               const uint8_t *ref, uint8_t *recon, const int16_t *levels,
                               int64_t nlevels, const uint32_t *index, const p64_mb_rec *mb,
                               const uint8_t *quant_mb, const uint8_t *coded_mask, void *stream);

/* ---- entropy coding on the device (p64vlc.hip) -------------------------- */
/* The H.261 bits of nframes coded pictures (QCIF/CIF/NTSC), identical to
 * p64s_write_picture (p64stream.h) and thus to the reference's WriteMDU/
 * WriteMBHeader/WriteGOBHeader/WritePictureHeader output.  Picture i is
 * written into out + i*out_stride starting at bit phase[i] (0..7) of its first
 * byte -- the bit position the sequence's stream has reached -- so the host
 * appends it by OR-ing the first byte into its pending byte.  bits[i] receives
 * the bit count including the phase, or 0xFFFFFFFF if a record was invalid.
 * Every pointer must be device-addressable: device memory, managed memory, or
 * host memory pinned by hipHostMalloc/hipHostRegister (e.g. `bits` straight
 * into pinned host memory, also under graph capture and replay: the kernel is
 * given the device pointer HIP reports for it); pageable host memory is
 * refused with P64GPU_E_INVALID (hipPointerGetAttributes, every call).
 * scratch holds 6*nframes*nmb uint32 and is 8-byte aligned, coef 16-byte, mb
 * 4-byte (else P64GPU_E_INVALID).  Batches whose levels exceed 2 GiB are
 * coded in several launches. */
typedef struct {
  int width, height, nframes;
  int flags;                /* 0 (was `reserved` before ABI version 2)        */
  const p64_mb_rec *mb;     /* [nframes][nmb] raster order (encoder output)   */
  const int16_t *coef;      /* [nframes][nmb][6][64] zigzag levels            */
  const uint8_t *gquant;    /* [nframes][ngob] GQUANT of each GOB header      */
  const uint8_t *mquant;    /* NULL or [nframes][nmb] MQUANT (types 1/3/6/9)  */
  const int32_t *tr;        /* [nframes] temporal references                  */
  const uint8_t *phase;     /* NULL (all 0) or [nframes] start bit 0..7       */
  uint8_t *out;             /* [nframes][out_stride]: every 32-bit word up to
                               the picture's last bit written (the phase bits
                               before its first as zeros), later ones left   */
  int64_t out_stride;       /* >= p64gpu_vlc_max_bytes, multiple of 4         */
  uint32_t *bits;           /* [nframes]                                      */
  uint32_t *scratch;        /* [6][nframes][nmb], 8-byte aligned              */
  uint16_t *blk_bits;       /* NULL, or [nframes][nmb][8] block bits from the
                               encoder (p64gpu_encode_args.vlc_bits, same
                               records and levels), 16-byte aligned, read
                               only: the blocks are not counted again        */
  int64_t *seq_bits;        /* (ABI v3) NULL, or [nframes] 8-byte aligned: the
                               running bit count of each picture's sequence;
                               the picture starts at phase seq_bits[i] & 7
                               (`phase` is then not read) and seq_bits[i]
                               advances by the picture's bits (not for an
                               invalid picture) -- a sequence's pictures coded
                               call after call without a host round trip    */
  uint32_t *max_bits;       /* (ABI v3) NULL, or [1]: set to the largest
                               bits[i] of the call's valid pictures         */
} p64gpu_vlc_args;
int64_t p64gpu_vlc_max_bytes(int width, int height);
int p64gpu_vlc_pictures(const p64gpu_vlc_args *args, void *stream);

/* ---- host-buffer encoder context (drop-in for a C host loop) ------------ */
typedef struct p64gpu_encoder p64gpu_encoder;
int p64gpu_encoder_open(int device, int width, int height, int me_mode,
                        int search_limit, p64gpu_encoder **out);
/* Encodes one picture (host Y|U|V, w*h*3/2 bytes).  intra=1 starts a new
 * sequence.  mtype_override may be NULL.  coef/mb are host outputs sized for
 * nmb macroblocks; me and recon may be NULL.  The reconstruction stays on the
 * device as the reference for the next call. */
int p64gpu_encoder_frame(p64gpu_encoder *enc, const uint8_t *picture, int intra,
                         int quant, const int8_t *mtype_override, int16_t *coef,
                         p64_mb_rec *mb, p64_me_rec *me, uint8_t *recon);
void p64gpu_encoder_close(p64gpu_encoder *enc);

/* ---- deterministic synthetic input (integer only) ----------------------- */
/* Two contents:
 *   P64_SYNTH_VNOISE  value-noise texture, per-seed motion in [-3,3]x[-2,2],
 *                     small temporal noise; seed classes mod 8: 5 scene cut at
 *                     picture 12, 6 noise-free, 7 low contrast (synth.c)
 *   P64_SYNTH_SURVEY  SURVEY.md 8(d): 128 + 50 sin(x/7) cos(y/11)
 *                     + 30 sin((x+y)/23) + N(0,12) texture translated by
 *                     (+3,-2) px per picture + N(0,4) temporal noise; chroma
 *                     from the 2x2-averaged luma (synth_impl.h)            */
enum p64_synth_content { P64_SYNTH_VNOISE = 0, P64_SYNTH_SURVEY = 1 };
/* Host: picture `frame` of stream `seed` (Y|U|V, w*h*3/2 bytes). */
void p64_synth_motion(uint32_t seed, int *mvx, int *mvy); /* VNOISE only */
void p64_synth_frame(uint32_t seed, int frame, int width, int height,
                     uint8_t *out); /* = p64_synth_frame_content(VNOISE, ...) */
int p64_synth_frame_content(int content, uint32_t seed, int frame, int width,
                            int height, uint8_t *out);
/* Device: the same bytes for nslots x nseeds pictures, slot-major: picture
 * (t, s) = p64_synth_frame_content(content, seed0 + s, frame0 + t) at
 * out + (t*nseeds + s)*stride.  nseeds*nslots <= 65535. */
int p64gpu_synth_frames(int width, int height, uint32_t seed0, int nseeds,
                        int frame0, int nslots, int64_t frame_stride,
                        uint8_t *out, void *stream); /* VNOISE */
int p64gpu_synth_content(int content, int width, int height, uint32_t seed0,
                         int nseeds, int frame0, int nslots,
                         int64_t frame_stride, uint8_t *out, void *stream);

/* Clock probe (measurement aid; no reference counterpart): runs
 * v_sad_u8 chains on every SIMD for `microseconds`, then reports the median
 * shader clock the waves held (s_memtime ticks / s_memrealtime ticks x
 * 100 MHz).  Synchronises the stream.  bench.py reads the clock a timed
 * region left the chip at with a short probe after it. */
int p64gpu_clock_probe(int microseconds, int *mhz, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* P64GPU_H */
