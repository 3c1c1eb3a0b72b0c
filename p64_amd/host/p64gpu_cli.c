/*
 * p64gpu_cli.c -- the reference CLI's encode and decode modes over the C ABI.
 *
 * Encode (p64EncodeSequence p64.c:524 / p64EncodeFrame p64.c:622):
 *   y4m in -> p64seq (GPU: ME, decision, DCT/quant, closed-loop reconstruction
 *   kept on the device; host: VLC and rate control) -> .p64, byte-identical to
 *   the reference's for the same flags.
 * Decode (p64DecodeSequence p64.c:1022):
 *   .p64 -> p64s_read_picture (host VLC parse) -> p64gpu_decode_recon (GPU:
 *   IQ/IDCT/prediction/filter) -> component files "<prefix><n>.Y/.U/.V"
 *   (MakeFileNames p64.c:1581, SaveMem) or one y4m (WriteIob io.c:686).
 *
 * Flags follow the reference (p64.c:262-404, p64.1):
 *   -NTSC | -CIF | -QCIF   picture format (checked against the y4m header)
 *   -y4m                    y4m input (encode) / output (decode)
 *   -a n  -b n  -k n        first / last frame, frame skip (TR = frame mod 32)
 *   -q n  -i n              quantiser 1..31, search limit 1..31 (BoundValue)
 *   -r bits/s  -x bits      rate control (buffer-driven GQUANT per GOB, MTYPE 4
 *                           on overflow) from a rate or a total file size
 *   -f rate                 frame rate (30000/1001 default; enters -r/-x)
 *   -s file                 stream file (default <prefix>.p64)
 *   -z suffix               component file suffix (default .y4m with -y4m)
 *   -d                      decode
 *   -c                      decode: ForceCIF, CIF geometry whatever PTYPE says
 *                           (p64.c:308-310, 1071-1072)
 *   -v                      print BufferContents / GQUANT at every rate-control
 *                           update (ExecuteQuantization p64.c:466-470)
 *   -l n                    Loud level: accepted; the statistics it prints
 *                           (stat.c) are not reproduced
 *   -p                      ParityEnable: accepted; it changes the stream only in
 *                           the VERSION_1_0 syntax the reference does not build
 *   -                       y4m from stdin
 * Additions: -full / -tss (FastBME vs the shipped StepBME), -D device,
 * -hostvlc (entropy-code on the host instead of the GPU).
 *   -o                      program interpreter: program text on stdin (p64prog.h)
 *   (no -y4m)               raw component files <prefix><n>.Y/.U/.V per picture
 * Not supported here: -y floating-point reference DCT (a test option; see
 * DESIGN.md).
 *
 * Differences from the reference: a y4m that ends before -b finishes the
 * stream (trailer written) instead of exit(ERROR_BOUNDS) with an unterminated
 * file; raw-file input ends with a complete stream (the reference crashes in
 * video_input_close before swclose, SURVEY.md 0.8, leaving it unflushed); every
 * failure exits non-zero with a message, never a segfault.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/p64gpu.h"
#include "../../include/p64prog.h"
#include "../../include/p64seq.h"
#include "../../include/p64stream.h"

static const char *const FMT_NAME[3] = {"QCIF", "CIF", "NTSC"};
static p64prog *g_prog; /* -o program */

static int die(const char *what, int s) {
  fprintf(stderr, "p64gpu: %s: %s (%s)\n", what, p64gpu_strerror(s), p64gpu_last_error());
  return 2;
}

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

static int drain(p64s_writer *wr, FILE *o) {
  size_t n;
  const uint8_t *d = p64s_writer_data(wr, &n, NULL);
  if (n && fwrite(d, 1, n, o) != n) return -1;
  return n ? p64s_writer_consume(wr, n) : 0;
}

typedef struct {
  int format, y4m, first, last, skip, quant, sl, mode, device, decode, from_stdin;
  int rate, file_size_bits, frame_rate, frame_rate_div, oracle, host_vlc;
  int force_cif, loud, verbose;
  const char *prefix, *suffix, *stream;
} opts;

/* raw component files <prefix><frame><suffix>, suffixes .Y .U .V by default
 * (MakeFileNames p64.c:1581, LoadMem mem.c) -- one file per plane and picture */
static int read_raw(const opts *o, int frame, int w, int h, unsigned char *buf) {
  static const char *const sfx[3] = {".Y", ".U", ".V"};
  const size_t n[3] = {(size_t)w * h, (size_t)w * h / 4, (size_t)w * h / 4};
  size_t off = 0;
  for (int c = 0; c < 3; c++) {
    char path[4096];
    snprintf(path, sizeof path, "%s%d%s", o->prefix, frame, sfx[c]);
    FILE *f = fopen(path, "rb");
    const size_t got = f ? fread(buf + off, 1, n[c], f) : 0;
    if (f) fclose(f);
    if (got != n[c]) return 0;
    off += n[c];
  }
  return 1;
}

static int encode(const opts *o) {
  char path[4096];
  FILE *f = NULL;
  int w, h, s;
  if (o->y4m) {
    if (o->from_stdin) {
      f = stdin;
    } else {
      snprintf(path, sizeof path, "%s%s", o->prefix, o->suffix ? o->suffix : ".y4m");
      f = fopen(path, "rb");
    }
    if (!f || read_y4m_header(f, &w, &h)) {
      fprintf(stderr, "p64gpu: cannot read y4m input\n");
      return 1;
    }
  } else { /* raw planes: the format comes from the flags (ImageType default NTSC, p64.c:114) */
    p64s_geometry(o->format >= 0 ? o->format : P64S_NTSC, &w, &h, NULL);
  }
  const int fmt = p64s_format_of(w, h);
  if (fmt < 0 || (o->format >= 0 && fmt != o->format)) {
    fprintf(stderr, "p64gpu: y4m is %dx%d, not %s\n", w, h,
            o->format >= 0 ? FMT_NAME[o->format] : "QCIF/CIF/NTSC");
    return 1;
  }
  const size_t pic = (size_t)w * h * 3 / 2;
  unsigned char *buf = malloc(pic);
  /* seek to StartFrame (p64.c:562-565) */
  for (int i = 0; f && i < o->first; i++)
    if (read_frame(f, buf, pic) != 1) {
      fprintf(stderr, "p64gpu: input ends before frame %d\n", o->first);
      return 1;
    }
  char spath[4096];
  if (o->stream) snprintf(spath, sizeof spath, "%s", o->stream);
  else snprintf(spath, sizeof spath, "%s.p64", o->prefix);
  FILE *out = fopen(spath, "wb");
  if (!out) {
    fprintf(stderr, "p64gpu: cannot open %s\n", spath);
    return 1;
  }
  p64seq_config cfg;
  p64seq_default_config(&cfg);
  cfg.format = fmt;
  cfg.me_mode = o->mode;
  cfg.search_limit = o->sl;
  cfg.quant = o->quant;
  cfg.rate = o->rate;
  cfg.file_size_bits = o->file_size_bits;
  cfg.start_frame = o->first;
  cfg.last_frame = o->last < o->first ? o->first : o->last;
  cfg.frame_skip = o->skip;
  cfg.frame_rate = o->frame_rate;
  cfg.frame_rate_div = o->frame_rate_div;
  cfg.device = o->device;
  cfg.program = g_prog;
  cfg.host_vlc = o->host_vlc;
  cfg.verbose = o->verbose;
  p64seq *sq = NULL;
  if ((s = p64seq_open(&cfg, &sq))) return die("p64seq_open", s);
  p64seq_stats st;
  p64seq_get_stats(sq, &st);
  if (st.rate) printf("Rate: %d   QDFact: %d  QOffs: %d\nStarting Quantization: %d\n", st.rate, st.rate / 320, 1, st.gquant);
  printf("START>SEQUENCE\n");
  while (p64seq_more(sq)) {
    p64seq_get_stats(sq, &st);
    /* y4m pictures are read in sequence whatever -k says (ReadIob io.c:629-645);
     * raw files are named by the frame number */
    const int r = f ? read_frame(f, buf, pic) : read_raw(o, st.next_frame, w, h, buf);
    if (r <= 0) {
      if (r < 0 || !f) fprintf(stderr, "p64gpu: cannot read frame %d\n", st.next_frame);
      break;
    }
    if ((s = p64seq_encode(sq, buf))) return die("encode", s);
    p64seq_get_stats(sq, &st);
    printf("END>Frame: %d  bits %lld  GQuant %d\n", st.next_frame - o->skip, (long long)st.last_bits, st.gquant);
    if (drain(p64seq_writer(sq), out)) {
      fprintf(stderr, "p64gpu: write error on %s\n", spath);
      return 1;
    }
  }
  if ((s = p64seq_finish(sq))) return die("finish", s);
  if (drain(p64seq_writer(sq), out) || fclose(out)) {
    fprintf(stderr, "p64gpu: write error on %s\n", spath);
    return 1;
  }
  p64seq_get_stats(sq, &st);
  printf("END>SEQUENCE\n");
  printf("Bits for first frame: %lld   Number of buffer overflows: %d\n", (long long)st.first_frame_bits,
         st.overflows);
  printf("frames %d  MTYPE histogram:", st.frames);
  for (int k = 0; k < 10; k++) printf(" %d", st.mtype_hist[k]);
  printf("\n");
  p64seq_close(sq);
  if (f && f != stdin) fclose(f);
  free(buf);
  return 0;
}

static int save(const char *path, const uint8_t *d, size_t n) {
  FILE *f = fopen(path, "wb");
  if (!f || fwrite(d, 1, n, f) != n || fclose(f)) {
    fprintf(stderr, "p64gpu: cannot write %s\n", path);
    return 1;
  }
  return 0;
}

static int decode(const opts *o) {
  if (!o->stream) {
    fprintf(stderr, "p64gpu: -d needs -s stream\n");
    return 1;
  }
  FILE *f = fopen(o->stream, "rb");
  if (!f) {
    fprintf(stderr, "p64gpu: cannot read %s\n", o->stream);
    return 1;
  }
  fseek(f, 0, SEEK_END);
  const long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *data = malloc(len > 0 ? (size_t)len : 1);
  if (len < 0 || fread(data, 1, (size_t)len, f) != (size_t)len) {
    fprintf(stderr, "p64gpu: read error on %s\n", o->stream);
    return 1;
  }
  fclose(f);
  p64s_reader *rd;
  p64s_picture_info info;
  int s;
  if ((s = p64s_reader_open(data, (size_t)len, &rd))) return die("reader_open", s);
  if (o->force_cif && (s = p64s_reader_force_cif(rd))) return die("reader_force_cif", s);
  p64s_reader_info(rd, &info);
  const int w = info.width, h = info.height, nmb = info.ngob * 33;
  const size_t pic = (size_t)w * h * 3 / 2;
  if ((s = p64gpu_set_device(o->device))) return die("set_device", s);
  p64_mb_rec *mb = malloc(nmb * sizeof *mb);
  uint8_t *qm = malloc(nmb), *coded = malloc(nmb), *host = calloc(pic, 1);
  int16_t *coef = malloc((size_t)nmb * 384 * sizeof *coef);
  /* the packed layout of p64gpu_decode_recon_packed: the transmitted blocks'
   * levels only, and the per-group index (p64s_pack_levels) */
  const size_t ngr = ((size_t)nmb * 6 + 63) / 64;
  int16_t *levels = malloc((size_t)nmb * 384 * sizeof *levels);
  uint32_t *index = malloc(ngr * 16);
  uint8_t *d_pic[2], *d_qm, *d_coded;
  int16_t *d_coef;
  uint32_t *d_index;
  p64_mb_rec *d_mb;
  if ((s = p64gpu_alloc((void **)&d_pic[0], pic)) || (s = p64gpu_alloc((void **)&d_pic[1], pic)) ||
      (s = p64gpu_alloc((void **)&d_qm, nmb)) || (s = p64gpu_alloc((void **)&d_coded, nmb)) ||
      (s = p64gpu_alloc((void **)&d_coef, (size_t)nmb * 384 * sizeof *coef)) ||
      (s = p64gpu_alloc((void **)&d_index, ngr * 16)) ||
      (s = p64gpu_alloc((void **)&d_mb, nmb * sizeof *mb)) ||
      (s = p64gpu_copy_to_device(d_pic[0], host, pic, NULL))) /* ClearFS */
    return die("device buffers", s);
  FILE *y4m = NULL;
  char path[4096];
  if (o->y4m) {
    snprintf(path, sizeof path, "%s%s", o->prefix, o->suffix ? o->suffix : ".y4m");
    y4m = fopen(path, "wb");
    if (!y4m) {
      fprintf(stderr, "p64gpu: cannot open %s\n", path);
      return 1;
    }
    fprintf(y4m, "YUV4MPEG2 W%d H%d C420jpeg Ip F30000:1001\n", w, h); /* p64.c:249-251, 1102 */
  }
  /* frame output schedule, p64DecodeSequence p64.c:1047-1056 */
  int frame = o->first, offset = 0, npics = 0, written = 0, prev = 0;
  for (;;) {
    const int r = p64s_read_picture(rd, &info, mb, qm, coded, coef);
    if (r < 0) return die("bitstream", r);
    if (npics) { /* the previous picture is complete: write it until TR matches */
      int guard = 0;
      while ((frame + offset) % 32 != info.tr && guard++ < 32) {
        if (y4m) {
          if (fwrite("FRAME\n", 1, 6, y4m) != 6 || fwrite(host, 1, pic, y4m) != pic) return 1;
        } else {
          const char *sfx[3] = {".Y", ".U", ".V"};
          const size_t off[3] = {0, (size_t)w * h, (size_t)w * h * 5 / 4};
          const size_t n[3] = {(size_t)w * h, (size_t)w * h / 4, (size_t)w * h / 4};
          for (int c = 0; c < 3; c++) {
            snprintf(path, sizeof path, "%s%d%s", o->prefix, frame, sfx[c]);
            if (save(path, host + off[c], n[c])) return 1;
          }
        }
        printf("END> Frame: %d\n", frame);
        frame++;
        written++;
      }
    }
    if (r == 0) break;
    if (!npics) offset = (info.tr - frame) % 32;
    /* recon starts as the previous picture: untransmitted MBs keep it */
    uint8_t *ref = d_pic[prev], *rec = d_pic[prev ^ 1];
    const int64_t nlev = p64s_pack_levels(info.format, 1, mb, coded, coef, levels, index);
    if (nlev < 0) return die("pack_levels", (int)nlev);
    if ((s = p64gpu_copy_on_device(rec, ref, pic, NULL)) ||
        (s = p64gpu_copy_to_device(d_mb, mb, nmb * sizeof *mb, NULL)) ||
        (s = p64gpu_copy_to_device(d_qm, qm, nmb, NULL)) ||
        (s = p64gpu_copy_to_device(d_coded, coded, nmb, NULL)) ||
        (s = p64gpu_copy_to_device(d_coef, levels, (size_t)nlev * 64 * sizeof *levels, NULL)) ||
        (s = p64gpu_copy_to_device(d_index, index, ngr * 16, NULL)) ||
        (s = p64gpu_decode_recon_packed(w, h, 1, (int64_t)pic, ref, rec, d_coef, nlev, d_index, d_mb, d_qm,
                                        d_coded, NULL)) ||
        (s = p64gpu_copy_to_host(host, rec, pic, NULL)) || (s = p64gpu_synchronize(NULL)))
      return die("decode", s);
    prev ^= 1;
    npics++;
  }
  printf("pictures %d  frames written %d\n", npics, written);
  if (y4m && fclose(y4m)) return 1;
  p64s_reader_close(rd);
  free(data);
  return 0;
}

int main(int argc, char **argv) {
  opts o = {.format = -1, .first = 0, .last = 0, .skip = 1, .quant = 0, .sl = 15,
            .mode = P64GPU_ME_TSS, .frame_rate = 30000, .frame_rate_div = 1001};
  for (int i = 1; i < argc; i++) {
    const char *a = argv[i];
    const int more = i + 1 < argc;
    if (!strcmp(a, "-NTSC")) o.format = P64S_NTSC;
    else if (!strcmp(a, "-CIF")) o.format = P64S_CIF;
    else if (!strcmp(a, "-QCIF")) o.format = P64S_QCIF;
    else if (!strcmp(a, "-y4m")) o.y4m = 1;
    else if (!strcmp(a, "-full")) o.mode = P64GPU_ME_FULL;
    else if (!strcmp(a, "-tss")) o.mode = P64GPU_ME_TSS;
    else if (!strcmp(a, "-D") && more) o.device = atoi(argv[++i]);
    else if (!strcmp(a, "-a") && more) o.first = atoi(argv[++i]);
    else if (!strcmp(a, "-b") && more) o.last = atoi(argv[++i]);
    else if (!strcmp(a, "-k") && more) o.skip = atoi(argv[++i]);
    else if (!strcmp(a, "-q") && more) {
      o.quant = atoi(argv[++i]); /* BoundValue(InitialQuant, 1, 31) p64.c:357-358 */
      if (o.quant < 1) o.quant = 1;
      if (o.quant > 31) o.quant = 31;
    }
    else if (!strcmp(a, "-i") && more) o.sl = atoi(argv[++i]);
    else if (!strcmp(a, "-s") && more) o.stream = argv[++i];
    else if (!strcmp(a, "-z") && more) o.suffix = argv[++i];
    else if (!strcmp(a, "-d")) o.decode = 1;
    else if (!strcmp(a, "-o")) o.oracle = 1;
    else if (!strcmp(a, "-hostvlc")) o.host_vlc = 1;
    else if (!strcmp(a, "-c")) o.force_cif = 1;
    else if (!strcmp(a, "-l") && more) o.loud = atoi(argv[++i]);
    else if (!strcmp(a, "-p")) (void)0; /* ParityEnable: no stream effect outside VERSION_1_0 */
    else if (!strcmp(a, "-v")) o.verbose = 1;
    else if (!strcmp(a, "-r") && more) o.rate = atoi(argv[++i]);
    else if (!strcmp(a, "-x") && more) o.file_size_bits = atoi(argv[++i]);
    else if (!strcmp(a, "-f") && more) {
      /* -f rate[.frac | /div | :div] (p64.c:314-339) */
      const char *v = argv[++i];
      const size_t numlen = strcspn(v, "./:");
      o.frame_rate = atoi(v);
      o.frame_rate_div = 1;
      if (v[numlen] == '.') {
        for (size_t k = strlen(v + numlen + 1); k > 0; --k) o.frame_rate_div *= 10;
        o.frame_rate = o.frame_rate * o.frame_rate_div + atoi(v + numlen + 1);
      } else if (v[numlen]) {
        o.frame_rate_div = atoi(v + numlen + 1);
        if (o.frame_rate_div < 1) o.frame_rate_div = 1;
      }
    }
    else if (!strcmp(a, "-")) {
      o.from_stdin = 1;
      o.prefix = "stdin";
    } else if (a[0] == '-') {
      fprintf(stderr, "p64gpu: unsupported option %s\n", a);
      return 1;
    } else {
      o.prefix = a;
    }
  }
  if (!o.prefix) {
    fprintf(stderr,
            "usage: p64gpu [-NTSC|-CIF|-QCIF] -y4m [-a n] [-b n] [-k n] [-q q] [-i sl] [-full|-tss]\n"
            "              [-r bits/s | -x bits] [-f rate] [-o] [-v] [-l n] [-p] [-D dev]\n"
            "              [-s out.p64] [-z suffix] prefix|-\n"
            "       p64gpu -d [-c] [-y4m] -s in.p64 [-z suffix] prefix\n");
    return 1;
  }
  /* BoundValue (p64.c:341-352); -q absent leaves 0 (default / rate-derived) */
  if (o.sl < 1) o.sl = 1;
  if (o.sl > 31) o.sl = 31;
  if (o.skip < 1) o.skip = 1;
  if (o.oracle && !o.decode) {
    /* -o: the program is read from stdin and its top-level statements run
     * after the command line, so they override it (p64.c:409-413) */
    size_t cap = 1 << 16, len = 0;
    char *text = malloc(cap);
    for (size_t n; (n = fread(text + len, 1, cap - len, stdin)) > 0;) {
      len += n;
      if (len == cap) text = realloc(text, cap *= 2);
    }
    int s = p64prog_load(text, len, stdout, &g_prog);
    free(text);
    if (s) return die("program", s);
    p64prog_settings ps;
    p64prog_settings_get(g_prog, &ps);
    if (ps.quantization >= 0) o.quant = ps.quantization;
    if (ps.search_limit >= 0) o.sl = ps.search_limit;
    if (ps.frame_rate >= 0) o.frame_rate = ps.frame_rate, o.frame_rate_div = 1;
    if (ps.frame_skip >= 0) o.skip = ps.frame_skip;
    if (ps.image_type >= 0) o.format = ps.image_type;
    if (o.from_stdin) {
      fprintf(stderr, "p64gpu: -o reads the program from stdin; give the y4m as a file\n");
      return 1;
    }
  }
  return o.decode ? decode(&o) : encode(&o);
}
