/*
 * p64stream.c -- H.261 bitstream writer/reader (include/p64stream.h).
 *
 * Host C.  The GPU produces per-macroblock records; this file is the entropy
 * coding either side of them, byte-compatible with the reference's .p64:
 *   - bit order: MSB first, last byte padded with ones (stream.c:89-190, :121)
 *   - VLC tables: ITU-T H.261 tables 1-5 as the reference loads them
 *     (ctables.h via huffman.c:102-160); written here in the standard's own
 *     bit-string notation and expanded at first use into direct-lookup encode
 *     arrays and prefix-indexed decode tables (the reference walks a binary
 *     state machine per bit, huffman.c:255-330)
 *   - syntax: marker.c (headers), codec.c (levels), p64.c (MDU order)
 */
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/p64stream.h"

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

/* ---- coding-control tables, p64.c:217-222 -------------------------------- */
static const unsigned char QUANT_MT[10] = {0, 1, 0, 1, 0, 0, 1, 0, 0, 1};
static const unsigned char CBP_MT[10] = {0, 0, 1, 1, 0, 1, 1, 0, 1, 1};
static const unsigned char MF_MT[10] = {0, 0, 0, 0, 1, 1, 1, 1, 1, 1};
static const unsigned char TC_MT[10] = {1, 1, 1, 1, 0, 1, 1, 0, 1, 1};

/* ---- formats (SetCCITT p64.c:1373; PType p64.c:414-431) ------------------ */
int p64s_geometry(int format, int *width, int *height, int *ngob) {
  static const int W[3] = {176, 352, 352}, H[3] = {144, 288, 240}, G[3] = {3, 12, 10};
  if (format < 0 || format > 2) return fail(P64GPU_E_INVALID, "unknown picture format %d", format);
  if (width) *width = W[format];
  if (height) *height = H[format];
  if (ngob) *ngob = G[format];
  return 0;
}

int p64s_format_of(int width, int height) {
  for (int f = 0; f < 3; f++) {
    int w, h;
    p64s_geometry(f, &w, &h, NULL);
    if (w == width && h == height) return f;
  }
  return fail(P64GPU_E_INVALID, "%dx%d is not QCIF, CIF or NTSC", width, height);
}

/* GOB g, MDU m -> raster macroblock index (Bpos/MoveTo io.c:719-783). */
int p64s_raster_mb(int format, int g, int m) {
  if (format < 0 || format > 2 || g < 0 || m < 0 || m >= 33) return -1;
  return (format == P64S_QCIF) ? (3 * g + m / 11) * 11 + m % 11
                               : ((g >> 1) * 3 + m / 11) * 22 + (g & 1) * 11 + m % 11;
}
static int raster_mb(int format, int g, int m) {
  if (format == P64S_QCIF) return (3 * g + m / 11) * 11 + m % 11;
  return ((g >> 1) * 3 + m / 11) * 22 + (g & 1) * 11 + m % 11;
}

/* ---- VLC tables ---------------------------------------------------------- */
/* H.261 Table 1 (MBA): value 1..33, 34 = stuffing, 35 = start code */
static const char *const MBA_BITS[36] = {
    NULL,          "1",           "011",         "010",         "0011",        "0010",
    "0001 1",      "0001 0",      "0000 111",    "0000 110",    "0000 1011",   "0000 1010",
    "0000 1001",   "0000 1000",   "0000 0111",   "0000 0110",   "0000 0101 11",
    "0000 0101 10", "0000 0101 01", "0000 0101 00", "0000 0100 11", "0000 0100 10",
    "0000 0100 011", "0000 0100 010", "0000 0100 001", "0000 0100 000", "0000 0011 111",
    "0000 0011 110", "0000 0011 101", "0000 0011 100", "0000 0011 011", "0000 0011 010",
    "0000 0011 001", "0000 0011 000", "0000 0001 111", "0000 0000 0000 0001"};
/* Table 2 (MTYPE 0..9) */
static const char *const MTYPE_BITS[10] = {"0001",      "0000 001", "1",          "0000 1",
                                           "0000 0000 1", "0000 0001", "0000 0000 01", "001",
                                           "01",        "0000 01"};
/* Table 3 (MVD): magnitude 1..15 -> code of +k (code of -k = same with the last
 * bit set); 0 -> "1"; -16 (== +16 mod 32) -> its own code */
static const char *const MVD_POS_BITS[16] = {
    "1",           "010",         "0010",        "0001 0",      "0000 110",    "0000 1010",
    "0000 1000",   "0000 0110",   "0000 0101 10", "0000 0101 00", "0000 0100 10",
    "0000 0100 010", "0000 0100 000", "0000 0011 110", "0000 0011 100", "0000 0011 010"};
static const char *const MVD_M16_BITS = "0000 0011 001";
/* Table 4 (CBP 1..63) */
static const struct {
  int cbp;
  const char *bits;
} CBP_TAB[63] = {
    {60, "111"},        {4, "1101"},        {8, "1100"},        {16, "1011"},
    {32, "1010"},       {12, "1001 1"},     {48, "1001 0"},     {20, "1000 1"},
    {40, "1000 0"},     {28, "0111 1"},     {44, "0111 0"},     {52, "0110 1"},
    {56, "0110 0"},     {1, "0101 1"},      {61, "0101 0"},     {2, "0100 1"},
    {62, "0100 0"},     {24, "0011 11"},    {36, "0011 10"},    {3, "0011 01"},
    {63, "0011 00"},    {5, "0010 111"},    {9, "0010 110"},    {17, "0010 101"},
    {33, "0010 100"},   {6, "0010 011"},    {10, "0010 010"},   {18, "0010 001"},
    {34, "0010 000"},   {7, "0001 1111"},   {11, "0001 1110"},  {19, "0001 1101"},
    {35, "0001 1100"},  {13, "0001 1011"},  {49, "0001 1010"},  {21, "0001 1001"},
    {41, "0001 1000"},  {14, "0001 0111"},  {50, "0001 0110"},  {22, "0001 0101"},
    {42, "0001 0100"},  {15, "0001 0011"},  {51, "0001 0010"},  {23, "0001 0001"},
    {43, "0001 0000"},  {25, "0000 1111"},  {37, "0000 1110"},  {26, "0000 1101"},
    {38, "0000 1100"},  {29, "0000 1011"},  {45, "0000 1010"},  {53, "0000 1001"},
    {57, "0000 1000"},  {30, "0000 0111"},  {46, "0000 0110"},  {54, "0000 0101"},
    {58, "0000 0100"},  {31, "0000 0011 1"}, {47, "0000 0011 0"}, {55, "0000 0010 1"},
    {59, "0000 0010 0"}, {27, "0000 0001 1"}, {39, "0000 0001 0"}};
/* Table 5 (TCOEFF), codes without the trailing sign bit.  (0,1) is "11" except
 * as the first coefficient of a CBP block, where it is "1" (TCoeff2 vs TCoeff1,
 * codec.c:141 / :96). */
static const struct {
  int run, level;
  const char *bits;
} TC_TAB[] = {
    {0, 1, "11"},            {0, 2, "0100"},           {0, 3, "0010 1"},
    {0, 4, "0000 110"},      {0, 5, "0010 0110"},      {0, 6, "0010 0001"},
    {0, 7, "0000 0010 10"},  {0, 8, "0000 0001 1101"}, {0, 9, "0000 0001 1000"},
    {0, 10, "0000 0001 0011"}, {0, 11, "0000 0001 0000"}, {0, 12, "0000 0000 1101 0"},
    {0, 13, "0000 0000 1100 1"}, {0, 14, "0000 0000 1100 0"}, {0, 15, "0000 0000 1011 1"},
    {1, 1, "011"},           {1, 2, "0001 10"},        {1, 3, "0010 0101"},
    {1, 4, "0000 0011 00"},  {1, 5, "0000 0001 1011"}, {1, 6, "0000 0000 1011 0"},
    {1, 7, "0000 0000 1010 1"}, {2, 1, "0101"},        {2, 2, "0000 100"},
    {2, 3, "0000 0010 11"},  {2, 4, "0000 0001 0100"}, {2, 5, "0000 0000 1010 0"},
    {3, 1, "0011 1"},        {3, 2, "0010 0100"},      {3, 3, "0000 0001 1100"},
    {3, 4, "0000 0000 1001 1"}, {4, 1, "0011 0"},      {4, 2, "0000 0011 11"},
    {4, 3, "0000 0001 0010"}, {5, 1, "0001 11"},       {5, 2, "0000 0010 01"},
    {5, 3, "0000 0000 1001 0"}, {6, 1, "0001 01"},     {6, 2, "0000 0001 1110"},
    {7, 1, "0001 00"},       {7, 2, "0000 0001 0101"}, {8, 1, "0000 111"},
    {8, 2, "0000 0001 0001"}, {9, 1, "0000 101"},      {9, 2, "0000 0000 1000 1"},
    {10, 1, "0010 0111"},    {10, 2, "0000 0000 1000 0"}, {11, 1, "0010 0011"},
    {12, 1, "0010 0010"},    {13, 1, "0010 0000"},     {14, 1, "0000 0011 10"},
    {15, 1, "0000 0011 01"}, {16, 1, "0000 0010 00"},  {17, 1, "0000 0001 1111"},
    {18, 1, "0000 0001 1010"}, {19, 1, "0000 0001 1001"}, {20, 1, "0000 0001 0111"},
    {21, 1, "0000 0001 0110"}, {22, 1, "0000 0000 1111 1"}, {23, 1, "0000 0000 1111 0"},
    {24, 1, "0000 0000 1110 1"}, {25, 1, "0000 0000 1110 0"}, {26, 1, "0000 0000 1101 1"}};
static const char *const TC_EOB_BITS = "10";
static const char *const TC_ESC_BITS = "0000 01";
static const char *const TC_FIRST01_BITS = "1";

#define TC_RUNS 27
#define TC_LEVELS 16
/* decoded TCOEFF symbols: run << 8 | level, or these */
#define SYM_EOB 0
#define SYM_ESC 0x7fff

typedef struct {
  uint16_t code;
  uint8_t len;
} venc;
typedef struct {
  int16_t val;
  uint8_t len;  /* 0 = invalid prefix */
} vdec;

#define MBA_BITS_MAX 16
#define MTYPE_BITS_MAX 10
#define MVD_BITS_MAX 11
#define CBP_BITS_MAX 9
#define TC_BITS_MAX 13

static venc E_MBA[36], E_MTYPE[10], E_MVD[32], E_CBP[64], E_TC[TC_RUNS][TC_LEVELS];
static venc E_TC_FIRST01, E_EOB, E_ESC;
static vdec D_MBA[1 << MBA_BITS_MAX], D_MTYPE[1 << MTYPE_BITS_MAX], D_MVD[1 << MVD_BITS_MAX],
    D_CBP[1 << CBP_BITS_MAX], D_TC_NEXT[1 << TC_BITS_MAX], D_TC_FIRST[1 << TC_BITS_MAX];
static int g_tables_ok;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static venc parse_bits(const char *s) {
  venc e = {0, 0};
  for (; *s; s++) {
    if (*s == ' ') continue;
    e.code = (uint16_t)(e.code << 1 | (*s == '1'));
    e.len++;
  }
  return e;
}

/* fills every decode entry whose top bits are the code; 0 on a prefix clash */
static int add_dec(vdec *tab, int maxbits, venc e, int val) {
  const int lo = e.code << (maxbits - e.len), n = 1 << (maxbits - e.len);
  for (int i = 0; i < n; i++) {
    if (tab[lo + i].len) return 0;
    tab[lo + i].val = (int16_t)val;
    tab[lo + i].len = e.len;
  }
  return 1;
}

static void build_tables(void) {
  int ok = 1;
  for (int v = 1; v < 36; v++) {
    E_MBA[v] = parse_bits(MBA_BITS[v]);
    ok &= add_dec(D_MBA, MBA_BITS_MAX, E_MBA[v], v);
  }
  for (int v = 0; v < 10; v++) {
    E_MTYPE[v] = parse_bits(MTYPE_BITS[v]);
    ok &= add_dec(D_MTYPE, MTYPE_BITS_MAX, E_MTYPE[v], v);
  }
  for (int k = 0; k < 16; k++) {
    venc e = parse_bits(MVD_POS_BITS[k]);
    E_MVD[k] = e;
    if (k) {
      e.code |= 1;
      E_MVD[32 - k] = e;
    }
  }
  E_MVD[16] = parse_bits(MVD_M16_BITS);
  for (int v = 0; v < 32; v++) ok &= add_dec(D_MVD, MVD_BITS_MAX, E_MVD[v], v);
  for (int i = 0; i < 63; i++) {
    E_CBP[CBP_TAB[i].cbp] = parse_bits(CBP_TAB[i].bits);
    ok &= add_dec(D_CBP, CBP_BITS_MAX, E_CBP[CBP_TAB[i].cbp], CBP_TAB[i].cbp);
  }
  E_EOB = parse_bits(TC_EOB_BITS);
  E_ESC = parse_bits(TC_ESC_BITS);
  E_TC_FIRST01 = parse_bits(TC_FIRST01_BITS);
  for (size_t i = 0; i < sizeof TC_TAB / sizeof TC_TAB[0]; i++) {
    const venc e = parse_bits(TC_TAB[i].bits);
    const int sym = TC_TAB[i].run << 8 | TC_TAB[i].level;
    E_TC[TC_TAB[i].run][TC_TAB[i].level] = e;
    ok &= add_dec(D_TC_NEXT, TC_BITS_MAX, e, sym);
    if (sym != 1) ok &= add_dec(D_TC_FIRST, TC_BITS_MAX, e, sym);
  }
  ok &= add_dec(D_TC_NEXT, TC_BITS_MAX, E_EOB, SYM_EOB);
  ok &= add_dec(D_TC_NEXT, TC_BITS_MAX, E_ESC, SYM_ESC);
  ok &= add_dec(D_TC_FIRST, TC_BITS_MAX, E_ESC, SYM_ESC);
  ok &= add_dec(D_TC_FIRST, TC_BITS_MAX, E_TC_FIRST01, 1);
  g_tables_ok = ok;
}

static int tables(void) {
  pthread_once(&g_once, build_tables);
  return g_tables_ok ? 0 : fail(P64GPU_E_STREAM, "VLC tables are not prefix-free");
}

/* internal (p64vlc.hip): the encode tables as code | len << 16 words --
 * mtype[10], mvd[32], cbp[64], tcoeff[27][16], then EOB, ESCAPE, first-(0,1) */
int p64s_vlc_tables_(uint32_t *t) {
  int s = tables();
  if (s) return s;
  uint32_t *p = t;
#define PUT(e) (*p++ = (uint32_t)(e).code | (uint32_t)(e).len << 16)
  for (int i = 0; i < 10; i++) PUT(E_MTYPE[i]);
  for (int i = 0; i < 32; i++) PUT(E_MVD[i]);
  for (int i = 0; i < 64; i++) PUT(E_CBP[i]);
  for (int r = 0; r < TC_RUNS; r++)
    for (int l = 0; l < TC_LEVELS; l++) PUT(E_TC[r][l]);
  PUT(E_EOB);
  PUT(E_ESC);
  PUT(E_TC_FIRST01);
#undef PUT
  return 0;
}

/* ---- writer -------------------------------------------------------------- */
struct p64s_writer {
  uint8_t *buf;
  size_t len, cap;
  uint64_t acc; /* pending bits, right-aligned */
  int nacc;
  int64_t bits;
  int ended, oom;
  /* position in the picture: format, GOB (-2 none yet, -1 header only) and the
   * MBA/MTYPE/MVD predictors of WriteMBHeader */
  int format, gob, last_mba, last_mt, pmx, pmy;
};

/* n <= 24 bits, MSB first (mputv stream.c:180-190) */
static void put(p64s_writer *w, int n, uint32_t v) {
  w->acc = (w->acc << n) | (v & ((1u << n) - 1u));
  w->nacc += n;
  w->bits += n;
  while (w->nacc >= 8) {
    if (w->len == w->cap) {
      size_t cap = w->cap ? 2 * w->cap : 1 << 16;
      uint8_t *b = (uint8_t *)realloc(w->buf, cap);
      if (!b) {
        w->oom = 1;
        w->nacc -= 8;
        continue;
      }
      w->buf = b;
      w->cap = cap;
    }
    w->nacc -= 8;
    w->buf[w->len++] = (uint8_t)(w->acc >> w->nacc);
  }
}

static inline void put_vlc(p64s_writer *w, venc e) { put(w, e.len, e.code); }

int p64s_writer_open(p64s_writer **out) {
  if (!out) return fail(P64GPU_E_INVALID, "writer: out is NULL");
  int s = tables();
  if (s) return s;
  *out = (p64s_writer *)calloc(1, sizeof(p64s_writer));
  if (!*out) return fail(P64GPU_E_NOMEM, "writer: calloc failed");
  (*out)->gob = -2;
  return 0;
}

void p64s_writer_close(p64s_writer *w) {
  if (!w) return;
  free(w->buf);
  free(w);
}

const uint8_t *p64s_writer_data(const p64s_writer *w, size_t *len, int64_t *bits) {
  if (len) *len = w ? w->len : 0;
  if (bits) *bits = w ? w->bits : 0;
  return w ? w->buf : NULL;
}

int p64s_writer_consume(p64s_writer *w, size_t n) {
  if (!w || n > w->len) return fail(P64GPU_E_INVALID, "writer_consume: %zu bytes", n);
  memmove(w->buf, w->buf + n, w->len - n);
  w->len -= n;
  return 0;
}

int p64s_writer_phase(const p64s_writer *w) { return w ? w->nacc : 0; }

int p64s_write_bits(p64s_writer *w, const uint8_t *data, int64_t bits, int phase) {
  if (!w || (!data && bits) || phase < 0 || phase > 7 || bits < phase)
    return fail(P64GPU_E_INVALID, "write_bits: bad arguments");
  if (w->ended) return fail(P64GPU_E_INVALID, "write after write_end");
  if (phase != w->nacc) return fail(P64GPU_E_INVALID, "write_bits: phase %d, writer at %d", phase, w->nacc);
  /* the coded picture continues the stream at bit `phase` of data[0] */
  int64_t pos = phase;
  while (pos < bits) {
    const int n = (int)((bits - pos) < 16 ? (bits - pos) : 16);
    const int64_t byte = pos >> 3;
    uint32_t v = (uint32_t)data[byte] << 16;
    if (pos + n > (byte + 1) * 8) v |= (uint32_t)data[byte + 1] << 8;
    if (pos + n > (byte + 2) * 8) v |= data[byte + 2];
    v = (v << (pos & 7)) >> (24 - n) & ((1u << n) - 1u);
    put(w, n, v);
    pos += n;
  }
  return w->oom ? fail(P64GPU_E_NOMEM, "writer: out of memory") : 0;
}

/* WritePictureHeader, marker.c:103-135 (non-VERSION_1_0): PSC, TR, PTYPE,
 * PSPARE for NTSC (p64.c:417-419), PEI = 0 */
static void write_picture_header(p64s_writer *w, int format, int tr) {
  put(w, 20, 0x10);
  put(w, 5, (uint32_t)tr & 31u);
  put(w, 6, format == P64S_QCIF ? 0x00 : 0x04);
  if (format == P64S_NTSC) {
    put(w, 1, 1);
    put(w, 8, 0x8c);
  }
  put(w, 1, 0);
}

/* one (run, level) event: the table code and sign bit, or ESCAPE + 6-bit run +
 * 8-bit two's-complement level when the pair has no code (codec.c:110-124;
 * Encode() huffman.c:232-252 declines values >= table size or without a code,
 * and the value 0x1b01 = run 27 level 1 collides with ESCAPE's own entry) */
static void write_level(p64s_writer *w, int run, int l, int first_of_cbp) {
  const int a = l < 0 ? -l : l;
  venc e = {0, 0};
  if (run < TC_RUNS && a < TC_LEVELS) e = (first_of_cbp && run == 0 && a == 1) ? E_TC_FIRST01 : E_TC[run][a];
  if (e.len) {
    put_vlc(w, e);
    put(w, 1, l < 0);
  } else {
    put_vlc(w, E_ESC);
    put(w, 6, (uint32_t)run);
    put(w, 8, (uint32_t)l);
  }
}

/* EncodeAC(1,...) codec.c:96 and CBPEncodeAC(0,...) codec.c:141 */
static void write_block(p64s_writer *w, const int16_t *z, int intra) {
  int k = 0, r = 0, first = !intra;
  if (intra) {
    int dc = z[0]; /* EncodeDC codec.c:343-352 */
    if (dc > 254) dc = 254;
    if (dc < 1) dc = 1;
    if (dc == 128) dc = 255;
    put(w, 8, (uint32_t)dc);
    k = 1;
  } else {
    int any = 0;
    for (int i = 0; i < 64; i++) any |= z[i];
    if (!any) return; /* "CBP block without any coefficients": nothing, no EOB */
  }
  for (; k < 64; k++) {
    const int l = z[k];
    if (!l) {
      r++;
      continue;
    }
    write_level(w, r, l, first);
    first = 0;
    r = 0;
  }
  put_vlc(w, E_EOB);
}

static int check_mb(const p64_mb_rec *r, int mquant, int k) {
  const int mt = r->mtype;
  if (mt < 0 || mt > 9) return fail(P64GPU_E_INVALID, "mb %d: mtype %d", k, mt);
  if (CBP_MT[mt] && (r->cbp < 1 || r->cbp > 63))
    return fail(P64GPU_E_INVALID, "mb %d: mtype %d with cbp %d", k, mt, r->cbp);
  if (QUANT_MT[mt] && (mquant < 1 || mquant > 31))
    return fail(P64GPU_E_INVALID, "mb %d: mtype %d needs MQUANT in 1..31, got %d", k, mt, mquant);
  return 0;
}

int p64s_write_picture_header(p64s_writer *w, int format, int tr) {
  int s;
  if (!w) return fail(P64GPU_E_INVALID, "write_picture_header: NULL writer");
  if (w->ended) return fail(P64GPU_E_INVALID, "write after write_end");
  if ((s = p64s_geometry(format, NULL, NULL, NULL))) return s;
  write_picture_header(w, format, tr);
  w->format = format;
  w->gob = -1;
  return 0;
}

/* WriteGOBHeader marker.c:171-198: GBSC, GN = GRead+1 (QCIF GRead = 2g,
 * p64.c:703-712), GQUANT, GEI = 0; resets the MBA/MVD predictors (p64.c:716) */
int p64s_write_gob_header(p64s_writer *w, int gob, int gquant) {
  int ngob;
  if (!w) return fail(P64GPU_E_INVALID, "write_gob_header: NULL writer");
  if (w->ended || w->gob == -2) return fail(P64GPU_E_INVALID, "GOB header outside a picture");
  p64s_geometry(w->format, NULL, NULL, &ngob);
  if (gob < 0 || gob >= ngob) return fail(P64GPU_E_INVALID, "gob %d of %d", gob, ngob);
  if (gquant < 1 || gquant > 31) return fail(P64GPU_E_INVALID, "gquant %d", gquant);
  put(w, 16, 1);
  put(w, 4, (uint32_t)(w->format == P64S_QCIF ? 2 * gob + 1 : gob + 1));
  put(w, 5, (uint32_t)gquant);
  put(w, 1, 0);
  w->gob = gob;
  w->last_mba = -1;
  w->last_mt = 0;
  w->pmx = w->pmy = 0;
  return w->oom ? fail(P64GPU_E_NOMEM, "writer: out of memory") : 0;
}

/* WriteMBHeader marker.c:288-357 + the coefficient half of WriteMDU p64.c:929-944 */
static void write_mb(p64s_writer *w, int mdu, const p64_mb_rec *r, const int16_t *coef, int mquant) {
  const int mt = r->mtype, mba = mdu - w->last_mba;
  put_vlc(w, E_MBA[mba]);
  put_vlc(w, E_MTYPE[mt]);
  if (QUANT_MT[mt]) put(w, 5, (uint32_t)mquant);
  if (MF_MT[mt]) {
    int dh = r->mvx, dv = r->mvy;
    if (MF_MT[w->last_mt] && mba == 1 && w->last_mba != -1 && w->last_mba != 10 && w->last_mba != 21) {
      dh -= w->pmx;
      dv -= w->pmy;
      if (dh < -16) dh += 32;
      if (dh > 15) dh -= 32;
      if (dv < -16) dv += 32;
      if (dv > 15) dv -= 32;
    }
    put_vlc(w, E_MVD[dh & 0x1f]);
    put_vlc(w, E_MVD[dv & 0x1f]);
    w->pmx = r->mvx;
    w->pmy = r->mvy;
  } else {
    w->pmx = w->pmy = 0;
  }
  const int cbp = CBP_MT[mt] ? r->cbp : 0x3f;
  if (CBP_MT[mt]) put_vlc(w, E_CBP[cbp]);
  w->last_mba = mdu;
  if (TC_MT[mt])
    for (int c = 0; c < 6; c++)
      if (cbp & (1 << (5 - c))) write_block(w, coef + c * 64, !CBP_MT[mt]);
  w->last_mt = mt;
}

int p64s_write_mb(p64s_writer *w, int mdu, const p64_mb_rec *mb, const int16_t *coef, int mquant) {
  int s;
  if (!w || !mb || !coef) return fail(P64GPU_E_INVALID, "write_mb: NULL argument");
  if (w->ended || w->gob < 0) return fail(P64GPU_E_INVALID, "macroblock outside a GOB");
  if (mdu <= w->last_mba || mdu >= 33 || mdu - w->last_mba > 33)
    return fail(P64GPU_E_INVALID, "mdu %d after %d", mdu, w->last_mba);
  if ((s = check_mb(mb, mquant, mdu))) return s;
  write_mb(w, mdu, mb, coef, mquant);
  return w->oom ? fail(P64GPU_E_NOMEM, "writer: out of memory") : 0;
}

int p64s_write_picture(p64s_writer *w, int format, int tr, const uint8_t *gquant,
                       const uint8_t *quant_mb, const p64_mb_rec *mb, const int16_t *coef) {
  int ngob, s;
  if (!w || !gquant || !mb || !coef) return fail(P64GPU_E_INVALID, "write_picture: NULL argument");
  if (w->ended) return fail(P64GPU_E_INVALID, "write_picture after write_end");
  if ((s = p64s_geometry(format, NULL, NULL, &ngob))) return s;
  for (int g = 0; g < ngob; g++)
    if (gquant[g] < 1 || gquant[g] > 31) return fail(P64GPU_E_INVALID, "gquant[%d] = %d", g, gquant[g]);
  /* validate before writing so a failed call leaves the stream unchanged */
  for (int k = 0; k < ngob * 33; k++)
    if ((s = check_mb(&mb[k], quant_mb ? quant_mb[k] : 0, k))) return s;
  p64s_write_picture_header(w, format, tr);
  for (int g = 0; g < ngob; g++) {
    p64s_write_gob_header(w, g, gquant[g]);
    for (int m = 0; m < 33; m++) {
      const int k = raster_mb(format, g, m);
      write_mb(w, m, &mb[k], coef + (size_t)k * 384, quant_mb ? quant_mb[k] : 0);
    }
  }
  return w->oom ? fail(P64GPU_E_NOMEM, "writer: out of memory") : 0;
}

int p64s_write_end(p64s_writer *w, int format, int tr) {
  int s;
  if (!w) return fail(P64GPU_E_INVALID, "write_end: NULL writer");
  if (w->ended) return fail(P64GPU_E_INVALID, "write_end called twice");
  if ((s = p64s_geometry(format, NULL, NULL, NULL))) return s;
  write_picture_header(w, format, tr);
  if (w->nacc) put(w, 8 - w->nacc, 0xff); /* mwclose: pad with ones */
  w->ended = 1;
  return w->oom ? fail(P64GPU_E_NOMEM, "writer: out of memory") : 0;
}

/* ---- reader -------------------------------------------------------------- */
struct p64s_reader {
  const uint8_t *data;
  size_t len;
  uint64_t pos; /* bit position */
  p64s_picture_info first;
  int have_psc;  /* a start code + GN 0 (picture header) has been consumed */
  int ended, end_tr, last_tr;
  int mt, mvx, mvy; /* ReadMBHeader's persistent MType / MVDH / MVDV */
  int force_cif;    /* -c: CIF geometry whatever PTYPE says (p64.c:1071-1072) */
  int started;      /* p64s_read_picture has been called */
};

/* n <= 25 bits at the current position without consuming them; bytes past
 * the end read as 0xff (mgetb on EOF, stream.c:154-163) */
static inline uint32_t peek(const p64s_reader *r, int n) {
  const uint64_t byte = r->pos >> 3;
  uint32_t v = 0;
  for (int i = 0; i < 4; i++) v = v << 8 | (byte + i < r->len ? r->data[byte + i] : 0xffu);
  return (v << (r->pos & 7)) >> (32 - n);
}
static inline uint32_t get(p64s_reader *r, int n) {
  const uint32_t v = peek(r, n);
  r->pos += (uint64_t)n;
  return v;
}
static inline int past_end(const p64s_reader *r) { return r->pos > (uint64_t)r->len * 8; }
static inline int at_end(const p64s_reader *r) { return r->pos >= (uint64_t)r->len * 8; }

static int get_vlc(p64s_reader *r, const vdec *tab, int maxbits, int *val) {
  const vdec d = tab[peek(r, maxbits)];
  if (!d.len) return 0;
  r->pos += d.len;
  *val = d.val;
  return 1;
}

#define BAD(...)                                               \
  do {                                                         \
    return fail(P64GPU_E_STREAM, __VA_ARGS__);                 \
  } while (0)

/* ReadPictureHeader marker.c:142-165 (after PSC and GN = 0) */
static void read_picture_header(p64s_reader *r, p64s_picture_info *pi) {
  pi->tr = (int)get(r, 5);
  pi->ptype = (int)get(r, 6);
  pi->pspare = -1;
  while (get(r, 1)) pi->pspare = (int)get(r, 8);
}

int p64s_reader_open(const uint8_t *data, size_t len, p64s_reader **out) {
  if (!out || (!data && len)) return fail(P64GPU_E_INVALID, "reader_open: NULL argument");
  int s = tables();
  if (s) return s;
  p64s_reader *r = (p64s_reader *)calloc(1, sizeof(p64s_reader));
  if (!r) return fail(P64GPU_E_NOMEM, "reader: calloc failed");
  r->data = data;
  r->len = len;
  /* ReadHeaderHeader + ReadHeaderTrailer: the stream must open with a PSC */
  if (len < 4 || get(r, 16) != 1 || get(r, 4) != 0) {
    free(r);
    return fail(P64GPU_E_STREAM, "stream does not start with a picture start code");
  }
  const uint64_t save = r->pos;
  p64s_picture_info pi;
  read_picture_header(r, &pi);
  r->pos = save;
  /* image type from PTYPE/PSPARE, p64.c:1071-1081 */
  pi.format = (pi.ptype & 0x04) ? (pi.pspare == 0x8c ? P64S_NTSC : P64S_CIF) : P64S_QCIF;
  p64s_geometry(pi.format, &pi.width, &pi.height, &pi.ngob);
  pi.coded_mbs = 0;
  r->first = pi;
  r->have_psc = 1;
  *out = r;
  return 0;
}

void p64s_reader_close(p64s_reader *r) { free(r); }

int p64s_reader_force_cif(p64s_reader *r) {
  if (!r) return fail(P64GPU_E_INVALID, "reader_force_cif: NULL reader");
  /* the caller sized its arrays from the geometry reader_info gave: changing
   * it once pictures are being read would overrun them */
  if (r->started) return fail(P64GPU_E_INVALID, "reader_force_cif: pictures already read");
  r->force_cif = 1;
  r->first.format = P64S_CIF;
  p64s_geometry(P64S_CIF, &r->first.width, &r->first.height, &r->first.ngob);
  return 0;
}

int p64s_reader_info(const p64s_reader *r, p64s_picture_info *info) {
  if (!r || !info) return fail(P64GPU_E_INVALID, "reader_info: NULL argument");
  *info = r->first;
  return 0;
}

/* one (run, level) event; returns 0 at EOB, 1 with an event, <0 on error */
static int read_level(p64s_reader *r, const vdec *tab, int *run, int *level) {
  int sym;
  if (!get_vlc(r, tab, TC_BITS_MAX, &sym)) BAD("invalid TCOEFF code at bit %llu", (unsigned long long)r->pos);
  if (sym == SYM_EOB) return 0;
  if (sym == SYM_ESC) {
    *run = (int)get(r, 6);
    int l = (int)get(r, 8);
    if (l & 0x80) l -= 256; /* extend_mask, codec.c:238 */
    *level = l;
  } else {
    *run = sym >> 8;
    *level = get(r, 1) ? -(sym & 0xff) : (sym & 0xff);
  }
  return 1;
}

/* DecodeAC codec.c:215 (index 1, after DecodeDC) / CBPDecodeAC codec.c:258 */
static int read_block(p64s_reader *r, int16_t *z, int intra) {
  int k = 0, run, level, s;
  if (intra) {
    int dc = (int)get(r, 8); /* DecodeDC codec.c:326-334 */
    z[0] = (int16_t)(dc == 255 ? 128 : dc);
    k = 1;
  } else {
    if ((s = read_level(r, D_TC_FIRST, &run, &level)) < 0) return s;
    if (s == 0) BAD("EOB as first coefficient of a CBP block");
    k += run;
    if (k > 63) BAD("coefficient run past the block end");
    z[k++] = (int16_t)level;
  }
  while (k < 64) {
    if ((s = read_level(r, D_TC_NEXT, &run, &level)) < 0) return s;
    if (s == 0) return 0;
    k += run;
    if (k > 63) BAD("coefficient run past the block end");
    z[k++] = (int16_t)level;
  }
  /* 64 coefficients without EOB: the reference reads one more code and
   * expects EOB (codec.c:248-252) */
  if ((s = read_level(r, D_TC_NEXT, &run, &level)) < 0) return s;
  if (s) BAD("EOB expected after 64 coefficients");
  return 0;
}

int p64s_read_picture(p64s_reader *r, p64s_picture_info *info, p64_mb_rec *mb, uint8_t *quant_mb,
                      uint8_t *coded, int16_t *coef) {
  if (!r || !info || !mb || !quant_mb || !coded || !coef)
    return fail(P64GPU_E_INVALID, "read_picture: NULL argument");
  r->started = 1;
  p64s_picture_info pi = r->first;
  const int nmb = pi.ngob * 33;
  memset(mb, 0, (size_t)nmb * sizeof *mb);
  memset(quant_mb, 0, (size_t)nmb);
  memset(coded, 0, (size_t)nmb);
  memset(coef, 0, (size_t)nmb * 384 * sizeof *coef);
  if (r->ended || !r->have_psc) {
    pi.tr = r->end_tr;
    *info = pi;
    return 0;
  }
  read_picture_header(r, &pi);
  if (!r->force_cif &&
      ((pi.ptype & 0x04) ? (pi.pspare == 0x8c ? P64S_NTSC : P64S_CIF) : P64S_QCIF) != r->first.format)
    BAD("picture format changes mid-stream");
  r->have_psc = 0;
  /* no start code after the header: it was the trailing picture header
   * (p64.c:1114-1115) */
  if (get(r, 16) != 1) {
    r->ended = 1;
    r->end_tr = pi.tr;
    *info = pi;
    return 0;
  }
  int gn = (int)get(r, 4), ncoded = 0;
  while (gn != 0) {
    /* ReadGOBHeader marker.c:245-267; GOB number p64DecodeGOB p64.c:1136-1148 */
    int gq = (int)get(r, 5), g = pi.format == P64S_QCIF ? (gn - 1) >> 1 : gn - 1;
    while (get(r, 1)) get(r, 8);
    if (g >= pi.ngob) BAD("GOB number %d out of range", gn);
    int last_mba = -1, end_of_data = 0;
    for (;;) { /* ReadMBHeader marker.c:372-418 */
      if (at_end(r)) {
        end_of_data = 1;
        break;
      }
      int mba;
      do {
        if (!get_vlc(r, D_MBA, MBA_BITS_MAX, &mba)) BAD("invalid MBA code at bit %llu", (unsigned long long)r->pos);
      } while (mba == 34);
      if (mba == 35) break; /* start code: next GOB or picture */
      const int last_mt = r->mt;
      int mt;
      if (!get_vlc(r, D_MTYPE, MTYPE_BITS_MAX, &mt)) BAD("invalid MTYPE code");
      r->mt = mt;
      if (QUANT_MT[mt]) gq = (int)get(r, 5); /* MQUANT becomes GQuant, p64.c:1205-1208 */
      if (MF_MT[mt]) {
        int dh, dv;
        if (!get_vlc(r, D_MVD, MVD_BITS_MAX, &dh) || !get_vlc(r, D_MVD, MVD_BITS_MAX, &dv))
          BAD("invalid MVD code");
        if (dh & 16) dh -= 32;
        if (dv & 16) dv -= 32;
        if (!MF_MT[last_mt] || mba != 1 || last_mba == -1 || last_mba == 10 || last_mba == 21) {
          r->mvx = dh;
          r->mvy = dv;
        } else {
          r->mvx += dh;
          r->mvy += dv;
          if (r->mvx < -16) r->mvx += 32;
          if (r->mvx > 15) r->mvx -= 32;
          if (r->mvy < -16) r->mvy += 32;
          if (r->mvy > 15) r->mvy -= 32;
        }
      } else {
        r->mvx = r->mvy = 0;
      }
      int cbp = 0x3f;
      if (CBP_MT[mt] && !get_vlc(r, D_CBP, CBP_BITS_MAX, &cbp)) BAD("invalid CBP code");
      const int mdu = last_mba + mba; /* DecompressMDU p64.c:1186-1201 */
      if (mdu >= 33) BAD("MDU %d out of range in GOB %d", mdu, gn);
      last_mba = mdu;
      const int k = raster_mb(pi.format, g, mdu);
      if (MF_MT[mt]) { /* the vector must keep the 16x16 source inside the picture */
        const int mbw = pi.width / 16, px = 16 * (k % mbw) + r->mvx, py = 16 * (k / mbw) + r->mvy;
        if (px < 0 || px > pi.width - 16 || py < 0 || py > pi.height - 16)
          BAD("motion vector (%d,%d) points outside the picture at MB %d", r->mvx, r->mvy, k);
      }
      mb[k].mtype = (int8_t)mt;
      mb[k].cbp = (int8_t)cbp;
      mb[k].mvx = (int8_t)r->mvx;
      mb[k].mvy = (int8_t)r->mvy;
      quant_mb[k] = (uint8_t)gq;
      if (!coded[k]) ncoded++;
      coded[k] = 1;
      int16_t *z = coef + (size_t)k * 384;
      memset(z, 0, 384 * sizeof *z);
      if (TC_MT[mt])
        for (int c = 0; c < 6; c++)
          if (cbp & (1 << (5 - c))) {
            int s = read_block(r, z + c * 64, !CBP_MT[mt]);
            if (s) return s;
          }
      if (past_end(r)) BAD("stream truncated inside a macroblock");
    }
    if (end_of_data) { /* EOF inside the picture: EndFrame, p64.c:1040-1046 */
      r->ended = 1;
      r->end_tr = (pi.tr + 1) & 31;
      break;
    }
    gn = (int)get(r, 4);
  }
  if (!r->ended) r->have_psc = 1; /* the PSC of the next picture was consumed */
  pi.coded_mbs = ncoded;
  r->last_tr = pi.tr;
  *info = pi;
  return 1;
}

/* the packed level layout of p64gpu_decode_recon_packed: the blocks the
 * stream carries (DecompressMDU p64.c:1200-1217: TCOEFF types, CBP bit) in
 * raster order, and per group of 64 blocks of a picture its first block's
 * index and its mask */
int64_t p64s_pack_levels(int format, int nframes, const p64_mb_rec *mb, const uint8_t *coded,
                         const int16_t *coef, int16_t *levels, uint32_t *index) {
  if (format < P64S_QCIF || format > P64S_NTSC || nframes < 0 || !mb || !coded || !coef || !levels || !index)
    return fail(P64GPU_E_INVALID, "pack_levels: bad arguments");
  int ngob = 0;
  p64s_geometry(format, NULL, NULL, &ngob);
  const int64_t nmb = (int64_t)ngob * 33, nball = 6 * nmb * nframes, ngr = (nball + 63) / 64;
  int64_t n = 0;
  for (int64_t j = 0; j < ngr; j++) {  // groups of 64 consecutive blocks of the batch
    uint64_t m = 0;
    const int64_t start = n;
    for (int i = 0; i < 64 && 64 * j + i < nball; i++) {
      const int64_t blk = 64 * j + i, k = blk / 6;  // (k: the MB over the batch)
      const int b = (int)(blk % 6), mt = mb[k].mtype;
      if (mt < 0 || mt > 9) return fail(P64GPU_E_INVALID, "pack_levels: MTYPE %d at MB %lld", mt, (long long)k);
      const int cbp = CBP_MT[mt] ? mb[k].cbp : 0x3f;
      if (coded[k] && TC_MT[mt] && ((cbp >> (5 - b)) & 1)) {
        memcpy(levels + n * 64, coef + (k * 6 + b) * 64, 64 * sizeof *levels);
        m |= 1ull << i;
        n++;
      }
    }
    uint32_t *e = index + 4 * j;
    e[0] = (uint32_t)start;
    e[1] = 0;
    e[2] = (uint32_t)m;
    e[3] = (uint32_t)(m >> 32);
  }
  return n;
}
