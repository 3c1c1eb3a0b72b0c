/*
 * p64prog.h -- the reference's program interpreter (the -o "oracle", lexer.l)
 * for the decision policy around the GPU hot path (host C, libp64gpu.so).
 *
 * A program file is a stream of top-level statements (executed as read) and
 * `open N ... close` blocks that define programs 0..9 for a small stack
 * machine over doubles (lexer.l:660-1090, mylex lexer.l:1440-1510).  The
 * encoder calls program 0 per macroblock to choose MTYPE and program 1 for
 * the quantiser under rate control (CallOracle p64.c:489-515), after storing
 * its state in Memory[1..14] (names GQUANT .. QOFFS, lexer.l:144-173).
 *
 * Semantics kept from the reference: case-insensitive words, nested comments,
 * the number syntaxes of the scanner (decimal, 0x/0o, ...h/...b suffixes,
 * 'c' characters, reals), global labels and equ names, a data stack and
 * Memory that persist across calls, EXIT/running off the end returning to
 * the caller.  Where the reference would read or write outside its arrays,
 * this implementation stops with P64GPU_E_INVALID instead.
 */
#ifndef P64PROG_H
#define P64PROG_H

#include <stddef.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Memory locations the encoder fills before a call (lexer.l:160-173) */
enum p64prog_loc {
  P64PROG_GQUANT = 1, P64PROG_MQUANT = 2, P64PROG_MQUANTENABLE = 3, P64PROG_MTYPE = 4,
  P64PROG_BD = 5, P64PROG_DBD = 6, P64PROG_VAROR = 7, P64PROG_VAR = 8, P64PROG_MWOR = 9,
  P64PROG_RATE = 10, P64PROG_BUFFERSIZE = 11, P64PROG_BUFFERCONTENTS = 12, P64PROG_QDFACT = 13,
  P64PROG_QOFFS = 14
};

/* Settings a program file may make at top level (lexer.l:1033-1083);
 * -1 / NULL where the file leaves the command line's value. */
typedef struct {
  int quantization, search_limit, frame_rate, frame_skip;
  int image_type;   /* 0 QCIF, 1 CIF, 2 NTSC (P64S_*), -1 unset */
  int abort_code;   /* ABORT n at top level: the reference exits with n; -1 none */
} p64prog_settings;

typedef struct p64prog p64prog;
/* Scans and runs the top-level statements of text (len bytes).  out receives
 * what ECHO/PRINTSTACK/PRINTPROGRAM and diagnostics print (NULL: silent). */
int p64prog_load(const char *text, size_t len, FILE *out, p64prog **prog);
void p64prog_free(p64prog *p);
int p64prog_settings_get(const p64prog *p, p64prog_settings *s);
/* 1 if program n (0..9) has been defined with at least one instruction */
int p64prog_defined(const p64prog *p, int n);
/* 1 if running program n may read Memory[loc] (RCL loc in n or in a program
 * it can EXE, transitively) */
int p64prog_reads(const p64prog *p, int n, int loc);
/* Execute(n) (lexer.l:1517): runs program n to its EXIT; no-op if undefined */
int p64prog_execute(p64prog *p, int n);
double *p64prog_memory(p64prog *p); /* Memory[0..1023] */

#ifdef __cplusplus
}
#endif

#endif /* P64PROG_H */
