/*
 * p64prog.c -- the reference's program interpreter (include/p64prog.h).
 *
 * Structure follows the behaviour of lexer.l, re-expressed: a scanner over the
 * program text, a top-level executor, a compiler of `open N ... close` blocks
 * into (opcode, operand) cells with a constant pool, and one token source that
 * feeds the executor either from the text or from the running program (the
 * role of mylex, lexer.l:1440-1510), so top-level code and programs share the
 * same operation semantics, data stack and Memory.
 */
#include <ctype.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/p64gpu.h"
#include "../../include/p64prog.h"

int p64gpu_fail_(int status, const char *msg); /* p64gpu_abi.hip: sets last error */

/* reserved words, lexer.l:27-79, in token order 1..52 */
static const char *const WORDS[] = {
    "ADD",  "SUB",   "MUL",    "DIV",   "NOT",   "AND",   "OR",   "XOR",        "LT",
    "LTE",  "EQ",    "GT",     "GTE",   "NEG",   "SQRT",  "ABS",  "FLOOR",      "CEIL",
    "ROUND", "DUP",  "POP",    "EXCH",  "COPY",  "ROLL",  "INDEX", "CLEAR",     "STO",
    "RCL",  "GOTO",  "IFG",    "IFNG",  "EXIT",  "EXE",   "ABORT", "PRINTSTACK", "PRINTPROGRAM",
    "PRINTIMAGE", "PRINTFRAME", "ECHO", "OPEN", "CLOSE", "EQU", "VAL", "STREAMNAME", "COMPONENT",
    "FRAMERATE", "FRAMESKIP", "QUANTIZATION", "SEARCHLIMIT", "NTSC", "CIF", "QCIF"};
enum {
  T_ADD = 1, T_SUB, T_MUL, T_DIV, T_NOT, T_AND, T_OR, T_XOR, T_LT, T_LTE, T_EQ, T_GT, T_GTE,
  T_NEG, T_SQRT, T_ABS, T_FLOOR, T_CEIL, T_ROUND, T_DUP, T_POP, T_EXCH, T_COPY, T_ROLL, T_INDEX,
  T_CLEAR, T_STO, T_RCL, T_GOTO, T_IFG, T_IFNG, T_EXIT, T_EXE, T_ABORT, T_PRINTSTACK,
  T_PRINTPROGRAM, T_PRINTIMAGE, T_PRINTFRAME, T_ECHO, T_OPEN, T_CLOSE, T_EQU, T_VAL,
  T_STREAMNAME, T_COMPONENT, T_FRAMERATE, T_FRAMESKIP, T_QUANTIZATION, T_SEARCHLIMIT, T_NTSC,
  T_CIF, T_QCIF,
  T_INTEGER = 1000, T_LBRACKET, T_RBRACKET, T_ID, T_STRING, T_REAL, T_EOF = 0
};
/* Memory names, lexer.l:144-158 */
static const char *const EQU_NAMES[] = {"GQUANT", "MQUANT", "MQUANTENABLE", "MTYPE", "BD", "DBD",
                                        "VAROR", "VAR", "MWOR", "RATE", "BUFFERSIZE",
                                        "BUFFERCONTENTS", "QDFACT", "QOFFS"};

#define NPROG 10
#define MEMTOP 1024
#define MAXLINES 2000
#define MAXNAMES 1024
#define MAXDEPTH 16

typedef struct {
  char name[64];
  int token; /* reserved word token, 0 for an identifier */
  int value; /* equ value / label position; -1 = unset (MakeLink lexer.l:530) */
} name_t;

typedef struct {
  int type;
  int ival;
  double rval;
  name_t *id;
  char str[256];
} token_t;

struct p64prog {
  const char *src;
  size_t len, pos;
  int comment_depth;
  FILE *out;
  name_t names[MAXNAMES];
  int nnames;
  double stack[MEMTOP];
  int level; /* DataLevel */
  double mem[MEMTOP];
  int code[NPROG][MAXLINES];
  double consts[NPROG][MAXLINES];
  int ncode[NPROG], nconst[NPROG];
  name_t *labels[1000];
  int nlabels;
  /* running programs (SourceLevel stack) */
  int depth, cur_prog, cur_line;
  int saved_prog[MAXDEPTH], saved_line[MAXDEPTH];
  int next_val; /* NextVal: operands to pass through as integers */
  p64prog_settings set;
  int err;
  char errmsg[200];
};

static int bad(p64prog *p, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static int bad(p64prog *p, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  if (!p->err) vsnprintf(p->errmsg, sizeof p->errmsg, fmt, ap);
  va_end(ap);
  p->err = 1;
  return -1;
}
static void say(p64prog *p, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static void say(p64prog *p, const char *fmt, ...) {
  if (!p->out) return;
  va_list ap;
  va_start(ap, fmt);
  vfprintf(p->out, fmt, ap);
  va_end(ap);
}

/* enter() lexer.l:538-573: names are upper-cased */
static name_t *lookup(p64prog *p, const char *s, size_t n, int token) {
  char up[64];
  if (n >= sizeof up) n = sizeof up - 1;
  for (size_t i = 0; i < n; i++) up[i] = (char)toupper((unsigned char)s[i]);
  up[n] = 0;
  for (int i = 0; i < p->nnames; i++)
    if (!strcmp(p->names[i].name, up)) return &p->names[i];
  if (p->nnames == MAXNAMES) {
    bad(p, "too many names");
    return &p->names[0];
  }
  name_t *e = &p->names[p->nnames++];
  memcpy(e->name, up, n + 1);
  e->token = token;
  e->value = -1;
  return e;
}

/* ---- scanner (the flex rules of lexer.l:224-346) ------------------------- */
static int at(const p64prog *p, size_t i) { return i < p->len ? (unsigned char)p->src[i] : -1; }

/* longest match among the number rules from position i; returns length, fills
 * type/value; ties go to the earlier rule (Real, Dec, Hex, Hex2, Oct, Oct2, Char) */
static size_t scan_number(const p64prog *p, size_t i, token_t *t) {
  size_t best = 0;
  int btype = 0;
  long bval = 0;
  double brval = 0;
  /* Real: D+ "." D* E? | D* "." D+ E? | D+ E */
  {
    size_t j = i, d1 = 0, d2 = 0, n = 0;
    while (isdigit(at(p, j))) j++, d1++;
    int dot = at(p, j) == '.';
    if (dot) {
      j++;
      while (isdigit(at(p, j))) j++, d2++;
    }
    if ((dot && (d1 || d2)) || (!dot && d1)) {
      size_t e = j;
      if (at(p, e) == 'e' || at(p, e) == 'E') {
        size_t k = e + 1;
        if (at(p, k) == '+' || at(p, k) == '-') k++;
        if (isdigit(at(p, k))) {
          while (isdigit(at(p, k))) k++;
          e = k;
        }
      }
      if (dot || e > j) n = e - i;
    }
    if (n > best) {
      char buf[128];
      size_t m = n < sizeof buf - 1 ? n : sizeof buf - 1;
      memcpy(buf, p->src + i, m);
      buf[m] = 0;
      best = n, btype = T_REAL, brval = atof(buf);
    }
  }
  size_t s = i;
  if (at(p, s) == '+' || at(p, s) == '-') s++;
  char buf[128];
  /* DecInteger [-+]?D+ */
  {
    size_t j = s;
    while (isdigit(at(p, j))) j++;
    if (j > s && j - i > best) {
      size_t m = j - i < sizeof buf - 1 ? j - i : sizeof buf - 1;
      memcpy(buf, p->src + i, m);
      buf[m] = 0;
      best = j - i, btype = T_INTEGER, bval = atoi(buf);
    }
  }
  /* HexInteger [-+]?0[xX]H+ -> strtol(text+2) (sign dropped, lexer.l:277) */
  if (at(p, s) == '0' && (at(p, s + 1) == 'x' || at(p, s + 1) == 'X')) {
    size_t j = s + 2;
    while (isxdigit(at(p, j))) j++;
    if (j > s + 2 && j - i > best) {
      size_t m = j - i - 2 < sizeof buf - 1 ? j - i - 2 : sizeof buf - 1;
      memcpy(buf, p->src + i + 2, m);
      buf[m] = 0;
      best = j - i, btype = T_INTEGER, bval = strtol(buf, NULL, 16);
    }
  }
  /* HexInteger2 [-+]?H+[Hh] -> strtol(text) */
  {
    size_t j = s;
    while (isxdigit(at(p, j))) j++;
    if (j > s && (at(p, j) == 'h' || at(p, j) == 'H') && j + 1 - i > best) {
      size_t m = j + 1 - i < sizeof buf - 1 ? j + 1 - i : sizeof buf - 1;
      memcpy(buf, p->src + i, m);
      buf[m] = 0;
      best = j + 1 - i, btype = T_INTEGER, bval = strtol(buf, NULL, 16);
    }
  }
  /* OctInteger [-+]?0[oO]O+ -> strtol(text+2) */
  if (at(p, s) == '0' && (at(p, s + 1) == 'o' || at(p, s + 1) == 'O')) {
    size_t j = s + 2;
    while (at(p, j) >= '0' && at(p, j) <= '7') j++;
    if (j > s + 2 && j - i > best) {
      size_t m = j - i - 2 < sizeof buf - 1 ? j - i - 2 : sizeof buf - 1;
      memcpy(buf, p->src + i + 2, m);
      buf[m] = 0;
      best = j - i, btype = T_INTEGER, bval = strtol(buf, NULL, 8);
    }
  }
  /* OctInteger2 [-+]?O+[BCObco] -> strtol(text) */
  {
    size_t j = s;
    while (at(p, j) >= '0' && at(p, j) <= '7') j++;
    const int c = at(p, j);
    if (j > s && c > 0 && strchr("BCObco", c) && j + 1 - i > best) {
      size_t m = j + 1 - i < sizeof buf - 1 ? j + 1 - i : sizeof buf - 1;
      memcpy(buf, p->src + i, m);
      buf[m] = 0;
      best = j + 1 - i, btype = T_INTEGER, bval = strtol(buf, NULL, 8);
    }
  }
  /* CharInteger [-+]?'([^\\]|\\(.|O{1,3}))' (lexer.l:296-338) */
  if (at(p, s) == '\'') {
    size_t j = s + 1;
    long v = 0;
    int ok = 0;
    if (at(p, j) == '\\') {
      size_t k = j + 1, od = 0;
      while (od < 3 && at(p, k) >= '0' && at(p, k) <= '7') k++, od++;
      if (od && at(p, k) == '\'') { /* octal escape */
        size_t m = k - (s + 2) < sizeof buf - 1 ? k - (s + 2) : sizeof buf - 1;
        memcpy(buf, p->src + s + 2, m);
        buf[m] = 0;
        v = strtol(buf, NULL, 8), j = k + 1, ok = 1;
      } else if (at(p, j + 1) >= 0 && at(p, j + 2) == '\'') {
        switch (at(p, j + 1)) {
          case '0': v = 0; break;
          case 'b': v = 0x8; break;
          case 'i': v = 0x9; break;
          case 'n': v = 0xa; break;
          case 'v': v = 0xb; break;
          case 'f': v = 0xc; break;
          case 'r': v = 0xd; break;
          default: v = at(p, i) + 2; break; /* (*yytext+2), lexer.l:327 */
        }
        j += 3, ok = 1;
      }
    } else if (at(p, j) >= 0 && at(p, j + 1) == '\'') {
      v = at(p, j), j += 2, ok = 1;
    }
    if (ok && j - i > best) best = j - i, btype = T_INTEGER, bval = v;
  }
  if (best) {
    t->type = btype;
    t->ival = (int)bval;
    t->rval = brval;
  }
  return best;
}

static void scan(p64prog *p, token_t *t) {
  t->id = NULL;
  t->str[0] = 0;
  for (;;) {
    const int c = at(p, p->pos);
    if (c < 0) {
      t->type = T_EOF;
      return;
    }
    if (c == '/' && at(p, p->pos + 1) == '*') { /* nested comments */
      p->comment_depth++;
      p->pos += 2;
      continue;
    }
    if (p->comment_depth) {
      if (c == '*' && at(p, p->pos + 1) == '/') {
        p->comment_depth--;
        p->pos += 2;
      } else {
        p->pos++;
      }
      continue;
    }
    if (c == ' ' || c == '\t' || c == '\n') {
      p->pos++;
      continue;
    }
    if (isalpha(c)) { /* Id: letter (letter|digit)* ':'? -- earlier than numbers */
      size_t j = p->pos + 1;
      while (isalnum(at(p, j))) j++;
      if (at(p, j) == ':') j++;
      name_t *e = lookup(p, p->src + p->pos, j - p->pos, 0);
      p->pos = j;
      t->id = e;
      if (e->token) {
        t->type = e->token;
      } else {
        t->type = T_ID;
        t->ival = e->value;
      }
      return;
    }
    if (c == '[' || c == ']') {
      p->pos++;
      t->type = c == '[' ? T_LBRACKET : T_RBRACKET;
      return;
    }
    size_t n = scan_number(p, p->pos, t);
    if (n) {
      p->pos += n;
      return;
    }
    if (c == '"') { /* String \"([^\"]|\\\")*\" */
      size_t j = p->pos + 1, k = 0;
      while (at(p, j) >= 0 && at(p, j) != '"') {
        if (at(p, j) == '\\' && at(p, j + 1) == '"') j++;
        if (k < sizeof t->str - 1) t->str[k++] = (char)at(p, j);
        j++;
      }
      if (at(p, j) == '"') {
        t->str[k] = 0;
        p->pos = j + 1;
        t->type = T_STRING;
        return;
      }
    }
    say(p, "Bad input char '%c'\n", c);
    p->pos++;
  }
}

/* ---- program source (mylex lexer.l:1440-1510) ----------------------------- */
static void push(p64prog *p, double v) {
  if (p->level >= MEMTOP) {
    bad(p, "data stack overflow");
    return;
  }
  p->stack[p->level++] = v;
}
static double pop1(p64prog *p) {
  if (p->level <= 0) {
    bad(p, "data stack underflow");
    return 0;
  }
  return p->stack[--p->level];
}

static void enter_prog(p64prog *p, int n, int line) {
  if (n < 0 || n >= NPROG || p->depth >= MAXDEPTH) {
    bad(p, "EXE of program %d", n);
    return;
  }
  p->saved_prog[p->depth] = p->cur_prog;
  p->saved_line[p->depth] = p->cur_line;
  p->depth++;
  p->cur_prog = n;
  p->cur_line = line;
}
static void leave_prog(p64prog *p) {
  p->depth--;
  p->cur_prog = p->saved_prog[p->depth];
  p->cur_line = p->saved_line[p->depth];
}

static void next(p64prog *p, token_t *t) {
  for (;;) {
    if (p->err) {
      t->type = T_EOF;
      return;
    }
    if (!p->depth) {
      scan(p, t);
      return;
    }
    if (p->cur_line < 0 || p->cur_line >= MAXLINES) {
      bad(p, "program %d jumps outside itself", p->cur_prog);
      continue;
    }
    const int tok = p->code[p->cur_prog][p->cur_line++];
    if (p->next_val) {
      p->next_val--;
      t->type = T_INTEGER;
      t->ival = tok;
      return;
    }
    switch (tok) {
      case 0: /* ran off the end: "Abnormal break", back to the caller */
        leave_prog(p);
        break;
      case T_VAL: {
        const int k = p->code[p->cur_prog][p->cur_line++];
        push(p, (k >= 0 && k < MAXLINES) ? p->consts[p->cur_prog][k] : 0.0);
        break;
      }
      case T_GOTO:
        p->cur_line = p->code[p->cur_prog][p->cur_line];
        break;
      case T_IFG:
      case T_IFNG: {
        const double v = pop1(p);
        if ((tok == T_IFG) == (v != 0))
          p->cur_line = p->code[p->cur_prog][p->cur_line];
        else
          p->cur_line++;
        break;
      }
      case T_EXIT:
        leave_prog(p);
        break;
      case T_COPY: case T_INDEX: case T_STO: case T_RCL: case T_EXE: case T_ABORT:
      case T_PRINTPROGRAM:
        p->next_val = 1;
        t->type = tok;
        return;
      case T_ROLL:
        p->next_val = 2;
        t->type = tok;
        return;
      default:
        t->type = tok;
        return;
    }
  }
}

/* integer or label operand (STO/RCL/EXE/... lexer.l:892-905) */
static int operand(p64prog *p, int *v) {
  token_t t;
  next(p, &t);
  if (t.type != T_INTEGER && t.type != T_ID) return bad(p, "integer or label expected");
  *v = t.ival;
  return 0;
}

/* ---- compile `open n ... close` (MakeProgram/CompileProgram lexer.l:1250-1430) */
static void emit(p64prog *p, int n, int v) {
  if (p->ncode[n] >= MAXLINES - 1) {
    bad(p, "program %d too long", n);
    return;
  }
  p->code[n][p->ncode[n]++] = v;
}
static void emit_const(p64prog *p, int n, double v) {
  if (p->nconst[n] >= MAXLINES) {
    bad(p, "program %d has too many constants", n);
    return;
  }
  emit(p, n, T_VAL);
  p->consts[n][p->nconst[n]] = v;
  emit(p, n, p->nconst[n]++);
}

static void compile(p64prog *p, int n) {
  token_t t;
  p->ncode[n] = 0; /* PLevel = 0; the constant pool is kept (PLLevel) */
  int first_ref = p->nlabels;
  for (;;) {
    next(p, &t);
    if (p->err) return;
    if (t.type == T_CLOSE) break;
    switch (t.type) {
      case T_EOF:
        bad(p, "end of input inside program %d", n);
        return;
      case T_COPY: case T_INDEX: case T_STO: case T_RCL: case T_EXE: case T_ABORT:
      case T_PRINTPROGRAM: {
        emit(p, n, t.type);
        token_t o;
        next(p, &o);
        emit(p, n, (o.type == T_INTEGER || o.type == T_ID) ? o.ival : 0);
        break;
      }
      case T_ROLL:
        emit(p, n, t.type);
        for (int k = 0; k < 2; k++) {
          token_t o;
          next(p, &o);
          emit(p, n, (o.type == T_INTEGER || o.type == T_ID) ? o.ival : 0);
        }
        break;
      case T_GOTO: case T_IFG: case T_IFNG: {
        emit(p, n, t.type);
        token_t o;
        next(p, &o);
        if (o.type != T_ID || p->nlabels >= 1000) {
          bad(p, "label expected after jump");
          return;
        }
        p->labels[p->nlabels] = o.id;
        emit(p, n, p->nlabels++);
        break;
      }
      case T_VAL:
        emit_const(p, n, pop1(p));
        break;
      case T_INTEGER:
        emit_const(p, n, (double)t.ival);
        break;
      case T_REAL:
        emit_const(p, n, t.rval);
        break;
      case T_ID:
        if (t.id->value >= 0) {
          say(p, "Attempt to redefine label.\n");
          break;
        }
        t.id->value = p->ncode[n];
        break;
      default:
        if (t.type >= T_ADD && t.type < T_ECHO) { /* operations without operands */
          emit(p, n, t.type);
        } else {
          say(p, "Token type %d not allowed in programs.\n", t.type);
        }
        break;
    }
  }
  /* resolve jumps to label positions; a label at position 0 cannot be a
   * target (CompileProgram tests the position for zero, lexer.l:1415) */
  for (int i = 0; i < p->ncode[n]; i++) {
    const int op = p->code[n][i];
    if (op == T_COPY || op == T_INDEX || op == T_STO || op == T_RCL || op == T_EXE ||
        op == T_ABORT || op == T_VAL || op == T_PRINTPROGRAM) {
      i++;
    } else if (op == T_ROLL) {
      i += 2;
    } else if (op == T_GOTO || op == T_IFG || op == T_IFNG) {
      i++;
      const int li = p->code[n][i];
      if (li < first_ref || li >= p->nlabels || p->labels[li]->value <= 0) {
        bad(p, "bad reference to label in program %d", n);
        return;
      }
      p->code[n][i] = p->labels[li]->value;
    }
  }
}

static void print_program(p64prog *p, int n) {
  if (n < 0 || n >= NPROG) return;
  for (int i = 0; i < p->ncode[n]; i++) {
    const int op = p->code[n][i];
    const char *w = (op >= T_ADD && op <= T_QCIF) ? WORDS[op - 1] : "?";
    if (op == T_ROLL) {
      say(p, "%d: %s %d %d\n", i, w, p->code[n][i + 1], p->code[n][i + 2]);
      i += 2;
    } else if (op == T_VAL) {
      say(p, "%d: %s %f\n", i, w, p->consts[n][p->code[n][i + 1]]);
      i++;
    } else if (op == T_COPY || op == T_INDEX || op == T_STO || op == T_RCL || op == T_EXE ||
               op == T_ABORT || op == T_PRINTPROGRAM || op == T_GOTO || op == T_IFG ||
               op == T_IFNG) {
      say(p, "%d: %s %d\n", i, w, p->code[n][i + 1]);
      i++;
    } else {
      say(p, "%d: %s\n", i, w);
    }
  }
}

static int mem_index(p64prog *p, int a) {
  if (a < 0 || a >= MEMTOP) return bad(p, "memory address %d out of range", a), 0;
  return a;
}

/* parser() lexer.l:732-1090: runs tokens until the source returns EOF */
static void run(p64prog *p) {
  token_t t;
  int v = 0, v2 = 0;
  double a;
  for (;;) {
    next(p, &t);
    if (p->err || t.type == T_EOF) return;
    double *top = p->stack + p->level;
    switch (t.type) {
      case T_INTEGER: push(p, (double)t.ival); break;
      case T_REAL: push(p, t.rval); break;
#define BIN(expr)                                   \
  if (p->level < 2) {                               \
    say(p, "Not enough operands on stack.\n");      \
    break;                                          \
  }                                                 \
  a = p->stack[--p->level];                         \
  {                                                 \
    double *x = &p->stack[p->level - 1];            \
    expr;                                           \
  }
      case T_ADD: BIN(*x += a); break;
      case T_SUB: BIN(*x -= a); break;
      case T_MUL: BIN(*x *= a); break;
      case T_DIV: BIN(*x /= a); break;
      case T_AND: BIN(*x = (*x && a) ? 1.0 : 0.0); break;
      case T_OR: BIN(*x = (*x || a) ? 1.0 : 0.0); break;
      case T_XOR: BIN(*x = ((*x != 0) != (a != 0)) ? 1.0 : 0.0); break;
      case T_LT: BIN(*x = *x < a ? 1.0 : 0.0); break;
      case T_LTE: BIN(*x = *x <= a ? 1.0 : 0.0); break;
      case T_EQ: BIN(*x = *x == a ? 1.0 : 0.0); break;
      case T_GT: BIN(*x = *x > a ? 1.0 : 0.0); break;
      case T_GTE: BIN(*x = *x >= a ? 1.0 : 0.0); break;
#undef BIN
      case T_NOT: case T_NEG: case T_SQRT: case T_ABS: case T_FLOOR: case T_CEIL: case T_ROUND: {
        if (p->level < 1) {
          bad(p, "unary operation on an empty stack");
          break;
        }
        double *x = top - 1;
        switch (t.type) {
          case T_NOT: *x = *x ? 0.0 : 1.0; break;
          case T_NEG: *x = -*x; break;
          case T_SQRT: *x = sqrt(*x); break;
          case T_ABS: *x = fabs(*x); break;
          case T_FLOOR: *x = floor(*x); break;
          case T_CEIL: *x = ceil(*x); break;
          default: *x = *x < 0 ? ceil(*x - 0.5) : floor(*x + 0.5); break;
        }
        break;
      }
      case T_DUP:
        if (p->level < 1) bad(p, "DUP on an empty stack");
        else push(p, top[-1]);
        break;
      case T_POP:
        if (p->level) p->level--;
        else say(p, "Not enough stack elements.\n");
        break;
      case T_EXCH:
        if (p->level < 2) bad(p, "EXCH needs two elements");
        else a = top[-1], top[-1] = top[-2], top[-2] = a;
        break;
      case T_COPY:
        if (operand(p, &v)) break;
        if (v < 0 || p->level < v) {
          say(p, "Not enough elements\n");
          break;
        }
        for (int i = 0; i < v; i++) push(p, p->stack[p->level - v]);
        break;
      case T_ROLL: { /* lexer.l:836-848: rotate the top `dest` up by `value` */
        if (operand(p, &v) || operand(p, &v2)) break;
        const int dest = v;
        if (dest <= 0 || dest > p->level) {
          bad(p, "ROLL %d on %d elements", dest, p->level);
          break;
        }
        int value = v2 % dest;
        if (value < 0) value += dest;
        double tmp[MEMTOP];
        double *base = p->stack + p->level - dest;
        for (int i = 0; i < dest; i++) tmp[(i + value) % dest] = base[i];
        memcpy(base, tmp, (size_t)dest * sizeof(double));
        break;
      }
      case T_INDEX:
        if (operand(p, &v)) break;
        if (v < 0 || v > p->level) {
          say(p, "Index out of bounds\n");
          break;
        }
        if (v == 0) {
          bad(p, "INDEX 0 reads above the stack");
          break;
        }
        push(p, p->stack[p->level - v]);
        break;
      case T_CLEAR: p->level = 0; break;
      case T_STO:
        if (operand(p, &v)) break;
        if (!p->level) {
          bad(p, "STO on an empty stack");
          break;
        }
        p->mem[mem_index(p, v)] = pop1(p);
        break;
      case T_RCL:
        if (operand(p, &v)) break;
        push(p, p->mem[mem_index(p, v)]);
        break;
      case T_GOTO: case T_IFG: case T_IFNG: case T_EXIT:
        say(p, "Program commands not available on top-level.\n");
        break;
      case T_EXE:
        if (operand(p, &v)) break;
        enter_prog(p, v, 0);
        break;
      case T_ABORT:
        if (operand(p, &v)) break;
        p->set.abort_code = v;
        bad(p, "ABORT %d", v);
        return;
      case T_PRINTSTACK:
        for (int i = 0; i < p->level; i++) say(p, "%d: %f\n", i, p->stack[i]);
        break;
      case T_PRINTPROGRAM:
        if (operand(p, &v)) break;
        print_program(p, v);
        break;
      case T_PRINTIMAGE: case T_PRINTFRAME: break;
      case T_ECHO: {
        token_t s;
        next(p, &s);
        say(p, "%s\n", s.type == T_STRING ? s.str : "");
        break;
      }
      case T_OPEN:
        if (operand(p, &v)) break;
        if (v < 0 || v >= NPROG) {
          bad(p, "OPEN %d: programs are 0..%d", v, NPROG - 1);
          break;
        }
        compile(p, v);
        break;
      case T_CLOSE: say(p, "Close not available on top level.\n"); break;
      case T_EQU: {
        const double x = pop1(p);
        token_t id;
        next(p, &id);
        if (id.type != T_ID) {
          say(p, "Label expected.\n");
          break;
        }
        id.id->value = (int)x;
        break;
      }
      case T_VAL: say(p, "VAL is not a valid id on top level.\n"); break;
      case T_STREAMNAME: {
        token_t s;
        next(p, &s);
        break;
      }
      case T_COMPONENT: { /* component n ["prefix" "suffix"] -- file names, unused here */
        token_t s;
        do next(p, &s);
        while (s.type != T_EOF && s.type != T_RBRACKET && !p->err);
        break;
      }
      case T_FRAMERATE:
        if (!operand(p, &v)) p->set.frame_rate = v;
        break;
      case T_FRAMESKIP:
        if (!operand(p, &v)) p->set.frame_skip = v;
        break;
      case T_QUANTIZATION:
        if (!operand(p, &v)) p->set.quantization = v;
        break;
      case T_SEARCHLIMIT:
        if (!operand(p, &v)) p->set.search_limit = v < 1 ? 1 : v > 31 ? 31 : v;
        break;
      case T_NTSC: p->set.image_type = 2; break;
      case T_CIF: p->set.image_type = 1; break;
      case T_QCIF: p->set.image_type = 0; break;
      default:
        say(p, "Illegal token type encountered: %d\n", t.type);
        break;
    }
  }
}

int p64prog_load(const char *text, size_t len, FILE *out, p64prog **prog) {
  if (!prog || (!text && len)) return p64gpu_fail_(P64GPU_E_INVALID, "p64prog_load: NULL argument");
  p64prog *p = (p64prog *)calloc(1, sizeof *p);
  if (!p) return p64gpu_fail_(P64GPU_E_NOMEM, "p64prog: calloc");
  p->src = text;
  p->len = len;
  p->out = out;
  p->set.quantization = p->set.search_limit = p->set.frame_rate = p->set.frame_skip = -1;
  p->set.image_type = p->set.abort_code = -1;
  for (int i = 0; i < (int)(sizeof WORDS / sizeof WORDS[0]); i++) lookup(p, WORDS[i], strlen(WORDS[i]), i + 1);
  for (int i = 0; i < 14; i++) lookup(p, EQU_NAMES[i], strlen(EQU_NAMES[i]), 0)->value = i + 1;
  run(p);
  p->src = NULL; /* the text is not needed after loading */
  p->len = p->pos = 0;
  if (p->err) {
    char msg[256];
    snprintf(msg, sizeof msg, "program: %s", p->errmsg);
    free(p);
    return p64gpu_fail_(P64GPU_E_INVALID, msg);
  }
  *prog = p;
  return 0;
}

void p64prog_free(p64prog *p) { free(p); }

int p64prog_settings_get(const p64prog *p, p64prog_settings *s) {
  if (!p || !s) return p64gpu_fail_(P64GPU_E_INVALID, "p64prog_settings_get: NULL");
  *s = p->set;
  return 0;
}

int p64prog_defined(const p64prog *p, int n) { return p && n >= 0 && n < NPROG && p->ncode[n] > 0; }

int p64prog_reads(const p64prog *p, int n, int loc) {
  if (!p || n < 0 || n >= NPROG) return 0;
  int seen[NPROG] = {0}, todo[NPROG], nt = 0;
  todo[nt++] = n;
  seen[n] = 1;
  while (nt) {
    const int q = todo[--nt];
    for (int i = 0; i < p->ncode[q]; i++) {
      const int op = p->code[q][i];
      if (op == T_ROLL) {
        i += 2;
      } else if (op == T_COPY || op == T_INDEX || op == T_STO || op == T_RCL || op == T_EXE ||
                 op == T_ABORT || op == T_VAL || op == T_PRINTPROGRAM || op == T_GOTO ||
                 op == T_IFG || op == T_IFNG) {
        const int v = p->code[q][++i];
        if (op == T_RCL && v == loc) return 1;
        if (op == T_EXE && v >= 0 && v < NPROG && !seen[v]) seen[v] = 1, todo[nt++] = v;
      }
    }
  }
  return 0;
}

int p64prog_execute(p64prog *p, int n) {
  if (!p) return p64gpu_fail_(P64GPU_E_INVALID, "p64prog_execute: NULL");
  if (n < 0 || n >= NPROG) return p64gpu_fail_(P64GPU_E_INVALID, "program number out of range");
  if (!p->ncode[n]) return 0; /* Execute: only defined programs run (lexer.l:1521) */
  enter_prog(p, n, 0);
  run(p); /* returns when the program exits and the (finished) text gives EOF */
  p->depth = 0;
  p->next_val = 0;
  if (p->err) {
    char msg[256];
    snprintf(msg, sizeof msg, "program %d: %s", n, p->errmsg);
    p->err = 0;
    return p64gpu_fail_(P64GPU_E_INVALID, msg);
  }
  return 0;
}

double *p64prog_memory(p64prog *p) { return p ? p->mem : NULL; }
