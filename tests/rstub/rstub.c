/* rstub.c -- test stub of R's C API (TEST INFRASTRUCTURE, see R.h): SEXP records, R_alloc,
 * Rf_error via longjmp, routine registration, and a ctypes-facing call wrapper so Python can
 * run the package's .Call routines exactly as R would hand them their arguments. */
#define _POSIX_C_SOURCE 200809L  /* strdup */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "R.h"
#include "R_ext/Rdynload.h"
#include "Rinternals.h"

#define MAX_ATTR 8
struct SEXPREC {
  int type;
  R_xlen_t len;
  int nrow, ncol;   /* allocMatrix dims (0: plain vector) */
  void* data;       /* elements; SYMSXP / CHARSXP: the NUL-terminated name / string */
  int nattr;        /* attributes: (symbol, value) pairs, as setAttrib stores them */
  SEXP attr_name[MAX_ATTR], attr_val[MAX_ATTR];
};

static struct SEXPREC nil = {NILSXP, 0, 0, 0, NULL, 0, {0}, {0}};
SEXP R_NilValue = &nil;

/* R_alloc memory lives until the end of the current .Call (freed by rs_call) */
static void* g_ralloc[4096];
static int g_nralloc = 0;
static jmp_buf g_jmp;
static int g_in_call = 0;
static char g_err[1024];

void* R_alloc(size_t n, int size) {
  void* p = calloc(n ? n : 1, (size_t)size);
  if (g_nralloc < 4096) g_ralloc[g_nralloc++] = p;
  return p;
}

void Rf_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  if (g_in_call) longjmp(g_jmp, 1);
  fprintf(stderr, "Rf_error outside a call: %s\n", g_err);
  abort();
}

static size_t elt_size(int type) {
  switch (type) {
    case REALSXP: return sizeof(double);
    case INTSXP: case LGLSXP: return sizeof(int);
    case RAWSXP: return 1;
    case VECSXP: case STRSXP: return sizeof(SEXP);
    default: return 1;
  }
}

SEXP Rf_allocVector(int type, R_xlen_t n) {
  SEXP s = (SEXP)calloc(1, sizeof(struct SEXPREC));
  s->type = type;
  s->len = n;
  s->data = calloc((size_t)(n ? n : 1), elt_size(type));
  if (type == VECSXP || type == STRSXP)
    for (R_xlen_t i = 0; i < n; ++i) ((SEXP*)s->data)[i] = R_NilValue;
  return s;
}

/* symbols are interned (R compares attribute names by pointer) */
static SEXP g_syms[64];
static int g_nsyms = 0;
SEXP Rf_install(const char* name) {
  for (int i = 0; i < g_nsyms; ++i)
    if (strcmp((const char*)g_syms[i]->data, name) == 0) return g_syms[i];
  SEXP s = (SEXP)calloc(1, sizeof(struct SEXPREC));
  s->type = SYMSXP;
  s->data = strdup(name);
  s->len = (R_xlen_t)strlen(name);
  if (g_nsyms < 64) g_syms[g_nsyms++] = s;
  return s;
}
SEXP R_NamesSymbol, R_ClassSymbol, R_RowNamesSymbol;
__attribute__((constructor)) static void init_symbols(void) {
  R_NamesSymbol = Rf_install("names");
  R_ClassSymbol = Rf_install("class");
  R_RowNamesSymbol = Rf_install("row.names");
}

SEXP Rf_mkChar(const char* str) {
  SEXP s = (SEXP)calloc(1, sizeof(struct SEXPREC));
  s->type = CHARSXP;
  s->data = strdup(str);
  s->len = (R_xlen_t)strlen(str);
  return s;
}
SEXP Rf_mkString(const char* str) {
  SEXP s = Rf_allocVector(STRSXP, 1);
  ((SEXP*)s->data)[0] = Rf_mkChar(str);
  return s;
}
void SET_STRING_ELT(SEXP x, R_xlen_t i, SEXP v) {
  if (x->type != STRSXP || v->type != CHARSXP) Rf_error("SET_STRING_ELT: wrong types");
  ((SEXP*)x->data)[i] = v;
}
SEXP STRING_ELT(SEXP x, R_xlen_t i) { return ((SEXP*)x->data)[i]; }
SEXP Rf_setAttrib(SEXP x, SEXP name, SEXP value) {
  for (int i = 0; i < x->nattr; ++i)
    if (x->attr_name[i] == name) { x->attr_val[i] = value; return value; }
  if (x->nattr == MAX_ATTR) Rf_error("setAttrib: too many attributes");
  x->attr_name[x->nattr] = name;
  x->attr_val[x->nattr++] = value;
  return value;
}
SEXP Rf_getAttrib(SEXP x, SEXP name) {
  for (int i = 0; i < x->nattr; ++i)
    if (x->attr_name[i] == name) return x->attr_val[i];
  return R_NilValue;
}

SEXP Rf_allocMatrix(int type, int nrow, int ncol) {
  SEXP s = Rf_allocVector(type, (R_xlen_t)nrow * ncol);
  s->nrow = nrow;
  s->ncol = ncol;
  return s;
}

SEXP Rf_ScalarReal(double x) {
  SEXP s = Rf_allocVector(REALSXP, 1);
  ((double*)s->data)[0] = x;
  return s;
}

static void need(SEXP x, int type, const char* what) {
  if (x->type != type) Rf_error("%s() applied to a non-%s (type %d)", what, what, x->type);
}
double* REAL(SEXP x) { need(x, REALSXP, "REAL"); return (double*)x->data; }
int* INTEGER(SEXP x) { need(x, INTSXP, "INTEGER"); return (int*)x->data; }
int* LOGICAL(SEXP x) { need(x, LGLSXP, "LOGICAL"); return (int*)x->data; }
Rbyte* RAW(SEXP x) { need(x, RAWSXP, "RAW"); return (Rbyte*)x->data; }
R_xlen_t XLENGTH(SEXP x) { return x->len; }
int TYPEOF(SEXP x) { return x->type; }
int LENGTH(SEXP x) { return (int)x->len; }
int Rf_isNull(SEXP x) { return x->type == NILSXP; }

double Rf_asReal(SEXP x) {
  if (x->len < 1) return 0.0 / 0.0;
  switch (x->type) {
    case REALSXP: return ((double*)x->data)[0];
    case INTSXP: case LGLSXP: return (double)((int*)x->data)[0];
    default: return 0.0 / 0.0;
  }
}
int Rf_asInteger(SEXP x) {
  if (x->len < 1) return -2147483647 - 1;
  if (x->type == REALSXP) return (int)((double*)x->data)[0];
  if (x->type == INTSXP || x->type == LGLSXP) return ((int*)x->data)[0];
  return -2147483647 - 1;
}
int Rf_asLogical(SEXP x) {
  if (x->len < 1) return -2147483647 - 1;
  if (x->type == LGLSXP || x->type == INTSXP) return ((int*)x->data)[0] != 0;
  if (x->type == REALSXP) return ((double*)x->data)[0] != 0.0;
  return -2147483647 - 1;
}
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v) { ((SEXP*)x->data)[i] = v; return v; }
SEXP VECTOR_ELT(SEXP x, R_xlen_t i) { return ((SEXP*)x->data)[i]; }

/* ------------------------------------------------------------ registration */
static const R_CallMethodDef* g_calls = NULL;
int R_registerRoutines(DllInfo* info, const void* c, const R_CallMethodDef* call, const void* f,
                       const void* e) {
  (void)info; (void)c; (void)f; (void)e;
  g_calls = call;
  return 1;
}
int R_useDynamicSymbols(DllInfo* info, int value) { (void)info; (void)value; return 1; }

/* ---------------------------------------------------- ctypes-facing helpers */
extern void R_init_dcor_r(DllInfo* dll);

SEXP rs_nil(void) { return R_NilValue; }
SEXP rs_real(const double* v, R_xlen_t n) {
  SEXP s = Rf_allocVector(REALSXP, n);
  if (n) memcpy(s->data, v, (size_t)n * sizeof(double));
  return s;
}
SEXP rs_int(const int* v, R_xlen_t n, int logical) {
  SEXP s = Rf_allocVector(logical ? LGLSXP : INTSXP, n);
  if (n) memcpy(s->data, v, (size_t)n * sizeof(int));
  return s;
}
int rs_type(SEXP s) { return s->type; }
R_xlen_t rs_length(SEXP s) { return s->len; }
int rs_nrow(SEXP s) { return s->nrow; }
void* rs_data(SEXP s) { return s->data; }
SEXP rs_elt(SEXP s, R_xlen_t i) { return VECTOR_ELT(s, i); }
const char* rs_error(void) { return g_err; }
const char* rs_char(SEXP s) { return s->type == CHARSXP ? (const char*)s->data : NULL; }
SEXP rs_attr(SEXP s, const char* name) { return Rf_getAttrib(s, Rf_install(name)); }

/* Number of arguments a registered routine takes (-1: not registered). */
int rs_nargs(const char* name) {
  if (!g_calls) R_init_dcor_r(NULL);
  for (const R_CallMethodDef* c = g_calls; c && c->name; ++c)
    if (strcmp(c->name, name) == 0) return c->numArgs;
  return -1;
}

typedef SEXP (*F0)(void);
/* .Call(name, args...): 0 and *out on success, 1 if the routine called Rf_error (message in
 * rs_error()), -1 if `name` is not registered or nargs disagrees with its registration. */
int rs_call(const char* name, int nargs, SEXP* a, SEXP* out) {
  if (!g_calls) R_init_dcor_r(NULL);
  const R_CallMethodDef* def = NULL;
  for (const R_CallMethodDef* c = g_calls; c && c->name; ++c)
    if (strcmp(c->name, name) == 0) def = c;
  if (!def || def->numArgs != nargs) return -1;
  g_err[0] = 0;
  int rc = 0;
  g_in_call = 1;
  if (setjmp(g_jmp) == 0) {
    void* f = (void*)def->fun;
    SEXP r;
    switch (nargs) {
#define A(k) a[k]
      case 2: r = ((SEXP(*)(SEXP, SEXP))f)(A(0), A(1)); break;
      case 3: r = ((SEXP(*)(SEXP, SEXP, SEXP))f)(A(0), A(1), A(2)); break;
      case 4: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3)); break;
      case 5: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4)); break;
      case 6: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5)); break;
      case 8: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7)); break;
      case 9: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8)); break;
      case 10: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8), A(9)); break;
      case 12: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8), A(9), A(10), A(11)); break;
      case 13: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8), A(9), A(10), A(11), A(12)); break;
      case 16: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8), A(9), A(10), A(11), A(12), A(13), A(14), A(15)); break;
      case 20: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8), A(9), A(10), A(11), A(12), A(13), A(14), A(15), A(16), A(17), A(18), A(19)); break;
#undef A
      default: g_in_call = 0; return -1;
    }
    *out = r;
  } else {
    rc = 1;
  }
  g_in_call = 0;
  for (int i = 0; i < g_nralloc; ++i) free(g_ralloc[i]);
  g_nralloc = 0;
  return rc;
}
