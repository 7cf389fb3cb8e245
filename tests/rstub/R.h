/* Test stub of R's C API (TEST INFRASTRUCTURE): just enough of R.h / Rinternals.h /
 * R_ext/Rdynload.h to compile the package's .Call shim (distributed-correlation_amd/src/dcor_r.c)
 * without R, and to call its routines from Python (tests/test_r_shim.py).  Not R: SEXPs are
 * plain heap records, PROTECT is a no-op, Rf_error longjmps to the stub's call wrapper. */
#ifndef DCOR_RSTUB_R_H
#define DCOR_RSTUB_R_H
#include <stddef.h>
#include <stdint.h>

typedef ptrdiff_t R_xlen_t;
typedef unsigned char Rbyte;
typedef struct SEXPREC* SEXP;
typedef enum { FALSE = 0, TRUE } Rboolean;

#define NILSXP 0
#define SYMSXP 1
#define CHARSXP 9
#define LGLSXP 10
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
#define VECSXP 19
#define RAWSXP 24

#define NA_INTEGER (-2147483647 - 1)
#define NA_LOGICAL NA_INTEGER
#define ISNAN(x) __builtin_isnan(x)

void* R_alloc(size_t n, int size);
void Rf_error(const char* fmt, ...) __attribute__((noreturn));
#endif
