/* Test stub of Rinternals.h (see R.h). */
#ifndef DCOR_RSTUB_RINTERNALS_H
#define DCOR_RSTUB_RINTERNALS_H
#include "R.h"

extern SEXP R_NilValue;
SEXP Rf_allocVector(int type, R_xlen_t n);
SEXP Rf_allocMatrix(int type, int nrow, int ncol);
SEXP Rf_ScalarReal(double x);
double* REAL(SEXP x);
int* INTEGER(SEXP x);
int* LOGICAL(SEXP x);
Rbyte* RAW(SEXP x);
R_xlen_t XLENGTH(SEXP x);
int LENGTH(SEXP x);
double Rf_asReal(SEXP x);
int Rf_asLogical(SEXP x);
int Rf_asInteger(SEXP x);
int Rf_isNull(SEXP x);
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v);
SEXP VECTOR_ELT(SEXP x, R_xlen_t i);
extern SEXP R_NamesSymbol, R_ClassSymbol, R_RowNamesSymbol;
SEXP Rf_install(const char* name);
int TYPEOF(SEXP x);
SEXP Rf_mkChar(const char* s);
SEXP Rf_mkString(const char* s);
void SET_STRING_ELT(SEXP x, R_xlen_t i, SEXP v);
SEXP STRING_ELT(SEXP x, R_xlen_t i);
SEXP Rf_setAttrib(SEXP x, SEXP name, SEXP value);
SEXP Rf_getAttrib(SEXP x, SEXP name);
#define allocVector Rf_allocVector
#define allocMatrix Rf_allocMatrix
#define ScalarReal Rf_ScalarReal
#define mkChar Rf_mkChar
#define mkString Rf_mkString
#define setAttrib Rf_setAttrib
#define getAttrib Rf_getAttrib
#define install Rf_install
#define PROTECT(s) (s)
#define UNPROTECT(n) ((void)(n))
#endif
