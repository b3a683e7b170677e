/* see tests/r_api/R.h: declarations only, for the shim's compile check */
#ifndef BRR_TEST_RINTERNALS_H
#define BRR_TEST_RINTERNALS_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef struct SEXPREC *SEXP;
typedef ptrdiff_t R_xlen_t;
typedef unsigned int SEXPTYPE;
#define LGLSXP 10
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
extern SEXP R_NilValue;
SEXP Rf_protect(SEXP);
void Rf_unprotect(int);
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
SEXP Rf_coerceVector(SEXP, SEXPTYPE);
int TYPEOF(SEXP);
double *REAL(SEXP);
int *INTEGER(SEXP);
R_xlen_t XLENGTH(SEXP);
int Rf_nrows(SEXP);
int Rf_ncols(SEXP);
int Rf_isMatrix(SEXP);
int Rf_isNumeric(SEXP);
int Rf_isLogical(SEXP);
int Rf_isString(SEXP);
int Rf_asInteger(SEXP);
double Rf_asReal(SEXP);
SEXP STRING_ELT(SEXP, R_xlen_t);
const char *CHAR(SEXP);
#ifdef __cplusplus
}
#endif
#endif
