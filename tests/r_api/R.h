/* Declarations of the part of R's C API (R >= 3.5, Rinternals.h / R.h / R_ext/Rdynload.h) that
 * r_shim/RcppExports.cpp uses, so the shim can be compile-checked in a container without R
 * (tests/test_r_shim.py).  Test infrastructure only: signatures as R documents them in
 * "Writing R Extensions"; no implementation, nothing here is linked or run. */
#ifndef BRR_TEST_R_H
#define BRR_TEST_R_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef enum { FALSE = 0, TRUE } Rboolean;
void REprintf(const char *, ...);
void GetRNGstate(void);
void PutRNGstate(void);
double unif_rand(void);
void Rf_error(const char *, ...);
#ifdef __cplusplus
}
#endif
#endif
