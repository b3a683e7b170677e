// r_shim/RcppExports.cpp -- drop-in replacement for the reference's src/RcppExports.cpp
// (medical-genomics-group/BayesRRcpp): the same four .Call symbols with the same arities
// (src/RcppExports.cpp:110-121), forwarding to libbrr.so's C ABI (include/brr.h) instead of
// the Eigen/Rcpp sampler bodies.  R's matrices are passed as borrowed column-major pointers
// (REAL(x)), so X is never copied on the host (the reference copies it into an Eigen::MatrixXd,
// src/RcppExports.cpp:48).  Not built in this repository (no R toolchain here); see
// INTEGRATION.md for the Makevars.
#include <R.h>
#include <R_ext/Rdynload.h>
#include <Rinternals.h>

#include <cstdint>
#include <vector>

#include "brr.h"

namespace {

void r_log(const char *msg, void *) { REprintf("%s", msg); }  // the reference prints to Rcerr

brr_options options_for(int seed) {
  brr_options o;
  brr_options_default(&o);
  o.log = r_log;
  o.verbose = 1;  // "iteration: i" progress lines like the reference (BayesRv2.cpp:173-175)
  (void)seed;
  return o;
}

// the reference keys nothing on `seed`; libbrr keys its Philox streams on it.
// A negative seed draws one from R's stream so set.seed() still controls the chain.
int resolve_seed(int seed) {
  if (seed >= 0) return seed;
  GetRNGstate();
  const int s = (int)(unif_rand() * 2147483646.0);
  PutRNGstate();
  return s;
}

std::vector<int32_t> as_int32(SEXP x) {
  SEXP xi = PROTECT(Rf_coerceVector(x, INTSXP));
  std::vector<int32_t> v(INTEGER(xi), INTEGER(xi) + XLENGTH(xi));
  UNPROTECT(1);
  return v;
}

void check(int rc) {
  if (rc < 0) Rf_error("BayesRRcpp (MI355X): %s", brr_last_error());
  // rc == 1: validation message already printed, return normally (reference behaviour)
}

}  // namespace

extern "C" {

// BRV2Grstart(outputFile, seed, max_iterations, burn_in, thinning, mu, beta, sigmaE, sigmaGG,
//             X, epsilon, components, sigma0, v0E, s02E, v0G, s02G, cva, groups, gAssign)
SEXP _BayesRRcpp_BRV2Grstart(SEXP outputFile, SEXP seed, SEXP max_iterations, SEXP burn_in,
                             SEXP thinning, SEXP mu, SEXP beta, SEXP sigmaE, SEXP sigmaGG, SEXP X,
                             SEXP epsilon, SEXP components, SEXP sigma0, SEXP v0E, SEXP s02E,
                             SEXP v0G, SEXP s02G, SEXP cva, SEXP groups, SEXP gAssign) {
  const int s = resolve_seed(Rf_asInteger(seed));
  brr_options o = options_for(s);
  std::vector<int32_t> ga = as_int32(gAssign);
  const int G = Rf_asInteger(groups);
  check(brr_BRV2Grstart(CHAR(STRING_ELT(outputFile, 0)), s, Rf_asInteger(max_iterations),
                        Rf_asInteger(burn_in), Rf_asInteger(thinning), Rf_asReal(mu), REAL(beta),
                        Rf_asReal(sigmaE), REAL(sigmaGG), REAL(X), Rf_nrows(X), Rf_ncols(X),
                        REAL(epsilon), REAL(components), Rf_asReal(sigma0), Rf_asReal(v0E),
                        Rf_asReal(s02E), Rf_asReal(v0G), Rf_asReal(s02G), REAL(cva), Rf_ncols(cva),
                        G, ga.data(), &o));
  return R_NilValue;
}

SEXP _BayesRRcpp_BayesRSamplerV2(SEXP outputFile, SEXP seed, SEXP max_iterations, SEXP burn_in,
                                 SEXP thinning, SEXP X, SEXP Y, SEXP sigma0, SEXP v0E, SEXP s02E,
                                 SEXP v0G, SEXP s02G, SEXP cva) {
  const int s = resolve_seed(Rf_asInteger(seed));
  brr_options o = options_for(s);
  check(brr_BayesRSamplerV2(CHAR(STRING_ELT(outputFile, 0)), s, Rf_asInteger(max_iterations),
                            Rf_asInteger(burn_in), Rf_asInteger(thinning), REAL(X), Rf_nrows(X),
                            Rf_ncols(X), REAL(Y), Rf_asReal(sigma0), Rf_asReal(v0E), Rf_asReal(s02E),
                            Rf_asReal(v0G), Rf_asReal(s02G), REAL(cva), (int32_t)XLENGTH(cva), &o));
  return R_NilValue;
}

SEXP _BayesRRcpp_BayesRSamplerV2Groups(SEXP outputFile, SEXP seed, SEXP max_iterations,
                                       SEXP burn_in, SEXP thinning, SEXP X, SEXP Y, SEXP sigma0,
                                       SEXP v0E, SEXP s02E, SEXP v0G, SEXP s02G, SEXP cva,
                                       SEXP groups, SEXP gAssign, SEXP fixed) {
  const int s = resolve_seed(Rf_asInteger(seed));
  brr_options o = options_for(s);
  std::vector<int32_t> ga = as_int32(gAssign);
  check(brr_BayesRSamplerV2Groups(
      CHAR(STRING_ELT(outputFile, 0)), s, Rf_asInteger(max_iterations), Rf_asInteger(burn_in),
      Rf_asInteger(thinning), REAL(X), Rf_nrows(X), Rf_ncols(X), REAL(Y), Rf_asReal(sigma0),
      Rf_asReal(v0E), Rf_asReal(s02E), Rf_asReal(v0G), Rf_asReal(s02G), REAL(cva), Rf_ncols(cva),
      Rf_asInteger(groups), ga.data(), REAL(fixed), Rf_ncols(fixed), &o));
  return R_NilValue;
}

SEXP _BayesRRcpp_HorseshoeR(SEXP outputFile, SEXP seed, SEXP max_iterations, SEXP burn_in,
                            SEXP thinning, SEXP X, SEXP Y, SEXP A, SEXP v0E, SEXP s02E, SEXP vL,
                            SEXP vT, SEXP c2, SEXP vC, SEXP sC) {
  const int s = resolve_seed(Rf_asInteger(seed));
  brr_options o = options_for(s);
  check(brr_HorseshoeR(CHAR(STRING_ELT(outputFile, 0)), s, Rf_asInteger(max_iterations),
                       Rf_asInteger(burn_in), Rf_asInteger(thinning), REAL(X), Rf_nrows(X),
                       Rf_ncols(X), REAL(Y), Rf_asReal(A), Rf_asReal(v0E), Rf_asReal(s02E),
                       Rf_asReal(vL), Rf_asReal(vT), Rf_asReal(c2), Rf_asReal(vC), Rf_asReal(sC), &o));
  return R_NilValue;
}

static const R_CallMethodDef CallEntries[] = {
    {"_BayesRRcpp_BRV2Grstart", (DL_FUNC)&_BayesRRcpp_BRV2Grstart, 20},
    {"_BayesRRcpp_BayesRSamplerV2", (DL_FUNC)&_BayesRRcpp_BayesRSamplerV2, 13},
    {"_BayesRRcpp_BayesRSamplerV2Groups", (DL_FUNC)&_BayesRRcpp_BayesRSamplerV2Groups, 16},
    {"_BayesRRcpp_HorseshoeR", (DL_FUNC)&_BayesRRcpp_HorseshoeR, 15},
    {NULL, NULL, 0}};

void R_init_BayesRRcpp(DllInfo *dll) {
  R_registerRoutines(dll, NULL, CallEntries, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}

}  // extern "C"
