// r_shim/RcppExports.cpp -- drop-in replacement for the reference's src/RcppExports.cpp
// (medical-genomics-group/BayesRRcpp): the same four .Call symbols with the same arities
// (src/RcppExports.cpp:110-121), forwarding to libbrr.so's C ABI (include/brr.h) instead of
// the Eigen/Rcpp sampler bodies.
//
// Argument conversion follows what Rcpp's input_parameter<> does for the reference's types
// (src/RcppExports.cpp:14-33, 43-55, 65-80, 90-104): every numeric argument is coerced to double
// (an integer 0/1/2 genotype matrix or an integer `components` vector is accepted, as
// input_parameter<Eigen::MatrixXd> accepts it), gAssign to int, scalars through Rf_asReal /
// Rf_asInteger.  A double matrix is passed as a borrowed column-major pointer (REAL(x)), so X is
// never copied on the host (the reference copies it into an Eigen::MatrixXd,
// src/RcppExports.cpp:48); only a non-double X is converted (one copy, as Rcpp makes).
// Sizes are taken where the reference takes them: N = epsilon.size() for BRV2Grstart
// (src/BRv2Grstart.cpp:81), N = Y.size() otherwise (src/BayesRv2.cpp:64), M = X.cols().
// tests/test_r_shim.py compiles this file against declarations of the R API it uses.
#include <R.h>
#include <R_ext/Rdynload.h>
#include <Rinternals.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "brr.h"

namespace {

void r_log(const char *msg, void *) { REprintf("%s", msg); }  // the reference prints to Rcerr

brr_options options_for() {
  brr_options o;
  brr_options_default(&o);
  o.log = r_log;
  o.verbose = 1;  // "iteration: i" progress lines like the reference (BayesRv2.cpp:173-175)
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

// Errors inside an entry point are C++ exceptions, so every C++ object (coerced copies, vectors)
// is destroyed before R's longjmp; `guarded` turns them into an R error (the role of Rcpp's
// BEGIN_RCPP / END_RCPP, src/RcppExports.cpp:12,36) from a frame without live C++ objects.
[[noreturn]] void fail(const std::string &m) { throw std::runtime_error("BayesRRcpp (MI355X): " + m); }

template <class F>
SEXP guarded(F &&body) {
  char msg[1024];
  msg[0] = 0;
  try {
    body();
  } catch (const std::exception &e) {
    std::snprintf(msg, sizeof msg, "%s", e.what());
  }
  if (msg[0]) Rf_error("%s", msg);
  return R_NilValue;
}

// Every coerced object stays PROTECTed until the call returns (the destructor unprotects them).
struct Protect {
  int n = 0;
  ~Protect() { if (n) UNPROTECT(n); }
  SEXP operator()(SEXP x) { ++n; return PROTECT(x); }
};

// A numeric argument as doubles: REAL() of the object itself when it already is a double
// vector / matrix, else of a coerced copy.  nrow / ncol as Eigen would see them (a plain vector
// is one column).
struct Real {
  const double *p;
  int64_t len, nrow, ncol;
};

Real as_real(Protect &prot, SEXP x, const char *name) {
  if (!Rf_isNumeric(x) && !Rf_isLogical(x)) fail(std::string("'") + name + "' must be numeric");
  SEXP d = TYPEOF(x) == REALSXP ? x : prot(Rf_coerceVector(x, REALSXP));
  Real r;
  r.p = REAL(d);
  r.len = (int64_t)XLENGTH(d);
  r.nrow = Rf_isMatrix(x) ? (int64_t)Rf_nrows(x) : r.len;
  r.ncol = Rf_isMatrix(x) ? (int64_t)Rf_ncols(x) : 1;
  return r;
}

std::vector<int32_t> as_int32(SEXP x) {
  SEXP xi = PROTECT(Rf_coerceVector(x, INTSXP));
  std::vector<int32_t> v(INTEGER(xi), INTEGER(xi) + XLENGTH(xi));
  UNPROTECT(1);
  return v;
}

// cva as the groups x (K-1) column-major block the C ABI reads (leading dimension = groups).  The
// reference indexes cva(g, k) of an Eigen matrix of any row count >= groups
// (src/BayesRv2Groups.cpp:237-240); rows beyond `groups` are never read, so they are dropped here.
std::vector<double> cva_block(const Real &c, int groups) {
  if (c.nrow < groups)
    fail("cva has " + std::to_string(c.nrow) + " rows, fewer than groups = " + std::to_string(groups));
  std::vector<double> out((size_t)groups * (size_t)c.ncol);
  for (int64_t k = 0; k < c.ncol; ++k)
    for (int g = 0; g < groups; ++g) out[(size_t)k * groups + g] = c.p[k * c.nrow + g];
  return out;
}

void check(int rc) {
  if (rc < 0) fail(brr_last_error());
  // rc == 1: validation message already printed, return normally (reference behaviour)
}

const char *path_of(SEXP outputFile) {
  if (!Rf_isString(outputFile) || XLENGTH(outputFile) < 1) fail("outputFile must be a character string");
  return CHAR(STRING_ELT(outputFile, 0));
}

}  // namespace

extern "C" {

// BRV2Grstart(outputFile, seed, max_iterations, burn_in, thinning, mu, beta, sigmaE, sigmaGG,
//             X, epsilon, components, sigma0, v0E, s02E, v0G, s02G, cva, groups, gAssign)
SEXP _BayesRRcpp_BRV2Grstart(SEXP outputFile, SEXP seed, SEXP max_iterations, SEXP burn_in,
                             SEXP thinning, SEXP mu, SEXP beta, SEXP sigmaE, SEXP sigmaGG, SEXP X,
                             SEXP epsilon, SEXP components, SEXP sigma0, SEXP v0E, SEXP s02E,
                             SEXP v0G, SEXP s02G, SEXP cva, SEXP groups, SEXP gAssign) {
  return guarded([&] {
    Protect prot;
    const int s = resolve_seed(Rf_asInteger(seed));
    brr_options o = options_for();
    const Real x = as_real(prot, X, "X"), b = as_real(prot, beta, "beta"), e = as_real(prot, epsilon, "epsilon");
    const Real sg = as_real(prot, sigmaGG, "sigmaGG"), cm = as_real(prot, components, "components");
    const Real cv = as_real(prot, cva, "cva");
    const int G = Rf_asInteger(groups);
    const std::vector<int32_t> ga = as_int32(gAssign);
    const int64_t N = e.len, M = x.ncol;  // N = epsilon.size() (src/BRv2Grstart.cpp:81)
    if (x.nrow != N)
      fail("X has " + std::to_string(x.nrow) + " rows but epsilon has " + std::to_string(N) + " entries");
    if (b.len < M || cm.len < M || (int64_t)ga.size() < M || sg.len < G)
      fail("beta, components and gAssign need one entry per column of X, sigmaGG one per group");
    const std::vector<double> cvb = cva_block(cv, G);
    check(brr_BRV2Grstart(path_of(outputFile), s, Rf_asInteger(max_iterations), Rf_asInteger(burn_in),
                          Rf_asInteger(thinning), Rf_asReal(mu), b.p, Rf_asReal(sigmaE), sg.p, x.p, N, M, e.p,
                          cm.p, Rf_asReal(sigma0), Rf_asReal(v0E), Rf_asReal(s02E), Rf_asReal(v0G),
                          Rf_asReal(s02G), cvb.data(), (int32_t)cv.ncol, G, ga.data(), &o));
  });
}

SEXP _BayesRRcpp_BayesRSamplerV2(SEXP outputFile, SEXP seed, SEXP max_iterations, SEXP burn_in,
                                 SEXP thinning, SEXP X, SEXP Y, SEXP sigma0, SEXP v0E, SEXP s02E,
                                 SEXP v0G, SEXP s02G, SEXP cva) {
  return guarded([&] {
    Protect prot;
    const int s = resolve_seed(Rf_asInteger(seed));
    brr_options o = options_for();
    const Real x = as_real(prot, X, "X"), y = as_real(prot, Y, "Y"), cv = as_real(prot, cva, "cva");
    // N = Y.size(), M = X.cols() (src/BayesRv2.cpp:64-65)
    if (x.nrow != y.len) fail("X has " + std::to_string(x.nrow) + " rows but Y has " + std::to_string(y.len) + " entries");
    check(brr_BayesRSamplerV2(path_of(outputFile), s, Rf_asInteger(max_iterations), Rf_asInteger(burn_in),
                              Rf_asInteger(thinning), x.p, y.len, x.ncol, y.p, Rf_asReal(sigma0), Rf_asReal(v0E),
                              Rf_asReal(s02E), Rf_asReal(v0G), Rf_asReal(s02G), cv.p, (int32_t)cv.len, &o));
  });
}

SEXP _BayesRRcpp_BayesRSamplerV2Groups(SEXP outputFile, SEXP seed, SEXP max_iterations,
                                       SEXP burn_in, SEXP thinning, SEXP X, SEXP Y, SEXP sigma0,
                                       SEXP v0E, SEXP s02E, SEXP v0G, SEXP s02G, SEXP cva,
                                       SEXP groups, SEXP gAssign, SEXP fixed) {
  return guarded([&] {
    Protect prot;
    const int s = resolve_seed(Rf_asInteger(seed));
    brr_options o = options_for();
    const Real x = as_real(prot, X, "X"), y = as_real(prot, Y, "Y"), cv = as_real(prot, cva, "cva");
    const Real f = as_real(prot, fixed, "fixed");
    const int G = Rf_asInteger(groups);
    const std::vector<int32_t> ga = as_int32(gAssign);
    // N = Y.size(), M = X.cols(), F = fixed.cols() (src/BayesRv2Groups.cpp:79-81)
    if (x.nrow != y.len || f.nrow != y.len)
      fail("X (" + std::to_string(x.nrow) + " rows) and fixed (" + std::to_string(f.nrow) +
           " rows) must have one row per entry of Y (" + std::to_string(y.len) + ")");
    if ((int64_t)ga.size() < x.ncol) fail("gAssign needs one entry per column of X");
    const std::vector<double> cvb = cva_block(cv, G);
    check(brr_BayesRSamplerV2Groups(path_of(outputFile), s, Rf_asInteger(max_iterations), Rf_asInteger(burn_in),
                                    Rf_asInteger(thinning), x.p, y.len, x.ncol, y.p, Rf_asReal(sigma0),
                                    Rf_asReal(v0E), Rf_asReal(s02E), Rf_asReal(v0G), Rf_asReal(s02G), cvb.data(),
                                    (int32_t)cv.ncol, G, ga.data(), f.p, f.ncol, &o));
  });
}

SEXP _BayesRRcpp_HorseshoeR(SEXP outputFile, SEXP seed, SEXP max_iterations, SEXP burn_in,
                            SEXP thinning, SEXP X, SEXP Y, SEXP A, SEXP v0E, SEXP s02E, SEXP vL,
                            SEXP vT, SEXP c2, SEXP vC, SEXP sC) {
  return guarded([&] {
    Protect prot;
    const int s = resolve_seed(Rf_asInteger(seed));
    brr_options o = options_for();
    const Real x = as_real(prot, X, "X"), y = as_real(prot, Y, "Y");
    // N = Y.size(), M = X.cols() (src/HorseshoeR.cpp:113-114)
    if (x.nrow != y.len) fail("X has " + std::to_string(x.nrow) + " rows but Y has " + std::to_string(y.len) + " entries");
    check(brr_HorseshoeR(path_of(outputFile), s, Rf_asInteger(max_iterations), Rf_asInteger(burn_in),
                         Rf_asInteger(thinning), x.p, y.len, x.ncol, y.p, Rf_asReal(A), Rf_asReal(v0E),
                         Rf_asReal(s02E), Rf_asReal(vL), Rf_asReal(vT), Rf_asReal(c2), Rf_asReal(vC), Rf_asReal(sC),
                         &o));
  });
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
