// Test driver for r_shim/RcppExports.cpp without R: a minimal in-memory implementation of the R API
// the shim declares (tests/r_api/*.h) and a recording stand-in for libbrr's one-shot entry points,
// so tests/test_r_shim.py can check what the shim hands to the C ABI: coercion of integer inputs
// to double (as Rcpp's input_parameter<Eigen::MatrixXd> does), N from epsilon for BRV2Grstart,
// cva repacked to groups rows, errors for inconsistent sizes.  Test infrastructure only.
#include <R.h>
#include <R_ext/Rdynload.h>
#include <Rinternals.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <csetjmp>
#include <string>
#include <vector>

#include "brr.h"

struct SEXPREC {
  int type = REALSXP;
  bool matrix = false;
  int nrow = 0, ncol = 0;
  std::vector<double> r;
  std::vector<int> i;
  std::string s;
};
static SEXPREC nil;
SEXP R_NilValue = &nil;
static std::vector<SEXPREC *> pool;
static int nprot = 0;
static jmp_buf on_error;
static std::string last_r_error;

extern "C" {
void REprintf(const char *fmt, ...) { (void)fmt; }
void GetRNGstate(void) {}
void PutRNGstate(void) {}
double unif_rand(void) { return 0.25; }
void Rf_error(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  last_r_error = buf;
  longjmp(on_error, 1);
}
SEXP Rf_protect(SEXP x) { ++nprot; return x; }
void Rf_unprotect(int n) { nprot -= n; }
int TYPEOF(SEXP x) { return x->type; }
double *REAL(SEXP x) { return x->r.data(); }
int *INTEGER(SEXP x) { return x->i.data(); }
R_xlen_t XLENGTH(SEXP x) { return x->type == REALSXP ? (R_xlen_t)x->r.size() : x->type == STRSXP ? 1 : (R_xlen_t)x->i.size(); }
int Rf_nrows(SEXP x) { return x->matrix ? x->nrow : (int)XLENGTH(x); }
int Rf_ncols(SEXP x) { return x->matrix ? x->ncol : 1; }
int Rf_isMatrix(SEXP x) { return x->matrix; }
int Rf_isNumeric(SEXP x) { return x->type == REALSXP || x->type == INTSXP; }
int Rf_isLogical(SEXP x) { return x->type == LGLSXP; }
int Rf_isString(SEXP x) { return x->type == STRSXP; }
int Rf_asInteger(SEXP x) { return x->type == REALSXP ? (int)x->r[0] : x->i[0]; }
double Rf_asReal(SEXP x) { return x->type == REALSXP ? x->r[0] : (double)x->i[0]; }
SEXP STRING_ELT(SEXP x, R_xlen_t) { return x; }
const char *CHAR(SEXP x) { return x->s.c_str(); }
SEXP Rf_coerceVector(SEXP x, SEXPTYPE t) {
  SEXPREC *c = new SEXPREC(*x);
  pool.push_back(c);
  c->type = (int)t;
  if (t == REALSXP && x->type != REALSXP) { c->r.assign(x->i.begin(), x->i.end()); c->i.clear(); }
  if (t == INTSXP && x->type == REALSXP) { c->i.assign(x->r.begin(), x->r.end()); c->r.clear(); }
  return c;
}
int R_registerRoutines(DllInfo *, const void *, const R_CallMethodDef *, const void *, const void *) { return 1; }
Rboolean R_useDynamicSymbols(DllInfo *, Rboolean) { return TRUE; }

// ---- recording stand-ins for libbrr ----
static std::string rec;
static void put(const char *k, double v) { char b[64]; snprintf(b, sizeof b, "%s=%.17g ", k, v); rec += b; }
static void putv(const char *k, const double *p, int64_t n) { rec += k; rec += "=["; for (int64_t j = 0; j < n; ++j) { char b[40]; snprintf(b, sizeof b, "%s%.17g", j ? "," : "", p[j]); rec += b; } rec += "] "; }
static void puti(const char *k, const int32_t *p, int64_t n) { rec += k; rec += "=["; for (int64_t j = 0; j < n; ++j) { char b[24]; snprintf(b, sizeof b, "%s%d", j ? "," : "", p[j]); rec += b; } rec += "] "; }
void brr_options_default(brr_options *o) { memset(o, 0, sizeof *o); o->abi_version = BRR_ABI_VERSION; o->shard_count = 1; }
const char *brr_last_error(void) { return "mock"; }
int brr_BayesRSamplerV2(const char *f, int seed, int mi, int bi, int th, const double *X, int64_t N, int64_t M,
                        const double *Y, double, double, double, double, double, const double *cva, int32_t ncva,
                        const brr_options *) {
  rec = std::string("V2 file=") + f + " "; put("seed", seed); put("it", mi); put("burn", bi); put("thin", th);
  put("N", (double)N); put("M", (double)M); putv("X", X, N * M); putv("Y", Y, N); putv("cva", cva, ncva);
  return 0;
}
int brr_BayesRSamplerV2Groups(const char *, int, int, int, int, const double *X, int64_t N, int64_t M, const double *Y,
                              double, double, double, double, double, const double *cva, int32_t ncva, int G,
                              const int32_t *ga, const double *fixed, int64_t F, const brr_options *) {
  rec = "GROUPS "; put("N", (double)N); put("M", (double)M); put("F", (double)F); put("G", G); putv("X", X, N * M);
  putv("Y", Y, N); putv("cva", cva, (int64_t)G * ncva); puti("gA", ga, M); putv("fixed", fixed, N * F);
  return 0;
}
int brr_BRV2Grstart(const char *, int, int, int, int, double mu, const double *beta, double sigmaE, const double *sgg,
                    const double *X, int64_t N, int64_t M, const double *eps, const double *comp, double, double,
                    double, double, double, const double *cva, int32_t ncva, int G, const int32_t *ga,
                    const brr_options *) {
  rec = "RESTART "; put("N", (double)N); put("M", (double)M); put("mu", mu); put("sigmaE", sigmaE);
  putv("beta", beta, M); putv("sgg", sgg, G); putv("X", X, N * M); putv("eps", eps, N); putv("comp", comp, M);
  putv("cva", cva, (int64_t)G * ncva); puti("gA", ga, M);
  return 0;
}
int brr_HorseshoeR(const char *, int, int, int, int, const double *X, int64_t N, int64_t M, const double *Y, double A,
                   double, double, double, double, double, double, double, const brr_options *) {
  rec = "HS "; put("N", (double)N); put("M", (double)M); put("A", A); putv("X", X, N * M); putv("Y", Y, N);
  return 0;
}
SEXP _BayesRRcpp_BayesRSamplerV2(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP);
SEXP _BayesRRcpp_BayesRSamplerV2Groups(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP,
                                       SEXP, SEXP, SEXP);
SEXP _BayesRRcpp_BRV2Grstart(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP,
                             SEXP, SEXP, SEXP, SEXP, SEXP);
SEXP _BayesRRcpp_HorseshoeR(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP);
}

static SEXP mk(SEXPREC v) { SEXPREC *c = new SEXPREC(std::move(v)); pool.push_back(c); return c; }
static SEXP dbl(std::vector<double> v) { SEXPREC s; s.r = std::move(v); return mk(s); }
static SEXP num(double v) { return dbl({v}); }
static SEXP integer(std::vector<int> v) { SEXPREC s; s.type = INTSXP; s.i = std::move(v); return mk(s); }
static SEXP imat(int nr, int nc, std::vector<int> v) { SEXPREC s; s.type = INTSXP; s.matrix = true; s.nrow = nr; s.ncol = nc; s.i = std::move(v); return mk(s); }
static SEXP dmat(int nr, int nc, std::vector<double> v) { SEXPREC s; s.matrix = true; s.nrow = nr; s.ncol = nc; s.r = std::move(v); return mk(s); }
static SEXP str(const char *v) { SEXPREC s; s.type = STRSXP; s.s = v; return mk(s); }

template <class F>
static void run(const char *name, F f) {
  rec.clear();
  last_r_error.clear();
  nprot = 0;
  if (setjmp(on_error) == 0) f();
  printf("%s|%s|%s|%d\n", name, rec.c_str(), last_r_error.c_str(), nprot);
}

int main() {
  // integer 3 x 2 genotype matrix (0/1/2) and integer Y: coerced to double like Rcpp does
  run("v2_int", [] {
    _BayesRRcpp_BayesRSamplerV2(str("out.csv"), integer({7}), integer({20}), integer({10}), integer({2}),
                                imat(3, 2, {0, 1, 2, 2, 1, 0}), integer({1, 2, 3}), num(0.01), num(1e-4), num(1e-3),
                                num(1e-4), num(1e-3), dbl({1e-4, 1e-3, 1e-2}));
  });
  run("v2_rows_mismatch", [] {
    _BayesRRcpp_BayesRSamplerV2(str("out.csv"), integer({7}), integer({20}), integer({10}), integer({2}),
                                dmat(3, 2, {0, 1, 2, 2, 1, 0}), dbl({1, 2}), num(0.01), num(1e-4), num(1e-3),
                                num(1e-4), num(1e-3), dbl({1e-4}));
  });
  // cva with 3 rows for 2 groups: rows beyond `groups` dropped; integer gAssign, fixed N x 1
  run("groups_cva", [] {
    _BayesRRcpp_BayesRSamplerV2Groups(str("g.csv"), integer({1}), integer({5}), integer({1}), integer({1}),
                                      dmat(2, 3, {1, 2, 3, 4, 5, 6}), dbl({0.5, -0.5}), num(0.01), num(1e-4),
                                      num(1e-3), num(1e-4), num(1e-3), dmat(3, 2, {1, 2, 3, 10, 20, 30}),
                                      integer({2}), dbl({0, 1, 1}), dmat(2, 1, {0, 0}));
  });
  run("groups_cva_short", [] {
    _BayesRRcpp_BayesRSamplerV2Groups(str("g.csv"), integer({1}), integer({5}), integer({1}), integer({1}),
                                      dmat(2, 3, {1, 2, 3, 4, 5, 6}), dbl({0.5, -0.5}), num(0.01), num(1e-4),
                                      num(1e-3), num(1e-4), num(1e-3), dmat(1, 2, {1, 10}), integer({2}),
                                      integer({0, 1, 1}), dmat(2, 1, {0, 0}));
  });
  // restart: N = length(epsilon); integer components and beta as an M x 1 matrix
  run("restart", [] {
    _BayesRRcpp_BRV2Grstart(str("r.csv"), integer({3}), integer({5}), integer({1}), integer({1}), num(0.1),
                            dmat(2, 1, {0.5, 0}), num(0.9), dbl({0.2}), imat(3, 2, {0, 1, 2, 1, 1, 0}),
                            dbl({0.1, 0.2, 0.3}), integer({2, 0}), num(0.01), num(1e-4), num(1e-3), num(1e-4),
                            num(1e-3), dmat(1, 3, {1e-4, 1e-3, 1e-2}), integer({1}), integer({0, 0}));
  });
  run("restart_eps_mismatch", [] {
    _BayesRRcpp_BRV2Grstart(str("r.csv"), integer({3}), integer({5}), integer({1}), integer({1}), num(0.1),
                            dmat(2, 1, {0.5, 0}), num(0.9), dbl({0.2}), imat(3, 2, {0, 1, 2, 1, 1, 0}),
                            dbl({0.1, 0.2}), integer({2, 0}), num(0.01), num(1e-4), num(1e-3), num(1e-4),
                            num(1e-3), dmat(1, 3, {1e-4, 1e-3, 1e-2}), integer({1}), integer({0, 0}));
  });
  run("hs_logical_x", [] {
    SEXPREC l;
    l.type = LGLSXP; l.matrix = true; l.nrow = 2; l.ncol = 1; l.i = {1, 0};
    _BayesRRcpp_HorseshoeR(str("h.csv"), integer({1}), integer({5}), integer({1}), integer({1}), mk(l),
                           dbl({1.5, 2.5}), num(0.3), num(1e-3), num(1e-3), num(1), num(1), num(1), num(10),
                           num(10));
  });
  run("v2_string_x", [] {
    _BayesRRcpp_BayesRSamplerV2(str("out.csv"), integer({7}), integer({20}), integer({10}), integer({2}), str("x"),
                                dbl({1}), num(0.01), num(1e-4), num(1e-3), num(1e-4), num(1e-3), dbl({1e-4}));
  });
  return 0;
}
