/*
 * sanitize_driver.c -- TEST INFRASTRUCTURE (a sanitizer-built CPU oracle).
 *
 * Drives every path of the CPU oracle (brr_oracle.c) on a small synthetic cohort so that a build
 * with -fsanitize=address,undefined (oracle/Makefile target `sanitize`, run by
 * tests/test_oracle_sanitized.py) checks the restatement for out-of-bounds accesses, leaks and
 * undefined behaviour: BayesRSamplerV2 in the three visit orders, Groups with fixed effects and
 * gAssign, BRV2Grstart from a Groups state, HorseshoeR, the in-process 2-shard emulation, the
 * shard_only exchange protocol, forced-state setters and the reference CSV writers.  Prints one
 * checksum line per case; exits non-zero on any failed call.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "brr_oracle.h"

#define NROW 150
#define NCOL 96
#define CHECK(x)                                               \
  do {                                                         \
    if ((x) != 0) {                                            \
      fprintf(stderr, "FAILED: %s (line %d)\n", #x, __LINE__); \
      exit(1);                                                 \
    }                                                          \
  } while (0)

static double X[NROW * NCOL], Y[NROW], FX[NROW * 2], BT[NCOL];
static const double CVA[3] = {1e-4, 1e-3, 1e-2};

static double checksum(const orc *o) {
  double buf[NROW > NCOL ? NROW : NCOL], acc = 0.0;
  const int which[] = {ORC_V_BETA, ORC_V_EPS, ORC_V_COMP, ORC_V_PI};
  for (int w = 0; w < 4; ++w) {
    const int64_t n = orc_get_vector(o, which[w], NULL);
    if (n < 0 || n > (int64_t)(sizeof buf / sizeof buf[0])) exit(2);
    orc_get_vector(o, which[w], buf);
    for (int64_t i = 0; i < n; ++i) acc += fabs(buf[i]) * (1.0 + 1e-3 * (double)i);
  }
  return acc + orc_get_scalar(o, ORC_S_SIGMAE) + orc_get_scalar(o, ORC_S_MU);
}

static orc_config base(int model) {
  orc_config c;
  memset(&c, 0, sizeof c);
  c.model = model;
  c.N = NROW;
  c.P = NCOL;
  c.K = model == ORC_HORSESHOE ? 1 : 4;
  c.G = 1;
  c.X = X;
  c.Y = Y;
  c.cva = CVA;
  c.sigma0 = 0.01; c.v0E = 1e-4; c.s02E = 1e-3; c.v0G = 1e-4; c.s02G = 1e-3;
  c.A = 0.02; c.vL = 1.0; c.vT = 1.0; c.c2 = 1.0; c.vC = 10.0; c.sC = 10.0;
  c.seed = 7;
  c.block_size = 32;
  c.n_shards = 1;
  c.shard_only = -1;
  return c;
}

static orc *run(const orc_config *c, int sweeps, const char *tag) {
  orc *o = orc_create(c);
  if (!o) { fprintf(stderr, "FAILED: orc_create %s\n", tag); exit(1); }
  CHECK(orc_init(o));
  CHECK(orc_sweep(o, sweeps));
  printf("%-22s %.12e\n", tag, checksum(o));
  return o;
}

int main(int argc, char **argv) {
  const char *dir = argc > 1 ? argv[1] : ".";
  CHECK(orc_synth_x(20261015, NROW, NCOL, 0, X));
  CHECK(orc_synth_beta(20261015, NCOL, 10, 0, NCOL, BT));
  for (int i = 0; i < NROW; ++i) {
    double g = 0.0;
    for (int j = 0; j < NCOL; ++j) g += X[(size_t)j * NROW + i] * BT[j];
    Y[i] = g + 0.3 * orc_normal(1, ORC_T_DATA_NOISE, (uint32_t)i, 0, 0);
    FX[i] = 1.0;
    FX[NROW + i] = (double)(i % 3) - 1.0;
  }
  /* V2, three visit orders */
  for (int m = 0; m < 3; ++m) {
    orc_config c = base(ORC_V2);
    c.order_mode = m;
    char tag[32];
    snprintf(tag, sizeof tag, "v2 order %d", m);
    orc_destroy(run(&c, 4, tag));
  }
  /* r_compat stream (R's generators) through V2 / Horseshoe init and sweeps */
  for (int model = 0; model < 2; ++model) {
    orc_config c = base(model ? ORC_HORSESHOE : ORC_V2);
    c.order_mode = ORC_ORDER_REFERENCE;
    orc *o = orc_create(&c);
    if (!o) { fprintf(stderr, "FAILED: orc_create r_compat\n"); exit(1); }
    CHECK(orc_set_rng_r(o, 1, 2024u));
    CHECK(orc_init(o));
    CHECK(orc_sweep(o, 4));
    printf("%-22s %.12e\n", model ? "hs r_compat" : "v2 r_compat", checksum(o));
    orc_destroy(o);
  }
  /* Groups: 3 groups, 2 fixed-effect columns */
  static int32_t gA[NCOL];
  static double cva3[3 * 3];
  for (int j = 0; j < NCOL; ++j) gA[j] = j % 3;
  for (int g = 0; g < 3; ++g)
    for (int k = 0; k < 3; ++k) cva3[k * 3 + g] = CVA[k];
  orc_config cg = base(ORC_GROUPS);
  cg.G = 3;
  cg.F = 2;
  cg.fixed = FX;
  cg.cva = cva3;
  cg.gAssign = gA;
  orc *og = run(&cg, 4, "groups G=3 F=2");
  /* restart from the Groups state */
  static double beta0[NCOL], comp0[NCOL], eps0[NROW], sgg0[3];
  orc_get_vector(og, ORC_V_BETA, beta0);
  orc_get_vector(og, ORC_V_COMP, comp0);
  orc_get_vector(og, ORC_V_EPS, eps0);
  orc_get_vector(og, ORC_V_SIGMAGG, sgg0);
  orc_config cr = cg;
  cr.model = ORC_RESTART;
  cr.F = 0;
  cr.fixed = NULL;
  cr.Y = NULL;
  cr.mu0 = orc_get_scalar(og, ORC_S_MU);
  cr.sigmaE0 = orc_get_scalar(og, ORC_S_SIGMAE);
  cr.beta0 = beta0; cr.comp0 = comp0; cr.eps0 = eps0; cr.sigmaGG0 = sgg0;
  orc_destroy(run(&cr, 3, "restart"));
  orc_destroy(og);
  /* Horseshoe, blocked and reference order */
  for (int m = 0; m < 2; ++m) {
    orc_config c = base(ORC_HORSESHOE);
    c.order_mode = m;
    orc_destroy(run(&c, 3, m ? "horseshoe ref order" : "horseshoe"));
  }
  /* column shards: in-process emulation, then the per-shard exchange protocol */
  {
    orc_config c = base(ORC_V2);
    c.n_shards = 2;
    orc_destroy(run(&c, 3, "v2 2-shard emulation"));
    orc *sh[2];
    for (int r = 0; r < 2; ++r) {
      orc_config cs = base(ORC_V2);
      cs.n_shards = 2;
      cs.shard_only = r;
      sh[r] = orc_create(&cs);
      if (!sh[r]) { fprintf(stderr, "FAILED: shard create\n"); return 1; }
      CHECK(orc_init(sh[r]));
    }
    const int64_t ns = orc_stats_size(sh[0]);
    double *de[2], *st[2], *des = calloc(NROW, sizeof(double)), *sts = calloc((size_t)ns, sizeof(double));
    for (int r = 0; r < 2; ++r) {
      de[r] = calloc(NROW, sizeof(double));
      st[r] = calloc((size_t)ns, sizeof(double));
    }
    for (int it = 0; it < 3; ++it) {
      for (int r = 0; r < 2; ++r) {
        CHECK(orc_sweep_local(sh[r]));
        CHECK(orc_exchange_get(sh[r], de[r], st[r]));
      }
      for (int i = 0; i < NROW; ++i) des[i] = de[0][i] + de[1][i];
      for (int64_t q = 0; q < ns; ++q) sts[q] = st[0][q] + st[1][q];
      for (int r = 0; r < 2; ++r) {
        CHECK(orc_exchange_set(sh[r], des, sts));
        CHECK(orc_sweep_finish(sh[r]));
      }
    }
    printf("%-22s %.12e\n", "v2 shard protocol", checksum(sh[0]) + checksum(sh[1]));
    for (int r = 0; r < 2; ++r) { orc_destroy(sh[r]); free(de[r]); free(st[r]); }
    free(des);
    free(sts);
  }
  /* forced state, one sweep */
  {
    orc_config c = base(ORC_V2);
    orc *o = orc_create(&c);
    CHECK(orc_init(o));
    static double b[NCOL], cm[NCOL];
    for (int j = 0; j < NCOL; ++j) { b[j] = (j % 5 == 0) ? 0.01 * (j % 7) : 0.0; cm[j] = b[j] != 0.0 ? 1 + j % 3 : 0; }
    const double pi[4] = {0.6, 0.2, 0.15, 0.05};
    CHECK(orc_set_vector(o, ORC_V_BETA, b));
    CHECK(orc_set_vector(o, ORC_V_COMP, cm));
    CHECK(orc_set_vector(o, ORC_V_PI, pi));
    CHECK(orc_set_scalar(o, ORC_S_SIGMAE, 0.6));
    CHECK(orc_sweep(o, 1));
    printf("%-22s %.12e\n", "v2 forced state", checksum(o));
    orc_destroy(o);
  }
  /* the reference CSV writers of the four samplers */
  {
    char path[1024];
    orc_config cs[4] = {base(ORC_V2), cg, cr, base(ORC_HORSESHOE)};
    const char *names[4] = {"v2", "groups", "restart", "horseshoe"};
    for (int m = 0; m < 4; ++m) {
      snprintf(path, sizeof path, "%s/sanitize_%s.csv", dir, names[m]);
      CHECK(orc_run_csv(&cs[m], path, 12, 4, 2));
      printf("%-22s written\n", names[m]);
    }
  }
  return 0;
}
