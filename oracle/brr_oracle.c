/*
 * brr_oracle.c -- CPU restatement of the BayesRRcpp samplers. TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker; the product path never calls it.  See brr_oracle.h for scope and the
 * parity status ("parity unpinned" against reference-produced outputs: none exist).
 *
 * Build: gcc -O2 -std=c99 -ffp-contract=off -fPIC -shared (oracle/Makefile).
 * -ffp-contract=off mirrors the reference's Eigen expressions compiled without FMA
 * (R's default package flags carry no -march, so no FMA contraction on x86-64).
 */
#define _POSIX_C_SOURCE 200809L
#include "brr_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAXK 16
#define ORC_LN2 0.693147180559945309417232121458
#define ORC_GAMMA_MAX_ATTEMPTS 64

/* ------------------------------------------------------------------------- */
/* Philox4x32-10 (Salmon et al., SC'11; Random123).  Counter = {slot, tag, entity,
 * iteration}, key = seed.  The GPU side uses rocRAND's engine for the same block
 * function (bayesrrcpp_amd/csrc/brr_rng.hpp). */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void philox_draw(uint64_t seed, uint32_t slot, uint32_t tag, uint32_t entity,
                        uint32_t it, uint32_t w[4]) {
  uint32_t ctr[4] = {slot, tag, entity, it};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  orc_philox4x32_10(ctr, key, w);
}

/* 53-bit uniform strictly inside (0,1): exact in double on every IEEE machine */
double orc_u53(uint32_t hi, uint32_t lo) {
  uint64_t x = ((((uint64_t)hi) << 32) | (uint64_t)lo) >> 11;
  return ((double)x + 0.5) * 0x1p-53;
}

/* ------------------------------------------------------------------------- */
/* r_compat backend: R's default generators, restated from R's published
 * nmath / RNG.c algorithms (R itself is not in this image): Mersenne-Twister unif_rand with
 * set.seed's scrambling, Inversion norm_rand (qnorm5, Wichura AS241), exp_rand (Ahrens &
 * Dieter 1972 SA), rgamma (Ahrens & Dieter 1982 GD for a >= 1, 1974 GS for a < 1) and
 * rbeta(1,1) (Cheng 1978 BC, the only beta the reference draws: src/distributions.cpp:58).
 * The draws are taken from ONE sequential stream in the reference's call order (the
 * samplers below call them in that order), so given R's set.seed value the chain would be
 * the reference's own.  Pinned: unif_rand / norm_rand against R's documented outputs
 * (tests/test_oracle.py, set.seed(42) runif, set.seed(1) / set.seed(123) rnorm);
 * exp_rand / rgamma / rbeta: parity unpinned (no R here), checked by moments only. */
#define R_MT_N 624
#define R_MT_M 397
struct orc_rstream {
  uint32_t mt[R_MT_N];
  int mti;
  double aa, aaa, s, s2, d, q0, b, si, c; /* rgamma's saved constants (rgamma.c statics) */
};

/* set.seed(seed) with kind = "Mersenne-Twister" (RNG.c Randomize / RNG_Init / FixupSeeds):
 * 50 initial LCG scrambles, then 625 LCG outputs: dummy[0] (mti, forced to 624) and mt[] */
orc_rstream *orc_rstream_create(uint32_t seed) {
  orc_rstream *r = (orc_rstream *)calloc(1, sizeof(orc_rstream));
  for (int j = 0; j < 50; ++j) seed = 69069u * seed + 1u;
  seed = 69069u * seed + 1u; /* i_seed[0] = dummy[0] (mti), reset to N by FixupSeeds */
  for (int j = 0; j < R_MT_N; ++j) {
    seed = 69069u * seed + 1u;
    r->mt[j] = seed;
  }
  r->mti = R_MT_N;
  r->aa = r->aaa = 0.0;
  return r;
}
void orc_rstream_destroy(orc_rstream *r) { free(r); }

static double r_mt_genrand(orc_rstream *r) {
  static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
  uint32_t y;
  if (r->mti >= R_MT_N) {
    int kk;
    for (kk = 0; kk < R_MT_N - R_MT_M; ++kk) {
      y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
      r->mt[kk] = r->mt[kk + R_MT_M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < R_MT_N - 1; ++kk) {
      y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
      r->mt[kk] = r->mt[kk + (R_MT_M - R_MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (r->mt[R_MT_N - 1] & 0x80000000u) | (r->mt[0] & 0x7fffffffu);
    r->mt[R_MT_N - 1] = r->mt[R_MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    r->mti = 0;
  }
  y = r->mt[r->mti++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return (double)y * 2.3283064365386963e-10; /* [0,1) */
}

/* unif_rand(): MT_genrand through fixup() (strictly inside (0,1)) */
double orc_r_unif(orc_rstream *r) {
  const double i2_32m1 = 2.328306437080797e-10; /* 1/(2^32 - 1) */
  double v = r_mt_genrand(r);
  if (v <= 0.0) return 0.5 * i2_32m1;
  if (1.0 - v <= 0.0) return 1.0 - 0.5 * i2_32m1;
  return v;
}

/* qnorm(p, 0, 1, lower = TRUE, log = FALSE): Wichura (1988) AS241 PPND16 */
static double r_qnorm(double p) {
  const double q = p - 0.5;
  double r, val;
  if (fabs(q) <= 0.425) {
    r = 0.180625 - q * q;
    return q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r +
                    45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
                 133.14166789178437745) * r + 3.387132872796366608) /
           (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r +
                21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
             42.313330701600911252) * r + 1.0);
  }
  r = q < 0 ? p : 1.0 - p;
  r = sqrt(-log(r));
  if (r <= 5.0) {
    r += -1.6;
    val = (((((((r * 7.7454501427834140764e-4 + 0.0227238449892691845833) * r + 0.24178072517745061177) * r +
               1.27045825245236838258) * r + 3.64784832476320460504) * r + 5.7694972214606914055) * r +
            4.6303378461565452959) * r + 1.42343711074968357734) /
          (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r + 0.0151986665636164571966) * r +
               0.14810397642748007459) * r + 0.68976733498510000455) * r + 1.6763848301838038494) * r +
            2.05319162663775882187) * r + 1.0);
  } else {
    r += -5.0;
    val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r + 0.0012426609473880784386) * r +
               0.026532189526576123093) * r + 0.29656057182850489123) * r + 1.7848265399172913358) * r +
            5.4637849111641143699) * r + 6.6579046435011037772) /
          (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r + 1.8463183175100546818e-5) * r +
               7.868691311456132591e-4) * r + 0.0148753612908506148525) * r + 0.13692988092273580531) * r +
            0.59983220655588793769) * r + 1.0);
  }
  return q < 0.0 ? -val : val;
}

/* norm_rand() with normal.kind = "Inversion": two uniforms for 2^27-fold resolution */
double orc_r_norm(orc_rstream *r) {
  const double BIG = 134217728.0; /* 2^27 */
  double u = orc_r_unif(r);
  u = (int)(BIG * u) + orc_r_unif(r);
  return r_qnorm(u / BIG);
}

/* exp_rand(): Ahrens & Dieter (1972) algorithm SA; q[k] = sum_{i=1..k+1} ln2^i / i! */
double orc_r_exp(orc_rstream *r) {
  static double q[16];
  static int qinit = 0;
  if (!qinit) {
    double term = 1.0, s = 0.0;
    for (int k = 0; k < 16; ++k) {
      term *= ORC_LN2 / (double)(k + 1);
      s += term;
      q[k] = s;
    }
    q[15] = 1.0;
    qinit = 1;
  }
  double a = 0.0;
  double u = orc_r_unif(r);
  while (u <= 0.0 || u >= 1.0) u = orc_r_unif(r);
  for (;;) {
    u += u;
    if (u > 1.0) break;
    a += q[0];
  }
  u -= 1.0;
  if (u <= q[0]) return a + u;
  int i = 0;
  double ustar = orc_r_unif(r), umin = ustar;
  do {
    ustar = orc_r_unif(r);
    if (umin > ustar) umin = ustar;
    i++;
  } while (u > q[i]);
  return a + umin * q[0];
}

/* rgamma(a, scale = 1) (nmath/rgamma.c) */
double orc_r_gamma(orc_rstream *r, double a) {
  const double sqrt32 = 5.656854, exp_m1 = 0.36787944117144233;
  const double q1 = 0.04166669, q2 = 0.02083148, q3 = 0.00801191, q4 = 0.00144121, q5 = -7.388e-5,
               q6 = 2.4511e-4, q7 = 2.424e-4;
  const double a1 = 0.3333333, a2 = -0.250003, a3 = 0.2000062, a4 = -0.1662921, a5 = 0.1423657,
               a6 = -0.1367177, a7 = 0.1233795;
  double e, p, q, t, u, v, w, x, ret_val;
  if (!(a > 0.0)) return 0.0;
  if (a < 1.0) { /* GS */
    e = 1.0 + exp_m1 * a;
    for (;;) {
      p = e * orc_r_unif(r);
      if (p >= 1.0) {
        x = -log((e - p) / a);
        if (orc_r_exp(r) >= (1.0 - a) * log(x)) break;
      } else {
        x = exp(log(p) / a);
        if (orc_r_exp(r) >= x) break;
      }
    }
    return x;
  }
  if (a != r->aa) {
    r->aa = a;
    r->s2 = a - 0.5;
    r->s = sqrt(r->s2);
    r->d = sqrt32 - r->s * 12.0;
  }
  const double s = r->s, s2 = r->s2, d = r->d;
  t = orc_r_norm(r);
  x = s + 0.5 * t;
  ret_val = x * x;
  if (t >= 0.0) return ret_val;
  u = orc_r_unif(r);
  if (d * u <= t * t * t) return ret_val;
  if (a != r->aaa) {
    r->aaa = a;
    const double rr = 1.0 / a;
    r->q0 = ((((((q7 * rr + q6) * rr + q5) * rr + q4) * rr + q3) * rr + q2) * rr + q1) * rr;
    if (a <= 3.686) {
      r->b = 0.463 + s + 0.178 * s2;
      r->si = 1.235;
      r->c = 0.195 / s - 0.079 + 0.16 * s;
    } else if (a <= 13.022) {
      r->b = 1.654 + 0.0076 * s2;
      r->si = 1.68 / s + 0.275;
      r->c = 0.062 / s + 0.024;
    } else {
      r->b = 1.77;
      r->si = 0.75;
      r->c = 0.1515 / s;
    }
  }
  const double q0 = r->q0, b = r->b, si = r->si, c = r->c;
  if (x > 0.0) {
    v = t / (s + s);
    if (fabs(v) <= 0.25)
      q = q0 + 0.5 * t * t * ((((((a7 * v + a6) * v + a5) * v + a4) * v + a3) * v + a2) * v + a1) * v;
    else
      q = q0 - s * t + 0.25 * t * t + (s2 + s2) * log(1.0 + v);
    if (log(1.0 - u) <= q) return ret_val;
  }
  for (;;) {
    e = orc_r_exp(r);
    u = orc_r_unif(r);
    u = u + u - 1.0;
    t = u < 0.0 ? b - si * e : b + si * e;
    if (t >= -0.71874483771719) {
      v = t / (s + s);
      if (fabs(v) <= 0.25)
        q = q0 + 0.5 * t * t * ((((((a7 * v + a6) * v + a5) * v + a4) * v + a3) * v + a2) * v + a1) * v;
      else
        q = q0 - s * t + 0.25 * t * t + (s2 + s2) * log(1.0 + v);
      if (q > 0.0) {
        w = expm1(q);
        if (c * fabs(u) <= w * exp(e - 0.5 * t * t)) break;
      }
    }
  }
  x = s + 0.5 * t;
  return x * x;
}

/* rbeta(1, 1): Cheng (1978) algorithm BC with a = b = 1 (beta = 1, delta = 1, k1 = 0.25,
 * k2 = 1, alpha = 2), returning a / (a + w) as rbeta.c does when aa == max(aa, bb) */
double orc_r_beta11(orc_rstream *r) {
  const double a = 1.0, alpha = 2.0, beta = 1.0, k1 = 0.25, k2 = 1.0;
  const double expmax = DBL_MAX_EXP * ORC_LN2;
  double u1, u2, v = 0.0, w = 0.0, y, z;
  for (;;) {
    u1 = orc_r_unif(r);
    u2 = orc_r_unif(r);
    if (u1 < 0.5) {
      y = u1 * u2;
      z = u1 * y;
      if (0.25 * u2 + z - y >= k1) continue;
    } else {
      z = u1 * u1 * u2;
      if (z <= 0.25) {
        v = beta * log(u1 / (1.0 - u1));
        w = v <= expmax ? a * exp(v) : DBL_MAX;
        if (!isfinite(w)) w = DBL_MAX;
        break;
      }
      if (z >= k2) continue;
    }
    v = beta * log(u1 / (1.0 - u1));
    w = v <= expmax ? a * exp(v) : DBL_MAX;
    if (!isfinite(w)) w = DBL_MAX;
    if (alpha * (log(alpha / (a + w)) + v) - 1.3862944 >= log(z)) break;
  }
  return a / (a + w);
}

/* the stream of the orc being driven (set by the public entry points): NULL = Philox */
static __thread orc_rstream *g_rs = NULL;

double orc_uniform(uint64_t seed, uint32_t tag, uint32_t entity, uint32_t it, uint32_t slot) {
  if (g_rs) return orc_r_unif(g_rs); /* R::runif(0, 1) = unif_rand() */
  uint32_t w[4];
  philox_draw(seed, slot, tag, entity, it, w);
  return orc_u53(w[0], w[1]);
}

/* beta_rng(1,1) call sites (src/distributions.cpp:58): a uniform under Philox, R::rbeta(1,1)
 * under r_compat */
static double orc_beta11(uint64_t seed, uint32_t tag, uint32_t entity, uint32_t it, uint32_t slot) {
  if (g_rs) return orc_r_beta11(g_rs);
  return orc_uniform(seed, tag, entity, it, slot);
}

static double box_muller(const uint32_t w[4]) {
  double u1 = orc_u53(w[0], w[1]);
  double u2 = orc_u53(w[2], w[3]);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586476925286766559 * u2);
}

double orc_normal(uint64_t seed, uint32_t tag, uint32_t entity, uint32_t it, uint32_t slot) {
  if (g_rs) return orc_r_norm(g_rs); /* R::rnorm(mean, sd) = mean + sd * norm_rand() */
  uint32_t w[4];
  philox_draw(seed, slot, tag, entity, it, w);
  return box_muller(w);
}

/* Gamma(shape, 1): Marsaglia-Tsang (ACM TOMS 26(3) 2000) with the U^(1/a) boost for a<1.
 * Attempt t uses slots 2t (normal) and 2t+1 (acceptance uniform); the boost uniform uses
 * slot 0xFFFFFFFF.  Replaces R::rgamma (src/distributions.cpp:17,22,25,31). */
double orc_gamma(uint64_t seed, double shape, uint32_t tag, uint32_t entity, uint32_t it) {
  if (!(shape > 0.0)) return 0.0;
  if (g_rs) return orc_r_gamma(g_rs, shape); /* R::rgamma(shape, 1); callers apply the scale */
  double boost = 1.0;
  double a = shape;
  if (a < 1.0) {
    double u = orc_uniform(seed, tag, entity, it, 0xFFFFFFFFu);
    boost = pow(u, 1.0 / a);
    a += 1.0;
  }
  double d = a - 1.0 / 3.0;
  double c = 1.0 / sqrt(9.0 * d);
  for (uint32_t t = 0; t < ORC_GAMMA_MAX_ATTEMPTS; ++t) {
    uint32_t w[4];
    philox_draw(seed, 2u * t, tag, entity, it, w);
    double z = box_muller(w);
    double v = 1.0 + c * z;
    if (v <= 0.0) continue;
    v = v * v * v;
    philox_draw(seed, 2u * t + 1u, tag, entity, it, w);
    double u = orc_u53(w[0], w[1]);
    if (log(u) < 0.5 * z * z + d - d * v + d * log(v)) return d * v * boost;
  }
  return d * boost;
}

/* ---- distributions.cpp restatement (src/distributions.cpp:21-39) ---- */
/* inv_gamma_rng(shape, scale) = 1/R::rgamma(shape, 1/scale)           :21-23 */
static double inv_gamma_rng(uint64_t s, double shape, double scale, uint32_t tag,
                            uint32_t ent, uint32_t it) {
  return 1.0 / ((1.0 / scale) * orc_gamma(s, shape, tag, ent, it));
}
/* inv_gamma_rate_rng(shape, rate) = 1/R::rgamma(shape, 1/rate)        :27-32 */
static double inv_gamma_rate_rng(uint64_t s, double shape, double rate, uint32_t tag,
                                 uint32_t ent, uint32_t it) {
  return 1.0 / ((1.0 / rate) * orc_gamma(s, shape, tag, ent, it));
}
/* inv_scaled_chisq_rng(dof, scale) = inv_gamma_rng(dof/2, dof*scale/2) :34-36 */
static double inv_scaled_chisq_rng(uint64_t s, double dof, double scale, uint32_t tag,
                                   uint32_t ent, uint32_t it) {
  return inv_gamma_rng(s, 0.5 * dof, 0.5 * dof * scale, tag, ent, it);
}
/* dirichilet_rng(alpha): normalised gammas                             :12-20 */
static void dirichlet_rng(uint64_t s, const double *alpha, int K, double *out,
                          uint32_t tag, uint32_t ent0, uint32_t it) {
  double sum = 0.0;
  for (int k = 0; k < K; ++k) {
    out[k] = orc_gamma(s, alpha[k], tag, ent0 + (uint32_t)k, it);
  }
  for (int k = 0; k < K; ++k) sum += out[k];
  for (int k = 0; k < K; ++k) out[k] /= sum;
}

/* ------------------------------------------------------------------------- */
/* glibc rand() (random_r TYPE_3: x[i] = x[i-3] + x[i-31], output x >> 1) seeded by
 * srand(s).  std::random_shuffle calls rand() (stl_algo.h:4576-4580). */
typedef struct glibc_rand {
  int32_t r[34];
  int idx;        /* ring position: r holds x[i-34..i-1] */
} glibc_rand;

static void glibc_srand(glibc_rand *g, uint32_t seed) {
  int32_t x[344 + 34];
  if (seed == 0) seed = 1;
  x[0] = (int32_t)seed;
  for (int i = 1; i < 31; ++i) {
    /* x[i] = (16807 * x[i-1]) % 2147483647 via Schrage, as glibc srandom_r */
    int32_t hi = x[i - 1] / 127773;
    int32_t lo = x[i - 1] % 127773;
    int32_t word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    x[i] = word;
  }
  for (int i = 31; i < 34; ++i) x[i] = x[i - 31];
  for (int i = 34; i < 344; ++i) x[i] = (int32_t)((uint32_t)x[i - 31] + (uint32_t)x[i - 3]);
  for (int i = 0; i < 34; ++i) g->r[i] = x[310 + i];
  g->idx = 0;
}

static int32_t glibc_next(glibc_rand *g) {
  /* ring holds the last 34 values; new = old[-31] + old[-3] */
  int i = g->idx;
  int32_t v = (int32_t)((uint32_t)g->r[(i + 34 - 31) % 34] + (uint32_t)g->r[(i + 34 - 3) % 34]);
  g->r[i] = v;
  g->idx = (i + 1) % 34;
  return (int32_t)(((uint32_t)v) >> 1);
}

void orc_glibc_rand(uint32_t s, int n, int32_t *out) {
  glibc_rand g;
  glibc_srand(&g, s);
  for (int i = 0; i < n; ++i) out[i] = glibc_next(&g);
}

/* libstdc++ std::random_shuffle(first,last) (stl_algo.h:4575-4583) */
static void random_shuffle_ref(glibc_rand *g, int32_t *a, int64_t n) {
  if (n <= 0) return;
  for (int64_t i = 1; i < n; ++i) {
    int64_t j = (int64_t)(glibc_next(g) % (int32_t)(i + 1));
    if (i != j) { int32_t t = a[i]; a[i] = a[j]; a[j] = t; }
  }
}

/* Philox Fisher-Yates (device fast-path spec for the order inside a block, DESIGN.md "visit order") */
static void fisher_yates(uint64_t seed, int32_t *a, int64_t n, uint32_t tag, uint32_t entity,
                         uint32_t it) {
  for (int64_t i = n - 1; i >= 1; --i) {
    uint32_t w[4];
    philox_draw(seed, (uint32_t)(i >> 2), tag, entity, it, w);
    uint32_t word = w[i & 3];
    int64_t j = (int64_t)(((uint64_t)word * (uint64_t)(i + 1)) >> 32);
    int32_t t = a[i]; a[i] = a[j]; a[j] = t;
  }
}

void orc_blocked_order(uint64_t seed, uint32_t it, int64_t P, int32_t B, int32_t shard,
                       int64_t col_offset, int32_t *order) {
  int64_t nb = (P + B - 1) / B;
  int32_t *blk = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nb > 0 ? nb : 1));
  int32_t *w = (int32_t *)malloc(sizeof(int32_t) * (size_t)B);
  /* block cycle with a random rotation and direction: consecutive blocks in the visit order
     are neighbours in the cycle, so the device path can precompute their cross-Gram blocks */
  {
    uint32_t w4[4];
    philox_draw(seed, 0, ORC_T_PERM_BLOCK, (uint32_t)shard, it, w4);
    int64_t rot = (int64_t)(((uint64_t)w4[0] * (uint64_t)nb) >> 32);
    int64_t dir = (w4[1] & 1u) ? 1 : -1;
    for (int64_t s2 = 0; s2 < nb; ++s2) blk[s2] = (int32_t)(((rot + dir * s2) % nb + nb) % nb);
  }
  int64_t pos = 0;
  for (int64_t s = 0; s < nb; ++s) {
    int64_t b = blk[s];
    int64_t size = P - b * B < B ? P - b * B : B;
    for (int64_t i = 0; i < size; ++i) w[i] = (int32_t)i;
    fisher_yates(seed, w, size, ORC_T_PERM_WITHIN, (uint32_t)(col_offset / B + b), it);
    for (int64_t i = 0; i < size; ++i) order[pos++] = (int32_t)(col_offset + b * B + w[i]);
  }
  free(blk);
  free(w);
}

/* ------------------------------------------------------------------------- */
struct orc {
  orc_config c;
  int64_t N, P;
  int K, G, F;
  uint64_t seed;
  double *eps, *ytilde, *beta, *comp, *xsq, *sigmaGG, *pi, *v, *betaAcum, *alpha, *lambda,
      *hsv, *eps_start, *eps_acc;
  int32_t *order, *forder;
  int32_t *visit;     /* REFERENCE order over column shards: each shard's columns in global order */
  double mu, sigmaE, sigmaF, tau, eta, c2;
  int32_t it;
  glibc_rand grand;
  double *stats;      /* [sum b^2, sum b^2/lambda, betaAcum[G], v[G*K]] used by the epilogue */
  double *deps;       /* shard_only: this shard's eps - eps_start */
  orc_rstream *rs;    /* r_compat stream (orc_set_rng_r), NULL = Philox */
  int seg;            /* shard_only: the exchange segment of the current sweep (n_exchanges) */
};

static double *dalloc(int64_t n) { return (double *)calloc((size_t)(n > 0 ? n : 1), sizeof(double)); }

orc *orc_create(const orc_config *cfg) {
  if (!cfg || cfg->N < 1 || cfg->P < 1) return NULL;
  if (cfg->model != ORC_HORSESHOE && (cfg->K < 2 || cfg->K > ORC_MAXK)) return NULL;
  orc *o = (orc *)calloc(1, sizeof(orc));
  o->c = *cfg;
  o->N = cfg->N;
  o->P = cfg->P;
  o->K = cfg->model == ORC_HORSESHOE ? 1 : cfg->K;
  o->G = (cfg->model == ORC_GROUPS || cfg->model == ORC_RESTART) ? cfg->G : 1;
  if (o->G < 1) o->G = 1;
  o->F = cfg->model == ORC_GROUPS ? cfg->F : 0;
  if (o->c.n_shards < 1) o->c.n_shards = 1;
  if (o->c.shard_only >= o->c.n_shards) o->c.shard_only = -1;
  if (o->c.n_exchanges < 1 || o->c.n_shards <= 1) o->c.n_exchanges = 1;
  if (o->c.block_size < 1) o->c.block_size = 256;
  o->seed = (uint64_t)(int64_t)cfg->seed;
  o->eps = dalloc(o->N);
  o->ytilde = dalloc(o->N);
  o->eps_start = dalloc(o->N);
  o->eps_acc = dalloc(o->N);
  o->beta = dalloc(o->P);
  o->comp = dalloc(o->P);
  o->xsq = dalloc(o->P);
  o->lambda = dalloc(o->P);
  o->hsv = dalloc(o->P);
  o->sigmaGG = dalloc(o->G);
  o->pi = dalloc((int64_t)o->G * o->K);
  o->v = dalloc((int64_t)o->G * o->K);
  o->betaAcum = dalloc(o->G);
  o->alpha = dalloc(o->F);
  o->stats = dalloc(2 + o->G + (int64_t)o->G * o->K);
  o->deps = dalloc(o->N);
  o->order = (int32_t *)malloc(sizeof(int32_t) * (size_t)o->P);
  o->forder = (int32_t *)malloc(sizeof(int32_t) * (size_t)(o->F > 0 ? o->F : 1));
  for (int64_t i = 0; i < o->P; ++i) o->order[i] = (int32_t)i;
  for (int i = 0; i < o->F; ++i) o->forder[i] = i;
  glibc_srand(&o->grand, 1); /* a fresh process: rand() unseeded == srand(1) */
  return o;
}

void orc_destroy(orc *o) {
  if (!o) return;
  free(o->eps); free(o->ytilde); free(o->eps_start); free(o->eps_acc); free(o->beta);
  free(o->comp); free(o->xsq); free(o->lambda); free(o->hsv); free(o->sigmaGG); free(o->pi);
  free(o->v); free(o->betaAcum); free(o->alpha); free(o->order); free(o->forder); free(o->visit);
  free(o->stats); free(o->deps);
  orc_rstream_destroy(o->rs);
  free(o);
}

int32_t orc_iteration(const orc *o) { return o->it; }

static inline const double *xcol(const orc *o, int64_t m) { return o->c.X + m * o->N; }
static inline int group_of(const orc *o, int64_t m) {
  return o->c.gAssign ? o->c.gAssign[m] : 0;
}
static inline double cva_at(const orc *o, int g, int k /* 1..K-1 */) {
  return o->c.cva[g + (int64_t)o->G * (k - 1)];
}

static double sqnorm(const double *x, int64_t n) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += x[i] * x[i];
  return s;
}

int orc_set_rng_r(orc *o, int on, uint32_t r_seed) {
  orc_rstream_destroy(o->rs);
  o->rs = on ? orc_rstream_create(r_seed) : NULL;
  return 0;
}

static int orc_init_body(orc *o);
int orc_init(orc *o) {
  g_rs = o->rs;
  const int rc = orc_init_body(o);
  g_rs = NULL;
  return rc;
}

static int orc_init_body(orc *o) {
  const int64_t N = o->N, P = o->P;
  const int K = o->K, G = o->G;
  const uint32_t IT = ORC_INIT_IT;
  o->it = 0;
  /* xsquared = X.colwise().squaredNorm()   (BayesRv2.cpp:170, Groups :205, restart :156) */
  for (int64_t m = 0; m < P; ++m) o->xsq[m] = sqnorm(xcol(o, m), N);
  switch (o->c.model) {
    case ORC_V2:
    case ORC_GROUPS: {
      /* priorPi: Groups convention (0.5, 0.5/K, ...) (BayesRv2Groups.cpp:170-175); V2's
       * BayesRv2.cpp:150 reads cVa before assignment (UB) -- SURVEY Appendix B decision. */
      for (int g = 0; g < G; ++g) {
        o->pi[g * K + 0] = 0.5;
        for (int k = 1; k < K; ++k) o->pi[g * K + k] = 0.5 / K;
      }
      if (o->c.pi0) memcpy(o->pi, o->c.pi0, sizeof(double) * (size_t)(G * K));
      for (int64_t m = 0; m < P; ++m) { o->beta[m] = 0.0; o->comp[m] = 0.0; }
      o->mu = 0.0;
      if (o->c.model == ORC_V2) {
        o->sigmaGG[0] = orc_beta11(o->seed, ORC_T_INIT, 0, IT, 0); /* beta_rng(1,1) :162 */
      } else {
        for (int g = 0; g < G; ++g) /* :194-195 */
          o->sigmaGG[g] = orc_beta11(o->seed, ORC_T_INIT, (uint32_t)g, IT, 0);
        o->sigmaF = orc_uniform(o->seed, ORC_T_INIT, 0x10000000u, IT, 0); /* R::runif :197 */
        for (int f = 0; f < o->F; ++f) o->alpha[f] = 0.0;
      }
      /* epsilon = Y - mu - X*beta, beta = 0 (:168) ; Groups: Y - mu (:203) */
      for (int64_t i = 0; i < N; ++i) o->eps[i] = o->c.Y[i] - o->mu - 0.0;
      o->sigmaE = sqnorm(o->eps, N) / (double)N * 0.5; /* :169 */
      break;
    }
    case ORC_RESTART: {
      o->mu = o->c.mu0;
      o->sigmaE = o->c.sigmaE0;
      for (int64_t m = 0; m < P; ++m) { o->beta[m] = o->c.beta0[m]; o->comp[m] = o->c.comp0[m]; }
      for (int g = 0; g < G; ++g) o->sigmaGG[g] = o->c.sigmaGG0[g];
      for (int64_t i = 0; i < N; ++i) o->eps[i] = o->c.eps0[i];
      /* v(gAssign(i), components(i)) += 1 ; pi.row(g) = Dirichlet(v.row(g)+1) (:157-165) */
      memset(o->v, 0, sizeof(double) * (size_t)(G * K));
      for (int64_t m = 0; m < P; ++m) o->v[group_of(o, m) * K + (int)o->comp[m]] += 1.0;
      for (int g = 0; g < G; ++g) {
        double a[ORC_MAXK];
        for (int k = 0; k < K; ++k) a[k] = o->v[g * K + k] + 1.0;
        dirichlet_rng(o->seed, a, K, o->pi + g * K, ORC_T_PI, (uint32_t)(g * K), IT);
      }
      if (o->c.pi0) memcpy(o->pi, o->c.pi0, sizeof(double) * (size_t)(G * K));
      break;
    }
    case ORC_HORSESHOE: {
      /* HorseshoeR.cpp:168-195.  The 2*M discarded init draws (:176,:179) and the
       * overwritten tau=rbeta(1,1) (:171) consume R's stream only; counter-based draws
       * make them no-ops, so they are skipped; a sequential R stream consumes them. */
      if (g_rs) {
        (void)orc_r_beta11(g_rs);                                                /* :171 */
        for (int64_t m = 0; m < P; ++m) (void)orc_r_gamma(g_rs, 0.5);            /* :176 */
        for (int64_t m = 0; m < P; ++m) (void)orc_r_gamma(g_rs, 0.5 * o->c.vL);  /* :179 */
      }
      for (int64_t m = 0; m < P; ++m) { o->beta[m] = 0.0; o->hsv[m] = 1.0; o->lambda[m] = 1.0; }
      o->mu = 0.0;
      o->c2 = o->c.c2;
      for (int64_t i = 0; i < N; ++i) o->eps[i] = o->c.Y[i] - o->mu - 0.0; /* :186 */
      o->sigmaE = sqnorm(o->eps, N) / (double)N * 0.5;                      /* :187 */
      o->eta = inv_gamma_rate_rng(o->seed, 0.5, 1.0 / (o->sigmaE * pow(o->c.A, 2)),
                                  ORC_T_HS_ETA, 0, IT);                      /* :189 */
      o->tau = (1.0 / o->eta) *
               inv_gamma_rate_rng(o->seed, 0.5 * o->c.vT, o->c.vT, ORC_T_HS_TAU, 0, IT); /* :192 */
      break;
    }
    default:
      return -1;
  }
  return 0;
}

/* ---- visit order for the current iteration ---- */
static int64_t shard_range(const orc *o, int s, int64_t *col_off) {
  const int B = o->c.block_size;
  int64_t nb = (o->P + B - 1) / B;
  int S = o->c.n_shards;
  int64_t b0 = nb * s / S, b1 = nb * (s + 1) / S;
  int64_t c0 = b0 * B, c1 = b1 * B < o->P ? b1 * B : o->P;
  *col_off = c0;
  return c1 - c0;
}

static void make_orders(orc *o) {
  switch (o->c.order_mode) {
    case ORC_ORDER_REFERENCE:
      /* Groups: fixedI shuffled first (BayesRv2Groups.cpp:216), then markerI (:227);
       * both arrays persist across iterations, exactly like the reference. */
      if (o->F > 0) random_shuffle_ref(&o->grand, o->forder, o->F);
      random_shuffle_ref(&o->grand, o->order, o->P);
      if (o->c.n_shards > 1) {
        /* column shards: shard s visits ITS columns in the order the (persisting, global)
         * permutation lists them -- the reference's order restricted to the shard */
        if (!o->visit) o->visit = (int32_t *)malloc(sizeof(int32_t) * (size_t)o->P);
        int64_t pos = 0;
        for (int sh = 0; sh < o->c.n_shards; ++sh) {
          int64_t off;
          const int64_t ps = shard_range(o, sh, &off);
          for (int64_t i = 0; i < o->P; ++i)
            if (o->order[i] >= off && o->order[i] < off + ps) o->visit[pos++] = o->order[i];
        }
      }
      break;
    case ORC_ORDER_BLOCKED: {
      for (int f = 0; f < o->F; ++f) o->forder[f] = f;
      fisher_yates(o->seed, o->forder, o->F, ORC_T_PERM_FIXED, 0, (uint32_t)o->it);
      int64_t pos = 0;
      for (int s = 0; s < o->c.n_shards; ++s) {
        int64_t off;
        int64_t ps = shard_range(o, s, &off);
        orc_blocked_order(o->seed, (uint32_t)o->it, ps, o->c.block_size, s, off, o->order + pos);
        pos += ps;
      }
      break;
    }
    default:
      for (int64_t i = 0; i < o->P; ++i) o->order[i] = (int32_t)i;
      for (int f = 0; f < o->F; ++f) o->forder[f] = f;
      break;
  }
}

/* ---- per-marker mixture update: BayesRv2.cpp:188-243 / Groups :234-295 / restart :185-247 */
static void bayesr_marker(orc *o, int64_t m, double *eps) {
  const int64_t N = o->N;
  const int K = o->K;
  const double *x = xcol(o, m);
  const int g = group_of(o, m);
  const double sigmaG = o->sigmaGG[g];
  const double sigmaE = o->sigmaE;
  double cVa[ORC_MAXK], cVaI[ORC_MAXK], denom[ORC_MAXK], muk[ORC_MAXK], logL[ORC_MAXK];
  cVa[0] = 0.0;
  cVaI[0] = 0.0;
  for (int k = 1; k < K; ++k) { cVa[k] = cva_at(o, g, k); cVaI[k] = 1.0 / cVa[k]; }
  double *yt = o->ytilde;
  const double bm = o->beta[m];
  for (int64_t i = 0; i < N; ++i) yt[i] = eps[i] + x[i] * bm;               /* :191 */
  muk[0] = 0.0;
  for (int k = 1; k < K; ++k) denom[k - 1] = o->xsq[m] + (sigmaE / sigmaG) * cVaI[k]; /* :199 */
  double num = 0.0;
  for (int64_t i = 0; i < N; ++i) num += x[i] * yt[i];                       /* :201 */
  for (int k = 1; k < K; ++k) muk[k] = num / denom[k - 1];                   /* :203 */
  for (int k = 0; k < K; ++k) logL[k] = log(o->pi[g * K + k]);               /* :207 */
  for (int k = 1; k < K; ++k)                                                /* :211 */
    logL[k] = logL[k] - 0.5 * log(((sigmaG / sigmaE) * o->xsq[m]) * cVa[k] + 1.0) +
              (0.5 * (muk[k] * num)) / sigmaE;
  const uint32_t mg = (uint32_t)m;
  /* V2 :213 / restart :217 beta_rng(1,1); Groups :266 R::runif(0,1) */
  const double p = o->c.model == ORC_GROUPS ? orc_uniform(o->seed, ORC_T_MARKER, mg, (uint32_t)o->it, 0)
                                            : orc_beta11(o->seed, ORC_T_MARKER, mg, (uint32_t)o->it, 0);
  double acum;
  int guard = 0;
  for (int i = 1; i < K; ++i) guard |= fabs(logL[i] - logL[0]) > 700.0;     /* :216 */
  if (guard) {
    acum = 0.0;
  } else {
    double s = 0.0;
    for (int i = 0; i < K; ++i) s += exp(logL[i] - logL[0]);
    acum = 1.0 / s;                                                          /* :219 */
  }
  for (int k = 0; k < K; ++k) {                                              /* :222-242 */
    if (p <= acum) {
      if (k == 0) {
        o->beta[m] = 0.0;
      } else {
        const double z = orc_normal(o->seed, ORC_T_MARKER, mg, (uint32_t)o->it, 1);
        o->beta[m] = muk[k] + sqrt(sigmaE / denom[k - 1]) * z;              /* :228 */
        if (o->c.model != ORC_V2) o->betaAcum[g] += pow(o->beta[m], 2);     /* Groups :280 */
      }
      o->v[g * K + k] += 1.0;
      o->comp[m] = (double)k;
      break;
    } else if (k + 1 < K) {
      /* the reference evaluates logL[k+1] even at k = K-1 (one past the end); that value
       * can never be used because the loop ends -- in-bounds here. */
      int gk = 0;
      for (int i = 1; i < K; ++i) gk |= fabs(logL[i] - logL[k + 1]) > 700.0;
      if (!gk) {
        double s = 0.0;
        for (int i = 0; i < K; ++i) s += exp(logL[i] - logL[k + 1]);
        acum += 1.0 / s;
      }
    }
  }
  const double bn = o->beta[m];
  for (int64_t i = 0; i < N; ++i) eps[i] = yt[i] - x[i] * bn;                /* :243 */
}

/* ---- Horseshoe per-marker Gaussian update: HorseshoeR.cpp:221-238 ---- */
static void horseshoe_marker(orc *o, int64_t m, double *eps) {
  const int64_t N = o->N;
  const double *x = xcol(o, m);
  double *yt = o->ytilde;
  const double bm = o->beta[m];
  for (int64_t i = 0; i < N; ++i) yt[i] = eps[i] + x[i] * bm;               /* :224 */
  double dot = 0.0;
  for (int64_t i = 0; i < N; ++i) dot += x[i] * yt[i];
  const double tau = o->tau, c2 = o->c2, lam = o->lambda[m], sigmaE = o->sigmaE;
  const double xsq = o->xsq[m]; /* X.col(marker).squaredNorm(), same summation */
  const double s = tau * c2 * lam / (tau * lam + c2);
  const double D = xsq + (sigmaE / s);
  const double z = orc_normal(o->seed, ORC_T_MARKER, (uint32_t)m, (uint32_t)o->it, 1);
  o->beta[m] = dot / D + sqrt(sigmaE / D) * z;                               /* :234 */
  const double bn = o->beta[m];
  for (int64_t i = 0; i < N; ++i) eps[i] = yt[i] - x[i] * bn;                /* :238 */
}

static void mu_update(orc *o) {
  /* epsilon += mu ; mu = norm_rng(sum/N, sigmaE/N) ; epsilon -= mu  (BayesRv2.cpp:177-179) */
  const int64_t N = o->N;
  for (int64_t i = 0; i < N; ++i) o->eps[i] = o->eps[i] + o->mu;
  double s = 0.0;
  for (int64_t i = 0; i < N; ++i) s += o->eps[i];
  const double z = orc_normal(o->seed, ORC_T_MU, 0, (uint32_t)o->it, 0);
  o->mu = s / (double)N + sqrt(o->sigmaE / (double)N) * z;
  for (int64_t i = 0; i < N; ++i) o->eps[i] = o->eps[i] - o->mu;
}

static void fixed_effects(orc *o) {
  /* BayesRv2Groups.cpp:216-225 */
  const int64_t N = o->N;
  for (int cf = 0; cf < o->F; ++cf) {
    const int cur = o->forder[cf];
    const double *f = o->c.fixed + (int64_t)cur * N;
    const double ca = o->alpha[cur];
    for (int64_t i = 0; i < N; ++i) o->ytilde[i] = o->eps[i] + f[i] * ca;
    const double denom_f = (double)(N - 1) + (o->sigmaE / o->sigmaF);
    double num_f = 0.0;
    for (int64_t i = 0; i < N; ++i) num_f += f[i] * o->ytilde[i];
    const double z = orc_normal(o->seed, ORC_T_FIXED, (uint32_t)cur, (uint32_t)o->it, 0);
    o->alpha[cur] = num_f / denom_f + sqrt(o->sigmaE / denom_f) * z;
    const double an = o->alpha[cur];
    for (int64_t i = 0; i < N; ++i) o->eps[i] = o->ytilde[i] - f[i] * an;
  }
}

/* positions [*p0, *p1) of a shard's ps visit positions that form exchange segment e: whole
 * blocks of B positions, blocks [nbl e / E, nbl (e + 1) / E) of the shard's nbl blocks (the
 * device splits a shard's block positions the same way, brr_session.cpp seg_range) */
static void seg_positions(const orc *o, int64_t ps, int e, int64_t *p0, int64_t *p1) {
  const int64_t B = o->c.block_size, E = o->c.n_exchanges;
  const int64_t nbl = (ps + B - 1) / B;
  const int64_t b0 = nbl * e / E, b1 = nbl * (e + 1) / E;
  *p0 = b0 * B < ps ? b0 * B : ps;
  *p1 = b1 * B < ps ? b1 * B : ps;
}

/* column-sharded protocol for exchange segment e: every shard sweeps its segment's
 * positions against its own copy of epsilon from the segment start; then
 * eps = eps_start + sum_s (eps_s - eps_start).  shard_only >= 0: this process's shard only, the
 * delta left in deps for the caller's all-reduce. */
static void marker_segment(orc *o, int e) {
  const int64_t N = o->N;
  const int hs = o->c.model == ORC_HORSESHOE;
  memcpy(o->eps_start, o->eps, sizeof(double) * (size_t)N);
  memset(o->eps_acc, 0, sizeof(double) * (size_t)N);
  int64_t pos = 0;
  const int32_t *ord = (o->c.order_mode == ORC_ORDER_REFERENCE && o->visit) ? o->visit : o->order;
  for (int s = 0; s < o->c.n_shards; ++s) {
    int64_t off;
    int64_t ps = shard_range(o, s, &off);
    if (o->c.shard_only >= 0 && s != o->c.shard_only) { pos += ps; continue; }
    memcpy(o->eps, o->eps_start, sizeof(double) * (size_t)N);
    int64_t j0, j1;
    seg_positions(o, ps, e, &j0, &j1);
    for (int64_t j = j0; j < j1; ++j) {
      int64_t m = ord[pos + j];
      if (hs) horseshoe_marker(o, m, o->eps); else bayesr_marker(o, m, o->eps);
    }
    for (int64_t i = 0; i < N; ++i) o->eps_acc[i] += o->eps[i] - o->eps_start[i];
    pos += ps;
  }
  if (o->c.shard_only >= 0) {  /* the caller sums eps_acc over processes */
    memcpy(o->deps, o->eps_acc, sizeof(double) * (size_t)N);
    return;
  }
  for (int64_t i = 0; i < N; ++i) o->eps[i] = o->eps_start[i] + o->eps_acc[i];
}

static void marker_pass(orc *o) {
  const int hs = o->c.model == ORC_HORSESHOE;
  if (o->c.n_shards <= 1) {
    for (int64_t j = 0; j < o->P; ++j) {
      int64_t m = o->order[j];
      if (hs) horseshoe_marker(o, m, o->eps); else bayesr_marker(o, m, o->eps);
    }
    return;
  }
  if (o->c.shard_only >= 0) {
    marker_segment(o, o->seg);
    return;
  }
  for (int e = 0; e < o->c.n_exchanges; ++e) marker_segment(o, e);
}

/* shard_only: this sweep's last exchange segment (the statistics and the epilogue follow it) */
static int last_seg(const orc *o) { return o->c.shard_only < 0 || o->seg == o->c.n_exchanges - 1; }

/* statistics the epilogue needs, over this process's markers (all markers unless shard_only) */
static void compute_stats(orc *o) {
  const int G = o->G, K = o->K;
  double *st = o->stats;
  memset(st, 0, sizeof(double) * (size_t)(2 + G + G * K));
  /* per-shard partial sums added in shard order: what an all-reduce over the shards' local
   * statistics computes (exact match for two shards); one shard = one sequential sum */
  for (int sh = 0; sh < o->c.n_shards; ++sh) {
    if (o->c.shard_only >= 0 && sh != o->c.shard_only) continue;
    int64_t m0;
    const int64_t m1 = shard_range(o, sh, &m0) + m0;
    double b2 = 0.0, b2l = 0.0;
    for (int64_t m = m0; m < m1; ++m) b2 += o->beta[m] * o->beta[m];
    if (o->c.model == ORC_HORSESHOE)
      for (int64_t m = m0; m < m1; ++m) b2l += pow(o->beta[m], 2) / o->lambda[m];
    st[0] += b2;
    st[1] += b2l;
  }
  for (int g = 0; g < G; ++g) st[2 + g] = o->betaAcum[g];
  for (int q = 0; q < G * K; ++q) st[2 + G + q] = o->v[q];
}
static void bayesr_epilogue(orc *o);

static void sweep_bayesr(orc *o) {
  const int K = o->K, G = o->G;
  const orc_config *c = &o->c;
  if (o->seg == 0) {
    mu_update(o);
    make_orders(o);
    if (c->model == ORC_GROUPS) fixed_effects(o);
    memset(o->v, 0, sizeof(double) * (size_t)(G * K));
    memset(o->betaAcum, 0, sizeof(double) * (size_t)G);
  }
  marker_pass(o);
  if (!last_seg(o)) {  /* an earlier exchange segment: nothing but the residual delta */
    memset(o->stats, 0, sizeof(double) * (size_t)orc_stats_size(o));
    return;
  }
  compute_stats(o);
  if (c->model != ORC_HORSESHOE && o->c.shard_only >= 0) return; /* epilogue after exchange */
  bayesr_epilogue(o);
}

static void bayesr_epilogue(orc *o) {
  const int64_t N = o->N, P = o->P;
  const int K = o->K, G = o->G;
  const uint32_t it = (uint32_t)o->it;
  const orc_config *c = &o->c;
  (void)N;
  const double *v = o->stats + 2 + G;
  const double *bacc = o->stats + 2;
  if (c->model == ORC_V2) {
    /* BayesRv2.cpp:247-255 */
    const int m0 = (int)(P - (int64_t)v[0]);
    const double bsq = o->stats[0];
    o->sigmaGG[0] = inv_scaled_chisq_rng(o->seed, c->v0G + m0,
                                         (bsq * m0 + c->v0G * c->s02G) / (c->v0G + m0),
                                         ORC_T_SIGMAG, 0, it);
    o->sigmaE = inv_scaled_chisq_rng(o->seed, c->v0E + N,
                                     (sqnorm(o->eps, N) + c->v0E * c->s02E) / (c->v0E + N),
                                     ORC_T_SIGMAE, 0, it);
    double a[ORC_MAXK];
    for (int k = 0; k < K; ++k) a[k] = v[k] + 1.0;
    dirichlet_rng(o->seed, a, K, o->pi, ORC_T_PI, 0, it);
  } else {
    if (c->model == ORC_GROUPS) {
      /* BayesRv2Groups.cpp:301 */
      o->sigmaF = inv_scaled_chisq_rng(o->seed, c->v0E + o->F,
                                       (sqnorm(o->alpha, o->F) + c->v0E * c->s02E) / (c->v0E + o->F),
                                       ORC_T_SIGMAF, 0, it);
    }
    /* Groups :304 / restart :254 */
    o->sigmaE = inv_scaled_chisq_rng(o->seed, c->v0E + N,
                                     (sqnorm(o->eps, N) + c->v0E * c->s02E) / (c->v0E + N),
                                     ORC_T_SIGMAE, 0, it);
    for (int g = 0; g < G; ++g) { /* Groups :307-312 / restart :257-262 */
      double rs = 0.0;
      for (int k = 0; k < K; ++k) rs += v[g * K + k];
      const int m0 = (int)(rs - v[g * K + 0]);
      o->sigmaGG[g] = inv_scaled_chisq_rng(
          o->seed, c->v0G + m0, (bacc[g] * m0 + c->v0G * c->s02G) / (c->v0G + m0),
          ORC_T_SIGMAG, (uint32_t)g, it);
      double a[ORC_MAXK];
      for (int k = 0; k < K; ++k) a[k] = v[g * K + k] + 1.0;
      dirichlet_rng(o->seed, a, K, o->pi + g * K, ORC_T_PI, (uint32_t)(g * K), it);
    }
  }
}

static void hs_epilogue(orc *o);

static void sweep_horseshoe(orc *o) {
  /* HorseshoeR.cpp:210-253 */
  const int64_t P = o->P;
  const uint32_t it = (uint32_t)o->it;
  const orc_config *c = &o->c;
  if (o->seg == 0) {
    mu_update(o);
    make_orders(o);
    o->eta = inv_gamma_rate_rng(o->seed, 0.5 + 0.5 * c->vT,
                                (1.0 / (o->sigmaE * c->A * c->A)) + c->vT / o->tau,
                                ORC_T_HS_ETA, 0, it);                               /* :217 */
    for (int64_t j = 0; j < P; ++j)                                                 /* :218 */
      o->hsv[j] = inv_gamma_rate_rng(o->seed, 0.5 + 0.5 * c->vL, c->vL / o->lambda[j] + 1.0,
                                     ORC_T_HS_V, (uint32_t)j, it);
  }
  marker_pass(o);                                                                   /* :219-240 */
  if (!last_seg(o)) {
    memset(o->stats, 0, sizeof(double) * (size_t)orc_stats_size(o));
    return;
  }
  int64_t j0 = 0, j1 = P;
  if (o->c.shard_only >= 0) j1 = j0 + shard_range(o, o->c.shard_only, &j0);
  for (int64_t j = j0; j < j1; ++j)                                                 /* :242 */
    o->lambda[j] = inv_gamma_rate_rng(
        o->seed, 0.5 + 0.5 * c->vL,
        c->vL * (1.0 / o->hsv[j]) + (0.5 * (o->beta[j] * o->beta[j])) * (1.0 / o->tau),
        ORC_T_HS_LAMBDA, (uint32_t)j, it);
  compute_stats(o);
  if (o->c.shard_only >= 0) return; /* epilogue after exchange */
  hs_epilogue(o);
}

static void hs_epilogue(orc *o) {
  const int64_t N = o->N, P = o->P;
  const uint32_t it = (uint32_t)o->it;
  const orc_config *c = &o->c;
  const double sb = o->stats[1];
  o->tau = inv_gamma_rate_rng(o->seed, 0.5 * (P + c->vT), c->vT / o->eta + (0.5) * sb,
                              ORC_T_HS_TAU, 0, it);                                 /* :245 */
  o->c2 = inv_gamma_rate_rng(o->seed, 0.5 * c->vC + 0.5 * P,
                             c->vC * c->sC * 0.5 + 0.5 * o->stats[0], ORC_T_HS_C2, 0,
                             it);                                                   /* :248 */
  o->sigmaE = inv_scaled_chisq_rng(o->seed, c->v0E + N,
                                   (sqnorm(o->eps, N) + c->v0E * c->s02E) / (c->v0E + N),
                                   ORC_T_SIGMAE, 0, it);                            /* :253 */
}

int orc_sweep_local(orc *o) {
  if (o->c.shard_only < 0) return -1;
  g_rs = o->rs;
  if (o->c.model == ORC_HORSESHOE) sweep_horseshoe(o); else sweep_bayesr(o);
  g_rs = NULL;
  return 0;
}

int64_t orc_stats_size(const orc *o) { return 2 + o->G + (int64_t)o->G * o->K; }

int orc_exchange_get(const orc *o, double *deps, double *stats) {
  if (deps) memcpy(deps, o->deps, sizeof(double) * (size_t)o->N);
  if (stats) memcpy(stats, o->stats, sizeof(double) * (size_t)orc_stats_size(o));
  return 0;
}

int orc_exchange_set(orc *o, const double *deps_sum, const double *stats_sum) {
  for (int64_t i = 0; i < o->N; ++i) o->eps[i] = o->eps_start[i] + deps_sum[i];
  memcpy(o->stats, stats_sum, sizeof(double) * (size_t)orc_stats_size(o));
  return 0;
}

int orc_sweep_finish(orc *o) {
  if (o->c.shard_only >= 0 && o->seg < o->c.n_exchanges - 1) {  /* the next exchange segment */
    o->seg++;
    return 0;
  }
  o->seg = 0;
  g_rs = o->rs;
  if (o->c.model == ORC_HORSESHOE) hs_epilogue(o); else bayesr_epilogue(o);
  g_rs = NULL;
  o->it++;
  return 0;
}

int orc_sweep(orc *o, int n) {
  g_rs = o->rs;
  for (int r = 0; r < n; ++r) {
    if (o->c.model == ORC_HORSESHOE) sweep_horseshoe(o); else sweep_bayesr(o);
    o->it++;
  }
  g_rs = NULL;
  return 0;
}

double orc_get_scalar(const orc *o, int which) {
  switch (which) {
    case ORC_S_MU: return o->mu;
    case ORC_S_SIGMAE: return o->sigmaE;
    case ORC_S_SIGMAG: return o->sigmaGG[0];
    case ORC_S_SIGMAF: return o->sigmaF;
    case ORC_S_TAU: return o->tau;
    case ORC_S_ETA: return o->eta;
    case ORC_S_C2: return o->c2;
    case ORC_S_SUMSQ_BETA: return sqnorm(o->beta, o->P);
    default: return NAN;
  }
}

int orc_set_scalar(orc *o, int which, double v) {
  switch (which) {
    case ORC_S_MU: o->mu = v; return 0;
    case ORC_S_SIGMAE: o->sigmaE = v; return 0;
    case ORC_S_SIGMAG: o->sigmaGG[0] = v; return 0;
    case ORC_S_SIGMAF: o->sigmaF = v; return 0;
    case ORC_S_TAU: o->tau = v; return 0;
    case ORC_S_ETA: o->eta = v; return 0;
    case ORC_S_C2: o->c2 = v; return 0;
    default: return -1;
  }
}

static double *vec_ptr(const orc *o, int which, int64_t *len) {
  switch (which) {
    case ORC_V_BETA: *len = o->P; return o->beta;
    case ORC_V_COMP: *len = o->P; return o->comp;
    case ORC_V_EPS: *len = o->N; return o->eps;
    case ORC_V_SIGMAGG: *len = o->G; return o->sigmaGG;
    case ORC_V_PI: *len = (int64_t)o->G * o->K; return o->pi;
    case ORC_V_ALPHA: *len = o->F; return o->alpha;
    case ORC_V_LAMBDA: *len = o->P; return o->lambda;
    case ORC_V_XSQ: *len = o->P; return o->xsq;
    case ORC_V_VCOUNT: *len = (int64_t)o->G * o->K; return o->v;
    case ORC_V_BETAACUM: *len = o->G; return o->betaAcum;
    case ORC_V_HSV: *len = o->P; return o->hsv;
    default: *len = -1; return NULL;
  }
}

int64_t orc_get_vector(const orc *o, int which, double *out) {
  int64_t len = 0;
  if (which == ORC_V_ORDER) {
    if (out) for (int64_t i = 0; i < o->P; ++i) out[i] = (double)o->order[i];
    return o->P;
  }
  double *p = vec_ptr(o, which, &len);
  if (!p) return -1;
  if (out) memcpy(out, p, sizeof(double) * (size_t)len);
  return len;
}

int orc_set_vector(orc *o, int which, const double *in) {
  int64_t len = 0;
  double *p = vec_ptr(o, which, &len);
  if (!p || len < 0) return -1;
  memcpy(p, in, sizeof(double) * (size_t)len);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* synthetic cohort: DESIGN.md "synthetic data spec" (shared with the device generator) */
static double data_uniform(uint64_t ds, uint32_t slot, uint32_t tag, uint32_t ent, uint32_t it) {
  uint32_t w[4];
  philox_draw(ds, slot, tag, ent, it, w);
  return orc_u53(w[0], w[1]);
}

static int genotype(uint64_t ds, int64_t i, int64_t j, uint32_t attempt, double t0, double t1) {
  uint32_t w[4];
  philox_draw(ds, (uint32_t)(i >> 3), ORC_T_DATA_GENO, (uint32_t)j, attempt, w);
  uint32_t word = w[(i >> 1) & 3];
  uint32_t half = (i & 1) ? (word >> 16) : (word & 0xFFFFu);
  double u = ((double)half + 0.5) * (1.0 / 65536.0);
  return u < t0 ? 0 : (u < t1 ? 1 : 2);
}

int orc_synth_x(uint64_t ds, int64_t N, int64_t P, int64_t col0, double *X) {
  for (int64_t jl = 0; jl < P; ++jl) {
    const int64_t j = col0 + jl;
    const double f = 0.05 + 0.45 * data_uniform(ds, 0, ORC_T_DATA_FREQ, (uint32_t)j, 0);
    const double t0 = (1.0 - f) * (1.0 - f);
    const double t1 = 1.0 - f * f;
    double *x = X + jl * N;
    uint32_t attempt = 0;
    int64_t S = 0, Q = 0;
    for (; attempt < 16; ++attempt) {
      S = 0; Q = 0;
      for (int64_t i = 0; i < N; ++i) {
        int g = genotype(ds, i, j, attempt, t0, t1);
        S += g; Q += g * g;
      }
      if (N > 1 && (double)Q * (double)N != (double)S * (double)S) break;
    }
    if (attempt == 16 || N < 2) {
      for (int64_t i = 0; i < N; ++i) x[i] = 0.0;
      continue;
    }
    const double mean = (double)S / (double)N;
    const double var = ((double)Q - (double)S * (double)S / (double)N) / (double)(N - 1);
    const double sd = sqrt(var);
    for (int64_t i = 0; i < N; ++i) {
      int g = genotype(ds, i, j, attempt, t0, t1);
      x[i] = (double)(float)(((double)g - mean) / sd);
    }
  }
  return 0;
}

int orc_synth_beta(uint64_t ds, int64_t P_total, int64_t n_causal, int64_t col0, int64_t P,
                   double *beta) {
  const double pc = (double)n_causal / (double)P_total;
  for (int64_t jl = 0; jl < P; ++jl) {
    const int64_t j = col0 + jl;
    const double u = data_uniform(ds, 1, ORC_T_DATA_FREQ, (uint32_t)j, 0);
    if (u < pc) {
      uint32_t w[4];
      philox_draw(ds, 2, ORC_T_DATA_FREQ, (uint32_t)j, 0, w);
      beta[jl] = box_muller(w);
    } else {
      beta[jl] = 0.0;
    }
  }
  return 0;
}

/* ------------------------------------------------------------------------- */
/* reference-faithful one-shot runs writing the reference CSV format */
static void csv_row(FILE *f, const double *v, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    if (i) fputs(", ", f);
    fprintf(f, "%g", v[i]);
  }
  fputc('\n', f);
}

int orc_run_csv(const orc_config *cfg, const char *path, int max_iterations, int burn_in,
                int thinning) {
  const int bad_iter = (max_iterations < burn_in || max_iterations < 1 || burn_in < 1 ||
                        thinning < 1);
  FILE *f = NULL;
  const int64_t N = cfg->N, M = cfg->P;
  const int G = cfg->G < 1 ? 1 : cfg->G;
  const int F = cfg->model == ORC_GROUPS ? cfg->F : 0;
  if (cfg->model == ORC_HORSESHOE && bad_iter) return 1; /* HorseshoeR.cpp:119-123 */
  f = fopen(path, "w");
  if (!f) return -3;
  if (cfg->model == ORC_V2) { /* header before validation: BayesRv2.cpp:69-70 */
    fputs("iteration,mu,", f);
    for (int64_t i = 0; i < M; ++i) fprintf(f, "beta[%lld],", (long long)(i + 1));
    fputs("sigmaE,sigmaG,", f);
    for (int64_t i = 0; i < M; ++i) fprintf(f, "comp[%lld],", (long long)(i + 1));
    for (int64_t i = 0; i < N - 1; ++i) fprintf(f, "epsilon[%lld],", (long long)(i + 1));
    fprintf(f, "epsilon[%lld]\n", (long long)N);
  }
  if (bad_iter) { fclose(f); return 1; }
  if (cfg->model == ORC_GROUPS) { /* BayesRv2Groups.cpp:25-54, after validation (:113) */
    fputs("iteration,mu,", f);
    for (int64_t i = 0; i < M; ++i) fprintf(f, "beta[%lld],", (long long)(i + 1));
    fputs("sigmaE,", f);
    for (int64_t i = 0; i < M; ++i) fprintf(f, "comp[%lld],", (long long)(i + 1));
    for (int g = 0; g < G; ++g) fprintf(f, "sigmaG[%d],", g + 1);
    for (int64_t i = 0; i < N - 1; ++i) fprintf(f, "epsilon[%lld],", (long long)(i + 1));
    fprintf(f, "epsilon[%lld],", (long long)N);
    for (int i = 0; i < F; ++i) fprintf(f, "alpha[%d],", i + 1);
    fputs("sigmaF\n", f);
  } else if (cfg->model == ORC_HORSESHOE) { /* HorseshoeR.cpp:279-291 */
    fputs("iteration,mu,", f);
    for (int64_t i = 0; i < M; ++i) fprintf(f, "beta[%lld],", (long long)(i + 1));
    fputs("sigmaE,tau,", f);
    for (int64_t i = 0; i < M; ++i) fprintf(f, "lambda[%lld],", (long long)(i + 1));
    for (int64_t i = 0; i < N; ++i) fprintf(f, "epsilon[%lld],", (long long)(i + 1));
    fputc('\n', f);
  } /* BRV2Grstart never writes a header (initialize_file unused, BRv2Grstart.cpp:26) */
  orc *o = orc_create(cfg);
  if (!o) { fclose(f); return -1; }
  orc_init(o);
  double *row = (double *)malloc(sizeof(double) * (size_t)(2 * M + N + G + F + 8));
  for (int it = 0; it < max_iterations; ++it) {
    orc_sweep(o, 1);
    if (it >= burn_in && it % thinning == 0) {
      int64_t n = 0;
      row[n++] = it;
      row[n++] = o->mu;
      memcpy(row + n, o->beta, sizeof(double) * (size_t)M); n += M;
      row[n++] = o->sigmaE;
      if (cfg->model == ORC_V2) {
        row[n++] = o->sigmaGG[0];
        memcpy(row + n, o->comp, sizeof(double) * (size_t)M); n += M;
        memcpy(row + n, o->eps, sizeof(double) * (size_t)N); n += N;
      } else if (cfg->model == ORC_HORSESHOE) {
        row[n++] = o->tau;
        memcpy(row + n, o->lambda, sizeof(double) * (size_t)M); n += M;
        memcpy(row + n, o->eps, sizeof(double) * (size_t)N); n += N;
        row[n++] = 0.0; /* sample has 2M+4+N slots but 2M+N+3 values (HorseshoeR.cpp:157,258) */
      } else {
        memcpy(row + n, o->comp, sizeof(double) * (size_t)M); n += M;
        memcpy(row + n, o->sigmaGG, sizeof(double) * (size_t)G); n += G;
        memcpy(row + n, o->eps, sizeof(double) * (size_t)N); n += N;
        if (cfg->model == ORC_GROUPS) {
          memcpy(row + n, o->alpha, sizeof(double) * (size_t)F); n += F;
          row[n++] = o->sigmaF;
        }
      }
      csv_row(f, row, n);
    }
  }
  free(row);
  orc_destroy(o);
  fclose(f);
  return 0;
}
