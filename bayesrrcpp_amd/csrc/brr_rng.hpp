// brr_rng.hpp -- device random-number library: the MI355X replacement of the reference's
// distributions.h / distributions.cpp (src/distributions.h:8-18, src/distributions.cpp:12-62).
//
// The reference draws from R's single global stream (R::rnorm/rgamma/rbeta/runif), which
// cannot be reproduced on a GPU at speed and does not exist here.  Every draw is instead a
// pure function of (seed, slot, tag, entity, iteration): one Philox4x32-10 block, computed by
// rocRAND's engine (rocrand_philox4x32_10.h), so conditional draws never shift later ones
// and any thread can produce any marker's draw.  Spec (shared with the CPU oracle, which
// re-implements it independently): DESIGN.md "RNG spec".
#pragma once
#include <hip/hip_runtime.h>
#include <rocrand/rocrand_philox4x32_10.h>
#include <stdint.h>

namespace brr {

enum RngTag : uint32_t {
  T_MARKER = 1, T_MU = 2, T_SIGMAE = 3, T_SIGMAG = 4, T_PI = 5, T_SIGMAF = 6, T_FIXED = 7,
  T_HS_V = 8, T_HS_LAMBDA = 9, T_HS_ETA = 10, T_HS_TAU = 11, T_HS_C2 = 12, T_INIT = 13,
  T_PERM_BLOCK = 14, T_PERM_WITHIN = 15, T_PERM_FIXED = 16,
  T_DATA_FREQ = 32, T_DATA_GENO = 33, T_DATA_NOISE = 34
};
constexpr uint32_t INIT_IT = 0xFFFFFFFFu;
constexpr int GAMMA_MAX_ATTEMPTS = 64;

// rocRAND's Philox4x32-10 engine exposes its block function only to derived classes.
struct PhiloxBlock : public rocrand_device::philox4x32_10_engine {
  __host__ __device__ __forceinline__ uint4 block(uint4 ctr, uint2 key) {
    return this->ten_rounds(ctr, key);
  }
};

__host__ __device__ __forceinline__ uint4 philox(uint64_t seed, uint32_t slot, uint32_t tag,
                                                 uint32_t entity, uint32_t it) {
  PhiloxBlock e;
  uint4 c;
  c.x = slot; c.y = tag; c.z = entity; c.w = it;
  uint2 k;
  k.x = (uint32_t)seed; k.y = (uint32_t)(seed >> 32);
  return e.block(c, k);
}

// 53-bit uniform strictly inside (0,1); exact (no rounding) on host and device.
__host__ __device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
  uint64_t x = ((((uint64_t)hi) << 32) | (uint64_t)lo) >> 11;
  return ((double)x + 0.5) * 0x1p-53;
}

__host__ __device__ __forceinline__ double uniform(uint64_t seed, uint32_t tag, uint32_t ent,
                                                   uint32_t it, uint32_t slot) {
  uint4 w = philox(seed, slot, tag, ent, it);
  return u53(w.x, w.y);
}

// Box-Muller (cosine branch) from one Philox block.
__host__ __device__ __forceinline__ double box_muller(uint4 w) {
  double u1 = u53(w.x, w.y);
  double u2 = u53(w.z, w.w);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586476925286766559 * u2);
}

__host__ __device__ __forceinline__ double normal(uint64_t seed, uint32_t tag, uint32_t ent,
                                                  uint32_t it, uint32_t slot) {
  return box_muller(philox(seed, slot, tag, ent, it));
}

// Gamma(shape, 1): Marsaglia-Tsang with U^(1/a) boost for a < 1.  Attempt t: slot 2t normal,
// slot 2t+1 acceptance uniform; boost uniform slot 0xFFFFFFFF.  Replaces R::rgamma.
__host__ __device__ inline double gamma(uint64_t seed, double shape, uint32_t tag, uint32_t ent,
                                        uint32_t it) {
  if (!(shape > 0.0)) return 0.0;
  double boost = 1.0, a = shape;
  if (a < 1.0) {
    boost = pow(uniform(seed, tag, ent, it, 0xFFFFFFFFu), 1.0 / a);
    a += 1.0;
  }
  const double d = a - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  for (uint32_t t = 0; t < (uint32_t)GAMMA_MAX_ATTEMPTS; ++t) {
    const double z = box_muller(philox(seed, 2u * t, tag, ent, it));
    double v = 1.0 + c * z;
    if (v <= 0.0) continue;
    v = v * v * v;
    uint4 w = philox(seed, 2u * t + 1u, tag, ent, it);
    const double u = u53(w.x, w.y);
    if (log(u) < 0.5 * z * z + d - d * v + d * log(v)) return d * v * boost;
  }
  return d * boost;
}

// --- distributions.cpp equivalents (same argument meaning as the reference) ---
// inv_gamma_rng(shape, scale) = 1/R::rgamma(shape, 1/scale)         (:21-23)
__host__ __device__ inline double inv_gamma_rng(uint64_t s, double shape, double scale,
                                                uint32_t tag, uint32_t ent, uint32_t it) {
  return 1.0 / ((1.0 / scale) * gamma(s, shape, tag, ent, it));
}
// inv_gamma_rate_rng(shape, rate) = 1/R::rgamma(shape, 1/rate)      (:27-32)
__host__ __device__ inline double inv_gamma_rate_rng(uint64_t s, double shape, double rate,
                                                     uint32_t tag, uint32_t ent, uint32_t it) {
  return 1.0 / ((1.0 / rate) * gamma(s, shape, tag, ent, it));
}
// inv_scaled_chisq_rng(dof, scale)                                   (:34-36)
__host__ __device__ inline double inv_scaled_chisq_rng(uint64_t s, double dof, double scale,
                                                       uint32_t tag, uint32_t ent, uint32_t it) {
  return inv_gamma_rng(s, 0.5 * dof, 0.5 * dof * scale, tag, ent, it);
}

// Fisher-Yates step source for the visit-order spec: word (i & 3) of block (i >> 2).
__host__ __device__ __forceinline__ uint32_t fy_index(uint64_t seed, int64_t i, uint32_t tag,
                                                      uint32_t ent, uint32_t it) {
  uint4 w = philox(seed, (uint32_t)(i >> 2), tag, ent, it);
  uint32_t word = (i & 3) == 0 ? w.x : (i & 3) == 1 ? w.y : (i & 3) == 2 ? w.z : w.w;
  return (uint32_t)(((uint64_t)word * (uint64_t)(i + 1)) >> 32);
}

}  // namespace brr
