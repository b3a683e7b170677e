// brr_chain.hpp -- serial chain of the Horseshoe block solve (one wave), shared by the fused
// sweep kernel (brr_kernels.hip, solve_block step 3) and its microbenchmark
// (scripts/mb_chain2.hip).
//
// Every Horseshoe position changes (beta ~ N(num/D, sigmaE/D), HorseshoeR.cpp:219-240), so the
// block's chain is a forward substitution in visit order.  With num_j = r0_j - sum_{i<j} G_ij
// delta_i, the scaled quantity
//     s_j = num_j / D_j + (z_j - beta_old_j) - sum_{i<j visited} (G_ij / D_j) delta_i
// IS delta_j when position j is reached.  Lane l holds positions l + 64 q (q < B / 64) in
// registers.  The positions are processed in sub-blocks of SB = 16: the coefficients G_ij of a
// sub-block's 16 positions i at every lane's positions are gathered from the LDS Gram block in
// ONE batch (2 x 16 LDS reads per lane at B = 128) one sub-block ahead (double buffer), so the
// dependency chain of a step is only readlane(owner's s_i) -> FMA into the later positions; no
// LDS latency and no branch sits on it (the sub-block loop is unrolled at compile time; steps
// past the block's end are no-ops: their s is 0).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

namespace brr {

template <class F, int... K>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, K...>) {
  (f(std::integral_constant<int, K>{}), ...);
}
// f(integral_constant<int, 0>), ..., f(integral_constant<int, N-1>) in order, unrolled
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ double chain_readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// Correctly rounded num / D: q0 = num * RN(1/D), one exact-remainder correction (Markstein).
__device__ __forceinline__ double chain_quot_rn(double num, double den, double inv) {
  const double q0 = num * inv;
  return __builtin_fma(__builtin_fma(-q0, den, num), inv, q0);
}

// The chain's coefficient matrix, made in place from the block's Gram in LDS before the chain:
// element (row g, column c) becomes G_gc / D_pos(c) (RN(1/D) times G) when position pos(g) comes
// before position pos(c) in visit order, else 0.  Linv_gi[c] = RN(1/D) of the position whose Gram
// index is c, Lpos_gi[c] = that position (B = unused index: its column is zeroed).  All NT threads
// of the workgroup take part; the caller synchronises before the chain.
template <int B, int NT>
__device__ __forceinline__ void chain_coefficients(double *slots, const double *Linv_gi, const int *Lpos_gi) {
  if constexpr (NT % B == 0) {  // a thread keeps one column
    const int c = threadIdx.x % B;
    const double ic = Linv_gi[c];
    const int pc = Lpos_gi[c];
#pragma unroll 8
    for (int r = threadIdx.x / B; r < B; r += NT / B) {
      double *e = slots + r * B + c;
      *e = Lpos_gi[r] < pc ? *e * ic : 0.0;
    }
  } else {
    for (int e = threadIdx.x; e < B * B; e += NT) {
      const int r = e / B, c = e % B;
      slots[e] = Lpos_gi[r] < Lpos_gi[c] ? slots[e] * Linv_gi[c] : 0.0;
    }
  }
}

// bs positions (bs <= B); Lr0 = num at the block start, Ldsel = D, Lsdz = sqrt(sigmaE / D) z,
// Lbo = beta_old, Lgi = Gram index of each position (a permutation of 0 .. bs - 1); coef =
// chain_coefficients (G_ij / D_j at coef[gi_i B + gi_j] for i before j, else 0).  Writes Lbn = beta_new.  One whole wave.  The
// zeros make every update unconditional (positions at or before step i subtract 0), so a step
// is readlane + FMAs and nothing else.
template <int B>
__device__ __forceinline__ void chain_hs_blocked(int bs, const double *Lr0, const double *Ldsel, const double *Lsdz,
                                                 const double *Lbo, double *Lbn, const int *Lgi,
                                                 const double *coef) {
#pragma clang fp contract(off)
  constexpr int NS = B / 64;
  constexpr int SB = 16;
  constexpr int NSB = B / SB;
  const int lane = threadIdx.x & 63;
  double sv[NS], bo[NS];
  int gg[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane + 64 * q;
    const bool in = pos < bs;
    const double dv = in ? Ldsel[pos] : 1.0;
    const double iv = 1.0 / dv;
    bo[q] = in ? Lbo[pos] : 0.0;
    const double r = in ? Lr0[pos] : 0.0;
    const double z = in ? Lsdz[pos] : 0.0;
    sv[q] = in ? chain_quot_rn(r, dv, iv) + (z - bo[q]) : 0.0;
    // past the block's end: Gram index B - 1, unused in a ragged block (its valid positions hold
    // the indices 0 .. bs - 1), so that row and column of coef are zero and those steps no-ops
    gg[q] = in ? Lgi[pos] : B - 1;
  }
  double hb[2][NS][SB];
  // coefficients of sub-block k's positions at this lane's positions (planes qk.. only)
  auto gather = [&](auto kc, double (&h)[NS][SB]) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    constexpr int qk = (SB * k) / 64;
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int gi = __builtin_amdgcn_readlane(gg[qk], (SB * k + u) & 63);
      const double *row = coef + gi * B;
#pragma unroll
      for (int q = qk; q < NS; ++q) h[q][u] = row[gg[q]];
    }
  };
  gather(std::integral_constant<int, 0>{}, hb[0]);
  auto sub = [&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    constexpr int qk = (SB * k) / 64;
    if constexpr (k + 1 < NSB) gather(std::integral_constant<int, k + 1>{}, hb[(k + 1) & 1]);
    double(&h)[NS][SB] = hb[k & 1];
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const double delta = chain_readlane_f64(sv[qk], (SB * k + u) & 63);
#pragma unroll
      for (int q = qk; q < NS; ++q) sv[q] = __builtin_fma(-h[q][u], delta, sv[q]);
    }
  };
  static_for<NSB>(sub);
#pragma unroll
  for (int q = 0; q < NS; ++q)
    if (lane + 64 * q < bs) Lbn[lane + 64 * q] = bo[q] + sv[q];  // HorseshoeR.cpp:234
}

}  // namespace brr
