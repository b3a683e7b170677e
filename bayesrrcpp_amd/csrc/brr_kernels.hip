// brr_kernels.hip -- HIP kernels (gfx950 / CDNA4) of the MI355X BayesR / BayesRR / Horseshoe
// Gibbs sweep.  Host-side orchestration lives in brr_session.cpp.
//
// The reference's hot loop (src/BayesRv2.cpp:186-245, Groups :232-298, restart :183-250,
// Horseshoe :219-240) visits markers one at a time: y~ = eps + x_m b_m, num = x_m . y~,
// mixture draw, eps = y~ - x_m b_m.  Here the markers of a sweep are processed in blocks of
// B (visit order = block order x order inside the block):
//
//   k_stream(s)  all CUs: apply the previous block's residual updates (one re-read of its
//                changed columns) and stream block s's B columns once from HBM to form the
//                partial dots x_j . eps over row slices; 2-level deterministic reduction.
//   k_solve(s)   one CU: exact single-site updates of the B markers in visit order.  The dot
//                of marker j with the CURRENT residual is d_j + xsq_j b_j - sum_{i<j} G_ji db_i
//                (G = X_b^T X_b, precomputed), so no further pass over X is needed.  Each
//                marker's component decision is pre-evaluated in parallel together with a
//                t = num^2 interval in which it cannot change; the serial chain then costs a
//                few f64 ops per marker and skips runs of unchanged markers with a ballot.
//
// Everything is double precision except X, which is stored as f32 (products are exact in
// f64).  No FMA contraction where the reference's elementwise arithmetic is restated.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "brr_device.hpp"
#include "brr_rng.hpp"

namespace brr {



// ------------------------------------------------------------------------------------
// small helpers
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// deterministic block sum (fixed tree), result valid in every thread
template <int NT>
__device__ __forceinline__ double block_sum(double v, double *lds /* NT/64 */) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += lds[i];
  return s;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// Last-arriver ticket (cdna_hip_programming.md section 5, in-launch split-K reduction):
// payload stores -> vmcnt(0) -> barrier -> release(agent) -> vmcnt(0) -> relaxed agent add;
// the last arriver acquires (agent) before reading the other workgroups' payload.
__device__ __forceinline__ bool last_arriver(int *cnt, int total, int *lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (old == total - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// Write-through variant (MI355X_MICROARCH.md "Valid forms", row 1): every payload byte stored
// sc1 (8-B agent-scope relaxed atomic stores) and drained by every storing wave, one relaxed
// agent add per workgroup; the last arriver reads the payload with sc1 loads only -- no
// release / acquire fences (no L2 write-back, no L1 invalidate).
__device__ __forceinline__ void st_sc1(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
  return __longlong_as_double(__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ bool last_arriver_wt(int *cnt, int total, int *lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_flag = (old == total - 1);
  }
  __syncthreads();
  return *lds_flag != 0;
}

// ------------------------------------------------------------------------------------
// Synthetic cohort (DESIGN.md "synthetic data spec"; mirrored by oracle orc_synth_x).
__device__ __forceinline__ int genotype(uint64_t ds, int64_t i, int64_t j, uint32_t att, double t0,
                                        double t1) {
  uint4 w = philox(ds, (uint32_t)(i >> 3), T_DATA_GENO, (uint32_t)j, att);
  const int q = (int)((i >> 1) & 3);
  uint32_t word = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
  uint32_t half = (i & 1) ? (word >> 16) : (word & 0xFFFFu);
  double u = ((double)half + 0.5) * (1.0 / 65536.0);
  return u < t0 ? 0 : (u < t1 ? 1 : 2);
}

__global__ __launch_bounds__(256) void k_synth_x(float *X, int64_t ld, int64_t N, int64_t col0,
                                                 uint64_t ds) {
#pragma clang fp contract(off)
  __shared__ double red[8];
  __shared__ int s_att;
  const int64_t jl = blockIdx.x;
  const int64_t j = col0 + jl;
  const double f = 0.05 + 0.45 * uniform(ds, T_DATA_FREQ, (uint32_t)j, 0, 0);
  const double t0 = (1.0 - f) * (1.0 - f);
  const double t1 = 1.0 - f * f;
  float *x = X + jl * ld;
  uint32_t att = 0;
  double S = 0.0, Q = 0.0;
  for (; att < 16; ++att) {
    double s = 0.0, q = 0.0;
    for (int64_t i = threadIdx.x; i < N; i += 256) {
      int g = genotype(ds, i, j, att, t0, t1);
      s += g;
      q += g * g;
    }
    S = block_sum<256>(s, red);
    Q = block_sum<256>(q, red);
    if (N > 1 && Q * (double)N != S * S) break;
  }
  if (threadIdx.x == 0) s_att = (int)att;
  __syncthreads();
  if (s_att == 16 || N < 2) {
    for (int64_t i = threadIdx.x; i < ld; i += 256) x[i] = 0.f;
    return;
  }
  const double mean = S / (double)N;
  const double var = (Q - S * S / (double)N) / (double)(N - 1);
  const double sd = sqrt(var);
  for (int64_t i = threadIdx.x; i < ld; i += 256) {
    float v = 0.f;
    if (i < N) v = (float)(((double)genotype(ds, i, j, att, t0, t1) - mean) / sd);
    x[i] = v;
  }
}

// y_i = sum_{causal j} x_ij beta_j  (causal list from the host)
__global__ __launch_bounds__(256) void k_synth_y(const float *X, int64_t ld, int64_t N,
                                                 const int *cidx, const double *cbeta, int nc,
                                                 double *y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  double acc = 0.0;
  for (int c = 0; c < nc; ++c) acc += (double)X[(int64_t)cidx[c] * ld + i] * cbeta[c];
  y[i] = acc;
}

__global__ void k_cast_f64_f32(const double *src, int64_t lds, float *dst, int64_t ldd,
                               int64_t N, int64_t M) {
  const int64_t j = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ldd; i += (int64_t)gridDim.x * 256)
    dst[j * ldd + i] = i < N ? (float)src[j * lds + i] : 0.f;
}

__global__ void k_copy_f32(const float *src, int64_t lds, float *dst, int64_t ldd, int64_t N,
                           int64_t M) {
  const int64_t j = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ldd; i += (int64_t)gridDim.x * 256)
    dst[j * ldd + i] = i < N ? src[j * lds + i] : 0.f;
}

// ------------------------------------------------------------------------------------
// Block Gram matrices: G[gb][i][j] = sum_r x(col(gb,i))[r] * x(col(gb,j))[r] in f64.
// 64x64 output tile per workgroup, 4x4 per thread, 64-row chunks staged in LDS.
// Element (i,j) and (j,i) accumulate identical products in identical order -> symmetric.
__global__ __launch_bounds__(256) void k_gram(const float *X, int64_t ld, const int *member,
                                              const int *bsz, int B, double *G) {
  __shared__ float As[64][65];
  __shared__ float Bs[64][65];
  const int gb = blockIdx.x;
  const int ntile = (B + 63) / 64;
  const int ti = blockIdx.y / ntile, tj = blockIdx.y % ntile;
  const int bs = bsz[gb];
  const int t = threadIdx.x;
  const int ty = t >> 4, tx = t & 15;
  double acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
  // loader: column c = t >> 2 (0..63), rows (t & 3) * 16 .. +16
  const int lc = t >> 2, lr = (t & 3) * 16;
  const int ci = ti * 64 + lc, cj = tj * 64 + lc;
  const float *pa = (ci < bs) ? X + (int64_t)member[(int64_t)gb * B + ci] * ld : nullptr;
  const float *pb = (cj < bs) ? X + (int64_t)member[(int64_t)gb * B + cj] * ld : nullptr;
  for (int64_t r0 = 0; r0 < ld; r0 += 64) {
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      float4 va = pa ? *reinterpret_cast<const float4 *>(pa + r0 + lr + q) : make_float4(0, 0, 0, 0);
      float4 vb = pb ? *reinterpret_cast<const float4 *>(pb + r0 + lr + q) : make_float4(0, 0, 0, 0);
      As[lr + q + 0][lc] = va.x; As[lr + q + 1][lc] = va.y; As[lr + q + 2][lc] = va.z; As[lr + q + 3][lc] = va.w;
      Bs[lr + q + 0][lc] = vb.x; Bs[lr + q + 1][lc] = vb.y; Bs[lr + q + 2][lc] = vb.z; Bs[lr + q + 3][lc] = vb.w;
    }
    __syncthreads();
#pragma unroll 4
    for (int r = 0; r < 64; ++r) {
      double a[4], b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) { a[q] = (double)As[r][ty * 4 + q]; b[q] = (double)Bs[r][tx * 4 + q]; }
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[p][q] = fma(a[p], b[q], acc[p][q]);
    }
    __syncthreads();
  }
  double *g = G + (int64_t)gb * B * B;
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = ti * 64 + ty * 4 + p, jj = tj * 64 + tx * 4 + q;
      if (i < B && jj < B) g[(int64_t)i * B + jj] = (i < bs && jj < bs) ? acc[p][q] : 0.0;
    }
}

__global__ void k_xsq_from_gram(const double *G, const int *member, const int *bsz, int B, int nb,
                                double *xsq) {
  const int s = blockIdx.x;
  const int i = threadIdx.x;
  if (s < nb && i < bsz[s]) xsq[member[(int64_t)s * B + i]] = G[(int64_t)s * B * B + (int64_t)i * B + i];
}

// ------------------------------------------------------------------------------------
// Row pass over the residual.  flags select: apply the mu shift of the sweep start
// (BayesRv2.cpp:177-179), apply the pending per-marker updates (:191,:243), snapshot /
// residual delta for the column-sharded exchange, and the sum(eps+mu), ||eps||^2 reductions.
enum RowFlags : int {
  ROW_SHIFT = 1, ROW_PENDING = 2, ROW_WRITE = 4, ROW_SNAPSHOT = 8, ROW_DEPS = 16,
  ROW_EXCHANGE = 32, ROW_REDUCE = 64, ROW_INIT_Y = 128
};

__global__ __launch_bounds__(256) void k_rows(Dev d, int flags, const double *deps_in) {
#pragma clang fp contract(off)
  __shared__ double red[8];
  __shared__ int s_last;
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = row < d.N;
  double e = 0.0;
  if (valid) {
    if (flags & ROW_INIT_Y) e = d.Y[row] - d.sc->mu - 0.0;  // eps = Y - mu - X*beta, beta=0
    else if (flags & ROW_EXCHANGE) e = d.eps_start[row] + deps_in[row];
    else e = d.eps[row];
  }
  if (flags & ROW_SHIFT) e = (e + d.sc->mu_prev) - d.sc->mu;
  if (flags & ROW_PENDING) {
    const int np = d.sc->n_pend;  // multiple of 8, neutral padding
    const float *Xr = d.X + (valid ? row : 0);
    for (int p0 = 0; p0 < np; p0 += 8) {
      double x[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) x[q] = (double)Xr[(int64_t)d.pend_idx[p0 + q] * d.ld];
#pragma unroll
      for (int q = 0; q < 8; ++q) e = (e + x[q] * d.pend_bo[p0 + q]) - x[q] * d.pend_bn[p0 + q];
    }
  }
  if (valid) {
    if (flags & ROW_WRITE) d.eps[row] = e;
    if (flags & ROW_SNAPSHOT) d.eps_start[row] = e;
    if (flags & ROW_DEPS) d.deps[row] = e - d.eps_start[row];
  }
  if (flags & ROW_REDUCE) {
    const double mu = d.sc->mu;
    const double s1 = block_sum<256>(valid ? e + mu : 0.0, red);
    const double s2 = block_sum<256>(valid ? e * e : 0.0, red);
    if (threadIdx.x == 0) { d.rslab[2 * blockIdx.x] = s1; d.rslab[2 * blockIdx.x + 1] = s2; }
    if (last_arriver(d.rcnt, gridDim.x, &s_last)) {
      double a = 0.0, b = 0.0;
      for (int w = threadIdx.x; w < (int)gridDim.x; w += 256) { a += d.rslab[2 * w]; b += d.rslab[2 * w + 1]; }
      // fixed-order combine: per-thread strided partials, then the deterministic tree
      a = block_sum<256>(a, red);
      b = block_sum<256>(b, red);
      if (threadIdx.x == 0) { d.sc->S1 = a; d.sc->S2 = b; *d.rcnt = 0; }
    }
  }
}

// ------------------------------------------------------------------------------------
// Sweep start: mu draw (BayesRv2.cpp:177-179; Groups :212-214; restart :173-175; HS :210-212)
// and, for the Horseshoe, eta (HorseshoeR.cpp:217).  The eps shift is applied by k_rows.
__global__ void k_sweep_start(Dev d, uint32_t it) {
  if (threadIdx.x != 0) return;
  Scal *sc = d.sc;
  sc->mu_prev = sc->mu;
  const double z = normal(d.seed, T_MU, 0, it, 0);
  sc->mu = sc->S1 / (double)d.N + sqrt(sc->sigmaE / (double)d.N) * z;
  sc->n_pend = 0;
  if (d.model == MODEL_HORSESHOE) {
    const Hyper &h = d.hyp;
    sc->eta = inv_gamma_rate_rng(d.seed, 0.5 + 0.5 * h.vT,
                                 (1.0 / (sc->sigmaE * h.A * h.A)) + h.vT / sc->tau, T_HS_ETA, 0, it);
  }
}

// ------------------------------------------------------------------------------------
// Visit order (BLOCKED mode): Philox Fisher-Yates of the block order and inside each block.
__device__ void fisher_yates_dev(uint64_t seed, int *a, int n, uint32_t tag, uint32_t ent, uint32_t it) {
  uint4 w = make_uint4(0, 0, 0, 0);
  int64_t cached = -1;
  for (int64_t i = n - 1; i >= 1; --i) {
    if ((i >> 2) != cached) { cached = i >> 2; w = philox(seed, (uint32_t)cached, tag, ent, it); }
    const int q = (int)(i & 3);
    uint32_t word = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
    int64_t j = (int64_t)(((uint64_t)word * (uint64_t)(i + 1)) >> 32);
    int tmp = a[i]; a[i] = a[j]; a[j] = tmp;
  }
}

// Block order: Fisher-Yates in LDS (serial by definition), then one coalesced write.
constexpr int PERM_LDS_MAX = 32768;  // blocks per shard handled in LDS (128 KiB)
__global__ __launch_bounds__(256) void k_perm_blockorder(Dev d, uint32_t it, int shard) {
  extern __shared__ __attribute__((aligned(16))) int ord[];
  const int nb = d.nb;
  if (nb <= PERM_LDS_MAX) {
    for (int b = threadIdx.x; b < nb; b += blockDim.x) ord[b] = b;
    __syncthreads();
    if (threadIdx.x == 0) fisher_yates_dev(d.seed, ord, nb, T_PERM_BLOCK, (uint32_t)shard, it);
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += blockDim.x) d.blkorder[b] = ord[b];
  } else if (threadIdx.x == 0) {
    for (int b = 0; b < nb; ++b) d.blkorder[b] = b;
    fisher_yates_dev(d.seed, d.blkorder, nb, T_PERM_BLOCK, (uint32_t)shard, it);
  }
}

__global__ void k_perm_within(Dev d, uint32_t it, int identity) {
  __shared__ int w[BMAX];
  const int s = blockIdx.x;
  const int b = identity ? s : d.blkorder[s];
  const int size = (int)min((int64_t)d.B, d.M - (int64_t)b * d.B);
  for (int i = threadIdx.x; i < size; i += blockDim.x) w[i] = i;
  __syncthreads();
  if (threadIdx.x == 0 && !identity)
    fisher_yates_dev(d.seed, w, size, T_PERM_WITHIN, (uint32_t)(d.col_offset / d.B + b), it);
  __syncthreads();
  for (int i = threadIdx.x; i < d.B; i += blockDim.x) {
    d.member[(int64_t)s * d.B + i] = i < size ? b * d.B + w[i] : 0;
    d.gidx[(int64_t)s * d.B + i] = i < size ? w[i] : 0;
  }
  if (threadIdx.x == 0) { d.bsz[s] = size; d.gblk[s] = b; }
}

// ------------------------------------------------------------------------------------
// Fixed effects (BayesRv2Groups.cpp:216-225), one workgroup, sequential over F columns.
__global__ __launch_bounds__(1024) void k_fixed(Dev d, uint32_t it, int perm_on_device) {
#pragma clang fp contract(off)
  __shared__ double red[16];
  __shared__ int ford[1024];
  const int F = d.F;
  if (F > 1024) return;
  if (threadIdx.x == 0) {
    for (int f = 0; f < F; ++f) ford[f] = perm_on_device ? f : d.forder[f];
    if (perm_on_device) fisher_yates_dev(d.seed, ford, F, T_PERM_FIXED, 0, it);
  }
  __syncthreads();
  const int64_t N = d.N;
  for (int cf = 0; cf < F; ++cf) {
    const int cur = ford[cf];
    const double *f = d.fixed + (int64_t)cur * N;
    const double ca = d.alpha[cur];
    double part = 0.0;
    for (int64_t i = threadIdx.x; i < N; i += 1024) {
      const double yt = d.eps[i] + f[i] * ca;
      part += f[i] * yt;
    }
    const double num_f = block_sum<1024>(part, red);
    const double sigmaE = d.sc->sigmaE;
    const double denom_f = (double)(N - 1) + (sigmaE / d.sc->sigmaF);
    const double z = normal(d.seed, T_FIXED, (uint32_t)cur, it, 0);
    const double an = num_f / denom_f + sqrt(sigmaE / denom_f) * z;
    for (int64_t i = threadIdx.x; i < N; i += 1024) {
      const double yt = d.eps[i] + f[i] * ca;
      d.eps[i] = yt - f[i] * an;
    }
    __syncthreads();
    if (threadIdx.x == 0) d.alpha[cur] = an;
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
// k_stream: residual update for the previous block + partial dots for block position s.
// grid = RG workgroups, each owns rows [rg*R, rg*R + R) (R <= 256, one row per thread).
// Partial dots: 32 columns at a time, wave transpose-reduction (32 shuffles / 32 columns),
// cross-wave via LDS -> slab1[rg][c]; the last of each group of STREAM_GROUP workgroups
// sums its group's rows -> slab2[group][c] (read by k_solve).
__device__ __forceinline__ double wave_reduce32(double (&v)[32], int lane) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const bool hi = lane & 32;
    const double send = hi ? v[j] : v[j + 16];
    const double keep = hi ? v[j + 16] : v[j];
    v[j] = keep + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool hi = lane & 16;
    const double send = hi ? v[j] : v[j + 8];
    const double keep = hi ? v[j + 8] : v[j];
    v[j] = keep + __shfl_xor(send, 16);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool hi = lane & 8;
    const double send = hi ? v[j] : v[j + 4];
    const double keep = hi ? v[j + 4] : v[j];
    v[j] = keep + __shfl_xor(send, 8);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const bool hi = lane & 4;
    const double send = hi ? v[j] : v[j + 2];
    const double keep = hi ? v[j + 2] : v[j];
    v[j] = keep + __shfl_xor(send, 4);
  }
  {
    const bool hi = lane & 2;
    const double send = hi ? v[0] : v[1];
    const double keep = hi ? v[1] : v[0];
    v[0] = keep + __shfl_xor(send, 2);
  }
  return v[0] + __shfl_xor(v[0], 1);
}

__device__ __forceinline__ int reduce32_col(int lane) {
  return ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 +
         ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
}

// Geometry: workgroup rg owns rows [rg*R, rg*R + R), R <= 256 a multiple of 4; lane l owns the
// 4 consecutive rows rg*R + 4l .. +3 (one 16-B load per column), wave w owns the B/4 columns
// [w B/4, (w+1) B/4) of the block.  X and eps are padded to ld rows (zeros), so every load is
// unconditional.  The residual update is applied redundantly by the 4 waves (the re-read
// columns hit the CU's L1/L2) and written back by wave 0: no barrier in the streaming part.
template <int B>
__global__ __launch_bounds__(256, 2) void k_stream(Dev d, int s) {
#pragma clang fp contract(off)
  constexpr int CW = B / 4;  // columns per wave (<= 32)
  __shared__ int s_last;
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int rg = blockIdx.x;
  const int64_t row0 = (int64_t)rg * d.R + 4 * lane;
  const bool valid = 4 * lane < d.R && row0 < d.N;
  const int64_t rowc = valid ? row0 : 0;
  const float *Xr = d.X + rowc;
  const int64_t ld = d.ld;
  // block columns first: their loads do not depend on the residual update
  const int *mem = d.member + (int64_t)s * B + w * CW;
  float4 x[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(Xr + (int64_t)mem[j] * ld);
  const double2 ea = *reinterpret_cast<const double2 *>(d.eps + rowc);
  const double2 eb = *reinterpret_cast<const double2 *>(d.eps + rowc + 2);
  double e0 = ea.x, e1 = ea.y, e2 = eb.x, e3 = eb.y;
  // residual update for the previous block's changed markers, eps = (eps + x b_old) - x b_new
  // (BayesRv2.cpp:191,243); list padded to a multiple of 32 with neutral b_old = b_new = 0
  const int np = d.sc->n_pend;
  for (int p0 = 0; p0 < np; p0 += 16) {
    float4 xp[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) xp[q] = *reinterpret_cast<const float4 *>(Xr + (int64_t)d.pend_idx[p0 + q] * ld);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const double bo = d.pend_bo[p0 + q], bn = d.pend_bn[p0 + q];
      const double a0 = xp[q].x, a1 = xp[q].y, a2 = xp[q].z, a3 = xp[q].w;
      e0 = (e0 + a0 * bo) - a0 * bn;
      e1 = (e1 + a1 * bo) - a1 * bn;
      e2 = (e2 + a2 * bo) - a2 * bn;
      e3 = (e3 + a3 * bo) - a3 * bn;
    }
  }
  if (np > 0 && w == 0 && valid) {
    *reinterpret_cast<double2 *>(d.eps + row0) = make_double2(e0, e1);
    *reinterpret_cast<double2 *>(d.eps + row0 + 2) = make_double2(e2, e3);
  }
  if (!valid) e0 = e1 = e2 = e3 = 0.0;
  // partial dots: 4 rows per lane, then the wave transpose-reduction over the 64 lanes
  double v[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    if (j < CW) {
      v[j] = (((double)x[j].x * e0 + (double)x[j].y * e1) + (double)x[j].z * e2) + (double)x[j].w * e3;
    } else {
      v[j] = 0.0;
    }
  }
  const double r = wave_reduce32(v, lane);
  const int col = reduce32_col(lane);
  if ((lane & 1) == 0 && col < CW) st_sc1(d.slab1 + (int64_t)rg * B + w * CW + col, r);
  // level-2: last arriver of the group sums the group's partials in workgroup order
  const int bs = d.bsz[s];
  const int grp = rg / STREAM_GROUP;
  const int g0 = grp * STREAM_GROUP;
  const int gsz = min(STREAM_GROUP, d.RG - g0);
  if (last_arriver_wt(d.cnt1 + grp, gsz, &s_last)) {
    if (t < bs) {
      double v16[STREAM_GROUP];
#pragma unroll
      for (int q = 0; q < STREAM_GROUP; ++q) v16[q] = q < gsz ? ld_sc1(d.slab1 + (int64_t)(g0 + q) * B + t) : 0.0;
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < STREAM_GROUP; ++q) acc += v16[q];
      d.slab2[(int64_t)grp * B + t] = acc;
    }
    if (t == 0) d.cnt1[grp] = 0;
  }
}

// ------------------------------------------------------------------------------------
// Per-marker mixture decision, restating BayesRv2.cpp:195-242 exactly (f64).
// Returns the selected component (0..K-1) or FALLTHROUGH, and the quantities needed to
// bound the t = num^2 interval in which the decision cannot change.
struct Decision {
  int k;
  double denom;   // denom[k-1] of the selected k >= 1
  double margin;  // half-width in t = num^2 of a decision-invariant interval (0 = none)
};

__device__ Decision decide_bayesr(double num, double xsq, double sigmaE, double sigmaG,
                                  const double *pi_g, const double *cva_g /* stride Gs */,
                                  int Gs, int K, double p, bool want_margin) {
#pragma clang fp contract(off)
  double cVa[MAXK], denom[MAXK], muk[MAXK], logL[MAXK], slope[MAXK], A[MAXK];
  cVa[0] = 0.0;
  for (int k = 1; k < K; ++k) cVa[k] = cva_g[(int64_t)Gs * (k - 1)];
  muk[0] = 0.0;
  slope[0] = 0.0;
  double smax = 0.0;
  for (int k = 1; k < K; ++k) {
    const double cVaI = 1.0 / cVa[k];
    denom[k - 1] = xsq + (sigmaE / sigmaG) * cVaI;
    muk[k] = num / denom[k - 1];
    slope[k] = 0.5 / (denom[k - 1] * sigmaE);  // d logL_k / d num^2
    smax = fmax(smax, slope[k]);
  }
  for (int k = 0; k < K; ++k) logL[k] = log(pi_g[k]);
  for (int k = 1; k < K; ++k)
    logL[k] = logL[k] - 0.5 * log(((sigmaG / sigmaE) * xsq) * cVa[k] + 1.0) + (0.5 * (muk[k] * num)) / sigmaE;
  double gmargin = 1e300;  // distance (in t) to the nearest 700-guard flip
  auto guard = [&](int kk) -> bool {
    bool gd = false;
    for (int i = 1; i < K; ++i) {
      const double df = logL[i] - logL[kk];
      gd |= fabs(df) > 700.0;
      if (want_margin) {
        const double sl = fabs(slope[i] - slope[kk]);
        if (sl > 0.0) gmargin = fmin(gmargin, fabs(fabs(df) - 700.0) / sl);
      }
    }
    return gd;
  };
  double acum;
  if (guard(0)) {
    acum = 0.0;
  } else {
    double sum = 0.0;
    for (int i = 0; i < K; ++i) sum += exp(logL[i] - logL[0]);
    acum = 1.0 / sum;
  }
  A[0] = acum;
  int sel = FALLTHROUGH;
  for (int k = 0; k < K; ++k) {
    if (p <= acum) { sel = k; break; }
    if (k + 1 < K) {
      if (!guard(k + 1)) {
        double sum = 0.0;
        for (int i = 0; i < K; ++i) sum += exp(logL[i] - logL[k + 1]);
        acum += 1.0 / sum;
      }
      A[k + 1] = acum;
    }
  }
  Decision r;
  r.k = sel;
  r.denom = (sel != FALLTHROUGH && sel > 0) ? denom[sel - 1] : 1.0;
  r.margin = 0.0;
  if (want_margin && smax > 0.0) {
    // Decision-invariant window in t = num^2 (DESIGN.md "decision margins").  Without active
    // guards A_k(t) = sum_{j<=k} P_j(t) with P = softmax(logL), logL_j = a_j + b_j t, so
    //   dA_k/dt = A_k (1 - A_k) (bbar_{<=k} - bbar_{>k}),  |.| <= min(A_k, 1-A_k) b_max,
    // and over |t - t0| <= delta <= 1/b_max both A_k and 1-A_k grow by at most e^{b_max delta}
    // <= e.  So A_k stays on its side of p while delta <= gap / (e b_max min(A_k, 1-A_k)).
    bool any_guard = false;
    for (int kk = 0; kk < K; ++kk)
      for (int i = 1; i < K; ++i) any_guard |= fabs(logL[i] - logL[kk]) > 700.0;
    const double E = 2.718281828459045;
    auto side = [&](double gap, double Ak) -> double {
      if (!(gap > 1e-12)) return 0.0;
      if (any_guard) return gap / smax;
      const double m = fmin(Ak, 1.0 - Ak);
      return m > 0.0 ? gap / (E * smax * m) : 1e300;
    };
    double w;
    if (sel == FALLTHROUGH) {
      w = side(p - A[K - 1], A[K - 1]);
    } else {
      w = side(A[sel] - p, A[sel]);
      if (sel > 0) w = fmin(w, side(p - A[sel - 1], A[sel - 1]));
    }
    w = fmin(w, 1.0 / smax);
    r.margin = 0.5 * fmin(w, gmargin);
  }
  return r;
}

// ------------------------------------------------------------------------------------
// k_solve: one workgroup.  Exact single-site updates of block position s in visit order.
// Slow path of the serial chain: exact re-evaluation (reference formula) of position i with
// its corrected dot product, when the corrected num^2 left the decision-invariant interval.
__device__ __forceinline__ int chain_slow(const Dev &d, double num, double x2, int g,
                                                    double p, double z, double sigmaE,
                                                    double *bnew, double bold) {
  Decision dc = decide_bayesr(num, x2, sigmaE, d.sigmaGG[g], d.pi + (int64_t)g * d.K, d.cva + g, d.G,
                              d.K, p, false);
  *bnew = dc.k == 0 ? 0.0 : (dc.k == FALLTHROUGH ? bold : num / dc.denom + sqrt(sigmaE / dc.denom) * z);
  return dc.k;
}

template <bool HS, int B>
__global__ __launch_bounds__(256) void k_solve(Dev d, int s, uint32_t it) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double *Gl = reinterpret_cast<double *>(smem);  // B*B
  double *r_ = Gl + (int64_t)B * B;                 // B each:
  double *tlo = r_ + B, *thi = tlo + B, *ide = thi + B, *sdz = ide + B, *bold = sdz + B,
         *bnw = bold + B, *pz = bnw + B, *xq = pz + B, *pu = xq + B;
  int *k0 = reinterpret_cast<int *>(pu + B);
  int *gi = k0 + B, *grp = gi + B, *ksel = grp + B, *mrk = ksel + B, *misc = mrk + B;

  const int t = threadIdx.x;
  const int bs = d.bsz[s];
  const int gb = d.gblk[s];
  // 1) Gram block -> LDS (row-major, stride B), overlapped with the first batch of the
  //    dot-product reduction loads (slab2 rows padded to a multiple of 32 with zeros)
  const int tc = t < B ? t : 0;
  double sv[32];
#pragma unroll
  for (int q = 0; q < 32; ++q) sv[q] = d.slab2[(int64_t)q * B + tc];
  {
    const double2 *src = reinterpret_cast<const double2 *>(d.gram + (int64_t)gb * B * B) + t;
    double2 *dst = reinterpret_cast<double2 *>(Gl) + t;
    constexpr int NQ = B * B / 2 / 256;
    double2 tmp[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) tmp[q] = src[q * 256];
#pragma unroll
    for (int q = 0; q < NQ; ++q) dst[q * 256] = tmp[q];
  }
  double dsum = 0.0;
#pragma unroll
  for (int q = 0; q < 32; ++q) dsum += sv[q];
  for (int q0 = 32; q0 < d.NG; q0 += 32) {
#pragma unroll
    for (int q = 0; q < 32; ++q) sv[q] = d.slab2[(int64_t)(q0 + q) * B + tc];
#pragma unroll
    for (int q = 0; q < 32; ++q) dsum += sv[q];
  }
  // 2) per-marker preparation, one thread per position
  const Scal sc = *d.sc;
  if (t < bs) {
    const int m = d.member[(int64_t)s * B + t];
    const int64_t gm = d.col_offset + m;
    const double bo = d.beta[m];
    const double x2 = d.xsq[m];
    const double r = dsum + x2 * bo;  // num = x.(eps + x b_old)
    const double p = uniform(d.seed, T_MARKER, (uint32_t)gm, it, 0);
    const double z = normal(d.seed, T_MARKER, (uint32_t)gm, it, 1);
    const int g = (d.gAssign && !HS) ? d.gAssign[m] : 0;
    mrk[t] = m;
    gi[t] = d.gidx[(int64_t)s * B + t];
    grp[t] = g;
    bold[t] = bo;
    xq[t] = x2;
    pz[t] = z;
    pu[t] = p;
    r_[t] = r;
    if (HS) {
      const double lam = d.lambda[m];
      const double sv = sc.tau * sc.c2 * lam / (sc.tau * lam + sc.c2);
      const double D = x2 + (sc.sigmaE / sv);
      ide[t] = 1.0 / D;
      sdz[t] = sqrt(sc.sigmaE / D) * z;  // HorseshoeR.cpp:234
      k0[t] = 1;
      tlo[t] = 0.0;
      thi[t] = 1e308;
    } else {
      Decision dc = decide_bayesr(r, x2, sc.sigmaE, d.sigmaGG[g], d.pi + (int64_t)g * d.K,
                                  d.cva + g, d.G, d.K, p, true);
      k0[t] = dc.k;
      ide[t] = 1.0 / dc.denom;
      sdz[t] = sqrt(sc.sigmaE / dc.denom) * z;  // BayesRv2.cpp:228
      const double t0 = r * r;
      tlo[t] = t0 - dc.margin;
      thi[t] = dc.margin > 0.0 ? t0 + dc.margin : -1.0;  // empty interval -> slow path
    }
  }
  __syncthreads();
  // 3) serial chain on wave 0 (lane l owns positions l + 64 q).  A ballot finds the next
  //    position whose update may change beta (fast decision changes it, or its corrected num^2
  //    left the invariant window); runs of unchanged positions are committed in one step.  The
  //    owner's new beta is broadcast by readlane and every later position subtracts G_ji*delta.
  if (t < 64) {
    const int lane = t;
    constexpr int NS = B / 64;
    double r[NS], lo[NS], hi[NS], id[NS], sz[NS], bo[NS], bf[NS];
    int kk[NS], gg[NS], kf[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const int pos = q * 64 + lane;
      const bool in = pos < bs;
      r[q] = in ? r_[pos] : 0.0;
      lo[q] = in ? tlo[pos] : 0.0;
      hi[q] = in ? thi[pos] : -1.0;
      id[q] = in ? ide[pos] : 0.0;
      sz[q] = in ? sdz[pos] : 0.0;
      bo[q] = in ? bold[pos] : 0.0;
      kk[q] = in ? k0[pos] : 0;
      gg[q] = in ? gi[pos] : 0;
      bf[q] = bo[q];
      kf[q] = kk[q];
    }
    int nslow = 0;
    int i = 0;
    while (i < bs) {
      int first = bs;
#pragma unroll
      for (int q = NS - 1; q >= 0; --q) {
        const int pos = q * 64 + lane;
        const double tt = r[q] * r[q];
        const bool fast = tt >= lo[q] && tt <= hi[q];
        const bool nochange = !HS && fast && (kk[q] == FALLTHROUGH || (kk[q] == 0 && bo[q] == 0.0));
        const uint64_t bal = __ballot(pos >= i && pos < bs && !nochange);
        if (bal) first = q * 64 + __builtin_ctzll(bal);
      }
      if (first >= bs) break;  // the rest keep their fast decisions (no change)
      const int qs = first >> 6, l = first & 63;  // wave-uniform
      double rv = r[0], lov = lo[0], hiv = hi[0], idv = id[0], szv = sz[0], bov = bo[0];
      int kv = kk[0], gv = gg[0];
#pragma unroll
      for (int q = 1; q < NS; ++q)
        if (qs == q) { rv = r[q]; lov = lo[q]; hiv = hi[q]; idv = id[q]; szv = sz[q]; bov = bo[q]; kv = kk[q]; gv = gg[q]; }
      double bn;
      int ks;
      if (HS) {
        bn = rv * idv + szv;
        ks = 1;
      } else {
        const double tt = rv * rv;
        const int fast = __builtin_amdgcn_readlane((int)(tt >= lov && tt <= hiv), l);
        if (fast) {
          ks = kv;
          bn = kv == 0 ? 0.0 : (kv == FALLTHROUGH ? bov : rv * idv + szv);
        } else {
          const double ri = readlane_f64(rv, l);  // uniform inputs -> uniform result
          const double boi = readlane_f64(bov, l);
          ks = chain_slow(d, ri, xq[first], grp[first], pu[first], pz[first], sc.sigmaE, &bn, boi);
          ++nslow;
        }
      }
      const double delta = readlane_f64(bn - bov, l);
      const int ksu = __builtin_amdgcn_readlane(ks, l);
      const int gf = __builtin_amdgcn_readlane(gv, l);
      const double *grow = Gl + gf * B;
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        const int pos = q * 64 + lane;
        if (pos == first) { bf[q] = bn; kf[q] = ksu; }
        if (pos > first && delta != 0.0) r[q] = r[q] - grow[gg[q]] * delta;
      }
      i = first + 1;
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const int pos = q * 64 + lane;
      if (pos < bs) { ksel[pos] = kf[q]; bnw[pos] = bf[q]; }
    }
    if (lane == 0 && nslow) atomicAdd(&d.sc->n_slow, (unsigned long long)nslow);
  }
  __syncthreads();
  // 4) write back, compact the changed markers into the pending list (position order)
  int changed = 0;
  if (t < bs) {
    const int m = mrk[t];
    const int ks = ksel[t];
    d.beta[m] = bnw[t];
    if (!HS) {
      if (ks != FALLTHROUGH) d.comp[m] = ks;
      d.sel[m] = ks != FALLTHROUGH;
    }
    changed = bnw[t] != bold[t];
  }
  const uint64_t bal = __ballot(changed);
  const int lane = t & 63, wv = t >> 6;
  if (lane == 0) misc[wv] = __popcll(bal);
  __syncthreads();
  int base = 0;
  for (int q = 0; q < wv; ++q) base += misc[q];
  if (changed) {
    const int idx = base + __popcll(bal & ((1ull << lane) - 1ull));
    d.pend_idx[idx] = mrk[t];
    d.pend_bo[idx] = bold[t];
    d.pend_bn[idx] = bnw[t];
  }
  const int npend = misc[0] + misc[1] + misc[2] + misc[3];
  const int npad = (npend + 31) & ~31;  // k_stream reads the list in batches of 32
  if (t >= npend && t < npad) {  // neutral padding: eps + x*0 - x*0 == eps exactly
    d.pend_idx[t] = 0;
    d.pend_bo[t] = 0.0;
    d.pend_bn[t] = 0.0;
  }
  if (t == 0) {
    d.sc->n_pend = npad;
    if (npend) atomicAdd(&d.sc->n_changed, (unsigned long long)npend);
  }
}

// ------------------------------------------------------------------------------------
// Marker pass: Horseshoe v / lambda draws (HorseshoeR.cpp:218,242) and the statistics the
// hyper-parameter draws need: sum beta^2, sum beta^2/lambda, betaAcum[g], v[g][k].
enum MarkerMode : int { MR_BAYESR = 0, MR_HS = 1, MR_COUNT_ALL = 2 };

__global__ __launch_bounds__(256) void k_markers(Dev d, int mode, uint32_t it) {
#pragma clang fp contract(off)
  __shared__ double red[8];
  __shared__ int cnt[MAXG * MAXK];
  __shared__ int s_last, s_gmin, s_gmax;
  const int NS = stats_size(d.G, d.K);
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = m < d.M;
  for (int q = threadIdx.x; q < d.G * d.K; q += 256) cnt[q] = 0;
  if (threadIdx.x == 0) { s_gmin = 1 << 30; s_gmax = -1; }
  __syncthreads();
  double b2 = 0.0, b2l = 0.0, bacc = 0.0;
  int g = 0;
  if (valid) {
    const double b = d.beta[m];
    b2 = b * b;
    if (mode == MR_HS) {
      const Hyper &h = d.hyp;
      const uint32_t gm = (uint32_t)(d.col_offset + m);
      const double v = inv_gamma_rate_rng(d.seed, 0.5 + 0.5 * h.vL, h.vL / d.lambda[m] + 1.0, T_HS_V, gm, it);
      const double lam = inv_gamma_rate_rng(
          d.seed, 0.5 + 0.5 * h.vL, h.vL * (1.0 / v) + (0.5 * (b * b)) * (1.0 / d.sc->tau), T_HS_LAMBDA, gm, it);
      d.hsv[m] = v;
      d.lambda[m] = lam;
      b2l = (b * b) / lam;
    } else {
      g = d.gAssign ? d.gAssign[m] : 0;
      const int c = d.comp[m];
      if (mode == MR_COUNT_ALL) {
        atomicAdd(&cnt[g * d.K + c], 1);
      } else if (d.sel[m]) {
        atomicAdd(&cnt[g * d.K + c], 1);
        if (c > 0) bacc = b * b;
      }
      atomicMin(&s_gmin, g);
      atomicMax(&s_gmax, g);
    }
  }
  const double s0 = block_sum<256>(b2, red);
  const double s1 = block_sum<256>(b2l, red);
  double *out = d.mslab + (int64_t)blockIdx.x * NS;
  if (threadIdx.x == 0) { out[0] = s0; out[1] = s1; }
  const int gmin = s_gmin, gmax = s_gmax;
  for (int q = threadIdx.x; q < d.G; q += 256) out[2 + q] = 0.0;
  __syncthreads();
  for (int gg = gmin; gg <= gmax; ++gg) {
    const double sg = block_sum<256>(g == gg ? bacc : 0.0, red);
    if (threadIdx.x == 0) out[2 + gg] = sg;
  }
  for (int q = threadIdx.x; q < d.G * d.K; q += 256) out[2 + d.G + q] = (double)cnt[q];
  if (last_arriver(d.mcnt, gridDim.x, &s_last)) {
    for (int q = threadIdx.x; q < NS; q += 256) {
      double acc = 0.0;
      for (int w = 0; w < (int)gridDim.x; ++w) acc += d.mslab[(int64_t)w * NS + q];
      d.stats[q] = acc;
    }
    if (threadIdx.x == 0) *d.mcnt = 0;
  }
}

// ------------------------------------------------------------------------------------
// Hyper-parameter draws at the end of a sweep.
//   V2:        BayesRv2.cpp:247-255        Groups: BayesRv2Groups.cpp:301-312
//   restart:   BRv2Grstart.cpp:254-262     Horseshoe: HorseshoeR.cpp:245-253
__device__ void dirichlet_dev(uint64_t seed, const double *alpha, int K, double *out, uint32_t ent0,
                              uint32_t it) {
  double sum = 0.0;
  for (int k = 0; k < K; ++k) out[k] = gamma(seed, alpha[k], T_PI, ent0 + (uint32_t)k, it);
  for (int k = 0; k < K; ++k) sum += out[k];
  for (int k = 0; k < K; ++k) out[k] /= sum;
}

__global__ void k_hyper(Dev d, uint32_t it, const double *stats) {
#pragma clang fp contract(off)
  const int t = threadIdx.x;
  Scal *sc = d.sc;
  const Hyper &h = d.hyp;
  const int G = d.G, K = d.K;
  const double N = (double)d.N;
  const double *bacc = stats + 2;
  const double *v = stats + 2 + G;
  const double sigmaE_new = inv_scaled_chisq_rng(d.seed, h.v0E + N, (sc->S2 + h.v0E * h.s02E) / (h.v0E + N),
                                                 T_SIGMAE, 0, it);
  if (d.model == MODEL_HORSESHOE) {
    if (t == 0) {
      const double M = (double)d.M_total;
      sc->tau = inv_gamma_rate_rng(d.seed, 0.5 * (M + h.vT), h.vT / sc->eta + (0.5) * stats[1], T_HS_TAU, 0, it);
      sc->c2 = inv_gamma_rate_rng(d.seed, 0.5 * h.vC + 0.5 * M, h.vC * h.sC * 0.5 + 0.5 * stats[0], T_HS_C2, 0, it);
      sc->sigmaE = sigmaE_new;
    }
    return;
  }
  if (d.model == MODEL_V2) {
    if (t == 0) {
      const int m0 = (int)(d.M_total - (int64_t)v[0]);
      d.sigmaGG[0] = inv_scaled_chisq_rng(d.seed, h.v0G + m0, (stats[0] * m0 + h.v0G * h.s02G) / (h.v0G + m0),
                                          T_SIGMAG, 0, it);
      sc->sigmaE = sigmaE_new;
      double a[MAXK];
      for (int k = 0; k < K; ++k) a[k] = v[k] + 1.0;
      dirichlet_dev(d.seed, a, K, d.pi, 0, it);
    }
    return;
  }
  // Groups / restart
  if (t == 0) {
    if (d.model == MODEL_GROUPS) {
      double asq = 0.0;
      for (int f = 0; f < d.F; ++f) asq += d.alpha[f] * d.alpha[f];
      sc->sigmaF = inv_scaled_chisq_rng(d.seed, h.v0E + d.F, (asq + h.v0E * h.s02E) / (h.v0E + d.F), T_SIGMAF, 0, it);
    }
    sc->sigmaE = sigmaE_new;
  }
  for (int g = t; g < G; g += blockDim.x) {
    double rs = 0.0;
    for (int k = 0; k < K; ++k) rs += v[g * K + k];
    const int m0 = (int)(rs - v[g * K + 0]);
    d.sigmaGG[g] = inv_scaled_chisq_rng(d.seed, h.v0G + m0, (bacc[g] * m0 + h.v0G * h.s02G) / (h.v0G + m0),
                                        T_SIGMAG, (uint32_t)g, it);
    double a[MAXK];
    for (int k = 0; k < K; ++k) a[k] = v[g * K + k] + 1.0;
    dirichlet_dev(d.seed, a, K, d.pi + (int64_t)g * K, (uint32_t)(g * K), it);
  }
}

// Init draws: BayesRv2.cpp:158-169, Groups :185-204, restart :157-165, Horseshoe :168-195
__global__ void k_hyper_init(Dev d, const double *stats, int pi_given) {
#pragma clang fp contract(off)
  const int t = threadIdx.x;
  Scal *sc = d.sc;
  const Hyper &h = d.hyp;
  const int G = d.G, K = d.K;
  const double N = (double)d.N;
  if (d.model != MODEL_RESTART && t == 0) sc->sigmaE = sc->S2 / N * 0.5;
  if (d.model == MODEL_V2 && t == 0) d.sigmaGG[0] = uniform(d.seed, T_INIT, 0, INIT_IT, 0);
  if (d.model == MODEL_GROUPS) {
    for (int g = t; g < G; g += blockDim.x) d.sigmaGG[g] = uniform(d.seed, T_INIT, (uint32_t)g, INIT_IT, 0);
    if (t == 0) sc->sigmaF = uniform(d.seed, T_INIT, 0x10000000u, INIT_IT, 0);
  }
  if (d.model == MODEL_RESTART && !pi_given) {
    const double *v = stats + 2 + G;
    for (int g = t; g < G; g += blockDim.x) {
      double a[MAXK];
      for (int k = 0; k < K; ++k) a[k] = v[g * K + k] + 1.0;
      dirichlet_dev(d.seed, a, K, d.pi + (int64_t)g * K, (uint32_t)(g * K), INIT_IT);
    }
  }
  if (d.model == MODEL_HORSESHOE && t == 0) {
    const double sE = sc->S2 / N * 0.5;
    sc->sigmaE = sE;
    sc->eta = inv_gamma_rate_rng(d.seed, 0.5, 1.0 / (sE * pow(h.A, 2)), T_HS_ETA, 0, INIT_IT);
    sc->tau = (1.0 / sc->eta) * inv_gamma_rate_rng(d.seed, 0.5 * h.vT, h.vT, T_HS_TAU, 0, INIT_IT);
  }
}

}  // namespace brr

// ======================================================================================
// host-side launch wrappers (called by brr_session.cpp)
#include "brr_launch.hpp"

namespace brr {

static inline unsigned cdiv64(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

hipError_t launch_synth_x(float *X, int64_t ld, int64_t N, int64_t M, int64_t col0, uint64_t ds,
                          hipStream_t st) {
  hipLaunchKernelGGL(k_synth_x, dim3((unsigned)M), dim3(256), 0, st, X, ld, N, col0, ds);
  return hipGetLastError();
}

hipError_t launch_synth_y(const float *X, int64_t ld, int64_t N, const int *cidx, const double *cb,
                          int nc, double *y, hipStream_t st) {
  hipLaunchKernelGGL(k_synth_y, dim3(cdiv64(N, 256)), dim3(256), 0, st, X, ld, N, cidx, cb, nc, y);
  return hipGetLastError();
}

hipError_t launch_cast_x(const void *src, bool is_f64, int64_t lds, float *dst, int64_t ldd,
                         int64_t N, int64_t M, hipStream_t st) {
  dim3 grid(cdiv64(ldd, 256) > 64 ? 64 : cdiv64(ldd, 256), (unsigned)M);
  if (is_f64)
    hipLaunchKernelGGL(k_cast_f64_f32, grid, dim3(256), 0, st, (const double *)src, lds, dst, ldd, N, M);
  else
    hipLaunchKernelGGL(k_copy_f32, grid, dim3(256), 0, st, (const float *)src, lds, dst, ldd, N, M);
  return hipGetLastError();
}

hipError_t launch_gram(const Dev &d, int nblocks, hipStream_t st) {
  const int nt = (d.B + 63) / 64;
  hipLaunchKernelGGL(k_gram, dim3((unsigned)nblocks, (unsigned)(nt * nt)), dim3(256), 0, st, d.X, d.ld,
                     d.member, d.bsz, d.B, d.gram);
  return hipGetLastError();
}

hipError_t launch_xsq(const Dev &d, hipStream_t st) {
  hipLaunchKernelGGL(k_xsq_from_gram, dim3((unsigned)d.nb), dim3(BMAX), 0, st, d.gram, d.member, d.bsz, d.B,
                     d.nb, d.xsq);
  return hipGetLastError();
}

hipError_t launch_rows(const Dev &d, int flags, const double *deps_in, hipStream_t st) {
  hipLaunchKernelGGL(k_rows, dim3(cdiv64(d.N, 256)), dim3(256), 0, st, d, flags, deps_in);
  return hipGetLastError();
}

hipError_t launch_sweep_start(const Dev &d, uint32_t it, hipStream_t st) {
  hipLaunchKernelGGL(k_sweep_start, dim3(1), dim3(64), 0, st, d, it);
  return hipGetLastError();
}

hipError_t launch_perm(const Dev &d, uint32_t it, int shard, bool identity, hipStream_t st) {
  if (!identity) {
    const size_t lds = d.nb <= PERM_LDS_MAX ? sizeof(int) * (size_t)d.nb : 0;
    hipLaunchKernelGGL(k_perm_blockorder, dim3(1), dim3(256), lds, st, d, it, shard);
  }
  hipLaunchKernelGGL(k_perm_within, dim3((unsigned)d.nb), dim3(64), 0, st, d, it, identity ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_fixed(const Dev &d, uint32_t it, bool perm_on_device, hipStream_t st) {
  hipLaunchKernelGGL(k_fixed, dim3(1), dim3(1024), 0, st, d, it, perm_on_device ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_stream(const Dev &d, int s, hipStream_t st) {
  if (d.B == 64)
    hipLaunchKernelGGL(k_stream<64>, dim3((unsigned)d.RG), dim3(256), 0, st, d, s);
  else
    hipLaunchKernelGGL(k_stream<128>, dim3((unsigned)d.RG), dim3(256), 0, st, d, s);
  return hipGetLastError();
}

size_t solve_lds_bytes(int B) { return (size_t)B * B * 8 + (size_t)B * 10 * 8 + (size_t)B * 5 * 4 + 64; }

hipError_t launch_solve(const Dev &d, int s, uint32_t it, hipStream_t st) {
  const size_t lds = solve_lds_bytes(d.B);
  const bool hs = d.model == MODEL_HORSESHOE;
  if (d.B == 64) {
    if (hs) hipLaunchKernelGGL((k_solve<true, 64>), dim3(1), dim3(256), lds, st, d, s, it);
    else hipLaunchKernelGGL((k_solve<false, 64>), dim3(1), dim3(256), lds, st, d, s, it);
  } else {
    if (hs) hipLaunchKernelGGL((k_solve<true, 128>), dim3(1), dim3(256), lds, st, d, s, it);
    else hipLaunchKernelGGL((k_solve<false, 128>), dim3(1), dim3(256), lds, st, d, s, it);
  }
  return hipGetLastError();
}

hipError_t set_solve_lds_limit(int /*B*/) {
  // One limit for every variant, the largest any block size needs: lowering it for one
  // session silently shrank the LDS window of later launches (out-of-range LDS writes are
  // dropped, no fault).
  const int lds = (int)solve_lds_bytes(BMAX);
  const void *fns[4] = {(const void *)k_solve<true, 64>, (const void *)k_solve<false, 64>,
                        (const void *)k_solve<true, 128>, (const void *)k_solve<false, 128>};
  for (const void *f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
  }
  return hipFuncSetAttribute((const void *)k_perm_blockorder, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)(sizeof(int) * PERM_LDS_MAX));
}

hipError_t launch_markers(const Dev &d, int mode, uint32_t it, hipStream_t st) {
  hipLaunchKernelGGL(k_markers, dim3((unsigned)d.MRG), dim3(256), 0, st, d, mode, it);
  return hipGetLastError();
}

hipError_t launch_hyper(const Dev &d, uint32_t it, const double *stats, hipStream_t st) {
  hipLaunchKernelGGL(k_hyper, dim3(1), dim3(64), 0, st, d, it, stats);
  return hipGetLastError();
}

hipError_t launch_hyper_init(const Dev &d, const double *stats, bool pi_given, hipStream_t st) {
  hipLaunchKernelGGL(k_hyper_init, dim3(1), dim3(64), 0, st, d, stats, pi_given ? 1 : 0);
  return hipGetLastError();
}

}  // namespace brr
