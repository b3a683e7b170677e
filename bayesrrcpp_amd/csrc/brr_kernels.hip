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
#include <cstdlib>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "brr_device.hpp"
#include "brr_rng.hpp"
#include "brr_chain.hpp"

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

// Workgroup barrier that orders LDS only: no vmcnt wait (a __syncthreads' release fence makes every
// wave first wait for ALL its outstanding global accesses, LDS-DMA copies included).  For barriers
// whose only cross-wave data is in LDS, where some waves have a copy in flight they wait for later.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// ------------------------------------------------------------------------------------
// Genotype storage: f32 X, or 2-bit codes + a 4-entry value table per column (brr_device.hpp).
// x_selk picks the value of the code in bits 2k, 2k+1 of b: two sign-extended bit extracts give
// all-ones / all-zero masks and three bitfield inserts select (v_bfe_i32 + v_bfi_b32: no compare,
// no VCC dependency, so the values of a byte decode in parallel).
// (inline asm: written in C the compiler turns the masks back into compares and VCC selects)
__device__ __forceinline__ uint32_t bfe_i1(uint32_t b, int pos) {
  uint32_t m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(b), "v"(pos));
  return m;
}
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {  // (m & a) | (~m & b)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float x_selk(float4 l, uint32_t b, int k) {
  const uint32_t m0 = bfe_i1(b, 2 * k), m1 = bfe_i1(b, 2 * k + 1);
  const uint32_t lo = bfi(m0, __float_as_uint(l.y), __float_as_uint(l.x));
  const uint32_t hi = bfi(m0, __float_as_uint(l.w), __float_as_uint(l.z));
  return __uint_as_float(bfi(m1, hi, lo));
}
__device__ __forceinline__ float x_sel(float4 l, uint32_t c) { return x_selk(l, c, 0); }
// rows 4k .. 4k+3 of a column from their code byte
__device__ __forceinline__ float4 x_decode4(uint32_t b, float4 l) {
  return make_float4(x_selk(l, b, 0), x_selk(l, b, 1), x_selk(l, b, 2), x_selk(l, b, 3));
}
__device__ __forceinline__ float4 x_lut(const Dev &d, int64_t col) {
  return *reinterpret_cast<const float4 *>(d.xlut + 4 * col);
}
// 2-bit code tiles (brr_device.hpp): byte of (column col, row quad g) -- column col = b B + i of
// block b, group i / 16 of 16 columns, quad g: ((b B/16 + i/16) nq + g) 16 + i % 16, nq = ldc
__host__ __device__ __forceinline__ int64_t code_off(int64_t col, int64_t g, int B, int64_t nq) {
  const int64_t b = col / B, i = col - b * B;
  return ((b * (B >> 4) + (i >> 4)) * nq + g) * 16 + (i & 15);
}
// one value (scattered reads: change lists, synthetic Y)
__device__ __forceinline__ float x_at(const Dev &d, int64_t col, int64_t row) {
  if (d.Xc) return x_sel(x_lut(d, col), (uint32_t)d.Xc[code_off(col, row >> 2, d.B, d.ldc)] >> (2 * (row & 3)));
  return d.X[col * d.ld + row];
}
// four consecutive rows row4 .. row4+3 (row4 a multiple of 4)
__device__ __forceinline__ float4 x_at4(const Dev &d, int64_t col, int64_t row4) {
  if (d.Xc) return x_decode4(d.Xc[code_off(col, row4 >> 2, d.B, d.ldc)], x_lut(d, col));
  return *reinterpret_cast<const float4 *>(d.X + col * d.ld + row4);
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
__device__ __forceinline__ unsigned long long ld_sc1_u64(const double *p) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_u64(double *p, unsigned long long v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_int(int *p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_sc1_int(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The persistent solver's hand-over of the reduced dots (slab2): a slot holds the sentinel of the block
// that will use it next until its reducer overwrites it with the dot -- a signalling-NaN bit pattern
// that arithmetic never produces (it yields quiet NaNs), carrying the block's session-wide epoch
// (Dev::sbase + s) so that a stale value of an earlier block is never mistaken for ready data.
__host__ __device__ inline unsigned long long slab_sentinel(int epoch) {
  return 0x7FF4000000000000ull | (unsigned long long)(unsigned)epoch;
}

// Bounded wait (one lane) for a device counter published by a kernel running concurrently on
// the other queue.  Never spins forever: after ~0.5 s the protocol error flag is raised and the
// caller proceeds (the host reports the error after the sweep).
constexpr uint32_t SPIN_MAX = 1u << 22;
__device__ __forceinline__ void stamp(int *sync, int k) {  // first writer wins
  unsigned long long *ts = reinterpret_cast<unsigned long long *>(sync + SY_TS) + k;
  atomicCAS(ts, 0ull, (unsigned long long)wall_clock64());
}

#ifndef BRR_SPIN_SLEEP
#define BRR_SPIN_SLEEP 8  // s_sleep units (64 clocks) between polls of a hand-over counter
#endif
__device__ __forceinline__ void wait_geq(const int *cnt, int target, int *sync, int where) {
  for (uint32_t n = 0;; ++n) {
    const int v = ld_sc1_int(cnt);
    if ((int)((unsigned)v - (unsigned)target) >= 0) return;  // cumulative counters: wrap-safe
    if (n == 0 && where == 2) stamp(sync, 6);
    if (n > SPIN_MAX) {
      stamp(sync, 7);
      if (atomicCAS(sync + SY_ERR, 0, 1) == 0) {  // the first failure records where it happened
        st_sc1_int(sync + SY_ERR + 1, where);
        st_sc1_int(sync + SY_ERR + 2, target);
        st_sc1_int(sync + SY_ERR + 3, v);
        st_sc1_int(sync + SY_ERR + 4, (int)blockIdx.x);
      }
      return;
    }
    if ((n & 255) == 255 && ld_sc1_int(sync + SY_ERR)) return;  // an earlier wait already failed
    __builtin_amdgcn_s_sleep(BRR_SPIN_SLEEP);
  }
}

// Publish a count after this workgroup's sc1 payload stores: every storing wave drains, then
// one relaxed agent-scope add (MI355X_MICROARCH.md "Valid forms", row 1).
__device__ __forceinline__ void publish_add(int *cnt, int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// Diagnostics (prof_on): per-block wall-clock events of the fused sweep, Dev::trace[s][16].
// "first" events store ~t with atomicMax (the host inverts them).
enum TraceEv : int {
  TR_SOLVE0 = 0, TR_GDONE_SEEN = 1, TR_CHAIN = 2, TR_PUB = 3, TR_PEND_FIRST = 4, TR_PEND_LAST = 5,
  TR_APPLY_LAST = 6, TR_ITEMS_LAST = 7, TR_L2_LAST = 8, TR_L2_FIRST = 9, TR_ITEMS_FIRST = 10
};
__device__ __forceinline__ void tr_last(const Dev &d, int s, int ev) {
  atomicMax(d.trace + (int64_t)s * 16 + ev, (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void tr_first(const Dev &d, int s, int ev) {
  atomicMax(d.trace + (int64_t)s * 16 + ev, ~(unsigned long long)wall_clock64());
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

// f32 storage (X) or 2-bit codes (Xc, code = genotype, 3 = padding) + value table (xlut).
// Row shards: the column statistics run over all Ntot rows of the cohort (the
// genotypes are counter-based, so every shard draws them), only rows [row0, row0 + N) are stored.
__global__ __launch_bounds__(256) void k_synth_x(float *X, uint8_t *Xc, float *xlut, int64_t ld, int64_t ldc,
                                                 int64_t N, int64_t col0, uint64_t ds, int64_t Ntot, int64_t row0,
                                                 int B) {
#pragma clang fp contract(off)
  __shared__ double red[8];
  __shared__ int s_att;
  const int64_t jl = blockIdx.x;
  const int64_t j = col0 + jl;
  const double f = 0.05 + 0.45 * uniform(ds, T_DATA_FREQ, (uint32_t)j, 0, 0);
  const double t0 = (1.0 - f) * (1.0 - f);
  const double t1 = 1.0 - f * f;
  float *x = X ? X + jl * ld : nullptr;
  uint32_t att = 0;
  double S = 0.0, Q = 0.0;
  for (; att < 16; ++att) {
    double s = 0.0, q = 0.0;
    for (int64_t i = threadIdx.x; i < Ntot; i += 256) {
      int g = genotype(ds, i, j, att, t0, t1);
      s += g;
      q += g * g;
    }
    S = block_sum<256>(s, red);
    Q = block_sum<256>(q, red);
    if (Ntot > 1 && Q * (double)Ntot != S * S) break;
  }
  if (threadIdx.x == 0) s_att = (int)att;
  __syncthreads();
  const bool mono = s_att == 16 || Ntot < 2;
  const double mean = S / (double)Ntot;
  const double var = (Q - S * S / (double)Ntot) / (double)(Ntot - 1);
  const double sd = sqrt(var);
  if (Xc) {
    // value of genotype g = f32((g - mean) / sd), exactly the f32 storage's value
    if (threadIdx.x < 4) {
      const int g = threadIdx.x;
      xlut[4 * jl + g] = (mono || g == 3) ? 0.f : (float)(((double)g - mean) / sd);
    }
    for (int64_t b = threadIdx.x; b < ldc; b += 256) {
      uint32_t byte = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t i = 4 * b + k;
        const uint32_t c = (mono || i >= N) ? 3u : (uint32_t)genotype(ds, row0 + i, j, att, t0, t1);
        byte |= c << (2 * k);
      }
      Xc[code_off(jl, b, B, ldc)] = (uint8_t)byte;
    }
    return;
  }
  if (mono) {
    for (int64_t i = threadIdx.x; i < ld; i += 256) x[i] = 0.f;
    return;
  }
  for (int64_t i = threadIdx.x; i < ld; i += 256) {
    float v = 0.f;
    if (i < N) v = (float)(((double)genotype(ds, row0 + i, j, att, t0, t1) - mean) / sd);
    x[i] = v;
  }
}

// 2-bit upload: a chunk of nc column-major code columns (ldc bytes each) into the code tiles
__global__ __launch_bounds__(256) void k_codes_tile(const uint8_t *src, uint8_t *Xc, int64_t c0, int64_t nc,
                                                    int64_t ldc, int B) {
  const int64_t jj = blockIdx.y;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < ldc; g += (int64_t)gridDim.x * 256)
    Xc[code_off(c0 + jj, g, B, ldc)] = src[jj * ldc + g];
}

// 2-bit storage: a column-major copy of the code tiles (ldc bytes per column, PLINK packing), the source of
// the streamers' change-list apply where no LDS code cache holds the recent blocks: a wave reads one
// column's 64 row quads as 64 contiguous bytes instead of one byte of each of 64 16-B tile granules
// (1 KiB of lines).  Thread = one column and four row quads (one 4-byte word).
__global__ __launch_bounds__(256) void k_codes_cm(Dev d, uint8_t *xcm) {
  const int64_t nw = d.ldc / 4;  // words per column (ldc = ld / 4, ld a multiple of 256)
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= nw * ((d.M + 15) / 16 * 16)) return;  // (whole tile groups: the last one may be short)
  // consecutive threads: the 16 columns of a tile group at the same four quads (their reads share 64 B)
  const int64_t grp = idx / (16 * nw), rem = idx - grp * 16 * nw;
  const int64_t wq = rem / 16, col = grp * 16 + rem % 16;
  if (col >= d.M) return;
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) v |= (uint32_t)d.Xc[code_off(col, 4 * wq + k, d.B, d.ldc)] << (8 * k);
  reinterpret_cast<uint32_t *>(xcm + col * d.ldc)[wq] = v;
}

// y_i = sum_{causal j} x_ij beta_j  (causal list from the host)
__global__ __launch_bounds__(256) void k_synth_y(Dev d, const int *cidx, const double *cbeta, int nc,
                                                 double *y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= d.N) return;
  double acc = 0.0;
  for (int c = 0; c < nc; ++c) acc += (double)x_at(d, cidx[c], i) * cbeta[c];
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
#ifndef GRAM_TILE
#define GRAM_TILE 128
#endif
#ifndef GRAM_KC
#define GRAM_KC 128
#endif
constexpr size_t GRAM_LDS = 2 * sizeof(float) * GRAM_KC * (GRAM_TILE + 1);
// Block Gram matrices: G[b][i][j] = sum_r x(col(b,i))[r] * x(col(b2,j))[r] in f64 with
// b2 = (b + shift) mod nb: shift 0 gives the diagonal blocks X_b^T X_b, shift 1 the cross-Gram
// of cycle neighbours (also stored transposed in GT when GT != nullptr).  GRAM_TILE^2 output tile
// per workgroup (a quadrant per wave in 16 x 16 tiles of the FP64 matrix core's 16 x 16 x 4 op),
// 32-row chunks staged in LDS as f32 (the genotype values), converted to f64 as operands.  The
// f32 x f32 products are exact in f64; element (i,j) and (j,i) of a diagonal block accumulate the
// same products in the same k order.
__global__ __launch_bounds__(256) void k_gram(Dev d, const int *member, const int *bsz, int B, int nb, int shift,
                                              double *G, double *GT) {
  constexpr int T = GRAM_TILE;  // output tile T x T per workgroup, a (T/2) x (T/2) quadrant per wave
  constexpr int KC = GRAM_KC;   // rows per LDS chunk (512 B per column: DRAM page locality)
  constexpr int NQ = T / 32;    // 16 x 16 MFMA tiles per wave and dimension
  const float *X = d.X;
  const int64_t ld = d.ld;
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  float (*As)[T + 1] = reinterpret_cast<float (*)[T + 1]>(gsm);
  float (*Bs)[T + 1] = reinterpret_cast<float (*)[T + 1]>(gsm + sizeof(float) * KC * (T + 1));
  const int gb = blockIdx.x;
  const int gb2 = (gb + shift) % nb;
  const int ntile = (B + T - 1) / T;
  const int ti = blockIdx.y / ntile, tj = blockIdx.y % ntile;
  const int bs = bsz[gb], bs2 = bsz[gb2];
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const int wi = wv >> 1, wj = wv & 1;  // this wave's quadrant of the tile
  typedef double f64x4 __attribute__((ext_vector_type(4)));
  f64x4 acc[NQ][NQ];
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int b = 0; b < NQ; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
  // loader: the chunk's KC rows of the tile's T columns of each operand, in (column, row quad)
  // elements with consecutive threads on consecutive quads of one column (a wave reads KC / 4 x
  // 16 B = 512 B contiguous per column); the columns' global indices staged once in LDS
  __shared__ int64_t s_ca[T], s_cb[T];
  __shared__ float4 s_la[T], s_lb[T];
  for (int c = t; c < T; c += 256) {
    const int ci = ti * T + c, cj = tj * T + c;
    s_ca[c] = ci < bs ? member[(int64_t)gb * B + ci] : -1;
    s_cb[c] = cj < bs2 ? member[(int64_t)gb2 * B + cj] : -1;
    const float4 z = make_float4(0, 0, 0, 0);
    s_la[c] = (s_ca[c] >= 0 && d.Xc) ? x_lut(d, s_ca[c]) : z;
    s_lb[c] = (s_cb[c] >= 0 && d.Xc) ? x_lut(d, s_cb[c]) : z;
  }
  __syncthreads();
  constexpr int QPC = KC / 4;  // row quads per column and chunk
  const float4 z4 = make_float4(0, 0, 0, 0);
  for (int64_t r0 = 0; r0 < ld; r0 += KC) {
    static_assert((T * QPC) % 256 == 0, "whole loader rounds");
#pragma unroll 4
    for (int k = 0; k < T * QPC / 256; ++k) {
      const int e = t + 256 * k;
      const int c = e / QPC, rq = (e - c * QPC) * 4;
      const int64_t ca = s_ca[c], cb = s_cb[c];
      float4 va, vb;
      if (d.Xc) {  // 2-bit codes: the same f32 values, decoded
        va = ca >= 0 ? x_decode4(d.Xc[code_off(ca, (r0 + rq) >> 2, d.B, d.ldc)], s_la[c]) : z4;
        vb = cb >= 0 ? x_decode4(d.Xc[code_off(cb, (r0 + rq) >> 2, d.B, d.ldc)], s_lb[c]) : z4;
      } else {
        va = ca >= 0 ? *reinterpret_cast<const float4 *>(X + ca * ld + r0 + rq) : z4;
        vb = cb >= 0 ? *reinterpret_cast<const float4 *>(X + cb * ld + r0 + rq) : z4;
      }
      As[rq + 0][c] = va.x; As[rq + 1][c] = va.y; As[rq + 2][c] = va.z; As[rq + 3][c] = va.w;
      Bs[rq + 0][c] = vb.x; Bs[rq + 1][c] = vb.y; Bs[rq + 2][c] = vb.z; Bs[rq + 3][c] = vb.w;
    }
    __syncthreads();
    // v_mfma_f64_16x16x4_f64 over the chunk's rows, 4 per step: lane l supplies A[i = l&15]
    // [k = l>>4] = x(col i)[row k] and B[k][j = l&15] = x(col j)[row k] (f32 values, exact in
    // f64); the products are exact and accumulated in f64
#pragma unroll 2
    for (int kb = 0; kb < KC; kb += 4) {  // (KC rows)
      const int k = kb + (lane >> 4);
      double a[NQ], b[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        a[q] = (double)As[k][wi * (T / 2) + q * 16 + (lane & 15)];
        b[q] = (double)Bs[k][wj * (T / 2) + q * 16 + (lane & 15)];
      }
#pragma unroll
      for (int p = 0; p < NQ; ++p)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[p], b[q], acc[p][q], 0, 0, 0);
    }
    __syncthreads();
  }
  double *g = G + (int64_t)gb * B * B;
  double *gt = GT ? GT + (int64_t)gb * B * B : nullptr;
  // C/D map of the f64 MFMA: element r of lane l is (row (l>>4) + 4 r, column l&15) of the tile
#pragma unroll
  for (int p = 0; p < NQ; ++p)
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = ti * T + wi * (T / 2) + p * 16 + (lane >> 4) + 4 * r;
        const int jj = tj * T + wj * (T / 2) + q * 16 + (lane & 15);
        if (i < B && jj < B) {
          const double v = (i < bs && jj < bs2) ? acc[p][q][r] : 0.0;
          g[(int64_t)i * B + jj] = v;
          if (gt) gt[(int64_t)jj * B + i] = v;
        }
      }
}

// ------------------------------------------------------------------------------------
// Value classes of a column ("integer Gram"): the distinct values of its N rows,
// ascending, with their row counts, when there are at most 4 -- genotype columns in either storage
// (2-bit: the table values of the codes that occur; f32: the values themselves, so both storages
// give the same classes).  Rejected (cls_info = 0): more than 4 values, or nonzero values whose
// binary exponents span more than 20 (k_gram_int sums exactly in 128 bits).  flags[0] |= 1 for a
// rejected column, flags[1] = max ncls.
__device__ __forceinline__ int f32_key(float v) {  // order-preserving int of a float (+0 for -0)
  const int b = __float_as_int(v == 0.f ? 0.f : v);
  return b >= 0 ? b : b ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float key_f32(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF); }

__global__ __launch_bounds__(256) void k_classes(Dev d, int *flags) {
  const int64_t j = blockIdx.x;
  const int t = threadIdx.x;
  __shared__ int s_key[5], s_cnt[4], s_n, s_over, s_min;
  float lv[4] = {0.f, 0.f, 0.f, 0.f};  // this thread's distinct values and their rows
  int lc[4] = {0, 0, 0, 0};
  int ln = 0;
  bool over = false;
  if (d.Xc) {
    // the codes' row counts; each code is one value of the column's table
    for (int64_t g = t; 4 * g < d.N; g += 256) {
      const uint32_t b = d.Xc[code_off(j, g, d.B, d.ldc)];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t cd = (b >> (2 * k)) & 3u;
        const int in = 4 * g + k < d.N;
#pragma unroll
        for (int q = 0; q < 4; ++q) lc[q] += (cd == (uint32_t)q) ? in : 0;
      }
    }
    const float4 l = x_lut(d, j);
    lv[0] = l.x; lv[1] = l.y; lv[2] = l.z; lv[3] = l.w;
    ln = 4;  // (codes that never occur have no rows and are skipped below)
  } else {
    const float *x = d.X + j * d.ld;
    for (int64_t i = t; i < d.N; i += 256) {
      const float v = x[i] == 0.f ? 0.f : x[i];
      int k = -1;
#pragma unroll
      for (int q = 0; q < 4; ++q) k = (q < ln && lv[q] == v) ? q : k;
      if (k >= 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) lc[q] += q == k;
      } else if (ln < 4 && v == v) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (q == ln) { lv[q] = v; lc[q] = 1; }
        ++ln;
      } else {
        over = true;  // a fifth value, or NaN
      }
    }
  }
  if (t == 0) { s_n = 0; s_over = 0; }
  if (t < 4) s_cnt[t] = 0;
  __syncthreads();
  if (over) s_over = 1;
  // the classes in ascending order: every round adds the smallest value not yet a class
  for (int r = 0; r < 5; ++r) {
    if (t == 0) s_min = 0x7FFFFFFF;
    __syncthreads();
    const int nk = s_n;
    int mine = 0x7FFFFFFF;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= ln || lc[q] == 0) continue;
      const int key = f32_key(lv[q]);
      bool seen = false;
      for (int c = 0; c < nk; ++c) seen |= s_key[c] == key;
      if (!seen) mine = min(mine, key);
    }
    if (mine != 0x7FFFFFFF) atomicMin(&s_min, mine);
    __syncthreads();
    const int m = s_min;
    __syncthreads();
    if (m == 0x7FFFFFFF) break;
    if (t == 0) {
      if (nk < 4) s_key[nk] = m; else s_over = 1;
      s_n = nk + 1;
    }
    __syncthreads();
    if (s_n > 4) break;
  }
  const int nc = min(s_n, 4);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q >= ln || lc[q] == 0) continue;
    const int key = f32_key(lv[q]);
    for (int c = 0; c < nc; ++c)
      if (s_key[c] == key) atomicAdd(&s_cnt[c], lc[q]);
  }
  __syncthreads();
  if (t == 0) {
    bool bad = s_over != 0 || s_n > 4;
    int emin = 1 << 20, emax = -(1 << 20);
    for (int c = 0; c < nc; ++c) {
      const float v = key_f32(s_key[c]);
      if (v != 0.f) {
        int e;
        frexpf(v, &e);
        emin = min(emin, e);
        emax = max(emax, e);
      }
    }
    if (emax - emin > 20) bad = true;
    int cmap = 0;  // 2-bit storage: class of each code (codes without rows: 0)
    if (d.Xc && !bad) {
      const float4 l = x_lut(d, j);
      const float tv[4] = {l.x, l.y, l.z, l.w};
      for (int k = 0; k < 4; ++k)
        for (int c = 0; c < nc; ++c)
          if (s_key[c] == f32_key(tv[k])) cmap |= c << (2 * k);
    }
    d.cls_info[j] = bad ? 0 : (nc | cmap << 8);
    for (int c = 0; c < 4; ++c) {
      d.cls_val[4 * j + c] = (!bad && c < nc) ? key_f32(s_key[c]) : 0.f;
      d.cls_cnt[4 * j + c] = (!bad && c < nc) ? s_cnt[c] : 0;
    }
    if (bad) atomicOr(flags, 1);
    atomicMax(flags + 1, bad ? 0 : nc);
  }
}

// Class codes of the current Gram layout (k_gram_int's input): byte of (block position b, in-block
// index i, row quad g) at code_off(b B + i, g) of Xk = the classes (2 bits per row) of the 4 rows of
// column member[b B + i] -- the column's value classes looked up from its 2-bit codes or found by
// comparing its f32 values with the class values.  A block's columns are then 16-B groups in row
// order whatever columns the visit order put in it (REFERENCE order re-encodes every sweep).
// Thread: (position group of 16, row quad); 16 columns' classes written as one 16-B store.
__global__ __launch_bounds__(256) void k_encode_layout(Dev d, uint8_t *Xk) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int ng = d.B / 16;
  for (int64_t bq = blockIdx.y; bq < (int64_t)d.nb * ng; bq += gridDim.y) {
    if (g >= d.ldc) return;
    const int b = (int)(bq / ng), q = (int)(bq % ng);
    const int bs = d.bsz[b];
    uint32_t out[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int pos = 16 * q + i;
      uint32_t byte = 0;
      if (pos < bs && 4 * g < d.N) {
        const int64_t col = d.member[(int64_t)b * d.B + pos];
        const int info = d.cls_info[col];
        if (d.Xc) {
          const uint32_t c = d.Xc[code_off(col, g, d.B, d.ldc)];
#pragma unroll
          for (int k = 0; k < 4; ++k) byte |= (((uint32_t)info >> (8 + 2 * ((c >> (2 * k)) & 3u))) & 3u) << (2 * k);
        } else {
          const float4 x = *reinterpret_cast<const float4 *>(d.X + col * d.ld + 4 * g);
          const int nc = info & 7;
          const float *v = d.cls_val + 4 * col;
          const float v1 = v[1], v2 = v[2], v3 = v[3];
          auto cl = [&](float xv) -> uint32_t {
            return (nc > 1 && xv == v1) ? 1u : (nc > 2 && xv == v2) ? 2u : (nc > 3 && xv == v3) ? 3u : 0u;
          };
          byte = cl(x.x) | cl(x.y) << 2 | cl(x.z) << 4 | cl(x.w) << 6;
        }
      }
      out[i >> 2] |= byte << (8 * (i & 3));
    }
    *reinterpret_cast<uint4 *>(Xk + (bq * d.ldc + g) * 16) = make_uint4(out[0], out[1], out[2], out[3]);
  }
}

// REFERENCE order: every column's class codes once, column-major (ldc bytes per column, the classes of
// rows 4g .. 4g+3 in byte g, PLINK packing), so that each sweep's layout encoding is a gather of
// contiguous bytes (k_encode_gather) instead of a pass over X (f32: 4 N P bytes) or over the 2-bit
// tiles (16-B granules, one useful byte each).  Rows beyond N: class 0 (k_gram_int masks them).
__global__ __launch_bounds__(256) void k_xcls(Dev d, uint8_t *xcls) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= d.ldc) return;
  for (int64_t col = blockIdx.y; col < d.M; col += gridDim.y) {
    const int info = d.cls_info[col];
    uint32_t byte = 0;
    if (4 * g < d.N) {
      if (d.Xc) {
        const uint32_t c = d.Xc[code_off(col, g, d.B, d.ldc)];
#pragma unroll
        for (int k = 0; k < 4; ++k) byte |= (((uint32_t)info >> (8 + 2 * ((c >> (2 * k)) & 3u))) & 3u) << (2 * k);
      } else {
        const float4 x = *reinterpret_cast<const float4 *>(d.X + col * d.ld + 4 * g);
        const int nc = info & 7;
        const float *v = d.cls_val + 4 * col;
        const float v1 = v[1], v2 = v[2], v3 = v[3];
        auto cl = [&](float xv) -> uint32_t {
          return (nc > 1 && xv == v1) ? 1u : (nc > 2 && xv == v2) ? 2u : (nc > 3 && xv == v3) ? 3u : 0u;
        };
        byte = cl(x.x) | cl(x.y) << 2 | cl(x.z) << 4 | cl(x.w) << 6;
      }
    }
    xcls[col * d.ldc + g] = (uint8_t)byte;
  }
}

// The layout's class codes gathered from the column-major codes (k_xcls): thread = (16-position group q
// of block b, 4 consecutive row quads); per position one 4-byte load (a wave reads 256 contiguous bytes
// of a column), then the 16 positions' bytes of each quad as one 16-B store.  Same bytes as
// k_encode_layout.
__global__ __launch_bounds__(256) void k_encode_gather(Dev d, const uint8_t *xcls, uint8_t *Xk) {
  const int64_t g0 = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  const int ng = d.B / 16;
  if (g0 >= d.ldc) return;
  for (int64_t bq = blockIdx.y; bq < (int64_t)d.nb * ng; bq += gridDim.y) {
    const int b = (int)(bq / ng), q = (int)(bq % ng);
    const int bs = d.bsz[b];
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int pos = 16 * q + i;
      w[i] = pos < bs ? *reinterpret_cast<const uint32_t *>(xcls + (int64_t)d.member[(int64_t)b * d.B + pos] * d.ldc + g0)
                      : 0u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = ((w[4 * j] >> (8 * k)) & 0xFFu) | ((w[4 * j + 1] >> (8 * k)) & 0xFFu) << 8 |
               ((w[4 * j + 2] >> (8 * k)) & 0xFFu) << 16 | ((w[4 * j + 3] >> (8 * k)) & 0xFFu) << 24;
      *reinterpret_cast<uint4 *>(Xk + (bq * d.ldc + g0 + k) * 16) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}

// Exact integer Gram of class-coded columns on the i8 matrix cores.  For columns i, j with class
// values u_a, w_b and n_ab = #rows where column i is in class a and column j in class b,
//     G_ij = sum_ab n_ab u_a w_b
// exactly: the NP x NP explicit counts are I_a^T I_b of 0/1 class indicator bytes
// (v_mfma_i32_16x16x64_i8 over the rows, int32 accumulation is exact), the counts of the last
// class follow from the per-column class totals, and the sum of the (NP+1)^2 integer multiples of
// u_a w_b (each a 24-bit x 24-bit mantissa product times a power of two) is formed in a 128-bit
// integer and rounded once -- the correctly rounded dot product of the f32 columns, in either
// storage, in any order (symmetric on the diagonal blocks).  GI_T x GI_T output columns per
// workgroup of 4 waves, each wave a quadrant of the (NP GI_T)^2 count matrix.  Input: the layout's
// class codes (k_encode_layout), GI_KC-row chunks read as 16-B groups (16 columns x 4 rows) GI_D
// chunks ahead in registers (a ring unrolled by its depth: each chunk waits for its own loads only),
// expanded to indicator planes in LDS as [side][plane][column][row] bytes (pitch GI_KC + 16: the 16-B
// operand reads of 16 consecutive columns hit 16 distinct 4-bank groups).
constexpr int GI_T = 64;
constexpr int GI_KC = 256;
constexpr int GI_D = 4;
constexpr int GI_PITCH = GI_KC + 16;
__host__ __device__ constexpr size_t gram_int_lds(int NP) {
  return (size_t)2 * NP * GI_T * GI_PITCH > (size_t)NP * GI_T * NP * GI_T * 4 ? (size_t)2 * NP * GI_T * GI_PITCH
                                                                             : (size_t)NP * GI_T * NP * GI_T * 4;
}
typedef int i32x4 __attribute__((ext_vector_type(4)));

// (NP <= 2, the genotype case: two workgroups per CU -- 8 waves, one's class-plane expansion beside
// the other's matrix-core products; the register budget of two waves per SIMD)
template <int NP>
__global__ __launch_bounds__(256, NP <= 2 ? 2 : 1) void k_gram_int(Dev d, const uint8_t *Xk, const int *member, const int *bsz, int B,
                                                  int nb, int shift, double *G, double *GT) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  uint8_t *stg = reinterpret_cast<uint8_t *>(gsm);  // the k loop's indicator planes
  int *cntm = reinterpret_cast<int *>(gsm);         // then the count matrix [NP GI_T][NP GI_T]
  __shared__ int s_emin[2][GI_T];
  __shared__ uint32_t s_cv[2][GI_T / 16];  // column-group validity: bit i = column 16 q + i exists
  __shared__ int s_h[2][GI_T][4], s_M[2][GI_T][4], s_E[2][GI_T][4];
  const int gb = blockIdx.x, gb2 = (gb + shift) % nb;
  const int ntile = B / GI_T;
  int ti = blockIdx.y / ntile, tj = blockIdx.y % ntile;
  const bool mirror = shift == 0 && GT == nullptr;  // a diagonal block: the tiles on and above its diagonal
  if (mirror) {
    int y = blockIdx.y;
    ti = 0;
    while (y >= ntile - ti) { y -= ntile - ti; ++ti; }
    tj = ti + y;
  }
  const int bs = bsz[gb], bs2 = bsz[gb2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, wi = wv >> 1, wj = wv & 1;
  const int64_t N = d.N, nq = d.ldc;
  if (t < 2 * GI_T / 16) s_cv[t / (GI_T / 16)][t % (GI_T / 16)] = 0u;
  __syncthreads();
  if (t < 2 * GI_T) {
    // this tile's columns: class tables, each class value as M 2^(E + emin) with M a 24-bit integer
    const int side = t / GI_T, c = t % GI_T;
    const int idx = (side ? tj : ti) * GI_T + c;
    const int64_t col = idx < (side ? bs2 : bs) ? member[(int64_t)(side ? gb2 : gb) * B + idx] : -1;
    const int nc = col >= 0 ? d.cls_info[col] & 7 : 0;
    if (col >= 0) atomicOr(&s_cv[side][c / 16], 1u << (c % 16));
    int emin = 1 << 20, E[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool in = col >= 0 && k < nc;
      const float v = in ? d.cls_val[4 * col + k] : 0.f;
      s_h[side][c][k] = in ? d.cls_cnt[4 * col + k] : 0;
      int e = 0;
      const float f = frexpf(v, &e);  // v = f 2^e, f in [0.5, 1)
      s_M[side][c][k] = v != 0.f ? (int)(f * 16777216.0f) : 0;
      E[k] = e - 24;
      if (v != 0.f) emin = min(emin, E[k]);
    }
    if (emin == (1 << 20)) emin = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) s_E[side][c][k] = s_M[side][c][k] != 0 ? E[k] - emin : 0;
    s_emin[side][c] = emin;
  }
  __syncthreads();
  constexpr int W = NP * GI_T;  // count matrix rows (plane a, column i) = a GI_T + i; columns likewise
  constexpr int NQ = W / 2 / 16;  // 16 x 16 count tiles per wave and dimension
  i32x4 acc[NQ][NQ];
#pragma unroll
  for (int p = 0; p < NQ; ++p)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[p][q] = i32x4{0, 0, 0, 0};
  // loader elements (side, column group q, row quad g), g fastest: one 16-B group of codes each
  constexpr int QPC = GI_KC / 4;                   // row quads per chunk
  constexpr int EPT = 2 * (GI_T / 16) * QPC / 256;  // elements per thread and chunk
  static_assert(EPT * 256 == 2 * (GI_T / 16) * QPC, "whole loader rounds");
  const int64_t nch = (N + GI_KC - 1) / GI_KC;
  const uint4 *src[EPT];
  int e_side[EPT], e_q[EPT], e_g[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = t + 256 * k;
    e_g[k] = e % QPC;
    e_q[k] = (e / QPC) % (GI_T / 16);
    e_side[k] = e / (QPC * (GI_T / 16));
    const int64_t grp = (int64_t)(e_side[k] ? gb2 : gb) * (B / 16) + (e_side[k] ? tj : ti) * (GI_T / 16) + e_q[k];
    src[k] = reinterpret_cast<const uint4 *>(Xk) + grp * nq + e_g[k];
  }
  auto load = [&](int64_t ch, uint4 (&r)[EPT]) __attribute__((always_inline)) {
    const int64_t c = ch < nch ? ch : nch - 1;  // (clamped: an unconditional load per slot)
#pragma unroll
    for (int k = 0; k < EPT; ++k) r[k] = src[k][min(c * QPC + e_g[k], nq - 1) - e_g[k]];
  };
  uint4 ring[GI_D][EPT];
#pragma unroll
  for (int u = 0; u < GI_D; ++u) load(u, ring[u]);
  for (int64_t c0 = 0; c0 < nch; c0 += GI_D) {
#pragma unroll
    for (int u = 0; u < GI_D; ++u) {
      const int64_t ch = c0 + u;
      if (ch >= nch) break;
      // expand: per column of the group, 4 rows' classes -> one 0/1 byte per row and plane.  Four
      // columns at a time (a code word: byte = column, 2-bit field k = row k): the fields equal to
      // class p are ~(w ^ p 0x55555555) with both bits set, kept as bit 2k of the column's byte; the
      // bits 0, 2, 4, 6 of a byte y spread to bytes 0..3 as (y * 0x41041) & 0x01010101 (the partial
      // products' other bits never carry into bits 0, 8, 16, 24)
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int64_t row4 = ch * GI_KC + 4 * e_g[k];
        // valid rows of this quad as bits 0, 2, 4, 6 (row k: bit 2 k)
        const uint32_t vrow = row4 >= N ? 0u : row4 + 4 <= N ? 0x55u : (0x55u >> (2 * (int)(4 - (N - row4))));
        const uint32_t cv = s_cv[e_side[k]][e_q[k]];
        const uint32_t wd[4] = {ring[u][k].x, ring[u][k].y, ring[u][k].z, ring[u][k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // column validity (bytes) of columns 4 j .. 4 j + 3, times the row validity
          const uint32_t cb = (cv >> (4 * j)) & 0xFu;
          const uint32_t cm = ((cb & 1u) ? 0xFFu : 0u) | ((cb & 2u) ? 0xFF00u : 0u) | ((cb & 4u) ? 0xFF0000u : 0u) |
                              ((cb & 8u) ? 0xFF000000u : 0u);
          const uint32_t m = cm & (vrow * 0x01010101u);
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            const uint32_t eq = ~(wd[j] ^ (0x55555555u * (uint32_t)p));
            const uint32_t ind = eq & (eq >> 1) & m;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const uint32_t y = __builtin_amdgcn_ubfe(ind, 8 * c, 8);
              uint8_t *dst = stg + (e_side[k] * NP * GI_T + 16 * e_q[k] + 4 * j + c) * GI_PITCH + 4 * e_g[k];
              *reinterpret_cast<uint32_t *>(dst + p * GI_T * GI_PITCH) = (y * 0x41041u) & 0x01010101u;
            }
          }
        }
      }
      load(ch + GI_D, ring[u]);  // this slot's next chunk, in flight during the products
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < GI_KC / 64; ++kk) {
        i32x4 a[NQ], bb[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int R = wi * (W / 2) + 16 * q, C = wj * (W / 2) + 16 * q;
          a[q] = *reinterpret_cast<const i32x4 *>(stg + ((0 * NP + R / GI_T) * GI_T + R % GI_T + (lane & 15)) * GI_PITCH +
                                                   kk * 64 + 16 * (lane >> 4));
          bb[q] = *reinterpret_cast<const i32x4 *>(stg + ((1 * NP + C / GI_T) * GI_T + C % GI_T + (lane & 15)) * GI_PITCH +
                                                    kk * 64 + 16 * (lane >> 4));
        }
#pragma unroll
        for (int p = 0; p < NQ; ++p)
#pragma unroll
          for (int q = 0; q < NQ; ++q) acc[p][q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[p], bb[q], acc[p][q], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  // C/D map of the 16 x 16 MFMA: element r of lane l is (row 4 (l >> 4) + r, column l & 15)
#pragma unroll
  for (int p = 0; p < NQ; ++p)
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cntm[(wi * (W / 2) + 16 * p + 4 * (lane >> 4) + r) * W + wj * (W / 2) + 16 * q + (lane & 15)] = acc[p][q][r];
  __syncthreads();
  double *g = G + (int64_t)gb * B * B;
  double *gt = GT ? GT + (int64_t)gb * B * B : nullptr;
  for (int e = t; e < GI_T * GI_T; e += 256) {
    const int i = e / GI_T, j = e % GI_T;
    const int ii = ti * GI_T + i, jj = tj * GI_T + j;
    double v = 0.0;
    if (ii < bs && jj < bs2) {
      int64_t n[NP + 1][NP + 1];
      int64_t hi = 0;
#pragma unroll
      for (int a = 0; a < NP; ++a) {
        int64_t sa = 0;
#pragma unroll
        for (int b = 0; b < NP; ++b) {
          n[a][b] = cntm[(a * GI_T + i) * W + b * GI_T + j];
          sa += n[a][b];
        }
        n[a][NP] = s_h[0][i][a] - sa;  // column j in the last class
        hi += s_h[0][i][a];
      }
      int64_t sl = 0;
#pragma unroll
      for (int b = 0; b < NP; ++b) {
        int64_t sb = 0;
#pragma unroll
        for (int a = 0; a < NP; ++a) sb += n[a][b];
        n[NP][b] = s_h[1][j][b] - sb;  // column i in the last class
        sl += n[NP][b];
      }
      n[NP][NP] = (N - hi) - sl;
      __int128 s = 0;
#pragma unroll
      for (int a = 0; a <= NP; ++a)
#pragma unroll
        for (int b = 0; b <= NP; ++b) {
          const int64_t m = (int64_t)s_M[0][i][a] * s_M[1][j][b];
          if (n[a][b] != 0 && m != 0)
            s += (__int128)n[a][b] * m * ((__int128)1 << (s_E[0][i][a] + s_E[1][j][b]));
        }
      v = ldexp((double)s, s_emin[0][i] + s_emin[1][j]);
    }
    g[(int64_t)ii * B + jj] = v;
    if (gt) gt[(int64_t)jj * B + ii] = v;
    // (a diagonal block's tile below its diagonal: the mirror -- the same correctly rounded dot products)
    if (mirror && ti != tj) g[(int64_t)jj * B + ii] = v;
  }
}

// The class-pair sum of one Gram entry from its explicit counts n[a][b] (a, b < NP), exactly as
// k_gram_int forms it: the last class's counts from the per-column class totals, the (NP + 1)^2
// integer multiples of u_a w_b summed in 128 bits, rounded once.
template <int NP>
__device__ __forceinline__ double gram_entry(const int64_t (&ne)[NP][NP], const int *h0, const int *h1, const int *M0,
                                             const int *M1, const int *E0, const int *E1, int emin0, int emin1, int64_t N) {
  int64_t n[NP + 1][NP + 1];
  int64_t hi = 0;
#pragma unroll
  for (int a = 0; a < NP; ++a) {
    int64_t sa = 0;
#pragma unroll
    for (int b = 0; b < NP; ++b) {
      n[a][b] = ne[a][b];
      sa += n[a][b];
    }
    n[a][NP] = h0[a] - sa;
    hi += h0[a];
  }
  int64_t sl = 0;
#pragma unroll
  for (int b = 0; b < NP; ++b) {
    int64_t sb = 0;
#pragma unroll
    for (int a = 0; a < NP; ++a) sb += n[a][b];
    n[NP][b] = h1[b] - sb;
    sl += n[NP][b];
  }
  n[NP][NP] = (N - hi) - sl;
  __int128 s = 0;
#pragma unroll
  for (int a = 0; a <= NP; ++a)
#pragma unroll
    for (int b = 0; b <= NP; ++b) {
      const int64_t m = (int64_t)M0[a] * M1[b];
      if (n[a][b] != 0 && m != 0) s += (__int128)n[a][b] * m * ((__int128)1 << (E0[a] + E1[b]));
    }
  return ldexp((double)s, emin0 + emin1);
}

// k_gram_int with whole 128-column tiles (NP <= 2, the genotype case; B a multiple of 128): one
// workgroup of 8 waves per GB_T x GB_T output tile, wave w the output rows 32 (w >> 1) .. + 31 and
// columns 64 (w & 1) .. + 63 with EVERY plane pair of them in its accumulators (NP^2 x 2 x 4 MFMA
// tiles), so the epilogue forms G from registers (no count matrix in LDS), and a tile whose two sides
// are the same columns (a diagonal block's diagonal tiles: every block of a B = 128 Gram set) expands
// its codes once.  The indicator planes are double-buffered by chunks of GB_KC rows: chunk c + 1 is
// expanded while chunk c's products run, one barrier per chunk.  Against k_gram_int's 64-column tiles
// the class-plane expansion -- which bounded it, not the matrix cores -- falls to a third (diagonal
// blocks) or a half (cross blocks) per MFMA and overlaps the products.  The counts and the exact sums
// are the same: the blocks are bit-identical (the correctly rounded dot products, tests/test_gpu_gram.py).
constexpr int GB_T = 128;
constexpr int GB_KC = 128;
#ifndef BRR_GB_D
#define BRR_GB_D 4
#endif
constexpr int GB_D = BRR_GB_D;
constexpr int GB_PITCH = GB_KC + 16;
__host__ __device__ constexpr size_t gram_blk_buf(int NP) { return (size_t)2 * NP * GB_T * GB_PITCH; }
__host__ __device__ constexpr size_t gram_blk_lds(int NP) { return 2 * gram_blk_buf(NP); }

template <int NP>
__global__ __launch_bounds__(512, 1) void k_gram_blk(Dev d, const uint8_t *Xk, const int *member, const int *bsz, int B,
                                                     int nb, int shift, double *G, double *GT) {
  static_assert(NP >= 1 && NP <= 2, "whole-tile accumulators for at most 2 explicit planes");
  constexpr int NC = NP + 1;  // classes
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  uint8_t *stg = reinterpret_cast<uint8_t *>(gsm);  // [buffer][side][plane][column][row] indicator bytes
  __shared__ int s_emin[2][GB_T];
  __shared__ uint32_t s_cv[2][GB_T / 16];
  __shared__ int s_h[2][GB_T][NC], s_M[2][GB_T][NC], s_E[2][GB_T][NC];
  const int gb = blockIdx.x, gb2 = (gb + shift) % nb;
  const int ntile = B / GB_T;
  int ti = blockIdx.y / ntile, tj = blockIdx.y % ntile;
  const bool mirror = shift == 0 && GT == nullptr;
  if (mirror) {
    int y = blockIdx.y;
    ti = 0;
    while (y >= ntile - ti) { y -= ntile - ti; ++ti; }
    tj = ti + y;
  }
  const bool same = gb2 == gb && ti == tj;  // both sides the same columns: one expansion
  const int bs = bsz[gb], bs2 = bsz[gb2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, wi = wv >> 1, wj = wv & 1;
  const int64_t N = d.N, nq = d.ldc;
  if (t < 2 * GB_T / 16) s_cv[t / (GB_T / 16)][t % (GB_T / 16)] = 0u;
  __syncthreads();
  if (t < 2 * GB_T) {
    const int side = t / GB_T, c = t % GB_T;
    const int idx = (side ? tj : ti) * GB_T + c;
    const int64_t col = idx < (side ? bs2 : bs) ? member[(int64_t)(side ? gb2 : gb) * B + idx] : -1;
    const int nc = col >= 0 ? d.cls_info[col] & 7 : 0;  // (<= NC: d.gram_np is the cohort's most explicit planes)
    if (col >= 0) atomicOr(&s_cv[side][c / 16], 1u << (c % 16));
    int emin = 1 << 20, E[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const bool in = col >= 0 && k < nc;
      const float v = in ? d.cls_val[4 * col + k] : 0.f;
      s_h[side][c][k] = in ? d.cls_cnt[4 * col + k] : 0;
      int e = 0;
      const float f = frexpf(v, &e);
      s_M[side][c][k] = v != 0.f ? (int)(f * 16777216.0f) : 0;
      E[k] = e - 24;
      if (v != 0.f) emin = min(emin, E[k]);
    }
    if (emin == (1 << 20)) emin = 0;
#pragma unroll
    for (int k = 0; k < NC; ++k) s_E[side][c][k] = s_M[side][c][k] != 0 ? E[k] - emin : 0;
    s_emin[side][c] = emin;
  }
  i32x4 acc[NP][NP][2][4];
#pragma unroll
  for (int a = 0; a < NP; ++a)
#pragma unroll
    for (int b = 0; b < NP; ++b)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[a][b][x][y] = i32x4{0, 0, 0, 0};
  // loader: per chunk of GB_KC rows, thread t the 16-B code group (side t >> 8, column group (t >> 5) & 7,
  // row quad t & 31); side-1 threads idle when both sides are the same columns
  constexpr int QPC = GB_KC / 4;
  static_assert(2 * (GB_T / 16) * QPC == 512, "one element per thread and chunk");
  const int eside = t >> 8, eq = (t >> 5) & 7, eg = t & 31;
  const bool eon = !(same && eside == 1);
  const int64_t nch = (N + GB_KC - 1) / GB_KC;
  // (side-1 threads of a same-columns tile load side 0's groups and skip the expansion: no load under a
  // branch, which would make the compiler drain the ring at the join -- see k_gram_fp4)
  const int lside = same ? 0 : eside;
  const uint4 *src = reinterpret_cast<const uint4 *>(Xk) +
                     ((int64_t)(lside ? gb2 : gb) * (B / 16) + (lside ? tj : ti) * (GB_T / 16) + eq) * nq;
  auto load = [&](int64_t ch) __attribute__((always_inline)) -> uint4 {
    const int64_t c = ch < nch ? ch : nch - 1;
    return src[min(c * QPC + eg, nq - 1)];
  };
  // expand (k_gram_int's bit spread) chunk ch's group into buffer bf: column 16 eq + 4 j + c, rows 4 eg .. 4 eg + 3
  auto expand = [&](const uint4 &v, int64_t ch, uint8_t *bf) __attribute__((always_inline)) {
    if (!eon) return;
    const int64_t row4 = ch * GB_KC + 4 * eg;
    const uint32_t vrow = row4 >= N ? 0u : row4 + 4 <= N ? 0x55u : (0x55u >> (2 * (int)(4 - (N - row4))));
    const uint32_t cv = s_cv[eside][eq];
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
    uint8_t *base = bf + ((eside * NP) * GB_T + 16 * eq) * GB_PITCH + 4 * eg;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t cb = (cv >> (4 * j)) & 0xFu;
      const uint32_t cm = ((cb & 1u) ? 0xFFu : 0u) | ((cb & 2u) ? 0xFF00u : 0u) | ((cb & 4u) ? 0xFF0000u : 0u) |
                          ((cb & 8u) ? 0xFF000000u : 0u);
      const uint32_t m = cm & (vrow * 0x01010101u);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const uint32_t e = ~(wd[j] ^ (0x55555555u * (uint32_t)p));
        const uint32_t ind = e & (e >> 1) & m;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t y = __builtin_amdgcn_ubfe(ind, 8 * c, 8);
          *reinterpret_cast<uint32_t *>(base + (p * GB_T + 4 * j + c) * GB_PITCH) = (y * 0x41041u) & 0x01010101u;
        }
      }
    }
  };
  uint4 ring[GB_D];  // ring[k]: the chunk of index = k (mod GB_D) next to be expanded
#pragma unroll
  for (int u = 0; u < GB_D; ++u) ring[u] = load(u);
  __syncthreads();  // (the class tables, s_cv)
  expand(ring[0], 0, stg);
  ring[0] = load(GB_D);
  __syncthreads();
  for (int64_t c0 = 0; c0 < nch; c0 += GB_D) {
#pragma unroll
    for (int u = 0; u < GB_D; ++u) {
      const int64_t ch = c0 + u;
      if (ch >= nch) break;
      // chunk ch + 1 into the other buffer (its last readers passed the barrier that ended chunk ch - 1)
      // chunk ch + 1 (clamped: past the last chunk the other buffer is written and never read)
      expand(ring[(u + 1) % GB_D], ch + 1, stg + ((ch + 1) & 1) * gram_blk_buf(NP));
      ring[(u + 1) % GB_D] = load(ch + 1 + GB_D);
      const uint8_t *sa = stg + (ch & 1) * gram_blk_buf(NP);
      const uint8_t *sb = same ? sa : sa + (size_t)NP * GB_T * GB_PITCH;
#pragma unroll
      for (int kk = 0; kk < GB_KC / 64; ++kk) {
        i32x4 fa[NP][2], fb[NP][4];
        const int ko = kk * 64 + 16 * (lane >> 4);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
          for (int x = 0; x < 2; ++x)
            fa[p][x] = *reinterpret_cast<const i32x4 *>(sa + (p * GB_T + 32 * wi + 16 * x + (lane & 15)) * GB_PITCH + ko);
#pragma unroll
          for (int y = 0; y < 4; ++y)
            fb[p][y] = *reinterpret_cast<const i32x4 *>(sb + (p * GB_T + 64 * wj + 16 * y + (lane & 15)) * GB_PITCH + ko);
        }
#pragma unroll
        for (int a = 0; a < NP; ++a)
#pragma unroll
          for (int b = 0; b < NP; ++b)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
              for (int y = 0; y < 4; ++y)
                acc[a][b][x][y] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[a][x], fb[b][y], acc[a][b][x][y], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  // epilogue from the accumulators: element r of lane l of a 16 x 16 tile is (row 4 (l >> 4) + r, column l & 15)
  double *g = G + (int64_t)gb * B * B;
  double *gt = GT ? GT + (int64_t)gb * B * B : nullptr;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 32 * wi + 16 * x + 4 * (lane >> 4) + r, j = 64 * wj + 16 * y + (lane & 15);
        const int ii = ti * GB_T + i, jj = tj * GB_T + j;
        int64_t ne[NP][NP];
#pragma unroll
        for (int a = 0; a < NP; ++a)
#pragma unroll
          for (int b = 0; b < NP; ++b) ne[a][b] = acc[a][b][x][y][r];
        // (entries past a short block's columns: 0, as k_gram_int writes them)
        const double v = (ii < bs && jj < bs2) ? gram_entry<NP>(ne, s_h[0][i], s_h[1][j], s_M[0][i], s_M[1][j], s_E[0][i],
                                                                s_E[1][j], s_emin[0][i], s_emin[1][j], N)
                                               : 0.0;
        g[(int64_t)ii * B + jj] = v;
        if (gt) gt[(int64_t)jj * B + ii] = v;
        if (mirror && ti != tj) g[(int64_t)jj * B + ii] = v;
      }
}

// REFERENCE order (Dev::xcls, the column-major class codes, present) with at most 3 classes per column:
// the same exact Gram blocks from fp4 planes on the block-scaled matrix cores, read straight from the
// column-major codes (no per-sweep layout encoding, k_encode_gather).  Per column two planes of e2m1
// values, the class code c (0, 1, 2) and c^2 (0, 1, 4) -- one plane c for 2 classes -- so the four plane
// products S_pq = sum_rows c^p c'^q (p, q = 1, 2) are V n V^T with V = [[1, 2], [1, 4]] and n the class-pair
// counts of classes 1 and 2 (invertible: 4 n is integer arithmetic on S); class 0 follows from the totals
// (gram_entry's last class, the class tables stored in the order 1, 2, 0).  The f32 accumulators are exact
// while 16 N < 2^24 (every product is an integer <= 16).  v_mfma_scale_f32_16x16x128_f8f6f4, unit scales:
// twice the i8 form's K per instruction at the same cycles and half its operand bytes; lane l's operand is
// row (column) l & 15, K = 32 (l >> 4) .. + 31 as 16 bytes, element 2q in the low nibble of byte q
// (scripts/mb_fp4_layout.hip).  A thread expands 64 rows of one column (16 code bytes) into 32 bytes per
// plane, two 16-B LDS stores each.  Tiles, waves and the epilogue as k_gram_blk.
constexpr int GF_KC = 256;               // rows per chunk
constexpr int GF_PITCH = GF_KC / 2;      // bytes per column and plane (nibbles)
// 16-B slot c of LDS row R at slot c ^ ((R >> 1) & 7) ^ (R & 1): the MFMA operand reads (ds_read_b128, lane l
// row R = 16 m + (l & 15), slot 4 kk + (l >> 4)) are conflict-free in each of the instruction's 16-lane
// groups (MI355X_MICROARCH.md LDS: groups {0-3, 12-15, 20-27}, ...; with 144-B rows, 2-way:
// SQ_LDS_BANK_CONFLICT 1.2e9 cycles per call, profiles/r06x_gram_fp4_pmc.csv), and so are the expansion's
// 16-B stores (8-lane groups: rows 2m and 2m + 1, slots of opposite parity)
__device__ __forceinline__ int gf_slot(int R, int c) { return (c ^ ((R >> 1) & 7) ^ (R & 1)) << 4; }
__host__ __device__ constexpr size_t gram_fp4_buf(int NP) { return (size_t)2 * NP * GB_T * GF_PITCH; }
__host__ __device__ constexpr size_t gram_fp4_lds(int NP) { return 2 * gram_fp4_buf(NP); }
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// 8 rows' 2-bit class codes (16 bits) -> 8 nibbles, each code in the low two bits of its nibble
__device__ __forceinline__ uint32_t spread2to4(uint32_t h) {
  uint32_t x = h & 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  return x;
}

template <int NP>
__global__ __launch_bounds__(512, 1) void k_gram_fp4(Dev d, const uint8_t *xcls, const int *member, const int *bsz, int B,
                                                     int nb, int shift, double *G, double *GT) {
  static_assert(NP >= 1 && NP <= 2, "planes c (and c^2) for at most 3 classes");
  constexpr int NC = NP + 1;
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  uint8_t *stg = reinterpret_cast<uint8_t *>(gsm);  // [buffer][side][plane][column][row nibbles]
  __shared__ int s_emin[2][GB_T];
  __shared__ int s_h[2][GB_T][NC], s_M[2][GB_T][NC], s_E[2][GB_T][NC];  // slot (k + NP) % NC: class k
  __shared__ int64_t s_col[2][GB_T];
  const int gb = blockIdx.x, gb2 = (gb + shift) % nb;
  const int ntile = B / GB_T;
  int ti = blockIdx.y / ntile, tj = blockIdx.y % ntile;
  const bool mirror = shift == 0 && GT == nullptr;
  if (mirror) {
    int y = blockIdx.y;
    ti = 0;
    while (y >= ntile - ti) { y -= ntile - ti; ++ti; }
    tj = ti + y;
  }
  const bool same = gb2 == gb && ti == tj;
  const int bs = bsz[gb], bs2 = bsz[gb2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, wi = wv >> 1, wj = wv & 1;
  const int64_t N = d.N, ldc = d.ldc;
  if (t < 2 * GB_T) {
    const int side = t / GB_T, c = t % GB_T;
    const int idx = (side ? tj : ti) * GB_T + c;
    const int64_t col = idx < (side ? bs2 : bs) ? member[(int64_t)(side ? gb2 : gb) * B + idx] : -1;
    s_col[side][c] = col >= 0 ? col : 0;  // (a missing column reads column 0; its entries are written 0)
    const int nc = col >= 0 ? d.cls_info[col] & 7 : 0;
    int emin = 1 << 20, E[NC], Mv[NC], H[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const bool in = col >= 0 && k < nc;
      const float v = in ? d.cls_val[4 * col + k] : 0.f;
      H[k] = in ? d.cls_cnt[4 * col + k] : 0;
      int e = 0;
      const float f = frexpf(v, &e);
      Mv[k] = v != 0.f ? (int)(f * 16777216.0f) : 0;
      E[k] = e - 24;
      if (v != 0.f) emin = min(emin, E[k]);
    }
    if (emin == (1 << 20)) emin = 0;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int sl = (k + NP) % NC;
      s_h[side][c][sl] = H[k];
      s_M[side][c][sl] = Mv[k];
      s_E[side][c][sl] = Mv[k] != 0 ? E[k] - emin : 0;
    }
    s_emin[side][c] = emin;
  }
  __syncthreads();
  f32x4 acc[NP][NP][2][4];
#pragma unroll
  for (int a = 0; a < NP; ++a)
#pragma unroll
    for (int b = 0; b < NP; ++b)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[a][b][x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  // loader: per chunk and side, thread t the 16 code bytes (64 rows) part t & 3 of column t >> 2
  const int ec = t >> 2, ep = t & 3;
  const int nsd = same ? 1 : 2;
  const int64_t nch = (N + GF_KC - 1) / GF_KC;  // (<= ldc / 64: ld is a multiple of 256)
  // (unconditional loads -- side 1 re-reads side 0's bytes when both are the same columns -- and no load
  // under a branch: a load on one path of a branch makes the compiler drain every load at the join,
  // i.e. the whole ring, before each chunk's products)
  const uint4 *src[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) src[k] = reinterpret_cast<const uint4 *>(xcls + s_col[same ? 0 : k][ec] * ldc) + ep;
  auto load = [&](int64_t ch, uint4 (&r)[2]) __attribute__((always_inline)) {
    const int64_t c = (ch < nch ? ch : nch - 1) * (GF_KC / 64);
    r[0] = src[0][c];
    r[1] = src[1][c];
  };
  auto expand = [&](const uint4 (&v)[2], uint8_t *bf) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k >= nsd) break;
      const uint32_t wd[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
      uint32_t pc[8], pq[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t lo = spread2to4(wd[q]), hi = spread2to4(wd[q] >> 16);
        pc[2 * q] = lo << 1;
        pc[2 * q + 1] = hi << 1;
        pq[2 * q] = (lo << 1) | (lo & 0x22222222u);  // c^2: 2 -> 0110 (4.0), 1 -> 0010 (1.0)
        pq[2 * q + 1] = (hi << 1) | (hi & 0x22222222u);
      }
      // slots 2 ep and 2 ep + 1 of row ec
      uint8_t *row = bf + ((k * NP) * GB_T + ec) * GF_PITCH;
      uint8_t *d0 = row + gf_slot(ec, 2 * ep), *d1 = row + gf_slot(ec, 2 * ep + 1);
      *reinterpret_cast<uint4 *>(d0) = make_uint4(pc[0], pc[1], pc[2], pc[3]);
      *reinterpret_cast<uint4 *>(d1) = make_uint4(pc[4], pc[5], pc[6], pc[7]);
      if (NP == 2) {
        *reinterpret_cast<uint4 *>(d0 + GB_T * GF_PITCH) = make_uint4(pq[0], pq[1], pq[2], pq[3]);
        *reinterpret_cast<uint4 *>(d1 + GB_T * GF_PITCH) = make_uint4(pq[4], pq[5], pq[6], pq[7]);
      }
    }
  };
  uint4 ring[GB_D][2];
#pragma unroll
  for (int u = 0; u < GB_D; ++u) load(u, ring[u]);
  expand(ring[0], stg);
  load(GB_D, ring[0]);
  __syncthreads();
  for (int64_t c0 = 0; c0 < nch; c0 += GB_D) {
#pragma unroll
    for (int u = 0; u < GB_D; ++u) {
      const int64_t ch = c0 + u;
      if (ch >= nch) break;
      // chunk ch + 1 (clamped: past the last chunk the other buffer is written and never read)
      expand(ring[(u + 1) % GB_D], stg + ((ch + 1) & 1) * gram_fp4_buf(NP));
      load(ch + 1 + GB_D, ring[(u + 1) % GB_D]);
      const uint8_t *sa = stg + (ch & 1) * gram_fp4_buf(NP);
      const uint8_t *sb = same ? sa : sa + (size_t)NP * GB_T * GF_PITCH;
#pragma unroll
      for (int kk = 0; kk < GF_KC / 128; ++kk) {
        i32x8 fa[NP][2], fb[NP][4];
        const int ko = gf_slot(lane & 15, 4 * kk + (lane >> 4));  // (row bits 1-3 = those of lane & 15)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
          for (int x = 0; x < 2; ++x) {
            const i32x4 v = *reinterpret_cast<const i32x4 *>(sa + (p * GB_T + 32 * wi + 16 * x + (lane & 15)) * GF_PITCH + ko);
            fa[p][x] = i32x8{v.x, v.y, v.z, v.w, 0, 0, 0, 0};
          }
#pragma unroll
          for (int y = 0; y < 4; ++y) {
            const i32x4 v = *reinterpret_cast<const i32x4 *>(sb + (p * GB_T + 64 * wj + 16 * y + (lane & 15)) * GF_PITCH + ko);
            fb[p][y] = i32x8{v.x, v.y, v.z, v.w, 0, 0, 0, 0};
          }
        }
#pragma unroll
        for (int a = 0; a < NP; ++a)
#pragma unroll
          for (int b = 0; b < NP; ++b)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
              for (int y = 0; y < 4; ++y)
                acc[a][b][x][y] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[a][x], fb[b][y], acc[a][b][x][y], 4, 4, 0,
                                                                                 0x7F7F7F7F, 0, 0x7F7F7F7F);
      }
      __syncthreads();
    }
  }
  double *g = G + (int64_t)gb * B * B;
  double *gt = GT ? GT + (int64_t)gb * B * B : nullptr;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 32 * wi + 16 * x + 4 * (lane >> 4) + r, j = 64 * wj + 16 * y + (lane & 15);
        const int ii = ti * GB_T + i, jj = tj * GB_T + j;
        int64_t ne[NP][NP];
        if constexpr (NP == 1) {
          ne[0][0] = (int64_t)acc[0][0][x][y][r];
        } else {
          // S = V n V^T, V = [[1, 2], [1, 4]]: U = 2 V^-1 S, 4 n = U (2 V^-T)
          const int64_t S11 = (int64_t)acc[0][0][x][y][r], S12 = (int64_t)acc[0][1][x][y][r];
          const int64_t S21 = (int64_t)acc[1][0][x][y][r], S22 = (int64_t)acc[1][1][x][y][r];
          const int64_t U00 = 4 * S11 - 2 * S21, U01 = 4 * S12 - 2 * S22, U10 = S21 - S11, U11 = S22 - S12;
          ne[0][0] = (4 * U00 - 2 * U01) / 4;
          ne[0][1] = (U01 - U00) / 4;
          ne[1][0] = (4 * U10 - 2 * U11) / 4;
          ne[1][1] = (U11 - U10) / 4;
        }
        const double v = (ii < bs && jj < bs2) ? gram_entry<NP>(ne, s_h[0][i], s_h[1][j], s_M[0][i], s_M[1][j], s_E[0][i],
                                                                s_E[1][j], s_emin[0][i], s_emin[1][j], N)
                                               : 0.0;
        g[(int64_t)ii * B + jj] = v;
        if (gt) gt[(int64_t)jj * B + ii] = v;
        if (mirror && ti != tj) g[(int64_t)jj * B + ii] = v;
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

__global__ __launch_bounds__(256) void k_rows(Dev d, int flags, const double *deps_in, const double *eps_in,
                                              int slot_a, int slot_b) {
#pragma clang fp contract(off)
  __shared__ double red[8];
  __shared__ int s_last;
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = row < d.N;
  double e = 0.0;
  if (valid) {
    if (flags & ROW_INIT_Y) e = d.Y[row] - d.sc->mu - 0.0;  // eps = Y - mu - X*beta, beta=0
    else if (flags & ROW_EXCHANGE) e = d.eps_start[row] + deps_in[row];
    else e = (eps_in ? eps_in : d.eps)[row];
  }
  if (flags & ROW_SHIFT) e = (e + d.sc->mu_prev) - d.sc->mu;
  if (flags & ROW_PENDING) {
    // the last one or two blocks' changes (slots slot_a then slot_b; -1 = none), lists padded
    // to a multiple of 16 with neutral entries
    const int64_t rowc = valid ? row : 0;
    for (int k = 0; k < 2; ++k) {
      const int slot = k == 0 ? slot_a : slot_b;
      if (slot < 0) continue;
      const int np = d.pend_n[slot];
      const int *pidx = d.pend_idx + slot * d.pend_stride;
      const double *pbo = d.pend_bo + slot * d.pend_stride, *pbn = d.pend_bn + slot * d.pend_stride;
      for (int p0 = 0; p0 < np; p0 += 8) {
        double x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = (double)x_at(d, pidx[p0 + q], rowc);
#pragma unroll
        for (int q = 0; q < 8; ++q) e = (e + x[q] * pbo[p0 + q]) - x[q] * pbn[p0 + q];
      }
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
  sc->mu = sc->S1 / (double)d.Ntot + sqrt(sc->sigmaE / (double)d.Ntot) * z;  // all rows (row shards: summed S1)
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

// Block order: a rotation of the block cycle, forwards or backwards (Philox draw, entity =
// shard), so consecutive blocks of a sweep are cycle neighbours (cross-Gram precomputed).
__global__ __launch_bounds__(256) void k_perm_blockorder(Dev d, uint32_t it, int shard, int identity) {
  const int64_t nb = d.nb;
  const uint4 w = philox(d.seed, 0, T_PERM_BLOCK, (uint32_t)shard, it);
  const int64_t rot = identity ? 0 : (int64_t)(((uint64_t)w.x * (uint64_t)nb) >> 32);
  const int64_t dir = identity ? 1 : ((w.y & 1u) ? 1 : -1);
  for (int64_t s = threadIdx.x; s < nb; s += blockDim.x) d.blkorder[s] = (int)(((rot + dir * s) % nb + nb) % nb);
}

// The same Fisher-Yates permutation as fisher_yates_dev: the draws do not depend on the swaps, so the
// workgroup forms them in parallel first (step i uses word i & 3 of Philox counter i >> 2) and one
// thread then only swaps in LDS (94 -> ~20 µs per sweep at C2: the Philox rounds were on the serial path)
__global__ void k_perm_within(Dev d, uint32_t it, int identity) {
  __shared__ int w[BMAX];
  __shared__ uint32_t jr[BMAX];
  const int s = blockIdx.x;
  const int b = d.blkorder[s];
  const int size = (int)min((int64_t)d.B, d.M - (int64_t)b * d.B);
  const uint32_t ent = (uint32_t)(d.col_offset / d.B + b);
  for (int i = threadIdx.x; i < size; i += blockDim.x) w[i] = i;
  if (!identity)
    for (int g = threadIdx.x; 4 * g < size; g += blockDim.x) {
      const uint4 r = philox(d.seed, (uint32_t)g, T_PERM_WITHIN, ent, it);
      jr[4 * g] = r.x;
      if (4 * g + 1 < BMAX) jr[4 * g + 1] = r.y;
      if (4 * g + 2 < BMAX) jr[4 * g + 2] = r.z;
      if (4 * g + 3 < BMAX) jr[4 * g + 3] = r.w;
    }
  __syncthreads();
  if (threadIdx.x == 0 && !identity)
    for (int i = size - 1; i >= 1; --i) {
      const int j = (int)(((uint64_t)jr[i] * (uint64_t)(i + 1)) >> 32);
      const int tmp = w[i];
      w[i] = w[j];
      w[j] = tmp;
    }
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
    const double denom_f = (double)(d.Ntot - 1) + (sigmaE / d.sc->sigmaF);
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

// Row shards: fixed effect cf of the sweep in two launches around the cross-shard
// sum of the dot product f . (eps + f alpha) (BayesRv2Groups.cpp:218-224).  Phase 0 forms this
// shard's part (into sc->fx; cf == 0 also draws the sweep's fixed-effect order), phase 1 draws
// alpha from the summed dot (identical on every shard) and updates this shard's residual rows.
// With one shard it performs k_fixed's operations in k_fixed's order.
__global__ __launch_bounds__(1024) void k_fixed_row(Dev d, uint32_t it, int cf, int phase, int perm_on_device) {
#pragma clang fp contract(off)
  __shared__ double red[16];
  __shared__ int ford[1024];
  const int F = d.F;
  if (F > 1024) return;
  if (phase == 0 && cf == 0) {
    if (threadIdx.x == 0) {
      for (int f = 0; f < F; ++f) ford[f] = perm_on_device ? f : d.forder[f];
      if (perm_on_device) fisher_yates_dev(d.seed, ford, F, T_PERM_FIXED, 0, it);
    }
    __syncthreads();
    for (int f = threadIdx.x; f < F; f += 1024) d.forder[f] = ford[f];  // read by the later launches
  } else if (threadIdx.x == 0) {
    ford[cf] = d.forder[cf];
  }
  __syncthreads();
  const int64_t N = d.N;
  const int cur = ford[cf];
  const double *f = d.fixed + (int64_t)cur * N;
  const double ca = d.alpha[cur];
  if (phase == 0) {
    double part = 0.0;
    for (int64_t i = threadIdx.x; i < N; i += 1024) {
      const double yt = d.eps[i] + f[i] * ca;
      part += f[i] * yt;
    }
    const double num_f = block_sum<1024>(part, red);
    if (threadIdx.x == 0) d.sc->fx = num_f;
    return;
  }
  const double num_f = d.sc->fx;
  const double sigmaE = d.sc->sigmaE;
  const double denom_f = (double)(d.Ntot - 1) + (sigmaE / d.sc->sigmaF);
  const double z = normal(d.seed, T_FIXED, (uint32_t)cur, it, 0);
  const double an = num_f / denom_f + sqrt(sigmaE / denom_f) * z;
  for (int64_t i = threadIdx.x; i < N; i += 1024) {
    const double yt = d.eps[i] + f[i] * ca;
    d.eps[i] = yt - f[i] * an;
  }
  if (threadIdx.x == 0) d.alpha[cur] = an;
}

// Row shards: block s's level-2 partial dots (slab2 rows 0 .. NG-1 of ring index s % NPAR)
// summed into row 0, in group order -- the order in which k_solve sums them -- so the value the
// solver reads with NG = 1 after the cross-shard sum is, on one shard, bit-identical to its own.
__global__ void k_slab_total(Dev d, int s) {
#pragma clang fp contract(off)
  double *slab2 = d.slab2 + (s % NPAR) * d.slab2_stride;
  for (int pos = threadIdx.x; pos < d.B; pos += blockDim.x) {
    double acc = 0.0;
    for (int g = 0; g < d.NG; ++g) acc += slab2[(int64_t)g * d.B + pos];
    slab2[pos] = acc;
  }
}

// In-process row-shard group: sum of the members' buffers in rank order, written back to every
// member (one device, or peer-mapped devices).
__global__ __launch_bounds__(256) void k_group_sum(GroupPtrs p, int64_t n) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    double acc = p.ptr[0][i];
    for (int r = 1; r < p.n; ++r) acc += p.ptr[r][i];
    for (int r = 0; r < p.n; ++r) p.ptr[r][i] = acc;
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

__device__ __forceinline__ Decision decide_bayesr(double num, double xsq, double sigmaE, double sigmaG,
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
// Per-position constants of a sweep (k_prep), field-major mc[f * nbB + s * B + i] in visit
// order.  BayesR: p (uniform), z (normal), beta_old, xsq, a_0..a_{K-1}, den_1..den_{K-1} with
//   logL_k(t) = a_k + t / (2 den_k sigmaE),  t = num^2           (BayesRv2.cpp:200-209)
//   a_0 = log pi_0,  a_k = log pi_k - 0.5 log((sigmaG/sigmaE) xsq cVa_k + 1),
//   den_k = xsq + (sigmaE/sigmaG) / cVa_k                          (denom[k-1], :200)
// Horseshoe: z, beta_old, xsq, D = xsq + sigmaE / (tau c2 lambda / (tau lambda + c2))
// (HorseshoeR.cpp:226-234).  sigmaE, sigmaG, pi, tau, c2, lambda are constant during the
// marker loop, and a marker's beta only changes at its own visit.
enum McField : int { MC_P = 0, MC_Z = 1, MC_BO = 2, MC_XSQ = 3, MC_A = 4 };

template <bool HS>
__global__ __launch_bounds__(256) void k_prep(Dev d, uint32_t it) {
#pragma clang fp contract(off)
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= d.nbB) return;
  const int s = (int)(q / d.B), i = (int)(q % d.B);
  if (i >= d.bsz[s]) return;
  const int m = d.member[q];
  const uint32_t gm = (uint32_t)(d.col_offset + m);
  const int64_t S = d.nbB;
  double *mc = d.mc;
  const double bo = d.beta[m], x2 = d.xsq[m];
  const double sigmaE = d.sc->sigmaE;
  mc[MC_Z * S + q] = normal(d.seed, T_MARKER, gm, it, 1);
  mc[MC_BO * S + q] = bo;
  mc[MC_XSQ * S + q] = x2;
  if (HS) {
    const double lam = d.lambda[m], tau = d.sc->tau, c2 = d.sc->c2;
    const double sv = tau * c2 * lam / (tau * lam + c2);
    mc[MC_A * S + q] = x2 + (sigmaE / sv);
  } else {
    const int K = d.K, G = d.G;
    const int g = d.gAssign ? d.gAssign[m] : 0;
    const double sigmaG = d.sigmaGG[g];
    const double *pi_g = d.pi + (int64_t)g * K;
    mc[MC_P * S + q] = uniform(d.seed, T_MARKER, gm, it, 0);
    mc[MC_A * S + q] = log(pi_g[0]);
    for (int k = 1; k < K; ++k) {
      const double cVa = d.cva[g + (int64_t)G * (k - 1)];
      const double cVaI = 1.0 / cVa;
      mc[(MC_A + K + k - 1) * S + q] = x2 + (sigmaE / sigmaG) * cVaI;
      mc[(MC_A + k) * S + q] = log(pi_g[k]) - 0.5 * log(((sigmaG / sigmaE) * x2) * cVa + 1.0);
    }
  }
}

// Fast decision at num = r from the precomputed constants: P = softmax(logL(t)), A_k its
// cumulative sums, selected k = first with p <= A_k.  Also returns a decision-invariant
// window [lo, hi] in t (DESIGN.md "decision margins"): with logL_j = a_j + b_j t,
//   dA_k/dt = A_k (1 - A_k)(bbar_{<=k} - bbar_{>k}),  |.| <= min(A_k, 1-A_k) b_max,
// and over |t - t0| <= delta <= 1/b_max, A_k and 1-A_k grow by at most e^{b_max delta} <= e,
// so A_k stays on its side of p while delta <= gap / (e b_max min(A_k, 1-A_k)); half of that
// is used.  The reference's arithmetic differs from the softmax by a few ulps, so any gap
// below 1e-12 -- and any spread of logL near the 700-guard (BayesRv2.cpp:212-240) -- is
// handed to the exact evaluation (ex = true).
struct FastDec {
  int k;
  double lo, hi;
  bool ex;
};

__device__ __forceinline__ FastDec decide_fast(double r, const double *a, const double *den, int64_t stride, int K,
                                               double sigmaE, double p) {
#pragma clang fp contract(off)
  FastDec o;
  o.ex = false;
  const double t = r * r;
  if (K == 1) { o.k = 0; o.lo = -1e308; o.hi = 1e308; return o; }
  double L[MAXK], A[MAXK];
  double mx = -1e308, mn = 1e308, smax = 0.0;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    if (k < K) {
      const double sl = k == 0 ? 0.0 : 0.5 / (den[(k - 1) * stride] * sigmaE);
      L[k] = a[k * stride] + sl * t;
      mx = fmax(mx, L[k]);
      mn = fmin(mn, L[k]);
      smax = fmax(smax, sl);
    }
  }
  if (!(mx - mn < 690.0) || !(smax > 0.0)) { o.ex = true; o.k = 0; o.lo = 1.0; o.hi = -1.0; return o; }
  double S = 0.0;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    if (k < K) { A[k] = exp(L[k] - mx); S += A[k]; }
  }
  double acc = 0.0;
  int sel = FALLTHROUGH;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    if (k < K) {
      acc += A[k];
      A[k] = acc / S;
      if (sel == FALLTHROUGH && p <= A[k]) sel = k;
    }
  }
  const double E = 2.718281828459045;
  auto side = [&](double gap, double Ak) -> double {
    if (!(gap > 1e-12)) return 0.0;
    const double m = fmin(Ak, 1.0 - Ak);
    return m > 0.0 ? gap / (E * smax * m) : 1e300;
  };
  double w;
  if (sel == FALLTHROUGH) {
    w = 0.0;  // p above the last cumulative sum: only the exact formula decides
  } else {
    double Asel = A[0], Aprev = 0.0;
#pragma unroll
    for (int k = 1; k < MAXK; ++k)
      if (k == sel) { Asel = A[k]; Aprev = A[k - 1]; }
    w = side(Asel - p, Asel);
    if (sel > 0) w = fmin(w, side(p - Aprev, Aprev));
  }
  w = fmin(w, 1.0 / smax);
  const double mg = 0.5 * w;
  o.k = sel;
  if (!(mg > 0.0)) { o.ex = true; o.lo = 1.0; o.hi = -1.0; return o; }
  o.lo = t - mg;
  o.hi = t + mg;
  return o;
}

// The lane index, formed where it is used: the chains' re-decisions index their components' LDS
// constants by lane, and an index hoisted out of the chain loop is spilled in the solver kernel and its
// scratch reload (a full vmcnt wait) lands on the re-decision's path (~40 % of C1's re-decision time)
__device__ __forceinline__ int lane_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// quad_perm DPP move of a double within each group of four lanes (CTRL = sel0 | sel1 << 2 | sel2 << 4 |
// sel3 << 6): a VALU operation, no round trip through a scalar register as a readlane takes
template <int CTRL>
__device__ __forceinline__ double quad_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readfirstlane_f64(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// decide_fast for ONE position and K = 4, on a whole wave with every lane active: every quad of lanes holds
// the four components (component k on lane 4 j + k), maxima and minima run as two quad exchanges, and the
// exponentials, cumulative sums and side widths reach every lane of the quad by quad broadcasts; each lane
// then sums in component order.  Element operations, their order and the sums' order are decide_fast's
// (BayesRv2.cpp:206-220; maxima and minima are exact in any order): bit-identical results, and every quad
// computes the same values, so the outputs are taken from the first lane.
__device__ __forceinline__ FastDec decide_fast_quad(double r, const double *a, const double *den, int64_t stride,
                                                    double sigmaE, double p) {
#pragma clang fp contract(off)
  FastDec o;
  o.ex = false;
  const double t = r * r;
  const int kl = lane_here() & 3;
  const double dk = den[(max(kl, 1) - 1) * stride];
  const double sl = kl == 0 ? 0.0 : 0.5 / (dk * sigmaE);
  const double Lk = a[kl * stride] + sl * t;
  double mx = fmax(Lk, quad_f64<0xB1>(Lk));
  mx = fmax(-1e308, fmax(mx, quad_f64<0x4E>(mx)));
  double mn = fmin(Lk, quad_f64<0xB1>(Lk));
  mn = fmin(1e308, fmin(mn, quad_f64<0x4E>(mn)));
  double smax = fmax(sl, quad_f64<0xB1>(sl));
  smax = fmax(0.0, fmax(smax, quad_f64<0x4E>(smax)));
  if (__builtin_amdgcn_readfirstlane((int)(!(mx - mn < 690.0) || !(smax > 0.0)))) {
    o.ex = true; o.k = 0; o.lo = 1.0; o.hi = -1.0;
    return o;
  }
  const double ek = exp(Lk - mx);
  const double e0 = quad_f64<0x00>(ek), e1 = quad_f64<0x55>(ek), e2 = quad_f64<0xAA>(ek), e3 = quad_f64<0xFF>(ek);
  double S = 0.0;
  S += e0; S += e1; S += e2; S += e3;
  double acc = 0.0, myacc;
  acc += e0; myacc = acc;
  acc += e1; myacc = kl == 1 ? acc : myacc;
  acc += e2; myacc = kl == 2 ? acc : myacc;
  acc += e3; myacc = kl == 3 ? acc : myacc;
  const double Ak = myacc / S;  // lane 4 j + k: A[k]
  const double A[4] = {quad_f64<0x00>(Ak), quad_f64<0x55>(Ak), quad_f64<0xAA>(Ak), quad_f64<0xFF>(Ak)};
  int sel = FALLTHROUGH;
  double Asel = 0.0, Aprev = 0.0, Al = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool hit = sel == FALLTHROUGH && p <= A[k];
    Asel = hit ? A[k] : Asel;
    Aprev = hit ? Al : Aprev;
    sel = hit ? k : sel;
    Al = A[k];
  }
  const double E = 2.718281828459045;
  // the side above p on even lanes, the side below on odd lanes, exchanged by one quad move
  const bool below = (kl & 1) != 0;
  const double gap = below ? p - Aprev : Asel - p;
  const double Ag = below ? Aprev : Asel;
  double sw;
  if (!(gap > 1e-12)) sw = 0.0;
  else {
    const double m = fmin(Ag, 1.0 - Ag);
    sw = m > 0.0 ? gap / (E * smax * m) : 1e300;
  }
  const double swo = quad_f64<0xB1>(sw);
  const double sw0 = below ? swo : sw, sw1 = below ? sw : swo;
  const double ism = 1.0 / smax;
  double w = sel == FALLTHROUGH ? 0.0 : (sel > 0 ? fmin(sw0, sw1) : sw0);
  w = fmin(w, ism);
  const double mg = readfirstlane_f64(0.5 * w);
  o.k = __builtin_amdgcn_readfirstlane(sel);
  if (!(mg > 0.0)) { o.ex = true; o.lo = 1.0; o.hi = -1.0; return o; }
  o.lo = t - mg;
  o.hi = t + mg;
  return o;
}

// decide_fast for ONE position, evaluated by a whole wave with every lane active (the serial chains'
// re-decision, wave-uniform arguments): component k on lane k, so the K exponentials and the K quotients
// of the softmax issue once, side by side, instead of K times on the chain.  Every element is the same
// operation on the same values as in decide_fast and every sum runs in the same order (maxima and minima
// are exact in any order): the result is bit-identical to decide_fast's.  KT > 0: K = KT known at compile
// time (the loops over components lose their per-component branches: the default K = 4 runs this form).
template <int KT = 0>
__device__ __forceinline__ FastDec decide_fast_wave(double r, const double *a, const double *den, int64_t stride, int Kr,
                                                    double sigmaE, double p) {
#pragma clang fp contract(off)
  if constexpr (KT == 4) return decide_fast_quad(r, a, den, stride, sigmaE, p);
  constexpr int KM = KT > 0 ? KT : MAXK;
  const int K = KT > 0 ? KT : Kr;
  FastDec o;
  o.ex = false;
  const double t = r * r;
  if (K == 1) { o.k = 0; o.lo = -1e308; o.hi = 1e308; return o; }
  const int lane = threadIdx.x & 63;
  const int kl = lane < K ? lane : 0;  // this lane's component
  const double dk = den[(max(kl, 1) - 1) * stride];  // (read for every lane: no divergent load)
  const double sl = kl == 0 ? 0.0 : 0.5 / (dk * sigmaE);
  const double Lk = a[kl * stride] + sl * t;
  double mx = -1e308, mn = 1e308, smax = 0.0;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k < K) {
      const double v = readlane_f64(Lk, k);
      mx = fmax(mx, v);
      mn = fmin(mn, v);
      smax = fmax(smax, readlane_f64(sl, k));
    }
  }
  if (!(mx - mn < 690.0) || !(smax > 0.0)) { o.ex = true; o.k = 0; o.lo = 1.0; o.hi = -1.0; return o; }
  const double ek = exp(Lk - mx);
  double S = 0.0, ev[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k < K) { ev[k] = readlane_f64(ek, k); S += ev[k]; }
  }
  double acc = 0.0, myacc = 0.0;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k < K) {
      acc += ev[k];
      myacc = kl == k ? acc : myacc;
    }
  }
  const double Ak = myacc / S;  // lane k: A[k]
  int sel = FALLTHROUGH;
  double Asel = 0.0, Aprev = 0.0, Al = 0.0;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k < K) {
      const double A = readlane_f64(Ak, k);
      if (sel == FALLTHROUGH && p <= A) { sel = k; Asel = A; Aprev = Al; }
      Al = A;
    }
  }
  const double E = 2.718281828459045;
  // the two side widths and 1 / smax on lanes 0, 1, 2
  const double gap = lane == 0 ? Asel - p : p - Aprev;
  const double Ag = lane == 0 ? Asel : Aprev;
  double sw;
  if (!(gap > 1e-12)) sw = 0.0;
  else {
    const double m = fmin(Ag, 1.0 - Ag);
    sw = m > 0.0 ? gap / (E * smax * m) : 1e300;
  }
  const double ism = 1.0 / smax;
  double w;
  if (sel == FALLTHROUGH) {
    w = 0.0;  // p above the last cumulative sum: only the exact formula decides
  } else {
    w = readlane_f64(sw, 0);
    if (sel > 0) w = fmin(w, readlane_f64(sw, 1));
  }
  w = fmin(w, ism);
  const double mg = 0.5 * w;
  o.k = sel;
  if (!(mg > 0.0)) { o.ex = true; o.lo = 1.0; o.hi = -1.0; return o; }
  o.lo = t - mg;
  o.hi = t + mg;
  return o;
}

// Decision with the window, exact fallback included (parallel phases: prep and refresh).
__device__ __forceinline__ FastDec decide_pos(const Dev &d, double r, const double *a, const double *den, int64_t stride,
                                              double sigmaE, double p, double x2, int m) {
  FastDec o = decide_fast(r, a, den, stride, d.K, sigmaE, p);
  if (o.ex) {
    const int g = d.gAssign ? d.gAssign[m] : 0;
    Decision dc = decide_bayesr(r, x2, sigmaE, d.sigmaGG[g], d.pi + (int64_t)g * d.K, d.cva + g, d.G, d.K, p, true);
    if (dc.margin > 0.0) {
      const double t = r * r;
      o.k = dc.k;
      o.lo = t - dc.margin;
      o.hi = t + dc.margin;
      o.ex = false;
    }
  }
  return o;
}

// Out-of-line copies for the serial chains' rare paths (re-decision, exact formula): inlined, their
// MAXK-wide arrays raise the register pressure of the whole fused kernel into spills, and spill
// reloads on the chain wait behind the streaming workgroups' HBM traffic.
__device__ __noinline__ Decision decide_bayesr_ool(double num, double xsq, double sigmaE, double sigmaG,
                                                   const double *pi_g, const double *cva_g, int Gs, int K, double p,
                                                   bool want_margin) {
  return decide_bayesr(num, xsq, sigmaE, sigmaG, pi_g, cva_g, Gs, K, p, want_margin);
}
// decide_pos for the chains (a whole wave, uniform arguments): the fast decision inline and spread over the
// K lanes, the exact fallback out of line
template <int KT = 0>
__device__ __forceinline__ FastDec decide_pos_ool(const int *gAssign, const double *sigmaGG, const double *pi,
                                                  const double *cva, int G, int K, double r, const double *a,
                                                  const double *den, int64_t stride, double sigmaE, double p,
                                                  double x2, int m) {
  FastDec o = decide_fast_wave<KT>(r, a, den, stride, K, sigmaE, p);
  if (o.ex) {
    const int g = gAssign ? gAssign[m] : 0;
    Decision dc = decide_bayesr_ool(r, x2, sigmaE, sigmaGG[g], pi + (int64_t)g * K, cva + g, G, K, p, true);
    if (dc.margin > 0.0) {
      const double t = r * r;
      o.k = dc.k;
      o.lo = t - dc.margin;
      o.hi = t + dc.margin;
      o.ex = false;
    }
  }
  return o;
}

// A serial chain's re-decision of position `first` (a whole wave, uniform arguments).  K = 4 (the default
// mixture) runs the compile-time form of decide_fast_wave; BRR_DECIDE_K4 = 0 keeps the runtime-K form for
// every K, 2 moves the runtime-K form out of line.
#ifndef BRR_DECIDE_K4
#define BRR_DECIDE_K4 1
#endif
__device__ __noinline__ FastDec decide_pos_generic_ool(const int *gAssign, const double *sigmaGG, const double *pi,
                                                       const double *cva, int G, int K, double r, const double *a,
                                                       const double *den, int64_t stride, double sigmaE, double p,
                                                       double x2, int m) {
  return decide_pos_ool(gAssign, sigmaGG, pi, cva, G, K, r, a, den, stride, sigmaE, p, x2, m);
}
__device__ __forceinline__ FastDec chain_redecide(const Dev &d, double rf, const double *a, const double *den,
                                                  int64_t stride, double sigmaE, double p, double x2, int m) {
#if BRR_DECIDE_K4 == 1
  return d.K == 4 ? decide_pos_ool<4>(d.gAssign, d.sigmaGG, d.pi, d.cva, d.G, 4, rf, a, den, stride, sigmaE, p, x2, m)
                  : decide_pos_ool(d.gAssign, d.sigmaGG, d.pi, d.cva, d.G, d.K, rf, a, den, stride, sigmaE, p, x2, m);
#elif BRR_DECIDE_K4 == 2
  return d.K == 4 ? decide_pos_ool<4>(d.gAssign, d.sigmaGG, d.pi, d.cva, d.G, 4, rf, a, den, stride, sigmaE, p, x2, m)
                  : decide_pos_generic_ool(d.gAssign, d.sigmaGG, d.pi, d.cva, d.G, d.K, rf, a, den, stride, sigmaE, p, x2, m);
#else
  return decide_pos_ool(d.gAssign, d.sigmaGG, d.pi, d.cva, d.G, d.K, rf, a, den, stride, sigmaE, p, x2, m);
#endif
}

// ------------------------------------------------------------------------------------
// k_stream(s): residual update for block s-2 + partial dots of block s (lag-1 pipeline).
// While k_solve(s-1) runs on the other queue, k_stream(s) forms d = X_s^T E_{s-1}, with E_t
// the residual at the start of block t: it reads E_{s-2} (written by k_stream(s-1)), applies
// block s-2's changes (published by k_solve(s-2)) and writes E_{s-1} to the other buffer.
// k_solve(s) then subtracts the cross-Gram term X_s^T X_{s-1} delta_{s-1} exactly.
// Tile = SROWS (256) rows x 4*CW columns; lane l owns the 4 consecutive rows 4l..4l+3 of the
// tile (one 16-B load per column: 1 KiB = 8 whole 128-B lines per column and wave), wave w
// owns CW columns.  Partial dots: wave transpose-reduction (32 shuffles / 32 columns) ->
// slab1[rg][col]; the last of each group of STREAM_GROUP row tiles sums its group's rows ->
// slab2[group][col] and counts the group in gdone (read by k_solve(s)).
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

// Grid: roundup(RG, 8) * NC workgroups, NC = B / (4 CW) column chunks.  Workgroup ids are
// dispatched round-robin over the 8 XCDs; the mapping puts the NC chunks of one row tile on
// the same XCD (bid % 8 == rg % 8), so the redundant residual update of the tile (each chunk
// applies it to its own copy of the rows) re-reads the changed columns and eps from one L2.
// Only chunk 0 writes eps_out, and no workgroup reads eps_out, so the update is race-free.
// X and eps are padded to ld rows.
template <int CW>
__global__ __launch_bounds__(256, 2) void k_stream(Dev d, int s, const double *eps_in, double *eps_out) {
#pragma clang fp contract(off)
  constexpr int CB = 4 * CW;  // columns per workgroup
  __shared__ int s_last, s_np;
  __shared__ int s_pidx[BMAX + 16];
  __shared__ double s_pbo[BMAX + 16], s_pbn[BMAX + 16];
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int B = d.B;
  const int NC = B / CB;
  const int bid = blockIdx.x;
  const int rest = bid >> 3;
  const int cc = rest % NC;
  const int rg = (rest / NC) * 8 + (bid & 7);
  if (rg >= d.RG) return;
  const int64_t row0 = (int64_t)rg * SROWS + 4 * lane;
  const bool valid = row0 < d.N;
  const int64_t rowc = valid ? row0 : 0;
  const int par = s % NPAR;
  // block columns first: their loads depend on nothing
  const int *mem = d.member + (int64_t)s * B + cc * CB + w * CW;
  float4 x[CW];
  if (d.Xc) {
#pragma unroll
    for (int j = 0; j < CW; ++j) x[j] = x_at4(d, mem[j], rowc);
  } else {
#pragma unroll
    for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(d.X + rowc + (int64_t)mem[j] * d.ld);
  }
  const double2 ea = *reinterpret_cast<const double2 *>(eps_in + rowc);
  const double2 eb = *reinterpret_cast<const double2 *>(eps_in + rowc + 2);
  double e0 = ea.x, e1 = ea.y, e2 = eb.x, e3 = eb.y;
  // residual update for block s-2, eps = (eps + x b_old) - x b_new (BayesRv2.cpp:191,243): wait
  // until k_solve(s-2) has published (normally long done), then read its list with sc1 loads;
  // lists are padded to a multiple of 16 with neutral b_old = b_new = 0
  if (s >= d.seg0 + 2) {  // (blocks before the launch's first are in eps_in already)
    // one wave stages the list in LDS (one sc1 request per line per workgroup, instead of one
    // per wave and entry hammering the same few lines from every workgroup)
    if (w == 0) {
      if (lane == 0) wait_geq(d.sync + SY_PEND, d.sbase + s - 1, d.sync, 1);
      const int slot = (s - 2) % NSLOT;
      const int np = ld_sc1_int(d.pend_n + slot);
      const int *pidx = d.pend_idx + slot * d.pend_stride;
      const double *pbo = d.pend_bo + slot * d.pend_stride, *pbn = d.pend_bn + slot * d.pend_stride;
      for (int e = lane; e < np; e += 64) {
        s_pidx[e] = ld_sc1_int(pidx + e);
        s_pbo[e] = ld_sc1(pbo + e);
        s_pbn[e] = ld_sc1(pbn + e);
      }
      if (lane == 0) s_np = np;
    }
    __syncthreads();
    const int np = s_np;
    for (int p0 = 0; p0 < np; p0 += 16) {
      float4 xp[16];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        xp[q] = d.Xc ? x_at4(d, s_pidx[p0 + q], rowc)
                     : *reinterpret_cast<const float4 *>(d.X + rowc + (int64_t)s_pidx[p0 + q] * d.ld);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const double bo = s_pbo[p0 + q], bn = s_pbn[p0 + q];
        const double a0 = xp[q].x, a1 = xp[q].y, a2 = xp[q].z, a3 = xp[q].w;
        e0 = (e0 + a0 * bo) - a0 * bn;
        e1 = (e1 + a1 * bo) - a1 * bn;
        e2 = (e2 + a2 * bo) - a2 * bn;
        e3 = (e3 + a3 * bo) - a3 * bn;
      }
    }
  }
  if (cc == 0 && w == 0 && valid) {
    *reinterpret_cast<double2 *>(eps_out + row0) = make_double2(e0, e1);
    *reinterpret_cast<double2 *>(eps_out + row0 + 2) = make_double2(e2, e3);
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
  double *slab1 = d.slab1 + par * d.slab1_stride;
  double *slab2 = d.slab2 + par * d.slab2_stride;
  int *cnt1 = d.cnt1 + par * (d.NG * NC);
  if ((lane & 1) == 0 && col < CW) st_sc1(slab1 + (int64_t)rg * B + cc * CB + w * CW + col, r);
  // level-2: last arriver of the group sums the group's partials in row-tile order
  const int grp = rg / STREAM_GROUP;
  const int g0 = grp * STREAM_GROUP;
  const int gsz = min(STREAM_GROUP, d.RG - g0);
  const int use = d.gbase[par] + s / NPAR;  // earlier blocks of this ring index (cumulative counters)
  if (last_arriver_wt(cnt1 + grp * NC + cc, (use + 1) * gsz, &s_last)) {
    if (t < CB) {
      double v16[STREAM_GROUP];
#pragma unroll
      for (int q = 0; q < STREAM_GROUP; ++q)
        v16[q] = q < gsz ? ld_sc1(slab1 + (int64_t)(g0 + q) * B + cc * CB + t) : 0.0;
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < STREAM_GROUP; ++q) acc += v16[q];
      st_sc1(slab2 + (int64_t)grp * B + cc * CB + t, acc);
    }
    publish_add(d.sync + SY_GDONE + 32 * par, 1);  // k_solve(s) waits for NG * NC groups
  }
}

// 16-column wave transpose-reduction (persistent streamer).
__device__ __forceinline__ double wave_reduce16(double (&v)[16], int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool hi = lane & 32;
    const double send = hi ? v[j] : v[j + 8];
    const double keep = hi ? v[j + 8] : v[j];
    v[j] = keep + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool hi = lane & 16;
    const double send = hi ? v[j] : v[j + 4];
    const double keep = hi ? v[j + 4] : v[j];
    v[j] = keep + __shfl_xor(send, 16);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const bool hi = lane & 8;
    const double send = hi ? v[j] : v[j + 2];
    const double keep = hi ? v[j + 2] : v[j];
    v[j] = keep + __shfl_xor(send, 8);
  }
  {
    const bool hi = lane & 4;
    const double send = hi ? v[0] : v[1];
    const double keep = hi ? v[1] : v[0];
    v[0] = keep + __shfl_xor(send, 4);
  }
  const double a = v[0] + __shfl_xor(v[0], 2);
  return a + __shfl_xor(a, 1);
}
// 8-column wave transpose-reduction: lanes with (lane & 7) == 0 hold column reduce8_col(lane)
__device__ __forceinline__ double wave_reduce8(double (&v)[8], int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool hi = lane & 32;
    const double send = hi ? v[j] : v[j + 4];
    const double keep = hi ? v[j + 4] : v[j];
    v[j] = keep + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const bool hi = lane & 16;
    const double send = hi ? v[j] : v[j + 2];
    const double keep = hi ? v[j + 2] : v[j];
    v[j] = keep + __shfl_xor(send, 16);
  }
  {
    const bool hi = lane & 8;
    const double send = hi ? v[0] : v[1];
    const double keep = hi ? v[1] : v[0];
    v[0] = keep + __shfl_xor(send, 8);
  }
  double a = v[0] + __shfl_xor(v[0], 4);
  a = a + __shfl_xor(a, 2);
  return a + __shfl_xor(a, 1);
}
__device__ __forceinline__ int reduce8_col(int lane) {
  return ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1);
}

// 16-B load through a global (address space 1) pointer: global_load_dwordx4 with an SGPR base
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldg4(const float *p) {
  const v4f v = *(const __attribute__((address_space(1))) v4f *)(p);
  return make_float4(v.x, v.y, v.z, v.w);
}
// The streamers' X / code-tile loads: every byte is read once per sweep and the shard is far larger
// than the Infinity Cache, so they carry the non-temporal hint (MI355X_MICROARCH.md "nt-weights":
// bytes streamed once; BRR_STREAM_NT=0 builds the default policy for comparison)
#ifndef BRR_STREAM_NT
#define BRR_STREAM_NT 1
#endif
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldg4_stream(const float *p) {
#if BRR_STREAM_NT
  const v4f v = __builtin_nontemporal_load((const __attribute__((address_space(1))) v4f *)(p));
#else
  const v4f v = *(const __attribute__((address_space(1))) v4f *)(p);
#endif
  return make_float4(v.x, v.y, v.z, v.w);
}
// (2-bit code tiles keep the default policy: nt measured 46.1 -> 45.0 sweeps/s at C2 2-bit, while
// the f32 stream gained 29.8 -> 30.8; profiles/r03nt_ab.log)
__device__ __forceinline__ uint4 ldg16_stream(const uint8_t *p) {
  const v4u v = *(const __attribute__((address_space(1))) v4u *)(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// column held (lanes with (lane & 3) == 0) after wave_reduce16
__device__ __forceinline__ int reduce16_col(int lane) {
  return ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
}

// ------------------------------------------------------------------------------------
// k_solve(s): one workgroup.  Exact single-site updates of block position s in visit order.
//   num_j = d_j - sum_{i changed in block s-1} C_ij delta_i + xsq_j b_j - sum_{i<j in s} G_ji delta_i
// with d = X_s^T E_{s-1} from k_stream(s) and C the cross-Gram of the two blocks.  Waits (device
// counter) for k_stream(s)'s reduction groups, publishes block s's changes for k_solve(s+1)
// and k_stream(s+2).
// LDS layout (B positions):
//   doubles  r0, lo, hi, dsel, sdz, inv, bo, bn, x2, p, z [B each], a [K][B], den [K-1][B]
//   ints     fl, ks, gi, m, slot, spos [B each], misc [32]; (persistent) nlb change lists
//   slots    nslot Gram rows (B doubles each), staged for the positions predicted to change
enum PrFlag : int { PF_EX = 1 << 8, PF_LIKELY = 1 << 9 };

// pipeline lag of this fused sweep: Dev::lag, or 1 while the previous sweep changed many markers
// (k_hyper sets Scal::lag_next; 0 before the first sweep = 1).  Both kernels of a sweep read it once.
__device__ __forceinline__ int sweep_lag(const Dev &d) { return d.sc->lag_next >= 2 ? d.lag : 1; }

// nlb: change-list buffers kept in LDS from block to block (persistent solver: one per pipeline lag,
// block s's list in buffer s % nlb, each B + 16 doubles of deltas and B + 16 Gram indices)
__host__ __device__ inline size_t solve_fixed_bytes(int B, int K, int nlb = 0) {
  return (size_t)(11 + K + (K > 1 ? K - 1 : 0)) * 8 * B + (size_t)6 * 4 * B + 128 + (size_t)nlb * 12 * (B + 16);
}
constexpr size_t SOLVE_LDS_MAX = 160 * 1024;
// phase A scratch in the slot area (doubles): the change list (deltas, gram indices) and the
// partial sums of NT / B thread groups.  nslot * B always covers it for K <= MAXK.
__host__ __device__ inline size_t solve_scratch_doubles(int B, int NT) {
  return (size_t)(B + 16) + (B + 16) / 2 + 1 + (size_t)(B < NT ? NT / B : 1) * B;
}
// Resident-Gram mode (B <= RESIDENT_BMAX and LDS for B + scratch rows): the whole Gram block
// is copied into LDS during phase A (LDS-DMA, before the wait for the streaming side), the
// slot of a row is its Gram index, the phase-A scratch moves behind the rows, and the chain
// keeps every per-position constant in registers (solve_block step 3).
constexpr int RESIDENT_BMAX = 128;
__host__ __device__ inline int solve_scratch_rows(int B, int NT) {
  return (int)((solve_scratch_doubles(B, NT) + B - 1) / B);
}
__host__ __device__ inline int solve_max_slots(int B, int NT) {
  return B <= RESIDENT_BMAX ? B + solve_scratch_rows(B, NT) : B;
}

// One block position s, by one workgroup (called per launch, or in a loop by the persistent
// solver).  Phase A needs nothing from k_stream(s): per-position constants, the previous
// block's changes and their cross-Gram correction.  Phase B waits for k_stream(s)'s reduction
// groups, then decides, stages Gram rows, runs the serial chain and publishes.
// Gram-row ring of the solver (waves of one workgroup, LDS only).
constexpr int RING_DONE = 1 << 30;
constexpr uint32_t RING_SPIN_MAX = 1u << 20;
__device__ __forceinline__ int lds_ld_acq(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st_rel(int *p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Chain side: release the entries below k, then wait (bounded) until entry k is in its ring
// slot.  False on timeout: the caller then reads the row from global memory.
__device__ __forceinline__ bool ring_take(int *Lcons, const int *Lready, int RS, int k) {
  if ((threadIdx.x & 63) == 0) lds_st_rel(Lcons, k);
  for (uint32_t n = 0; n < RING_SPIN_MAX; ++n) {
    if (lds_ld_acq(Lready + k % RS) == k + 1) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}
// Producer waves 1..NW-1: entry k (k = wave-1, wave-1 + NW-1, ...) = Gram row of position
// Lspos[nst + k] into ring slot k % RS, once the chain has released entry k - RS.
template <int B, int NW>
__device__ __forceinline__ void ring_produce(const double *Gblk, const int *Lgi, const int *Lspos, int nst, int nov,
                                             double *ring, int RS, int *Lcons, int *Lready) {
  constexpr int H = B / 2, U = H >= 64 ? H / 64 : 1;
  const int lane = threadIdx.x & 63, pw = (int)(threadIdx.x >> 6) - 1;
  const double2 *G2 = reinterpret_cast<const double2 *>(Gblk);
  double2 *R2 = reinterpret_cast<double2 *>(ring);
  for (int k = pw; k < nov; k += NW - 1) {
    int c = 0;
    uint32_t n = 0;
    while ((c = lds_ld_acq(Lcons)) <= k - RS && ++n < RING_SPIN_MAX) __builtin_amdgcn_s_sleep(1);
    if (c >= RING_DONE || n >= RING_SPIN_MAX) break;
    const int64_t gi = Lgi[Lspos[nst + k]];
    double2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = G2[gi * H + min(u * 64 + lane, H - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u * 64 + lane < H) R2[(k % RS) * H + u * 64 + lane] = v[u];
    if (lane == 0) lds_st_rel(Lready + k % RS, k + 1);
  }
}

// Correctly rounded num / D on the chain: q0 = num * RN(1/D), one exact-remainder correction
// (Markstein) -- three dependent operations instead of the division sequence.
__device__ __forceinline__ double quot_rn(double num, double den, double inv) {
  const double q0 = num * inv;
  return __builtin_fma(__builtin_fma(-q0, den, num), inv, q0);
}

// The new-beta arms of a chain's re-decision: lane c < K holds quot_rn(num, D_c) + sqrt(sigmaE / D_c) z, the
// new beta if component c >= 1 is drawn (BayesRv2.cpp:226-230) -- the operations the chain's fast step
// applies to the selected component's constants, on the same values, formed beside the decision (off its
// dependency chain); the decision picks one arm by a readlane.  The chains need nothing else of the
// selected component: a re-decided position is stepped at once or left, never examined again.
__device__ __forceinline__ double refresh_arm(double num, const double *den, int64_t stride, int K, double sigmaE,
                                              double z) {
#pragma clang fp contract(off)
  const int lane = lane_here();
  const int kl = lane < K ? lane : 0;
  const double dk = kl >= 1 ? den[(kl - 1) * stride] : 1.0;
  const double iv = 1.0 / dk;
  return quot_rn(num, dk, iv) + sqrt(sigmaE / dk) * z;
}

// Resident-Gram serial chain, Horseshoe (wave 0).  Every position changes
// (beta ~ N(num/D, sigmaE/D), HorseshoeR.cpp:226-234): a forward substitution through the block in
// position order,
//     delta_j = (num_j - sum_{i<j} G_ij delta_i) / D_j + (z_j - beta_old_j).
// Lane l holds positions l + 64 q in registers as the scaled quantity
//     s_j = num_j / D_j + (z_j - beta_old_j) - sum_{i<j, visited} (G_ij / D_j) delta_i,
// which IS delta_j when position j is reached: a step is one read of the owner's s_j and one FMA
// per later position with the pre-scaled coefficient G_ij / D_j (zero at positions <= j).  The
// dependency chain per step is readlane + FMA; the Gram values are gathered GD steps ahead and
// scaled off the chain.  beta_new = beta_old + delta (same value as num/D + z up to rounding).
template <int B>
__device__ __forceinline__ void chain_hs_resident(int bs, const double *Lr0, const double *Ldsel, const double *Lsdz,
                                                  const double *Lbo, double *Lbn, const int *Lgi,
                                                  const double *slots) {
#pragma clang fp contract(off)
  constexpr int NS = B / 64;
  const int lane = threadIdx.x & 63;
  double sv[NS], iv[NS], bo[NS];
  int gg[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane + 64 * q;
    const bool in = pos < bs;
    const double dv = in ? Ldsel[pos] : 1.0;
    iv[q] = 1.0 / dv;
    bo[q] = in ? Lbo[pos] : 0.0;
    const double r = in ? Lr0[pos] : 0.0;
    const double z = in ? Lsdz[pos] : 0.0;
    sv[q] = quot_rn(r, dv, iv[q]) + (z - bo[q]);
    gg[q] = in ? Lgi[pos] : 0;
  }
  // Gram row of position j (lane j & 63 of plane j >> 6) gathered at this lane's positions
  auto gather = [&](int j, double (&g)[NS]) __attribute__((always_inline)) {
    int gi = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q)
      if ((j >> 6) == q) gi = __builtin_amdgcn_readlane(gg[q], j & 63);
    const double *row = slots + (int64_t)gi * B;
#pragma unroll
    for (int q = 0; q < NS; ++q) g[q] = row[gg[q]];
  };
  // ring of GD gathered rows, unrolled by GD: a set is consumed before it is refilled.  The
  // scheduling barrier at the end of each step keeps the gather GD steps ahead of its use (the
  // machine scheduler otherwise sinks it next to the use and the step waits for the LDS
  // latency: 84 -> ~31 cycles per step on an idle GPU, scripts/mb_chain.hip)
  constexpr int GD = 4;
  double gb[GD][NS];
#pragma unroll
  for (int u = 0; u < GD; ++u)
    if (u < bs) gather(u, gb[u]);
#pragma unroll
  for (int qo = 0; qo < NS; ++qo) {
    const int jend = min(bs, 64 * (qo + 1));
    for (int j0 = 64 * qo; j0 < jend; j0 += GD) {
#pragma unroll
      for (int u = 0; u < GD; ++u) {
        const int j = j0 + u;
        if (j >= jend) break;
        double h[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) h[q] = lane + 64 * q > j ? gb[u][q] * iv[q] : 0.0;
        if (j + GD < bs) gather(j + GD, gb[u]);
        const double delta = readlane_f64(sv[qo], j - 64 * qo);
#pragma unroll
        for (int q = qo; q < NS; ++q) sv[q] = __builtin_fma(-h[q], delta, sv[q]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NS; ++q)
    if (lane + 64 * q < bs) Lbn[lane + 64 * q] = bo[q] + sv[q];  // HorseshoeR.cpp:234
}

// Resident-Gram serial chain, BayesR family (wave 0).  Lane l holds positions l NS .. l NS + NS-1
// with their current num (r), decision window [lo, hi] in num^2, chosen component and its
// constants in registers.  The next position to visit is the lowest one that is predicted to
// change (act), needs the exact formula (ex) or whose num^2 left its window; every lane forms
// the new beta of its own lowest candidate in parallel with the wave's search, so a fast step
// is: ballot -> owner lane -> read delta -> update the later positions from the LDS Gram row.
// A position found outside its window is re-decided at its current num (wave-uniform) and
// re-examined; an exact-formula position is evaluated by decide_bayesr (BayesRv2.cpp:195-242).
// coef is the block's raw Gram in LDS (rows and columns by Gram index); a step updates the later
// positions by a select on the position, so the fast step has no divergent branch: branches cost
// the persistent solver far more than their instructions (Horseshoe chain).
// (Until round 3 a coefficient pass zeroed the entries of earlier positions first: 128 KiB of LDS
// rewritten per block at B = 128.)
template <int B>
__device__ __forceinline__ void chain_bayesr_resident(const Dev &d, int bs, double sigmaE, const double *Lr0,
                                                      const double *Llo, const double *Lhi, const double *Ldsel,
                                                      const double *Lsdz, const double *Lbo, double *Lbn,
                                                      const int *Lfl, int *Lks, const int *Lgi, const double *La,
                                                      const double *Lden, const double *Lp, const double *Lx2,
                                                      const double *Lz, const int *Lm, const double *coef,
                                                      bool prof) {
#pragma clang fp contract(off)
  constexpr int NS = B / 64;
  constexpr uint32_t ALLQ = (1u << NS) - 1u;
  const int lane = threadIdx.x & 63;
  double r[NS], lo[NS], hi[NS], dv[NS], iv[NS], sz[NS], bo[NS], bn[NS];
  int gg[NS], ks[NS];
  uint32_t act = 0, win = 0, valid = 0, exb = 0;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane * NS + q;
    const bool in = pos < bs;
    const int fl = in ? Lfl[pos] : 0;
    r[q] = in ? Lr0[pos] : 0.0;
    lo[q] = in ? Llo[pos] : 1.0;
    hi[q] = in ? Lhi[pos] : -1.0;
    dv[q] = in ? Ldsel[pos] : 1.0;
    iv[q] = 1.0 / dv[q];
    sz[q] = in ? Lsdz[pos] : 0.0;
    bo[q] = in ? Lbo[pos] : 0.0;
    bn[q] = bo[q];
    gg[q] = in ? Lgi[pos] : B - 1;  // past the end: an unused Gram index (zero row and column)
    ks[q] = fl & 0xFF;
    const double tt = r[q] * r[q];
    valid |= (uint32_t)in << q;
    act |= (uint32_t)(in && (fl & PF_LIKELY)) << q;
    exb |= (uint32_t)(in && (fl & PF_EX)) << q;
    win |= (uint32_t)(in && tt >= lo[q] && tt <= hi[q]) << q;
  }
  int nslow = 0, nsteps = 0, nref = 0;
  int i = 0;
  uint64_t tslow = 0;
  const uint64_t tl0 = prof ? wall_clock64() : 0;
  while (true) {
    const int lowq = min(max(i - lane * NS, 0), NS);
    const uint32_t ge = ALLQ & ~((1u << lowq) - 1u);
    const uint32_t cand = valid & (act | ~win | exb) & ge;
    const int ql = cand ? __builtin_ctz(cand) : 0;
    // this lane's lowest candidate, by selects (a divergent branch here costs more than all of it)
    double rv = r[0], dvv = dv[0], ivv = iv[0], szv = sz[0], bov = bo[0];
    int ksv = ks[0], ggv = gg[0];
#pragma unroll
    for (int q = 1; q < NS; ++q) {
      const bool h = ql == q;
      rv = h ? r[q] : rv;
      dvv = h ? dv[q] : dvv;
      ivv = h ? iv[q] : ivv;
      szv = h ? sz[q] : szv;
      bov = h ? bo[q] : bov;
      ksv = h ? ks[q] : ksv;
      ggv = h ? gg[q] : ggv;
    }
    // speculative new beta of this lane's lowest candidate (BayesRv2.cpp:226-230), every arm
    // evaluated and selected
    const double qv = quot_rn(rv, dvv, ivv) + szv;
    const double bnl = ksv == 0 ? 0.0 : (ksv == FALLTHROUGH ? bov : qv);
    const int fastl = (int)(((win & ~exb) >> ql) & 1u);
    const uint64_t bal = __ballot(cand != 0);
    if (!bal) break;  // the rest keep their decisions (no change)
    const int L = __builtin_ctzll(bal);
    const int qf = __builtin_amdgcn_readlane(ql, L);
    const int first = L * NS + qf;  // wave-uniform
    const double *grow = coef + (int64_t)__builtin_amdgcn_readlane(ggv, L) * B;
    double delta;
    if (__builtin_expect(__builtin_amdgcn_readlane(fastl, L) != 0, 1)) {
      delta = readlane_f64(bnl - bov, L);
#pragma unroll
      for (int q = 0; q < NS; ++q) bn[q] = (lane == L && q == qf) ? bnl : bn[q];
    } else {
      const uint64_t ts0 = prof ? wall_clock64() : 0;
      const double rf = readlane_f64(rv, L);
      const bool exf = (__builtin_amdgcn_readlane((int)exb, L) >> qf) & 1;
      if (!exf) {
        // outside its window: re-decide at the current num, then re-examine
        FastDec o = decide_pos_ool(d.gAssign, d.sigmaGG, d.pi, d.cva, d.G, d.K, rf, La + first, Lden + first, B, sigmaE, Lp[first], Lx2[first], Lm[first]);
        const bool lk = o.ex || !(o.k == FALLTHROUGH || (o.k == 0 && readlane_f64(bov, L) == 0.0));
        const double dsel = (!o.ex && o.k >= 1 && o.k != FALLTHROUGH) ? Lden[(o.k - 1) * B + first] : 1.0;
        const double sdz = sqrt(sigmaE / dsel) * Lz[first];
        if (lane == L) {
#pragma unroll
          for (int q = 0; q < NS; ++q)
            if (q == qf) { lo[q] = o.lo; hi[q] = o.hi; ks[q] = o.k; dv[q] = dsel; iv[q] = 1.0 / dsel; sz[q] = sdz; }
          act = (act & ~(1u << qf)) | ((uint32_t)lk << qf);
          win = (win & ~(1u << qf)) | ((uint32_t)(!o.ex) << qf);
          exb = (exb & ~(1u << qf)) | ((uint32_t)o.ex << qf);
        }
        ++nref;
        if (prof) tslow += wall_clock64() - ts0;
        continue;
      }
      const double bof = readlane_f64(bov, L);
      const int m = Lm[first];
      const int g = d.gAssign ? d.gAssign[m] : 0;
      Decision dc = decide_bayesr_ool(rf, Lx2[first], sigmaE, d.sigmaGG[g], d.pi + (int64_t)g * d.K, d.cva + g, d.G,
                                      d.K, Lp[first], false);
      const double bnf = dc.k == 0 ? 0.0 : (dc.k == FALLTHROUGH ? bof : rf / dc.denom + sqrt(sigmaE / dc.denom) * Lz[first]);
      if (lane == L) {
#pragma unroll
        for (int q = 0; q < NS; ++q)
          if (q == qf) { bn[q] = bnf; ks[q] = dc.k; }
      }
      delta = bnf - bof;
      ++nslow;
      if (prof) tslow += wall_clock64() - ts0;
    }
    // the positions after `first` subtract G delta (a select, not a branch: the raw Gram block is
    // in LDS, no coefficient pass zeroes the entries of earlier positions)
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const double g = grow[gg[q]];
      const bool later = lane * NS + q > first && ((valid >> q) & 1u);
      r[q] = later ? r[q] - g * delta : r[q];
      const double tt = r[q] * r[q];
      win = (win & ~(1u << q)) | ((uint32_t)(tt >= lo[q] && tt <= hi[q]) << q);
    }
    i = first + 1;
    ++nsteps;
  }
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane * NS + q;
    if (pos < bs) { Lbn[pos] = bn[q]; Lks[pos] = ks[q]; }
  }
  if (lane == 0 && nslow) atomicAdd(&d.sc->n_slow, (unsigned long long)nslow);
  if (prof && lane == 0) {
    atomicAdd(&d.sc->prof[6], (unsigned long long)nsteps);
    atomicAdd(&d.sc->prof[7], (unsigned long long)nref);
    atomicAdd(&d.sc->prof[8], (unsigned long long)tslow);                  // solve_refresh_us: slow paths
    atomicAdd(&d.sc->prof[9], (unsigned long long)(wall_clock64() - tl0));  // solve_correct_us: whole loop
  }
}

// The same chain in sub-blocks (blocked forward substitution).  Lane l holds positions l + 64 q, so
// sub-block q (positions 64 q .. 64 q + 63) is one position per lane: a step examines and updates ONE
// register set per lane (its position in the current sub-block) instead of NS, and the sub-block's
// changes reach the later sub-blocks' positions in one batch when the sub-block ends (the flush: for
// each change in chain order, r -= G delta at every later position).  Every position still receives the
// same subtractions in the same (chain) order as in chain_bayesr_resident, and is decided only after all
// of them, so the chain is bit-identical to it; the flush's reads are independent of each other (off the
// step's dependency chain).  scripts/mb_chain_br.hip: 733 against 861 shader cycles per step at B = 128
// (24 changes per block), bit-identical new betas.
template <int B>
__device__ __forceinline__ void chain_bayesr_resident_blk(const Dev &d, int bs, double sigmaE, const double *Lr0,
                                                          const double *Llo, const double *Lhi, const double *Ldsel,
                                                          const double *Lsdz, const double *Lbo, double *Lbn,
                                                          const int *Lfl, int *Lks, const int *Lgi, const double *La,
                                                          const double *Lden, const double *Lp, const double *Lx2,
                                                          const double *Lz, const int *Lm, const double *coef,
                                                          bool prof) {
#pragma clang fp contract(off)
  constexpr int NS = B / 64;
  const int lane = threadIdx.x & 63;
  double r[NS], lo[NS], hi[NS], dv[NS], iv[NS], sz[NS], bo[NS], bn[NS];
  int gg[NS], ks[NS];
  uint32_t act = 0, win = 0, valid = 0, exb = 0;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane + 64 * q;
    const bool in = pos < bs;
    const int fl = in ? Lfl[pos] : 0;
    r[q] = in ? Lr0[pos] : 0.0;
    lo[q] = in ? Llo[pos] : 1.0;
    hi[q] = in ? Lhi[pos] : -1.0;
    dv[q] = in ? Ldsel[pos] : 1.0;
    iv[q] = 1.0 / dv[q];
    sz[q] = in ? Lsdz[pos] : 0.0;
    bo[q] = in ? Lbo[pos] : 0.0;
    bn[q] = bo[q];
    gg[q] = in ? Lgi[pos] : B - 1;  // past the end: an unused Gram index (zero row and column)
    ks[q] = fl & 0xFF;
    const double tt = r[q] * r[q];
    valid |= (uint32_t)in << q;
    act |= (uint32_t)(in && (fl & PF_LIKELY)) << q;
    exb |= (uint32_t)(in && (fl & PF_EX)) << q;
    win |= (uint32_t)(in && tt >= lo[q] && tt <= hi[q]) << q;
  }
  int nslow = 0, nsteps = 0, nref = 0;
  uint64_t tslow = 0;
  const uint64_t tl0 = prof ? wall_clock64() : 0;
  static_for<NS>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    constexpr uint32_t bk = 1u << k;
    if (64 * k >= bs) return;
    int i = 64 * k;                   // the next position to examine
    int np = 0, pgi = 0;              // this sub-block's changes: lane c holds change c's Gram index
    double pdl = 0.0;                 // and its delta
    while (true) {
      const bool mine = (lane + 64 * k >= i) && ((valid & (act | ~win | exb) & bk) != 0);
      // speculative new beta of this lane's position (BayesRv2.cpp:226-230), every arm evaluated and selected
      const double qv = quot_rn(r[k], dv[k], iv[k]) + sz[k];
      const double bnl = ks[k] == 0 ? 0.0 : (ks[k] == FALLTHROUGH ? bo[k] : qv);
      const int fastl = (int)(((win & ~exb) >> k) & 1u);
      const uint64_t bal = __ballot(mine);
      if (!bal) break;  // the rest of the sub-block keeps its decisions
      const int L = __builtin_ctzll(bal);
      const int first = 64 * k + L;  // wave-uniform
      const int gif = __builtin_amdgcn_readlane(gg[k], L);
      double delta;
      if (__builtin_expect(__builtin_amdgcn_readlane(fastl, L) != 0, 1)) {
        delta = readlane_f64(bnl - bo[k], L);
        bn[k] = lane == L ? bnl : bn[k];
      } else {
        const uint64_t ts0 = prof ? wall_clock64() : 0;
        const double rf = readlane_f64(r[k], L);
        const bool exf = (__builtin_amdgcn_readlane((int)exb, L) >> k) & 1;
        if (!exf) {
          // outside its window: re-decide at the current num.  A fast decision that changes the position is
          // its step at once (the re-examination would find it inside its new window and take the fast arm
          // with these constants: the same delta); the exact formula's cases are re-examined
          const double arm = refresh_arm(rf, Lden + first, B, d.K, sigmaE, Lz[first]);
          const double pf = Lp[first], x2f = Lx2[first];
          const int mf = Lm[first];
          FastDec o = chain_redecide(d, rf, La + first, Lden + first, B, sigmaE, pf, x2f, mf);
          const double bof = readlane_f64(bo[k], L);
          const bool lk = o.ex || !(o.k == FALLTHROUGH || (o.k == 0 && bof == 0.0));
          // (its D, 1 / D and noise are not needed again: the position is stepped now or left)
          if (lane == L) {
            lo[k] = o.lo; hi[k] = o.hi; ks[k] = o.k;
            act = (act & ~bk) | ((uint32_t)lk << k);
            win = (win & ~bk) | ((uint32_t)(!o.ex) << k);
            exb = (exb & ~bk) | ((uint32_t)o.ex << k);
          }
          ++nref;
          if (o.ex || !lk) {
            if (prof) tslow += wall_clock64() - ts0;
            continue;
          }
          const double bnr = o.k == 0 ? 0.0 : readlane_f64(arm, o.k);
          bn[k] = lane == L ? bnr : bn[k];
          delta = bnr - bof;
          if (prof) tslow += wall_clock64() - ts0;
        } else {
          const double bof = readlane_f64(bo[k], L);
          const int m = Lm[first];
          const int g = d.gAssign ? d.gAssign[m] : 0;
          Decision dc = decide_bayesr_ool(rf, Lx2[first], sigmaE, d.sigmaGG[g], d.pi + (int64_t)g * d.K, d.cva + g, d.G,
                                          d.K, Lp[first], false);
          const double bnf = dc.k == 0 ? 0.0 : (dc.k == FALLTHROUGH ? bof : rf / dc.denom + sqrt(sigmaE / dc.denom) * Lz[first]);
          if (lane == L) { bn[k] = bnf; ks[k] = dc.k; }
          delta = bnf - bof;
          ++nslow;
          if (prof) tslow += wall_clock64() - ts0;
        }
      }
      // the sub-block's later positions subtract G delta now (the raw Gram block is in LDS); the later
      // sub-blocks' positions at the flush
      {
        const double g = coef[(int64_t)gif * B + gg[k]];
        const bool later = lane > L && (valid & bk);
        r[k] = later ? r[k] - g * delta : r[k];
        const double tt = r[k] * r[k];
        win = (win & ~bk) | ((uint32_t)(tt >= lo[k] && tt <= hi[k]) << k);
      }
      if (k + 1 < NS && delta != 0.0) {  // (a zero delta subtracts exactly nothing)
        pgi = lane == np ? gif : pgi;
        pdl = lane == np ? delta : pdl;
        ++np;
      }
      i = first + 1;
      ++nsteps;
    }
    if constexpr (k + 1 < NS) {
      // flush: this sub-block's changes, in chain order, into every later position
      for (int c = 0; c < np; ++c) {
        const int gic = __builtin_amdgcn_readlane(pgi, c);
        const double dc = readlane_f64(pdl, c);
        const double *row = coef + (int64_t)gic * B;
#pragma unroll
        for (int q = k + 1; q < NS; ++q) r[q] = r[q] - row[gg[q]] * dc;
      }
#pragma unroll
      for (int q = k + 1; q < NS; ++q) {
        const double tt = r[q] * r[q];
        win = (win & ~(1u << q)) | ((uint32_t)(((valid >> q) & 1u) && tt >= lo[q] && tt <= hi[q]) << q);
      }
    }
  });
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane + 64 * q;
    if (pos < bs) { Lbn[pos] = bn[q]; Lks[pos] = ks[q]; }
  }
  if (lane == 0 && nslow) atomicAdd(&d.sc->n_slow, (unsigned long long)nslow);
  if (prof && lane == 0) {
    atomicAdd(&d.sc->prof[6], (unsigned long long)nsteps);
    atomicAdd(&d.sc->prof[7], (unsigned long long)nref);
    atomicAdd(&d.sc->prof[8], (unsigned long long)tslow);                  // solve_refresh_us: slow paths
    atomicAdd(&d.sc->prof[9], (unsigned long long)(wall_clock64() - tl0));  // solve_correct_us: whole loop
  }
}

// Serial chain, BayesR family, for blocks whose Gram block does not fit in LDS (B = 256, 512): lane
// l holds positions l NS .. l NS + NS-1 with num and its decision window in registers; the Gram rows
// are the raw rows of the positions predicted to change (static LDS slots, then the ring the idle
// waves fill from HBM, else HBM itself), so an update is masked to the positions after the visited
// one.  Each lane reads the constants of ITS lowest candidate (flags, D, noise, beta_old, slot) from
// LDS and forms that candidate's new beta while the wave's ballot / owner-lane search runs, so a fast
// step is ballot -> readlane of the owner's delta -> row update: the position's constants, the
// division and the slot look-up are off the wave-uniform dependency chain (in the form it replaces,
// four dependent LDS round trips and the division sat on it per step).  Operations and values are
// those of that form (new beta = num / D + noise, BayesRv2.cpp:226-230).  Measured against it (C2,
// same run, twice): sweeps 5-24 of a fresh chain 37.4 / 37.8 against 37.9 / 37.4 ms -- the burn-in
// sweeps are bound by the solver's HBM round trips (Gram rows, corrections), not by this arithmetic.
template <int B>
__device__ __forceinline__ void chain_bayesr_rows(const Dev &d, int bs, double sigmaE, const double *Lr0,
                                                  const double *Llo, const double *Lhi, double *Ldsel, double *Lsdz,
                                                  double *Linv, const double *Lbo, double *Lbn, int *Lfl, int *Lks, const int *Lgi,
                                                  const double *La, const double *Lden, const double *Lp,
                                                  const double *Lx2, const double *Lz, const int *Lm, const int *Lslot,
                                                  const int *Lspos, const double *slots, const double *Ggl, int RS,
                                                  int nst, int nov, int npred, int *Lcons, int *Lready, bool prof) {
#pragma clang fp contract(off)
  constexpr int NS = B / 64;
  constexpr uint32_t ALLQ = NS >= 32 ? 0xFFFFFFFFu : ((1u << NS) - 1u);
  const int lane = threadIdx.x & 63;
  double r[NS], lo[NS], hi[NS];
  int gg[NS];
  uint32_t act = 0, win = 0, valid = 0;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane * NS + q;
    const bool in = pos < bs;
    r[q] = in ? Lr0[pos] : 0.0;
    lo[q] = in ? Llo[pos] : 1.0;
    hi[q] = in ? Lhi[pos] : -1.0;
    gg[q] = in ? Lgi[pos] : 0;
    const int fl = in ? Lfl[pos] : 0;
    const double tt = r[q] * r[q];
    valid |= (uint32_t)in << q;
    act |= (uint32_t)(in && (fl & PF_LIKELY)) << q;
    win |= (uint32_t)(in && tt >= lo[q] && tt <= hi[q]) << q;
  }
  int nslow = 0, nsteps = 0, nref = 0, nglob = 0;
  int kc = 0;  // ring cursor: entries below kc are released
  // the Gram row of the next predicted position with a static slot (Lspos[kp], kp < nsp), gathered one
  // step ahead -- before this step's update -- so that a step that visits it finds the row in
  // registers (its LDS latency off the step's dependency chain).  B = 256 only: at B = 512 its NS more
  // live registers spill in the solver kernel (C1 146 -> 152 sweeps/s; C2 30.2 -> 28.4 with it at 512)
  constexpr bool PREF = B <= 256;
  const int nsp = PREF ? min(npred, nst) : 0;
  int kp = 0, pre = -1;
  double gpre[NS];
  uint64_t tref = 0;
  const uint64_t tl0 = prof ? wall_clock64() : 0;
  int i = 0;
  while (i < bs) {
    const int lowq = min(max(i - lane * NS, 0), NS);
    const uint32_t ge = ALLQ & ~((1u << lowq) - 1u);
    const uint32_t cand = valid & (act | ~win) & ge;
    const int ql = cand ? __builtin_ctz(cand) : 0;
    // this lane's lowest candidate: its constants and its new beta (the fast arm)
    const int posl = min(lane * NS + ql, bs - 1);
    const int fll = Lfl[posl];
    const double dsl = Ldsel[posl], ivl = Linv[posl], szl = Lsdz[posl], bol = Lbo[posl];
    const int sll = Lslot[posl];
    double rv = r[0];
#pragma unroll
    for (int q = 1; q < NS; ++q) rv = ql == q ? r[q] : rv;
    const int ksl = fll & 0xFF;
    // BayesRv2.cpp:226-230; num / D as q0 = num RN(1/D) plus one exact-remainder correction (the
    // resident chain's quotient): three dependent operations on the step's path instead of a division
    const double bnl = ksl == 0 ? 0.0 : (ksl == FALLTHROUGH ? bol : quot_rn(rv, dsl, ivl) + szl);
    const int fastl = (int)((win >> ql) & 1u) & (int)((fll & PF_EX) == 0);
    const uint64_t bal = __ballot(cand != 0);
    if (!bal) break;  // the rest keep their decisions (no change)
    const int L = __builtin_ctzll(bal);
    const int qf = __builtin_amdgcn_readlane(ql, L);
    const int first = L * NS + qf;  // wave-uniform
    double delta;
    if (__builtin_expect(__builtin_amdgcn_readlane(fastl, L) != 0, 1)) {
      delta = readlane_f64(bnl - bol, L);
      if (lane == L) Lbn[first] = bnl;
    } else {
      const double rf = readlane_f64(rv, L);
      const bool exf = (__builtin_amdgcn_readlane(fll, L) & PF_EX) != 0;
      if (!exf) {
        // outside its window: re-decide `first` at its current num (wave-uniform), then re-examine it (the
        // re-decision's runtime-K form: at B = 256 / 512 re-decisions are rare, and the compile-time form's
        // registers spill in this kernel)
        const uint64_t tr0 = prof ? wall_clock64() : 0;
        FastDec o = decide_pos_ool(d.gAssign, d.sigmaGG, d.pi, d.cva, d.G, d.K, rf, La + first, Lden + first, B, sigmaE,
                                   Lp[first], Lx2[first], Lm[first]);
        const double bo = Lbo[first];
        const bool lk = o.ex || !(o.k == FALLTHROUGH || (o.k == 0 && bo == 0.0));
        const double dsel = (!o.ex && o.k >= 1 && o.k != FALLTHROUGH) ? Lden[(o.k - 1) * B + first] : 1.0;
        if (lane == 0) {
          Lfl[first] = (o.k & 0xFF) | (o.ex ? PF_EX : 0) | (lk ? PF_LIKELY : 0);
          Lks[first] = o.k;
          Ldsel[first] = dsel;
          Linv[first] = 1.0 / dsel;
          Lsdz[first] = sqrt(sigmaE / dsel) * Lz[first];
        }
        if (lane == L) {
#pragma unroll
          for (int q = 0; q < NS; ++q)
            if (q == qf) { lo[q] = o.lo; hi[q] = o.hi; }
          act = (act & ~(1u << qf)) | ((uint32_t)lk << qf);
          win = (win & ~(1u << qf)) | ((uint32_t)(!o.ex) << qf);
        }
        ++nref;
        if (prof) tref += wall_clock64() - tr0;
        continue;
      }
      const double bof = Lbo[first];
      const int m = Lm[first];
      const int g = d.gAssign ? d.gAssign[m] : 0;
      Decision dc = decide_bayesr_ool(rf, Lx2[first], sigmaE, d.sigmaGG[g], d.pi + (int64_t)g * d.K, d.cva + g, d.G,
                                      d.K, Lp[first], false);
      const double bnf = dc.k == 0 ? 0.0 : (dc.k == FALLTHROUGH ? bof : rf / dc.denom + sqrt(sigmaE / dc.denom) * Lz[first]);
      if (lane == 0) { Lbn[first] = bnf; Lks[first] = dc.k; }
      delta = bnf - bof;
      ++nslow;
    }
    if (delta != 0.0) {
      // the visited position's Gram row: its static slot, its ring entry, or HBM
      const int slf = __builtin_amdgcn_readlane(sll, L);
      int lrow = slf;  // LDS slot of the row, or -1: HBM
      bool from_ring = false;
      if (slf < 0 && RS > 0) {  // predicted beyond the static slots: its ring entry
        while (kc < nov && Lspos[nst + kc] < first) ++kc;  // entries passed without a change
        if (kc < nov && Lspos[nst + kc] == first && ring_take(Lcons, Lready, RS, kc)) {
          lrow = nst + kc % RS;
          from_ring = true;
        }
      }
      nglob += lrow < 0;
      // the row's NS entries of this lane's positions, through a pointer of the row's own address
      // space (a pointer that may be LDS or HBM compiles to FLAT loads, and the masked update
      // below then became NS branches, each a FLAT load and a full vmcnt / lgkmcnt wait: ~3,300
      // shader clocks per step at B = 512), all issued before any is used
      double g[NS];
      if (PREF && first == pre) {
#pragma unroll
        for (int q = 0; q < NS; ++q) g[q] = gpre[q];
      } else if (lrow >= 0) {
        const __attribute__((address_space(3))) double *row =
            (const __attribute__((address_space(3))) double *)(slots + (int64_t)lrow * B);
#pragma unroll
        for (int q = 0; q < NS; ++q) g[q] = row[gg[q]];
      } else {
        const __attribute__((address_space(1))) double *row =
            (const __attribute__((address_space(1))) double *)(Ggl + (int64_t)Lgi[first] * B);
#pragma unroll
        for (int q = 0; q < NS; ++q) g[q] = row[gg[q]];
      }
      // the next predicted position's row, in flight during this step's update
      while (PREF && kp < nsp && __builtin_amdgcn_readfirstlane(Lspos[kp]) <= first) ++kp;
      pre = -1;
      if (PREF && kp < nsp) {
        pre = __builtin_amdgcn_readfirstlane(Lspos[kp]);
        const __attribute__((address_space(3))) double *row =
            (const __attribute__((address_space(3))) double *)(slots + (int64_t)__builtin_amdgcn_readfirstlane(Lslot[pre]) * B);
#pragma unroll
        for (int q = 0; q < NS; ++q) gpre[q] = row[gg[q]];
      }
#pragma unroll
      for (int q = 0; q < NS; ++q) asm volatile("" ::"v"(g[q]));  // every load lands before the update
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        const int pos = lane * NS + q;
        const bool later = pos > first && pos < bs;
        r[q] = later ? r[q] - g[q] * delta : r[q];
        const double tt = r[q] * r[q];
        const uint32_t bw = (uint32_t)(tt >= lo[q] && tt <= hi[q]);
        win = later ? ((win & ~(1u << q)) | (bw << q)) : win;
      }
      if (from_ring) {
        ++kc;
        if (lane == 0) lds_st_rel(Lcons, kc);
      }
    }
    i = first + 1;
    ++nsteps;
  }
  if (lane == 0) lds_st_rel(Lcons, RING_DONE);
  if (lane == 0 && nslow) atomicAdd(&d.sc->n_slow, (unsigned long long)nslow);
  if (prof && lane == 0) {
    atomicAdd(&d.sc->prof[6], (unsigned long long)nsteps);
    atomicAdd(&d.sc->prof[7], (unsigned long long)nref);
    atomicAdd(&d.sc->prof[4], (unsigned long long)nglob);
    atomicAdd(&d.sc->prof[8], (unsigned long long)tref);
    atomicAdd(&d.sc->prof[9], (unsigned long long)(wall_clock64() - tl0));
  }
}

// The chains as separate (not inlined) functions: inside the persistent k_sweep the solver's
// chain shares the register allocation of every role (256 VGPRs and several hundred spilled SGPRs
// whose reloads land in the chain's loop); called, a chain gets its own allocation (Horseshoe:
// 220 -> 53 shader cycles per step in the fused kernel, the isolated microbenchmark's rate).  The LDS
// operands travel as address-space-3 pointers so the callee still addresses them with ds_*
// instructions (a generic pointer would make every read a flat access).
#ifndef BRR_CHAIN_INLINE
#define BRR_CHAIN_INLINE 0
#endif
// (the BayesR chain stays inline: called, its caller keeps ~400 VGPRs of live state in scratch
// across the call and the streaming role of the same kernel slowed 2x at C3, measured)
#ifndef BRR_BAYESR_CHAIN_CALL
#define BRR_BAYESR_CHAIN_CALL 0
#endif
#define BRR_LDS __attribute__((address_space(3)))
template <class T>
__device__ __forceinline__ BRR_LDS T *to_lds(T *p) { return (BRR_LDS T *)p; }
template <class T>
__device__ __forceinline__ T *from_lds(BRR_LDS T *p) { return (T *)p; }

template <int B>
__device__ __attribute__((noinline)) void chain_hs_call(int bs, BRR_LDS const double *Lr0, BRR_LDS const double *Ldsel,
                                                        BRR_LDS const double *Lsdz, BRR_LDS const double *Lbo,
                                                        BRR_LDS double *Lbn, BRR_LDS const int *Lgi,
                                                        BRR_LDS const double *coef) {
  chain_hs_blocked<B>(bs, from_lds(Lr0), from_lds(Ldsel), from_lds(Lsdz), from_lds(Lbo), from_lds(Lbn), from_lds(Lgi),
                      from_lds(coef));
}

template <int B>
__device__ __attribute__((noinline)) void chain_bayesr_call(
    const Dev &d, int bs, double sigmaE, BRR_LDS const double *Lr0, BRR_LDS const double *Llo, BRR_LDS const double *Lhi,
    BRR_LDS const double *Ldsel, BRR_LDS const double *Lsdz, BRR_LDS const double *Lbo, BRR_LDS double *Lbn,
    BRR_LDS const int *Lfl, BRR_LDS int *Lks, BRR_LDS const int *Lgi, BRR_LDS const double *La,
    BRR_LDS const double *Lden, BRR_LDS const double *Lp, BRR_LDS const double *Lx2, BRR_LDS const double *Lz,
    BRR_LDS const int *Lm, BRR_LDS const double *coef, bool prof) {
  chain_bayesr_resident<B>(d, bs, sigmaE, from_lds(Lr0), from_lds(Llo), from_lds(Lhi), from_lds(Ldsel), from_lds(Lsdz),
                           from_lds(Lbo), from_lds(Lbn), from_lds(Lfl), from_lds(Lks), from_lds(Lgi), from_lds(La),
                           from_lds(Lden), from_lds(Lp), from_lds(Lx2), from_lds(Lz), from_lds(Lm), from_lds(coef), prof);
}

#ifndef BRR_CHAIN_BLK
#define BRR_CHAIN_BLK 1  // the resident BayesR chain in sub-blocks of 64 positions (chain_bayesr_resident_blk); 0: per step
#endif

#ifndef BRR_EARLY_GRAM
#define BRR_EARLY_GRAM 0
#endif

// persistent: one workgroup solves every block of the sweep in order (LDS persists between blocks)
template <bool HS, int B, int NT>
__device__ __forceinline__ void solve_block(const Dev &d, int s, uint32_t it, int nslot, char *smem,
                                            bool persistent, int lag) {
#pragma clang fp contract(off)
  constexpr int NPT = (B + NT - 1) / NT;  // positions per thread, parallel phases
  constexpr int NW = NT / 64;             // waves
  constexpr int NS = B / 64;            // positions per lane (contiguous), serial chain
  const int K = HS ? 1 : d.K;
  const int KD = K > 1 ? K - 1 : 0;
  double *Lr0 = reinterpret_cast<double *>(smem);
  // (Linv: 1 / D of each position's decision, for the row chain's quotient; Lbo .. Lden stay contiguous
  // for the constants' LDS-DMA)
  double *Llo = Lr0 + B, *Lhi = Llo + B, *Ldsel = Lhi + B, *Lsdz = Ldsel + B, *Linv = Lsdz + B, *Lbo = Linv + B, *Lbn = Lbo + B,
         *Lx2 = Lbn + B, *Lp = Lx2 + B, *Lz = Lp + B, *La = Lz + B, *Lden = La + (int64_t)K * B;
  int *Lfl = reinterpret_cast<int *>(Lden + (int64_t)KD * B);
  int *Lks = Lfl + B, *Lgi = Lks + B, *Lm = Lgi + B, *Lslot = Lm + B, *Lspos = Lslot + B, *misc = Lspos + B;
  // persistent solver: the change lists of the last nlb blocks stay in LDS (buffer j: deltas at
  // Llist + j (B + 16), Gram indices at Lligi + j (B + 16); misc[16 + 2 j] = padded length, misc[17 + 2 j]
  // = its block), so the cross-Gram correction of the next blocks needs no round trip for them
  const int nlb = persistent ? d.lag : 0;
  double *Llist = reinterpret_cast<double *>(misc + 32);
  int *Lligi = reinterpret_cast<int *>(Llist + (int64_t)nlb * (B + 16));
  double *slots = reinterpret_cast<double *>(Lligi + (int64_t)nlb * (B + 16));

  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const int bs = d.bsz[s];
  const int gb = d.gblk[s];
  const int par = s % NPAR;
  const bool prof = d.sc->prof_on;
  uint64_t tp0 = prof ? wall_clock64() : 0, tp1 = 0, tp2 = 0, tp3 = 0, tw = 0, tce = 0;
  const double sigmaE = d.sc->sigmaE;
  const int64_t S = d.nbB;
  const int64_t q0 = (int64_t)s * B;
  const bool resident = B <= RESIDENT_BMAX && nslot >= B + solve_scratch_rows(B, NT);
  // misc[12]: block whose Gram copy into LDS the previous block already started; misc[17 + 2 j]:
  // block of the change list in LDS buffer j
  if (t == 0 && s == d.seg0) {
    misc[12] = -2;
    for (int j = 0; j < LAG_MAX; ++j) misc[17 + 2 * j] = -2;
  }
  const bool pipelined = persistent && resident;

  // A) everything that does not depend on k_stream(s): the per-position constants, the cross-Gram
  // correction for the changes of the blocks the streamed dots have not seen, and (resident mode) the
  // LDS-DMA of block s's Gram block.  The constants go straight from HBM into their LDS arrays by
  // LDS-DMA (no registers, no wait at the issue), so they are in flight together with the
  // correction's loads: one HBM round trip under the streaming load instead of two.  Deferred-DMA mode
  // (persistent resident BayesR solver): waves NW/2 .. NW-1 alone copy the Gram block and do not wait
  // for it until the chain -- the barriers between here and the chain only order LDS (lds_barrier), so
  // the copy lands during the correction, the wait for the streaming side and the decisions -- while
  // waves 0 .. NW/2-1 load the constants and form the correction; otherwise every wave does both (the
  // Horseshoe's coefficient pass needs the Gram block before the wait).
  const bool defer_dma = pipelined && !HS;

  const int dma_w0 = defer_dma ? NW / 2 : 0;  // first wave of the Gram copy
  const int cw1 = defer_dma ? NW / 2 : NW;    // waves [0, cw1) load the constants
  {
    // LDS [Lbo, Lden + KD B): fields bo, bn (= bo), x2, p, z, a_k (K), den_k (KD), B doubles each, in
    // 16-B pieces (64 per wave instruction: 1 KiB contiguous in LDS, per-lane HBM sources); then
    // [Lgi, Lm + B): the Gram index and the member of every position
    const int nfd = 5 + K + KD;
    const int npd = nfd * B / 2, npi = 2 * B / 4;  // 16-B pieces
    const int ninst = (npd + 63) / 64 + (npi + 63) / 64;
    for (int w = wv; w < ninst; w += cw1) {
      const int nid = (npd + 63) / 64;
      const __attribute__((address_space(1))) void *src;
      __attribute__((address_space(3))) void *dst;
      if (w < nid) {
        const int pc = min(w * 64 + lane, npd - 1), f = pc / (B / 2), e = (pc % (B / 2)) * 2;
        const int mf = f < 2 ? MC_BO : f == 2 ? MC_XSQ : f == 3 ? MC_P : f == 4 ? MC_Z : MC_A + (f - 5);
        src = (const __attribute__((address_space(1))) void *)(d.mc + (int64_t)mf * S + q0 + e);
        dst = (__attribute__((address_space(3))) void *)(reinterpret_cast<char *>(Lbo) + (int64_t)w * 1024);
      } else {
        const int pc = min((w - nid) * 64 + lane, npi - 1), f = pc / (B / 4), e = (pc % (B / 4)) * 4;
        src = (const __attribute__((address_space(1))) void *)((f == 0 ? d.gidx : d.member) + q0 + e);
        dst = (__attribute__((address_space(3))) void *)(reinterpret_cast<char *>(Lgi) + (int64_t)(w - nid) * 1024);
      }
      if (lane < (w < nid ? npd - w * 64 : npi - (w - nid) * 64))
        __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
    }
  }
  if (resident && !(pipelined && s > d.seg0 && misc[12] == s) && wv >= dma_w0) {
    // row gi at slots + gi B, 1 KiB per wave-instruction; retired by each copying wave's vmcnt(0) and
    // the barrier after it (before the coefficients / the chain read it).  (The persistent solver can
    // start this copy at the end of the previous block already, see step 3.)
    constexpr int NCHUNK = B * B * 8 / 1024;
    const char *src = reinterpret_cast<const char *>(d.gram + (int64_t)gb * B * B);
    char *dst = reinterpret_cast<char *>(slots);
    for (int c = wv - dma_w0; c < NCHUNK; c += NW - dma_w0)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + c * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void *)(dst + c * 1024), 16, 0, 0);
  }
  const uint64_t tA1 = prof ? wall_clock64() : 0;  // constants and copy issued
  // sum_i (x_j . x_i) delta_i over the changes of the blocks the streamed dots have not seen:
  // block s-1 (cross-Gram of cycle neighbours), and with lag 2 also block s-2 (cross-Gram of
  // blocks two apart), added in that order -- blocks of this launch only (seg0 onwards: the
  // earlier ones' changes are in the residual the launch started from).  The persistent solver
  // keeps the lists in LDS (written by its own write-back); the per-block solve stages the one list
  // of its lag-1 pipeline from global memory into the slot area, which is free until step 2.  Each
  // round has up to 48 loads in flight: a chunk (16 entries) of every list, or with one list three
  // of its chunks; every list is summed in entry order.  With B < NT the thread groups (NT / B, or
  // the copy-free waves' share in deferred-DMA mode) take contiguous parts of each list and their
  // partial sums are added in group order.
  constexpr int PG0 = B < NT ? NT / B : 1;
  const int PG = defer_dma ? max(1, min(PG0, (dma_w0 * 64) / B)) : PG0;
  double *scr = resident ? slots + (int64_t)B * B : slots;
  double *Lpart = scr + (B + 16) + (B + 16) / 2 + 1;  // [PG][B] partial sums (PG > 1)
  const int nlist = lag;  // (<= d.lag: the persistent solver's lag of this sweep; per-block: 1)
  const double *Cl[LAG_MAX] = {nullptr, nullptr, nullptr};
  const double *Ldl[LAG_MAX] = {nullptr, nullptr, nullptr};
  const int *Lgl[LAG_MAX] = {nullptr, nullptr, nullptr};
  int npl[LAG_MAX] = {0, 0, 0};
  bool staged = false;
#pragma unroll
  for (int l = 0; l < LAG_MAX; ++l) {
    const int sp = s - 1 - l;  // the earlier block
    // (rcorr: the reducers subtract it -- all but block s-1's with rcsplit)
    if (l >= nlist || sp < d.seg0 || (persistent && d.rcorr && !(d.rcsplit && l == 0))) continue;
    const int gp = d.gblk[sp];
    if (l == 0)
      Cl[l] = (gb == (gp + 1) % d.nb) ? d.xgram + (int64_t)gp * B * B : d.xgramT + (int64_t)gb * B * B;
    else if (l == 1)
      Cl[l] = (gb == (gp + 2) % d.nb) ? d.xgram2 + (int64_t)gp * B * B : d.xgram2T + (int64_t)gb * B * B;
    else
      Cl[l] = (gb == (gp + 3) % d.nb) ? d.xgram3 + (int64_t)gp * B * B : d.xgram3T + (int64_t)gb * B * B;
    const int j = nlb > 0 ? sp % nlb : 0;
    if (nlb > 0 && misc[17 + 2 * j] == sp) {
      // this workgroup wrote block sp's list into LDS buffer j itself (its step 4)
      npl[l] = misc[16 + 2 * j];
      Ldl[l] = Llist + (int64_t)j * (B + 16);
      Lgl[l] = Lligi + (int64_t)j * (B + 16);
    } else if (!staged) {
      // (per-block solve: lag 1, one list) from global memory, written with sc1 stores
      double *Lcd = scr;
      int *Lcg = reinterpret_cast<int *>(scr + (B + 16));
      const int slot = sp % NSLOT;
      const int np = ld_sc1_int(d.pend_n + slot);
      const int *pv_gi = d.pend_gi + slot * d.pend_stride;
      const double *pv_bo = d.pend_bo + slot * d.pend_stride, *pv_bn = d.pend_bn + slot * d.pend_stride;
      for (int e = t; e < np; e += NT) {
        Lcg[e] = ld_sc1_int(pv_gi + e);
        Lcd[e] = ld_sc1(pv_bn + e) - ld_sc1(pv_bo + e);
      }
      npl[l] = np;
      Ldl[l] = Lcd;
      Lgl[l] = Lcg;
      staged = true;
    }
  }
  if (staged) __syncthreads();
  // The sums are formed per Gram index j of block s (the columns of a cross-Gram row are Gram
  // indices, so a wave's 64 loads of one entry are 512 contiguous bytes; by visit position they were
  // 64 scattered ones) into Lcor[j] (the correction of the position whose Gram index is j, read by
  // the decisions through Lgi); per j the same operations in the same order as by position.
  double *Lcor = Lpart;
#pragma unroll
  for (int c = 0; c < NPT; ++c) {
    const int pos = (t % (B < NT ? B : NT)) + NT * c;  // (here: the Gram index j)
    const int grp = B < NT ? t / B : 0;
    double corr[LAG_MAX] = {0.0, 0.0, 0.0};
    if (pos < bs && grp < PG) {
      const int gi = pos;
      int c0[LAG_MAX], c1[LAG_MAX];
#pragma unroll
      for (int l = 0; l < LAG_MAX; ++l) {
        const int nch = npl[l] / 16;
        c0[l] = grp * nch / PG;
        c1[l] = (grp + 1) * nch / PG;
      }
      // one list: three of its chunks per round (slot groups 0, 1, 2), else a chunk of every list
      const bool one = nlist == 1;
      for (int k = 0;; ++k) {
        bool more = false;
        double cv[LAG_MAX][16];
        int chs[LAG_MAX];
#pragma unroll
        for (int u3 = 0; u3 < LAG_MAX; ++u3) {
          const int l = one ? 0 : u3;
          const int ch = one ? c0[0] + 3 * k + u3 : c0[l] + k;
          chs[u3] = ch;
          if (ch < c1[l]) {
            more = true;
#pragma unroll
            for (int u = 0; u < 16; ++u) cv[u3][u] = Cl[l][(int64_t)Lgl[l][16 * ch + u] * B + gi];
          }
        }
        if (!more) break;
#pragma unroll
        for (int u3 = 0; u3 < LAG_MAX; ++u3) {
          const int l = one ? 0 : u3;
          const int ch = chs[u3];
          if (ch < c1[l]) {
#pragma unroll
            for (int u = 0; u < 16; ++u) corr[l] += cv[u3][u] * Ldl[l][16 * ch + u];
          }
        }
      }
    }
    // the lists' sums added in list order (per thread group, then the groups in group order)
    const double tot = (corr[0] + corr[1]) + corr[2];
    if (grp < PG) Lcor[grp * B + pos] = tot;
  }
  // the constant-loading waves' LDS-DMA has landed before any wave reads the constants (the
  // deferred Gram copy's waves wait for theirs just before the chain)
  if (wv < cw1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (PG > 1) {
    if (defer_dma) lds_barrier(); else __syncthreads();
    if (t < bs) {
      double tot = Lpart[t];
      for (int g = 1; g < PG; ++g) tot += Lpart[g * B + t];
      Lcor[t] = tot;
    }
  }
  const uint64_t tA2 = prof ? wall_clock64() : 0;  // cross-Gram correction done
  if (resident && HS) {
    // the Horseshoe chain's coefficients made in place from the resident Gram before the wait for
    // the streaming side: entry (i, j) = G_ij / D_j (D is a per-sweep constant,
    // HorseshoeR.cpp:226-232) when position i comes before position j, else 0; the scratch behind
    // the rows holds the scale and the position of every Gram index.  (The BayesR chain reads the
    // raw Gram block and masks by position.)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA pieces landed
    __syncthreads();  // (also: the correction's partial sums in the scratch are consumed)
    double *Linv = scr;
    int *Lposg = reinterpret_cast<int *>(scr + B);
    for (int g = t; g < B; g += NT) { Linv[g] = 0.0; Lposg[g] = B; }
    __syncthreads();
    for (int pos = t; pos < bs; pos += NT) { Linv[Lgi[pos]] = HS ? 1.0 / La[pos] : 1.0; Lposg[Lgi[pos]] = pos; }
    __syncthreads();
    chain_coefficients<B, NT>(slots, Linv, Lposg);
  }
  const uint64_t tA3 = prof ? wall_clock64() : 0;  // coefficients built
  // B) wait for k_stream(s)'s reduction groups (other queue; cumulative count).  The persistent
  // solver instead polls the reduced dots themselves in step 1 (each slot holds this block's
  // sentinel until its reducer writes it): one HBM round trip less than counter, barrier and loads.
  if (t == 0 && s == 0) stamp(d.sync, 3);
  if (t == 0 && !persistent) wait_geq(d.sync + SY_GDONE + 32 * par, (d.gbase[par] + s / NPAR + 1) * d.gtarget, d.sync, 3);
  if (t == 0 && s == 0) stamp(d.sync, 4);
  if (defer_dma) {
    lds_barrier();  // (the copying waves wait for their pieces just before the chain)
  } else {
    if (resident) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA pieces landed
    __syncthreads();
  }
  if (prof) tw = wall_clock64();
  const double *slab2 = d.slab2 + par * d.slab2_stride;
  // 1) num at the block start, decisions with their windows; Gram-row slots for the positions
  //    predicted to change (position order).  When the slot area cannot hold a row for every
  //    position, its last RS slots form a ring: the predicted positions beyond the nst static
  //    slots (Lspos[nst + k], k < nov) get their rows from global memory through the ring,
  //    filled in chain order by the otherwise idle waves while wave 0 runs the chain.
  const int RS = (nslot < B && NW > 1) ? min(6, nslot / 2) : 0;
  const int nst = nslot - RS;
  int *Lcons = misc + 8, *Lready = misc + 9;  // ring: entries released by the chain, entry k ready = k + 1
  int base = 0;
#pragma unroll
  for (int c = 0; c < NPT; ++c) {
    const int pos = t + NT * c;
    bool likely = false;
    double dsum = 0.0;
    // (persistent solver) every one of the B slot columns is polled by one thread -- a short last
    // block's unread columns too -- so that no reducer store can land after the sentinel stores below
    if (pos < bs || (persistent && pos < B)) {
      // the dots are by visit position, or by in-block (storage) index when the 2-bit streamers
      // read the block in storage order (a permutation of 0 .. bs-1; columns bs .. B-1 are unread)
      const int sidx = pos < bs && d.slab_storage ? Lgi[pos] : pos;
      // (this block's sentinel only: a stale one of another epoch cannot be here -- after a failed census
      // the error flag makes every later fused launch leave at its census until the host has switched
      // the session to the per-block kernels, which use no sentinels.  Testing for any sentinel instead
      // cost the B = 512 solver 16 more spilled VGPRs.)
      const unsigned long long sent = slab_sentinel(d.sbase + s);
      for (int g0 = 0; g0 < d.NG; g0 += 16) {
        unsigned long long v[16];
        for (uint32_t n = 0;; ++n) {
          bool ready = true;
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            v[u] = g0 + u < d.NG ? ld_sc1_u64(slab2 + (int64_t)(g0 + u) * B + sidx) : 0ull;
            ready = ready && (!persistent || v[u] != sent);
          }
          if (ready) break;
          if (n > SPIN_MAX) {  // bounded, as wait_geq: the host reports the protocol error
            if (atomicCAS(d.sync + SY_ERR, 0, 1) == 0) {
              st_sc1_int(d.sync + SY_ERR + 1, 3);
              st_sc1_int(d.sync + SY_ERR + 2, d.sbase + s);
              st_sc1_int(d.sync + SY_ERR + 3, g0);
              st_sc1_int(d.sync + SY_ERR + 4, (int)blockIdx.x);
            }
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) dsum += __longlong_as_double((long long)v[u]);
      }
    }
    if (pos < bs) {
      const double bo = Lbo[pos], x2 = Lx2[pos];
      // num = x.(eps + x b_old) (BayesRv2.cpp:191-193), x.eps = d - cross-Gram correction
      const double r = (dsum - Lcor[Lgi[pos]]) + x2 * bo;
      FastDec o;
      double dsel;
      if (HS) {
        o.k = 1; o.lo = -1e308; o.hi = 1e308; o.ex = false;
        dsel = La[pos];  // D (HorseshoeR.cpp:232-234)
        likely = true;
      } else {
        o = decide_pos(d, r, La + pos, Lden + pos, B, sigmaE, Lp[pos], x2, Lm[pos]);
        dsel = (!o.ex && o.k >= 1 && o.k != FALLTHROUGH) ? Lden[(o.k - 1) * B + pos] : 1.0;
        likely = o.ex || !(o.k == FALLTHROUGH || (o.k == 0 && bo == 0.0));
      }
      Lfl[pos] = (o.k & 0xFF) | (o.ex ? PF_EX : 0) | (likely ? PF_LIKELY : 0);
      Lks[pos] = o.k & 0xFF;
      Lr0[pos] = r;
      Llo[pos] = o.lo;
      Lhi[pos] = o.hi;
      Ldsel[pos] = dsel;
      Linv[pos] = 1.0 / dsel;
      Lsdz[pos] = sqrt(sigmaE / dsel) * Lz[pos];  // rnorm(muk, sqrt(sigmaE/denom)) noise
      if (HS) Lp[pos] = 1.0 / dsel;                 // RN(1/D) for the chain's quotient
    }
    const uint64_t bal = __ballot(likely);
    if (lane == 0) misc[wv] = __popcll(bal);
    if (defer_dma) lds_barrier(); else __syncthreads();
    int pre = base;
    for (int w = 0; w < wv; ++w) pre += misc[w];
    if (pos < bs) {
      const int idx = pre + __popcll(bal & ((1ull << lane) - 1ull));
      const int sl = likely && idx < nst ? idx : -1;
      Lslot[pos] = sl;
      if (likely) Lspos[idx] = pos;
    }
    for (int w = 0; w < NW; ++w) base += misc[w];
    if (defer_dma) lds_barrier(); else __syncthreads();
  }
  if (persistent) {
    // every position has read this block's dots (barrier above): the slots get the sentinel of the
    // next block that uses them -- s + NPAR in this sweep, else block s % NPAR of the next sweep (its
    // reducer can only write after this solver publishes later blocks, so these stores land first)
    const int nxt = s + NPAR < d.nb ? d.sbase + s + NPAR : d.sbase + d.nb + s % NPAR;
    const unsigned long long ns = slab_sentinel(nxt);
    double *slab2w = d.slab2 + par * d.slab2_stride;
    for (int i = t; i < d.NG * B; i += NT) st_sc1_u64(slab2w + i, ns);
  }
  const int nused = resident ? 0 : min(base, nst);  // resident: every row is in LDS already
  const int nov = max(base - nst, 0);  // predicted positions served by the ring
  const int npred = base;
  if (t == 0) {
    *Lcons = 0;
    for (int k = 0; k < RS; ++k) Lready[k] = 0;
  }
  if (prof) tp1 = wall_clock64();
  // 2) stage the predicted positions' Gram rows (8 double2 loads in flight per thread)
  {
    const double2 *G2 = reinterpret_cast<const double2 *>(d.gram + (int64_t)gb * B * B);
    double2 *S2 = reinterpret_cast<double2 *>(slots);
    constexpr int H = B / 2;
    const int tot = nused * H;
    for (int e0 = 0; e0 < tot; e0 += NT * 8) {
      double2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = min(e0 + u * NT + t, tot - 1);
        v[u] = G2[(int64_t)Lgi[Lspos[e / H]] * H + (e % H)];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + u * NT + t < tot) S2[e0 + u * NT + t] = v[u];
    }
  }
  if (defer_dma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the copying waves' Gram pieces landed
  __syncthreads();
  if (prof) tp2 = wall_clock64();
  const uint64_t tc2 = prof ? __builtin_amdgcn_s_memtime() : 0;  // shader clock (diagnostics)
  // 3) serial chain on wave 0; lane l owns positions l*NS .. l*NS+NS-1.  Per position: the
  //    current num (r), its decision window [lo, hi] in num^2, and two bits: act (the decision
  //    changes beta, or needs the exact formula) and win (num^2 inside the window).  The next
  //    position to visit is the lowest one with act or !win; runs of unchanged positions in
  //    between are committed as they are.  A position found outside its window is re-decided
  //    at its current num (wave-uniform) and re-examined.  A visited position's new beta is
  //    computed wave-uniformly and every later position subtracts G_ji * delta.
  if (resident) {
    if (t < 64) {
      if constexpr (HS) {
        const uint64_t tq0 = prof ? __builtin_amdgcn_s_memtime() : 0;
#if BRR_CHAIN_INLINE
        chain_hs_blocked<B>(bs, Lr0, Ldsel, Lsdz, Lbo, Lbn, Lgi, slots);
#else
        chain_hs_call<B>(bs, to_lds(Lr0), to_lds(Ldsel), to_lds(Lsdz), to_lds(Lbo), to_lds(Lbn), to_lds(Lgi),
                         to_lds(slots));
#endif
        if (prof && lane == 0) {
          atomicAdd(&d.sc->prof[6], (unsigned long long)bs);
          atomicAdd(&d.sc->prof[12], (unsigned long long)(__builtin_amdgcn_s_memtime() - tq0));  // chain loop, shader clocks
        }
      } else {
#if BRR_CHAIN_BLK
        chain_bayesr_resident_blk<B>(d, bs, sigmaE, Lr0, Llo, Lhi, Ldsel, Lsdz, Lbo, Lbn, Lfl, Lks, Lgi, La, Lden, Lp,
                                     Lx2, Lz, Lm, slots, prof);
#elif BRR_CHAIN_INLINE || !BRR_BAYESR_CHAIN_CALL
        chain_bayesr_resident<B>(d, bs, sigmaE, Lr0, Llo, Lhi, Ldsel, Lsdz, Lbo, Lbn, Lfl, Lks, Lgi, La, Lden, Lp,
                                 Lx2, Lz, Lm, slots, prof);
#else
        chain_bayesr_call<B>(d, bs, sigmaE, to_lds(Lr0), to_lds(Llo), to_lds(Lhi), to_lds(Ldsel), to_lds(Lsdz),
                             to_lds(Lbo), to_lds(Lbn), to_lds(Lfl), to_lds(Lks), to_lds(Lgi), to_lds(La), to_lds(Lden),
                             to_lds(Lp), to_lds(Lx2), to_lds(Lz), to_lds(Lm), to_lds(slots), prof);
#endif
      }
    }
  } else if (HS && t < 64) {
    // Horseshoe: every position changes (beta ~ N(num/D, sigmaE/D), HorseshoeR.cpp:226-234), so
    // the chain is a forward substitution through the block in position order.  The owner lane
    // of position j forms beta_j, the wave reads delta_j back from it and every later position
    // subtracts G_jk delta_j -- the same operations, in the same order, as the general chain.
    // The next step's Gram values are gathered one step ahead, off the dependency chain.
    // num / D on the chain: q0 = num * RN(1/D), one exact-remainder correction (Markstein) --
    // the correctly rounded quotient, in three dependent operations instead of the division
    // sequence; RN(1/D) is formed in step 1.  The position's constants are read from LDS one
    // step ahead (wave-uniform addresses); only num and the Gram values live in registers.
    // Layout: lane l holds positions l + 64 q, so the owner's register index is a constant of
    // the unrolled outer loop (no dynamically indexed register arrays).
    double r[NS], gn[NS];
    int gg[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const int pos = lane + 64 * q;
      const bool in = pos < bs;
      r[q] = in ? Lr0[pos] : 0.0;
      gg[q] = in ? Lgi[pos] : 0;
    }
    const double *Ggl = d.gram + (int64_t)gb * B * B;
    // every row in LDS (slot j = position j: all positions are predicted to change) -> LDS
    // loads only; otherwise rows without a static slot come through the ring (or global memory)
    auto chain = [&](auto all_lds) __attribute__((always_inline)) {
      constexpr bool ALL = decltype(all_lds)::value;
      auto row_of = [&](int j) __attribute__((always_inline)) -> const double * {
        if constexpr (ALL) {
          return slots + (int64_t)j * B;
        } else {
          const int sl = Lslot[j];
          if (sl >= 0) return slots + (int64_t)sl * B;
          // every position is predicted: position j >= nst is ring entry j - nst
          if (RS > 0 && ring_take(Lcons, Lready, RS, j - nst)) return slots + (int64_t)(nst + (j - nst) % RS) * B;
          return Ggl + (int64_t)Lgi[j] * B;
        }
      };
      double nd = Ldsel[0], ni = Lp[0], nz = Lsdz[0], nbo = Lbo[0];
      {
        const double *g0 = row_of(0);
#pragma unroll
        for (int q = 0; q < NS; ++q) gn[q] = g0[gg[q]];
      }
#pragma unroll
      for (int qo = 0; qo < NS; ++qo) {
        const int jend = min(bs, 64 * (qo + 1));
        for (int j = 64 * qo; j < jend; ++j) {
          const double dv = nd, iv = ni, zv = nz, bv = nbo;
          double gc[NS];
#pragma unroll
          for (int q = 0; q < NS; ++q) gc[q] = gn[q];
          if (j + 1 < bs) {
            nd = Ldsel[j + 1]; ni = Lp[j + 1]; nz = Lsdz[j + 1]; nbo = Lbo[j + 1];
            const double *g1 = row_of(j + 1);
#pragma unroll
            for (int q = 0; q < NS; ++q) gn[q] = g1[gg[q]];
          }
          const double rv = r[qo];
          const double q0 = rv * iv;
          const double quo = __builtin_fma(__builtin_fma(-q0, dv, rv), iv, q0);  // = num / D
          const double bn = quo + zv;  // HorseshoeR.cpp:234
          const double delta = readlane_f64(bn - bv, j - 64 * qo);
          if (lane == j - 64 * qo) Lbn[j] = bn;
#pragma unroll
          for (int q = qo; q < NS; ++q)
            if (lane + 64 * q > j) r[q] = r[q] - gc[q] * delta;
        }
      }
    };
    if (nused >= bs) chain(std::true_type{});
    else chain(std::false_type{});
    if (lane == 0) lds_st_rel(Lcons, RING_DONE);
    if (prof && lane == 0) atomicAdd(&d.sc->prof[6], (unsigned long long)bs);
  } else if (!HS && t < 64) {
    chain_bayesr_rows<B>(d, bs, sigmaE, Lr0, Llo, Lhi, Ldsel, Lsdz, Linv, Lbo, Lbn, Lfl, Lks, Lgi, La, Lden, Lp, Lx2, Lz, Lm,
                         Lslot, Lspos, slots, d.gram + (int64_t)gb * B * B, RS, nst, nov, npred, Lcons, Lready, prof);
    if (prof) tce = wall_clock64();
  } else if (RS > 0 && nov > 0) {
    ring_produce<B, NW>(d.gram + (int64_t)gb * B * B, Lgi, Lspos, nst, nov, slots + (int64_t)nst * B, RS, Lcons,
                        Lready);
  }
  __syncthreads();
  if (prof) tp3 = wall_clock64();
  const uint64_t tc3 = prof ? __builtin_amdgcn_s_memtime() : 0;
  if (BRR_EARLY_GRAM && pipelined && s + 1 < d.seg1) {
    // this block's coefficients are no longer read: the upper half of the waves starts copying
    // the next block's Gram block into LDS, in flight during the write-back and the next block's
    // constants and cross-Gram loads.  (Measured slower: every barrier of the write-back then waits
    // for the copy -- a workgroup barrier retires outstanding LDS-DMA -- so it is off by default.)
    if (wv >= NW / 2) {
      constexpr int NCHUNK = B * B * 8 / 1024;
      const char *src = reinterpret_cast<const char *>(d.gram + (int64_t)d.gblk[s + 1] * B * B);
      char *dst = reinterpret_cast<char *>(slots);
      for (int c = wv - NW / 2; c < NCHUNK; c += NW / 2)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + c * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void *)(dst + c * 1024), 16, 0, 0);
    }
    if (t == 0) misc[12] = s + 1;
  }
  // 4) write back, compact the changed markers into this block's list in Gram-index (storage) order: a
  //    list holding every position (the Horseshoe's) is then the block's columns in storage order, which
  //    the streamers' apply reads 16 at a time from their code tiles (apply_pending); every consumer
  //    (apply, cross-Gram corrections) sums a list in list order
  int *Lpg = Lspos;  // the position of each Gram index (the chain's prediction list is no longer read)
  for (int pos = t; pos < bs; pos += NT) Lpg[Lgi[pos]] = pos;
  __syncthreads();
  const int pslot = s % NSLOT;
  int *pidx = d.pend_idx + pslot * d.pend_stride, *pgi = d.pend_gi + pslot * d.pend_stride;
  int *ppos = d.pend_pos + pslot * d.pend_stride;
  double *pbo = d.pend_bo + pslot * d.pend_stride, *pbn = d.pend_bn + pslot * d.pend_stride;
  base = 0;
#pragma unroll
  for (int c = 0; c < NPT; ++c) {
    const int gi = t + NT * c;  // (Lgi is a permutation of 0 .. bs - 1)
    const int pos = gi < bs ? Lpg[gi] : 0;
    int changed = 0;
    double bnv = 0.0, bov = 0.0;
    int m = 0;
    if (gi < bs) {
      m = Lm[pos];
      bnv = Lbn[pos];
      bov = Lbo[pos];
      changed = bnv != bov;
    }
    const uint64_t bal = __ballot(changed);
    if (lane == 0) misc[wv] = __popcll(bal);
    __syncthreads();
    int pre = base;
    for (int w = 0; w < wv; ++w) pre += misc[w];
    if (changed) {
      const int idx = pre + __popcll(bal & ((1ull << lane) - 1ull));
      st_sc1_int(pidx + idx, m);
      st_sc1_int(pgi + idx, gi);
      st_sc1_int(ppos + idx, pos);
      st_sc1(pbo + idx, bov);
      st_sc1(pbn + idx, bnv);
      if (nlb > 0) {  // the next blocks' cross-Gram corrections read it from LDS (phase A)
        Llist[(int64_t)(s % nlb) * (B + 16) + idx] = bnv - bov;
        Lligi[(int64_t)(s % nlb) * (B + 16) + idx] = gi;
      }
    }
    for (int w = 0; w < NW; ++w) base += misc[w];
    __syncthreads();
  }
  const int npend = base;
  const int npad = (npend + 15) & ~15;  // lists are read in batches of 8 / 16
  if (nlb > 0) {
    if (npend + t < npad) {
      Llist[(int64_t)(s % nlb) * (B + 16) + npend + t] = 0.0;
      Lligi[(int64_t)(s % nlb) * (B + 16) + npend + t] = 0;
    }
    if (t == 0) { misc[16 + 2 * (s % nlb)] = npad; misc[17 + 2 * (s % nlb)] = s; }
  }
  if (npend + t < npad) {  // neutral padding: eps + x*0 - x*0 == eps exactly, delta = 0
    st_sc1_int(pidx + npend + t, 0);
    st_sc1_int(pgi + npend + t, 0);
    st_sc1_int(ppos + npend + t, 0);
    st_sc1(pbo + npend + t, 0.0);
    st_sc1(pbn + npend + t, 0.0);
  }
  if (t == 0) {
    st_sc1_int(d.pend_n + pslot, npad);
    st_sc1_int(d.pend_n + NSLOT + pslot, npend);
  }
  // publish: every storing wave drains its sc1 stores, then the block count (k_stream(s+2)).  The
  // stores above come from the position threads (t < B) only; with B <= NT / 2 the upper half of
  // the waves stored nothing and must not wait here for the next block's Gram copy it started
  if (!(pipelined && B <= NT / 2 && wv >= NW / 2)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __hip_atomic_store(d.sync + SY_PEND, d.sbase + s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 0) stamp(d.sync, 5);
    if (npend) atomicAdd(&d.sc->n_changed, (unsigned long long)npend);
    if (prof) {
      const uint64_t tp4 = wall_clock64();
      unsigned long long *tr = d.trace + (int64_t)s * 16;
      tr[TR_SOLVE0] = tp0; tr[TR_GDONE_SEEN] = tw; tr[TR_CHAIN] = tp3; tr[TR_PUB] = tp4;
      atomicAdd(&d.sc->prof[0], (unsigned long long)(tp1 - tw));
      atomicAdd(&d.sc->prof[1], (unsigned long long)(tp2 - tp1));
      atomicAdd(&d.sc->prof[2], (unsigned long long)(tp3 - tp2));
      atomicAdd(&d.sc->prof[3], (unsigned long long)(tp4 - tp3));
      atomicAdd(&d.sc->prof[5], 1ull);
      atomicAdd(&d.sc->prof[10], (unsigned long long)(tw - tp0));
      atomicAdd(&d.sc->prof[13], (unsigned long long)(tA1 - tp0));
      atomicAdd(&d.sc->prof[14], (unsigned long long)(tA2 - tA1));
      atomicAdd(&d.sc->prof[15], (unsigned long long)(tA3 - tA2));
      atomicAdd(&d.sc->prof[11], (unsigned long long)(tc3 - tc2));
      if (tce) atomicAdd(&d.sc->prof[17], (unsigned long long)(tp3 - tce));  // chain end -> all waves past it
      atomicAdd(&d.sc->prof[18], (unsigned long long)nov);                     // rows served by the ring
      atomicAdd(&d.sc->prof[19], (unsigned long long)npred);                   // positions predicted to change
    }
  }
  // the block's state for later sweeps (beta, comp, sel: BayesRv2.cpp:226-245) after the publish: off
  // the streamers' path (the drain above covers the change list only); these stores retire at the
  // wave's next vmcnt wait, the next block's phase A, and before the sweep's k_markers
#pragma unroll
  for (int c = 0; c < NPT; ++c) {
    const int pos = t + NT * c;
    if (pos < bs) {
      const int m = Lm[pos];
      d.beta[m] = Lbn[pos];
      if (!HS) {
        const int ks = Lks[pos];
        if (ks != FALLTHROUGH) d.comp[m] = ks;
        d.sel[m] = ks != FALLTHROUGH;
      }
    }
  }
}

template <bool HS, int B>
__global__ __launch_bounds__(256) void k_solve(Dev d, int s, uint32_t it, int nslot) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  solve_block<HS, B, 256>(d, s, it, nslot, smem, false, d.lag);
}


// ------------------------------------------------------------------------------------
// k_sweep: the whole marker loop of a sweep in ONE persistent launch.  Workgroup 0 is the
// solver (solve_block for s = 0..nb-1); workgroups 1..nsg stream; the last nred reduce.  Every
// workgroup has its own CU (the solver's LDS needs it), all are resident (census at the
// start), so the device counters of the lag-1 hand-over can be waited on (bounded).
//
// Streaming workgroup g owns the rows [g rpw, min(N, (g+1) rpw)) for the whole sweep (rpw a
// multiple of 4, so every workgroup has the same work) and keeps their residual in LDS, in
// npass passes of 256 rows (lane = 4 consecutive rows, 16-B loads).  Its 8 waves split the
// block's columns (B/8 each).  Per block s it applies block s-2's changes (after the solver's
// counter says they are published), forms the partial dots X_s^T E_{s-1} of its rows in
// (chunk, pass) items of CW columns per wave and publishes them (one slab row per workgroup,
// one arrival per block on its group's counter).  The next item's X loads, across block
// boundaries, are issued before the current item is consumed, so HBM stays busy while a
// workgroup waits.  At the end it applies the last two blocks' changes and writes eps back.
constexpr int SWEEP_NT = 512;
constexpr int SWEEP_NW = SWEEP_NT / 64;
#ifndef STREAM_CW
#define STREAM_CW 16  // columns per streaming item and wave
#endif
#ifndef STREAM_P
#define STREAM_P 1    // items in flight ahead of the one being consumed (2+ spills at CW = 16)
#endif
#ifndef STREAM_P2
#define STREAM_P2 3   // the same for 2-bit code tiles (one 16-byte load per item and lane; P + 1 = 4
                      // divides a 512-column block's items, so the static ring applies)
#endif
#ifndef BRR_STATIC_RING
#define BRR_STATIC_RING 1  // stream_role: the ring unrolled by its length where it divides a block's items
#endif
// streaming workgroups (slab rows) per level-2 reduction group: 64 -> 4 reducer workgroups at C2
// (16 / 32 / 64 measured 27.1 / 27.6 / 28.1 sweeps/s: fewer reducers, fewer slab2 rows for the
// solver to sum; 64 doubles per reducer thread is the register limit of the unrolled sum)
#ifndef FUSED_GROUP_N
#define FUSED_GROUP_N 64
#endif
constexpr int FUSED_GROUP = FUSED_GROUP_N;

// Block `slot`'s change list applied to this workgroup's residual rows (BayesRv2.cpp:191,243):
//     eps_i += sum_c x_ic (b_old_c - b_new_c)
// Lane = 4 consecutive rows (one 16-B load per column, as the stream reads them; 2-bit storage:
// one code byte), so a wave-instruction covers a 256-row pass.  The 8 waves split the passes,
// and when there are fewer than 8 passes also the list: wave w takes pass w % npass and the
// contiguous part w / npass of G = 8 / npass parts of the list (npass >= 8: every wave takes
// whole passes with the whole list).  Each wave keeps two batches of AB column loads in flight
// and sums its part in list order; the parts are added to eps in part order through LDS
// (s_part), so the result does not depend on timing.  (Round 1 loaded one 4-B value per lane
// and column, 16 in flight: the apply of a 128-change list took 11-18 us of HBM latency.)
// msrc != nullptr: also copy the B member indices at msrc to mdst (LDS); loaded before the first
// barrier, stored after the last (the buffer's previous block is then no longer read by any wave).
// ccode != nullptr (2-bit storage): the code bytes of the block being applied are in LDS
// (stream_role's code cache, tiles [group][row quad][16]); s_ppos receives the in-block indices.
// 2-bit storage: lsrc / ldst stage the next block's value tables (storage order, lcnt valid
// entries, f32 in HBM -> 4 doubles per column in LDS) the same way; lutb = the value tables of
// the block being applied (LDS, 4 doubles per column, by visit position).
#ifndef BRR_APPLY_AB
#define BRR_APPLY_AB 4
#endif
// Parts of a change list of np entries (padded length): a list of at most 16 entries -- the steady
// state's, a few real ones plus padding -- is applied by one wave per pass (no cross-wave sum and
// its barrier); a longer one in SWEEP_NW / npass parts per pass.  Every path applies a list the same
// way, so the residual does not depend on the storage or on whether the list was prefetched.
#ifndef BRR_DENSE_PIPE
#define BRR_DENSE_PIPE 1  // (class-code cache) the dense apply's whole groups software-pipelined (0: one pair at a time)
#endif
#ifndef BRR_APPLY_SMALL
#define BRR_APPLY_SMALL 16
#endif
// (The split is defined over APPLY_NW = 8 waves whatever the streaming workgroup's width: a wider
// workgroup's extra waves take whole passes of one-part lists or sit a long list out, so a residual
// row sees the same operations in the same order under every streamer geometry.)
constexpr int APPLY_NW = 8;
// Uniform integer division by a small run-time divisor in the apply: a scalar loop (the compiler's
// expansion goes through a VALU reciprocal whose loop-invariant constants it hoists into VGPRs).
__device__ __forceinline__ int small_div(int x, int d, int *rem) {  // x >= 0, d >= 1 uniform, x / d small
  int q = 0;
  while (x >= d) { x -= d; ++q; }
  *rem = x;
  return q;
}
__device__ __forceinline__ int apply_nparts(int np, int npass) {
  int r;
  return (npass >= APPLY_NW || np <= BRR_APPLY_SMALL) ? 1 : small_div(APPLY_NW, npass, &r);
}
// (G = 8 / npass is 8, 4, 2 or 1: the part bounds np part / G are shifts)
__device__ __forceinline__ int part_bound(int np, int part, int G) { return (np * part) >> (31 - __builtin_clz(G)); }
template <int XF, int NT = SWEEP_NT>
__device__ __forceinline__ void apply_pending(const Dev &d, int slot, int64_t r0, int64_t r1, int npass,
                                              double *eps_l, int *s_pidx, double *s_pbo, double *s_pbn,
                                              int *s_np, double *s_part, const int *msrc = nullptr,
                                              int *mdst = nullptr, const uint8_t *ccode = nullptr,
                                              int *s_ppos = nullptr, const float4 *lsrc = nullptr,
                                              double *ldst = nullptr, const double *lutb = nullptr, int lcnt = 0,
                                              uint64_t *ptime = nullptr, double *s_w = nullptr) {
#pragma clang fp contract(off)
  // diagnostics (ptime, thread 0): [0] += list staging incl. its barrier, [1] += this wave's
  // products, [2] += the wait for the other waves' parts, [3] += the staging stores and the last
  // barrier (bench.py --profile-solve: wg_apply_{list,products,partbar,stage}_ms_pct)
  const uint64_t tq0 = ptime ? wall_clock64() : 0;
  constexpr int AB = BRR_APPLY_AB;  // columns per batch (two batches in flight: 8 KiB per wave, 32 VGPRs, as many as the
                         // streaming ring leaves without spills)
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool mcopy = msrc != nullptr && t < d.B;
  const int mval = mcopy ? msrc[t] : 0;
  const bool lcopy = XF && lsrc != nullptr && t < d.B;
  const float4 lval = (lcopy && t < lcnt) ? lsrc[t] : make_float4(0.f, 0.f, 0.f, 0.f);
  double *s_pd = s_pbo;  // b_old - b_new per list entry
  // 2-bit: per entry the offset of its code byte at row quad 0 -- in the LDS code cache (tiles of
  // this workgroup's rows) or in the HBM code tiles -- so a lane adds only its quad
  int64_t *s_cb = reinterpret_cast<int64_t *>(s_pbn);
  if (t < 64) {
    const int *pidx = d.pend_idx + slot * d.pend_stride;
    const double *pbo = d.pend_bo + slot * d.pend_stride, *pbn = d.pend_bn + slot * d.pend_stride;
    // one round trip for the counts and every lane's first entry together (the list arrays hold
    // at least B >= 64 entries, so entry `lane` is always addressable; entries past np are unused)
    const int np = ld_sc1_int(d.pend_n + slot);
    const int nr = ld_sc1_int(d.pend_n + NSLOT + slot);  // entries before the neutral padding
    int col0 = ld_sc1_int(pidx + lane);
    int gi0 = XF ? ld_sc1_int(d.pend_gi + slot * d.pend_stride + lane) : 0;
    const double pd0 = ld_sc1(pbo + lane) - ld_sc1(pbn + lane);
    // (B >= 128) entries 64 + lane in the same round trip, before the counts are known (the arrays hold
    // B + 16 entries): a Horseshoe list -- every column of its block -- is staged in one round trip, not two
    const bool two = d.B >= 128;
    int col1 = two ? ld_sc1_int(pidx + 64 + lane) : 0;
    int gi1 = (XF && two) ? ld_sc1_int(d.pend_gi + slot * d.pend_stride + 64 + lane) : 0;
    const double pd1 = two ? ld_sc1(pbo + 64 + lane) - ld_sc1(pbn + 64 + lane) : 0.0;
    {
      // neutral padding entries (e >= nr: b_old = b_new = 0) take the last real entry's column: a
      // cache hit instead of column 0 from HBM, and no branch in the batched loads
      const int last = max(nr - 1, 0);
      const int lc0 = __shfl(col0, last & 63), lc1 = __shfl(col1, last & 63);
      const int lg0 = XF ? __shfl(gi0, last & 63) : 0, lg1 = XF ? __shfl(gi1, last & 63) : 0;
      const int lcol = last < 64 ? lc0 : lc1, lgi = last < 64 ? lg0 : lg1;
      auto stage = [&](int e, int col, int gi, double pd) __attribute__((always_inline)) {
        if (e >= nr) { col = lcol; gi = lgi; }
        s_pidx[e] = col;
        if (XF) {
          s_ppos[e] = gi;
          s_cb[e] = ccode ? (int64_t)(gi >> 4) * (npass * 64 * 16) + (gi & 15) : code_off(col, 0, d.B, d.ldc);
        }
        s_pd[e] = pd;
      };
      if (lane < np) stage(lane, col0, gi0, pd0);
      if (two && 64 + lane < np) stage(64 + lane, col1, gi1, pd1);
    }
    for (int e = lane + (two ? 128 : 64); e < np; e += 64) {
      // neutral padding entries (b_old = b_new = 0) load the last real column again: a cache
      // hit instead of column 0 from HBM, and no branch in the batched loads
      const int es = e < nr ? e : max(nr - 1, 0);
      const int col = ld_sc1_int(pidx + es);
      s_pidx[e] = col;
      const double pde = ld_sc1(pbo + e) - ld_sc1(pbn + e);
      if (XF) {
        const int gi = ld_sc1_int(d.pend_gi + slot * d.pend_stride + es);  // in-block (storage) index
        s_ppos[e] = gi;
        s_cb[e] = ccode ? (int64_t)(gi >> 4) * (npass * 64 * 16) + (gi & 15) : code_off(col, 0, d.B, d.ldc);
      }
      s_pd[e] = pde;
    }
    // (table storage) dense: the list is the block's first nr columns in storage order -- the
    // Horseshoe's every block (the solver writes lists in storage order, solve_block)
    bool dn = true;
    if (XF)
      for (int e = lane; e < nr; e += 64) dn = dn && s_ppos[e] == e;
    const bool dense_l = XF && __ballot(!dn) == 0;
    if (lane == 0) { s_np[0] = np; s_np[1] = nr | (dense_l ? 1 << 30 : 0); }
  }
  __syncthreads();
  const int np = __builtin_amdgcn_readfirstlane(s_np[0]);
  const int nr_d = __builtin_amdgcn_readfirstlane(s_np[1]);
  const int nr = nr_d & ((1 << 30) - 1);
  const bool dense = XF && (nr_d >> 30) != 0;
  if (XF && np > 0) {
    // the pair tables, by every thread: entries 2q and 2q + 1 add W[c0 | c1 << 2] = (x0(c0) d0) + (x1(c1) d1)
    // per row, the f32 path's (x0 d0 + x1 d1) (the same rounded products, then the same adds); an entry
    // without a real partner (2q + 1 >= nr) adds x0(c0) d0 alone, as the f32 path does
    for (int i = t; i < 8 * np; i += NT) {
      const int e = 2 * (i >> 4), c0 = i & 3, c1 = (i >> 2) & 3;
      const double w0 = lutb[4 * s_ppos[e] + c0] * s_pd[e];
      s_w[i] = e + 1 >= nr ? w0 : w0 + lutb[4 * s_ppos[e + 1] + c1] * s_pd[e + 1];
    }
    __syncthreads();
  }
  const uint64_t tq1 = ptime ? wall_clock64() : 0;
  const int G = apply_nparts(np, npass);  // parts of the list
  const int ldp = npass * SROWS;                          // doubles per part in s_part
  if (np > 0) {
    int wr;
    const int wq = small_div(w, npass, &wr);
    const int p0 = G == 1 ? w : wr, part = G == 1 ? 0 : wq;
    const int pstep = G == 1 ? NT / 64 : npass;  // (G > 1: one pass per wave)
    const int e0 = part < G ? part_bound(np, part, G) : np, e1 = part < G ? part_bound(np, part + 1, G) : np;
    // the part's real entries: the neutral padding's products are exact zeros and are skipped
    const int ee = min(e1, nr);
    for (int p = p0; p < npass && e0 < e1; p += pstep) {
      const int off = p * SROWS + 4 * lane;  // this lane's 4 rows, relative to r0
      const bool ok = r0 + off < r1;
      const int64_t src = ok ? r0 + off : r0;  // lanes past the rows re-read row r0 (not stored)
      auto xload = [&](int e) __attribute__((always_inline)) -> float4 {
        return ldg4(d.X + (int64_t)s_pidx[e] * d.ld + src);
      };
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      if constexpr (XF) {
        // table storage: per pair of entries one LDS read and one add per row (the pair tables).  The
        // byte of (entry e, this lane's quad) from LDS (code cache) or HBM in separate loops (concrete
        // address spaces).
        auto pair_load = [&](uint32_t b0, uint32_t b1, int e, double (&wv)[4]) __attribute__((always_inline)) {
          const double *wq = s_w + 8 * e;  // (e even: the tables of pair e / 2)
          const uint32_t m = b0 | (b1 << 8);
          wv[0] = wq[__builtin_amdgcn_ubfe(m, 0, 2) | (__builtin_amdgcn_ubfe(m, 8, 2) << 2)];
          wv[1] = wq[__builtin_amdgcn_ubfe(m, 2, 2) | (__builtin_amdgcn_ubfe(m, 10, 2) << 2)];
          wv[2] = wq[__builtin_amdgcn_ubfe(m, 4, 2) | (__builtin_amdgcn_ubfe(m, 12, 2) << 2)];
          wv[3] = wq[__builtin_amdgcn_ubfe(m, 6, 2) | (__builtin_amdgcn_ubfe(m, 14, 2) << 2)];
        };
        auto pair_add = [&](uint32_t b0, uint32_t b1, int e) __attribute__((always_inline)) {
          double wv[4];
          pair_load(b0, b1, e, wv);
          a0 = a0 + wv[0];
          a1 = a1 + wv[1];
          a2 = a2 + wv[2];
          a3 = a3 + wv[3];
        };
        auto run = [&](auto lds_c) __attribute__((always_inline)) {
          constexpr bool LDSC = decltype(lds_c)::value;
          const int64_t qo = LDSC ? (int64_t)(off >> 2) * 16 : (src >> 2) * 16;
          if (e0 >= ee) return;
          if (dense) {
            // the list is the block's first nr columns in storage order: entries 16 g .. 16 g + 15 are
            // one 16-byte code group at this lane's quad (1 read for 16 entries instead of 2 per entry)
            auto gload = [&](int gq) __attribute__((always_inline)) -> uint4 {
              if constexpr (LDSC) {
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(
                    (const __attribute__((address_space(3))) uint8_t *)ccode + s_cb[16 * gq] + qo);
                return make_uint4(v.x, v.y, v.z, v.w);
              } else
                return *reinterpret_cast<const uint4 *>(d.Xc + s_cb[16 * gq] + qo);
            };
            const int g1 = (ee - 1) >> 4;
            uint4 cur = gload(e0 >> 4);
            auto byte_of = [&](const uint4 &c, int k) __attribute__((always_inline)) -> uint32_t {  // k static
              const uint32_t word = k < 4 ? c.x : (k < 8 ? c.y : (k < 12 ? c.z : c.w));
              return __builtin_amdgcn_ubfe(word, 8 * (k & 3), 8);
            };
            for (int gq = e0 >> 4; gq <= g1; ++gq) {
              const uint4 nxt = gload(min(gq + 1, g1));
              if (BRR_DENSE_PIPE && XF == 2 && 16 * gq >= e0 && 16 * gq + 16 <= ee) {
                // a whole group, software-pipelined: pair j + 1's table reads are issued before pair
                // j's adds (a scheduling barrier keeps them there; without it the reads issue one at
                // a time under the prefetch ring's register pressure)
                double wv[4], wn[4];
                pair_load(byte_of(cur, 0), byte_of(cur, 1), 16 * gq, wv);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  if (j + 1 < 8) pair_load(byte_of(cur, 2 * j + 2), byte_of(cur, 2 * j + 3), 16 * gq + 2 * j + 2, wn);
                  __builtin_amdgcn_sched_barrier(0);
                  a0 = a0 + wv[0];
                  a1 = a1 + wv[1];
                  a2 = a2 + wv[2];
                  a3 = a3 + wv[3];
                  if (j + 1 < 8) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) wv[k] = wn[k];
                  }
                }
              } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  const int e = 16 * gq + 2 * j;
                  if (e >= e0 && e < ee) pair_add(byte_of(cur, 2 * j), byte_of(cur, 2 * j + 1), e);
                }
              }
              cur = nxt;
            }
            return;
          }
          auto rload = [&](int e) __attribute__((always_inline)) -> uint32_t {
            if constexpr (LDSC)
              return ((const __attribute__((address_space(3))) uint8_t *)ccode)[s_cb[e] + qo];
            else if (d.Xcm)  // (the column-major copy: 64 contiguous bytes per wave instead of 64 tile granules)
              return d.Xcm[(int64_t)s_pidx[e] * d.ldc + (src >> 2)];
            else
              return d.Xc[s_cb[e] + qo];
          };
          // raw code bytes in flight (2 batches of AB entries, AB even: whole pairs), decoded when
          // consumed; a pair's second byte past ee is read clamped and not used (its table is the
          // first entry's alone)
          uint32_t ra[AB], rb[AB];
          auto consume = [&](const uint32_t (&r)[AB], int e) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < AB; q += 2)
              if (e + q < ee) pair_add(r[q], r[q + 1], e + q);
          };
#pragma unroll
          for (int q = 0; q < AB; ++q) ra[q] = rload(min(e0 + q, ee - 1));
          for (int e = e0; e < ee; e += 2 * AB) {
            const bool more = e + AB < ee;
            if (more) {
#pragma unroll
              for (int q = 0; q < AB; ++q) rb[q] = rload(min(e + AB + q, ee - 1));
            }
            consume(ra, e);
            if (!more) break;
            if (e + 2 * AB < ee) {
#pragma unroll
              for (int q = 0; q < AB; ++q) ra[q] = rload(min(e + 2 * AB + q, ee - 1));
            }
            consume(rb, e + AB);
          }
        };
        if (ccode) run(std::true_type{});
        else run(std::false_type{});
      } else {
      float4 xa[AB], xb[AB];
      auto consume = [&](const float4 (&x)[AB], int e) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < AB; q += 2) {
          // pairs of entries: (x0 d0 + x1 d1) per row, then the add (rounded products: the table
          // storages' pair tables); an entry without a partner in the part alone
          if (e + q + 1 < ee) {
            const double d0 = s_pd[e + q], d1 = s_pd[e + q + 1];
            a0 = a0 + ((double)x[q].x * d0 + (double)x[q + 1].x * d1);
            a1 = a1 + ((double)x[q].y * d0 + (double)x[q + 1].y * d1);
            a2 = a2 + ((double)x[q].z * d0 + (double)x[q + 1].z * d1);
            a3 = a3 + ((double)x[q].w * d0 + (double)x[q + 1].w * d1);
          } else if (e + q < ee) {
            const double d0 = s_pd[e + q];
            a0 = a0 + (double)x[q].x * d0;
            a1 = a1 + (double)x[q].y * d0;
            a2 = a2 + (double)x[q].z * d0;
            a3 = a3 + (double)x[q].w * d0;
          }
        }
      };
      if (e0 < ee) {
#pragma unroll
      for (int q = 0; q < AB; ++q) xa[q] = xload(min(e0 + q, ee - 1));
      for (int e = e0; e < ee; e += 2 * AB) {
        const bool more = e + AB < ee;
        if (more) {
#pragma unroll
          for (int q = 0; q < AB; ++q) xb[q] = xload(min(e + AB + q, ee - 1));
        }
        consume(xa, e);
        if (!more) break;
        if (e + 2 * AB < ee) {
#pragma unroll
          for (int q = 0; q < AB; ++q) xa[q] = xload(min(e + 2 * AB + q, ee - 1));
        }
        consume(xb, e + AB);
      }
      }
      }
      if (G == 1) {
        if (ok) {
          double *ep = eps_l + off;
          ep[0] = ep[0] + a0;
          ep[1] = ep[1] + a1;
          ep[2] = ep[2] + a2;
          ep[3] = ep[3] + a3;
        }
      } else {
        double *pp = s_part + (int64_t)part * ldp + off;
        pp[0] = a0;
        pp[1] = a1;
        pp[2] = a2;
        pp[3] = a3;
      }
    }
    const uint64_t tq2 = ptime ? wall_clock64() : 0;
    if (ptime) { ptime[0] += tq1 - tq0; ptime[1] += tq2 - tq1; }
    if (G > 1) {
      // parts without a pass (G npass < 8 waves, or an empty part) hold nothing: zero them first
      for (int pt = 0; pt < G; ++pt)
        if (part_bound(np, pt, G) == part_bound(np, pt + 1, G))
          for (int i = t; i < ldp; i += NT) s_part[pt * ldp + i] = 0.0;
      __syncthreads();
      if (ptime) ptime[2] += wall_clock64() - tq2;
      for (int i = t; i < ldp; i += NT) {
        if (r0 + i < r1) {
          double acc = s_part[i];
          for (int part = 1; part < G; ++part) acc += s_part[part * ldp + i];
          eps_l[i] = eps_l[i] + acc;
        }
      }
    }
  }
  const uint64_t tq4 = ptime ? wall_clock64() : 0;
  if (mcopy) mdst[t] = mval;
  if (lcopy) {
    double *l = ldst + 4 * t;
    l[0] = lval.x; l[1] = lval.y; l[2] = lval.z; l[3] = lval.w;
  }
  __syncthreads();
  if (ptime) ptime[3] += wall_clock64() - tq4;
}

// The part (pass, entry range) of a change list of np entries that wave w applies (apply_pending's
// split; one pass per wave when npass <= 8, the case the prefetch serves).
struct ApplyPart {
  int p0, e0, e1;
};
__device__ __forceinline__ ApplyPart apply_part(int np, int npass, int w) {
  const int G = apply_nparts(np, npass);
  int wr;
  const int wq = small_div(w, npass, &wr);
  const int p0 = G == 1 ? w : wr, part = G == 1 ? 0 : wq;
  return {p0, part < G ? part_bound(np, part, G) : np, part < G ? part_bound(np, part + 1, G) : np};
}

// apply_pending for f32 storage when every wave of the workgroup prefetched the list during the
// previous block (stream_role's list prefetch): the list (np entries, nr real, lane e's
// b_old - b_new in lpd) is in registers and this wave's part of the columns' rows is in LDS
// (stage[(e npass + p) 256 + row], 16-B LDS-DMA of exactly the loads apply_pending would issue),
// so the boundary makes no HBM round trip.  Same parts, entry order and operations as
// apply_pending: the residual is bit-identical (the neutral padding entries, whose products are
// exact zeros, are skipped).  npass <= 8.
__device__ __forceinline__ void apply_staged(const Dev &d, int np, int nr, double lpd, int64_t r0, int64_t r1,
                                             int npass, double *eps_l, double *s_part, const float *stage,
                                             const int *msrc, int *mdst, uint64_t *ptime) {
#pragma clang fp contract(off)
  const uint64_t tq0 = ptime ? wall_clock64() : 0;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool mcopy = msrc != nullptr && t < d.B;
  const int mval = mcopy ? msrc[t] : 0;
  const int G = apply_nparts(np, npass);
  const int ldp = npass * SROWS;
  if (np > 0) {
    const ApplyPart ap = apply_part(np, npass, w);
    int wr;
    const int part = G == 1 ? 0 : small_div(w, npass, &wr);
    if (ap.p0 < npass && ap.e0 < ap.e1) {
      const int off = ap.p0 * SROWS + 4 * lane;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      const int ee = min(ap.e1, nr);
      for (int e = ap.e0; e < ee; e += 2) {  // pairs of entries, as apply_pending
        const double d0 = readlane_f64(lpd, e);
        const float4 x = *reinterpret_cast<const float4 *>(stage + ((int64_t)e * npass + ap.p0) * SROWS + 4 * lane);
        if (e + 1 < ee) {
          const double d1 = readlane_f64(lpd, e + 1);
          const float4 y = *reinterpret_cast<const float4 *>(stage + ((int64_t)(e + 1) * npass + ap.p0) * SROWS + 4 * lane);
          a0 = a0 + ((double)x.x * d0 + (double)y.x * d1);
          a1 = a1 + ((double)x.y * d0 + (double)y.y * d1);
          a2 = a2 + ((double)x.z * d0 + (double)y.z * d1);
          a3 = a3 + ((double)x.w * d0 + (double)y.w * d1);
        } else {
          a0 = a0 + (double)x.x * d0;
          a1 = a1 + (double)x.y * d0;
          a2 = a2 + (double)x.z * d0;
          a3 = a3 + (double)x.w * d0;
        }
      }
      if (G == 1) {
        if (r0 + off < r1) {
          double *ep = eps_l + off;
          ep[0] = ep[0] + a0;
          ep[1] = ep[1] + a1;
          ep[2] = ep[2] + a2;
          ep[3] = ep[3] + a3;
        }
      } else {
        double *pp = s_part + (int64_t)part * ldp + off;
        pp[0] = a0;
        pp[1] = a1;
        pp[2] = a2;
        pp[3] = a3;
      }
    }
    const uint64_t tq2 = ptime ? wall_clock64() : 0;
    if (ptime) ptime[1] += tq2 - tq0;
    if (G > 1) {
      for (int pt = 0; pt < G; ++pt)
        if (part_bound(np, pt, G) == part_bound(np, pt + 1, G))
          for (int i = t; i < ldp; i += SWEEP_NT) s_part[pt * ldp + i] = 0.0;
      __syncthreads();
      if (ptime) ptime[2] += wall_clock64() - tq2;
      for (int i = t; i < ldp; i += SWEEP_NT) {
        if (r0 + i < r1) {
          double acc = s_part[i];
          for (int pt = 1; pt < G; ++pt) acc += s_part[pt * ldp + i];
          eps_l[i] = eps_l[i] + acc;
        }
      }
    }
  }
  const uint64_t tq4 = ptime ? wall_clock64() : 0;
  if (mcopy) mdst[t] = mval;
  __syncthreads();
  if (ptime) ptime[3] += wall_clock64() - tq4;
}

// XF = 1: 2-bit genotype codes in tiles (brr_device.hpp).  A block is streamed in STORAGE order:
// item (chunk c of wave w, pass p) = the block's 16-column group w CPW / 16 + c and this lane's row
// quad, ONE 16-byte load per lane (1 KiB per wave instruction, 16 columns x 256 rows), so the
// partial dot of in-block column i lands in slab column i (the solver reads it by Gram index,
// Dev::slab_storage).  The value tables of the block being consumed are staged in LDS in storage
// order (s_lut, B entries) at each block boundary, after the previous block's last item and
// before the barrier that precedes the first item of the block.
#ifndef BRR_PF_DMA
#define BRR_PF_DMA 1  // (diagnostics: 0 compiles the f32 list prefetch out)
#endif
template <int CW, int P, int XF, int NT = SWEEP_NT, bool PROF = false>
__device__ __forceinline__ void stream_role(const Dev &d, int g, int rpw, int npass, double *eps_l, int *s_pidx,
                                            double *s_pbo, double *s_pbn, int *s_np, double *s_lut, int *s_mem,
                                            double *s_part, uint8_t *s_codes, int pfe = 0, int *s_pf = nullptr,
                                            float *s_stage = nullptr, double *s_w = nullptr) {
#pragma clang fp contract(off)
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  if (!XF && pfe > 0 && lane == 0) s_pf[w] = -1;  // (before the first barrier below)
  const int64_t r0 = (int64_t)g * rpw, r1 = min((int64_t)d.N, r0 + rpw);
  const int B = d.B, nb = d.nb;
  const int64_t ld = d.ld;
  // (the diagnostics' timers in a variant of their own: their registers cost the timed variant 46
  // spilled VGPRs at XF = 2, whose reloads in the apply wait for the whole prefetch ring)
  const bool prof = PROF && d.sc->prof_on;
  // 2-bit storage: the value tables of blocks s - 2 .. s + 1 in LDS (buffer s & 3): block s + 1's
  // are staged at boundary s (inside the apply), block s - 2's serve the apply
  const int LAG = sweep_lag(d);  // (buffer counts below are within the layout's d.lag)
  const int NLB = LAG + 3;  // value-table buffers: blocks s-1-LAG (apply) .. s+1 (staged)
  const int NCC = LAG + 2;  // code-cache buffers: blocks s-1-LAG (apply) .. s (being streamed)
  // (a column's table: its 4 f32 values as doubles, read per value by code, so a product is the
  // f32 path's (double) x * e without a decode or conversion)
  auto lut_of = [&](int s) __attribute__((always_inline)) { return s_lut + (int64_t)(s % NLB) * B * 4; };
  // XF = 2 (f32 storage, class-code cache): the class values play the value tables' part
  const float *lutsrc = XF == 2 ? d.cls_val : d.xlut;
  auto stage_lut = [&](int s) __attribute__((always_inline)) {
    if constexpr (XF) {
      const int gb = d.gblk[s], bs = d.bsz[s];
      const float4 *src = reinterpret_cast<const float4 *>(lutsrc) + (int64_t)gb * B;
      for (int i = t; i < B; i += NT) {
        const float4 l = i < bs ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        double *dl = lut_of(s) + 4 * i;
        dl[0] = l.x; dl[1] = l.y; dl[2] = l.z; dl[3] = l.w;
      }
    }
  };
  // this launch's block positions [sb0, sb1): the sweep, or one exchange segment of it
  const int sb0 = d.seg0, sb1 = d.seg1;
  for (int i = t; i < npass * SROWS; i += NT) eps_l[i] = r0 + i < r1 ? d.eps[r0 + i] : 0.0;
  stage_lut(sb0);
  if (sb0 + 1 < sb1) stage_lut(sb0 + 1);
  // (table storage) the storage block of block s in LDS (s_gb[s & 7]), written by thread 0 P blocks ahead
  // (at boundary s - P, before its barriers; an item is issued at most P items -- blocks -- ahead): an
  // item's loads then need no global load first.  (Read from HBM in issue(), that load's wait -- vmcnt
  // counts in issue order -- drained every load in flight before each item: no prefetch at all.)
  static_assert(P <= 6, "s_gb holds blocks s .. s + P");
  __shared__ int s_gb[8];
  if (XF && t == 0)
    for (int k = 0; k <= P && sb0 + k < sb1; ++k) s_gb[(sb0 + k) & 7] = d.gblk[sb0 + k];
  // f32 path: the member (column) indices of blocks s and s + 1 live in LDS (s_mem[(s & 1) B ..]),
  // so an item's loads need no scalar-cache miss first; block s + 1's are copied at boundary s
  if constexpr (!XF)
    for (int i = t; i < min(2, sb1 - sb0) * B; i += NT)
      s_mem[(((sb0 + i / B) & 1) * B) + i % B] = d.member[(int64_t)sb0 * B + i];
  __syncthreads();
  constexpr int NW = NT / 64;
  const int CPW = B / NW;  // columns per wave
  const int NCH = CPW / CW;      // chunks per wave and block
  // 2-bit storage with room in LDS: the code tiles of this workgroup's rows of the last LAG + 2
  // blocks (buffer s % NCC; [group][row quad][16 columns]), so the change list of block s-1-LAG is
  // applied from LDS, not HBM
  auto cache_of = [&](int s) __attribute__((always_inline)) -> const uint8_t * {
    return (XF && s_codes) ? s_codes + (int64_t)(s % NCC) * B * (npass * 64) : nullptr;
  };
  const int items = NCH * npass; // (chunk, pass) items per wave and block
  const int total = items * (sb1 - sb0);
  const int grp = g / FUSED_GROUP;
  // Lanes whose 4 rows start at or beyond r1 re-read the workgroup's first rows (their
  // residual rows are 0, so they add exactly 0); rows in [N, ld) are zero padding of X.  The
  // loads stay unconditional: a divergent branch here would turn the wave-uniform member
  // loads into vector loads whose wait drains the prefetch ring.
  // f32: one float4 (4 rows) per column and lane; 2-bit: one 16-byte code group (16 columns x 4
  // rows) per lane in x[0]
  // XF = 2: the item's CW float4 columns and, in x[CW], its 16-B class-code group (bits as a float4)
  using Raw = typename std::conditional<XF == 1, uint4, float4>::type;
  constexpr int NR = XF == 1 ? 1 : (XF == 2 ? CW + 1 : CW);
  auto issue = [&](int it, Raw (&x)[NR]) {
    const int s = sb0 + it / items, rem = it - (s - sb0) * items;
    const int c = rem / npass, p = rem - c * npass;
    const int64_t off = r0 + p * SROWS + 4 * lane < r1 ? r0 + p * SROWS + 4 * lane : r0;
    if constexpr (XF == 2) {
      // storage order, as the 2-bit path: the block's 16 contiguous columns of this chunk (clamped
      // to the last column in a short last block: those dots are never read) and their codes
      static_assert(CW == 16, "an item is one 16-column code group");
      const int64_t gb = __builtin_amdgcn_readfirstlane(s_gb[s & 7]);  // wave-uniform
      const int64_t c0 = gb * B + w * CPW + c * CW;
#pragma unroll
      for (int j = 0; j < CW; ++j) x[j] = ldg4_stream(d.X + min(c0 + j, d.M - 1) * ld + off);
      const uint4 cg = ldg16_stream(d.xcodes + ((c0 >> 4) * d.ldc + (off >> 2)) * 16);
      x[CW] = make_float4(__uint_as_float(cg.x), __uint_as_float(cg.y), __uint_as_float(cg.z), __uint_as_float(cg.w));
    } else if constexpr (XF) {
      static_assert(CW == 16, "a 2-bit item is one 16-column group");
      const int64_t gb = __builtin_amdgcn_readfirstlane(s_gb[s & 7]);  // wave-uniform
      const int64_t grp = gb * (B >> 4) + ((w * CPW + c * CW) >> 4);
      x[0] = ldg16_stream(d.Xc + (grp * d.ldc + (off >> 2)) * 16);
    } else {
      const float *base = d.X + off;
      // (scalar loads of the member indices instead: -6 % at C2, a K$ miss per item)
      const int4 *m4 = reinterpret_cast<const int4 *>(s_mem + (s & 1) * B + w * CPW + c * CW);
#pragma unroll
      for (int j = 0; j < CW; j += 4) {
        const int4 m = m4[j / 4];  // same LDS address in every lane: broadcast
        x[j + 0] = ldg4_stream(base + (int64_t)__builtin_amdgcn_readfirstlane(m.x) * ld);
        x[j + 1] = ldg4_stream(base + (int64_t)__builtin_amdgcn_readfirstlane(m.y) * ld);
        x[j + 2] = ldg4_stream(base + (int64_t)__builtin_amdgcn_readfirstlane(m.z) * ld);
        x[j + 3] = ldg4_stream(base + (int64_t)__builtin_amdgcn_readfirstlane(m.w) * ld);
      }
    }
  };
  // register ring of P + 1 items: item it + P is issued before item it is consumed
  Raw xq[P + 1][NR];
  double v[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) v[j] = 0.0;
#pragma unroll
  for (int q = 0; q < P; ++q)
    if (q < total) issue(q, xq[q]);
  // diagnostics (prof): this workgroup's accumulated wait / apply / streaming time of the sweep
  uint64_t acc_wait = 0, acc_apply = 0, acc_stream = 0, t_mark = prof ? wall_clock64() : 0;
  uint64_t acc_sub[4] = {0, 0, 0, 0};  // apply: list staging, products, part barrier, staging stores (ptime)
  // List prefetch (f32 storage, pfe > 0).  While block s streams, each wave fetches the change
  // list that boundary s + 1 applies (block s - LAG; with lag 2 the solver has usually published it
  // before block s starts) one step per item, so no step waits on memory: poll the solver's
  // counter, load the count and lane e's entry e, then LDS-DMA its own part's columns (16 B per
  // lane, the loads apply_pending would issue) and flag it in s_pf[w].  A list longer than pfe,
  // or one not yet published when block s ends, is applied the ordinary way.
  // Three VGPRs of state: pf_m (the counter, then lane e < 32: entry e's column, lane 62 / 63: the
  // padded / real length) and pf_d (lane e < 32: b_old, lane 32 + e: b_new; then lane e: the delta).
  int pf_st = 0;  // 0 poll next, 1 poll in flight, 2 list in flight, 3 staged, 4 too long
  int pf_m = 0, pf_np = 0, pf_nr = 0;
  double pf_d = 0.0;
  auto pf_step = [&](int s) __attribute__((always_inline)) {
    if constexpr (!XF && BRR_PF_DMA) {
      const int a = s - LAG;  // the list boundary s + 1 applies
      if (pfe == 0 || pf_st >= 3 || s + 1 >= sb1 || a < sb0) return;
      const int slot = a % NSLOT;
      if (pf_st == 2) {
        pf_np = __builtin_amdgcn_readlane(pf_m, 62);
        pf_nr = __builtin_amdgcn_readlane(pf_m, 63);
        if (pf_nr > pfe || pf_np > 48) { pf_st = 4; return; }
        pf_d = pf_d - __shfl(pf_d, (lane + 32) & 63);  // lane e < 32: b_old - b_new
        const ApplyPart ap = apply_part(pf_np, npass, w);
        if (ap.p0 < npass) {
          const int64_t off = r0 + ap.p0 * SROWS + 4 * lane < r1 ? r0 + ap.p0 * SROWS + 4 * lane : r0;
          const int ee = min(ap.e1, pf_nr);
          for (int e = ap.e0; e < ee; ++e) {
            const int64_t col = __builtin_amdgcn_readlane(pf_m, e);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(d.X + col * ld + off),
                (__attribute__((address_space(3))) void *)(s_stage + ((int64_t)e * npass + ap.p0) * SROWS), 16, 0, 0);
          }
        }
        pf_st = 3;
        if (lane == 0) s_pf[w] = a;  // read at boundary s + 1, after block s's closing barrier
        return;
      }
      if (pf_st == 1 && (int)((unsigned)__builtin_amdgcn_readfirstlane(pf_m) - (unsigned)(d.sbase + a + 1)) >= 0) {
        // (entries past nr are the neutral padding; lanes 32..61 load an unused word)
        const int *pidx = d.pend_idx + slot * d.pend_stride;
        pf_m = ld_sc1_int(lane < 32 ? pidx + lane : lane == 62 ? d.pend_n + slot : lane == 63 ? d.pend_n + NSLOT + slot : pidx);
        pf_d = ld_sc1(lane < 32 ? d.pend_bo + slot * d.pend_stride + lane : d.pend_bn + slot * d.pend_stride + (lane - 32));
        pf_st = 2;
        return;
      }
      pf_m = ld_sc1_int(d.sync + SY_PEND);
      pf_st = 1;
    }
  };
  auto boundary = [&](int s) __attribute__((always_inline)) {
    const int sr = s - sb0;  // position in this launch
    // (every boundary past the first has a barrier before block s's items: see s_gb)
    if (XF && sr >= 1 && t == 0 && s + P < sb1) s_gb[(s + P) & 7] = d.gblk[s + P];
    if (sr >= 1 && sr <= LAG) {
      // a boundary without a change list to apply yet: stage block s+1's tables / indices
      if constexpr (XF) {
        if (s + 1 < sb1) stage_lut(s + 1);  // (its buffer is not read before the barrier)
      } else if (s + 1 < sb1) {
        __syncthreads();  // every wave is done issuing block s-1's items (same member buffer)
        for (int i = t; i < B; i += NT) s_mem[((s + 1) & 1) * B + i] = d.member[(int64_t)(s + 1) * B + i];
      }
      __syncthreads();
    }
    if (sr >= LAG + 1) {
      // block boundary: apply block a = s-1-LAG's changes to the residual rows (lag 1: they
      // then hold every change before block s-1, which the solver corrects for through the
      // cross-Gram; lag 2: before block s-2, corrected for blocks s-2 and s-1)
      const int a = s - 1 - LAG;
      // every wave prefetched list a during block s-1 (pf_step; its flags were stored before the
      // barrier that ended block s-1): no wait, no list staging, the columns' rows are in LDS
      bool fast = false;
      if constexpr (!XF) {
        if (pfe > 0) {
          fast = true;
#pragma unroll
          for (int q = 0; q < NW; ++q) fast = fast && s_pf[q] == a;
        }
      }
      pf_st = 0;
      if (fast) {
        if (prof && t == 0) {
          const uint64_t tn = wall_clock64();
          acc_wait += tn - t_mark;
          t_mark = tn;
        }
        apply_staged(d, pf_np, pf_nr, pf_d,
                     r0, r1, npass, eps_l, s_part, s_stage,
                     s + 1 < sb1 ? d.member + (int64_t)(s + 1) * B : nullptr, s_mem + ((s + 1) & 1) * B,
                     (prof && t == 0) ? acc_sub : nullptr);
        if (prof && t == 0) {
          const uint64_t tn = wall_clock64();
          acc_apply += tn - t_mark;
          t_mark = tn;
          atomicAdd(&d.sc->prof[16], 1ull);  // boundaries served by the prefetch
        }
        return;
      }
      if (t == 0) {
        wait_geq(d.sync + SY_PEND, d.sbase + a + 1, d.sync, 2);
        if (prof) {
          tr_first(d, s, TR_PEND_FIRST);
          tr_last(d, s, TR_PEND_LAST);
          const uint64_t tn = wall_clock64();
          acc_wait += tn - t_mark;
          t_mark = tn;
        }
      }
      apply_pending<XF, NT>(d, a % NSLOT, r0, r1, npass, eps_l, s_pidx, s_pbo, s_pbn, s_np, s_part,
                        (!XF && s + 1 < sb1) ? d.member + (int64_t)(s + 1) * B : nullptr, s_mem + ((s + 1) & 1) * B,
                        cache_of(a), s_mem,
                        (XF && s + 1 < sb1) ? reinterpret_cast<const float4 *>(lutsrc) + (int64_t)d.gblk[s + 1] * B : nullptr,
                        lut_of(s + 1), lut_of(a), (XF && s + 1 < sb1) ? d.bsz[s + 1] : 0,
                        (prof && t == 0) ? acc_sub : nullptr, s_w);
      if (prof && t == 0) {
        tr_last(d, s, TR_APPLY_LAST);
        if (s == nb / 2) d.trace[(int64_t)nb * 16 + 1024 + g] = wall_clock64();  // per-workgroup probe
        const uint64_t tn = wall_clock64();
        acc_apply += tn - t_mark;
        t_mark = tn;
      }
    }
  };
  auto consume = [&](int it, const Raw (&xc)[NR]) __attribute__((always_inline)) {
    const int s = sb0 + it / items, rem = it - (s - sb0) * items;
    const int c = rem / npass, p = rem - c * npass;
    const double *e = eps_l + p * SROWS + 4 * lane;
    const double e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
    if constexpr (XF) {
      // code cache: block s's tile of group w CPW / 16 + c at this lane's row quad p 64 + lane
      uint4 cg;
      if constexpr (XF == 2)
        cg = make_uint4(__float_as_uint(xc[CW].x), __float_as_uint(xc[CW].y), __float_as_uint(xc[CW].z),
                        __float_as_uint(xc[CW].w));
      else
        cg = xc[0];
      if (s_codes)
        reinterpret_cast<uint4 *>(s_codes)[((s % NCC) * (B >> 4) + ((w * CPW + c * CW) >> 4)) * (npass * 64) + p * 64 +
                                           lane] = cg;
    }
    // one fused multiply-add per value into the column's accumulator, rows in order (the same
    // operations on the same f64 values for both storages: the chains are identical)
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      double x0, x1, x2, x3;
      if constexpr (XF == 1) {
        const uint32_t word = j < 4 ? xc[0].x : (j < 8 ? xc[0].y : (j < 12 ? xc[0].z : xc[0].w));
        const int sh = 8 * (j & 3);
        const double *lt = lut_of(s) + 4 * (w * CPW + c * CW + j);
        x0 = lt[__builtin_amdgcn_ubfe(word, sh, 2)];
        x1 = lt[__builtin_amdgcn_ubfe(word, sh + 2, 2)];
        x2 = lt[__builtin_amdgcn_ubfe(word, sh + 4, 2)];
        x3 = lt[__builtin_amdgcn_ubfe(word, sh + 6, 2)];
      } else {
        const float4 xv = xc[j];
        x0 = xv.x; x1 = xv.y; x2 = xv.z; x3 = xv.w;
      }
      v[j] = __builtin_fma(x3, e3, __builtin_fma(x2, e2, __builtin_fma(x1, e1, __builtin_fma(x0, e0, v[j]))));
    }
    if (p == npass - 1) {
      // chunk done over this workgroup's rows: wave-reduce its CW columns
      double r;
      int lcol;
      if constexpr (CW == 8) {
        r = wave_reduce8(v, lane);
        lcol = reduce8_col(lane);
      } else {
        r = wave_reduce16(v, lane);
        lcol = reduce16_col(lane);
      }
#pragma unroll
      for (int j = 0; j < CW; ++j) v[j] = 0.0;
      const int col = w * CPW + c * CW + lcol;
      if ((lane & (64 / CW - 1)) == 0) st_sc1(d.slab1 + (s % NPAR) * d.slab1_stride + (int64_t)g * B + col, r);
    }
  };
  auto block_end = [&](int it, int s, Raw (&xn)[NR], bool clamp) __attribute__((always_inline)) {
    // block done.  The partial-dot stores were issued before the next item's loads, so
    // waiting until only those loads are outstanding drains the stores (vmcnt counts in
    // issue order) without draining the prefetch.
    asm volatile("" ::: "memory");
    if (clamp || it + P < total) issue(clamp ? min(it + P, total - 1) : it + P, xn);
    if (clamp || it + P < total) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P * NR) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // then one arrival on the group counter for the reducer workgroup (one per workgroup:
    // per-wave arrivals measured 1.6x slower, contention on the group counters)
    __syncthreads();
    if (t == 0)
      __hip_atomic_fetch_add(d.cnt1 + (s % NPAR) * d.ngr + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == 0) {
      if (prof) {
        tr_first(d, s, TR_ITEMS_FIRST);
        tr_last(d, s, TR_ITEMS_LAST);
        if (s == nb / 2) d.trace[(int64_t)nb * 16 + g] = wall_clock64();
        const uint64_t tn = wall_clock64();
        acc_stream += tn - t_mark;
        t_mark = tn;
      }
    }
  };
  constexpr int R = P + 1;
  if (BRR_STATIC_RING && items % R == 0) {
    // static register ring: item it's data in xq[it % R], the loop unrolled by R so every slot
    // index is a constant, and one load issued per item (clamped past the end), so the wait
    // before a consume is for the oldest load only.  (A runtime ring shifts its elements, and
    // the compiler then waits for every outstanding load before each consume:
    // scripts/mb_decode.hip.)  R divides items: a block starts at u = 0 and ends at u = R - 1.
    for (int it0 = 0; it0 < total; it0 += R) {
      static_for<R>([&](auto uc) __attribute__((always_inline)) {
        constexpr int u = decltype(uc)::value;
        const int it = it0 + u;
        const int s = sb0 + it / items, rem = it - (s - sb0) * items;
        if constexpr (u == 0)
          if (rem == 0) boundary(s);
        const bool blk_end = u == R - 1 && rem == items - 1;
        if (!blk_end) issue(min(it + P, total - 1), xq[(u + P) % R]);
        consume(it, xq[u]);
        pf_step(s);
        if constexpr (u == R - 1)
          if (blk_end) block_end(it, s, xq[(u + P) % R], true);
      });
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int it = 0; it < total; ++it) {
      const int s = sb0 + it / items, rem = it - (s - sb0) * items;
      const bool blk_end = rem == items - 1;
      if (rem == 0) boundary(s);
      // prefetch P items ahead (across block boundaries) before consuming this one; at a block's
      // last item the prefetch is issued after the partial-dot stores instead (block_end)
      if (!blk_end && it + P < total) issue(it + P, xq[P]);
      consume(it, xq[0]);
      pf_step(s);
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int j = 0; j < NR; ++j) xq[q][j] = xq[q + 1][j];
      if (blk_end) block_end(it, s, xq[P - 1], false);
    }
  }
  if (prof && t == 0) {
    unsigned long long *acc = d.trace + (int64_t)nb * 16 + 2048;
    acc[g] = acc_wait;
    acc[1024 + g] = acc_apply;
    acc[2048 + g] = acc_stream;
    acc[3072 + g] = acc_sub[0];
    acc[4096 + g] = acc_sub[1];
    acc[5120 + g] = acc_sub[2];
    acc[6144 + g] = acc_sub[3];
  }
  // end of the launch: the last LAG + 1 blocks' changes, then the residual rows back to HBM
  if (t == 0) wait_geq(d.sync + SY_PEND, d.sbase + sb1, d.sync, 4);
  for (int a = max(sb0, sb1 - 1 - LAG); a < sb1; ++a)
    apply_pending<XF, NT>(d, a % NSLOT, r0, r1, npass, eps_l, s_pidx, s_pbo, s_pbn, s_np, s_part, nullptr, nullptr,
                          cache_of(a), s_mem, nullptr, nullptr, lut_of(a), 0, nullptr, s_w);
  for (int i = t; i < npass * SROWS; i += NT)
    if (r0 + i < r1) d.eps[r0 + i] = eps_l[i];
}

// Reducer workgroup r of nred: for every block, the whole sum over the nsg streaming workgroups'
// partial dots of ITS columns [r cw, (r + 1) cw), cw = B / nred, into slab2 row 0 (the solver
// reads one value per position).  Each of RED_NT logical threads sums a contiguous range of
// workgroups for one column (in workgroup order); the RED_NT / cw ranges are added in range order
// -- the same operations whatever the workgroup's width.  A column slice per reducer instead of a
// group of streamers per reducer: every reducer reads nsg cw partials (C2: 196 x 16 doubles) rather
// than a group's 64 B (256 KB at B = 512, ~9 us at one CU's share of HBM under the stream).
// Dev::rcorr: the reducer also subtracts the column's cross-Gram corrections (the changes of blocks
// s-1 .. s-lag, the solver's phase A sums, solve_block), each list's sum over RED_NT / cw contiguous
// entry ranges added in range order, the lists as (c_1 + c_2) + c_3: the solver then reads corrected
// dots and its phase A loads no cross-Gram rows (a C4 block's correction reads all 128 KB of its
// cross-Gram block: at one CU's share of HBM that was half of the solver's phase A).
constexpr int RED_NT = 512;
template <int NT = SWEEP_NT>
__device__ __forceinline__ void reduce_role(const Dev &d, int r, int nsg, int nred, bool prof, double *s_red) {
#pragma clang fp contract(off)
  const int t = threadIdx.x;
  const int B = d.B;
  const int cw = B / nred;            // columns of this reducer (a power of two, 8 .. RED_NT)
  const int np = RED_NT / cw;         // workgroup ranges per column
  const int cl = t % cw, part = t / cw;
  const int w0 = part * nsg / np, w1 = (part + 1) * nsg / np;
  const int col = r * cw + cl;
  const int lag = sweep_lag(d);
  double *s_ld = s_red + RED_NT;                            // a change list: deltas [B + 16]
  int *s_lg = reinterpret_cast<int *>(s_ld + (B + 16));     // and Gram indices [B + 16]
  // (Dev::rcpf) this reducer's columns of the cross-Gram blocks of the lists block s's dots have not seen,
  // [list l][row][cw]: their rows (the earlier block's Gram indices) and columns are known before those
  // lists are published (the visit order is), so they are loaded before the wait -- after the publication
  // only the list itself is read.  For the Horseshoe (every marker changes: the whole B x B block) this
  // takes the correction's 128 KB per block off the solver's phase A.
  double *s_C = reinterpret_cast<double *>(s_lg + (B + 16));
  // the cross-Gram block of block sp's changes against block s (l = s - 1 - sp)
  auto xblock = [&](int l, int sp, int s) -> const double * {
    const int gp = d.gblk[sp], gb = d.gblk[s];
    return l == 0 ? (gb == (gp + 1) % d.nb ? d.xgram + (int64_t)gp * B * B : d.xgramT + (int64_t)gb * B * B)
         : l == 1 ? (gb == (gp + 2) % d.nb ? d.xgram2 + (int64_t)gp * B * B : d.xgram2T + (int64_t)gb * B * B)
                  : (gb == (gp + 3) % d.nb ? d.xgram3 + (int64_t)gp * B * B : d.xgram3T + (int64_t)gb * B * B);
  };
  for (int s = d.seg0; s < d.seg1; ++s) {
    const int par = s % NPAR;
    const int use = d.gbase[par] + s / NPAR;
    const double *slab1 = d.slab1 + par * d.slab1_stride + col;
    if (d.rcpf && d.rcorr && s > d.seg0 && t < RED_NT) {
      const int bs = d.bsz[s];
      const int gic = col < bs ? (d.slab_storage ? col : d.gidx[(int64_t)s * B + col]) : 0;
      for (int l = 0; l < lag; ++l) {
        const int sp = s - 1 - l;
        if (sp < d.seg0) break;
        const int bsp = d.bsz[sp];  // (rows of a short earlier block past its size are never read)
        const double *C = xblock(l, sp, s);
        for (int row = part; row < bsp; row += np) s_C[((int64_t)l * B + row) * cw + cl] = C[(int64_t)row * B + gic];
      }
    }
    if (t == 0)
      for (int grp = 0; grp < d.ngr; ++grp)
        wait_geq(d.cnt1 + par * d.ngr + grp, (use + 1) * min(FUSED_GROUP, nsg - grp * FUSED_GROUP), d.sync, 6);
    __syncthreads();
    if (t < RED_NT) {
      double acc = 0.0;
      for (int w = w0; w < w1; w += 16) {
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = w + q < w1 ? ld_sc1(slab1 + (int64_t)(w + q) * B) : 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q)
          if (w + q < w1) acc += v[q];
      }
      s_red[part * cw + cl] = acc;
    }
    __syncthreads();
    double tot = 0.0;
    if (t < cw) {
      tot = s_red[t];
      for (int p = 1; p < np; ++p) tot += s_red[p * cw + t];
    }
    if (d.rcorr && s > d.seg0) {
      const int bs = d.bsz[s];
      // the column's Gram index (slab columns are visit positions, or storage indices = Gram indices)
      const int gic = col < bs ? (d.slab_storage ? col : d.gidx[(int64_t)s * B + col]) : 0;
      double cor[LAG_MAX] = {0.0, 0.0, 0.0};
      for (int l = LAG_MAX - 1; l >= 0; --l) {  // (the older lists are published first)
        const int sp = s - 1 - l;
        if (l >= lag || sp < d.seg0 || (d.rcsplit && l == 0)) continue;  // (rcsplit: the solver corrects for s-1)
        if (t == 0) wait_geq(d.sync + SY_PEND, d.sbase + sp + 1, d.sync, 7);
        __syncthreads();  // (also: the partial sums above are consumed)
        const int slot = sp % NSLOT;
        const int nr = ld_sc1_int(d.pend_n + NSLOT + slot);  // real entries (no padding)
        const int *pgi = d.pend_gi + slot * d.pend_stride;
        const double *pbo = d.pend_bo + slot * d.pend_stride, *pbn = d.pend_bn + slot * d.pend_stride;
        for (int e = t; e < nr; e += NT) {
          s_lg[e] = ld_sc1_int(pgi + e);
          s_ld[e] = ld_sc1(pbn + e) - ld_sc1(pbo + e);
        }
        __syncthreads();
        if (t < RED_NT) {
          const int e0 = part * nr / np, e1 = (part + 1) * nr / np;
          double a = 0.0;
          if (col < bs) {
            if (d.rcpf) {  // the slice in LDS (the same values, summed in the same order)
              const double *Cs = s_C + (int64_t)l * B * cw + cl;
              for (int e = e0; e < e1; e += 8) {
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = e + u < e1 ? Cs[(int64_t)s_lg[e + u] * cw] : 0.0;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                  if (e + u < e1) a += v[u] * s_ld[e + u];
              }
            } else {
              const double *C = xblock(l, sp, s);
              for (int e = e0; e < e1; e += 8) {
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = e + u < e1 ? C[(int64_t)s_lg[e + u] * B + gic] : 0.0;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                  if (e + u < e1) a += v[u] * s_ld[e + u];
              }
            }
          }
          s_red[part * cw + cl] = a;
        }
        __syncthreads();
        if (t < cw) {
          double c = s_red[t];
          for (int p = 1; p < np; ++p) c += s_red[p * cw + t];
          cor[l] = c;
        }
      }
      if (t < cw && col < bs) tot = tot - ((cor[0] + cor[1]) + cor[2]);
    }
    if (t < cw) st_sc1(d.slab2 + par * d.slab2_stride + col, tot);
    publish_add(d.sync + SY_GDONE + 32 * par, 1);
    if (prof && t == 0) { tr_first(d, s, TR_L2_FIRST); tr_last(d, s, TR_L2_LAST); }
  }
}

#ifndef BRR_SOLVER_CALL
#define BRR_SOLVER_CALL 0  // (diagnostics) the solver role as a called function: its own register allocation
#endif
#if BRR_SOLVER_CALL
#define BRR_SOLVER_INL __attribute__((noinline))
#else
#define BRR_SOLVER_INL __forceinline__
#endif
template <bool HS, int B, int NT = SWEEP_NT>
__device__ BRR_SOLVER_INL void solver_role(const Dev &d, uint32_t it, int nslot, char *smem) {
  const int lag = sweep_lag(d);
  for (int s = d.seg0; s < d.seg1; ++s) {
    solve_block<HS, B, NT>(d, s, it, nslot, smem, true, lag);
    __syncthreads();
  }
}

#include "brr_ovsolve.hpp"

// the persistent solver workgroup: the overlapped form where it applies (Dev::ovs), else solve_block
// per block
template <bool HS, int B, int NT = SWEEP_NT>
__device__ __forceinline__ void solver_any(const Dev &d, uint32_t it, int nslot, char *smem) {
  if constexpr (!HS && B == OVB && NT == 512) {
    if (d.ovs) {
      solver_role_ov<B>(d, it, smem);
      return;
    }
  }
  solver_role<HS, B, NT>(d, it, nslot, smem);
}

// XF: 0 f32 storage (with the list prefetch when pfe > 0), 1 2-bit codes, 2 f32 storage with the
// class-code cache -- the streaming roles of k_sweep_stream<XF> at 512 threads, so that a PMC pass of
// this form counts the path the two-kernel default times (C2 f32: XF 0 + pfe; C4: XF 2)
template <bool HS, int B, int XF>
__global__ __launch_bounds__(SWEEP_NT, 1) void k_sweep(Dev d, uint32_t it, int nslot, int nsg, int rpw, int npass,
                                                        int nred, int ccache, int pfe) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_np[2];
  __shared__ int s_ok;
  __shared__ int s_pf[SWEEP_NW];
  // residency census: every workgroup must be running before any waits on another.  A workgroup whose census
  // timed out -- or that arrives after another one's did -- leaves before touching any state,
  // so a failed census costs one sweep's marker loop, never the chain's consistency.
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(d.sync + SY_ARRIVE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    wait_geq(d.sync + SY_ARRIVE, d.abase + nsg + 1 + nred, d.sync, 5);
    s_ok = ld_sc1_int(d.sync + SY_ERR) == 0;
  }
  __syncthreads();
  if (!s_ok) return;
  if (blockIdx.x == 0) {
    solver_any<HS, B>(d, it, nslot, smem);
  } else if ((int)blockIdx.x > nsg) {
    reduce_role(d, (int)blockIdx.x - 1 - nsg, nsg, nred, d.sc->prof_on, reinterpret_cast<double *>(smem));
  } else {
    // streamer LDS: residual rows, [value tables of four blocks (2-bit codes)], the change list
    // being applied, member indices of two blocks (fused_config)
    double *eps_l = reinterpret_cast<double *>(smem);
    double *s_lut = eps_l + (int64_t)npass * SROWS;
    double *s_pbo = s_lut + (XF ? (int64_t)(d.lag + 3) * d.B * 4 : 0), *s_pbn = s_pbo + (d.B + 16);
    int *s_pidx = reinterpret_cast<int *>(s_pbn + (d.B + 16));
    int *s_mem = s_pidx + (d.B + 16);  // 16-B aligned: B + 16 is a multiple of 4
    // (2-bit storage: s_mem holds the change positions instead); the apply's partial sums; then
    // the code cache
    double *s_part = reinterpret_cast<double *>(s_mem + 2 * d.B);
    // (table storage) the apply's pair tables (16 doubles per pair of list entries), then the code cache
    double *s_w = XF ? s_part + SWEEP_NW * SROWS : nullptr;
    uint8_t *s_codes = (XF && ccache) ? reinterpret_cast<uint8_t *>(s_w + (int64_t)(d.B + 16) * 8) : nullptr;
    // (f32 storage) the list prefetch's staging area: pfe entries x npass passes x 1 KiB
    float *s_stage = reinterpret_cast<float *>(s_part + SWEEP_NW * SROWS);
    stream_role<STREAM_CW, XF == 1 ? STREAM_P2 : STREAM_P, XF>(d, (int)blockIdx.x - 1, rpw, npass, eps_l, s_pidx, s_pbo,
                                                         s_pbn, s_np, s_lut, s_mem, s_part, s_codes, XF ? 0 : pfe, s_pf,
                                                         s_stage, s_w);
  }
}


// The same marker loop as two kernels launched side by side (the default): the solver workgroup in
// k_sweep_solve, the streaming and reducing workgroups in k_sweep_stream.  Each gets its own
// register allocation (in k_sweep every role shares the largest role's, and the solver's serial
// chain reloads spilled registers from scratch memory).  Residency: the solver needs a whole CU's
// LDS and every streaming / reducing workgroup is padded to more than half of it, so no two
// workgroups of this launch pair share a CU and 1 + nsg + nred <= #CUs of them are resident at
// once; the census below (across both kernels) is the defence, as in k_sweep.
__device__ __forceinline__ bool sweep_census(const Dev &d, int total, int *s_ok) {
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(d.sync + SY_ARRIVE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    wait_geq(d.sync + SY_ARRIVE, d.abase + total, d.sync, 5);
    *s_ok = ld_sc1_int(d.sync + SY_ERR) == 0;
  }
  __syncthreads();
  return *s_ok != 0;
}

constexpr int SOLVE_NT = SWEEP_NT;  // the solver workgroup's threads
template <bool HS, int B>
__global__ __launch_bounds__(SOLVE_NT, 1) void k_sweep_solve(Dev d, uint32_t it, int nslot, int total) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_ok;
  if (!sweep_census(d, total, &s_ok)) return;
  solver_any<HS, B, SOLVE_NT>(d, it, nslot, smem);
}

// NT = 1024 (2-bit storage, B >= 256): 16 waves per streaming workgroup at <= 128 VGPRs -- four
// waves per SIMD instead of two to hide the decode-dot's LDS-read -> FMA latency; every column's
// partial dot and every residual update are the same operations in the same order as at NT = 512.
template <int XF, int NT = SWEEP_NT, bool PROF = false>
__global__ __launch_bounds__(NT, 1) void k_sweep_stream(Dev d, int nsg, int rpw, int npass, int nred, int ccache,
                                                         int pfe) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_np[2];
  __shared__ int s_ok;
  __shared__ int s_pf[NT / 64];
  if (!sweep_census(d, nsg + 1 + nred, &s_ok)) return;
  if ((int)blockIdx.x >= nsg) {
    reduce_role<NT>(d, (int)blockIdx.x - nsg, nsg, nred, d.sc->prof_on, reinterpret_cast<double *>(smem));
    return;
  }
  double *eps_l = reinterpret_cast<double *>(smem);
  double *s_lut = eps_l + (int64_t)npass * SROWS;
  double *s_pbo = s_lut + (XF ? (int64_t)(d.lag + 3) * d.B * 4 : 0), *s_pbn = s_pbo + (d.B + 16);
  int *s_pidx = reinterpret_cast<int *>(s_pbn + (d.B + 16));
  int *s_mem = s_pidx + (d.B + 16);
  double *s_part = reinterpret_cast<double *>(s_mem + 2 * d.B);
  // (table storage: 2-bit codes, f32 code cache) the apply's pair tables, then the code cache
  double *s_w = XF ? s_part + SWEEP_NW * SROWS : nullptr;
  uint8_t *s_codes = (XF && ccache) ? reinterpret_cast<uint8_t *>(s_w + (int64_t)(d.B + 16) * 8) : nullptr;
  // (f32 storage) the list prefetch's staging area: pfe entries x npass passes x 1 KiB
  float *s_stage = reinterpret_cast<float *>(s_part + SWEEP_NW * SROWS);
  stream_role<STREAM_CW, XF == 1 ? STREAM_P2 : STREAM_P, XF, NT, PROF>(d, (int)blockIdx.x, rpw, npass, eps_l, s_pidx, s_pbo,
                                                           s_pbn, s_np, s_lut, s_mem, s_part, s_codes, XF ? 0 : pfe,
                                                           s_pf, s_stage, s_w);
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
    const int nw = (int)gridDim.x;
    if (NS <= 64) {
      // wave per statistic, lanes stride over the workgroup slabs (fixed order), wave tree
      const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
      for (int q = wv; q < NS; q += 4) {
        double acc = 0.0;
        for (int w = lane; w < nw; w += 64) acc += d.mslab[(int64_t)w * NS + q];
        acc = wave_sum(acc);
        if (lane == 0) d.stats[q] = acc;
      }
    } else {
      for (int q = threadIdx.x; q < NS; q += 256) {
        double acc = 0.0;
        for (int w = 0; w < nw; ++w) acc += d.mslab[(int64_t)w * NS + q];
        d.stats[q] = acc;
      }
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
  const double N = (double)d.Ntot;
  const double *bacc = stats + 2;
  const double *v = stats + 2 + G;
  const double sigmaE_new = inv_scaled_chisq_rng(d.seed, h.v0E + N, (sc->S2 + h.v0E * h.s02E) / (h.v0E + N),
                                                 T_SIGMAE, 0, it);
  if (t == 0) {  // the next fused sweep's pipeline lag from this sweep's changes (Dev::lag_thresh)
    const unsigned long long nc = sc->n_changed;
    sc->lag_next = (double)(nc - sc->nch_mark) > d.lag_thresh ? 1 : 2;
    sc->nch_mark = nc;
  }
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
  const double N = (double)d.Ntot;
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

// Linear predictor X beta + F alpha of this shard (validation read-back, not on the sweep path):
// one thread per row, columns in index order, f64 accumulation of the stored f32 values.  A plain
// kernel sharing nothing with the sweep's streaming code, so the full-size residual invariant
// eps = Y - mu - X beta - F alpha checks the sweep's bookkeeping against an independent product.
__global__ __launch_bounds__(256) void k_linpred(Dev d, double *out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= d.N) return;
  double acc = 0.0;
  for (int64_t j = 0; j < d.M; ++j) {
    const double b = d.beta[j];
    if (b != 0.0) acc = __builtin_fma((double)x_at(d, j, i), b, acc);
  }
  for (int c = 0; c < d.F; ++c) acc = __builtin_fma(d.fixed[(int64_t)c * d.N + i], d.alpha[c], acc);
  out[i] = acc;
}

}  // namespace brr

// ======================================================================================
// host-side launch wrappers (called by brr_session.cpp)
#include "brr_launch.hpp"

namespace brr {

static inline unsigned cdiv64(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

hipError_t launch_synth_x(const Dev &d, uint64_t ds, hipStream_t st) {
  hipLaunchKernelGGL(k_synth_x, dim3((unsigned)d.M), dim3(256), 0, st, const_cast<float *>(d.X),
                     const_cast<uint8_t *>(d.Xc), const_cast<float *>(d.xlut), d.ld, d.ldc, d.N, d.col_offset, ds,
                     d.Ntot, d.row_offset, d.B);
  return hipGetLastError();
}

hipError_t launch_synth_y(const Dev &d, const int *cidx, const double *cb, int nc, double *y, hipStream_t st) {
  hipLaunchKernelGGL(k_synth_y, dim3(cdiv64(d.N, 256)), dim3(256), 0, st, d, cidx, cb, nc, y);
  return hipGetLastError();
}

hipError_t launch_codes_cm(const Dev &d, uint8_t *xcm, hipStream_t st) {
  const int64_t n = d.ldc / 4 * ((d.M + 15) / 16 * 16);
  if (n > 0) hipLaunchKernelGGL(k_codes_cm, dim3((unsigned)cdiv64(n, 256)), dim3(256), 0, st, d, xcm);
  return hipGetLastError();
}

hipError_t launch_codes_tile(const uint8_t *src, uint8_t *Xc, int64_t c0, int64_t nc, int64_t ldc, int B,
                             hipStream_t st) {
  for (int64_t j0 = 0; j0 < nc; j0 += 65535) {
    const dim3 grid(cdiv64(ldc, 256) > 64 ? 64 : cdiv64(ldc, 256), (unsigned)std::min<int64_t>(65535, nc - j0));
    hipLaunchKernelGGL(k_codes_tile, grid, dim3(256), 0, st, src + j0 * ldc, Xc, c0 + j0, grid.y, ldc, B);
  }
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

hipError_t launch_classes(const Dev &d, int *flags, hipStream_t st) {
  if (d.M <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_classes, dim3((unsigned)d.M), dim3(256), 0, st, d, flags);
  return hipGetLastError();
}

hipError_t launch_encode_layout(const Dev &d, hipStream_t st) {
  if (!d.gram_codes) return hipErrorInvalidValue;
  const unsigned gy = (unsigned)std::min<int64_t>((int64_t)d.nb * (d.B / 16), 65535);
  if (d.xcls && d.ldc % 4 == 0)
    hipLaunchKernelGGL(k_encode_gather, dim3(cdiv64(d.ldc / 4, 256), gy), dim3(256), 0, st, d, d.xcls, d.gram_codes);
  else
    hipLaunchKernelGGL(k_encode_layout, dim3(cdiv64(d.ldc, 256), gy), dim3(256), 0, st, d, d.gram_codes);
  return hipGetLastError();
}

hipError_t launch_xcls(const Dev &d, uint8_t *xcls, hipStream_t st) {
  if (d.M <= 0) return hipSuccess;
  const unsigned gy = (unsigned)std::min<int64_t>(d.M, 65535);
  hipLaunchKernelGGL(k_xcls, dim3(cdiv64(d.ldc, 256), gy), dim3(256), 0, st, d, xcls);
  return hipGetLastError();
}

template <int NP>
static hipError_t launch_gram_int_t(const Dev &d, int shift, double *G, double *GT, hipStream_t st) {
  constexpr size_t lds = gram_int_lds(NP);
  static const hipError_t attr =
      hipFuncSetAttribute((const void *)k_gram_int<NP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  const int nt = d.B / GI_T;
  // diagonal blocks (shift 0, no transposed copy): the nt (nt + 1) / 2 tiles on and above the diagonal,
  // each written to both halves (G is exactly symmetric)
  const int ntiles = (shift == 0 && GT == nullptr) ? nt * (nt + 1) / 2 : nt * nt;
  hipLaunchKernelGGL((k_gram_int<NP>), dim3((unsigned)d.nb, (unsigned)ntiles), dim3(256), lds, st, d, d.gram_codes,
                     d.member, d.bsz, d.B, d.nb, shift, G, GT);
  return hipGetLastError();
}

template <int NP>
static hipError_t launch_gram_blk_t(const Dev &d, int shift, double *G, double *GT, hipStream_t st) {
  constexpr size_t lds = gram_blk_lds(NP);
  static const hipError_t attr =
      hipFuncSetAttribute((const void *)k_gram_blk<NP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  const int nt = d.B / GB_T;
  const int ntiles = (shift == 0 && GT == nullptr) ? nt * (nt + 1) / 2 : nt * nt;
  hipLaunchKernelGGL((k_gram_blk<NP>), dim3((unsigned)d.nb, (unsigned)ntiles), dim3(512), lds, st, d, d.gram_codes,
                     d.member, d.bsz, d.B, d.nb, shift, G, GT);
  return hipGetLastError();
}

template <int NP>
static hipError_t launch_gram_fp4_t(const Dev &d, int shift, double *G, double *GT, hipStream_t st) {
  constexpr size_t lds = gram_fp4_lds(NP);
  static const hipError_t attr =
      hipFuncSetAttribute((const void *)k_gram_fp4<NP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  const int nt = d.B / GB_T;
  const int ntiles = (shift == 0 && GT == nullptr) ? nt * (nt + 1) / 2 : nt * nt;
  hipLaunchKernelGGL((k_gram_fp4<NP>), dim3((unsigned)d.nb, (unsigned)ntiles), dim3(512), lds, st, d, d.xcls, d.member,
                     d.bsz, d.B, d.nb, shift, G, GT);
  return hipGetLastError();
}

// the fp4 Gram kernel applies: REFERENCE order's column-major class codes, at most 3 classes, whole
// 128-column tiles, f32 sums exact (16 N < 2^24); BRR_GRAM_FP4=0 keeps the i8 kernels (A/B)
bool gram_reads_xcls(const Dev &d) {
  const char *f = getenv("BRR_GRAM_FP4");
  return d.xcls && d.gram_np >= 1 && d.gram_np <= 2 && d.B % GB_T == 0 && d.ldc % 64 == 0 &&
         16 * (int64_t)d.N < ((int64_t)1 << 24) && !(f && f[0] == '0');
}

hipError_t launch_gram(const Dev &d, int shift, double *G, double *GT, hipStream_t st) {
  if (d.gram_np > 0 && gram_reads_xcls(d))
    return d.gram_np == 1 ? launch_gram_fp4_t<1>(d, shift, G, GT, st) : launch_gram_fp4_t<2>(d, shift, G, GT, st);
  // whole 128-column tiles for the genotype case (BRR_GRAM_TILE64=1: k_gram_int's 64-column tiles, A/B)
  const char *t64 = getenv("BRR_GRAM_TILE64");
  if (d.gram_np > 0 && d.gram_np <= 2 && d.gram_codes && d.B % GB_T == 0 && !(t64 && t64[0] == '1'))
    return d.gram_np == 1 ? launch_gram_blk_t<1>(d, shift, G, GT, st) : launch_gram_blk_t<2>(d, shift, G, GT, st);
  if (d.gram_np > 0 && d.gram_codes && d.B % GI_T == 0) {
    switch (d.gram_np) {
      case 1: return launch_gram_int_t<1>(d, shift, G, GT, st);
      case 2: return launch_gram_int_t<2>(d, shift, G, GT, st);
      default: return launch_gram_int_t<3>(d, shift, G, GT, st);
    }
  }
  const int nt = (d.B + GRAM_TILE - 1) / GRAM_TILE;
  static const hipError_t attr = hipFuncSetAttribute((const void *)k_gram, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)GRAM_LDS);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(k_gram, dim3((unsigned)d.nb, (unsigned)(nt * nt)), dim3(256), GRAM_LDS, st, d, d.member, d.bsz,
                     d.B, d.nb, shift, G, GT);
  return hipGetLastError();
}

hipError_t launch_xsq(const Dev &d, hipStream_t st) {
  hipLaunchKernelGGL(k_xsq_from_gram, dim3((unsigned)d.nb), dim3(BMAX), 0, st, d.gram, d.member, d.bsz, d.B,
                     d.nb, d.xsq);
  return hipGetLastError();
}

hipError_t launch_rows(const Dev &d, int flags, const double *deps_in, hipStream_t st, const double *eps_in,
                       int slot_a, int slot_b) {
  hipLaunchKernelGGL(k_rows, dim3(cdiv64(d.N, 256)), dim3(256), 0, st, d, flags, deps_in, eps_in, slot_a, slot_b);
  return hipGetLastError();
}

__global__ void k_noop() {}

// A no-op dispatch right after an event record on the main queue: the event then completes
// with this kernel, never with the persistent streamer that follows (which waits for the
// solver queue that waits for the event).
hipError_t launch_noop(hipStream_t st) {
  hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, st);
  return hipGetLastError();
}

hipError_t launch_sweep_start(const Dev &d, uint32_t it, hipStream_t st) {
  hipLaunchKernelGGL(k_sweep_start, dim3(1), dim3(64), 0, st, d, it);
  return hipGetLastError();
}

hipError_t launch_perm(const Dev &d, uint32_t it, int shard, bool identity, hipStream_t st) {
  hipLaunchKernelGGL(k_perm_blockorder, dim3(1), dim3(256), 0, st, d, it, shard, identity ? 1 : 0);
  hipLaunchKernelGGL(k_perm_within, dim3((unsigned)d.nb), dim3(64), 0, st, d, it, identity ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_fixed(const Dev &d, uint32_t it, bool perm_on_device, hipStream_t st) {
  hipLaunchKernelGGL(k_fixed, dim3(1), dim3(1024), 0, st, d, it, perm_on_device ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_fixed_row(const Dev &d, uint32_t it, int cf, int phase, bool perm_on_device, hipStream_t st) {
  hipLaunchKernelGGL(k_fixed_row, dim3(1), dim3(1024), 0, st, d, it, cf, phase, perm_on_device ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_slab_total(const Dev &d, int s, hipStream_t st) {
  hipLaunchKernelGGL(k_slab_total, dim3(1), dim3(BMAX), 0, st, d, s);
  return hipGetLastError();
}

hipError_t launch_group_sum(const GroupPtrs &p, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const unsigned grid = cdiv64(n, 256) > 1024 ? 1024 : cdiv64(n, 256);
  hipLaunchKernelGGL(k_group_sum, dim3(grid), dim3(256), 0, st, p, n);
  return hipGetLastError();
}

hipError_t launch_stream(const Dev &d, int s, const double *eps_in, double *eps_out, hipStream_t st) {
  const int cw = d.B >= 128 ? 32 : 16;
  const unsigned grid = (unsigned)(((d.RG + 7) / 8) * 8 * (d.B / (4 * cw)));
  if (cw == 32)
    hipLaunchKernelGGL(k_stream<32>, dim3(grid), dim3(256), 0, st, d, s, eps_in, eps_out);
  else
    hipLaunchKernelGGL(k_stream<16>, dim3(grid), dim3(256), 0, st, d, s, eps_in, eps_out);
  return hipGetLastError();
}

// Fused sweep geometry: one solver, nsg streaming and nred reducing workgroups, one per CU (the
// solver's LDS), each streamer owning rpw rows (npass passes of 256).  Returns false when the
// configuration cannot be made resident (the per-block kernels are used then).
// (B = 64 never fuses: a block must give every wave whole STREAM_CW-column chunks)
template <bool HS, int B>
static const void *sweep_fn(int xv) {
  return xv == 1 ? (const void *)k_sweep<HS, B, 1> : xv == 2 ? (const void *)k_sweep<HS, B, 2> : (const void *)k_sweep<HS, B, 0>;
}

// xv: the streaming variant (stream_variant)
static const void *sweep_kernel(int model, int B, int xv) {
  const bool hs = model == MODEL_HORSESHOE;
  switch (B) {
    case 128: return hs ? sweep_fn<true, 128>(xv) : sweep_fn<false, 128>(xv);
    case 256: return hs ? sweep_fn<true, 256>(xv) : sweep_fn<false, 256>(xv);
    case 512: return hs ? sweep_fn<true, 512>(xv) : sweep_fn<false, 512>(xv);
    default: return nullptr;
  }
}

template <bool HS, int B>
static const void *solve_fn() { return (const void *)k_sweep_solve<HS, B>; }

static const void *solve_kernel(int model, int B) {
  const bool hs = model == MODEL_HORSESHOE;
  switch (B) {
    case 128: return hs ? solve_fn<true, 128>() : solve_fn<false, 128>();
    case 256: return hs ? solve_fn<true, 256>() : solve_fn<false, 256>();
    case 512: return hs ? solve_fn<true, 512>() : solve_fn<false, 512>();
    default: return nullptr;
  }
}

// 0: f32 storage, 1: 2-bit codes, 2: f32 storage with the class-code cache (Dev::xcodes); nt: threads
// per streaming workgroup (1024: 2-bit codes only); prof: the variant with the diagnostics' timers
template <bool PROF>
static const void *stream_kernel_t(int xf, int nt) {
  if (xf == 1)
    return nt == 1024 ? (const void *)k_sweep_stream<1, 1024, PROF> : (const void *)k_sweep_stream<1, SWEEP_NT, PROF>;
  return xf == 2 ? (const void *)k_sweep_stream<2, SWEEP_NT, PROF> : (const void *)k_sweep_stream<0, SWEEP_NT, PROF>;
}
static const void *stream_kernel(int xf, int nt = SWEEP_NT, bool prof = false) {
  return prof ? stream_kernel_t<true>(xf, nt) : stream_kernel_t<false>(xf, nt);
}
static int stream_variant(const Dev &d, const FusedCfg &c) { return d.Xc ? 1 : (c.f32cc && d.xcodes) ? 2 : 0; }

// streaming / reducing workgroups of the two-kernel sweep take more than half of a CU's LDS: one per CU
constexpr size_t STREAM_LDS_MIN = SOLVE_LDS_MAX / 2 + 1024;

bool fused_config(const Dev &d, int cus, int max_wg, FusedCfg *cfg, bool f32cc) {
  // the 8 waves of a streaming workgroup split a block's columns in chunks of STREAM_CW
  if (cus < 3 || d.B % (SWEEP_NW * STREAM_CW) != 0) return false;
  // one CU each: the solver, nsg streamers (rows split evenly, at least 256 rows each) and
  // nred reducers (one per group of 16 streamers)
  const auto ngr = [](int n) { return (n + FUSED_GROUP - 1) / FUSED_GROUP; };
  int cap = cus - 2;
  while (cap > 1 && 1 + cap + ngr(cap) > cus) --cap;
  if (max_wg > 0) cap = std::min(cap, max_wg);
  cap = std::max(cap, 1);
  // row ranges start on 256-B boundaries (64 rows): a range split inside a 128-B line costs
  // ~8 % of the streaming rate (measured); BRR_ROW_ALIGN overrides (diagnostics)
  // B >= 256 (C2): whole 256-row passes per streaming workgroup, i.e. fewer and fuller workgroups
  // (C2 f32: 196 x 512 rows instead of 224 x 448, 30.9 -> 31.8 sweeps/s, driver window 34.0 -> 33.3
  // ms; 2-bit 46.5 -> 46.2, within noise, taken too so that both storages keep one geometry and
  // bit-identical chains; profiles/r03_geometry_ab.log).  B = 128 (C3 / C4): unchanged within
  // noise, kept at 64.
  const char *al = getenv("BRR_ROW_ALIGN");
  const int64_t align = al && atoi(al) >= 4 ? (atoi(al) + 3) / 4 * 4 : (d.B >= 256 ? SROWS : 64);
  int64_t rpw = (d.N + cap - 1) / cap;
  rpw = std::max<int64_t>(SROWS, (rpw + align - 1) / align * align);
  const int nsg = (int)((d.N + rpw - 1) / rpw);
  const int npass = (int)((rpw + SROWS - 1) / SROWS);
  // reducers: 4 (BRR_NRED: another power of two, diagnostics), each owning B / nred columns
  // (reduce_role); the streamers still arrive in groups of FUSED_GROUP.  Same box, sweeps/s for
  // 1 / 2 / 4 / 8 reducers: C2 2-bit 45.2 / 51.2 / 53.0 / 52.9, C3 10.8 / 10.8 / 10.9 / 10.7, C2 f32
  // (ms per step, driver's window) 32.77 / 32.40 / 32.46 / 33.05 -- more reducer workgroups slow the
  // stream (32: C2 34.4 ms); the round-3 form (4 reducers, each a group of 64 streamers for all B
  // columns, the solver summing 4 rows) 47.5 / 10.35 / 32.64 (profiles/r04g_ab.log)
  const char *nre = getenv("BRR_NRED");
  const int nred_cap = nre && atoi(nre) >= 1 ? atoi(nre) : 4;
  int nred = 1;
  while (2 * nred <= nred_cap && 1 + nsg + 2 * nred <= cus && d.B % (2 * nred) == 0 && d.B / (2 * nred) >= 8) nred *= 2;
  if (RED_NT % (d.B / nred) != 0) return false;
  if (nsg > d.RG + 1) return false;  // slab1 rows
  const bool xf = d.Xc != nullptr;
  // BRR_FUSED_SINGLE=1: every role in one k_sweep grid (the PMC passes' form, launch_sweep_fused)
  const char *one = getenv("BRR_FUSED_SINGLE");
  const bool split = !(one && one[0] == '1');
  // 2-bit storage at B >= 256: 1,024-thread streaming workgroups (four waves per SIMD; each wave
  // still a whole number of 16-column chunks); BRR_STREAM_NT=512 keeps eight waves (diagnostics)
  const char *snt_env = getenv("BRR_STREAM_NT");
  const int stnt = (split && xf && d.B % (16 * STREAM_CW) == 0 && !(snt_env && atoi(snt_env) == 512)) ? 1024 : SWEEP_NT;
  const void *fn = split ? solve_kernel(d.model, d.B) : sweep_kernel(d.model, d.B, xf ? 1 : 0);
  const void *fst = split ? stream_kernel(xf ? 1 : 0, stnt) : nullptr;
  if (!fn) return false;
  hipFuncAttributes attr, attr_st;
  if (hipFuncGetAttributes(&attr, fn) != hipSuccess) return false;
  if (split && hipFuncGetAttributes(&attr_st, fst) != hipSuccess) return false;
  const size_t budget = SOLVE_LDS_MAX - attr.sharedSizeBytes;
  const int K = d.model == MODEL_HORSESHOE ? 1 : d.K;
  const size_t fixed = solve_fixed_bytes(d.B, K, d.lag);  // (the persistent solver keeps d.lag lists in LDS)
  if (fixed + 8 * (size_t)d.B > budget) return false;
  const int snt = split ? SOLVE_NT : SWEEP_NT;  // the solver workgroup's threads
  const int nslot = (int)std::min<size_t>((size_t)solve_max_slots(d.B, snt), (budget - fixed) / (8 * (size_t)d.B));
  if ((size_t)nslot * d.B < solve_scratch_doubles(d.B, snt)) return false;
  // streamers: residual rows, [the value tables of two blocks], the change list (indices, old and
  // new betas), the member indices of two blocks in LDS
  // (f32 storage with a class-code cache: the value tables and code tiles as for 2-bit storage)
  const bool tables = xf || f32cc;
  const size_t lut_bytes = (size_t)d.B * 32 * (d.lag + 3) + (size_t)(d.B + 16) * 64;  // + the apply's pair tables
  const size_t eps_base = (size_t)npass * SROWS * sizeof(double) + (size_t)(d.B + 16) * (2 * sizeof(double) + sizeof(int)) +
                          2 * sizeof(int) * d.B + (size_t)SWEEP_NW * SROWS * sizeof(double);
  const size_t code_bytes = (size_t)(d.lag + 2) * d.B * npass * 64;
  const size_t st_budget = split ? SOLVE_LDS_MAX - attr_st.sharedSizeBytes : budget;
  const bool ccache = tables && eps_base + lut_bytes + code_bytes <= st_budget && !getenv("BRR_NO_CODE_CACHE");
  const size_t st_lds = eps_base + (xf || ccache ? lut_bytes : 0) + (ccache ? code_bytes : 0);
  // (split, f32 storage) the list prefetch's staging area in the room left: up to 32 entries of
  // npass KiB, when every wave has at most one pass (BRR_LIST_PREFETCH=0: off)
  // (one-kernel form: the same staging area where the grid's LDS request leaves room, so that the PMC
  // passes count the prefetching stream)
  int pfe = 0;
  if (!xf && !ccache && npass <= SWEEP_NW && !(getenv("BRR_LIST_PREFETCH") && getenv("BRR_LIST_PREFETCH")[0] == '0')) {
    const size_t cap_lds = split ? st_budget : budget;
    const size_t room = cap_lds > st_lds ? cap_lds - st_lds : 0;
    pfe = (int)std::min<size_t>(32, room / ((size_t)npass * SROWS * sizeof(float))) / 16 * 16;
  }
  const size_t st_lds_pf = st_lds + (size_t)pfe * npass * SROWS * sizeof(float);
  const size_t lds = split ? fixed + (size_t)nslot * 8 * d.B : std::max(fixed + (size_t)nslot * 8 * d.B, st_lds_pf);
  if (lds > budget || st_lds > st_budget) return false;
  // (one-kernel form) the variant this configuration launches (launch_sweep_fused)
  const int xv1 = xf ? 1 : ccache ? 2 : 0;
  if (!split) fn = sweep_kernel(d.model, d.B, xv1);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)budget) != hipSuccess) return false;
  for (int pv = 0; pv < 2 && split; ++pv) {  // (both the timed and the diagnostics variant)
    if (hipFuncSetAttribute(stream_kernel(xf ? 1 : 0, stnt, pv), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)st_budget) != hipSuccess)
      return false;
    if (!xf && ccache &&
        hipFuncSetAttribute(stream_kernel(2, SWEEP_NT, pv), hipFuncAttributeMaxDynamicSharedMemorySize, (int)st_budget) !=
            hipSuccess)
      return false;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, snt, lds) != hipSuccess || per_cu < 1)
    return false;
  cfg->split = split ? 1 : 0;
  // (split) the streaming kernel's LDS request: padded past half a CU's LDS, one workgroup per CU
  cfg->st_lds = split ? std::min(st_budget, std::max(st_lds_pf, STREAM_LDS_MIN - attr_st.sharedSizeBytes)) : 0;
  cfg->pfe = pfe;
  if (split) {
    per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fst, stnt, cfg->st_lds) != hipSuccess || per_cu != 1)
      return false;
    cfg->stnt = stnt;
    if (1 + nsg + nred > cus) return false;
  }
  cfg->nsg = nsg;
  cfg->rpw = (int)rpw;
  cfg->npass = npass;
  cfg->nslot = nslot;
  cfg->ngroups = 1;  // slab2 rows: every column's whole sum
  cfg->nred = nred;
  cfg->narr = ngr(nsg);
  cfg->lds = lds;
  cfg->ccache = (xf && ccache) ? 1 : 0;
  cfg->f32cc = (!xf && ccache) ? 1 : 0;
  // room in a reducer's LDS for its cross-Gram slices (reduce_role, Dev::rcpf): the partial sums, a list,
  // and d.lag slices of B rows x B / nred columns
  const size_t red_need = 8 * ((size_t)RED_NT + (size_t)(d.B + 16) + (size_t)(d.B + 16) / 2 + (size_t)d.lag * d.B * (d.B / nred));
  cfg->rcpf = red_need <= (split ? cfg->st_lds : lds) ? 1 : 0;
  return true;
}

// The marker loop's launch.  Default: the solver kernel and the streaming kernel side by side on two
// queues.  BRR_FUSED_SINGLE=1: every role in one k_sweep grid (the form PMC counter passes count:
// counter collection serialises dispatches, so two co-dependent kernels cannot both run under it).
// Both are plain launches: the in-kernel residency census (every workgroup running before any waits
// on another, else all leave before touching state) guards the hand-over.  BRR_TEST_CENSUS_EXTRA
// (tests) raises the census target above the grid to exercise the failed-census exit.
// the overlapped solver (Dev::ovs, brr_ovsolve.hpp) fits this configuration: BayesR family, B = 128, K <= 4,
// pipeline lag <= 2, and its LDS layout within the solver workgroup's budget
bool ov_solver_ok(const Dev &d, const FusedCfg &c) {
  if (c.nsg == 0 || d.model == MODEL_HORSESHOE || d.B != OVB || d.K > OV_KMAX || d.K < 1 || d.lag > 2) return false;
  hipFuncAttributes attr;
  const void *fn = c.split ? solve_kernel(d.model, d.B) : sweep_kernel(d.model, d.B, 0);
  if (!fn || hipFuncGetAttributes(&attr, fn) != hipSuccess) return false;
  return OV_LDS + attr.sharedSizeBytes <= SOLVE_LDS_MAX;
}

hipError_t launch_sweep_fused(const Dev &d, uint32_t it, const FusedCfg &c_in, hipStream_t st, hipStream_t st_side,
                              hipEvent_t ev_go, hipEvent_t ev_done) {
  FusedCfg c = c_in;
  if (d.ovs) c.lds = std::max(c.lds, OV_LDS);
  Dev dd = d;
  if (const char *ex = getenv("BRR_TEST_CENSUS_EXTRA")) dd.abase += atoi(ex);
  int nslot = c.nslot, nsg = c.nsg, rpw = c.rpw, npass = c.npass, nred = c.nred, cc = c.ccache;
  if (c.split) {
    // the streaming kernel on the side stream, released by the same event that precedes the
    // solver on the session stream; the session stream waits for it before the next launch
    const int xv = stream_variant(d, c);
    const void *fs = solve_kernel(d.model, d.B), *ft = stream_kernel(xv, xv == 1 ? c.stnt : SWEEP_NT, c.prof != 0);
    if (xv == 2) cc = 1;  // (k_sweep_stream<2> always keeps the cache)
    if (!fs || !ft) return hipErrorInvalidValue;
    int total = nsg + 1 + nred;
    hipError_t e = hipEventRecord(ev_go, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(st_side, ev_go, 0);
    void *sargs[] = {&dd, &it, &nslot, &total};
    if (e == hipSuccess) e = hipLaunchKernel(fs, dim3(1), dim3(SOLVE_NT), sargs, (unsigned)c.lds, st);
    int pfe = xv == 0 ? c.pfe : 0;
    void *targs[] = {&dd, &nsg, &rpw, &npass, &nred, &cc, &pfe};
    if (e == hipSuccess)
      e = hipLaunchKernel(ft, dim3((unsigned)(nsg + nred)), dim3(xv == 1 ? c.stnt : SWEEP_NT), targs, (unsigned)c.st_lds,
                          st_side);
    if (e == hipSuccess) e = hipEventRecord(ev_done, st_side);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, ev_done, 0);
    return e;
  }
  // one kernel: the same streaming variant and list prefetch as the two-kernel form (at 512 threads)
  const int xv = stream_variant(d, c);
  const void *fn = sweep_kernel(d.model, d.B, xv);
  if (!fn) return hipErrorInvalidValue;
  if (xv == 2) cc = 1;
  int pfe = xv == 0 ? c.pfe : 0;
  void *args[] = {&dd, &it, &nslot, &nsg, &rpw, &npass, &nred, &cc, &pfe};
  return hipLaunchKernel(fn, dim3((unsigned)(c.nsg + 1 + c.nred)), dim3(SWEEP_NT), args, (unsigned)c.lds, st);
}

hipError_t launch_prep(const Dev &d, uint32_t it, hipStream_t st) {
  const unsigned grid = cdiv64(d.nbB, 256);
  if (d.model == MODEL_HORSESHOE)
    hipLaunchKernelGGL(k_prep<true>, dim3(grid), dim3(256), 0, st, d, it);
  else
    hipLaunchKernelGGL(k_prep<false>, dim3(grid), dim3(256), 0, st, d, it);
  return hipGetLastError();
}

// Gram-row slots that fit next to the per-position arrays (all rows when possible)
static int solve_slots(int B, int K) {
  const size_t fixed = solve_fixed_bytes(B, K);
  const int n = (int)((SOLVE_LDS_MAX - fixed) / (8 * (size_t)B));
  const int mx = solve_max_slots(B, 256);
  return n < mx ? n : mx;
}

size_t solve_lds_bytes(int B, int K) { return solve_fixed_bytes(B, K) + (size_t)solve_slots(B, K) * 8 * B; }

template <bool HS>
static void launch_solve_b(const Dev &d, int s, uint32_t it, hipStream_t st) {
  const int K = HS ? 1 : d.K;
  const int ns = solve_slots(d.B, K);
  const size_t lds = solve_lds_bytes(d.B, K);
  switch (d.B) {
    case 64: hipLaunchKernelGGL((k_solve<HS, 64>), dim3(1), dim3(256), lds, st, d, s, it, ns); break;
    case 128: hipLaunchKernelGGL((k_solve<HS, 128>), dim3(1), dim3(256), lds, st, d, s, it, ns); break;
    case 256: hipLaunchKernelGGL((k_solve<HS, 256>), dim3(1), dim3(256), lds, st, d, s, it, ns); break;
    default: hipLaunchKernelGGL((k_solve<HS, 512>), dim3(1), dim3(256), lds, st, d, s, it, ns); break;
  }
}

hipError_t launch_solve(const Dev &d, int s, uint32_t it, hipStream_t st) {
  if (d.model == MODEL_HORSESHOE) launch_solve_b<true>(d, s, it, st);
  else launch_solve_b<false>(d, s, it, st);
  return hipGetLastError();
}

hipError_t set_solve_lds_limit(int /*B*/) {
  // One limit for every variant, the largest any configuration uses: lowering it for one
  // session silently shrank the LDS window of later launches (out-of-range LDS writes are
  // dropped, no fault).
  const int lds = (int)SOLVE_LDS_MAX;
  const void *fns[8] = {(const void *)k_solve<true, 64>, (const void *)k_solve<false, 64>,
                        (const void *)k_solve<true, 128>, (const void *)k_solve<false, 128>,
                        (const void *)k_solve<true, 256>, (const void *)k_solve<false, 256>,
                        (const void *)k_solve<true, 512>, (const void *)k_solve<false, 512>};
  for (const void *f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_linpred(const Dev &d, double *out, hipStream_t st) {
  hipLaunchKernelGGL(k_linpred, dim3(cdiv64(d.N, 256)), dim3(256), 0, st, d, out);
  return hipGetLastError();
}

__global__ void k_slab_sentinels(double *slab2, int64_t stride, int nrow, int B, int epoch0) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int p = blockIdx.y;
  if (i < (int64_t)nrow * B) reinterpret_cast<unsigned long long *>(slab2 + p * stride)[i] = slab_sentinel(epoch0 + p);
}
// the persistent solver's slab2 slots before the session's first fused sweep: slot p holds block p's
// sentinel (epoch p); nrow = the padded row count (all of them)
hipError_t launch_slab_sentinels(const Dev &d, int nrow, hipStream_t st) {
  hipLaunchKernelGGL(k_slab_sentinels, dim3(cdiv64((int64_t)nrow * d.B, 256), NPAR), dim3(256), 0, st, d.slab2,
                     d.slab2_stride, nrow, d.B, 0);
  return hipGetLastError();
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
