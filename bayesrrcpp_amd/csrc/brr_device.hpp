// brr_device.hpp -- data layout shared by the HIP kernels and the host session.
//
// HBM layout (one session = one GPU = one column shard):
//   X        f32, column-major, ld = roundup(N, 64) rows (256-B aligned columns); the only
//            large array: streamed once per sweep by k_stream.
//   eps      f64 [N] residual (Y - mu - X beta), owned row-wise by k_stream workgroups.
//   beta,xsq f64 [M]; comp int32 [M]; sel uint8 [M] (marker selected a component this sweep)
//   gram     f64 [nb][B][B] block Gram matrices X_b^T X_b of the fixed column blocks.
//   member   int32 [nb*B] marker at (block position s, slot i); gidx = its row in the Gram.
//   slab1/2  f64 partial dot products (2-level deterministic reduction, see k_stream).
#pragma once
#include <stdint.h>

namespace brr {

constexpr int MAXK = 8;         // mixture components incl. zero
constexpr int MAXG = 64;        // groups
constexpr int BMAX = 128;       // marker block (f64 Gram block must fit LDS: 128 KiB)
constexpr int STREAM_GROUP = 16;  // k_stream workgroups per first-level reduction group
constexpr int FALLTHROUGH = 255;  // no component selected (700-guard, BayesRv2.cpp:216-242)

enum Model : int { MODEL_V2 = 0, MODEL_GROUPS = 1, MODEL_RESTART = 2, MODEL_HORSESHOE = 3 };

// Device-resident scalar state of a chain.
struct Scal {
  double mu, mu_prev, sigmaE, sigmaF, tau, eta, c2;
  double S1;   // sum(eps + mu)   (BayesRv2.cpp:177-178 operand), from the latest row pass
  double S2;   // ||eps||^2        (BayesRv2.cpp:251 operand)
  int n_pend;  // pending residual updates (previous block's changed markers)
  int pad;
  unsigned long long n_slow;     // diagnostics: serial steps that needed the exact re-evaluation
  unsigned long long n_changed;  // diagnostics: markers whose beta changed
};

struct Hyper {
  double sigma0, v0E, s02E, v0G, s02G;   // BayesR family
  double A, vL, vT, c2_0, vC, sC;         // Horseshoe
};

// Stats vector (reduced over markers, summed across shards):
//   [0] sum beta^2  [1] sum beta^2/lambda  [2 .. 2+G) betaAcum[g]  [2+G .. 2+G+G*K) v[g][k]
__host__ __device__ inline int stats_size(int G, int K) { return 2 + G + G * K; }

// Everything a kernel needs: dimensions, hyper-parameters and device pointers (by value).
struct Dev {
  int64_t N, ld, M, M_total, col_offset;
  int K, G, F, B, nb, model, R, RG, NG, MRG;
  uint64_t seed;
  Hyper hyp;
  const float *X;
  const double *Y, *fixed, *cva;
  const int *gAssign;
  double *eps, *eps_start, *deps, *beta, *xsq, *lambda, *hsv, *sigmaGG, *pi, *alpha;
  int *comp, *forder;
  uint8_t *sel;
  double *gram;
  int *member, *gidx, *bsz, *gblk, *blkorder;
  double *slab1, *slab2;
  int *cnt1;
  int *pend_idx;
  double *pend_bo, *pend_bn;
  double *rslab;
  int *rcnt;
  double *mslab;
  int *mcnt;
  double *stats;
  Scal *sc;
};

}  // namespace brr
