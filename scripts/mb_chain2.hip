// Microbenchmark of the blocked Horseshoe chain (bayesrrcpp_amd/csrc/brr_chain.hpp) on an idle
// GPU: cycles per step for B = 128 and 64, one wave, Gram block in LDS, against a plain
// sequential forward substitution on the host (values checked).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/mb_chain2.hip -o scripts/mb_chain2.bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../bayesrrcpp_amd/csrc/brr_chain.hpp"

template <int B>
__global__ void k_mb(const double *G, const int *gi, const double *r0, const double *D, const double *sdz,
                     const double *bo, double *bn, unsigned long long *cyc, int reps, int bs) {
  extern __shared__ double sm[];
  double *slots = sm;
  double *Lr0 = slots + B * B, *Ld = Lr0 + B, *Lz = Ld + B, *Lbo = Lz + B, *Lbn = Lbo + B;
  int *Lgi = reinterpret_cast<int *>(Lbn + B);
  for (int i = threadIdx.x; i < B * B; i += blockDim.x) slots[i] = G[i];
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    Lr0[i] = r0[i]; Ld[i] = D[i]; Lz[i] = sdz[i]; Lbo[i] = bo[i]; Lgi[i] = gi[i];
  }
  __syncthreads();
  // coefficient matrix as solve_block makes it (brr::chain_coefficients)
  double *Linv = Lbn;
  __shared__ int Lposg[B];
  for (int i = threadIdx.x; i < B; i += blockDim.x) { Linv[i] = 0.0; Lposg[i] = B; }
  __syncthreads();
  for (int i = threadIdx.x; i < bs; i += blockDim.x) { Linv[Lgi[i]] = 1.0 / Ld[i]; Lposg[Lgi[i]] = i; }
  __syncthreads();
  for (int e = threadIdx.x; e < B * B; e += blockDim.x) {
    const int r = e / B, c = e % B;
    slots[e] = Lposg[r] < Lposg[c] ? slots[e] * Linv[c] : 0.0;
  }
  __syncthreads();
  unsigned long long t0 = 0, t1 = 0;
  if (threadIdx.x < 64) {
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) brr::chain_hs_blocked<B>(bs, Lr0, Ld, Lz, Lbo, Lbn, Lgi, slots);
    t1 = __builtin_amdgcn_s_memtime();
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B; i += blockDim.x) bn[i] = Lbn[i];
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int B>
void run(int bs, int threads) {
  std::vector<double> G(B * B), r0(B), D(B), sdz(B), bo(B), bn(B), ref(B);
  std::vector<int> gi(B);
  srand(7);
  for (int i = 0; i < B; ++i) gi[i] = i;
  // a permutation of 0 .. bs-1 over the valid positions (as the sweep's within-block order is),
  // the rest past the end
  for (int i = bs - 1; i > 0; --i) std::swap(gi[i], gi[rand() % (i + 1)]);
  for (int a = 0; a < B; ++a)
    for (int b = 0; b <= a; ++b) {
      const double v = a == b ? 1000.0 : ((rand() % 2001) - 1000) * 0.05;
      G[a * B + b] = G[b * B + a] = v;
    }
  for (int i = 0; i < B; ++i) {
    r0[i] = ((rand() % 2001) - 1000) * 0.1;
    D[i] = G[gi[i] * B + gi[i]] + 3.0 + (rand() % 100);
    sdz[i] = ((rand() % 2001) - 1000) * 1e-4;
    bo[i] = ((rand() % 2001) - 1000) * 1e-3;
  }
  // host reference: sequential single-site updates in position order
  std::vector<double> num(r0);
  for (int j = 0; j < bs; ++j) {
    ref[j] = num[j] / D[j] + sdz[j];
    const double delta = ref[j] - bo[j];
    for (int k = j + 1; k < bs; ++k) num[k] -= G[gi[j] * B + gi[k]] * delta;
  }
  double *dG, *dr0, *dD, *dz, *dbo, *dbn;
  int *dgi;
  unsigned long long *dc;
  hipMalloc(&dG, 8 * B * B); hipMalloc(&dr0, 8 * B); hipMalloc(&dD, 8 * B); hipMalloc(&dz, 8 * B);
  hipMalloc(&dbo, 8 * B); hipMalloc(&dbn, 8 * B); hipMalloc(&dgi, 4 * B); hipMalloc(&dc, 8);
  hipMemcpy(dG, G.data(), 8 * B * B, hipMemcpyHostToDevice);
  hipMemcpy(dr0, r0.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dD, D.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dz, sdz.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dbo, bo.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dgi, gi.data(), 4 * B, hipMemcpyHostToDevice);
  const size_t lds = 8 * (size_t)B * B + 5 * 8 * B + 4 * B;
  hipFuncSetAttribute((const void *)k_mb<B>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int reps = 200;
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(k_mb<B>, dim3(1), dim3(threads), lds, 0, dG, dgi, dr0, dD, dz, dbo, dbn, dc, reps, bs);
    hipDeviceSynchronize();
  }
  unsigned long long c = 0;
  hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  hipMemcpy(bn.data(), dbn, 8 * B, hipMemcpyDeviceToHost);
  double err = 0;
  for (int j = 0; j < bs; ++j) err = fmax(err, fabs(bn[j] - ref[j]) / fmax(1e-300, fabs(ref[j])));
  std::printf("B=%d bs=%d threads=%d: %.1f cycles/step, max rel err vs sequential %.2e\n", B, bs, threads,
              (double)c / ((double)reps * B), err);
}

int main() {
  run<128>(128, 64);
  run<128>(128, 512);
  run<128>(100, 512);
  run<64>(64, 512);
  return 0;
}
