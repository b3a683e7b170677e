// Microbenchmark: cycles per step of the Horseshoe forward-substitution chain (one wave, B = 128,
// Gram block in LDS) on an idle GPU, in variants that remove one ingredient at a time:
//   0 full step (gathered Gram row ring + readlane + FMA)
//   1 contiguous row reads instead of the permuted gather
//   2 no Gram reads (constant coefficient)
//   3 no readlane (own lane's value)
// hipcc --offload-arch=gfx950 -O3 scripts/mb_chain.hip -o scripts/mb_chain.bin && ./scripts/mb_chain.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int B = 128, NS = 2, GD = 4;

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

template <int V>
__global__ void k_chain(const double *G, const int *perm, double *out, unsigned long long *cyc, int reps) {
  __shared__ double slots[B * B];
  const int lane = threadIdx.x;
  for (int i = lane; i < B * B; i += 64) slots[i] = G[i];
  __syncthreads();
  double sv[NS], iv[NS];
  int gg[NS];
  for (int q = 0; q < NS; ++q) {
    sv[q] = 1e-3 * (lane + 64 * q);
    iv[q] = 1.0 / (1e5 + lane);
    gg[q] = V == 1 ? lane + 64 * q : perm[lane + 64 * q];
  }
  auto gather = [&](int j, double (&g)[NS]) __attribute__((always_inline)) {
    int gi = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q)
      if ((j >> 6) == q) gi = __builtin_amdgcn_readlane(gg[q], j & 63);
    const double *row = slots + gi * B;
#pragma unroll
    for (int q = 0; q < NS; ++q) g[q] = V == 2 ? 1e-3 : row[gg[q]];
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < reps; ++rep) {
    double gb[GD][NS];
#pragma unroll
    for (int u = 0; u < GD; ++u) gather(u, gb[u]);
    if constexpr (V == 4) {
      // fully unrolled steps (no loop back-edge between a gather and its use)
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const int u = j % GD, qo = j >> 6;
        double h[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) h[q] = lane + 64 * q > j ? gb[u][q] * iv[q] : 0.0;
        if (j + GD < B) gather(j + GD, gb[u]);
        const double delta = readlane_f64(sv[qo], j & 63);
#pragma unroll
        for (int q = qo; q < NS; ++q) sv[q] = __builtin_fma(-h[q], delta, sv[q]);
        __builtin_amdgcn_sched_barrier(0);  // keep the gather GD steps ahead of its use
      }
    } else {
#pragma unroll
    for (int qo = 0; qo < NS; ++qo) {
      for (int j0 = 64 * qo; j0 < 64 * (qo + 1); j0 += GD) {
#pragma unroll
        for (int u = 0; u < GD; ++u) {
          const int j = j0 + u;
          double h[NS];
#pragma unroll
          for (int q = 0; q < NS; ++q) h[q] = lane + 64 * q > j ? gb[u][q] * iv[q] : 0.0;
          if (j + GD < B) gather(j + GD, gb[u]);
          const double delta = V == 3 ? sv[qo] : readlane_f64(sv[qo], j - 64 * qo);
#pragma unroll
          for (int q = qo; q < NS; ++q) sv[q] = __builtin_fma(-h[q], delta, sv[q]);
          if (V == 5) __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = sv[0] + sv[1];
  if (lane == 0) *cyc = t1 - t0;
}

int main() {
  std::vector<double> G(B * B);
  std::vector<int> perm(B);
  for (int i = 0; i < B * B; ++i) G[i] = (rand() % 1000) * 1e-6;
  for (int i = 0; i < B; ++i) perm[i] = i;
  for (int i = B - 1; i > 0; --i) std::swap(perm[i], perm[rand() % (i + 1)]);
  double *dG, *dout;
  int *dperm;
  unsigned long long *dcyc;
  hipMalloc(&dG, sizeof(double) * B * B);
  hipMalloc(&dperm, sizeof(int) * B);
  hipMalloc(&dout, sizeof(double) * 64);
  hipMalloc(&dcyc, sizeof(unsigned long long));
  hipMemcpy(dG, G.data(), sizeof(double) * B * B, hipMemcpyHostToDevice);
  hipMemcpy(dperm, perm.data(), sizeof(int) * B, hipMemcpyHostToDevice);
  const int reps = 200;
  const char *names[6] = {"full (permuted gather)", "contiguous row reads", "no Gram reads", "no readlane",
                          "full, steps unrolled + sched_barrier", "full, rolled + sched_barrier"};
  for (int v = 0; v < 6; ++v) {
    for (int pass = 0; pass < 2; ++pass) {
      switch (v) {
        case 0: hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, dG, dperm, dout, dcyc, reps); break;
        case 1: hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, dG, dperm, dout, dcyc, reps); break;
        case 2: hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, dG, dperm, dout, dcyc, reps); break;
        case 3: hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, dG, dperm, dout, dcyc, reps); break;
        case 4: hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(64), 0, 0, dG, dperm, dout, dcyc, reps); break;
        default: hipLaunchKernelGGL(k_chain<5>, dim3(1), dim3(64), 0, 0, dG, dperm, dout, dcyc, reps); break;
      }
      hipDeviceSynchronize();
    }
    unsigned long long cyc = 0;
    hipMemcpy(&cyc, dcyc, sizeof cyc, hipMemcpyDeviceToHost);
    std::printf("%-26s %.1f cycles/step\n", names[v], (double)cyc / (reps * B));
  }
  return 0;
}
