// Microbenchmark of the resident BayesR chain's re-decisions (chain_bayesr_resident_blk in
// bayesrrcpp_amd/csrc/brr_kernels.hip): every position starts with an empty decision window, so the
// chain re-decides each position when it reaches it (C1 re-decides ~24 of 128 positions per block,
// profiles/r05x_prof_c1.log) -- shader cycles per block and per re-decision, one wave, Gram block in
// LDS, K = 4 with C1-like constants (xsq ~ N = 2000, cva = 1e-4 / 1e-3 / 1e-2).  Prints a hash of the
// new betas and components, so two builds of brr_kernels.hip (the current one and an older copy given
// by -DKFILE) can be checked bit-identical on the same inputs.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bayesrrcpp_amd/csrc scripts/mb_refresh.hip -o scripts/mb_refresh.bin
#ifndef KFILE
#define KFILE "../bayesrrcpp_amd/csrc/brr_kernels.hip"
#endif
#include KFILE

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace brr;

template <int B>
__global__ __launch_bounds__(512, 1) void k_mb_ref(Dev d, const double *G, const int *gi, const double *r0,
                                                   const double *La0, const double *Lden0, const double *p0,
                                                   const double *z0, const double *bo, double *bn, int *kso,
                                                   unsigned long long *cyc, int reps, int bs) {
  extern __shared__ double sm[];
  double *coef = sm;
  double *Lr0 = coef + B * B, *Llo = Lr0 + B, *Lhi = Llo + B, *Ld = Lhi + B, *Lsz = Ld + B, *Lbo = Lsz + B,
         *Lbn = Lbo + B, *La = Lbn + B, *Lden = La + 4 * B, *Lp = Lden + 3 * B, *Lx2 = Lp + B, *Lz = Lx2 + B;
  int *Lgi = reinterpret_cast<int *>(Lz + B), *Lfl = Lgi + B, *Lks = Lfl + B, *Lm = Lks + B;
  for (int i = threadIdx.x; i < B * B; i += blockDim.x) coef[i] = G[i];
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    Lr0[i] = r0[i]; Llo[i] = 1.0; Lhi[i] = -1.0; Ld[i] = 1.0; Lsz[i] = 0.0; Lbo[i] = bo[i]; Lgi[i] = gi[i];
    Lfl[i] = PF_LIKELY; Lks[i] = 0; Lm[i] = i; Lp[i] = p0[i]; Lx2[i] = G[gi[i] * B + gi[i]]; Lz[i] = z0[i];
    for (int k = 0; k < 4; ++k) La[k * B + i] = La0[k * B + i];
    for (int k = 0; k < 3; ++k) Lden[k * B + i] = Lden0[k * B + i];
  }
  __syncthreads();
  unsigned long long t0 = 0, t1 = 0, tr = 0;
  if (threadIdx.x < 64) {
    // the chain rewrites its outputs (new beta, component): every repetition restores them first; the
    // restore alone is timed separately and subtracted
    const int l = threadIdx.x;
    const double ba = bo[l], bb = bo[l + 64];
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
      Lbn[l] = ba; Lbn[l + 64] = bb; Lks[l] = 0; Lks[l + 64] = 0;
      __builtin_amdgcn_wave_barrier();
    }
    tr = __builtin_amdgcn_s_memtime() - t0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
      Lbn[l] = ba; Lbn[l + 64] = bb; Lks[l] = 0; Lks[l + 64] = 0;
      __builtin_amdgcn_wave_barrier();
      chain_bayesr_resident_blk<B>(d, bs, 1.0, Lr0, Llo, Lhi, Ld, Lsz, Lbo, Lbn, Lfl, Lks, Lgi, La, Lden, Lp, Lx2, Lz,
                                   Lm, coef, r == 0);
    }
    t1 = __builtin_amdgcn_s_memtime() - tr;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B; i += blockDim.x) { bn[i] = Lbn[i]; kso[i] = Lks[i]; }
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

static uint64_t fnv(const void *p, size_t n, uint64_t h) {
  const unsigned char *c = (const unsigned char *)p;
  for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  return h;
}

template <int B>
void run(int bs, double rscale, unsigned seed) {
  const int K = 4;
  std::vector<double> G(B * B), r0(B), La(4 * B), Lden(3 * B), p(B), z(B), bo(B), bn(B);
  std::vector<int> gi(B), ks(B);
  srand(seed);
  for (int i = 0; i < B; ++i) gi[i] = i;
  for (int i = bs - 1; i > 0; --i) std::swap(gi[i], gi[rand() % (i + 1)]);
  for (int a = 0; a < B; ++a)
    for (int b = 0; b <= a; ++b) {
      const double v = a == b ? 2000.0 + (rand() % 100) : ((rand() % 2001) - 1000) * 0.05;
      G[a * B + b] = G[b * B + a] = v;
    }
  const double pi[4] = {0.5, 0.3, 0.15, 0.05}, cva[3] = {1e-4, 1e-3, 1e-2};
  for (int i = 0; i < B; ++i) {
    const double xsq = G[gi[i] * B + gi[i]];
    La[i] = std::log(pi[0]);
    for (int k = 1; k < K; ++k) {
      Lden[(k - 1) * B + i] = xsq + 1.0 / cva[k - 1];
      La[k * B + i] = std::log(pi[k]) - 0.5 * std::log(xsq * cva[k - 1] + 1.0);
    }
    r0[i] = ((rand() % 2001) - 1000) * rscale;
    p[i] = (rand() % 1000 + 0.5) / 1000.0;
    z[i] = ((rand() % 2001) - 1000) * 1e-3;
    bo[i] = ((rand() % 2001) - 1000) * 1e-4;
  }
  double *dG, *dr0, *dLa, *dLden, *dp, *dz, *dbo, *dbn, *dpi, *dcva, *dsg;
  int *dgi, *dks;
  unsigned long long *dc;
  hipMalloc(&dG, 8 * B * B); hipMalloc(&dr0, 8 * B); hipMalloc(&dLa, 8 * 4 * B); hipMalloc(&dLden, 8 * 3 * B);
  hipMalloc(&dp, 8 * B); hipMalloc(&dz, 8 * B); hipMalloc(&dbo, 8 * B); hipMalloc(&dbn, 8 * B);
  hipMalloc(&dgi, 4 * B); hipMalloc(&dks, 4 * B); hipMalloc(&dc, 8);
  hipMalloc(&dpi, 8 * 4); hipMalloc(&dcva, 8 * 3); hipMalloc(&dsg, 8);
  hipMemcpy(dG, G.data(), 8 * B * B, hipMemcpyHostToDevice);
  hipMemcpy(dr0, r0.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dLa, La.data(), 8 * 4 * B, hipMemcpyHostToDevice);
  hipMemcpy(dLden, Lden.data(), 8 * 3 * B, hipMemcpyHostToDevice);
  hipMemcpy(dp, p.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dz, z.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dbo, bo.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dgi, gi.data(), 4 * B, hipMemcpyHostToDevice);
  hipMemcpy(dpi, pi, 8 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dcva, cva, 8 * 3, hipMemcpyHostToDevice);
  const double one = 1.0;
  hipMemcpy(dsg, &one, 8, hipMemcpyHostToDevice);
  Dev d{};
  d.K = K; d.G = 1; d.pi = dpi; d.cva = dcva; d.sigmaGG = dsg;
  Scal *sc;
  hipMalloc(&sc, sizeof(Scal));
  hipMemset(sc, 0, sizeof(Scal));
  d.sc = sc;
  const size_t lds = 8 * (size_t)B * B + 8 * (size_t)B * 18 + 4 * (size_t)B * 4;
  hipFuncSetAttribute((const void *)k_mb_ref<B>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int reps = 200;
  for (int pass = 0; pass < 2; ++pass) {
    hipMemset(sc, 0, sizeof(Scal));
    hipLaunchKernelGGL((k_mb_ref<B>), dim3(1), dim3(512), lds, 0, d, dG, dgi, dr0, dLa, dLden, dp, dz, dbo, dbn, dks,
                       dc, reps, bs);
    hipDeviceSynchronize();
  }
  unsigned long long c = 0;
  Scal h{};
  hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  hipMemcpy(&h, sc, sizeof(Scal), hipMemcpyDeviceToHost);
  hipMemcpy(bn.data(), dbn, 8 * B, hipMemcpyDeviceToHost);
  hipMemcpy(ks.data(), dks, 4 * B, hipMemcpyDeviceToHost);
  const double steps = (double)h.prof[6], nref = (double)h.prof[7];
  int nch = 0;
  for (int i = 0; i < bs; ++i) nch += bn[i] != bo[i];
  const uint64_t hsh = fnv(ks.data(), 4 * (size_t)bs, fnv(bn.data(), 8 * (size_t)bs, 1469598103934665603ull));
  std::printf("B=%d bs=%d rscale=%.2f seed=%u: %.0f cycles/block, %.0f steps, %.0f re-decisions, %d changed, "
              "%.0f cycles per (step + re-decision), hash %016llx\n",
              B, bs, rscale, seed, (double)c / reps, steps, nref, nch, (double)c / reps / (steps + nref),
              (unsigned long long)hsh);
  hipFree(dG); hipFree(dr0); hipFree(dLa); hipFree(dLden); hipFree(dp); hipFree(dz); hipFree(dbo); hipFree(dbn);
  hipFree(dgi); hipFree(dks); hipFree(dc); hipFree(dpi); hipFree(dcva); hipFree(dsg); hipFree(sc);
}

int main() {
  run<128>(128, 0.05, 7);
  run<128>(128, 0.2, 11);
  run<128>(128, 0.5, 13);
  run<128>(100, 0.2, 17);
  return 0;
}
