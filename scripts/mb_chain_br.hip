// Microbenchmark of the BayesR resident serial chain, per-step form (chain_bayesr_resident) against the
// sub-block form (chain_bayesr_resident_blk; both in
// bayesrrcpp_amd/csrc/brr_kernels.hip) on an idle GPU: shader cycles per chain step for B = 128
// with `nact` positions predicted to change (C3-like: ~24 per block) and every position inside its
// decision window (the fast path), one wave, Gram block in LDS -- to separate the chain's own cost
// from the fused kernel's context.  Values are checked against a host forward substitution.
// The two forms must give bit-identical new betas (checked).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bayesrrcpp_amd/csrc scripts/mb_chain_br.hip -o scripts/mb_chain_br.bin
#include "../bayesrrcpp_amd/csrc/brr_kernels.hip"

#include <cstdio>
#include <cstring>
#include <vector>

using namespace brr;

template <int B, int BLK>
__global__ __launch_bounds__(512, 1) void k_mb_br(Dev d, const double *G, const int *gi, const double *r0, const double *D, const double *sdz,
                        const double *bo, const int *fl, double *bn, unsigned long long *cyc, int reps, int bs) {
  extern __shared__ double sm[];
  double *coef = sm;
  double *Lr0 = coef + B * B, *Llo = Lr0 + B, *Lhi = Llo + B, *Ld = Lhi + B, *Lz = Ld + B, *Lbo = Lz + B,
         *Lbn = Lbo + B, *La = Lbn + B, *Lden = La + 4 * B, *Lp = Lden + 3 * B, *Lx2 = Lp + B, *Lzz = Lx2 + B;
  int *Lgi = reinterpret_cast<int *>(Lzz + B), *Lfl = Lgi + B, *Lks = Lfl + B, *Lm = Lks + B;
  __shared__ int Lposg[B];
  for (int i = threadIdx.x; i < B * B; i += blockDim.x) coef[i] = G[i];
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    Lr0[i] = r0[i]; Llo[i] = 0.0; Lhi[i] = 1e300; Ld[i] = D[i]; Lz[i] = sdz[i]; Lbo[i] = bo[i]; Lgi[i] = gi[i];
    Lfl[i] = fl[i]; Lks[i] = fl[i] & 0xFF; Lm[i] = i; Lp[i] = 0.5; Lx2[i] = D[i]; Lzz[i] = 0.0;
    for (int k = 0; k < 4; ++k) La[k * B + i] = 0.0;
    for (int k = 0; k < 3; ++k) Lden[k * B + i] = D[i];
  }
  __syncthreads();
  // zero-masked Gram: entry (g_i, g_j) kept when position i comes before position j
  for (int i = threadIdx.x; i < B; i += blockDim.x) Lposg[i] = B;
  __syncthreads();
  for (int i = threadIdx.x; i < bs; i += blockDim.x) Lposg[Lgi[i]] = i;
  __syncthreads();
  for (int e = threadIdx.x; e < B * B; e += blockDim.x) {
    const int r = e / B, c = e % B;
    coef[e] = Lposg[r] < Lposg[c] ? coef[e] : 0.0;
  }
  __syncthreads();
  unsigned long long t0 = 0, t1 = 0, tr = 0;
  if (threadIdx.x < 64) {
    // the chain rewrites its inputs (current num, new beta): every repetition restores them
    // first; the restore alone is timed separately and subtracted
    const int l = threadIdx.x;
    const double ra = r0[l], rb = r0[l + 64], ba = bo[l], bb = bo[l + 64];
    const int fa = fl[l], fb = fl[l + 64];
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
      Lr0[l] = ra; Lr0[l + 64] = rb; Lbn[l] = ba; Lbn[l + 64] = bb; Lfl[l] = fa; Lfl[l + 64] = fb;
      __builtin_amdgcn_wave_barrier();
    }
    tr = __builtin_amdgcn_s_memtime() - t0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
      Lr0[l] = ra; Lr0[l + 64] = rb; Lbn[l] = ba; Lbn[l + 64] = bb; Lfl[l] = fa; Lfl[l + 64] = fb;
      __builtin_amdgcn_wave_barrier();
      if constexpr (BLK)
        chain_bayesr_resident_blk<B>(d, bs, 1.0, Lr0, Llo, Lhi, Ld, Lz, Lbo, Lbn, Lfl, Lks, Lgi, La, Lden, Lp, Lx2, Lzz,
                                     Lm, coef, false);
      else
        chain_bayesr_resident<B>(d, bs, 1.0, Lr0, Llo, Lhi, Ld, Lz, Lbo, Lbn, Lfl, Lks, Lgi, La, Lden, Lp, Lx2, Lzz, Lm,
                                 coef, false);
    }
    t1 = __builtin_amdgcn_s_memtime() - tr;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B; i += blockDim.x) bn[i] = Lbn[i];
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int B>
void run(int bs, int nact) {
  std::vector<double> G(B * B), r0(B), D(B), sdz(B), bo(B), bn(B), ref(B);
  std::vector<int> gi(B), fl(B, 0);
  srand(7);
  for (int i = 0; i < B; ++i) gi[i] = i;
  for (int i = bs - 1; i > 0; --i) std::swap(gi[i], gi[rand() % (i + 1)]);
  for (int a = 0; a < B; ++a)
    for (int b = 0; b <= a; ++b) {
      const double v = a == b ? 1000.0 : ((rand() % 2001) - 1000) * 0.05;
      G[a * B + b] = G[b * B + a] = v;
    }
  std::vector<int> idx(bs);
  for (int i = 0; i < bs; ++i) idx[i] = i;
  for (int i = bs - 1; i > 0; --i) std::swap(idx[i], idx[rand() % (i + 1)]);
  for (int i = 0; i < nact; ++i) fl[idx[i]] = 1 | (1 << 9);  // component 1, PF_LIKELY
  for (int i = 0; i < B; ++i) {
    r0[i] = ((rand() % 2001) - 1000) * 0.1;
    D[i] = G[gi[i] * B + gi[i]] + 3.0 + (rand() % 100);
    sdz[i] = ((rand() % 2001) - 1000) * 1e-4;
    bo[i] = ((rand() % 2001) - 1000) * 1e-3;
  }
  std::vector<double> num(r0);
  for (int j = 0; j < bs; ++j) {
    ref[j] = fl[j] ? num[j] / D[j] + sdz[j] : bo[j];
    const double delta = ref[j] - bo[j];
    for (int k = j + 1; k < bs; ++k) num[k] -= G[gi[j] * B + gi[k]] * delta;
  }
  double *dG, *dr0, *dD, *dz, *dbo, *dbn;
  int *dgi, *dfl;
  unsigned long long *dc;
  hipMalloc(&dG, 8 * B * B); hipMalloc(&dr0, 8 * B); hipMalloc(&dD, 8 * B); hipMalloc(&dz, 8 * B);
  hipMalloc(&dbo, 8 * B); hipMalloc(&dbn, 8 * B); hipMalloc(&dgi, 4 * B); hipMalloc(&dfl, 4 * B); hipMalloc(&dc, 8);
  hipMemcpy(dG, G.data(), 8 * B * B, hipMemcpyHostToDevice);
  hipMemcpy(dr0, r0.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dD, D.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dz, sdz.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dbo, bo.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dgi, gi.data(), 4 * B, hipMemcpyHostToDevice);
  hipMemcpy(dfl, fl.data(), 4 * B, hipMemcpyHostToDevice);
  Dev d{};
  d.K = 4; d.G = 1;
  Scal *sc;
  hipMalloc(&sc, sizeof(Scal));
  hipMemset(sc, 0, sizeof(Scal));
  d.sc = sc;
  const size_t lds = 8 * (size_t)B * B + 8 * (size_t)B * 18 + 4 * (size_t)B * 4;
  hipFuncSetAttribute((const void *)k_mb_br<B, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipFuncSetAttribute((const void *)k_mb_br<B, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int reps = 200;
  std::vector<double> bn0(B);
  for (int v = 0; v < 2; ++v) {
    for (int pass = 0; pass < 2; ++pass) {
      if (v == 0) hipLaunchKernelGGL((k_mb_br<B, 0>), dim3(1), dim3(512), lds, 0, d, dG, dgi, dr0, dD, dz, dbo, dfl, dbn, dc, reps, bs);
      else hipLaunchKernelGGL((k_mb_br<B, 1>), dim3(1), dim3(512), lds, 0, d, dG, dgi, dr0, dD, dz, dbo, dfl, dbn, dc, reps, bs);
      hipDeviceSynchronize();
    }
    unsigned long long c = 0;
    hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    hipMemcpy(bn.data(), dbn, 8 * B, hipMemcpyDeviceToHost);
    double err = 0;
    for (int j = 0; j < bs; ++j) err = fmax(err, fabs(bn[j] - ref[j]) / fmax(1e-300, fabs(ref[j])));
    int same = 1;
    if (v == 0) bn0 = bn;
    else for (int j = 0; j < bs; ++j) same &= std::memcmp(&bn[j], &bn0[j], 8) == 0;
    std::printf("BayesR resident chain %-9s B=%d bs=%d act=%d: %.1f cycles/step (%.0f cycles/block), max rel err %.2e%s\n",
                v ? "sub-block" : "per-step", B, bs, nact, (double)c / ((double)reps * nact), (double)c / reps, err,
                v ? (same ? ", bit-identical to per-step" : ", DIFFERS from per-step") : "");
  }
}

int main() {
  run<128>(128, 24);
  run<128>(128, 64);
  run<128>(128, 4);
  return 0;
}
