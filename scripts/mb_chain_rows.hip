// Microbenchmark of the BayesR row chain (chain_bayesr_rows in bayesrrcpp_amd/csrc/brr_kernels.hip, the
// B >= 256 chain of the C2 burn-in) on an idle GPU: shader cycles per chain step for B = 512 with `nact`
// positions predicted to change and every position inside its decision window (the fast path), one
// wave.  Rows from LDS static slots (the solver's staged rows) or, `hbm` = 1, every row from the Gram
// block in HBM (the unpredicted positions' path).  Values are checked against a host forward substitution.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bayesrrcpp_amd/csrc scripts/mb_chain_rows.hip -o scripts/mb_chain_rows.bin
#include "../bayesrrcpp_amd/csrc/brr_kernels.hip"

#include <cstdio>
#include <vector>

using namespace brr;

template <int B>
__global__ __launch_bounds__(512, 1) void k_mb_rows(Dev d, const double *G, const int *gi, const double *r0, const double *D,
                                                   const double *sdz, const double *bo, const int *fl, const int *spos,
                                                   int npred, int hbm, double *bn, unsigned long long *cyc, int reps) {
  extern __shared__ double sm[];
  double *Lr0 = sm, *Llo = Lr0 + B, *Lhi = Llo + B, *Ld = Lhi + B, *Lz = Ld + B, *Linv = Lz + B, *Lbo = Linv + B,
         *Lbn = Lbo + B, *La = Lbn + B, *Lden = La + 4 * B, *Lp = Lden + 3 * B, *Lx2 = Lp + B, *Lzz = Lx2 + B;
  int *Lgi = reinterpret_cast<int *>(Lzz + B), *Lfl = Lgi + B, *Lks = Lfl + B, *Lm = Lks + B, *Lslot = Lm + B,
      *Lspos = Lslot + B, *misc = Lspos + B;
  double *slots = reinterpret_cast<double *>(misc + 64);
  const int bs = B;
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    Lr0[i] = r0[i]; Llo[i] = 0.0; Lhi[i] = 1e300; Ld[i] = D[i]; Lz[i] = sdz[i]; Linv[i] = 1.0 / D[i]; Lbo[i] = bo[i];
    Lgi[i] = gi[i]; Lfl[i] = fl[i]; Lks[i] = fl[i] & 0xFF; Lm[i] = i; Lp[i] = 0.5; Lx2[i] = D[i]; Lzz[i] = 0.0;
    Lslot[i] = -1;
    Lbn[i] = bo[i];  // (the chain stores only the visited positions' new betas)
    for (int k = 0; k < 4; ++k) La[k * B + i] = 0.0;
    for (int k = 0; k < 3; ++k) Lden[k * B + i] = D[i];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < npred; k += blockDim.x) { Lspos[k] = spos[k]; if (!hbm) Lslot[spos[k]] = k; }
  __syncthreads();
  if (!hbm)
    for (int e = threadIdx.x; e < npred * B; e += blockDim.x) slots[e] = G[(int64_t)gi[spos[e / B]] * B + e % B];
  __syncthreads();
  unsigned long long t0 = 0, t1 = 0;
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    double rs[B / 64];
    for (int q = 0; q < B / 64; ++q) rs[q] = r0[l + 64 * q];
    for (int pass = 0; pass < 2; ++pass) {  // (pass 0 warms the caches)
      t0 = __builtin_amdgcn_s_memtime();
      for (int r = 0; r < reps; ++r) {
        for (int q = 0; q < B / 64; ++q) Lr0[l + 64 * q] = rs[q];
        __builtin_amdgcn_wave_barrier();
        chain_bayesr_rows<B>(d, bs, 1.0, Lr0, Llo, Lhi, Ld, Lz, Linv, Lbo, Lbn, Lfl, Lks, Lgi, La, Lden, Lp, Lx2, Lzz,
                             Lm, Lslot, Lspos, slots, G, 0, hbm ? 0 : npred, 0, npred, misc + 8, misc + 9, false);
      }
      t1 = __builtin_amdgcn_s_memtime();
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B; i += blockDim.x) bn[i] = Lbn[i];
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int B>
void run(int nact, int hbm) {
  std::vector<double> G((size_t)B * B), r0(B), D(B), sdz(B), bo(B), bn(B), ref(B);
  std::vector<int> gi(B), fl(B, 1), spos;
  srand(11);
  for (int i = 0; i < B; ++i) gi[i] = i;
  for (int i = B - 1; i > 0; --i) std::swap(gi[i], gi[rand() % (i + 1)]);
  for (int a = 0; a < B; ++a)
    for (int b = 0; b <= a; ++b) {
      const double v = a == b ? 5000.0 : ((rand() % 2001) - 1000) * 0.05;
      G[(size_t)a * B + b] = G[(size_t)b * B + a] = v;
    }
  std::vector<int> idx(B);
  for (int i = 0; i < B; ++i) idx[i] = i;
  for (int i = B - 1; i > 0; --i) std::swap(idx[i], idx[rand() % (i + 1)]);
  std::vector<char> act(B, 0);
  for (int i = 0; i < nact; ++i) act[idx[i]] = 1;
  for (int i = 0; i < B; ++i) {
    if (act[i]) { fl[i] = 1 | (1 << 9); spos.push_back(i); }  // component 1, PF_LIKELY (positions in order)
    r0[i] = ((rand() % 2001) - 1000) * 0.1;
    D[i] = G[(size_t)gi[i] * B + gi[i]] + 3.0 + (rand() % 100);
    sdz[i] = ((rand() % 2001) - 1000) * 1e-4;
    bo[i] = ((rand() % 2001) - 1000) * 1e-3;
  }
  std::vector<double> num(r0);
  for (int j = 0; j < B; ++j) {
    ref[j] = act[j] ? num[j] / D[j] + sdz[j] : bo[j];
    const double delta = ref[j] - bo[j];
    if (delta != 0.0)
      for (int k = j + 1; k < B; ++k) num[k] -= G[(size_t)gi[j] * B + gi[k]] * delta;
  }
  double *dG, *dr0, *dD, *dz, *dbo, *dbn;
  int *dgi, *dfl, *dsp;
  unsigned long long *dc;
  hipMalloc(&dG, 8 * (size_t)B * B); hipMalloc(&dr0, 8 * B); hipMalloc(&dD, 8 * B); hipMalloc(&dz, 8 * B);
  hipMalloc(&dbo, 8 * B); hipMalloc(&dbn, 8 * B); hipMalloc(&dgi, 4 * B); hipMalloc(&dfl, 4 * B); hipMalloc(&dsp, 4 * B);
  hipMalloc(&dc, 8);
  hipMemcpy(dG, G.data(), 8 * (size_t)B * B, hipMemcpyHostToDevice);
  hipMemcpy(dr0, r0.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dD, D.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dz, sdz.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dbo, bo.data(), 8 * B, hipMemcpyHostToDevice);
  hipMemcpy(dgi, gi.data(), 4 * B, hipMemcpyHostToDevice);
  hipMemcpy(dfl, fl.data(), 4 * B, hipMemcpyHostToDevice);
  hipMemcpy(dsp, spos.data(), 4 * (size_t)nact, hipMemcpyHostToDevice);
  Dev d{};
  d.K = 4; d.G = 1;
  Scal *sc;
  hipMalloc(&sc, sizeof(Scal));
  hipMemset(sc, 0, sizeof(Scal));
  d.sc = sc;
  const size_t lds = 8 * (size_t)B * 20 + 4 * (size_t)B * 6 + 256 + 8 * (size_t)nact * B;
  hipFuncSetAttribute((const void *)k_mb_rows<B>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int reps = 100;
  hipLaunchKernelGGL(k_mb_rows<B>, dim3(1), dim3(512), lds, 0, d, dG, dgi, dr0, dD, dz, dbo, dfl, dsp, nact, hbm, dbn, dc, reps);
  if (hipDeviceSynchronize() != hipSuccess) { std::printf("kernel failed\n"); return; }
  unsigned long long c = 0;
  hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  hipMemcpy(bn.data(), dbn, 8 * B, hipMemcpyDeviceToHost);
  double err = 0;
  for (int j = 0; j < B; ++j) err = fmax(err, fabs(bn[j] - ref[j]) / fmax(1e-300, fabs(ref[j])));
  std::printf("BayesR row chain B=%d act=%d rows from %s: %.1f cycles/step (%.0f cycles/block), max rel err %.2e\n", B,
              nact, hbm ? "HBM" : "LDS slots", (double)c / ((double)reps * nact), (double)c / reps, err);
}

int main() {
  run<512>(12, 0);
  run<512>(3, 0);
  run<512>(12, 1);
  run<256>(12, 0);
  return 0;
}
