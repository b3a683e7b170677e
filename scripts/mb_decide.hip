// Microbenchmark of one re-decision (decide_fast_wave in bayesrrcpp_amd/csrc/brr_kernels.hip) on one
// wave, its result fed into the next call's num (a dependent chain, as on the serial chain): shader
// cycles per call for the whole decision and for pieces of it (the denominator and the log-weights, the
// softmax's exponential, the cumulative sums and the quotient) to see where a re-decision's time goes.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bayesrrcpp_amd/csrc scripts/mb_decide.hip -o scripts/mb_decide.bin
#include "../bayesrrcpp_amd/csrc/brr_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstring>

using namespace brr;

template <int V>
__device__ __forceinline__ double piece(double r, const double *a, const double *den, int64_t stride, int K,
                                        double sigmaE, double p) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int kl = lane < K ? lane : 0;
  if constexpr (V == 0) {
    const FastDec o = decide_fast_wave(r, a, den, stride, K, sigmaE, p);
    return o.lo + (double)o.k;
  } else if constexpr (V == 6) {  // the compile-time K = 4 form the chains run for K = 4
    const FastDec o = decide_fast_wave<4>(r, a, den, stride, 4, sigmaE, p);
    return o.lo + (double)o.k;
  } else if constexpr (V == 1) {  // the log-weight of this lane's component: load, division, FMA
    const double dk = den[(max(kl, 1) - 1) * stride];
    const double sl = kl == 0 ? 0.0 : 0.5 / (dk * sigmaE);
    return a[kl * stride] + sl * (r * r);
  } else if constexpr (V == 2) {  // V1 + the maximum over the K lanes (readlanes)
    const double dk = den[(max(kl, 1) - 1) * stride];
    const double sl = kl == 0 ? 0.0 : 0.5 / (dk * sigmaE);
    const double Lk = a[kl * stride] + sl * (r * r);
    double mx = -1e308;
    for (int k = 0; k < 4; ++k)
      if (k < K) mx = fmax(mx, readlane_f64(Lk, k));
    return mx;
  } else if constexpr (V == 3) {  // the exponential alone
    return exp(r * 1e-3 - 1.0);
  } else if constexpr (V == 4) {  // one division alone
    return p / (r + 3.0);
  } else if constexpr (V == 5) {  // four readlanes of a double, summed
    double s = 0.0;
    for (int k = 0; k < 4; ++k)
      if (k < K) s += readlane_f64(r + (double)lane, k);
    return s;
  } else {
    return r;
  }
}

template <int V>
__global__ __launch_bounds__(64, 1) void k_mb_dec(const double *a0, const double *den0, double *out,
                                                 unsigned long long *cyc, int reps, int K) {
  __shared__ double La[4 * 64], Lden[3 * 64];
  for (int i = threadIdx.x; i < 4 * 64; i += 64) La[i] = a0[i];
  for (int i = threadIdx.x; i < 3 * 64; i += 64) Lden[i] = den0[i];
  __syncthreads();
  double r = 120.0, acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < reps; ++i) {
    const double v = piece<V>(r, La + (i & 63), Lden + (i & 63), 64, K, 1.0, 0.37);
    acc += v;
    r = 120.0 + (v - v);  // the next call depends on this one's result
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc + r;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int V>
void run(const char *name, const double *da, const double *dd, double *dout, unsigned long long *dc) {
  const int reps = 2000;
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL((k_mb_dec<V>), dim3(1), dim3(64), 0, 0, da, dd, dout, dc, reps, 4);
    hipDeviceSynchronize();
  }
  unsigned long long c = 0;
  double o0 = 0.0;
  hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  hipMemcpy(&o0, dout, 8, hipMemcpyDeviceToHost);
  unsigned long long bits;
  std::memcpy(&bits, &o0, 8);
  std::printf("%-40s %.0f cycles per call (result bits %016llx)\n", name, (double)c / reps, bits);
}

int main() {
  double a[4 * 64], den[3 * 64];
  const double pi[4] = {0.5, 0.3, 0.15, 0.05}, cva[3] = {1e-4, 1e-3, 1e-2};
  for (int i = 0; i < 64; ++i) {
    const double xsq = 2000.0 + i;
    a[i] = std::log(pi[0]);
    for (int k = 1; k < 4; ++k) {
      den[(k - 1) * 64 + i] = xsq + 1.0 / cva[k - 1];
      a[k * 64 + i] = std::log(pi[k]) - 0.5 * std::log(xsq * cva[k - 1] + 1.0);
    }
  }
  double *da, *dd, *dout;
  unsigned long long *dc;
  hipMalloc(&da, sizeof a); hipMalloc(&dd, sizeof den); hipMalloc(&dout, 8 * 64); hipMalloc(&dc, 8);
  hipMemcpy(da, a, sizeof a, hipMemcpyHostToDevice);
  hipMemcpy(dd, den, sizeof den, hipMemcpyHostToDevice);
  run<0>("decide_fast_wave (whole)", da, dd, dout, dc);
  run<6>("decide_fast_wave<4> (whole)", da, dd, dout, dc);
  run<1>("log-weight: load, division, FMA", da, dd, dout, dc);
  run<2>("log-weight + maximum over 4 lanes", da, dd, dout, dc);
  run<3>("exp (f64)", da, dd, dout, dc);
  run<4>("division (f64)", da, dd, dout, dc);
  run<5>("4 readlanes of a double, summed", da, dd, dout, dc);
  return 0;
}
