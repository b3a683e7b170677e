// Microbenchmark: column-block streaming (the k_stream access pattern) on one MI355X.
// X is N x P f32 column-major (ld = roundup(N, 256)); one "launch" reads the B columns of one
// block and forms B partial dot products with an f64 vector.  Variants isolate the cost of the
// read pattern, the in-wave reduction and the cross-workgroup reduction.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/mb_stream.hip -o /tmp/mb_stream
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int SROWS = 256;

__device__ __forceinline__ double wave_reduce32(double (&v)[32], int lane) {
#pragma unroll
  for (int j = 0; j < 16; ++j) { const bool hi = lane & 32; const double send = hi ? v[j] : v[j + 16]; const double keep = hi ? v[j + 16] : v[j]; v[j] = keep + __shfl_xor(send, 32); }
#pragma unroll
  for (int j = 0; j < 8; ++j) { const bool hi = lane & 16; const double send = hi ? v[j] : v[j + 8]; const double keep = hi ? v[j + 8] : v[j]; v[j] = keep + __shfl_xor(send, 16); }
#pragma unroll
  for (int j = 0; j < 4; ++j) { const bool hi = lane & 8; const double send = hi ? v[j] : v[j + 4]; const double keep = hi ? v[j + 4] : v[j]; v[j] = keep + __shfl_xor(send, 8); }
#pragma unroll
  for (int j = 0; j < 2; ++j) { const bool hi = lane & 4; const double send = hi ? v[j] : v[j + 2]; const double keep = hi ? v[j + 2] : v[j]; v[j] = keep + __shfl_xor(send, 4); }
  { const bool hi = lane & 2; const double send = hi ? v[0] : v[1]; const double keep = hi ? v[1] : v[0]; v[0] = keep + __shfl_xor(send, 2); }
  return v[0] + __shfl_xor(v[0], 1);
}

// V0: pure read, 4 rows per lane, CW columns per wave, 4 waves, XCD-aware (rg, cc) mapping
template <int CW>
__global__ __launch_bounds__(256, 2) void v0_read(const float *X, int64_t ld, int N, int RG, int B, int col0, double *out) {
  constexpr int CB = 4 * CW;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int NC = B / CB;
  const int bid = blockIdx.x, rest = bid >> 3, cc = rest % NC, rg = (rest / NC) * 8 + (bid & 7);
  if (rg >= RG) return;
  const int64_t row0 = (int64_t)rg * SROWS + 4 * lane;
  const int64_t rowc = row0 < N ? row0 : 0;
  const float *Xr = X + rowc;
  float4 x[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(Xr + (int64_t)(col0 + cc * CB + w * CW + j) * ld);
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < CW; ++j) a += x[j].x + x[j].y + x[j].z + x[j].w;
  if (a == 12345.f) out[bid] = a;
}

// V1: the k_stream dot + wave transpose-reduction + plain partial stores (no cross-WG reduction)
template <int CW>
__global__ __launch_bounds__(256, 2) void v1_dots(const float *X, int64_t ld, int N, int RG, int B, int col0,
                                                  const double *eps, double *slab1) {
  constexpr int CB = 4 * CW;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int NC = B / CB;
  const int bid = blockIdx.x, rest = bid >> 3, cc = rest % NC, rg = (rest / NC) * 8 + (bid & 7);
  if (rg >= RG) return;
  const int64_t row0 = (int64_t)rg * SROWS + 4 * lane;
  const bool valid = row0 < N;
  const int64_t rowc = valid ? row0 : 0;
  const float *Xr = X + rowc;
  float4 x[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(Xr + (int64_t)(col0 + cc * CB + w * CW + j) * ld);
  const double2 ea = *reinterpret_cast<const double2 *>(eps + rowc);
  const double2 eb = *reinterpret_cast<const double2 *>(eps + rowc + 2);
  double e0 = ea.x, e1 = ea.y, e2 = eb.x, e3 = eb.y;
  if (!valid) e0 = e1 = e2 = e3 = 0.0;
  double v[32];
#pragma unroll
  for (int j = 0; j < 32; ++j)
    v[j] = j < CW ? ((((double)x[j].x * e0 + (double)x[j].y * e1) + (double)x[j].z * e2) + (double)x[j].w * e3) : 0.0;
  const double r = wave_reduce32(v, lane);
  const int col = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
  if ((lane & 1) == 0 && col < CW) slab1[(int64_t)rg * B + cc * CB + w * CW + col] = r;
}

// V2: one workgroup per row tile, loops over all B columns in chunks of 32 per wave with the
// next chunk's loads issued before the current chunk's reduction (software pipelining)
__global__ __launch_bounds__(256, 1) void v2_pipelined(const float *X, int64_t ld, int N, int RG, int B, int col0,
                                                       const double *eps, double *slab1) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int rg = blockIdx.x;
  if (rg >= RG) return;
  const int64_t row0 = (int64_t)rg * SROWS + 4 * lane;
  const bool valid = row0 < N;
  const int64_t rowc = valid ? row0 : 0;
  const float *Xr = X + rowc;
  const double2 ea = *reinterpret_cast<const double2 *>(eps + rowc);
  const double2 eb = *reinterpret_cast<const double2 *>(eps + rowc + 2);
  double e0 = ea.x, e1 = ea.y, e2 = eb.x, e3 = eb.y;
  if (!valid) e0 = e1 = e2 = e3 = 0.0;
  const int nch = B / 128;  // chunks of 32 columns per wave
  float4 xa[32], xb[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) xa[j] = *reinterpret_cast<const float4 *>(Xr + (int64_t)(col0 + w * 32 + j) * ld);
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) {
#pragma unroll
      for (int j = 0; j < 32; ++j) xb[j] = *reinterpret_cast<const float4 *>(Xr + (int64_t)(col0 + (c + 1) * 128 + w * 32 + j) * ld);
    }
    double v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j)
      v[j] = (((double)xa[j].x * e0 + (double)xa[j].y * e1) + (double)xa[j].z * e2) + (double)xa[j].w * e3;
    const double r = wave_reduce32(v, lane);
    const int col = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
    if ((lane & 1) == 0) slab1[(int64_t)rg * B + c * 128 + w * 32 + col] = r;
#pragma unroll
    for (int j = 0; j < 32; ++j) xa[j] = xb[j];
  }
}

// V3: like V1 but 8 waves x 16 columns per workgroup (512 threads), 2 rows... (4 rows per lane)
template <int CW, int NW>
__global__ __launch_bounds__(64 * NW, 1) void v3_dots(const float *X, int64_t ld, int N, int RG, int B, int col0,
                                                       const double *eps, double *slab1) {
  constexpr int CB = NW * CW;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int NC = B / CB;
  const int bid = blockIdx.x, rest = bid >> 3, cc = rest % NC, rg = (rest / NC) * 8 + (bid & 7);
  if (rg >= RG) return;
  const int64_t row0 = (int64_t)rg * SROWS + 4 * lane;
  const bool valid = row0 < N;
  const int64_t rowc = valid ? row0 : 0;
  const float *Xr = X + rowc;
  float4 x[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(Xr + (int64_t)(col0 + cc * CB + w * CW + j) * ld);
  const double2 ea = *reinterpret_cast<const double2 *>(eps + rowc);
  const double2 eb = *reinterpret_cast<const double2 *>(eps + rowc + 2);
  double e0 = ea.x, e1 = ea.y, e2 = eb.x, e3 = eb.y;
  if (!valid) e0 = e1 = e2 = e3 = 0.0;
  double v[32];
#pragma unroll
  for (int j = 0; j < 32; ++j)
    v[j] = j < CW ? ((((double)x[j].x * e0 + (double)x[j].y * e1) + (double)x[j].z * e2) + (double)x[j].w * e3) : 0.0;
  const double r = wave_reduce32(v, lane);
  const int col = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
  if ((lane & 1) == 0 && col < CW) slab1[(int64_t)rg * B + cc * CB + w * CW + col] = r;
}


__device__ __forceinline__ void st_sc1(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), __double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
  return __longlong_as_double(__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// V4: v1 + options: bit0 sc1 partial stores, bit1 level-2 last arriver (16 row tiles) with
// write-through, bit2 16 pending columns applied (neutral), bit3 eps_out write
template <int CW>
__global__ __launch_bounds__(256, 2) void v4_full(const float *X, int64_t ld, int N, int RG, int B, int col0,
                                                  const double *eps, double *eps_out, double *slab1, double *slab2,
                                                  int *cnt1, const int *pidx, int opts) {
  constexpr int CB = 4 * CW;
  __shared__ int s_last;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int NC = B / CB;
  const int bid = blockIdx.x, rest = bid >> 3, cc = rest % NC, rg = (rest / NC) * 8 + (bid & 7);
  if (rg >= RG) return;
  const int64_t row0 = (int64_t)rg * SROWS + 4 * lane;
  const bool valid = row0 < N;
  const int64_t rowc = valid ? row0 : 0;
  const float *Xr = X + rowc;
  float4 x[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(Xr + (int64_t)(col0 + cc * CB + w * CW + j) * ld);
  const double2 ea = *reinterpret_cast<const double2 *>(eps + rowc);
  const double2 eb = *reinterpret_cast<const double2 *>(eps + rowc + 2);
  double e0 = ea.x, e1 = ea.y, e2 = eb.x, e3 = eb.y;
  if (opts & 4) {
    float4 xp[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) xp[q] = *reinterpret_cast<const float4 *>(Xr + (int64_t)pidx[q] * ld);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const double a0 = xp[q].x, a1 = xp[q].y, a2 = xp[q].z, a3 = xp[q].w;
      e0 = (e0 + a0 * 0.0) - a0 * 0.0; e1 = (e1 + a1 * 0.0) - a1 * 0.0;
      e2 = (e2 + a2 * 0.0) - a2 * 0.0; e3 = (e3 + a3 * 0.0) - a3 * 0.0;
    }
  }
  if ((opts & 8) && cc == 0 && w == 0 && valid) {
    *reinterpret_cast<double2 *>(eps_out + row0) = make_double2(e0, e1);
    *reinterpret_cast<double2 *>(eps_out + row0 + 2) = make_double2(e2, e3);
  }
  if (!valid) e0 = e1 = e2 = e3 = 0.0;
  double v[32];
#pragma unroll
  for (int j = 0; j < 32; ++j)
    v[j] = j < CW ? ((((double)x[j].x * e0 + (double)x[j].y * e1) + (double)x[j].z * e2) + (double)x[j].w * e3) : 0.0;
  const double r = wave_reduce32(v, lane);
  const int col = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
  double *dst = slab1 + (int64_t)rg * B + cc * CB + w * CW + col;
  if ((lane & 1) == 0 && col < CW) { if (opts & 1) st_sc1(dst, r); else *dst = r; }
  if (opts & 2) {
    const int grp = rg / 16, g0 = grp * 16, gsz = min(16, RG - g0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) s_last = (__hip_atomic_fetch_add(cnt1 + grp * NC + cc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsz - 1);
    __syncthreads();
    if (s_last) {
      if (t < CB) {
        double acc = 0.0;
        double v16[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v16[q] = q < gsz ? ld_sc1(slab1 + (int64_t)(g0 + q) * B + cc * CB + t) : 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc += v16[q];
        st_sc1(slab2 + (int64_t)grp * B + cc * CB + t, acc);
      }
      if (t == 0) cnt1[grp * NC + cc] = 0;
    }
  }
}

// fake solve: one workgroup that holds a CU (big LDS) for `us` microseconds
__global__ __launch_bounds__(256) void fake_solve(int us, double *out) {
  extern __shared__ double lds[];
  const uint64_t t0 = wall_clock64();
  lds[threadIdx.x] = threadIdx.x;
  while (wall_clock64() - t0 < (uint64_t)us * 100) { __builtin_amdgcn_s_sleep(1); }
  __syncthreads();
  if (threadIdx.x == 0) out[0] = lds[5];
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 100000;
  const int B = argc > 2 ? atoi(argv[2]) : 512;
  const int nblk = argc > 3 ? atoi(argv[3]) : 40;
  const int64_t ld = (N + 255) / 256 * 256;
  const int RG = (N + SROWS - 1) / SROWS;
  const int64_t P = (int64_t)B * nblk;
  float *X; double *eps, *slab1, *out;
  CHK(hipMalloc(&X, sizeof(float) * ld * P));
  CHK(hipMalloc(&eps, sizeof(double) * ld));
  CHK(hipMalloc(&slab1, sizeof(double) * (int64_t)RG * B));
  CHK(hipMalloc(&out, sizeof(double) * 100000));
  CHK(hipMemset(X, 0, sizeof(float) * ld * P));
  CHK(hipMemset(eps, 0, sizeof(double) * ld));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const double bytes = 4.0 * N * B;
  auto run = [&](const char *name, auto launch) {
    for (int b = 0; b < nblk; ++b) launch(b);  // warm
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    const int reps = 3;
    for (int r = 0; r < reps; ++r)
      for (int b = 0; b < nblk; ++b) launch(b);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / (reps * nblk);
    printf("%-28s %8.2f us/launch  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  const unsigned g32 = (unsigned)((RG + 7) / 8 * 8 * (B / 128));
  const unsigned g16 = (unsigned)((RG + 7) / 8 * 8 * (B / 64));
  printf("N=%d B=%d nblk=%d RG=%d (X %.1f GB)\n", N, B, nblk, RG, 4.0 * ld * P / 1e9);
  run("v0_read<32>", [&](int b) { hipLaunchKernelGGL(v0_read<32>, dim3(g32), dim3(256), 0, 0, X, ld, N, RG, B, b * B, out); });
  run("v0_read<16>", [&](int b) { hipLaunchKernelGGL(v0_read<16>, dim3(g16), dim3(256), 0, 0, X, ld, N, RG, B, b * B, out); });
  run("v1_dots<32>", [&](int b) { hipLaunchKernelGGL(v1_dots<32>, dim3(g32), dim3(256), 0, 0, X, ld, N, RG, B, b * B, eps, slab1); });
  run("v1_dots<16>", [&](int b) { hipLaunchKernelGGL(v1_dots<16>, dim3(g16), dim3(256), 0, 0, X, ld, N, RG, B, b * B, eps, slab1); });
  run("v2_pipelined", [&](int b) { hipLaunchKernelGGL(v2_pipelined, dim3((unsigned)RG), dim3(256), 0, 0, X, ld, N, RG, B, b * B, eps, slab1); });
  const unsigned g816 = (unsigned)((RG + 7) / 8 * 8 * (B / 128));
  run("v3_dots<16,8>", [&](int b) { hipLaunchKernelGGL((v3_dots<16, 8>), dim3(g816), dim3(512), 0, 0, X, ld, N, RG, B, b * B, eps, slab1); });
  const unsigned g3216 = (unsigned)((RG + 7) / 8 * 8 * (B / 256));
  if (B >= 256) run("v3_dots<16,16>", [&](int b) { hipLaunchKernelGGL((v3_dots<16, 16>), dim3(g3216), dim3(1024), 0, 0, X, ld, N, RG, B, b * B, eps, slab1); });
  run("v3_dots<32,8>", [&](int b) { hipLaunchKernelGGL((v3_dots<32, 8>), dim3(g3216), dim3(512), 0, 0, X, ld, N, RG, B, b * B, eps, slab1); });
  {
    double *slab2, *eps_out; int *cnt1, *pidx;
    CHK(hipMalloc(&slab2, sizeof(double) * 64 * B));
    CHK(hipMalloc(&eps_out, sizeof(double) * ld));
    CHK(hipMalloc(&cnt1, sizeof(int) * 4096));
    CHK(hipMalloc(&pidx, sizeof(int) * 16));
    CHK(hipMemset(cnt1, 0, sizeof(int) * 4096));
    CHK(hipMemset(pidx, 0, sizeof(int) * 16));
    const char *names[] = {"v4 plain", "v4 sc1", "v4 sc1+lvl2", "v4 sc1+lvl2+pend", "v4 all (+eps_out)", "v4 pend only", "v4 lvl2 plain-st"};
    const int optv[] = {0, 1, 3, 7, 15, 4, 2};
    for (int k = 0; k < 7; ++k) {
      const int o = optv[k];
      run(names[k], [&](int b) { hipLaunchKernelGGL(v4_full<32>, dim3(g32), dim3(256), 0, 0, X, ld, N, RG, B, b * B, eps, eps_out, slab1, slab2, cnt1, pidx, o); });
    }
  }
  // big single launch: all nblk blocks in one grid (upper bound, no per-launch ramp)
  {
    const unsigned gall = (unsigned)((RG + 7) / 8 * 8 * (P / 128));
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(v0_read<32>, dim3(gall), dim3(256), 0, 0, X, ld, N, RG, (int)P, 0, out);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(v0_read<32>, dim3(gall), dim3(256), 0, 0, X, ld, N, RG, (int)P, 0, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %8.2f us total    %7.1f GB/s\n", "v0_read<32> one grid", ms * 1e3, 4.0 * N * P / (ms * 1e-3) / 1e9);
  }
  // lag-1 pipeline rehearsal: stream(b) waits for solve(b-2), solve(b) waits for stream(b)
  {
    const int solve_us = argc > 4 ? atoi(argv[4]) : 15;
    const size_t lds = 150 * 1024;
    CHK(hipFuncSetAttribute((const void *)fake_solve, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int ncu = 0;
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    for (int masked = 0; masked < 2; ++masked) {
      hipStream_t sa, sb;
      if (masked) {
        std::vector<uint32_t> ma((ncu + 31) / 32, 0), mb((ncu + 31) / 32, 0);
        for (int c = 0; c < ncu; ++c) { if (c == 0) mb[0] |= 1u; else ma[c / 32] |= 1u << (c % 32); }
        CHK(hipExtStreamCreateWithCUMask(&sa, (uint32_t)ma.size(), ma.data()));
        CHK(hipExtStreamCreateWithCUMask(&sb, (uint32_t)mb.size(), mb.data()));
      } else {
        CHK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
        CHK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
      }
      std::vector<hipEvent_t> evs(nblk), evv(nblk);
      for (int b = 0; b < nblk; ++b) {
        CHK(hipEventCreateWithFlags(&evs[b], hipEventDisableTiming));
        CHK(hipEventCreateWithFlags(&evv[b], hipEventDisableTiming));
      }
      for (int rep = 0; rep < 2; ++rep) {
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0, sa));
        for (int b = 0; b < nblk; ++b) {
          if (b >= 2) CHK(hipStreamWaitEvent(sa, evv[b - 2], 0));
          hipLaunchKernelGGL(v1_dots<32>, dim3(g32), dim3(256), 0, sa, X, ld, N, RG, B, b * B, eps, slab1);
          CHK(hipEventRecord(evs[b], sa));
          CHK(hipStreamWaitEvent(sb, evs[b], 0));
          hipLaunchKernelGGL(fake_solve, dim3(1), dim3(256), lds, sb, solve_us, out);
          CHK(hipEventRecord(evv[b], sb));
        }
        CHK(hipStreamWaitEvent(sa, evv[nblk - 1], 0));
        CHK(hipEventRecord(e1, sa));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        if (rep) printf("lag-1 pipeline masked=%d solve=%dus: %8.2f us/block\n", masked, solve_us, ms * 1e3 / nblk);
      }
      // serial reference: stream then solve on one stream
      for (int rep = 0; rep < 2; ++rep) {
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0, sa));
        for (int b = 0; b < nblk; ++b) {
          hipLaunchKernelGGL(v1_dots<32>, dim3(g32), dim3(256), 0, sa, X, ld, N, RG, B, b * B, eps, slab1);
          hipLaunchKernelGGL(fake_solve, dim3(1), dim3(256), lds, sa, solve_us, out);
        }
        CHK(hipEventRecord(e1, sa));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        if (rep) printf("serial         masked=%d solve=%dus: %8.2f us/block\n", masked, solve_us, ms * 1e3 / nblk);
      }
    }
  }
  return 0;
}
