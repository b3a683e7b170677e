// Microbenchmark: the 2-bit streaming dot of k_sweep's streaming workgroups in isolation (no
// solver, no hand-over): 224 workgroups x 512 threads, 448 residual rows each in LDS, blocks of
// B = 512 columns in code tiles, one 16-byte code group (16 columns x 4 rows) per lane and item,
// P items in flight, a wave reduction per 16-column chunk.  Variants of the decode + f64 dot:
//   0  value tables as float4 in LDS, bit-select decode, f32 -> f64, mul + add (round-2 kernel)
//   1  value tables as 4 doubles in LDS, one indexed 8-byte LDS read per value, mul + add
//   2  as 1 with a fused multiply-add chain per value
//   3  codes read and summed as integers (the load / loop floor)
//   6, 7  as 2 and 1 with a static register ring and explicit bit-field address arithmetic
//   8, 9  as 6 with the LDS reads of 16 / 4 columns issued before their multiply-adds
//   4, 5  as 1 and 3 with the next block's value tables loaded one block ahead into registers
//         (no global-memory round trip between a block's last item and the boundary barrier)
// Results of 0 and 1 must be identical bit for bit (same products, same order).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/mb_decode.hip -o scripts/mb_decode.bin
#include "../bayesrrcpp_amd/csrc/brr_kernels.hip"

#include <cstdio>
#include <vector>

using namespace brr;

constexpr int NT = 512, NW = NT / 64, BB = 512, CPW = BB / NW, CWD = 16, NCH = CPW / CWD;

template <int V, int PP = 6, bool RED = true, bool UNR = false>
__global__ __launch_bounds__(NT, 1) void k_dec(const uint8_t *Xc, const float4 *lut, int nb, int64_t nq, int rpw,
                                               int npass, const double *eps, double *out) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char sm[];
  double *eps_l = reinterpret_cast<double *>(sm);
  float4 *lf = reinterpret_cast<float4 *>(eps_l + npass * SROWS);  // 3 blocks
  double *ld = reinterpret_cast<double *>(lf + 3 * BB);             // 3 blocks x 4 doubles
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = blockIdx.x;
  const int64_t r0 = (int64_t)g * rpw;
  for (int i = t; i < npass * SROWS; i += NT) eps_l[i] = i < rpw ? eps[r0 + i] : 0.0;
  auto put = [&](int s, int i, float4 l) {
    lf[(s % 3) * BB + i] = l;
    double *dd = ld + ((s % 3) * BB + i) * 4;
    dd[0] = l.x; dd[1] = l.y; dd[2] = l.z; dd[3] = l.w;
  };
  auto stage = [&](int s) {
    for (int i = t; i < BB; i += NT) put(s, i, lut[(int64_t)s * BB + i]);
  };
  constexpr bool PRE = V >= 4;
  static_assert(NT == BB, "one value table per thread");
  float4 lpre = make_float4(0.f, 0.f, 0.f, 0.f);
  stage(0);
  if (PRE && nb > 1) stage(1);
  if (PRE && nb > 2) lpre = lut[2 * BB + t];
  __syncthreads();
  const int items = NCH * npass, total = items * nb;
  auto issue = [&](int it) -> uint4 {
    const int s = it / items, rem = it - s * items;
    const int c = rem / npass, p = rem - c * npass;
    const int64_t o = p * SROWS + 4 * lane;
    const int64_t off = r0 + (o < rpw ? o : 0);  // lanes past the rows re-read the first quad (as k_sweep)
    const int64_t grp = (int64_t)s * (BB >> 4) + ((w * CPW + c * CWD) >> 4);
    return *reinterpret_cast<const uint4 *>(Xc + (grp * nq + (off >> 2)) * 16);
  };
  uint4 xq[PP + 1];
#pragma unroll
  for (int q = 0; q < PP; ++q) xq[q] = issue(q);
  double v[CWD];
#pragma unroll
  for (int j = 0; j < CWD; ++j) v[j] = 0.0;
  uint32_t iacc = 0;
  auto step = [&](int it, const uint4 &xc) __attribute__((always_inline)) {
    const int s = it / items, rem = it - s * items;
    const int c = rem / npass, p = rem - c * npass;
    if (rem == 0 && s >= 1) {
      if (PRE) {
        if (s + 1 < nb) put(s + 1, t, lpre);
        if (s + 2 < nb) lpre = lut[(int64_t)(s + 2) * BB + t];
      } else if (s + 1 < nb) {
        stage(s + 1);
      }
      __syncthreads();
    }
    if (!PRE && rem == 0 && s == 0 && nb > 1) { stage(1); __syncthreads(); }
    const double *e = eps_l + p * SROWS + 4 * lane;
    const double e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
    const int cb = (s % 3) * BB + w * CPW + c * CWD;
    if constexpr (V >= 8) {
      // LDS reads of CB columns (4 CB values) issued together, then their multiply-adds
      constexpr int CBT = V == 8 ? 16 : 4;
#pragma unroll
      for (int j0 = 0; j0 < CWD; j0 += CBT) {
        double xv[CBT][4];
#pragma unroll
        for (int jj = 0; jj < CBT; ++jj) {
          const int j = j0 + jj;
          const uint32_t word = j < 4 ? xc.x : (j < 8 ? xc.y : (j < 12 ? xc.z : xc.w));
          const uint32_t lb = (uint32_t)(uintptr_t)(ld + (int64_t)(cb + j) * 4);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            xv[jj][k] = *(const __attribute__((address_space(3))) double *)(uintptr_t)(
                __builtin_amdgcn_ubfe(word, 8 * (j & 3) + 2 * k, 2) * 8u + lb);
        }
#pragma unroll
        for (int jj = 0; jj < CBT; ++jj)
          v[j0 + jj] = __builtin_fma(xv[jj][3], e3, __builtin_fma(xv[jj][2], e2, __builtin_fma(xv[jj][1], e1, __builtin_fma(xv[jj][0], e0, v[j0 + jj]))));
      }
    } else
#pragma unroll
    for (int j = 0; j < CWD; ++j) {
      const uint32_t word = j < 4 ? xc.x : (j < 8 ? xc.y : (j < 12 ? xc.z : xc.w));
      const uint32_t b = (word >> (8 * (j & 3))) & 0xFFu;
      if constexpr (V == 0) {  // (V 4 / 5: as 1 / 3)
        const float4 xv = x_decode4(b, lf[cb + j]);
        v[j] += (((double)xv.x * e0 + (double)xv.y * e1) + (double)xv.z * e2) + (double)xv.w * e3;
      } else if constexpr (V >= 6) {
        // explicit bit-field extract + scaled add per value (2 integer ops), f64 tables in LDS
        const uint32_t lb = (uint32_t)(uintptr_t)(ld + (int64_t)(cb + j) * 4);
        const int sh = 8 * (j & 3);
        auto at = [&](int k) __attribute__((always_inline)) {
          const uint32_t a = __builtin_amdgcn_ubfe(word, sh + 2 * k, 2) * 8u + lb;
          return *(const __attribute__((address_space(3))) double *)(uintptr_t)a;
        };
        const double x0 = at(0), x1 = at(1), x2 = at(2), x3 = at(3);
        if constexpr (V == 7)
          v[j] += (((x0 * e0 + x1 * e1) + x2 * e2) + x3 * e3);
        else
          v[j] = __builtin_fma(x3, e3, __builtin_fma(x2, e2, __builtin_fma(x1, e1, __builtin_fma(x0, e0, v[j]))));
      } else if constexpr (V == 1 || V == 2 || V == 4) {
        const double *lt = ld + (int64_t)(cb + j) * 4;
        const double x0 = lt[b & 3], x1 = lt[(b >> 2) & 3], x2 = lt[(b >> 4) & 3], x3 = lt[b >> 6];
        if constexpr (V != 2)
          v[j] += (((x0 * e0 + x1 * e1) + x2 * e2) + x3 * e3);
        else
          v[j] = __builtin_fma(x3, e3, __builtin_fma(x2, e2, __builtin_fma(x1, e1, __builtin_fma(x0, e0, v[j]))));
      } else {
        iacc += b;
      }
    }
    if (p == npass - 1) {
      if constexpr (V == 3 || V == 5) v[0] += (double)iacc;
      const double r = RED ? wave_reduce16(v, lane) : v[0];
#pragma unroll
      for (int j = 0; j < CWD; ++j) v[j] = 0.0;
      const int col = w * CPW + c * CWD + reduce16_col(lane);
      if ((lane & 3) == 0) out[((int64_t)s * gridDim.x + g) * BB + col] = r;
    }
  };
  if constexpr (UNR) {
    // static register ring: item it's code group is xq[it % R] with R = PP + 1 and the loads
    // unconditional (clamped index), so the wait before a consume is vmcnt(PP), not vmcnt(0)
    constexpr int R = PP + 1;
    int it0 = 0;
    if constexpr (V >= 6) {
      // whole rounds of R items without a per-item condition, then the tail item by item
      for (; it0 + R <= total; it0 += R) {
#pragma unroll
        for (int u = 0; u < R; ++u) {
          xq[(u + PP) % R] = issue(min(it0 + u + PP, total - 1));
          step(it0 + u, xq[u]);
        }
      }
      for (int it = it0; it < total; ++it) {
        const uint4 xc = xq[0];
#pragma unroll
        for (int q = 0; q < R - 1; ++q) xq[q] = xq[q + 1];
        step(it, xc);
      }
      return;
    }
    for (; it0 < total; it0 += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int it = it0 + u;
        xq[(u + PP) % R] = issue(min(it + PP, total - 1));
        if (it < total) step(it, xq[u]);
      }
    }
  } else {
    for (int it = 0; it < total; ++it) {
      if (it + PP < total) xq[PP] = issue(it + PP);
      step(it, xq[0]);
#pragma unroll
      for (int q = 0; q < PP; ++q) xq[q] = xq[q + 1];
    }
  }
}

int main() {
  const int nsg = 224, rpw = 448, npass = 2, nb = 64;
  const int64_t N = (int64_t)nsg * rpw, nq = (N + 3) / 4;
  const int64_t P = (int64_t)nb * BB;
  std::vector<uint8_t> hc((size_t)(P / 16) * nq * 16);
  uint32_t x = 12345;
  for (auto &c : hc) { x = x * 1664525u + 1013904223u; c = (uint8_t)(x >> 24); }
  std::vector<float4> hl(P);
  for (int64_t i = 0; i < P; ++i) hl[i] = make_float4(-1.1f - 0.001f * (i % 97), 0.f, 0.3f + 0.002f * (i % 89), 1.7f + 0.003f * (i % 83));
  std::vector<double> he(N);
  for (int64_t i = 0; i < N; ++i) he[i] = std::sin(0.37 * i) * 0.8;
  uint8_t *dc; float4 *dl; double *de, *dout;
  const size_t nout = (size_t)nb * nsg * BB;
  if (hipMalloc(&dc, hc.size()) != hipSuccess) { std::printf("hipMalloc failed\n"); return 1; } hipMalloc(&dl, sizeof(float4) * P); hipMalloc(&de, 8 * N); hipMalloc(&dout, 8 * nout);
  hipMemcpy(dc, hc.data(), hc.size(), hipMemcpyHostToDevice);
  hipMemcpy(dl, hl.data(), sizeof(float4) * P, hipMemcpyHostToDevice);
  hipMemcpy(de, he.data(), 8 * N, hipMemcpyHostToDevice);
  const size_t lds = (size_t)npass * SROWS * 8 + 3 * BB * 16 + 3 * BB * 32;
  std::vector<double> ref(nout), got(nout);
  auto run = [&](auto kern, const char *name, int v) {
    hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(kern, dim3(nsg), dim3(NT), lds, 0, dc, dl, nb, nq, rpw, npass, de, dout);
    hipError_t er = hipDeviceSynchronize();
    if (er == hipSuccess) er = hipGetLastError();
    if (er != hipSuccess) { std::printf("%s: %s\n", name, hipGetErrorString(er)); return; }
    hipEventRecord(a);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(nsg), dim3(NT), lds, 0, dc, dl, nb, nq, rpw, npass, de, dout);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(v == 0 ? ref.data() : got.data(), dout, 8 * nout, hipMemcpyDeviceToHost);
    size_t ndiff = 0;
    double md = 0;
    if (v != 0)
      for (size_t i = 0; i < nout; ++i)
        if (got[i] != ref[i]) { ++ndiff; md = std::max(md, std::fabs(got[i] - ref[i]) / (std::fabs(ref[i]) + 1e-300)); }
    const double us = 1000.0 * ms / reps / nb;
    std::printf("%-34s %7.2f us per 512-column block (C2 sweep: %5.1f ms), %zu of %zu partials differ (max rel %.1e)\n", name,
                us, us * 977 / 1000.0, ndiff, nout, md);
  };
  run(k_dec<0>, "0 float4 LUT, bit-select, cvt", 0);
  run(k_dec<1>, "1 f64 LUT, indexed LDS read", 1);
  run(k_dec<2>, "2 f64 LUT, fma chain", 2);
  run(k_dec<3>, "3 integer sum (load floor)", 3);
  run(k_dec<4>, "4 = 1, tables one block ahead", 4);
  run(k_dec<5>, "5 = 3, tables one block ahead", 5);
  run(k_dec<3, 12>, "3 with 12 items in flight", 3);
  run(k_dec<3, 6, false>, "3 without the wave reduction", 3);
  run(k_dec<1, 12>, "1 with 12 items in flight", 1);
  run(k_dec<1, 3>, "1 with 3 items in flight", 1);
  run(k_dec<3, 6, true, true>, "3, static ring", 3);
  run(k_dec<1, 6, true, true>, "1, static ring", 1);
  run(k_dec<0, 6, true, true>, "0, static ring", 0);
  run(k_dec<2, 6, true, true>, "2, static ring", 2);
  run(k_dec<1, 3, true, true>, "1, static ring, 3 in flight", 1);
  run(k_dec<1, 11, true, true>, "1, static ring, 11 in flight", 1);
  run(k_dec<7, 6, true, true>, "7 = 1, static ring, bfe, no tail cond", 7);
  run(k_dec<6, 6, true, true>, "6 = 2, static ring, bfe, no tail cond", 6);
  run(k_dec<6, 3, true, true>, "6 with 3 in flight", 6);
  run(k_dec<6, 9, true, true>, "6 with 9 in flight", 6);
  run(k_dec<8, 6, true, true>, "8 = 6, 64 LDS reads batched", 8);
  run(k_dec<9, 6, true, true>, "9 = 6, 16 LDS reads batched", 9);
  return 0;
}
