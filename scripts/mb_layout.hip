// Microbenchmark: the fused sweep's streaming loop (8 waves, 16 columns x 256 rows per item, one
// item prefetched, npass row passes per workgroup) over nb blocks of B = 512 columns, with the
// X layout as a parameter:
//   layout 0: column-major, ld = roundup(N, 256)          (1-KiB pieces 400 KB apart)
//   layout 1: tiled [block][row tile][column][256 rows]    (a workgroup's block = rpw/256
//             contiguous 512-KiB tiles)
// Reports the achieved read rate of the whole grid (no hand-over, no solver).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/mb_layout.hip -o scripts/mb_layout.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int SROWS = 256, NT = 512, NW = 8, CW = 16, B = 512;

__global__ __launch_bounds__(NT, 1) void stream(const float *X, int64_t ld, int N, int RG, int nb, int rpw, int npass,
                                                int layout, double *out) {
  __shared__ double eps[8 * SROWS];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = blockIdx.x;
  const int64_t r0 = (int64_t)g * rpw, r1 = r0 + rpw < N ? r0 + rpw : N;
  for (int i = t; i < npass * SROWS; i += NT) eps[i] = 1.0 / (1 + i);
  __syncthreads();
  const int CPW = B / NW, NCH = CPW / CW, items = NCH * npass, total = items * nb;
  auto issue = [&](int it, float4 (&x)[CW]) {
    const int s = it / items, rem = it - s * items;
    const int c = rem / npass, p = rem - c * npass;
    const int64_t row = r0 + p * SROWS + 4 * lane;
    const int64_t off = row < r1 ? row : r0;
    const int cb = w * CPW + c * CW;  // column within the block
    if (layout == 0) {
      const float *base = X + off + (int64_t)(s * B + cb) * ld;
#pragma unroll
      for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(base + (int64_t)j * ld);
    } else {
      const int64_t tile = off / SROWS, rin = off % SROWS;
      const float *base = X + ((((int64_t)s * RG + tile) * B + cb) * SROWS) + rin;
#pragma unroll
      for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(base + (int64_t)j * SROWS);
    }
  };
  float4 xq[2][CW];
  double v[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) v[j] = 0.0;
  issue(0, xq[0]);
  double acc = 0.0;
  for (int it = 0; it < total; ++it) {
    const int rem = it % items, p = rem % npass;
    if (it + 1 < total) issue(it + 1, xq[1]);
    const double *e = eps + p * SROWS + 4 * lane;
    const double e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
#pragma unroll
    for (int j = 0; j < CW; ++j)
      v[j] += (((double)xq[0][j].x * e0 + (double)xq[0][j].y * e1) + (double)xq[0][j].z * e2) + (double)xq[0][j].w * e3;
#pragma unroll
    for (int j = 0; j < CW; ++j) xq[0][j] = xq[1][j];
    if (p == npass - 1) {
#pragma unroll
      for (int j = 0; j < CW; ++j) { acc += v[j]; v[j] = 0.0; }
    }
  }
  if (acc == 1234.5) out[g] = acc;
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 100000;
  const int nb = argc > 2 ? atoi(argv[2]) : 60;
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int RG = (N + SROWS - 1) / SROWS;
  const int64_t ld = (int64_t)RG * SROWS;
  const size_t elems = (size_t)ld * B * nb;
  float *X;
  double *out;
  CHK(hipMalloc(&X, elems * sizeof(float)));
  CHK(hipMalloc(&out, 4096 * sizeof(double)));
  CHK(hipMemset(X, 0, elems * sizeof(float)));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int rpws[] = {256, 420, 448, 512, 768, 1024};
  for (int layout = 0; layout < 2; ++layout)
    for (int rpw : rpws) {
      if (layout == 1 && rpw % SROWS) continue;  // tiled layout: whole tiles per workgroup
      const int nsg = (N + rpw - 1) / rpw;
      if (nsg > cus) continue;
      const int npass = (rpw + SROWS - 1) / SROWS;
      for (int rep = 0; rep < 2; ++rep) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(stream, dim3(nsg), dim3(NT), 0, 0, X, ld, N, RG, nb, rpw, npass, layout, out);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        const double bytes = 4.0 * N * B * nb;
        if (rep) printf("layout %d rpw %4d wgs %3d: %.3f ms  %.2f TB/s  (%.1f us per block)\n", layout, rpw, nsg, ms,
                        bytes / ms / 1e9, 1000.0 * ms / nb);
      }
    }
  return 0;
}
