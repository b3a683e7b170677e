// Microbenchmark: what the fused sweep's per-block synchronisation costs the streaming loop.
// The mb_layout loop (8 waves, CW columns x 256 rows per item, P items prefetched, npass row
// passes per workgroup, B = 512 column blocks, column-major X) plus, per block:
//   bar    the block-end workgroup barrier
//   apply  a change-list apply at every block boundary: barrier, each wave loads NA columns of
//          its 64-row slice (two batches of 16 scattered 4-B loads), updates the LDS residual,
//          barrier (the shape of apply_pending with NA changes)
// Reports the achieved read rate of X (no hand-over, no solver).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/mb_sync.hip -o scripts/mb_sync.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <utility>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int SROWS = 256, NT = 512, NW = 8, B = 512;

template <int CW, int P, bool BAR, int NA, bool IND = false>
__global__ __launch_bounds__(NT, 1) void stream(const float *X, int64_t ld, int N, int nb, int rpw, int npass,
                                                double *out, const int *member) {
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
    const int cb = w * CPW + c * CW;
    if (IND) {  // column indices from a member array (scalar loads), as k_sweep
      const int *mem = member + (int64_t)s * B + cb;
#pragma unroll
      for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(X + off + (int64_t)mem[j] * ld);
    } else {
      const float *base = X + off + (int64_t)(s * B + cb) * ld;
#pragma unroll
      for (int j = 0; j < CW; ++j) x[j] = *reinterpret_cast<const float4 *>(base + (int64_t)j * ld);
    }
  };
  float4 xq[P + 1][CW];
  double v[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) v[j] = 0.0;
#pragma unroll
  for (int q = 0; q < P; ++q) issue(q, xq[q]);
  double acc = 0.0;
  for (int it = 0; it < total; ++it) {
    const int s = it / items, rem = it - s * items, p = rem % npass;
    if (NA > 0 && rem == 0 && s >= 2) {
      __syncthreads();
      // apply: wave w updates the 64-row slices w, w + 8, ... with NA columns of block s-2
      for (int sl = w; sl < npass * 4; sl += NW) {
        const int off = sl * 64 + lane;
        const int64_t rr = r0 + off < r1 ? r0 + off : r0;
        double e = eps[off];
        for (int p0 = 0; p0 < NA; p0 += 16) {
          float xa[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) xa[q] = X[(int64_t)((s - 2) * B + 31 * (p0 + q) % B) * ld + rr];
#pragma unroll
          for (int q = 0; q < 16; ++q) e = (e + (double)xa[q] * 1e-3) - (double)xa[q] * 2e-3;
        }
        eps[off] = e;
      }
      __syncthreads();
    }
    if (it + P < total) issue(it + P, xq[P]);
    const double *e = eps + p * SROWS + 4 * lane;
    const double e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
#pragma unroll
    for (int j = 0; j < CW; ++j)
      v[j] += (((double)xq[0][j].x * e0 + (double)xq[0][j].y * e1) + (double)xq[0][j].z * e2) + (double)xq[0][j].w * e3;
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
      for (int j = 0; j < CW; ++j) xq[q][j] = xq[q + 1][j];
    if (p == npass - 1) {
#pragma unroll
      for (int j = 0; j < CW; ++j) { acc += v[j]; v[j] = 0.0; }
    }
    if (BAR && rem == items - 1) __syncthreads();
  }
  if (acc == 1234.5) out[g] = acc;
}

template <int CW, int P, bool BAR, int NA, bool IND = false>
void run(const char *name, const float *X, int64_t ld, int N, int nb, int rpw, double *out, const int *member = nullptr) {
  const int nsg = (N + rpw - 1) / rpw, npass = (rpw + SROWS - 1) / SROWS;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((stream<CW, P, BAR, NA, IND>), dim3(nsg), dim3(NT), 0, 0, X, ld, N, nb, rpw, npass, out, member);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep && ms < best) best = ms;
  }
  const double bytes = 4.0 * N * B * nb;
  printf("%-28s rpw %4d wgs %3d: %.3f ms  %.2f TB/s  (%.1f us per block)\n", name, rpw, nsg, best, bytes / best / 1e9,
         1000.0 * best / nb);
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 100000;
  const int nb = argc > 2 ? atoi(argv[2]) : 200;
  const int RG = (N + SROWS - 1) / SROWS;
  const int64_t ld = (int64_t)RG * SROWS;
  const size_t elems = (size_t)ld * B * nb;
  float *X;
  double *out;
  CHK(hipMalloc(&X, elems * sizeof(float)));
  CHK(hipMalloc(&out, 4096 * sizeof(double)));
  CHK(hipMemset(X, 0, elems * sizeof(float)));
  // member: a within-block permutation of every block's columns (as the BLOCKED visit order)
  int *member;
  {
    std::vector<int> m((size_t)nb * B);
    uint32_t r = 12345;
    for (int b = 0; b < nb; ++b) {
      for (int i = 0; i < B; ++i) m[(size_t)b * B + i] = b * B + i;
      for (int i = B - 1; i > 0; --i) {
        r = r * 1664525u + 1013904223u;
        const int k = (int)((r >> 8) % (uint32_t)(i + 1));
        std::swap(m[(size_t)b * B + i], m[(size_t)b * B + k]);
      }
    }
    CHK(hipMalloc(&member, m.size() * sizeof(int)));
    CHK(hipMemcpy(member, m.data(), m.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  for (int rpw : {448, 512}) {
    run<16, 1, false, 0, true>("cw16 p1 plain member", X, ld, N, nb, rpw, out, member);
    run<16, 1, true, 32, true>("cw16 p1 bar apply32 member", X, ld, N, nb, rpw, out, member);
    run<16, 1, false, 0>("cw16 p1 plain", X, ld, N, nb, rpw, out);
    run<16, 1, true, 0>("cw16 p1 bar", X, ld, N, nb, rpw, out);
    run<16, 1, true, 16>("cw16 p1 bar apply16", X, ld, N, nb, rpw, out);
    run<16, 1, true, 32>("cw16 p1 bar apply32", X, ld, N, nb, rpw, out);
    run<8, 3, false, 0>("cw8 p3 plain", X, ld, N, nb, rpw, out);
    run<8, 3, true, 32>("cw8 p3 bar apply32", X, ld, N, nb, rpw, out);
    run<8, 2, true, 32>("cw8 p2 bar apply32", X, ld, N, nb, rpw, out);
    run<4, 7, true, 32>("cw4 p7 bar apply32", X, ld, N, nb, rpw, out);
  }
  return 0;
}
