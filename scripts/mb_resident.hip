// Residency census: how many 256-thread workgroups (given VGPR / LDS use) run concurrently on a
// CU-masked queue.  Each workgroup counts itself in, then waits (bounded) for the full grid.
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_resident.hip -o scripts/mb_resident.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256, 2) void census(int *cnt, int *maxseen, int grid, int heavy) {
  extern __shared__ double lds[];
  __shared__ int s;
  double acc[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) acc[i] = threadIdx.x * 0.5 + i;  // hold VGPRs like the streamer
  if (threadIdx.x == 0) {
    int c = atomicAdd(cnt, 1) + 1;
    uint64_t t0 = wall_clock64();
    while (c < grid && wall_clock64() - t0 < 2000000) { __builtin_amdgcn_s_sleep(8); c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
    atomicMax(maxseen, c);
    s = c;
  }
  __syncthreads();
  double r = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) r += acc[i];
  lds[threadIdx.x] = r;
  if (heavy == 12345) maxseen[1] = (int)lds[5];
}

int main() {
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int per = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)census, 256, 16384));
  printf("CUs %d, occupancy API %d per CU\n", cus, per);
  int *cnt, *mx;
  CHK(hipMalloc(&cnt, 8)); CHK(hipMalloc(&mx, 8));
  for (int masked = 0; masked < 2; ++masked) {
    hipStream_t st;
    if (masked) {
      std::vector<uint32_t> m((cus + 31) / 32, 0);
      for (int c = 1; c < cus; ++c) m[c / 32] |= 1u << (c % 32);
      CHK(hipExtStreamCreateWithCUMask(&st, (uint32_t)m.size(), m.data()));
      std::vector<uint32_t> got(m.size());
      CHK(hipExtStreamGetCUMask(st, (uint32_t)got.size(), got.data()));
      int bits = 0; for (auto g : got) bits += __builtin_popcount(g);
      printf("masked stream: %d CUs in mask\n", bits);
    } else {
      CHK(hipStreamCreate(&st));
    }
    for (int grid : {128, 200, 255, 256, 300, 391, 450, 500, 510, 512, 600}) {
      CHK(hipMemset(cnt, 0, 8)); CHK(hipMemset(mx, 0, 8));
      hipLaunchKernelGGL(census, dim3(grid), dim3(256), 16384, st, cnt, mx, grid, 0);
      CHK(hipStreamSynchronize(st));
      int m; CHK(hipMemcpy(&m, mx, 4, hipMemcpyDeviceToHost));
      printf("masked=%d grid=%4d max co-resident=%d%s\n", masked, grid, m, m < grid ? "  <-- NOT all resident" : "");
    }
  }
  return 0;
}
