// Cross-XCD flag polling test: a producer workgroup (solve queue, CU 0) publishes epochs
// 1..E; `nwg` consumer workgroups (main queue, all other CUs) poll for each epoch, then ack.
// Variants of the consumer poll and producer store; counts consumer waits that time out.
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_poll.hip -o scripts/mb_poll.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

enum { POLL_SC1 = 0, POLL_SYS = 1, POLL_RMW = 2, POLL_SC1_INV = 3 };

__device__ __forceinline__ int poll_load(int *p, int mode) {
  if (mode == POLL_SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (mode == POLL_SYS) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (mode == POLL_RMW) return __hip_atomic_fetch_add(p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void producer(int *flag, int *ack, int nwg, int E, int *fail) {
  if (threadIdx.x != 0) return;
  for (int e = 1; e <= E; ++e) {
    // all consumers saw e-1
    uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(ack, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (e - 1) * nwg) {
      if (wall_clock64() - t0 > 20000000ull) { atomicAdd(fail + 1, 1); return; }  // 0.2 s
      __builtin_amdgcn_s_sleep(4);
    }
    __hip_atomic_store(flag, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(256, 2) void consumer(int *flag, int *ack, int E, int mode, int *fail, int *maxlat,
                                                   int prewarm) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    if (prewarm) (void)*(volatile int *)flag;  // plain read: leave the line in this XCD's L2
    for (int e = 1; e <= E; ++e) {
      uint64_t t0 = wall_clock64();
      int v;
      while ((v = poll_load(flag, mode)) < e) {
        if (wall_clock64() - t0 > 20000000ull) { atomicAdd(fail, 1); break; }
        __builtin_amdgcn_s_sleep(8);
      }
      atomicMax(maxlat, (int)((wall_clock64() - t0) / 100));  // microseconds
      __hip_atomic_fetch_add(ack, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_ok = 1;
  }
  __syncthreads();
}

int main(int argc, char **argv) {
  const int nwg = argc > 1 ? atoi(argv[1]) : 391;
  const int E = argc > 2 ? atoi(argv[2]) : 200;
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<uint32_t> ma((cus + 31) / 32, 0), mb((cus + 31) / 32, 0);
  for (int c = 0; c < cus; ++c) { if (c == 0) mb[0] |= 1u; else ma[c / 32] |= 1u << (c % 32); }
  hipStream_t sa, sb;
  CHK(hipExtStreamCreateWithCUMask(&sa, (uint32_t)ma.size(), ma.data()));
  CHK(hipExtStreamCreateWithCUMask(&sb, (uint32_t)mb.size(), mb.data()));
  int *buf;
  CHK(hipMalloc(&buf, 4096));
  int *flag = buf, *ack = buf + 32, *fail = buf + 64, *maxlat = buf + 96;
  const char *names[] = {"sc1 load (agent)", "sc0 sc1 load (system)", "atomic add 0", "acquire + sc1 load"};
  for (int prewarm = 0; prewarm < 2; ++prewarm)
    for (int mode = 0; mode < 4; ++mode) {
      CHK(hipMemset(buf, 0, 4096));
      CHK(hipDeviceSynchronize());
      hipLaunchKernelGGL(consumer, dim3(nwg), dim3(256), 0, sa, flag, ack, E, mode, fail, maxlat, prewarm);
      hipLaunchKernelGGL(producer, dim3(1), dim3(64), 0, sb, flag, ack, nwg, E, fail);
      CHK(hipDeviceSynchronize());
      int h[128];
      CHK(hipMemcpy(h, buf, sizeof h, hipMemcpyDeviceToHost));
      printf("prewarm=%d %-24s epochs %d: consumer timeouts %d, producer timeouts %d, max wait %d us\n", prewarm,
             names[mode], E, h[64], h[65], h[96]);
    }
  return 0;
}
