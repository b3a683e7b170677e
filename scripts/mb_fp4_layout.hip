// Probe: the operand lane map of v_mfma_scale_f32_16x16x128_f8f6f4 with fp4 (e2m1) operands and unit
// scales, checked with exact small-integer data against a CPU product (the assumed map: lane l holds row
// (or column) l & 15, K = 32 (l >> 4) .. + 31 as 16 bytes, element 2 q in the low nibble of byte q --
// the i8 16x16x64 byte layout read as nibble pairs).  Used by k_gram_fp4 (brr_kernels.hip).
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/mb_fp4 scripts/mb_fp4_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// fp4 e2m1 codes of 0, 1, 2, 4 (and 0.5, 1.5, 3, 6 for the check of the full code set)
static const float kval[8] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};

__global__ void k_probe(const uint8_t *A, const uint8_t *B, float *C) {
  // A: [16 rows][64 bytes] (128 nibbles of K), B: [16 columns][64 bytes]
  const int l = threadIdx.x;
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t *pa = reinterpret_cast<const uint32_t *>(A + (l & 15) * 64 + 16 * (l >> 4));
  const uint32_t *pb = reinterpret_cast<const uint32_t *>(B + (l & 15) * 64 + 16 * (l >> 4));
  for (int k = 0; k < 4; ++k) { a[k] = pa[k]; b[k] = pb[k]; }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
  uint8_t hA[16 * 64], hB[16 * 64];
  srand(7);
  for (int i = 0; i < 16 * 64; ++i) {
    hA[i] = (uint8_t)((rand() & 7) | ((rand() & 7) << 4));
    hB[i] = (uint8_t)((rand() & 7) | ((rand() & 7) << 4));
  }
  uint8_t *dA, *dB;
  float *dC, hC[256];
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dC, sizeof hC);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 128; ++k) {
        const int na = (hA[i * 64 + k / 2] >> (4 * (k & 1))) & 15, nb = (hB[j * 64 + k / 2] >> (4 * (k & 1))) & 15;
        s += (double)kval[na & 7] * kval[nb & 7];
      }
      if (s != hC[i * 16 + j]) {
        if (bad < 5) printf("mismatch (%d,%d): cpu %g gpu %g\n", i, j, s, hC[i * 16 + j]);
        ++bad;
      }
    }
  printf("fp4 16x16x128 layout: %s (%d of 256 mismatched)\n", bad ? "MISMATCH" : "OK", bad);
  return bad ? 1 : 0;
}
