// Fragment mapping of v_mfma_i32_32x32x32_i8 on gfx950: one wave computes D[32][32] = A[32][32] . B[32][32]^T
// (A rows = i, B rows = j, K = 32) with the hypothesised operand layout: lane l holds row l % 32 and
// K bytes 16 * (l / 32) .. + 16 of A (and of B), and D row 8 (r / 4) + 4 (l / 32) + r % 4, column
// l % 32 in accumulator register r. Prints whether the hypothesis holds, against a host reference.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma32_probe.hip -o tools/bin/mfma32_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x;
  const v4i a = *reinterpret_cast<const v4i*>(A + (l % 32) * 32 + 16 * (l / 32));
  const v4i b = *reinterpret_cast<const v4i*>(B + (l % 32) * 32 + 16 * (l / 32));
  v16i c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[(8 * (r / 4) + 4 * (l / 32) + r % 4) * 32 + l % 32] = c[r];
}

int main() {
  signed char hA[1024], hB[1024];
  int hD[1024];
  srand(7);
  for (int i = 0; i < 1024; ++i) hA[i] = (signed char)(rand() % 256 - 128), hB[i] = (signed char)(rand() % 256 - 128);
  signed char *dA, *dB;
  int* dD;
  if (hipMalloc(&dA, 1024) || hipMalloc(&dB, 1024) || hipMalloc(&dD, 4096)) return 1;
  (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  (void)hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      int s = 0;
      for (int kk = 0; kk < 32; ++kk) s += hA[i * 32 + kk] * hB[j * 32 + kk];
      bad += s != hD[i * 32 + j];
    }
  printf("{\"mfma_i32_32x32x32_i8_layout_ok\": %s, \"mismatches\": %d}\n", bad ? "false" : "true", bad);
  return 0;
}
