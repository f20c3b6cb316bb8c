// Register-only throughput ceilings on gfx950 for the two ways to multiply a sub-byte weight slice
// (north_star: "4/6-bit slices use DP4A-style integer dot on unpacked nibbles"; SURVEY.md 7 step 5
// asks for the choice to be measured): VALU dot products vs the int8 MFMA the conv kernel uses.
// No memory traffic at all — each number is an UPPER bound for a conv built on that instruction.
//
//   sdot4        v_dot4_i32_i8: 4 int8 x int8 MACs per lane (activation limb x unpacked weight)
//   unpack+sdot4 8 packed 4-bit codes per dword -> two int8 dwords (v_perm / shifts), 2 sdot4
//   sdot8        v_dot8_i32_i4: 8 int4 x int4 MACs per lane (would need 4-bit ACTIVATIONS too)
//   mfma_i8      v_mfma_i32_16x16x64_i8, 4 independent accumulators per wave
//
// hipcc --offload-arch=gfx950 -O3 tools/dp4a_peak.hip -o tools/bin/dp4a_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_sdot4(int* out, int seed) {
  int acc[8], a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    acc[i] = 0;
    a[i] = seed * (threadIdx.x + 3 * i + 1);
    b[i] = seed ^ (blockIdx.x + 7 * i);
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_sdot4(a[i], b[i], acc[i], false);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] ^= it;
  }
  int s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  if (s == 0x7654321) out[0] = s;
}

__global__ __launch_bounds__(256) void k_unpack_sdot4(int* out, int seed) {
  int acc[8], a[16];
  unsigned w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    acc[i] = 0;
    w[i] = (unsigned)(seed ^ (blockIdx.x + 7 * i));
    a[2 * i] = seed * (threadIdx.x + 3 * i + 1);
    a[2 * i + 1] = seed * (threadIdx.x + 5 * i + 2);
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // 8 signed nibbles -> 8 int8 (sign-extended): low nibbles and high nibbles, 2 dwords
      const unsigned lo = w[i] & 0x0f0f0f0fu, hi = (w[i] >> 4) & 0x0f0f0f0fu;
      const unsigned slo = (lo ^ 0x08080808u) - 0x08080808u, shi = (hi ^ 0x08080808u) - 0x08080808u;
      acc[i] = __builtin_amdgcn_sdot4(a[2 * i], (int)slo, acc[i], false);
      acc[i] = __builtin_amdgcn_sdot4(a[2 * i + 1], (int)shi, acc[i], false);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] ^= it;
  }
  int s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  if (s == 0x7654321) out[0] = s;
}

__global__ __launch_bounds__(256) void k_sdot8(int* out, int seed) {
  int acc[8], a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    acc[i] = 0;
    a[i] = seed * (threadIdx.x + 3 * i + 1);
    b[i] = seed ^ (blockIdx.x + 7 * i);
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_sdot8(a[i], b[i], acc[i], false);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] ^= it;
  }
  int s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  if (s == 0x7654321) out[0] = s;
}

__global__ __launch_bounds__(256) void k_mfma(int* out, int seed) {
  v4i acc[4], a, b;
  for (int i = 0; i < 4; ++i) acc[i] = v4i{0, 0, 0, 0};
  a = v4i{seed, (int)threadIdx.x, seed ^ 5, 7};
  b = v4i{(int)blockIdx.x, seed, 3, seed * 3};
  for (int it = 0; it < kIters / 4; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
    a.x ^= it;
  }
  int s = 0;
  for (int i = 0; i < 4; ++i) s ^= acc[i].x ^ acc[i].w;
  if (s == 0x7654321) out[0] = s;
}

template <typename K>
static double run(K kern, double macs_per_thread_iter, int iters, int* out) {
  const int blocks = 256 * 8, threads = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 3);  // warm-up
  (void)hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 3 + r);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double macs = macs_per_thread_iter * iters * (double)blocks * threads * reps;
  return macs / (ms * 1e-3) / 1e12;  // T MAC/s
}

int main() {
  int* out;
  if (hipMalloc(&out, 4) != hipSuccess) return 1;
  const double sdot4 = run(k_sdot4, 8 * 4, kIters, out);
  const double unpack = run(k_unpack_sdot4, 8 * 8, kIters, out);
  const double sdot8 = run(k_sdot8, 8 * 8, kIters, out);
  // per wave per iteration: 4 MFMAs x 16x16x64 MACs, i.e. per thread 4 * 16384 / 64
  const double mfma = run(k_mfma, 4.0 * 16 * 16 * 64 / 64, kIters / 4, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"unit\": \"T int MAC/s (register-only, whole chip)\", \"v_dot4_i32_i8\": %.1f, "
         "\"nibble_unpack_plus_v_dot4\": %.1f, \"v_dot8_i32_i4\": %.1f, \"v_mfma_i32_16x16x64_i8\": %.1f}\n",
         sdot4, unpack, sdot8, mfma);
  (void)hipFree(out);
  return 0;
}
