// How fast can a CU move L2-resident operand bytes into LDS (or registers) on gfx950? The conv
// kernel stages every operand piece (16 rows x 64 B) with one LDS-DMA wave-instruction; DESIGN.md
// 4a models its K loop as bound by that path. This measures the three candidate paths with no
// compute at all, 4 waves per block, 1 / 2 / 4 blocks per CU, a 2 MiB source (L2-resident):
//
//   dma      buffer_load_dwordx4 ... lds (1 KiB per wave-instruction), 8 in flight per wave
//   vgpr_ds  buffer_load_dwordx4 -> VGPRs -> ds_write_b128, 8 loads in flight per wave
//   vgpr     buffer_load_dwordx4 -> VGPRs only (xor-reduced), 8 in flight per wave
//
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I semilayer-wise-mixed-precision-quantization_amd/csrc \
//       tools/fill_bench.hip -o tools/bin/fill_bench
#include <hip/hip_runtime.h>

#include <cstdio>

#include "lds_dma.h"

using namespace smpq;

constexpr int kSrcBytes = 2 << 20;
constexpr int kPieces = 2048;  // per wave

__device__ __forceinline__ unsigned piece_off(int p, int wid) {
  return (unsigned)((((unsigned)wid * 977u + (unsigned)p * 7u) & ((kSrcBytes >> 10) - 1)) << 10);
}

// ROWB: bytes of one source row inside a piece (1024 = contiguous piece; 128 = 8 rows of one cache
// line each, 1 KiB apart; 64 = 16 half-line rows 256 B apart, the conv's BK = 64 pieces at cin 256)
template <int ROWB>
__device__ __forceinline__ unsigned lane_off(int lane) {
  if constexpr (ROWB == 1024) return 16 * lane;
  else return (unsigned)((lane / (ROWB / 16)) * (ROWB == 128 ? 1024 : 256) + 16 * (lane % (ROWB / 16)));
}

template <int ROWB>
__global__ __launch_bounds__(256) void k_dma(const int8_t* src, int* out) {
  extern __shared__ __attribute__((aligned(1024))) int8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wid = blockIdx.x * 4 + wave;
  const v4i rs = make_rsrc(src, kSrcBytes + 32768);
  const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lds) + wave * 8192;
  const unsigned lo = lane_off<ROWB>(lane);
  for (int p = 0; p < kPieces; ++p) {
    dma16(__builtin_amdgcn_readfirstlane(base + (p & 7) * 1024), rs, piece_off(p, wid) + lo, 0u);
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (lds[threadIdx.x * 16] == 123 && lds[threadIdx.x * 16 + 1] == 45) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_vgpr_ds(const int8_t* src, int* out) {
  extern __shared__ __attribute__((aligned(1024))) int8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wid = blockIdx.x * 4 + wave;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(src), 0, kSrcBytes, 0x00020000);
  v4u buf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) buf[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, piece_off(s, wid) + 16 * lane, 0, 0);
  int8_t* ring = lds + wave * 8192 + 16 * lane;
  for (int p = 0; p < kPieces; p += 8) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      *reinterpret_cast<v4u*>(ring + s * 1024) = buf[s];
      if (p + 8 + s < kPieces)
        buf[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, piece_off(p + 8 + s, wid) + 16 * lane, 0, 0);
    }
  }
  __syncthreads();
  if (lds[threadIdx.x * 16] == 123 && lds[threadIdx.x * 16 + 1] == 45) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_vgpr(const int8_t* src, int* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wid = blockIdx.x * 4 + wave;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(src), 0, kSrcBytes, 0x00020000);
  v4u buf[8], acc = v4u{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < 8; ++s) buf[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, piece_off(s, wid) + 16 * lane, 0, 0);
  for (int p = 0; p < kPieces; p += 8) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      acc ^= buf[s];
      if (p + 8 + s < kPieces)
        buf[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, piece_off(p + 8 + s, wid) + 16 * lane, 0, 0);
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x7654321u) out[0] = 1;
}

template <typename K>
static double run(K kern, int blocks, int lds, const int8_t* src, int* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, src, out);
  (void)hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, src, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)blocks * 4 * kPieces * 1024.0 * reps;
  return bytes / (ms * 1e-3) / 1e12;  // TB/s
}

int main() {
  int8_t* src;
  int* out;
  if (hipMalloc(&src, kSrcBytes + 32768) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  (void)hipMemset(src, 1, kSrcBytes + 32768);
  printf("{\"unit\": \"TB/s chip-wide (256 CUs), 2 MiB L2-resident source, 4 waves per block\"");
  for (int k : {1, 2, 4}) {
    const double d = run(k_dma<1024>, 256 * k, 32768, src, out);
    const double d128 = run(k_dma<128>, 256 * k, 32768, src, out);
    const double d64 = run(k_dma<64>, 256 * k, 32768, src, out);
    const double vd = run(k_vgpr_ds, 256 * k, 32768, src, out);
    const double v = run(k_vgpr, 256 * k, 0, src, out);
    printf(", \"blocks_per_cu_%d\": {\"lds_dma_contiguous_1k\": %.2f, \"lds_dma_8x128B_rows\": %.2f, "
           "\"lds_dma_16x64B_rows\": %.2f, \"vgpr_then_ds_write_b128\": %.2f, \"vgpr_only\": %.2f}", k, d, d128, d64,
           vd, v);
  }
  printf("}\n");
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  return 0;
}
