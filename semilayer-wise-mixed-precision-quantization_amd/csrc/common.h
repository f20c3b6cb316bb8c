// Shared helpers for libsmpq (gfx950 / CDNA4). Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/smpq.h"

namespace smpq {

// thread-local last-error message (abi.cpp)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

inline int check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    return fail(SMPQ_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  }
  return SMPQ_OK;
}

constexpr int kWave = 64;  // CDNA wavefront width

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// 16-B global store followed by two wait states (the gfx940-family count): on gfx950 a VMEM store of more than 8 bytes must
// not have its data VGPRs rewritten by the next instruction, and ROCm 7.2's hazard recognizer does
// not always keep them apart (conv_glds.hip store_limbs16 has the observed failure).
__device__ __forceinline__ void st16(void* p, v4i v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// atomic max on a non-negative float stored as its bit pattern (monotone for v >= 0)
__device__ __forceinline__ void atomic_max_nonneg(float* p, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}

}  // namespace smpq
