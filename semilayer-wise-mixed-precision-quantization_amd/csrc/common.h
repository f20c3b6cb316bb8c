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

// atomic max on a non-negative float stored as its bit pattern (monotone for v >= 0)
__device__ __forceinline__ void atomic_max_nonneg(float* p, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}

}  // namespace smpq
