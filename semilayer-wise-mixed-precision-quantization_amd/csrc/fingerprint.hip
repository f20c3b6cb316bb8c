// Content fingerprints of the tensors a cached forward depends on (conv weights, quantization
// metadata, BatchNorm buffers), so that a change the host cannot see is still caught.
//
// The reference and its drivers rewrite weights in place (functions.py:22 writes
// `tensor[i][:][:][:] = ...` into conv.weight.data; resnet50_main.py:191 assigns `.data`); writes
// through `.data` do not bump a Parameter's version counter, so the engine's host-side key
// (data_ptr, _version) misses them. The engine fingerprints those tensors on the device after
// each forward (inside the captured graph) and compares against the fingerprint taken when its
// caches were built; a mismatch is reported with the overflow flag it already reads once per
// forward, and the result is recomputed from freshly packed weights.
//
// Fingerprint of a tensor of N 32-bit words w_i: sum_i H(w_i, i) mod 2^64 with the 64-bit word hash
// H(w, i) = fmix32(w ^ i * 0x9E3779B9) | fmix32(w ^ (i * 0x85EBCA6B + 0xC2B2AE35)) << 32 (fmix32 =
// the MurmurHash3 finalizer, a bijection on 32-bit values). For a fixed i, H is injective in w, so
// changing any word changes its term by a pseudo-random non-zero amount; several changed words
// cancel with probability ~2^-64 whatever their structure. (A plain odd-multiplier sum
// sum (w_i (2i + 1) mod 2^32) cannot see through floats with many trailing zero bits: scaling a
// BatchNorm variance of 1.0 by 4 left it unchanged.) The sum is order-independent (exact integer
// atomics), hence deterministic. Work is split into chunks of kChunkWords words; chunk c belongs to
// tensor chunk_tensor[c] and starts at word chunk_word[c]. HBM-bound: one read of every byte
// (R50: ~100 MB of fp32 weights, ~20 us; 6 quarter-rate multiplies per word stay under it).
#include "common.h"

namespace smpq {

constexpr int kFpThreads = 256;

__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__host__ __device__ __forceinline__ unsigned long long word_hash(uint32_t w, uint32_t i) {
  const uint32_t lo = fmix32(w ^ (i * 0x9E3779B9u));
  const uint32_t hi = fmix32(w ^ (i * 0x85EBCA6Bu + 0xC2B2AE35u));
  return (unsigned long long)lo | ((unsigned long long)hi << 32);
}
constexpr long long kChunkWords = 16384;  // 64 KiB per block

// A tensor of nbytes bytes is hashed as ceil(nbytes / 4) words, the last one zero-padded (its
// missing bytes masked off; tensors start 4-B aligned, so the load stays inside the allocation).
__host__ __device__ __forceinline__ uint32_t tail_mask(long long nbytes) {
  const int r = (int)(nbytes & 3);
  return r == 0 ? 0xffffffffu : (0xffffffffu >> (8 * (4 - r)));
}

__global__ __launch_bounds__(kFpThreads) void fingerprint_kernel(const uint32_t* const* __restrict__ ptrs,
                                                                   const long long* __restrict__ nbytes,
                                                                   const int* __restrict__ chunk_tensor,
                                                                   const long long* __restrict__ chunk_word,
                                                                   unsigned long long* __restrict__ out) {
  __shared__ unsigned long long part[kFpThreads / kWave];
  const int c = blockIdx.x;
  const int t = chunk_tensor[c];
  const long long w0 = chunk_word[c];
  const long long nb = nbytes[t];
  const long long n = (nb + 3) >> 2;
  const uint32_t last_mask = tail_mask(nb);
  const long long w1 = w0 + kChunkWords < n ? w0 + kChunkWords : n;
  const uint32_t* p = ptrs[t];
  unsigned long long acc = 0;
  // 16-B loads where the chunk is whole quads (tensors start 16-B aligned: caching-allocator blocks)
  // and does not hold a partial last word
  const bool vec = ((reinterpret_cast<unsigned long long>(p) & 15) == 0) && ((w1 - w0) & 3) == 0 &&
                   (w1 < n || last_mask == 0xffffffffu);
  if (vec) {
    const uint4* q = reinterpret_cast<const uint4*>(p + w0);
    const int nq = (int)((w1 - w0) >> 2);
    for (int j = threadIdx.x; j < nq; j += kFpThreads) {
      const uint4 v = q[j];
      const uint32_t i = (uint32_t)w0 + 4u * (uint32_t)j;  // word index of v.x (tensors < 2^32 words)
      acc += word_hash(v.x, i) + word_hash(v.y, i + 1u) + word_hash(v.z, i + 2u) + word_hash(v.w, i + 3u);
    }
  } else {
    for (long long i = w0 + threadIdx.x; i < w1; i += kFpThreads)
      acc += word_hash(i == n - 1 ? (p[i] & last_mask) : p[i], (uint32_t)i);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, kWave);
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane == 0) part[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
#pragma unroll
    for (int i = 0; i < kFpThreads / kWave; ++i) s += part[i];
    atomicAdd(out + t, s);
  }
}

__global__ void fingerprint_zero_kernel(unsigned long long* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = 0ull;
}

__global__ void fingerprint_compare_kernel(const unsigned long long* __restrict__ a,
                                           const unsigned long long* __restrict__ b, int n,
                                           int32_t* __restrict__ flag) {
  bool diff = false;
  for (int i = threadIdx.x; i < n; i += blockDim.x) diff |= a[i] != b[i];
  if (__any(diff) && (threadIdx.x % kWave) == 0) atomicOr(flag, 1);
}

}  // namespace smpq

using namespace smpq;

extern "C" long long smpq_fingerprint_chunk_words(void) { return kChunkWords; }

extern "C" int smpq_fingerprint(const void* const* ptrs, const int64_t* nbytes, int ntensors,
                                const int32_t* chunk_tensor, const int64_t* chunk_word, int nchunks,
                                uint64_t* out, smpq_stream_t stream) {
  if (!ptrs || !nbytes || !chunk_tensor || !chunk_word || !out || ntensors <= 0 || nchunks <= 0)
    return fail(SMPQ_E_INVALID, "smpq_fingerprint: bad arguments");
  hipLaunchKernelGGL(fingerprint_zero_kernel, dim3((ntensors + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<unsigned long long*>(out), ntensors);
  hipLaunchKernelGGL(fingerprint_kernel, dim3(nchunks), dim3(kFpThreads), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint32_t* const*>(ptrs), reinterpret_cast<const long long*>(nbytes),
                     chunk_tensor, reinterpret_cast<const long long*>(chunk_word),
                     reinterpret_cast<unsigned long long*>(out));
  return check_hip(hipGetLastError(), "fingerprint_kernel launch");
}

extern "C" int smpq_fingerprint_compare(const uint64_t* a, const uint64_t* b, int n, int32_t* flag,
                                        smpq_stream_t stream) {
  if (!a || !b || !flag || n <= 0) return fail(SMPQ_E_INVALID, "smpq_fingerprint_compare: bad arguments");
  hipLaunchKernelGGL(fingerprint_compare_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const unsigned long long*>(a), reinterpret_cast<const unsigned long long*>(b),
                     n, flag);
  return check_hip(hipGetLastError(), "fingerprint_compare_kernel launch");
}

// Host twin (tests): the same sum over one tensor's nbytes bytes (last word zero-padded).
extern "C" uint64_t smpq_fingerprint_host(const void* p, int64_t nbytes) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  const long long n = (nbytes + 3) >> 2;
  unsigned long long acc = 0;
  for (long long i = 0; i < n; ++i) {
    uint32_t w = 0;
    for (int k = 0; k < 4 && 4 * i + k < nbytes; ++k) w |= (uint32_t)b[4 * i + k] << (8 * k);
    acc += word_hash(w, (uint32_t)i);
  }
  return acc;
}
