// Evaluation reductions that follow every quantized forward of the search:
//
//   functions.evaluate_acc_loss_softmax (functions.py:84-129): per batch `output.max(1)`, the
//   batch-mean CrossEntropyLoss and `Softmax(dim=1)` (:113-117), then top-1 accuracy and the mean
//   of the batch losses (:121-128);
//   functions.KLdiv (functions.py:131-149): per image sum_c p_ref * log(p_ref / p), averaged over
//   images — a Python loop over 50k rows in the reference.
//
// One wavefront per row (64 lanes stride the classes: 256-B coalesced loads), the row's
// max / sum-exp / argmax by cross-lane reduction, per-row results into a workspace, then one
// single-block pass that sums the rows in a FIXED order (double) into the caller's accumulators:
// deterministic, no float atomics, no host sync. Values follow torch's fp32 formulas
// (softmax = exp(x - max) / sum, CE = log(sum) + max - x_label, KL term = p_ref * log(p_ref / p)).
#include "common.h"

namespace smpq {

namespace {

constexpr int kRowsPerBlock = 4;  // 256 threads, one row per wave

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// row max and its FIRST index (ties -> lowest class index)
__device__ __forceinline__ void wave_argmax(float& v, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, kWave);
    const int oi = __shfl_xor(idx, o, kWave);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
}

__global__ __launch_bounds__(64 * kRowsPerBlock) void softmax_xent_kernel(const float* __restrict__ logits,
                                                                          const int64_t* __restrict__ labels,
                                                                          int rows, int cols, float* __restrict__ probs,
                                                                          float* __restrict__ row_ws) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole waves exit together
  const float* x = logits + (long long)row * cols;
  float m = -INFINITY;
  int mi = 0x7fffffff;
  for (int c = lane; c < cols; c += 64) {
    const float v = x[c];
    if (v > m || (v == m && c < mi)) {  // NaN never wins, as in a strict '>' scan
      m = v;
      mi = c;
    }
  }
  wave_argmax(m, mi);
  float s = 0.f;
  for (int c = lane; c < cols; c += 64) s += expf(x[c] - m);
  s = wave_sum(s);
  if (probs) {
    float* p = probs + (long long)row * cols;
    for (int c = lane; c < cols; c += 64) p[c] = __fdiv_rn(expf(x[c] - m), s);
  }
  if (lane == 0) {
    const long long y = labels[row];
    const bool ok = y >= 0 && y < cols;
    // -log_softmax(x)[y] = log(sum) + max - x[y]; an out-of-range label gives NaN (torch raises)
    row_ws[row] = ok ? (logf(s) + m) - x[y] : __int_as_float(0x7fc00000);
    row_ws[rows + row] = (ok && mi == (int)y) ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(64 * kRowsPerBlock) void kl_rows_kernel(const float* __restrict__ p_ref,
                                                                     const float* __restrict__ p, int rows, int cols,
                                                                     float* __restrict__ row_ws) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* a = p_ref + (long long)row * cols;
  const float* b = p + (long long)row * cols;
  float s = 0.f;
  for (int c = lane; c < cols; c += 64) {
    const float n = a[c];
    s += n * logf(__fdiv_rn(n, b[c]));  // n_out * (n_out / out).log() (functions.py:145)
  }
  s = wave_sum(s);
  if (lane == 0) row_ws[row] = s;
}

// stats[k] += w_k * (sum over rows r of ws[k * rows + r]) for k < nsums, in a fixed order (double);
// then stats[nsums] += rows and, with `batches`, stats[nsums + 1] += 1.
__global__ __launch_bounds__(256) void sum_rows_kernel(const float* __restrict__ ws, int rows, int nsums, double w0,
                                                       double w1, double* __restrict__ stats, int batches) {
  __shared__ double part[256];
  for (int k = 0; k < nsums; ++k) {
    double acc = 0.0;
    for (int r = threadIdx.x; r < rows; r += 256) acc += (double)ws[(long long)k * rows + r];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) stats[k] += part[0] * (k == 0 ? w0 : w1);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[nsums] += (double)rows;
    if (batches) stats[nsums + 1] += 1.0;
  }
}

}  // namespace
}  // namespace smpq

using namespace smpq;

extern "C" int smpq_softmax_xent(const float* logits, const int64_t* labels, int rows, int cols, float* probs,
                                 double* stats, float* row_ws, smpq_stream_t stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  if (rows < 0 || cols <= 0 || (rows > 0 && (!logits || !labels || !stats || !row_ws)))
    return fail(SMPQ_E_INVALID, "smpq_softmax_xent: bad arguments");
  if (rows == 0) return SMPQ_OK;
  hipLaunchKernelGGL(softmax_xent_kernel, dim3((rows + kRowsPerBlock - 1) / kRowsPerBlock), dim3(64 * kRowsPerBlock),
                     0, stream, logits, labels, rows, cols, probs, row_ws);
  int rc = check_hip(hipGetLastError(), "softmax_xent_kernel launch");
  if (rc) return rc;
  // [0] += batch-mean CE (criterion(output, y), functions.py:116), [1] += correct, [2] += rows, [3] += 1
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, stream, row_ws, rows, 2, 1.0 / rows, 1.0, stats, 1);
  return check_hip(hipGetLastError(), "sum_rows_kernel launch");
}

extern "C" int smpq_kl_rows(const float* p_ref, const float* p, int rows, int cols, double* stats, float* row_ws,
                            smpq_stream_t stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  if (rows < 0 || cols <= 0 || (rows > 0 && (!p_ref || !p || !stats || !row_ws)))
    return fail(SMPQ_E_INVALID, "smpq_kl_rows: bad arguments");
  if (rows == 0) return SMPQ_OK;
  hipLaunchKernelGGL(kl_rows_kernel, dim3((rows + kRowsPerBlock - 1) / kRowsPerBlock), dim3(64 * kRowsPerBlock), 0,
                     stream, p_ref, p, rows, cols, row_ws);
  int rc = check_hip(hipGetLastError(), "kl_rows_kernel launch");
  if (rc) return rc;
  // [0] += sum of the per-image KL terms, [1] += rows
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, stream, row_ws, rows, 1, 1.0, 1.0, stats, 0);
  return check_hip(hipGetLastError(), "sum_rows_kernel launch");
}
