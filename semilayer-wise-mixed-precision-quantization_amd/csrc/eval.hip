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


// ---- AdaptiveAvgPool2d(1) + flatten + fc (resnet.py:216-218), batch-invariant ----------------
// pooled[n][c] = (x[n][0][c] + x[n][1][c] + ... + x[n][hw-1][c]) / hw, summed in pixel order: one
// thread per 4 channels of one image (float4 loads, consecutive threads -> consecutive channels).
__global__ __launch_bounds__(256) void avgpool_kernel(const float* __restrict__ x, int n, int hw, int c,
                                                      float* __restrict__ pooled) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const int c4 = c / 4;
  if (t >= (long long)n * c4) return;
  const int img = (int)(t / c4), q = (int)(t - (long long)img * c4);
  const float4* p = reinterpret_cast<const float4*>(x + (long long)img * hw * c) + q;
  float4 s = p[0];
  // the pixels' loads in batches of 8 in flight (one at a time made this kernel latency-bound at
  // ~2 TB/s); the sum itself stays one chain in pixel order
  int i = 1;
  for (; i + 8 <= hw; i += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(long long)(i + u) * c4];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s.x = __fadd_rn(s.x, v[u].x);
      s.y = __fadd_rn(s.y, v[u].y);
      s.z = __fadd_rn(s.z, v[u].z);
      s.w = __fadd_rn(s.w, v[u].w);
    }
  }
  for (; i < hw; ++i) {
    const float4 v = p[(long long)i * c4];
    s.x = __fadd_rn(s.x, v.x);
    s.y = __fadd_rn(s.y, v.y);
    s.z = __fadd_rn(s.z, v.z);
    s.w = __fadd_rn(s.w, v.w);
  }
  const float d = (float)hw;
  reinterpret_cast<float4*>(pooled)[t] = make_float4(__fdiv_rn(s.x, d), __fdiv_rn(s.y, d), __fdiv_rn(s.z, d),
                                                     __fdiv_rn(s.w, d));
}

// logits[i][o] = fc_b[o] + ((s_0 + s_1) + s_2) + s_3, where s_q = sum over the q-th quarter of k
// (kFcK-aligned ranges fixed by c alone) as one fmaf chain in k order: the order depends on nothing
// but c, so a row's logits are the same bits in any batch. Block: 8 images x 64 outputs; its 512
// threads are 4 K-quarter groups of 128 (group g = threads 128 g ..), thread (i = t / 16, o4 = t % 16)
// of a group owns outputs 4 o4 .. 4 o4 + 3 of image i over the group's quarter. Each group stages
// its own 32-k chunks in LDS (k-major, two buffers), with the global loads of the next TWO chunks in
// flight (two register sets) under the current chunk's FMAs — with one in flight the kernel waited
// on each chunk's load latency in turn; the groups' partials meet in LDS and group 0 adds them in
// quarter order.
// (Round 4's one-chain kernel ran 16 x 64 tiles over all of k per thread: 110-190 us per R50 slice
// of 128 images, a fifth of the chip busy; this one splits the chain four ways over 4x the blocks.)
constexpr int kFcI = 8, kFcO = 64, kFcK = 32, kFcG = 4;
constexpr int kFcKQ = kFcK / 4;  // float4 per staged row
__global__ __launch_bounds__(512) void fc_kernel(const float* __restrict__ pooled, int n, int c,
                                                 const float* __restrict__ w, const float* __restrict__ b, int nout,
                                                 float* __restrict__ logits) {
  // per buffer and group, k-major LDS images (rows padded: the transposing writes stay at <= 4-way
  // conflicts)
  __shared__ __attribute__((aligned(16))) float sp[2][kFcG][kFcK][kFcI + 4];
  __shared__ __attribute__((aligned(16))) float sw[2][kFcG][kFcK][kFcO + 4];
  __shared__ __attribute__((aligned(16))) float part[kFcG - 1][kFcI][kFcO];
  const int grp = threadIdx.x >> 7, tid = threadIdx.x & 127;
  const int i0 = blockIdx.y * kFcI, o0 = blockIdx.x * kFcO;
  const int ti = tid / 16, to = tid % 16;
  // quarter ranges: whole kFcK chunks, fixed by c
  const int cq = ((c + kFcG - 1) / kFcG + kFcK - 1) / kFcK * kFcK;
  const int kb = min(c, grp * cq), ke = min(c, kb + cq);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // staging: pooled kFcI images x kFcK k (one float4 per thread of the group's first kFcI * kFcKQ);
  // weights kFcO x kFcK k (kFcO * kFcKQ / 128 float4 per thread)
  constexpr int kWR = kFcO * kFcKQ / 128;
  struct Regs {
    float4 p, w[kWR];
  };
  auto load = [&](Regs& r, int k0) {
    {
      const int ii = tid / kFcKQ, kq = tid % kFcKQ, img = i0 + ii, k = k0 + 4 * kq;
      r.p = (tid < kFcI * kFcKQ && img < n && k < ke) ? *reinterpret_cast<const float4*>(pooled + (long long)img * c + k)
                                                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < kWR; ++q) {
      const int e = tid + 128 * q, oo = e / kFcKQ, kq = e % kFcKQ, o = o0 + oo, k = k0 + 4 * kq;
      r.w[q] = (o < nout && k < ke) ? *reinterpret_cast<const float4*>(w + (long long)o * c + k)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](const Regs& r, int buf) {
    if (tid < kFcI * kFcKQ) {
      const int ii = tid / kFcKQ, kq = tid % kFcKQ;
      sp[buf][grp][4 * kq][ii] = r.p.x;
      sp[buf][grp][4 * kq + 1][ii] = r.p.y;
      sp[buf][grp][4 * kq + 2][ii] = r.p.z;
      sp[buf][grp][4 * kq + 3][ii] = r.p.w;
    }
#pragma unroll
    for (int q = 0; q < kWR; ++q) {
      const int e = tid + 128 * q, oo = e / kFcKQ, kq = e % kFcKQ;
      sw[buf][grp][4 * kq][oo] = r.w[q].x;
      sw[buf][grp][4 * kq + 1][oo] = r.w[q].y;
      sw[buf][grp][4 * kq + 2][oo] = r.w[q].z;
      sw[buf][grp][4 * kq + 3][oo] = r.w[q].w;
    }
  };
  auto compute = [&](int buf, int k0) {
    const int kn = max(0, min(kFcK, ke - k0));
    for (int kk = 0; kk < kn; ++kk) {
      const float pv = sp[buf][grp][kk][ti];
      const float4 wv = *reinterpret_cast<const float4*>(&sw[buf][grp][kk][4 * to]);
      acc[0] = __fmaf_rn(pv, wv.x, acc[0]);
      acc[1] = __fmaf_rn(pv, wv.y, acc[1]);
      acc[2] = __fmaf_rn(pv, wv.z, acc[2]);
      acc[3] = __fmaf_rn(pv, wv.w, acc[3]);
    }
  };
  // every group runs the same number of chunk steps (barriers are block-wide); a group past its
  // range computes nothing. Chunk s: register set / LDS buffer s % 2; the one barrier per chunk
  // also certifies that every wave finished computing chunk s - 1, whose buffer chunk s + 1 refills.
  const int steps = (cq + kFcK - 1) / kFcK;
  Regs ra, rb;
  load(ra, kb);
  if (steps > 1) load(rb, kb + kFcK);
  for (int s = 0; s < steps; s += 2) {
    store(ra, 0);
    __syncthreads();
    if (s + 2 < steps) load(ra, kb + (s + 2) * kFcK);
    compute(0, kb + s * kFcK);
    if (s + 1 < steps) {
      store(rb, 1);
      __syncthreads();
      if (s + 3 < steps) load(rb, kb + (s + 3) * kFcK);
      compute(1, kb + (s + 1) * kFcK);
    }
  }
  if (grp > 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) part[grp - 1][ti][4 * to + j] = acc[j];
  }
  __syncthreads();
  if (grp > 0) return;
  const int img = i0 + ti;
  if (img >= n) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = o0 + 4 * to + j;
    float v = acc[j];
#pragma unroll
    for (int q = 0; q < kFcG - 1; ++q) v = __fadd_rn(v, part[q][ti][4 * to + j]);
    if (o < nout) logits[(long long)img * nout + o] = b ? __fadd_rn(v, b[o]) : v;
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

extern "C" int smpq_avgpool_fc(const float* x, int n, int hw, int c, const float* fc_w, const float* fc_b, int nout,
                               float* pooled_ws, float* logits, smpq_stream_t stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  if (n < 0 || hw <= 0 || c <= 0 || (c % 4) != 0 || nout <= 0 ||
      (n > 0 && (!x || !fc_w || !pooled_ws || !logits)))
    return fail(SMPQ_E_INVALID, "smpq_avgpool_fc: bad arguments (c % 4 == 0)");
  if (n == 0) return SMPQ_OK;
  if ((long long)n * hw * c > 0x7fffffffLL * 4 || n > 65535 * kFcI)
    return fail(SMPQ_E_SHAPE, "smpq_avgpool_fc: tensor too large");
  const long long threads = (long long)n * (c / 4);
  hipLaunchKernelGGL(avgpool_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream, x, n, hw, c,
                     pooled_ws);
  int rc = check_hip(hipGetLastError(), "avgpool_kernel launch");
  if (rc) return rc;
  hipLaunchKernelGGL(fc_kernel, dim3((nout + kFcO - 1) / kFcO, (n + kFcI - 1) / kFcI), dim3(512), 0, stream,
                     pooled_ws, n, c, fc_w, fc_b, nout, logits);
  return check_hip(hipGetLastError(), "fc_kernel launch");
}
