// Weight fake-quantizer (bit-exact with the reference) and the int8 code packer.
//
// Reference arithmetic (functions.py:25-43, quantize_wgt), per output channel t:
//   mn, mx  = exact fp32 min / max of t                      (functions.py:35-36, .item())
//   scale   = (mx - mn) / (2^bit - 1)           IEEE double   (functions.py:39)
//   z       = round(mn / scale)                 half-even      (functions.py:40)
//   q       = (rne(t / f32(scale) + f32(z)) - f32(z)) * f32(scale)   fp32 ops (functions.py:41)
// What `t / scale` (scale a Python float) rounds to depends on where the reference's tensor lives:
//   SMPQ_QSEM_CPU     torch CPU: a correctly rounded fp32 division t / f32(scale) (__fdiv_rn);
//   SMPQ_QSEM_DEVICE  torch on the GPU: t * f32(1.0 / scale), a multiply by the reciprocal of the
//                     DOUBLE scale rounded once to fp32 (ATen's tensor-by-scalar division on
//                     device; pinned by tests/golden/quant_kat_device.npz, which torch itself
//                     produced on an MI355X: 2 of the 69 KAT channels round differently there).
// The reference's drivers quantize channels of a model already moved to the GPU
// (functions.py:97 net.to(device) before resnet50_main.py:189-197), so device tensors default to
// SMPQ_QSEM_DEVICE and host tensors to SMPQ_QSEM_CPU (smpq.quant). FP contraction is off.
//
// One workgroup per output channel: channels are at most 4608 elements (R50 layer4 conv2),
// so a 256-thread block covers a channel in <= 18 iterations and the launch is a single
// wave of blocks over all channels of a layer (22,656 channels for all of ResNet-50).
#include <cmath>
#include <cstring>
#include <string>

#include "common.h"

#pragma clang fp contract(off)

namespace smpq {

constexpr int kQThreads = 256;

__device__ __forceinline__ void block_minmax(float& mn, float& mx, float* smem) {
  // smem: 2 * (kQThreads / 64) floats
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane == 0) {
    smem[wid] = mn;
    smem[kQThreads / kWave + wid] = mx;
  }
  __syncthreads();
  mn = smem[0];
  mx = smem[kQThreads / kWave];
#pragma unroll
  for (int i = 1; i < kQThreads / kWave; ++i) {
    mn = fminf(mn, smem[i]);
    mx = fmaxf(mx, smem[kQThreads / kWave + i]);
  }
}

__global__ __launch_bounds__(kQThreads) void quantize_channels_kernel(
    float* __restrict__ w, int k, const int8_t* __restrict__ bits, float* __restrict__ scale_out,
    int32_t* __restrict__ status, int semantics) {
  __shared__ float smem[2 * kQThreads / kWave];
  const int c = blockIdx.x;
  const int b = bits[c];
  if (b <= 0) return;
  float* row = w + (size_t)c * k;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < k; i += kQThreads) {
    const float v = row[i];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  block_minmax(mn, mx, smem);
  if (mx == mn) {  // reference: ZeroDivisionError at functions.py:40
    if (threadIdx.x == 0) atomicCAS(reinterpret_cast<int*>(status), 0, c + 1);
    return;
  }
  const double scale = ((double)mx - (double)mn) / (double)((1 << b) - 1);
  const double zd = rint((double)mn / scale) + 0.0;  // Python round(): half-to-even; no -0
  const float s32 = (float)scale;
  const float z32 = (float)zd;
  const float inv32 = (float)(1.0 / scale);
  const bool dev = semantics == SMPQ_QSEM_DEVICE;
  for (int i = threadIdx.x; i < k; i += kQThreads) {
    const float t = row[i];
    const float d = dev ? __fmul_rn(t, inv32) : __fdiv_rn(t, s32);
    const float q = rintf(d + z32) - z32;
    row[i] = __fmul_rn(q, s32);
  }
  if (threadIdx.x == 0) scale_out[c] = s32;
}

// Weight codes for the conv's B operand, one workgroup per output channel.
//   w [cout][cin][kh][kw] fp32, step [cout] (0 = channel never quantized).
//   Exact mode (step > 0 and every w == fl32(m * step), |m| <= WMAX): the integer codes m of
//     the reference quantizer (functions.py:41) — recovered by m = rne(w / step), exact because
//     |w / step - m| < 2^-14 — verified bitwise.
//   Fixed mode (lw >= 2: unquantized / off-grid channels): per-channel fixed point with
//     WMAX = 32512 (lw 2, 16-bit) or 8323072 (lw 3, 24-bit): wscale = max|w| / WMAX,
//     m = rne(w / wscale).
//   lw == 1: m - offset stored as one int8 plane (offset != 0 only when [min m, max m] is not
//     inside [-128, 127]); lw >= 2: m stored as lw balanced int8 digit planes, no offset.
//   lw >= 2, exact channels: m is shifted left by the most bits that keep max|m| << sh <= WMAX
//     (wscale = step * 2^-sh, exact), so every channel's magnitude sits in the TOP weight limb.
//     The conv kernels skip the low-digit products (limb pairs l + lw < L + LW - 4); without the
//     shift an 8-bit code would live in limb 0 alone and lose the low activation limbs entirely
//     (a mixed exact / fixed-point conv of a mid-search layer was off by ~1e-3 of its logits).
//     The shift changes no value (m * step == (m << sh) * (step * 2^-sh) exactly), only which
//     limb products carry it.
//   Layout: codes[l][c][k], k = tap * cin_pad + ci (tap = r * kw + q), zero-padded to K.
//   status[0] += off-grid channels (lw == 1: error), status[1] += channels whose exact codes do
//   not fit (lw == 1: > 256 levels), status[2] += channels coded in fixed mode.
constexpr float kW16Max = 32512.f;    // 2-limb fixed-point code range (127 * 256)
constexpr float kW24Max = 8323072.f;  // 3-limb fixed-point code range (127 * 65536)

__global__ __launch_bounds__(kQThreads) void pack_weights_ex_kernel(
    const float* __restrict__ w, int cin, int kh, int kw, int cin_pad, int K, int lw, int s2d,
    const float* __restrict__ step, int8_t* __restrict__ codes, long long wplane,
    int32_t* __restrict__ offset, float* __restrict__ wscale, int32_t* __restrict__ status) {
  __shared__ int smem[4 * kQThreads / kWave];
  __shared__ float sabs[kQThreads / kWave];
  const int c = blockIdx.x;
  const int taps = kh * kw;
  const int kreal = cin * taps;
  const float* row = w + (size_t)c * kreal;
  const float s = step ? step[c] : 0.f;
  const float wmax = lw >= 3 ? kW24Max : kW16Max;
  int mmin = INT32_MAX, mmax = INT32_MIN, bad = (s > 0.f) ? 0 : 1;
  float amax = 0.f;
  for (int i = threadIdx.x; i < kreal; i += kQThreads) {
    const float v = row[i];
    amax = fmaxf(amax, fabsf(v));
    if (bad) continue;
    const float mf = rintf(__fdiv_rn(v, s));
    if (__fmul_rn(mf, s) != v || fabsf(mf) > wmax) {
      bad = 1;
      continue;
    }
    mmin = min(mmin, (int)mf);
    mmax = max(mmax, (int)mf);
  }
  mmin = wave_min_i(mmin);
  mmax = wave_max_i(mmax);
  bad = wave_max_i(bad);
  amax = wave_max(amax);
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane == 0) {
    smem[wid] = mmin;
    smem[4 + wid] = mmax;
    smem[8 + wid] = bad;
    sabs[wid] = amax;
  }
  __syncthreads();
  mmin = min(min(smem[0], smem[1]), min(smem[2], smem[3]));
  mmax = max(max(smem[4], smem[5]), max(smem[6], smem[7]));
  bad = smem[8] | smem[9] | smem[10] | smem[11];
  amax = fmaxf(fmaxf(sabs[0], sabs[1]), fmaxf(sabs[2], sabs[3]));
  int o = 0;
  bool fixed = false, range_bad = false;
  float sc = s;
  if (lw == 1) {
    if (!bad) {
      if (mmax - mmin > 255) range_bad = true;
      else if (mmin < -128 || mmax > 127) o = mmin + 128;
    }
  } else if (bad) {
    fixed = true;
    sc = amax > 0.f ? amax / wmax : 1.f;
  }
  int sh = 0;  // lw >= 2, exact channel: normalize the codes into the top limb
  if (lw >= 2 && !bad) {
    const int am = max(abs(mmin), abs(mmax));
    const int lim = (int)wmax;
    while (am > 0 && sh < 8 * (lw - 1) && (am << (sh + 1)) <= lim) ++sh;
    sc = ldexpf(s, -sh);
  }
  if (threadIdx.x == 0) {
    if (bad && s > 0.f) atomicAdd(&status[0], 1);
    if (lw == 1 && bad && !(s > 0.f)) atomicAdd(&status[0], 1);
    if (range_bad) atomicAdd(&status[1], 1);
    if (fixed) atomicAdd(&status[2], 1);
    if (offset) offset[c] = o;
    if (wscale) wscale[c] = sc;
  }
  const bool zero = (lw == 1) && (bad || range_bad);
  for (int k = threadIdx.x; k < K; k += kQThreads) {
    int src = -1;  // index of the weight in the [cin][kh][kw] row, or -1 for a zero code
    if (s2d) {
      // space-to-depth stem (smpq_pack_weights_s2d): k = [ty][tx][dy][dx][c] over a 4 x 4 x 16
      // kernel; original tap (2 ty + dy - 1, 2 tx + dx - 1) of channel c
      const int t = k >> 4, ch = k & 15;
      const int kr = 2 * (t >> 2) + (ch >> 3) - 1, kc = 2 * (t & 3) + ((ch >> 2) & 1) - 1, ci = ch & 3;
      if (ci < cin && kr >= 0 && kr < kh && kc >= 0 && kc < kw) src = ci * taps + kr * kw + kc;
    } else {
      const int tap = k / cin_pad;
      const int ci = k - tap * cin_pad;
      if (tap < taps && ci < cin) src = ci * taps + tap;
    }
    int m = 0;
    if (!zero && src >= 0) {
      const float v = row[src];
      // fixed point: round in double (at 24 bits an fp32 quotient cannot round exactly)
      if (fixed) m = (int)fmin(fmax(rint((double)v / (double)sc), -(double)wmax), (double)wmax);
      else m = ((int)rintf(__fdiv_rn(v, s)) - o) * (1 << sh);
    }
    for (int l = 0; l < lw; ++l) {  // balanced base-256 digits (the last one takes the rest)
      const int lo = (l == lw - 1) ? m : ((m + 128) & 255) - 128;
      codes[l * wplane + (size_t)c * K + k] = (int8_t)lo;
      m = (m - lo) >> 8;
    }
  }
}

// ------------------------------------------------------------------------------------------
// host twin (native C++, same arithmetic)
// ------------------------------------------------------------------------------------------
static int quantize_row_host(float* row, int k, int b, float* s_out, int semantics) {
  float mn = INFINITY, mx = -INFINITY;
  for (int i = 0; i < k; ++i) {
    mn = std::fmin(mn, row[i]);
    mx = std::fmax(mx, row[i]);
  }
  if (mx == mn) return SMPQ_E_CONSTANT;
  const double scale = ((double)mx - (double)mn) / (double)((1 << b) - 1);
  const double zd = std::nearbyint((double)mn / scale) + 0.0;
  const float s32 = (float)scale;
  const float z32 = (float)zd;
  const float inv32 = (float)(1.0 / scale);
  for (int i = 0; i < k; ++i) {
    // fp32 IEEE division, or the device's reciprocal multiply (contraction is off in this file)
    const float d = semantics == SMPQ_QSEM_DEVICE ? row[i] * inv32 : row[i] / s32;
    const float q = std::nearbyintf(d + z32) - z32;
    row[i] = q * s32;
  }
  *s_out = s32;
  return SMPQ_OK;
}

}  // namespace smpq

using namespace smpq;

extern "C" int smpq_quantize_channels_ex(float* w, int cout, int k_elems, const int8_t* bits,
                                         float* scale_out, int32_t* status, int semantics,
                                         smpq_stream_t stream) {
  if (!w || !bits || !scale_out || !status || cout <= 0 || k_elems <= 0)
    return fail(SMPQ_E_INVALID, "smpq_quantize_channels: bad arguments");
  if (semantics != SMPQ_QSEM_CPU && semantics != SMPQ_QSEM_DEVICE)
    return fail(SMPQ_E_INVALID, "smpq_quantize_channels: semantics must be SMPQ_QSEM_CPU or SMPQ_QSEM_DEVICE");
  hipLaunchKernelGGL(quantize_channels_kernel, dim3(cout), dim3(kQThreads), 0,
                     (hipStream_t)stream, w, k_elems, bits, scale_out, status, semantics);
  return check_hip(hipGetLastError(), "quantize_channels_kernel launch");
}

extern "C" int smpq_quantize_channels(float* w, int cout, int k_elems, const int8_t* bits,
                                      float* scale_out, int32_t* status, smpq_stream_t stream) {
  return smpq_quantize_channels_ex(w, cout, k_elems, bits, scale_out, status, SMPQ_QSEM_CPU, stream);
}

extern "C" int smpq_quantize_channels_host_ex(float* w, int cout, int k_elems, const int8_t* bits,
                                              float* scale_out, int semantics) {
  if (!w || !bits || cout <= 0 || k_elems <= 0)
    return fail(SMPQ_E_INVALID, "smpq_quantize_channels_host: bad arguments");
  if (semantics != SMPQ_QSEM_CPU && semantics != SMPQ_QSEM_DEVICE)
    return fail(SMPQ_E_INVALID, "smpq_quantize_channels_host: semantics must be SMPQ_QSEM_CPU or SMPQ_QSEM_DEVICE");
  for (int c = 0; c < cout; ++c) {
    const int b = bits[c];
    if (b <= 0) continue;
    if (b > 30) return fail(SMPQ_E_BITS, "smpq_quantize_channels_host: bit > 30");
    float* row = w + (size_t)c * k_elems;
    float s32 = 0.f;
    const int rc = quantize_row_host(row, k_elems, b, &s32, semantics);
    if (rc != SMPQ_OK)
      return fail(rc, "float division by zero (constant channel " + std::to_string(c) + ")");
    if (scale_out) scale_out[c] = s32;
  }
  return SMPQ_OK;
}

extern "C" int smpq_quantize_channels_host(float* w, int cout, int k_elems, const int8_t* bits,
                                           float* scale_out) {
  return smpq_quantize_channels_host_ex(w, cout, k_elems, bits, scale_out, SMPQ_QSEM_CPU);
}

extern "C" int smpq_pack_weights(const float* w, int cout, int cin, int kh, int kw,
                                 const float* step, int8_t* codes, int32_t* offset,
                                 int32_t* status, smpq_stream_t stream) {
  if (!w || !step || !codes || !offset || !status || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0)
    return fail(SMPQ_E_INVALID, "smpq_pack_weights: bad arguments");
  const int K = cin * kh * kw;
  hipLaunchKernelGGL(pack_weights_ex_kernel, dim3(cout), dim3(kQThreads), 0, (hipStream_t)stream, w,
                     cin, kh, kw, cin, K, 1, 0, step, codes, (long long)cout * K, offset, (float*)nullptr,
                     status);
  return check_hip(hipGetLastError(), "pack_weights_ex_kernel launch");
}

extern "C" int smpq_pack_weights_ex(const float* w, int cout, int cin, int kh, int kw, const float* step,
                                    int wlimbs, int8_t* codes, int32_t* offset, float* wscale,
                                    int32_t* status, smpq_stream_t stream) {
  if (!w || !codes || !wscale || !status || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0)
    return fail(SMPQ_E_INVALID, "smpq_pack_weights_ex: bad arguments");
  if (wlimbs < 1 || wlimbs > 3) return fail(SMPQ_E_INVALID, "smpq_pack_weights_ex: wlimbs must be 1, 2 or 3");
  if (wlimbs == 1 && (!step || !offset))
    return fail(SMPQ_E_INVALID, "smpq_pack_weights_ex: wlimbs == 1 needs step and offset");
  if (cin % 64 != 0)
    return fail(SMPQ_E_SHAPE,
                "smpq_pack_weights_ex: cin must be a multiple of 64 (the <= 4-channel stem: smpq_pack_weights_s2d_ex)");
  const int K = cin * kh * kw;
  hipLaunchKernelGGL(pack_weights_ex_kernel, dim3(cout), dim3(kQThreads), 0, (hipStream_t)stream, w,
                     cin, kh, kw, cin, K, wlimbs, 0, step, codes, (long long)cout * K, offset, wscale,
                     status);
  return check_hip(hipGetLastError(), "pack_weights_ex_kernel launch");
}

extern "C" int smpq_pack_weights_s2d_ex(const float* w, int cout, int cin, const float* step, int wlimbs,
                                        int8_t* codes, float* wscale, int32_t* status, smpq_stream_t stream) {
  if (!w || !codes || !wscale || !status || cout <= 0 || cin <= 0 || cin > 4)
    return fail(SMPQ_E_INVALID, "smpq_pack_weights_s2d: bad arguments (cin must be 1..4)");
  if (wlimbs < 2 || wlimbs > 3) return fail(SMPQ_E_INVALID, "smpq_pack_weights_s2d: wlimbs must be 2 or 3");
  constexpr int K = 256;  // 4 x 4 taps x 16 space-to-depth channels
  hipLaunchKernelGGL(pack_weights_ex_kernel, dim3(cout), dim3(kQThreads), 0, (hipStream_t)stream, w, cin, 7, 7,
                     16, K, wlimbs, 1, step, codes, (long long)cout * K, (int32_t*)nullptr, wscale, status);
  return check_hip(hipGetLastError(), "pack_weights_ex_kernel launch");
}

extern "C" int smpq_pack_weights_s2d(const float* w, int cout, int cin, int wlimbs, int8_t* codes, float* wscale,
                                     int32_t* status, smpq_stream_t stream) {
  return smpq_pack_weights_s2d_ex(w, cout, cin, nullptr, wlimbs, codes, wscale, status, stream);
}
