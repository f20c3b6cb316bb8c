// Quantized convolution forward for gfx950 (CDNA4): the C-ABI of the int8-MFMA conv (its kernel,
// qconv_glds_kernel, is in conv_glds_kernel.h) and the activation-side helper kernels
// (quantizers, max pools, per-image ranges, the K-major weight copy).
//
// Replaces nn.Conv2d on the fake-quantized weight (resnet.py:22-30) together with the eval
// BatchNorm, ReLU and residual add that follow it (resnet.py:55-68 / 97-116), and the
// unquantized stem / downsample convs (resnet.py:143, 188-192).
//
// GEMM view (NHWC activations):
//   M = n*ho*wo output pixels, N = cout, K = kh*kw*cin ordered [kh][kw][cin], cin % 64 == 0: one
//   64-wide K step is 64 contiguous channels of one tap (64 B per limb). The 7x7/2 stem on <= 4
//   channels runs as a 4x4/1 conv over 16-channel space-to-depth pixels (smpq_stem_conv_s2d_q).
//   A[m][k] = activation code at the tap's input pixel (0 outside the image: zero padding).
//   B[k][n] = weight code (int8 limbs, from smpq_pack_weights_ex).
//
// Weights: LW int8 limbs. LW = 1: the reference's integer codes m (functions.py:41: the weight is
// exactly fl32(m * step)), centred by a per-channel offset when needed — exact. LW = 2 / 3: 16 /
// 24-bit per-channel fixed point for fp32 (unquantized) weights (LW follows the activation width),
// or exact codes that do not fit int8.
// Activations: L int8 limbs of a per-image fixed point q = rne(x * QMAX / max|x_img|)
// (act_quantize_kernel), L = 1 / 2 / 3 -> int8 / int16 / int24.
// Each (activation limb, weight limb) pair is one MFMA pass; passes of equal total weight
// 256^(la+lw) share an int32 accumulator, recombined in fp32 in the epilogue. With 3-limb operands
// on both sides (24-bit x 24-bit) the passes with la + lw < SMIN = L + LW - 4 (products of two low
// digits, weight <= 2^-22 of the top product, i.e. below the 24-bit quantization step itself) are
// skipped: 6 passes instead of 9. All accumulation is exact integer arithmetic, so results are
// independent of the tile configuration and of the batch composition (per-image steps).
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "conv_common.h"

namespace smpq {

// ------------------------------------------------------------------------------------------
// x (fp32, any layout, n images of per_image elements) -> L int8 digit planes of
// q = clamp(rne(x * (QMAX / absmax[img])), +-QMAX). 8 elements per thread: two float4 loads,
// one 8-byte store per plane.
template <int L>
__global__ __launch_bounds__(256) void act_quantize_kernel(const float* __restrict__ x, long long total,
                                                           long long per_image,
                                                           const float* __restrict__ absmax,
                                                           int8_t* __restrict__ out, long long plane) {
  const float qmax = act_qmax<L>();
  const long long nvec = total / 8;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec;
       v += (long long)gridDim.x * blockDim.x) {
    const long long e = v * 8;
    const int img = (int)(e / per_image);
    const float am = absmax[img];
    const float inv = am > 0.f ? qmax / am : 0.f;
    const float4 x0 = *reinterpret_cast<const float4*>(x + e);
    const float4 x1 = *reinterpret_cast<const float4*>(x + e + 4);
    const float vals[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    unsigned int lo[L], hi[L];
#pragma unroll
    for (int l = 0; l < L; ++l) lo[l] = hi[l] = 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float qf = rintf(vals[k] * inv);
      qf = fminf(fmaxf(qf, -qmax), qmax);
      int d[L];
      split_limbs<L>((int)qf, d);
#pragma unroll
      for (int l = 0; l < L; ++l) {
        const unsigned int byte = (unsigned int)(d[l] & 255);
        if (k < 4) lo[l] |= byte << (8 * k);
        else hi[l] |= byte << (8 * (k - 4));
      }
    }
#pragma unroll
    for (int l = 0; l < L; ++l)
      *reinterpret_cast<uint2*>(out + l * plane + e) = make_uint2(lo[l], hi[l]);
  }
}

// NCHW fp32 images (c <= 4 channels) -> L int8 limb planes in space-to-depth layout
// [n][ceil(h/2)][ceil(w/2)][16], channel (dy * 2 + dx) * 4 + c = pixel (2i + dy, 2j + dx), channel c
// (zero for c >= c_in, and for a pixel past an odd h or w: the stem conv's own zero padding): the
// stem's 7x7/2 conv becomes a 4x4/1 conv over 16-channel pixels whose 64-B K steps are whole tap
// rows (smpq_stem_conv_s2d_q). One thread = one 16-channel pixel.
template <int L>
__global__ __launch_bounds__(256) void image_quantize_s2d_kernel(const float* __restrict__ x, int n, int c, int h,
                                                                 int w, const float* __restrict__ absmax,
                                                                 int8_t* __restrict__ out, long long plane) {
  const float qmax = act_qmax<L>();
  const int h2 = (h + 1) / 2, w2 = (w + 1) / 2;
  const bool even_w = (w & 1) == 0;
  const long long total = (long long)n * h2 * w2;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(p % w2);
    const long long t = p / w2;
    const int i = (int)(t % h2);
    const int img = (int)(t / h2);
    const float am = absmax[img];
    const float inv = am > 0.f ? qmax / am : 0.f;
    unsigned int word[L][4];
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int g = 0; g < 4; ++g) word[l][g] = 0u;
    for (int ch = 0; ch < c; ++ch) {
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        if (2 * i + dy >= h) continue;  // odd h: the zero row
        const float* row = x + (((size_t)img * c + ch) * h + 2 * i + dy) * w + 2 * j;
        float vals[2];
        if (even_w) {
          const float2 v = *reinterpret_cast<const float2*>(row);
          vals[0] = v.x;
          vals[1] = v.y;
        } else {  // odd w: rows are not 8-B aligned, and the last column pair has one pixel
          vals[0] = row[0];
          vals[1] = 2 * j + 1 < w ? row[1] : 0.f;
        }
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          const float qf = fminf(fmaxf(rintf(vals[dx] * inv), -qmax), qmax);
          int d[L];
          split_limbs<L>((int)qf, d);
          const int g = dy * 2 + dx;  // byte 4 g + ch of the 16
#pragma unroll
          for (int l = 0; l < L; ++l) word[l][g] |= (unsigned int)(d[l] & 255) << (8 * ch);
        }
      }
    }
#pragma unroll
    for (int l = 0; l < L; ++l)
      st16(out + l * plane + 16 * p, v4i{(int)word[l][0], (int)word[l][1], (int)word[l][2], (int)word[l][3]});
  }
}

// 3x3 / stride 2 / pad 1 max pool (resnet.py:147) on NHWC fp32, fused with the activation
// quantizer of its output (per-image range absmax = max of the pool input: max-pooling a
// non-negative ReLU output keeps the per-image maximum). Optional fp32 output.
// One thread = 4 channels of one output pixel.
template <int L>
__global__ __launch_bounds__(256) void maxpool_quantize_kernel(const float* __restrict__ x, int n, int h,
                                                               int w, int c, int ho, int wo,
                                                               const float* __restrict__ absmax,
                                                               int8_t* __restrict__ out, long long plane,
                                                               float* __restrict__ out_f32) {
  const float qmax = act_qmax<L>();
  const int c4 = c / 4;
  const long long total = (long long)n * ho * wo * c4;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int cq = (int)(t % c4);
    long long p = t / c4;
    const int ow = (int)(p % wo);
    p /= wo;
    const int oh = (int)(p % ho);
    const int img = (int)(p / ho);
    float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
    for (int dr = 0; dr < 3; ++dr) {
      const int ih = 2 * oh - 1 + dr;
      if ((unsigned)ih >= (unsigned)h) continue;
#pragma unroll
      for (int dc = 0; dc < 3; ++dc) {
        const int iw = 2 * ow - 1 + dc;
        if ((unsigned)iw >= (unsigned)w) continue;
        const float4 v = *reinterpret_cast<const float4*>(x + (((size_t)img * h + ih) * w + iw) * c + 4 * cq);
        m.x = fmaxf(m.x, v.x);
        m.y = fmaxf(m.y, v.y);
        m.z = fmaxf(m.z, v.z);
        m.w = fmaxf(m.w, v.w);
      }
    }
    const size_t o = (((size_t)img * ho + oh) * wo + ow) * c + 4 * cq;
    if (out_f32) st16(out_f32 + o, v4i{__float_as_int(m.x), __float_as_int(m.y), __float_as_int(m.z), __float_as_int(m.w)});
    const float am = absmax[img];
    const float inv = am > 0.f ? qmax / am : 0.f;
    const float vals[4] = {m.x, m.y, m.z, m.w};
    unsigned int word[L];
#pragma unroll
    for (int l = 0; l < L; ++l) word[l] = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float qf = fminf(fmaxf(rintf(vals[k] * inv), -qmax), qmax);
      int d[L];
      split_limbs<L>((int)qf, d);
#pragma unroll
      for (int l = 0; l < L; ++l) word[l] |= (unsigned int)(d[l] & 255) << (8 * k);
    }
#pragma unroll
    for (int l = 0; l < L; ++l) *reinterpret_cast<unsigned int*>(out + l * plane + o) = word[l];
  }
}

// 3x3 / stride 2 / pad 1 max pool on int8 limb planes [L][n][h][w][c] (c % 16 == 0): the codes of
// one activation share one step, so the max of the codes is the code of the max (the quantizer
// is monotone) — exact. One thread = 16 channels of one output pixel (16-B loads per limb).
template <int L>
__global__ __launch_bounds__(256) void maxpool_limbs_kernel(const int8_t* __restrict__ x, int n, int h, int w, int c,
                                                            int ho, int wo, long long iplane,
                                                            int8_t* __restrict__ out, long long oplane) {
  // one thread = 16 channels of one pooled pixel; all 9 taps x L limbs are loaded before any is
  // used (27 independent 16-B loads in flight). A tap outside the image re-reads the window's
  // centre (2 oh, 2 ow), which is always inside and already part of the max: no masks.
  const int c16 = c / 16;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;  // total < 2^31 (checked by the launcher)
  if (t >= n * ho * wo * c16) return;
  const int cq = t % c16;
  int p = t / c16;
  const int ow = p % wo;
  p /= wo;
  const int oh = p % ho;
  const int img = p / ho;
  const long long base = (long long)img * h * w;
  v4i d[9][L];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    int ih = 2 * oh - 1 + tap / 3, iw = 2 * ow - 1 + tap % 3;
    if ((unsigned)ih >= (unsigned)h || (unsigned)iw >= (unsigned)w) {
      ih = 2 * oh;
      iw = 2 * ow;
    }
    const long long off = ((base + (long long)ih * w + iw) * c) + 16 * cq;
#pragma unroll
    for (int l = 0; l < L; ++l) d[tap][l] = *reinterpret_cast<const v4i*>(x + l * iplane + off);
  }
  int m[16];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      unsigned wv[L];
#pragma unroll
      for (int l = 0; l < L; ++l) wv[l] = (unsigned)d[tap][l][k];
      int q[4];
      decode4<L>(wv, q);
#pragma unroll
      for (int r = 0; r < 4; ++r) m[4 * k + r] = tap == 0 ? q[r] : max(m[4 * k + r], q[r]);
    }
  const long long o = (((long long)img * ho + oh) * wo + ow) * c + 16 * cq;
  unsigned wd[4][L];
#pragma unroll
  for (int k = 0; k < 4; ++k) encode4<L>(&m[4 * k], wd[k]);
#pragma unroll
  for (int l = 0; l < L; ++l)
    st16(out + l * oplane + o, v4i{(int)wd[0][l], (int)wd[1][l], (int)wd[2][l], (int)wd[3][l]});
}

__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, int64_t per_image,
                                                     float* __restrict__ out) {
  const int img = blockIdx.y;
  const float* p = x + (size_t)img * per_image;
  float m = 0.f;
  const int64_t start = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  if ((per_image & 3) == 0) {
    // four independent 16-B loads in flight per iteration (one at a time left the kernel
    // latency-bound: 2.9 TB/s on the input images of the R50 bench)
    int64_t i = start;
    for (; i + 3 * stride < per_image; i += 4 * stride) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(p + i + u * stride);
#pragma unroll
      for (int u = 0; u < 4; ++u) m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
    for (; i < per_image; i += stride) {
      const float4 v = *reinterpret_cast<const float4*>(p + i);
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  } else {
    for (int64_t i = start / 4; i < per_image; i += stride / 4) m = fmaxf(m, fabsf(p[i]));
  }
  __shared__ float red[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f) atomic_max_nonneg(&out[img], m);
  }
}

__global__ void debug_mfma_kernel(const int8_t* a, const int8_t* b, int32_t* c) {
  const int lane = threadIdx.x;
  const int frow = lane & 15, fk = 16 * (lane >> 4);
  const v4i af = *reinterpret_cast<const v4i*>(a + frow * 64 + fk);
  const v4i bf = *reinterpret_cast<const v4i*>(b + frow * 64 + fk);
  v4i acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) c[(4 * (lane >> 4) + r) * 16 + frow] = acc[r];
}

}  // namespace smpq

using namespace smpq;

static int conv_args_q(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                                 const int8_t* codes, int wlimbs, const int32_t* offset, int cout, int kh,
                                 int kw, int stride, int pad, const float* col_scale,
                                 const float* col_shift, const float* residual, int relu, int limbs,
                                 float* y, float* y_absmax, int8_t* yq, float yq_range, int32_t* overflow,
                                 const int8_t* residual_q, float residual_range, ConvArgs& a) {
  if (!xq || !x_absmax || !codes || !col_scale || !col_shift || (!y && !yq))
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: null pointer");
  if (yq && (!overflow || !(yq_range > 0.f)))
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: yq needs overflow flag and a positive range");
  if ((yq || residual_q) && (cout & 3) != 0)
    return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: limb-plane output/residual needs cout % 4 == 0");
  if (residual_q && residual) return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: two residuals");
  if (n <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 || stride <= 0 ||
      pad < 0)
    return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: bad shape");
  if (cin % kKStep != 0)
    return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: cin must be a multiple of 64 (got " + std::to_string(cin) +
                                  "; the <= 4-channel 7x7/2 stem runs on smpq_stem_conv_s2d_q)");
  if (cout % 16 != 0) return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: cout must be a multiple of 16");
  if (wlimbs < 1 || wlimbs > 3) return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: wlimbs must be 1, 2 or 3");
  if (wlimbs == 3 && limbs != 3)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: 3 weight limbs are built for 3 activation limbs only");
  a = ConvArgs{};
  a.s2d = 0;
  a.xq = xq;
  a.plane = (long long)n * h * w * cin;
  a.x_absmax = x_absmax;
  a.codes = codes;
  a.w_off = offset;
  a.col_scale = col_scale;
  a.col_shift = col_shift;
  a.residual = residual;
  a.res_q = residual_q;
  a.res_scale = residual_q ? residual_range / (limbs == 1 ? 127.f : (limbs == 2 ? 32512.f : 8323072.f)) : 0.f;
  a.y = y;
  a.y_absmax = y_absmax;
  a.yq = yq;
  a.overflow = overflow;
  a.yq_inv = yq ? (limbs == 1 ? 127.f : (limbs == 2 ? 32512.f : 8323072.f)) / yq_range : 0.f;
  a.n = n;
  a.h = h;
  a.w = w;
  a.cin = cin;
  a.cout = cout;
  a.kh = kh;
  a.kw = kw;
  a.stride = stride;
  a.pad = pad;
  a.ho = (h + 2 * pad - kh) / stride + 1;
  a.wo = (w + 2 * pad - kw) / stride + 1;
  if (a.ho <= 0 || a.wo <= 0) return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: empty output");
  const long M = (long)n * a.ho * a.wo;
  if (M > 0x7fffffffL || a.plane > 0x7fffffffLL * 8 || (long)n * h * w > 0x7fffffffL)
    return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: tensor too large");
  a.M = (int)M;
  a.K = kh * kw * cin;
  a.cchunks = cin / kKStep;
  a.ksteps = kh * kw * a.cchunks;
  a.wplane = (long long)cout * a.K;
  a.relu = relu ? 1 : 0;
  a.has_offset = (offset && wlimbs == 1) ? 1 : 0;
  fast_div_init(a.ho * a.wo, a.hw_mul, a.hw_shr);
  fast_div_init(a.wo, a.wo_mul, a.wo_shr);
  {
    // outputs larger than this stream past the 256-MB MALL anyway: store them non-temporally
    static const long long nt_min = [] {
      const char* e = getenv("SMPQ_NT_MIN_MB");
      return (e ? atoll(e) : 64LL) << 20;
    }();
    a.nt_store = (yq && (long long)limbs * M * cout >= nt_min) ? 1 : 0;
  }
  if (limbs < 1 || limbs > 3) return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: limbs must be 1, 2 or 3");
  a.inv_qmax = 1.f / (limbs == 1 ? 127.f : (limbs == 2 ? 32512.f : 8323072.f));
  return SMPQ_OK;
}

extern "C" int smpq_conv2d_fwd_q_km(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                                    const int8_t* codes, const int8_t* codes_kmajor, int wlimbs,
                                    const int32_t* offset, int cout, int kh, int kw, int stride, int pad,
                                    const float* col_scale, const float* col_shift, const float* residual, int relu,
                                    int limbs, float* y, float* y_absmax, int8_t* yq, float yq_range,
                                    int32_t* overflow, const int8_t* residual_q, float residual_range, int tile_cfg,
                                    smpq_stream_t stream) {
  ConvArgs a;
  const int rc = conv_args_q(xq, x_absmax, n, h, w, cin, codes, wlimbs, offset, cout, kh, kw, stride, pad, col_scale,
                             col_shift, residual, relu, limbs, y, y_absmax, yq, yq_range, overflow, residual_q,
                             residual_range, a);
  if (rc) return rc;
  if (tile_cfg < 0) {
    tile_cfg = glds_default_cfg(a, limbs, wlimbs);
    // every operand and output plane is addressed with 32-bit buffer offsets: larger batches are
    // split by the caller (smpq.ops.conv2d_q chunks the images)
    if (tile_cfg < 0)
      return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: a limb plane of 2 GiB or more (split the batch)");
  }
  if (tile_cfg >= glds_num_cfgs()) return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: bad tile config");
  if (codes_kmajor) {  // the same codes, K-major (smpq_weights_kmajor): whole-line weight DMA pieces
    a.codes = codes_kmajor;
    a.w_kmajor = 1;
  }
  return launch_glds(tile_cfg, limbs, wlimbs, a, (hipStream_t)stream);
}

extern "C" int smpq_conv2d_fwd_q(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                                 const int8_t* codes, int wlimbs, const int32_t* offset, int cout, int kh,
                                 int kw, int stride, int pad, const float* col_scale,
                                 const float* col_shift, const float* residual, int relu, int limbs,
                                 float* y, float* y_absmax, int8_t* yq, float yq_range, int32_t* overflow,
                                 const int8_t* residual_q, float residual_range, int tile_cfg,
                                 smpq_stream_t stream) {
  return smpq_conv2d_fwd_q_km(xq, x_absmax, n, h, w, cin, codes, nullptr, wlimbs, offset, cout, kh, kw, stride, pad,
                              col_scale, col_shift, residual, relu, limbs, y, y_absmax, yq, yq_range, overflow,
                              residual_q, residual_range, tile_cfg, stream);
}

namespace {
// [LW][cout][K] -> [LW][K/64][cout][64], one 16-B chunk per thread
__global__ void weights_kmajor_kernel(const int4* __restrict__ src, int4* __restrict__ dst, int cout, int kc,
                                      long long chunks_per_limb, long long total) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long long lw = i / chunks_per_limb, r = i - lw * chunks_per_limb;
  const int q = (int)(r & 3);            // 16-B chunk in the 64-B slice
  const long long t = r >> 2;            // (row, slice) in the source order
  const int row = (int)(t / kc), sl = (int)(t - (long long)row * kc);
  dst[lw * chunks_per_limb + ((long long)sl * cout + row) * 4 + q] = src[i];
}
}  // namespace

extern "C" int smpq_weights_kmajor(const int8_t* codes, int wlimbs, int cout, int K, int8_t* out,
                                   smpq_stream_t stream) {
  if (!codes || !out) return fail(SMPQ_E_INVALID, "smpq_weights_kmajor: null pointer");
  if (wlimbs < 1 || wlimbs > 3 || cout <= 0 || K <= 0 || K % 64 != 0)
    return fail(SMPQ_E_SHAPE, "smpq_weights_kmajor: need 1..3 limbs, cout > 0, K % 64 == 0");
  if (((uintptr_t)codes | (uintptr_t)out) & 15) return fail(SMPQ_E_INVALID, "smpq_weights_kmajor: 16-B alignment");
  const long long per = (long long)cout * K / 16, total = per * wlimbs;
  if (total == 0) return 0;
  hipLaunchKernelGGL(weights_kmajor_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const int4*>(codes), reinterpret_cast<int4*>(out), cout, K / 64, per, total);
  return check_hip(hipGetLastError(), "weights_kmajor_kernel launch");
}

extern "C" int smpq_conv2d_fwd_ex(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                                  const int8_t* codes, int wlimbs, const int32_t* offset, int cout, int kh,
                                  int kw, int stride, int pad, const float* col_scale,
                                  const float* col_shift, const float* residual, int relu, int limbs,
                                  float* y, float* y_absmax, int tile_cfg, smpq_stream_t stream) {
  if (!y) return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: null pointer");
  return smpq_conv2d_fwd_q(xq, x_absmax, n, h, w, cin, codes, wlimbs, offset, cout, kh, kw, stride, pad,
                           col_scale, col_shift, residual, relu, limbs, y, y_absmax, nullptr, 0.f, nullptr,
                           nullptr, 0.f, tile_cfg, stream);
}

extern "C" int smpq_conv2d_fwd(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                               const int8_t* codes, const int32_t* offset, int cout, int kh, int kw,
                               int stride, int pad, const float* col_scale, const float* col_shift,
                               const float* residual, int relu, int limbs, float* y, float* y_absmax,
                               int tile_cfg, smpq_stream_t stream) {
  return smpq_conv2d_fwd_ex(xq, x_absmax, n, h, w, cin, codes, 1, offset, cout, kh, kw, stride, pad,
                            col_scale, col_shift, residual, relu, limbs, y, y_absmax, tile_cfg, stream);
}

extern "C" int smpq_conv2d_num_tile_configs(void) { return glds_num_cfgs(); }

extern "C" int smpq_conv2d_tile_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs) {
  if (cfg < 0 || cfg >= glds_num_cfgs() || limbs < 1 || limbs > 3 || wlimbs < 1 || wlimbs > 3) return 0;
  return glds_supported(cfg, cin, cout, kh, kw, limbs, wlimbs) ? 1 : 0;
}

extern "C" int smpq_conv2d_tile_kind(int cfg) {
  if (cfg < 0 || cfg >= glds_num_cfgs()) return fail(SMPQ_E_INVALID, "smpq_conv2d_tile_kind: bad config");
  if (glds_is_halo(cfg)) return SMPQ_TILE_HALO3X3;
  if (glds_is_resident(cfg)) return SMPQ_TILE_RESIDENT1X1;
  return glds_cfg_bk(cfg) == 128 ? SMPQ_TILE_LDS_DMA_K128 : SMPQ_TILE_LDS_DMA;
}

extern "C" int smpq_conv2d_tile_config(int cfg, int* bm, int* bn, int* threads) {
  if (cfg < 0 || cfg >= glds_num_cfgs() || !bm || !bn || !threads)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_tile_config: bad arguments");
  glds_cfg_info(cfg, bm, bn, threads);
  return SMPQ_OK;
}

extern "C" size_t smpq_conv2d_workspace_bytes(int, int, int, int, int, int, int, int, int, int) {
  return 0;
}

static long long grid_for(long long work) {
  long long blocks = (work + 255) / 256;
  if (blocks > 256 * 16) blocks = 256 * 16;
  if (blocks < 1) blocks = 1;
  return blocks;
}

extern "C" int smpq_act_quantize(const float* x, int n, int64_t per_image, const float* absmax, int limbs,
                                 int8_t* out, smpq_stream_t stream) {
  if (!x || !absmax || !out || n <= 0 || per_image <= 0)
    return fail(SMPQ_E_INVALID, "smpq_act_quantize: bad arguments");
  if (per_image % 8 != 0) return fail(SMPQ_E_SHAPE, "smpq_act_quantize: per_image % 8 != 0");
  const long long total = (long long)n * per_image;
  const dim3 grid((unsigned)grid_for(total / 8));
  hipStream_t s = (hipStream_t)stream;
  switch (limbs) {
    case 1: hipLaunchKernelGGL(act_quantize_kernel<1>, grid, dim3(256), 0, s, x, total, per_image, absmax, out, total); break;
    case 2: hipLaunchKernelGGL(act_quantize_kernel<2>, grid, dim3(256), 0, s, x, total, per_image, absmax, out, total); break;
    case 3: hipLaunchKernelGGL(act_quantize_kernel<3>, grid, dim3(256), 0, s, x, total, per_image, absmax, out, total); break;
    default: return fail(SMPQ_E_INVALID, "smpq_act_quantize: limbs must be 1, 2 or 3");
  }
  return check_hip(hipGetLastError(), "act_quantize_kernel launch");
}

extern "C" int smpq_image_quantize_s2d(const float* x, int n, int c, int h, int w, const float* absmax, int limbs,
                                       int8_t* out, smpq_stream_t stream) {
  if (!x || !absmax || !out || n <= 0 || c <= 0 || c > 4 || h <= 1 || w <= 1)
    return fail(SMPQ_E_INVALID, "smpq_image_quantize_s2d: need 1..4 channels and h, w >= 2");
  const long long total = (long long)n * ((h + 1) / 2) * ((w + 1) / 2);
  const long long plane = total * 16;
  const dim3 grid((unsigned)std::min<long long>((total + 255) / 256, 65535));
  hipStream_t s = (hipStream_t)stream;
  switch (limbs) {
    case 1: hipLaunchKernelGGL(image_quantize_s2d_kernel<1>, grid, dim3(256), 0, s, x, n, c, h, w, absmax, out, plane); break;
    case 2: hipLaunchKernelGGL(image_quantize_s2d_kernel<2>, grid, dim3(256), 0, s, x, n, c, h, w, absmax, out, plane); break;
    case 3: hipLaunchKernelGGL(image_quantize_s2d_kernel<3>, grid, dim3(256), 0, s, x, n, c, h, w, absmax, out, plane); break;
    default: return fail(SMPQ_E_INVALID, "smpq_image_quantize_s2d: limbs must be 1, 2 or 3");
  }
  return check_hip(hipGetLastError(), "image_quantize_s2d_kernel launch");
}

extern "C" int smpq_stem_conv_s2d_q(const int8_t* xq, const float* x_absmax, int n, int h, int w,
                                    const int8_t* codes, int wlimbs, int cout, const float* col_scale,
                                    const float* col_shift, int relu, int limbs, float* y, float* y_absmax,
                                    int8_t* yq, float yq_range, int32_t* overflow, int tile_cfg,
                                    smpq_stream_t stream) {
  if (!xq || !x_absmax || !codes || !col_scale || !col_shift || (!y && !yq))
    return fail(SMPQ_E_INVALID, "smpq_stem_conv_s2d_q: null pointer");
  if (yq && (!overflow || !(yq_range > 0.f)))
    return fail(SMPQ_E_INVALID, "smpq_stem_conv_s2d_q: yq needs overflow flag and a positive range");
  if (n <= 0 || h <= 1 || w <= 1 || cout <= 0 || cout % 16 != 0)
    return fail(SMPQ_E_SHAPE, "smpq_stem_conv_s2d_q: bad shape (h, w >= 2, cout % 16 == 0)");
  if (limbs < 1 || limbs > 3) return fail(SMPQ_E_INVALID, "smpq_stem_conv_s2d_q: limbs must be 1, 2 or 3");
  if (tile_cfg < 0) tile_cfg = 0;  // 64 x 64
  if (tile_cfg >= glds_num_cfgs()) return fail(SMPQ_E_INVALID, "smpq_stem_conv_s2d_q: bad tile config");
  ConvArgs a = {};
  a.s2d = 1;
  a.xq = xq;
  a.x_absmax = x_absmax;
  a.codes = codes;
  a.col_scale = col_scale;
  a.col_shift = col_shift;
  a.y = y;
  a.y_absmax = y_absmax;
  a.yq = yq;
  a.overflow = overflow;
  a.yq_inv = yq ? (limbs == 1 ? 127.f : (limbs == 2 ? 32512.f : 8323072.f)) / yq_range : 0.f;
  a.n = n;
  // space-to-depth geometry: 4x4 taps, stride 1, pad 2 (top / left; bottom / right by range). An odd
  // h or w gets a zero row / column from smpq_image_quantize_s2d: the conv's own zero padding there
  a.h = (h + 1) / 2;
  a.w = (w + 1) / 2;
  a.cin = 16;
  a.cout = cout;
  a.kh = a.kw = 4;
  a.stride = 1;
  a.pad = 2;
  a.ho = (h + 2 * 3 - 7) / 2 + 1;  // the original 7x7 / stride 2 / pad 3 output
  a.wo = (w + 2 * 3 - 7) / 2 + 1;
  a.M = n * a.ho * a.wo;
  a.K = 256;
  a.ksteps = 4;
  a.cchunks = 1;
  a.plane = (long long)n * a.h * a.w * 16;
  a.wplane = (long long)cout * a.K;
  a.relu = relu ? 1 : 0;
  a.inv_qmax = 1.f / (limbs == 1 ? 127.f : (limbs == 2 ? 32512.f : 8323072.f));
  fast_div_init(a.ho * a.wo, a.hw_mul, a.hw_shr);
  fast_div_init(a.wo, a.wo_mul, a.wo_shr);
  if ((long long)n * a.ho * a.wo > 0x7fffffffLL) return fail(SMPQ_E_SHAPE, "smpq_stem_conv_s2d_q: tensor too large");
  return launch_glds(tile_cfg, limbs, wlimbs, a, (hipStream_t)stream);
}

extern "C" int smpq_maxpool_quantize(const float* x, int n, int h, int w, int c, const float* absmax, int limbs,
                                     int8_t* out, float* out_f32, smpq_stream_t stream) {
  if (!x || !absmax || !out || n <= 0 || h <= 0 || w <= 0 || c <= 0 || c % 4 != 0)
    return fail(SMPQ_E_INVALID, "smpq_maxpool_quantize: bad arguments");
  const int ho = (h + 2 - 3) / 2 + 1, wo = (w + 2 - 3) / 2 + 1;
  const long long plane = (long long)n * ho * wo * c;
  const dim3 grid((unsigned)grid_for(plane / 4));
  hipStream_t s = (hipStream_t)stream;
  switch (limbs) {
    case 1: hipLaunchKernelGGL(maxpool_quantize_kernel<1>, grid, dim3(256), 0, s, x, n, h, w, c, ho, wo, absmax, out, plane, out_f32); break;
    case 2: hipLaunchKernelGGL(maxpool_quantize_kernel<2>, grid, dim3(256), 0, s, x, n, h, w, c, ho, wo, absmax, out, plane, out_f32); break;
    case 3: hipLaunchKernelGGL(maxpool_quantize_kernel<3>, grid, dim3(256), 0, s, x, n, h, w, c, ho, wo, absmax, out, plane, out_f32); break;
    default: return fail(SMPQ_E_INVALID, "smpq_maxpool_quantize: limbs must be 1, 2 or 3");
  }
  return check_hip(hipGetLastError(), "maxpool_quantize_kernel launch");
}

extern "C" int smpq_maxpool_limbs(const int8_t* x, int n, int h, int w, int c, int limbs, int8_t* out,
                                  smpq_stream_t stream) {
  if (!x || !out || n <= 0 || h <= 0 || w <= 0 || c <= 0 || (c % 16) != 0)
    return fail(SMPQ_E_INVALID, "smpq_maxpool_limbs: bad arguments (c % 16 == 0)");
  const int ho = (h + 2 - 3) / 2 + 1, wo = (w + 2 - 3) / 2 + 1;
  const long long iplane = (long long)n * h * w * c, oplane = (long long)n * ho * wo * c;
  const long long total = (long long)n * ho * wo * (c / 16);
  if (total > 0x7fffff00LL) return fail(SMPQ_E_SHAPE, "smpq_maxpool_limbs: too many outputs");
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  switch (limbs) {
    case 1: hipLaunchKernelGGL(maxpool_limbs_kernel<1>, grid, dim3(256), 0, s, x, n, h, w, c, ho, wo, iplane, out, oplane); break;
    case 2: hipLaunchKernelGGL(maxpool_limbs_kernel<2>, grid, dim3(256), 0, s, x, n, h, w, c, ho, wo, iplane, out, oplane); break;
    case 3: hipLaunchKernelGGL(maxpool_limbs_kernel<3>, grid, dim3(256), 0, s, x, n, h, w, c, ho, wo, iplane, out, oplane); break;
    default: return fail(SMPQ_E_INVALID, "smpq_maxpool_limbs: limbs must be 1, 2 or 3");
  }
  return check_hip(hipGetLastError(), "maxpool_limbs_kernel launch");
}

extern "C" int smpq_act_absmax(const float* x, int n, int64_t per_image, float* absmax,
                               smpq_stream_t stream) {
  if (!x || !absmax || n <= 0 || per_image <= 0)
    return fail(SMPQ_E_INVALID, "smpq_act_absmax: bad arguments");
  // ~4 workgroups per CU in total, few atomics per image (no contention on one address)
  int chunks = (1024 + n - 1) / n;
  const int maxc = (int)((per_image / 4 + 255) / 256);
  if (chunks > maxc) chunks = maxc;
  if (chunks < 1) chunks = 1;
  hipLaunchKernelGGL(absmax_kernel, dim3(chunks, n), dim3(256), 0, (hipStream_t)stream, x, per_image,
                     absmax);
  return check_hip(hipGetLastError(), "absmax_kernel launch");
}

extern "C" int smpq_debug_mfma_i8(const int8_t* a, const int8_t* b, int32_t* c, smpq_stream_t stream) {
  if (!a || !b || !c) return fail(SMPQ_E_INVALID, "smpq_debug_mfma_i8: null pointer");
  hipLaunchKernelGGL(debug_mfma_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, c);
  return check_hip(hipGetLastError(), "debug_mfma_kernel launch");
}

extern "C" int smpq_conv2d_pair_supported(int cin, int cout1, int cout2, int limbs) {
  return cout2 > 0 && resident_pair_supported(cin, cout1, cout2, limbs) ? 1 : 0;
}

extern "C" int smpq_conv2d_chain_supported(int cin, int cout1, int cout2, int limbs) {
  return resident_pair_supported(cin, cout1, cout2, limbs) ? 1 : 0;
}

extern "C" int smpq_conv2d_chain_ds_supported(int cin, int cout1, int ds_cin, int ds_stride, int limbs) {
  return resident_chain_ds_supported(cin, cout1, ds_cin, ds_stride, limbs) ? 1 : 0;
}

extern "C" int smpq_conv2d_chain_fwd(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                                     const int8_t* codes1, const int32_t* offset1, int cout1, const float* col_scale1,
                                     const float* col_shift1, const int8_t* residual_q, float residual_range,
                                     const int8_t* ds_xq, const float* ds_x_absmax, int ds_h, int ds_w,
                                     int ds_cin, int ds_stride, const int8_t* ds_codes,
                                     int ds_wlimbs, const float* ds_col_scale, const float* ds_col_shift,
                                     float ds_range, int8_t* yq1, float yq1_range, const float* y1_absmax,
                                     const int8_t* codes2, int cout2, const float* col_scale2,
                                     const float* col_shift2, int8_t* yq2, float yq2_range, int32_t* overflow,
                                     smpq_stream_t stream) {
  constexpr int limbs = 3;
  if (!yq1 || (!residual_q) == (!ds_xq)) return fail(SMPQ_E_INVALID, "smpq_conv2d_chain_fwd: yq1 and exactly one "
                                                                      "identity source (residual_q or ds_xq)");
  if (ds_xq && (!ds_x_absmax || !ds_codes || ds_wlimbs != 3 || !(ds_range > 0.f)))
    return fail(SMPQ_E_INVALID, "smpq_conv2d_chain_fwd: the fused downsample needs its input range, 3-limb "
                                "weights and a positive output range");
  if (codes2 && (!yq2 || !y1_absmax)) return fail(SMPQ_E_INVALID, "smpq_conv2d_chain_fwd: null pointer");
  ConvArgs a, b, d;
  // conv3; with a fused downsample its residual is the downsample's codes at scale ds_range / QMAX
  int rc = conv_args_q(xq, x_absmax, n, h, w, cin, codes1, 1, offset1, cout1, 1, 1, 1, 0, col_scale1, col_shift1,
                       nullptr, 1, limbs, nullptr, nullptr, yq1, yq1_range, overflow, residual_q, residual_range, a);
  if (rc) return rc;
  if (ds_xq) {
    a.res_scale = ds_range / 8323072.f;
    // the downsample as its own launch would run it (its output quantizer: yq1 stands in for the
    // planes it would write; the chain never writes them)
    rc = conv_args_q(ds_xq, ds_x_absmax, n, ds_h, ds_w, ds_cin, ds_codes, 3, nullptr, cout1, 1, 1, ds_stride, 0,
                     ds_col_scale, ds_col_shift, nullptr, 0, limbs, nullptr, nullptr, yq1, ds_range, overflow, nullptr,
                     0.f, d);
    if (rc) return rc;
  }
  if (codes2) {
    rc = conv_args_q(yq1, y1_absmax, n, h, w, cout1, codes2, 1, nullptr, cout2, 1, 1, 1, 0, col_scale2, col_shift2,
                     nullptr, 1, limbs, nullptr, nullptr, yq2, yq2_range, overflow, nullptr, 0.f, b);
    if (rc) return rc;
  }
  long long big = (long long)limbs * a.M * (cout1 > cin ? cout1 : cin);
  if (ds_xq && (long long)limbs * d.plane > big) big = (long long)limbs * d.plane;
  if (big > 0x7fffff00LL) return fail(SMPQ_E_SHAPE, "smpq_conv2d_chain_fwd: a limb plane of 2 GiB or more");
  return launch_resident_chain(a, codes2 ? &b : nullptr, ds_xq ? &d : nullptr, limbs, (hipStream_t)stream);
}

extern "C" int smpq_conv2d_pair_fwd(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                                    const int8_t* codes1, int cout1, const float* col_scale1,
                                    const float* col_shift1, const int8_t* residual_q, float residual_range,
                                    int8_t* yq1, float yq1_range, const float* y1_absmax, const int8_t* codes2,
                                    int cout2, const float* col_scale2, const float* col_shift2, int8_t* yq2,
                                    float yq2_range, int32_t* overflow, smpq_stream_t stream) {
  if (!residual_q || !codes2) return fail(SMPQ_E_INVALID, "smpq_conv2d_pair_fwd: null pointer");
  return smpq_conv2d_chain_fwd(xq, x_absmax, n, h, w, cin, codes1, nullptr, cout1, col_scale1, col_shift1, residual_q,
                               residual_range, nullptr, nullptr, 0, 0, 0, 0, nullptr, 0, nullptr, nullptr, 0.f, yq1, yq1_range,
                               y1_absmax, codes2, cout2, col_scale2, col_shift2, yq2, yq2_range, overflow, stream);
}
