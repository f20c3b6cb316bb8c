// Shared by the two quantized-conv kernels (conv.hip: register-staged, any cin; conv_glds.hip:
// LDS-DMA staged, cin % 64 == 0). Not part of the public ABI.
#pragma once

#include "common.h"

namespace smpq {

constexpr int kKStep = 64;  // K per MFMA (i8 16x16x64)

struct ConvArgs {
  const int8_t* xq;       // [L][n][h][w][cin] activation limb planes
  long long plane;        // elements per activation plane
  const float* x_absmax;  // [n]
  const int8_t* codes;    // [LW][cout][K] weight limb planes
  long long wplane;       // elements per weight plane (cout*K)
  const int32_t* w_off;   // [cout] (LW == 1 only) or NULL
  const float* col_scale;
  const float* col_shift;
  const float* residual;  // fp32 NHWC residual, or NULL
  const int8_t* res_q;    // [L][M][cout] residual limb planes (static range), or NULL
  float res_scale;        // residual value = res_scale * sum_l 256^l digit_l
  float* y;               // fp32 NHWC output, or NULL
  float* y_absmax;
  int8_t* yq;             // [L][M][cout] output limb planes (static range), or NULL
  float yq_inv;           // QMAX / range of the output quantizer
  int32_t* overflow;      // set to 1 when |y| exceeded the static range (then clamped)
  int n, h, w, cin, cout, kh, kw, stride, pad, ho, wo;
  int M, K, ksteps, cchunks;
  int relu, has_offset;
  float inv_qmax;
  int s2d;  // space-to-depth stem (smpq_stem_conv_s2d_q): cin 16, 4 x 4 taps, K step = one tap row
};

template <int L>
__device__ __host__ constexpr float act_qmax() {
  return L == 1 ? 127.f : (L == 2 ? 32512.f : 8323072.f);
}

template <int L>
__device__ __forceinline__ void split_limbs(int q, int* d) {
  // balanced base-256 digits, each in [-128, 127]
#pragma unroll
  for (int l = 0; l < L - 1; ++l) {
    const int lo = ((q + 128) & 255) - 128;
    d[l] = lo;
    q = (q - lo) >> 8;
  }
  d[L - 1] = q;
}

// Epilogue arithmetic shared by both kernels, written with explicit rounding so that every tile
// configuration of either kernel produces bitwise-identical outputs (no compiler contraction).
// v = sum_s fl(acc_s) * 256^(SMIN+s), accumulated in fp32 from the lowest limb weight up.
__device__ __forceinline__ float affine(float v, float rscale, float cscale, float cshift) {
  return __fmaf_rn(v, __fmul_rn(rscale, cscale), cshift);
}

// LDS-DMA staged kernel (conv_glds.hip)
int glds_num_cfgs();
void glds_cfg_info(int cfg, int* bm, int* bn, int* threads);
int glds_cfg_bk(int cfg);
bool glds_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs);
int launch_glds(int cfg, int limbs, int wlimbs, const ConvArgs& a, hipStream_t s);

}  // namespace smpq
