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
  int nt_store;  // limb-plane output stores with the non-temporal policy (outputs too big for the MALL)
  // x / d = (x * mul) >> shr for 0 <= x < 2^31 (fast_div_init): output pixels per image, output
  // width, and (set by the tile launcher) channel tiles
  unsigned hw_mul, wo_mul, ntc_mul;
  int hw_shr, wo_shr, ntc_shr;
  float inv_qmax;
  int s2d;  // space-to-depth stem (smpq_stem_conv_s2d_q): cin 16, 4 x 4 taps, K step = one tap row
  // codes in the K-major layout [LW][K/64][cout][64] (smpq_conv2d_fwd_q_km; LDS-DMA kernel only):
  // the 64-B K slices of 16 consecutive output channels are one contiguous KiB, so every weight
  // DMA piece is whole cache lines instead of 16 half lines
  int w_kmajor;
};

// Division by a runtime constant d >= 1 for numerators in [0, 2^31): p = 31 + ceil(log2 d),
// mul = ceil(2^p / d) (< 2^32), x / d == (x * mul) >> p. Two instructions instead of the ~20 of a
// generic 32-bit division (the conv prologues decompose pixel indices with it).
inline void fast_div_init(int d, unsigned& mul, int& shr) {
  int l = 0;
  while ((1LL << l) < (long long)d) ++l;
  shr = 31 + l;
  mul = (unsigned)(((1ULL << shr) + (unsigned long long)d - 1) / (unsigned long long)d);
}
__device__ __forceinline__ int fast_div(int x, unsigned mul, int shr) {
  return (int)(((unsigned long long)(unsigned)x * mul) >> shr);
}

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
int glds_default_cfg(const ConvArgs& a, int limbs, int wlimbs);
bool glds_is_halo(int cfg);

// halo-patch 3x3 kernel (conv_halo.hip); its tile configs follow the LDS-DMA ones in the C-ABI's
// numbering (cfg = glds count + halo index)
int halo_num_cfgs();
void halo_cfg_info(int cfg, int* bm, int* bn, int* threads);
bool halo_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs);
int launch_halo(int cfg, int limbs, int wlimbs, const ConvArgs& a, hipStream_t s);

// weight-stationary 1x1 tiles (conv_resident.hip); their configs follow the halo ones
int resident_num_cfgs();
void resident_cfg_info(int cfg, int* bm, int* bn, int* threads);
bool resident_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs);
int launch_resident(int cfg, int limbs, int wlimbs, const ConvArgs& a, hipStream_t s);
bool glds_is_resident(int cfg);
// the Bottleneck tail chains: conv3 (+ fused downsample) (-> next conv1) (smpq_conv2d_chain_fwd)
bool resident_pair_supported(int cin, int cout1, int cout2, int limbs);
bool resident_chain_ds_supported(int cin, int cout1, int ds_cin, int ds_stride, int limbs);
int launch_resident_chain(const ConvArgs& a, const ConvArgs* b, const ConvArgs* d, int limbs, hipStream_t s);

// The 4 codes (channels 0..3) held by one dword per limb plane, w[l] = the 4 balanced digits of
// limb l: q = sum_l d_l 256^l. With u_l = d_l + 128 (byte ^ 0x80) for the low limbs,
// q = sext24(u0 | u1 << 8 | d2 << 16) - 0x8080 (L = 3), sext16(u0 | d1 << 8) - 0x80 (L = 2).
template <int L>
__device__ __forceinline__ void decode4(const unsigned* w, int* q) {
  if constexpr (L == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) q[r] = __builtin_amdgcn_sbfe((int)w[0], 8 * r, 8);
  } else if constexpr (L == 2) {
    const unsigned x0 = w[0] ^ 0x80808080u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned b = __builtin_amdgcn_perm(w[1], x0, (unsigned)r | ((unsigned)(r + 4) << 8) | 0x0c0c0000u);
      q[r] = __builtin_amdgcn_sbfe((int)b, 0, 16) - 0x80;
    }
  } else {
    const unsigned x0 = w[0] ^ 0x80808080u, x1 = w[1] ^ 0x80808080u;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // [u0(2h), u1(2h), u0(2h+1), u1(2h+1)]
      const unsigned a = __builtin_amdgcn_perm(x1, x0, h == 0 ? 0x05010400u : 0x07030602u);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int r = 2 * h + e;
        const unsigned sel = (e == 0 ? 0x0100u : 0x0302u) | ((unsigned)(4 + r) << 16) | 0x0c000000u;
        const unsigned b = __builtin_amdgcn_perm(w[2], a, sel);
        q[r] = __mul24((int)b, 1) - 0x8080;  // 24-bit operand: sign from bit 23 (v_mad_i32_i24)
      }
    }
  }
}

// The digit dwords of 4 clamped codes (inverse of decode4): with Q = q + 0x8080 (L = 3) / q + 0x80
// (L = 2), digit l of q is byte l of Q, xor 0x80 for every limb below the top one.
template <int L>
__device__ __forceinline__ void encode4(const int* q, unsigned* w) {
  constexpr int bias = L == 3 ? 0x8080 : (L == 2 ? 0x80 : 0);
  const unsigned Q0 = (unsigned)(q[0] + bias), Q1 = (unsigned)(q[1] + bias), Q2 = (unsigned)(q[2] + bias),
                 Q3 = (unsigned)(q[3] + bias);
  const unsigned a = __builtin_amdgcn_perm(Q1, Q0, 0x05010400u);  // [Q0.b0, Q1.b0, Q0.b1, Q1.b1]
  const unsigned b = __builtin_amdgcn_perm(Q3, Q2, 0x05010400u);
  constexpr unsigned flip = 0x80808080u;
  w[0] = __builtin_amdgcn_perm(b, a, 0x05040100u) ^ (L > 1 ? flip : 0u);
  if constexpr (L >= 2) w[1] = __builtin_amdgcn_perm(b, a, 0x07060302u) ^ (L > 2 ? flip : 0u);
  if constexpr (L >= 3) {
    const unsigned c = __builtin_amdgcn_perm(Q1, Q0, 0x07030602u);  // [Q0.b2, Q1.b2, Q0.b3, Q1.b3]
    const unsigned d = __builtin_amdgcn_perm(Q3, Q2, 0x07030602u);
    w[2] = __builtin_amdgcn_perm(d, c, 0x05040100u);
  }
}

}  // namespace smpq
