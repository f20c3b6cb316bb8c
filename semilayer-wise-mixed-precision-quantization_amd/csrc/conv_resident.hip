// Weight-stationary 1x1 conv tiles for gfx950 (round 6; tile kind SMPQ_TILE_RESIDENT1X1): 1x1 convs
// whose epilogue only emits the next conv's limb planes (optionally adding a limb-plane residual)
// and whose weights — for a slab of output channels — fit in the VGPRs of a workgroup. In the R50
// forward: the 1x1 convs of the Bottlenecks and the four downsample convs
// (resnet.py:188-192, conv1x1 + BN, 24-bit fixed-point weights: 3 weight limbs, 6 MFMA passes),
// where the LDS-DMA kernel spends most of its operand staging on the weights (a 128 x 32 tile of
// the 64 -> 256 downsample re-stages 24 KB of weight limbs for 6 KB of activations, 50,176 times per
// 256 images; the strided 256 -> 512 / 512 -> 1024 ones 3 bytes of weights per K element and output
// channel).
//
// A persistent workgroup (4 waves) owns one slab of BN = 64 CW output channels (wave w: channels
// 16 CW w .. 16 CW (w + 1) - 1 of the slab) and loads the slab's weight limbs for the whole K ONCE,
// straight into VGPRs (LW x KC x CW A fragments per wave: each lane's 16 bytes are one buffer load).
// It then walks pixel tiles of BP pixels (tiles t0, t0 + stride, ...): the activation tile of the
// next tile ([L][BP][K] bytes, K = 64 KC, rows swizzled by 16-B chunk) arrives by LDS-DMA into the
// other of two stages while this tile's MFMAs and epilogue run. The epilogue is the LDS-DMA kernel's
// lean static-range epilogue (lean_quad: limb recombination, folded BN, optional ReLU, rounding,
// clamp, digit encode), staged in LDS as a [L][BP][BN] tile and copied out row-major. Integer
// accumulation is exact and the epilogue is the same function, so the outputs and the overflow flag
// are bitwise those of every other tile config (tests/test_gpu_resident.py). A limb-plane residual
// (conv3 + the block input, resnet.py:111-113) arrives by LDS-DMA with the activations, one tile
// ahead, as a [L][BP][BN] tile in the output tile's layout. The slabs of a conv
// walk the same pixel tiles in the same order, so a tile's activations are read from HBM once and
// from L2 / MALL by the other slabs.
//
// Chained pair (CW2 > 0; smpq_conv2d_pair_fwd, round 6): a Bottleneck's conv3 (+ limb-plane identity,
// ReLU) followed by the NEXT block's conv1 (1x1, ReLU), which reads nothing but conv3's output
// (resnet.py:108-113 then :99-101). One slab holds all of conv3's channels, so the staged output tile
// [L][BP][BN] is exactly conv1's activation tile for the same pixels: after it is written, its limb
// rows are read straight back as conv1's MFMA B fragments (conv1's weights: a second set of VGPR
// fragments), and conv1's own [L][BP][64 CW2] tile is staged and copied out beside it. Both outputs
// are bitwise those of the two separate launches (the same codes, the same epilogue); conv1's
// activation read from HBM disappears.
//
// Fused downsample (LWD > 0): in the first block of a stage the identity conv3 adds is the
// downsample's output (resnet.py:108-113 with :188-192), written as limb planes by one launch and
// read back by conv3. Where the downsample is a 1x1 / stride-1 conv over the same pixels and K as
// conv3 (the R50 layer1 block 0: 64 -> 256 at 56^2), its activation tile arrives beside conv3's, its
// 24-bit fixed-point weight limbs sit in VGPRs too, and its epilogue's clamped codes (the values its
// own launch would have written) feed conv3's residual directly: both HBM round trips of the
// downsample output and its launch disappear; the overflow flag covers both outputs.
//
// Weight offsets (OFF; exact-code channels whose codes sit off-centre): acc_l += offset_c * (sum of
// the pixel's limb-l digits), the digit sums taken with v_dot4 on the B fragments — the LDS-DMA
// kernel's exact integer correction.
#include "conv_common.h"
#include "lds_dma.h"

namespace smpq {

namespace {

struct ResCfg {
  int cw, wp;   // 16-channel fragments per wave (slab = 64 cw channels), 16-pixel fragments per tile
  int kc_mask;  // bit k: K = 64 k supported (chunks of 64 bytes per activation row)
};
constexpr ResCfg kRes[] = {
    {4, 2, 1 << 1},                                // 0: slab 256, 32 px, K 64 (the 64 -> 256 downsample)
    {4, 1, (1 << 1) | (1 << 2) | (1 << 4)},        // 1: slab 256, 16 px, K 64..256 (the expansions)
    {1, 1, 0x10116},                               // 2: slab 64, 16 px, K 64..1024 (strided ds, reductions)
    {2, 1, 0x10116},                               // 3: slab 128, 16 px, K 64..1024
    // (slab 64 x 32 px at K 256 / 512 measured 1.1-2.1x slower than 16 px: one workgroup per CU)
};
// the weight fragments a wave holds: at most 32 (128 VGPRs)
constexpr bool res_fits(int lw, int kc, int cw) { return lw * kc * cw <= 32; }
constexpr int kNumRes = sizeof(kRes) / sizeof(kRes[0]);
constexpr int kResThreads = 256;
// Per-image input scales staged in LDS at the start (up to kNTab images; more: read from memory).
// A global load inside the tile loop would end in an s_waitcnt vmcnt the compiler places for it —
// which also waits for the next tile's activation DMA and the copy-out stores issued before it,
// serialising every tile on a full memory round trip.
constexpr int kNTab = 256;

// the 16-B chunk c of activation row r is stored at chunk ach<KC>(c, r): conflict-free DMA writes and
// fragment reads (16 rows, chunk fixed per lane group) for 64-B rows (KC = 1, the LDS-DMA kernel's
// swizzle) and for rows of 16 or more chunks (KC >= 4: XOR by the row's low 4 bits)
template <int KC>
__device__ __forceinline__ int ach(int c, int r) {
  if constexpr (KC == 1) return c ^ swz<64>(r & 15);
  else if constexpr (KC == 2) return c ^ swz<128>(r);
  else return c ^ (r & 15);
}

template <int L, int LW, int KC, int CW, int WP, bool RES, int CW2 = 0, int LWD = 0, bool OFF = false,
          int KCD = KC>
struct ResShape {
  static constexpr int SMIN = (L + LW - 4) > 0 ? (L + LW - 4) : 0;
  static constexpr int NACC = L + LW - 1 - SMIN;
  static constexpr int BN = 64 * CW, BP = 16 * WP, K = 64 * KC;
  static constexpr int ATILE = L * BP * K;                     // activation tile bytes
  static constexpr int ATILE_D = LWD > 0 ? L * BP * 64 * KCD : 0;  // the fused downsample's tile
  static constexpr int ASTAGE = ATILE + ATILE_D;
  static constexpr int OTILE = L * BP * BN;  // output (and residual) tile bytes
  static constexpr int OTILE2 = L * BP * 64 * CW2;  // the chained conv's output tile
  static constexpr int LDS = 2 * ASTAGE + (RES ? 3 : 1) * OTILE + OTILE2;
  // VGPRs: weights (+ the chained conv's) + accumulators + one chunk's B fragments + addressing /
  // epilogue (~40)
  // (+ the fused downsample's accumulators and epilogue constants; the offsets and digit sums: the
  // compiler's counts, tools/ resource usage, need this much margin to stay spill-free)
  static constexpr int NACC_D = LWD > 0 ? L + LWD - 1 - ((L + LWD - 4) > 0 ? (L + LWD - 4) : 0) : 0;
  static constexpr int REGS = 4 * (LW * KC * CW + CW * CW2 + LWD * KCD * CW + NACC * CW * WP + L * WP) + 40 +
                              (LWD > 0 ? 8 * CW + 4 * CW * WP + (CW2 > 0 ? 4 * NACC_D * CW * WP : 0) : 0) +
                              (OFF ? 8 * CW + L * WP : 0) + (CW2 > 0 ? 8 * CW2 + 4 * L * CW2 * WP : 0);
  // workgroups per CU (1 wave per SIMD each; past 256 the accumulators move to AGPRs)
  static constexpr int MINW_R = REGS <= 120 ? 4 : (REGS <= 152 ? 3 : (REGS <= 240 ? 2 : 1));
  // + the per-image input scales (x_absmax / QMAX) of each conv, staged once (kNTab images)
  static constexpr int NTABS = 1 + (LWD > 0 ? 1 : 0) + (CW2 > 0 ? 1 : 0);
  static constexpr int LDS_TOTAL = LDS + NTABS * kNTab * 4;
  static constexpr int MINW_L = (160 * 1024) / LDS_TOTAL;
  static constexpr int MINW = MINW_R < MINW_L ? MINW_R : MINW_L;
};

template <int L, int LW, int KC, int CW, int WP, bool RELU, bool RES, int MINW, int CW2 = 0, bool OFF = false,
          int LWD = 0, int KCD = KC>
__global__ __launch_bounds__(kResThreads, MINW) void qconv_resident_kernel(ConvArgs a, ConvArgs b, ConvArgs d,
                                                                           int ntiles, int nslabs) {
  using S = ResShape<L, LW, KC, CW, WP, RES, CW2, LWD, OFF, KCD>;
  constexpr int SMIN = S::SMIN, NACC = S::NACC, BN = S::BN, BP = S::BP, K = S::K, ASTAGE = S::ASTAGE;
  constexpr int ATILE = S::ATILE;
  static_assert(!OFF || (LW == 1 && SMIN == 0), "weight offsets: exact codes only");
  static_assert(!(RES && LWD > 0), "one residual source");
  constexpr int SMIN_D = (L + LWD - 4) > 0 ? (L + LWD - 4) : 0, NACC_D = LWD > 0 ? L + LWD - 1 - SMIN_D : 1;
  constexpr int CH = K / 16;       // 16-B chunks per activation row
  constexpr int RP = 1024 / K;     // activation rows per 1-KiB DMA piece
  constexpr int APIECES = L * BP / RP;
  constexpr float qmax = act_qmax<L>();
  extern __shared__ __attribute__((aligned(1024))) int8_t lds[];  // 2 act stages, output tile, 2 residual tiles
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, grp = lane >> 4;
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  int8_t* const otile = lds + 2 * ASTAGE;
  constexpr int OTILE = S::OTILE;
  const unsigned rtile0 = lds0 + 2 * ASTAGE + OTILE;  // residual tile of stage s at rtile0 + s OTILE
  // per-image scales: [0] this conv's input, [1] the fused downsample's, [2] the chained conv's
  float* const rtab = reinterpret_cast<float*>(lds + S::LDS);
  const bool tab_ok = a.n <= kNTab;
  if (tab_ok) {
    for (int i = threadIdx.x; i < a.n; i += kResThreads) {
      rtab[i] = a.x_absmax[i] * a.inv_qmax;
      if constexpr (LWD > 0) rtab[kNTab + i] = d.x_absmax[i] * d.inv_qmax;
      if constexpr (CW2 > 0) rtab[(S::NTABS - 1) * kNTab + i] = b.x_absmax[i] * b.inv_qmax;
    }
  }  // (visible to every wave after the tile loop's first barrier)
  const int slab = blockIdx.x % nslabs;
  const int n0 = slab * BN;
  const int tstride = gridDim.x / nslabs;

  // ---- the slab's weight limbs -> VGPRs once: A fragment (lw, kc, i) of lane (g, p) = the 16
  // bytes of K chunk 4 kc + g of output channel n0 + 16 (CW wave + i) + p
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.codes), 0, (int)(LW * a.wplane), 0x00020000);
  v4i wa[LW][KC][CW];
#pragma unroll
  for (int lw = 0; lw < LW; ++lw)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int i = 0; i < CW; ++i) {
        const int row = n0 + (wave * CW + i) * 16 + frow;
        const unsigned off = a.w_kmajor ? (unsigned)(kc * a.cout * 64 + row * 64 + 16 * grp)
                                        : (unsigned)(row * K + kc * 64 + 16 * grp);
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(wrs, off, (unsigned)(lw * a.wplane), 0);
        wa[lw][kc][i] = v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
      }
  // the chained conv's weights (CW2 > 0: exact codes, K = BN = this conv's output channels, KC2 = CW
  // chunks of 64; wave w: its output channels 16 (CW2 w + i) + p)
  constexpr int KC2 = CW2 > 0 ? CW : 0, BN2 = 64 * CW2;
  v4i wb[KC2 > 0 ? KC2 : 1][CW2 > 0 ? CW2 : 1];
  if constexpr (CW2 > 0) {
    const auto wrs2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(b.codes), 0, (int)b.wplane, 0x00020000);
#pragma unroll
    for (int kc = 0; kc < KC2; ++kc)
#pragma unroll
      for (int i = 0; i < CW2; ++i) {
        const int row = (wave * CW2 + i) * 16 + frow;
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(wrs2, (unsigned)(row * BN + kc * 64 + 16 * grp), 0u, 0);
        wb[kc][i] = v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
      }
  }
  // the fused downsample's weight limbs (LWD > 0: same slab, K = 64 KCD)
  constexpr int KD = 64 * KCD;
  v4i wd[LWD > 0 ? LWD : 1][LWD > 0 ? KCD : 1][LWD > 0 ? CW : 1];
  if constexpr (LWD > 0) {
    const auto wrsd = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(d.codes), 0, (int)(LWD * d.wplane), 0x00020000);
#pragma unroll
    for (int lw = 0; lw < LWD; ++lw)
#pragma unroll
      for (int kc = 0; kc < KCD; ++kc)
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          const int row = n0 + (wave * CW + i) * 16 + frow;
          const unsigned off = d.w_kmajor ? (unsigned)(kc * d.cout * 64 + row * 64 + 16 * grp)
                                          : (unsigned)(row * KD + kc * 64 + 16 * grp);
          const v4u v = __builtin_amdgcn_raw_buffer_load_b128(wrsd, off, (unsigned)(lw * d.wplane), 0);
          wd[lw][kc][i] = v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
        }
  }

  // ---- activation DMA: piece = RP pixel rows x K bytes of one limb; lane -> (row, physical chunk)
  const int prow = lane / CH, pphys = lane % CH;
  const v4i xrs = make_rsrc(a.xq, (long long)L * a.plane);
  const v4i xrsd = make_rsrc(LWD > 0 ? d.xq : nullptr, LWD > 0 ? (long long)L * d.plane : 0);
  const int hw_out = a.ho * a.wo;
  // the fused downsample's tile: the same output pixels, sampled from its own input (h, w, stride,
  // K = KD); piece = RPD rows x KD bytes
  constexpr int CHD = KD / 16, RPD = 1024 / KD, DPIECES = LWD > 0 ? L * BP / RPD : 0;
  const int prowd = lane / CHD, pphysd = lane % CHD;
  auto issue_acts = [&](int t, int stage) {
    for (int p = wave; p < APIECES; p += 4) {
      const int l = p / (BP / RP), r = (p % (BP / RP)) * RP + prow;  // tile row (pixel) of this lane
      const int m = t * BP + r;
      unsigned src = kOOB;
      if (m < a.M) {
        const int img = fast_div(m, a.hw_mul, a.hw_shr);
        const int rem = m - img * hw_out;
        const int oh = fast_div(rem, a.wo_mul, a.wo_shr), ow = rem - oh * a.wo;
        src = (unsigned)(((img * a.h + oh * a.stride) * a.w + ow * a.stride) * K + 16 * ach<KC>(pphys, r));
      }
      dma16(lds0 + stage * ASTAGE + p * 1024, xrs, src, __builtin_amdgcn_readfirstlane((unsigned)((long long)l * a.plane)));
    }
    if constexpr (LWD > 0) {
      for (int p = wave; p < DPIECES; p += 4) {
        const int l = p / (BP / RPD), r = (p % (BP / RPD)) * RPD + prowd;
        const int m = t * BP + r;
        unsigned src = kOOB;
        if (m < a.M) {
          const int img = fast_div(m, a.hw_mul, a.hw_shr);
          const int rem = m - img * hw_out;
          const int oh = fast_div(rem, a.wo_mul, a.wo_shr), ow = rem - oh * a.wo;
          src = (unsigned)(((img * d.h + oh * d.stride) * d.w + ow * d.stride) * KD + 16 * ach<KCD>(pphysd, r));
        }
        dma16(lds0 + stage * ASTAGE + ATILE + p * 1024, xrsd, src,
              __builtin_amdgcn_readfirstlane((unsigned)((long long)l * d.plane)));
      }
    }
  };
  // the residual tile [L][BP][BN] of tile t (RES): piece = 1024 / BN rows x BN bytes of one limb, 16-B
  // chunk c of tile row r at c ^ swze<BN>(r & 15) (the output tile's layout: the epilogue reads it
  // with the same addressing)
  const long long oplane = (long long)a.M * a.cout;
  const v4i rrs = make_rsrc(a.res_q, RES ? (long long)L * oplane : 0);
  auto issue_res = [&](int t, int stage) {
    if constexpr (RES) {
      constexpr int RROWS = 1024 / BN, RCPR = BN / 16, RPIECES = L * BP / RROWS;
      const int rrow = lane / RCPR, rpc = lane % RCPR;
      for (int p = wave; p < RPIECES; p += 4) {
        const int l = p / (BP / RROWS), rt = (p % (BP / RROWS)) * RROWS + rrow;
        const int m = t * BP + rt;
        const unsigned src = m < a.M ? (unsigned)((long long)m * a.cout + n0 + 16 * (rpc ^ swze<BN>(rt & 15))) : kOOB;
        dma16(rtile0 + stage * OTILE + p * 1024, rrs, src, __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane)));
      }
    }
  };
  int t = blockIdx.x / nslabs;
  if (t < ntiles) {
    issue_acts(t, 0);
    issue_res(t, 0);
  }

  // ---- epilogue constants of this lane's channels -----------------------------------------------
  const float inv = a.yq_inv;
  float csq[CW][4], shq[CW][4];
#pragma unroll
  for (int i = 0; i < CW; ++i) {
    const int c = n0 + (wave * CW + i) * 16 + 4 * grp;
    const float4 cs = *reinterpret_cast<const float4*>(a.col_scale + c);
    const float4 csh = *reinterpret_cast<const float4*>(a.col_shift + c);
    csq[i][0] = cs.x * inv, csq[i][1] = cs.y * inv, csq[i][2] = cs.z * inv, csq[i][3] = cs.w * inv;
    shq[i][0] = csh.x * inv, shq[i][1] = csh.y * inv, shq[i][2] = csh.z * inv, shq[i][3] = csh.w * inv;
  }
  const float lo = RELU ? 0.f : -qmax;
  const float rsq = a.res_scale * inv;
  // the fused downsample's epilogue constants, and this lane's weight offsets
  float csqd[LWD > 0 ? CW : 1][4], shqd[LWD > 0 ? CW : 1][4];
  if constexpr (LWD > 0) {
    const float invd = d.yq_inv;
#pragma unroll
    for (int i = 0; i < CW; ++i) {
      const int c = n0 + (wave * CW + i) * 16 + 4 * grp;
      const float4 cs = *reinterpret_cast<const float4*>(d.col_scale + c);
      const float4 csh = *reinterpret_cast<const float4*>(d.col_shift + c);
      csqd[i][0] = cs.x * invd, csqd[i][1] = cs.y * invd, csqd[i][2] = cs.z * invd, csqd[i][3] = cs.w * invd;
      shqd[i][0] = csh.x * invd, shqd[i][1] = csh.y * invd, shqd[i][2] = csh.z * invd, shqd[i][3] = csh.w * invd;
    }
  }
  int woff[OFF ? CW : 1][4];
  if constexpr (OFF) {
#pragma unroll
    for (int i = 0; i < CW; ++i) {
      const int4 o = *reinterpret_cast<const int4*>(a.w_off + n0 + (wave * CW + i) * 16 + 4 * grp);
      woff[i][0] = o.x, woff[i][1] = o.y, woff[i][2] = o.z, woff[i][3] = o.w;
    }
  }
  const v4i qrs4 = make_rsrc(a.yq, (long long)L * oplane);
  // the chained conv's epilogue constants, output planes and staged tile
  const float inv2 = CW2 > 0 ? b.yq_inv : 0.f;
  float csq2[CW2 > 0 ? CW2 : 1][4], shq2[CW2 > 0 ? CW2 : 1][4];
  if constexpr (CW2 > 0) {
#pragma unroll
    for (int i = 0; i < CW2; ++i) {
      const int c = (wave * CW2 + i) * 16 + 4 * grp;
      const float4 cs = *reinterpret_cast<const float4*>(b.col_scale + c);
      const float4 csh = *reinterpret_cast<const float4*>(b.col_shift + c);
      csq2[i][0] = cs.x * inv2, csq2[i][1] = cs.y * inv2, csq2[i][2] = cs.z * inv2, csq2[i][3] = cs.w * inv2;
      shq2[i][0] = csh.x * inv2, shq2[i][1] = csh.y * inv2, shq2[i][2] = csh.z * inv2, shq2[i][3] = csh.w * inv2;
    }
  }
  const long long oplane2 = CW2 > 0 ? (long long)a.M * BN2 : 0;
  const v4i qrs4b = make_rsrc(CW2 > 0 ? b.yq : nullptr, (long long)L * oplane2);
  int8_t* const otile2 = lds + 2 * ASTAGE + (RES ? 3 : 1) * OTILE;
  const bool nt = __builtin_amdgcn_readfirstlane(a.nt_store) != 0;
  float vmax = 0.f;

  // copy-out of a staged output tile: BN-byte pixel rows of the slab, 16 B per lane
  auto copy_out = [&](int m0) {
    constexpr int RC = BN / 16, ITEMS = L * BP * RC;
#pragma unroll
    for (int k = 0; k < (ITEMS + kResThreads - 1) / kResThreads; ++k) {
      const int it = threadIdx.x + kResThreads * k;
      if (ITEMS % kResThreads == 0 || it < ITEMS) {
        const int l = it / (BP * RC), rem = it - l * (BP * RC);
        const int rt = rem / RC, c = rem - rt * RC;
        const v4i v = *reinterpret_cast<const v4i*>(otile + l * BP * BN + rt * BN + 16 * (c ^ swze<BN>(rt & 15)));
        const unsigned off = m0 + rt < a.M ? (unsigned)((long long)(m0 + rt) * a.cout + n0 + 16 * c) : kOOB;
        store_limbs16(v4u{(unsigned)v.x, (unsigned)v.y, (unsigned)v.z, (unsigned)v.w}, qrs4, off,
                      __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane)), nt);
      }
    }
    if constexpr (CW2 > 0) {
      constexpr int RC2 = BN2 / 16, ITEMS2 = L * BP * RC2;
#pragma unroll
      for (int k = 0; k < (ITEMS2 + kResThreads - 1) / kResThreads; ++k) {
        const int it = threadIdx.x + kResThreads * k;
        if (ITEMS2 % kResThreads == 0 || it < ITEMS2) {
          const int l = it / (BP * RC2), rem = it - l * (BP * RC2);
          const int rt = rem / RC2, c = rem - rt * RC2;
          const v4i v = *reinterpret_cast<const v4i*>(otile2 + l * BP * BN2 + rt * BN2 + 16 * (c ^ swze<BN2>(rt & 15)));
          const unsigned off = m0 + rt < a.M ? (unsigned)((long long)(m0 + rt) * BN2 + 16 * c) : kOOB;
          store_limbs16(v4u{(unsigned)v.x, (unsigned)v.y, (unsigned)v.z, (unsigned)v.w}, qrs4b, off,
                        __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane2)), nt);
        }
      }
    }
  };
  // Tile loop. The copy-out of tile i-1 and the DMA of tile i+1 are issued at the top of
  // iteration i, before tile i's MFMAs and epilogue, so both fly under a tile's work; raw s_barriers
  // with explicit waits (a __syncthreads would also wait for the stores and the DMA).
  int stage = 0, prev_m0 = -1;
  for (; t < ntiles; t += tstride) {
    const int m0 = t * BP;
    // tile t's activations (and residual) have landed and the last copy-out's stores are done (this
    // wave's); every wave's epilogue writes of the staged output tile and its reads of the other
    // stage are done (lgkmcnt) — after the barrier, every wave's
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (prev_m0 >= 0) copy_out(prev_m0);
    if (t + tstride < ntiles) {
      issue_acts(t + tstride, stage ^ 1);
      issue_res(t + tstride, stage ^ 1);
    }
    const int8_t* as = lds + stage * ASTAGE;
    v4i acc[NACC][CW][WP];
#pragma unroll
    for (int s = 0; s < NACC; ++s)
#pragma unroll
      for (int i = 0; i < CW; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j) acc[s][i][j] = v4i{0, 0, 0, 0};
    v4i accd[NACC_D][LWD > 0 ? CW : 1][LWD > 0 ? WP : 1];
    if constexpr (LWD > 0) {
#pragma unroll
      for (int s = 0; s < NACC_D; ++s)
#pragma unroll
        for (int i = 0; i < CW; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j) accd[s][i][j] = v4i{0, 0, 0, 0};
    }
    // the fused downsample first: its MFMAs, then its epilogue's clamped codes (conv3's residual),
    // so that its accumulators are dead before conv3's are live
    int dq[LWD > 0 ? CW : 1][LWD > 0 ? WP : 1][4];
    if constexpr (LWD > 0) {
#pragma unroll
      for (int kc = 0; kc < KCD; ++kc) {
        v4i fd[L][WP];
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
          for (int j = 0; j < WP; ++j) {
            const int r = j * 16 + frow;
            fd[l][j] = *reinterpret_cast<const v4i*>(as + ATILE + (l * BP + r) * KD + 16 * ach<KCD>(4 * kc + grp, r));
          }
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
          for (int lw = 0; lw < LWD; ++lw) {
            if (l + lw < SMIN_D) continue;
#pragma unroll
            for (int i = 0; i < CW; ++i)
#pragma unroll
              for (int j = 0; j < WP; ++j)
                accd[l + lw - SMIN_D][i][j] =
                    __builtin_amdgcn_mfma_i32_16x16x64_i8(wd[lw][kc][i], fd[l][j], accd[l + lw - SMIN_D][i][j], 0, 0, 0);
          }
      }
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        const int m = m0 + j * 16 + frow;
        const int img = m < a.M ? fast_div(m, a.hw_mul, a.hw_shr) : 0;
        const float rscd = m < a.M ? (tab_ok ? rtab[kNTab + img] : d.x_absmax[img] * d.inv_qmax) : 0.f;
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          v4i accqd[NACC_D];
#pragma unroll
          for (int s2 = 0; s2 < NACC_D; ++s2) accqd[s2] = accd[s2][i][j];
          const int rq0[4] = {0, 0, 0, 0};
          const float md = lean_codes<L, NACC_D, SMIN_D>(accqd, rscd, csqd[i], shqd[i], false, rq0, 0.f, false, -qmax,
                                                         dq[i][j]);
          vmax = m < a.M ? fmaxf(vmax, md) : vmax;
        }
      }
    }
    int rs[OFF ? L : 1][OFF ? WP : 1];  // digit sums of this lane's 16-B slices (OFF)
    if constexpr (OFF) {
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int j = 0; j < WP; ++j) rs[l][j] = 0;
    }
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      v4i fb[L][WP];
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          const int r = j * 16 + frow;
          fb[l][j] = *reinterpret_cast<const v4i*>(as + (l * BP + r) * K + 16 * ach<KC>(4 * kc + grp, r));
        }
      if constexpr (OFF) {
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
          for (int j = 0; j < WP; ++j) {
            int sdig = rs[l][j];
            sdig = __builtin_amdgcn_sdot4(fb[l][j].x, 0x01010101, sdig, false);
            sdig = __builtin_amdgcn_sdot4(fb[l][j].y, 0x01010101, sdig, false);
            sdig = __builtin_amdgcn_sdot4(fb[l][j].z, 0x01010101, sdig, false);
            sdig = __builtin_amdgcn_sdot4(fb[l][j].w, 0x01010101, sdig, false);
            rs[l][j] = sdig;
          }
      }
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int lw = 0; lw < LW; ++lw) {
          if (l + lw < SMIN) continue;  // compile-time: skipped low-digit product (as the LDS-DMA kernel)
#pragma unroll
          for (int i = 0; i < CW; ++i)
#pragma unroll
            for (int j = 0; j < WP; ++j)
              acc[l + lw - SMIN][i][j] =
                  __builtin_amdgcn_mfma_i32_16x16x64_i8(wa[lw][kc][i], fb[l][j], acc[l + lw - SMIN][i][j], 0, 0, 0);
        }
    }
    if constexpr (OFF) {
      // whole-row digit sums (the 4 lane groups hold 16 B each), then acc_l += offset_c * sum_l: the
      // LDS-DMA kernel's integer correction (|offset| < 2^15, |sum| < 2^22: exact 24-bit products)
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          int sdig = rs[l][j];
          sdig += __shfl_xor(sdig, 16, 64);
          sdig += __shfl_xor(sdig, 32, 64);
          rs[l][j] = sdig;
        }
#pragma unroll
      for (int i = 0; i < CW; ++i)
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
          for (int j = 0; j < WP; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[l][i][j][r] += __mul24(woff[i][r], rs[l][j]);
    }
    // every wave's copy-out reads of the staged output tile are done before it is overwritten
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // lean epilogue -> the [L][BP][BN] output tile in LDS (16-B chunk c of tile row r at
    // c ^ swze<BN>(r & 15), as the LDS-DMA kernel's staged tiles)
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const int m = m0 + j * 16 + frow;
      const int img = m < a.M ? fast_div(m, a.hw_mul, a.hw_shr) : 0;
      const float rscale = m < a.M ? (tab_ok ? rtab[img] : a.x_absmax[img] * a.inv_qmax) : 0.f;
#pragma unroll
      for (int i = 0; i < CW; ++i) {
        v4i accq[NACC];
#pragma unroll
        for (int s = 0; s < NACC; ++s) accq[s] = acc[s][i][j];
        const int rt = j * 16 + frow, cc = wave * CW + i;
        int rqv[4] = {0, 0, 0, 0};
        if constexpr (LWD > 0) {  // the downsample's clamped output codes (what its own launch writes)
#pragma unroll
          for (int r = 0; r < 4; ++r) rqv[r] = dq[i][j][r];
        }
        if constexpr (RES) {
          unsigned rw[L];
#pragma unroll
          for (int l = 0; l < L; ++l)
            rw[l] = *reinterpret_cast<const unsigned*>(lds + 2 * ASTAGE + (1 + stage) * OTILE + l * BP * BN + rt * BN +
                                                       16 * (cc ^ swze<BN>(frow)) + 4 * grp);
          decode4<L>(rw, rqv);
        }
        unsigned wq[L];
        const float mm = lean_quad<L, NACC, SMIN>(accq, rscale, csq[i], shq[i], RES || LWD > 0, rqv, rsq, RELU, lo, wq);
        vmax = m < a.M ? fmaxf(vmax, mm) : vmax;
#pragma unroll
        for (int l = 0; l < L; ++l)
          *reinterpret_cast<unsigned*>(otile + l * BP * BN + rt * BN + 16 * (cc ^ swze<BN>(frow)) + 4 * grp) = wq[l];
      }
    }
    if constexpr (CW2 > 0) {
      // the chained conv on the staged tile: every wave's epilogue writes are done (barrier), then
      // its limb rows are the B fragments (row r, K chunk 4 kc + g at (4 kc + g) ^ swze<BN>(r & 15))
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      v4i acc2[L][CW2][WP];
#pragma unroll
      for (int s = 0; s < L; ++s)
#pragma unroll
        for (int i = 0; i < CW2; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j) acc2[s][i][j] = v4i{0, 0, 0, 0};
#pragma unroll
      for (int kc = 0; kc < KC2; ++kc) {
        v4i fb[L][WP];
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
          for (int j = 0; j < WP; ++j) {
            const int r = j * 16 + frow;
            fb[l][j] = *reinterpret_cast<const v4i*>(otile + l * BP * BN + r * BN + 16 * ((4 * kc + grp) ^ swze<BN>(frow)));
          }
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
          for (int i = 0; i < CW2; ++i)
#pragma unroll
            for (int j = 0; j < WP; ++j)
              acc2[l][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wb[kc][i], fb[l][j], acc2[l][i][j], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        const int m = m0 + j * 16 + frow;
        const int img = m < a.M ? fast_div(m, a.hw_mul, a.hw_shr) : 0;
        const float rscale =
            m < a.M ? (tab_ok ? rtab[(S::NTABS - 1) * kNTab + img] : b.x_absmax[img] * b.inv_qmax) : 0.f;
#pragma unroll
        for (int i = 0; i < CW2; ++i) {
          v4i accq[L];
#pragma unroll
          for (int s = 0; s < L; ++s) accq[s] = acc2[s][i][j];
          const int rt = j * 16 + frow, cc = wave * CW2 + i;
          const int rq0[4] = {0, 0, 0, 0};
          unsigned wq[L];
          const float mm = lean_quad<L, L, 0>(accq, rscale, csq2[i], shq2[i], false, rq0, 0.f, true, 0.f, wq);
          vmax = m < a.M ? fmaxf(vmax, mm) : vmax;
#pragma unroll
          for (int l = 0; l < L; ++l)
            *reinterpret_cast<unsigned*>(otile2 + l * BP * BN2 + rt * BN2 + 16 * (cc ^ swze<BN2>(frow)) + 4 * grp) = wq[l];
        }
      }
    }
    prev_m0 = m0;
    stage ^= 1;
  }
  if (prev_m0 >= 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    copy_out(prev_m0);
  }
  if (__any(vmax > qmax) && lane == 0) atomicMax(a.overflow, 1);
}

int device_cus_res() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
      c = 256;
    cus = c;
  }
  return cus;
}

template <int L, int LW, int CFG, int KC, bool RELU, bool RES, bool OFF>
int launch_res_one(const ConvArgs& a, hipStream_t s) {
  constexpr int CW = kRes[CFG].cw, WP = kRes[CFG].wp;
  if constexpr (!((kRes[CFG].kc_mask >> KC) & 1) || !res_fits(LW, KC, CW)) {
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tile: cin not built for this configuration");
  } else {
  using S = ResShape<L, LW, KC, CW, WP, RES, 0, 0, OFF>;
  static_assert(S::MINW >= 1, "LDS per CU");
  auto k = qconv_resident_kernel<L, LW, KC, CW, WP, RELU, RES, S::MINW, 0, OFF>;
  static const hipError_t attr = [&] {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS_TOTAL);
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
  }();
  if (attr != hipSuccess) return check_hip(attr, "qconv_resident_kernel LDS attribute");
  const long long ntiles = ((long long)a.M + S::BP - 1) / S::BP;
  const int nslabs = a.cout / S::BN;
  if (ntiles > 0x7fffffffLL) return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: grid too large");
  // persistent: as many workgroups as fit the CUs at once, a multiple of the slab count (every slab
  // walks the tiles with the same stride), at most one per (slab, tile)
  long long per_slab = (long long)device_cus_res() * S::MINW / nslabs;
  if (per_slab < 1) per_slab = 1;
  if (per_slab > ntiles) per_slab = ntiles;
  const long long blocks = per_slab * nslabs;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(kResThreads), S::LDS_TOTAL, s, a, a, a, (int)ntiles, nslabs);
  return check_hip(hipGetLastError(), "qconv_resident_kernel launch");
  }
}

template <int L, int LW, int CFG, bool RELU, bool RES, bool OFF>
int launch_res_kc(int kc, const ConvArgs& a, hipStream_t s) {
  switch (kc) {  // only the K sizes of the configuration's mask are instantiated
    case 1: return launch_res_one<L, LW, CFG, 1, RELU, RES, OFF>(a, s);
    case 2: return launch_res_one<L, LW, CFG, 2, RELU, RES, OFF>(a, s);
    case 4: return launch_res_one<L, LW, CFG, 4, RELU, RES, OFF>(a, s);
    case 8: return launch_res_one<L, LW, CFG, 8, RELU, RES, OFF>(a, s);
    case 16: return launch_res_one<L, LW, CFG, 16, RELU, RES, OFF>(a, s);
    default: return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tile: cin not built");
  }
}

template <int L, int LW, bool RELU, bool RES, bool OFF = false>
int launch_res_l(int cfg, const ConvArgs& a, hipStream_t s) {
  const int kc = a.cin / 64;
  switch (cfg) {
    case 0: return launch_res_kc<L, LW, 0, RELU, RES, OFF>(kc, a, s);
    case 1: return launch_res_kc<L, LW, 1, RELU, RES, OFF>(kc, a, s);
    case 2: return launch_res_kc<L, LW, 2, RELU, RES, OFF>(kc, a, s);
    default: return launch_res_kc<L, LW, 3, RELU, RES, OFF>(kc, a, s);
  }
}

// the Bottleneck tail chain: conv3 (one slab with all its output channels, 16-pixel tiles) with
// its identity as limb planes (LWD == 0) or as the fused downsample (LWD == 3), optionally the next
// block's conv1 (CW2 > 0), conv3's weight offsets or not
template <int L, int KC, int CW, int CW2, bool OFF, int LWD, int KCD = KC>
int launch_chain_one(const ConvArgs& a, const ConvArgs& b, const ConvArgs& d, hipStream_t s) {
  using S = ResShape<L, 1, KC, CW, 1, LWD == 0, CW2, LWD, OFF, KCD>;
  static_assert(S::MINW >= 1, "LDS per CU");
  auto k = qconv_resident_kernel<L, 1, KC, CW, 1, true, LWD == 0, S::MINW, CW2, OFF, LWD, KCD>;
  static const hipError_t attr = [&] {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS_TOTAL);
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
  }();
  if (attr != hipSuccess) return check_hip(attr, "qconv_resident_kernel (chain) LDS attribute");
  const long long ntiles = ((long long)a.M + S::BP - 1) / S::BP;
  const int nslabs = a.cout / S::BN;  // 1 with a chained conv (it needs every channel of the tile)
  long long per_slab = (long long)device_cus_res() * S::MINW / nslabs;
  if (per_slab > ntiles) per_slab = ntiles;
  if (per_slab < 1) per_slab = 1;
  hipLaunchKernelGGL(k, dim3((unsigned)(per_slab * nslabs)), dim3(kResThreads), S::LDS_TOTAL, s, a, b, d, (int)ntiles,
                     nslabs);
  return check_hip(hipGetLastError(), "qconv_resident_kernel (chain) launch");
}

}  // namespace

int resident_num_cfgs() { return kNumRes; }

void resident_cfg_info(int cfg, int* bm, int* bn, int* threads) {
  *bm = 16 * kRes[cfg].wp;
  *bn = 64 * kRes[cfg].cw;
  *threads = kResThreads;
}

// What tile_supported can see; the launcher also needs pad 0, no weight offsets and the
// static-range limb-plane epilogue without a residual (yq set; y, y_absmax, residual, residual_q NULL).
bool resident_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs) {
  if (cfg < 0 || cfg >= kNumRes || kh != 1 || kw != 1 || limbs != 3 || !(wlimbs == 1 || wlimbs == 3)) return false;
  const ResCfg& c = kRes[cfg];
  return cin % 64 == 0 && cin / 64 < 31 && ((c.kc_mask >> (cin / 64)) & 1) && cout % (64 * c.cw) == 0 &&
         res_fits(wlimbs, cin / 64, c.cw);
}

int launch_resident(int cfg, int limbs, int wlimbs, const ConvArgs& a, hipStream_t s) {
  if (!resident_supported(cfg, a.cin, a.cout, a.kh, a.kw, limbs, wlimbs) || a.pad != 0 || a.s2d)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tiles take 1x1 / pad 0 convs with 3 activation limbs, "
                                "1 or 3 weight limbs and the tile's cin (64 .. 1024) and slab of couts");
  if (!a.yq || a.y || a.residual || a.y_absmax)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tiles run the static-range limb-plane epilogue (with a "
                                "limb-plane residual or none) only");
  if (a.has_offset) {  // exact codes off-centre (ReLU convs: conv1 / conv3)
    if (wlimbs != 1 || !a.relu)
      return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tiles with weight offsets: one weight limb and ReLU");
    return a.res_q ? launch_res_l<3, 1, true, true, true>(cfg, a, s) : launch_res_l<3, 1, true, false, true>(cfg, a, s);
  }
  // built variants: the downsamples (3 weight limbs, no ReLU, no residual), conv1 / conv2 (ReLU), conv3
  // (ReLU + limb-plane residual) and plain (neither)
  if (wlimbs == 3) {
    if (a.relu || a.res_q)
      return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tiles with 3 weight limbs: no ReLU or residual");
    return launch_res_l<3, 3, false, false>(cfg, a, s);
  }
  if (a.res_q) {
    if (!a.relu) return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tiles: a residual needs ReLU");
    return launch_res_l<3, 1, true, true>(cfg, a, s);
  }
  return a.relu ? launch_res_l<3, 1, true, false>(cfg, a, s) : launch_res_l<3, 1, false, false>(cfg, a, s);
}

// Bottleneck conv3 (+ identity, ReLU) chained with the next block's conv1 (ReLU; cout2 = 0: none)
// and / or its fused downsample: (cin, cout1, cout2) = (64, 256, 64 or 0), the R50 layer1 blocks. (The
// layer2 chain 128 -> 512 -> 128,
// one 512-channel slab: 452 registers per lane, one workgroup per CU, measured 0.82-0.85x the two
// launches and the R50 step 1.2 % slower: profiles/r06_pair_chain.txt; not built.)
bool resident_pair_supported(int cin, int cout1, int cout2, int limbs) {
  // cout2 = 64: the layer-1 blocks' conv1; 128: layer 2's first conv1 (on layer 1's last output)
  return limbs == 3 && cin == 64 && cout1 == 256 && (cout2 == 64 || cout2 == 128 || cout2 == 0);
}

// conv3 (cin -> cout1) with a fused 1x1 downsample (ds_cin -> cout1, stride ds_stride) and no chained
// conv1: the first Bottleneck of R50's layer1 (64 -> 256, downsample 64 -> 256 / 1), layer2 (128 ->
// 512, downsample 256 -> 512 / 2) and layer3 (256 -> 1024, downsample 512 -> 1024 / 2)
bool resident_chain_ds_supported(int cin, int cout1, int ds_cin, int ds_stride, int limbs) {
  return limbs == 3 && ((cin == 64 && cout1 == 256 && ds_cin == 64 && ds_stride == 1) ||
                        (cin == 128 && cout1 == 512 && ds_cin == 256 && ds_stride == 2) ||
                        (cin == 256 && cout1 == 1024 && ds_cin == 512 && ds_stride == 2));
}

int launch_resident_chain(const ConvArgs& a, const ConvArgs* b, const ConvArgs* d, int limbs, hipStream_t s) {
  auto conv1x1 = [](const ConvArgs& c) { return c.kh == 1 && c.kw == 1 && c.stride == 1 && c.pad == 0 && !c.s2d; };
  auto ds1x1 = [](const ConvArgs& c) { return c.kh == 1 && c.kw == 1 && c.pad == 0 && !c.s2d; };
  const bool shapes_ok =
      conv1x1(a) && (d ? resident_chain_ds_supported(a.cin, a.cout, d->cin, d->stride, limbs) && ds1x1(*d) &&
                             d->cout == a.cout && d->ho == a.ho && d->wo == a.wo && d->n == a.n
                       : resident_pair_supported(a.cin, a.cout, b ? b->cout : 0, limbs)) &&
      (!b || (conv1x1(*b) && b->cin == a.cout && b->M == a.M));
  if (!shapes_ok)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_chain_fwd: shapes not built (conv3 1x1 stride 1, 3 activation limbs: "
                                "64->256 with the next conv1 256->64 on its output, or with its downsample over the "
                                "same output pixels: 64->256 / 1, 256->512 / 2 under 128->512, 512->1024 / 2 under "
                                "256->1024)");
  if (!a.yq || a.y || a.residual || a.y_absmax || !a.relu || (!a.res_q) == (d == nullptr) ||
      (b && (!b->yq || b->y || b->residual || b->res_q || b->y_absmax || b->has_offset || !b->relu ||
             b->overflow != a.overflow)) ||
      (d && (!d->yq_inv || d->y || d->residual || d->res_q || d->has_offset || d->relu || d->overflow != a.overflow)))
    return fail(SMPQ_E_INVALID, "smpq_conv2d_chain_fwd: static-range limb-plane outputs, ReLU, the identity as "
                                "limb planes or as the fused downsample (exactly one), one overflow flag");
  const ConvArgs& bb = b ? *b : a;
  const ConvArgs& dd = d ? *d : a;
  const bool off = a.has_offset != 0;
  if (d) {
    // conv3 + the fused downsample: 128-channel slabs (three workgroups per CU). With the chained
    // conv1 as well it needs one 256-channel slab, ~410 registers per lane and one workgroup per
    // CU: measured 4-5 % slower on the R50 step than without (profiles/r06_chain_fused_ds.txt); not built
    if (b) return fail(SMPQ_E_INVALID, "smpq_conv2d_chain_fwd: the fused downsample is built without a chained conv1");
    // (layer2 / layer3: 128- / 64-channel slabs, the downsample's K 256 / 512 beside conv3's 128 / 256)
    if (a.cin == 128) return off ? launch_chain_one<3, 2, 2, 0, true, 3, 4>(a, bb, dd, s) : launch_chain_one<3, 2, 2, 0, false, 3, 4>(a, bb, dd, s);
    if (a.cin == 256) return off ? launch_chain_one<3, 4, 1, 0, true, 3, 8>(a, bb, dd, s) : launch_chain_one<3, 4, 1, 0, false, 3, 8>(a, bb, dd, s);
    return off ? launch_chain_one<3, 1, 2, 0, true, 3>(a, bb, dd, s) : launch_chain_one<3, 1, 2, 0, false, 3>(a, bb, dd, s);
  }
  if (!b) return fail(SMPQ_E_INVALID, "smpq_conv2d_chain_fwd: nothing to chain (plain conv3: smpq_conv2d_fwd_q)");
  if (b->cout == 128)
    return off ? launch_chain_one<3, 1, 4, 2, true, 0>(a, bb, dd, s) : launch_chain_one<3, 1, 4, 2, false, 0>(a, bb, dd, s);
  return off ? launch_chain_one<3, 1, 4, 1, true, 0>(a, bb, dd, s) : launch_chain_one<3, 1, 4, 1, false, 0>(a, bb, dd, s);
}

}  // namespace smpq
