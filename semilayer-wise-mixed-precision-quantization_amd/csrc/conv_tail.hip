// Fused Bottleneck tail for gfx950: conv2 (kxk, stride s) + bn2 + relu -> t2 -> conv3 (1x1) + bn3
// + residual add + relu (resnet.py:103-114), static-range mode, in ONE launch.
//
// The two-launch path writes t2 (the 3x3 conv's output, 64..512 channels) to HBM as limb planes and
// reads it straight back as the 1x1 expansion's input. Here a block owns BP output pixels and ALL
// cmid channels of conv2, so its t2 tile is complete in LDS after phase 1 and phase 2 (conv3) reads
// its A operand from there: t2 never leaves the CU. Phase 1 is the LDS-DMA implicit GEMM of
// conv_glds.hip (weights = MFMA A operand, activations = B, two DMA stages, XCD-aware tile order);
// its lean epilogue writes the t2 codes into an LDS image laid out exactly like the DMA stages
// (K steps of 64 channels, 64-B rows, the same XOR swizzle), so phase 2's fragment reads are the
// kernel's ordinary ds_read_b128 pattern. Phase 2 walks conv3's cout3 = 4 cmid channels in four
// chunks of cmid (the phase-1 wave layout again), its weight fragments straight from L2 into
// registers one K step ahead, the residual's limb planes as 16-B pieces (the next chunk's requested
// under the current chunk's stores); the output
// leaves through the lane-group-transposed 16-B stores.
//
// Every value is computed as the two launches compute it: exact integer accumulation, the same
// lean_quad epilogue (lds_dma.h) with the same operands, so the output planes and the overflow
// flag are bitwise those of conv2d_q(conv2) followed by conv2d_q(conv3) (tests/test_gpu.py).
#include "conv_common.h"
#include "lds_dma.h"

namespace smpq {

struct TailArgs {
  ConvArgs a;              // conv2: xq = t1 planes, codes = w2, yq_inv = t2 quantizer, relu, overflow
  const int8_t* codes3;    // [cout3][cmid] conv3 weight codes (one limb)
  const int32_t* w_off3;   // [cout3] or NULL
  const float* col_scale3;
  const float* col_shift3;
  const int8_t* res_q;     // [L][M][cout3] residual limb planes
  float res_scale;         // residual value = res_scale * code
  int8_t* yq;              // [L][M][cout3] output limb planes
  float yq_inv3;           // QMAX / output range
  float range2;            // t2's static range (conv3's input scale = range2 * inv_qmax)
  int cout3, relu3, has_offset3, nt_store3;
};

template <int L, int WAVES_C, int WAVES_P, int WC, int WP, int BK>
__global__ __launch_bounds__(64 * WAVES_C * WAVES_P, 2) void qconv_tail_kernel(TailArgs ta) {
  static_assert(BK == 64 || BK == 128, "BK");
  static_assert(WC % 4 == 0, "16-B limb-plane epilogue needs 4k channel blocks per wave");
  const ConvArgs& a = ta.a;
  constexpr int NW = WAVES_C * WAVES_P;
  constexpr int BC = 16 * WC * WAVES_C;  // == cmid: all conv2 output channels of the tile
  constexpr int BP = 16 * WP * WAVES_P;  // output pixels per tile
  constexpr int NACC = L;                // one weight limb: SMIN = 0
  constexpr int KH = BK / 64;
  constexpr int RPP = 1024 / BK;
  constexpr int CPR = BK / 16;
  constexpr int WPIECES = BC / RPP;
  constexpr int APIECES = L * (BP / RPP);
  constexpr int STAGE = (WPIECES + APIECES) * 1024;
  constexpr int WSLOTS = (WPIECES + NW - 1) / NW;
  constexpr int ASLOTS = (APIECES + NW - 1) / NW;
  constexpr int NST = 2;
  constexpr int T2OFF = NST * STAGE;     // t2 image: [BC / 64][L][BP][64 B], swz<64> chunks
  constexpr int KS3 = BC / 64;           // conv3 K steps
  constexpr int NQ = WC / 4;
  constexpr int NCH = 4;                 // conv3 channel chunks of BC (cout3 == 4 cmid)
  constexpr float qmax = act_qmax<L>();
  extern __shared__ __attribute__((aligned(1024))) int8_t lds[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < NW);
  const int wc = wave / WAVES_P, wp = wave % WAVES_P;
  const int frow = lane & 15;

  // ---- XCD-aware tile order (consecutive pixel tiles share 3x3 halos in one XCD's L2) ------
  const int total = (int)gridDim.x;
  const int full = total & ~7;
  int t = blockIdx.x;
  if (t < full) t = (t & 7) * (full >> 3) + (t >> 3);
  const int m0 = t * BP;
  const int hw_out = a.ho * a.wo;

  const v4i wrs = make_rsrc(a.codes, a.wplane);
  const v4i xrs = make_rsrc(a.xq, (long long)L * a.plane);

  // ---- phase 1: conv2 (LDS-DMA implicit GEMM, as qconv_glds_kernel with LW = 1, NST = 2) ----
  const int prow = lane / CPR;
  auto pchunk_of = [&](int q) { return (lane % CPR) ^ swz<BK>((RPP * q + prow) & 15); };
  unsigned wsrc[WSLOTS];
#pragma unroll
  for (int s = 0; s < WSLOTS; ++s) {
    const int p = wave + NW * s;
    const int row = RPP * p + prow;
    wsrc[s] = (p < WPIECES) ? (unsigned)((long long)row * a.K + 16 * pchunk_of(p)) : kOOB;
  }
  int apix[ASLOTS], aih[ASLOTS], aiw[ASLOTS];
#pragma unroll
  for (int s = 0; s < ASLOTS; ++s) {
    const int p = wave + NW * s;
    const int bj = p % (BP / RPP);
    const int m = m0 + RPP * bj + prow;
    if (p < APIECES && m < a.M) {
      const int img = fast_div(m, a.hw_mul, a.hw_shr);
      const int rem = m - img * hw_out;
      const int oh = fast_div(rem, a.wo_mul, a.wo_shr), ow = rem - oh * a.wo;
      aih[s] = oh * a.stride - a.pad;
      aiw[s] = ow * a.stride - a.pad;
      apix[s] = ((img * a.h + aih[s]) * a.w + aiw[s]) * a.cin + 16 * pchunk_of(bj);
    } else {
      aih[s] = -(1 << 28);
      aiw[s] = 0;
      apix[s] = 0;
    }
  }
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  auto issue = [&](int buf, int kr, int kc, int c0, int ks) {
    const unsigned sb = lds0 + buf * STAGE;
#pragma unroll
    for (int s = 0; s < WSLOTS; ++s) {
      const int p = wave + NW * s;
      if (p < WPIECES) dma16(sb + p * 1024, wrs, wsrc[s], __builtin_amdgcn_readfirstlane(ks * BK));
    }
    const int tapoff = (kr * a.w + kc) * a.cin + c0;
#pragma unroll
    for (int s = 0; s < ASLOTS; ++s) {
      const int p = wave + NW * s;
      if (p < APIECES) {
        const int l = p / (BP / RPP);
        const bool ok = (unsigned)(aih[s] + kr) < (unsigned)a.h && (unsigned)(aiw[s] + kc) < (unsigned)a.w;
        const unsigned voff = ok ? (unsigned)(apix[s] + tapoff) : kOOB;
        dma16(sb + (WPIECES + p) * 1024, xrs, voff, __builtin_amdgcn_readfirstlane((unsigned)((long long)l * a.plane)));
      }
    }
  };

  // output coordinates of this lane (both phases): channels chan_i + 0..3 (relative to the chunk)
  // of pixel mrow[j]
  int mrow[WP];
  bool mok[WP];
#pragma unroll
  for (int j = 0; j < WP; ++j) {
    const int m = m0 + (wp * WP + j) * 16 + frow;
    mok[j] = m < a.M;
    mrow[j] = mok[j] ? m : 0;
  }
  int chan[WC];
#pragma unroll
  for (int i = 0; i < WC; ++i) chan[i] = (wc * WC + i) * 16 + 4 * (lane >> 4);

  // conv3's residual limb planes [L][M][cout3]: 16-B pieces, one chunk at a time
  const long long oplane = (long long)a.M * ta.cout3;
  const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(ta.res_q), 0, (int)(L * oplane), 0x00020000);
  auto qoff_of = [&](int n3, int q, int j) {
    const int c16 = n3 + (wc * WC + 4 * q + (lane >> 4)) * 16;
    return mok[j] ? (unsigned)(mrow[j] * ta.cout3 + c16) : kOOB;
  };
  unsigned rq[WC][WP][L];
  auto load_res = [&](int n3) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < WP; ++j)
#pragma unroll
        for (int l = 0; l < L; ++l) {
          const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rrs, qoff_of(n3, q, j), (unsigned)((long long)l * oplane), 0);
#pragma unroll
          for (int c = 0; c < 4; ++c) rq[4 * q + c][j][l] = v[c];
        }
  };

  v4i acc[NACC][WC][WP];
#pragma unroll
  for (int s = 0; s < NACC; ++s)
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) acc[s][i][j] = v4i{0, 0, 0, 0};
  const bool do_off = a.has_offset != 0;
  int rs[L][WP];
#pragma unroll
  for (int l = 0; l < L; ++l)
#pragma unroll
    for (int j = 0; j < WP; ++j) rs[l][j] = 0;

  int rd[KH];
#pragma unroll
  for (int h = 0; h < KH; ++h) rd[h] = frow * BK + 16 * ((4 * h + (lane >> 4)) ^ swz<BK>(frow));
  const int nsteps = a.ksteps / KH;
  int kr = 0, kc = 0, c0 = 0, nissued = 0, wbuf = 0, rbuf = 0;
  auto issue_next = [&]() {
    if (nissued < nsteps) {
      issue(wbuf, kr, kc, c0, nissued);
      c0 += BK;
      if (c0 == a.cin) {
        c0 = 0;
        if (++kc == a.kw) {
          kc = 0;
          ++kr;
        }
      }
      ++nissued;
      wbuf ^= 1;
    }
  };
  struct Frags {
    v4i w[WC], a[L][WP];
  };
  auto pix_sums = [&](const v4i (&fa)[L][WP]) {  // offset correction: per-pixel digit sums
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        int s = rs[l][j];
        s = __builtin_amdgcn_sdot4(fa[l][j].x, 0x01010101, s, false);
        s = __builtin_amdgcn_sdot4(fa[l][j].y, 0x01010101, s, false);
        s = __builtin_amdgcn_sdot4(fa[l][j].z, 0x01010101, s, false);
        s = __builtin_amdgcn_sdot4(fa[l][j].w, 0x01010101, s, false);
        rs[l][j] = s;
      }
  };
  auto mma = [&](const v4i (&fw)[WC], const v4i (&fa)[L][WP]) {
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j)
          acc[l][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fw[i], fa[l][j], acc[l][i][j], 0, 0, 0);
  };
  issue_next();
  for (int ks = 0; ks < nsteps; ++ks) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int8_t* sb = lds + rbuf * STAGE;
    rbuf ^= 1;
#pragma unroll
    for (int h = 0; h < KH; ++h) {
      Frags f;
#pragma unroll
      for (int i = 0; i < WC; ++i) f.w[i] = *reinterpret_cast<const v4i*>(sb + ((wc * WC + i) * 16) * BK + rd[h]);
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int j = 0; j < WP; ++j)
          f.a[l][j] = *reinterpret_cast<const v4i*>(sb + WPIECES * 1024 + (l * BP + (wp * WP + j) * 16) * BK + rd[h]);
      if (h == 0) issue_next();  // the DMA of step ks + 1 into the other stage
      if (do_off) pix_sums(f.a);
      mma(f.w, f.a);
    }
  }

  // conv3's residual for chunk 0 (16-B pieces: lane group g loads the 16 channels of block 4q + g of
  // its pixel; transposed to the accumulator layout in the epilogue), under epilogue 1
  load_res(0);

  // weight-offset correction: acc_l += offset_c * (sum of the pixel's digits of limb l)
  auto offset_fix = [&](const int32_t* w_off, int n3) {
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        int s = rs[l][j];
        s += __shfl_xor(s, 16, kWave);
        s += __shfl_xor(s, 32, kWave);
        rs[l][j] = s;
      }
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const int4 coff = *reinterpret_cast<const int4*>(w_off + n3 + chan[i]);
      const int cor[4] = {coff.x, coff.y, coff.z, coff.w};
#pragma unroll
      for (int s = 0; s < L; ++s)
#pragma unroll
        for (int j = 0; j < WP; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[s][i][j][r] += __mul24(cor[r], rs[s][j]);
    }
  };

  // ---- epilogue 1: t2 codes (lean static epilogue of conv2) into the LDS image ---------------
  {
    if (do_off) offset_fix(a.w_off, 0);
    float rscale[WP];
#pragma unroll
    for (int j = 0; j < WP; ++j) rscale[j] = mok[j] ? a.x_absmax[fast_div(mrow[j], a.hw_mul, a.hw_shr)] * a.inv_qmax : 0.f;
    const float inv = a.yq_inv;
    const float lo = a.relu ? 0.f : -qmax;
    const bool relu = a.relu != 0;
    float vmax = 0.f;
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const float4 cs = *reinterpret_cast<const float4*>(a.col_scale + chan[i]);
      const float4 csh = *reinterpret_cast<const float4*>(a.col_shift + chan[i]);
      const float csq[4] = {cs.x * inv, cs.y * inv, cs.z * inv, cs.w * inv};
      const float shq[4] = {csh.x * inv, csh.y * inv, csh.z * inv, csh.w * inv};
      const int ch = (wc * WC + i) * 16;  // this quad's 16-channel block; 64-channel K step ch / 64
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        unsigned wq[L];
        const int rqdummy[4] = {0, 0, 0, 0};
        v4i accq[NACC];
#pragma unroll
        for (int s = 0; s < NACC; ++s) accq[s] = acc[s][i][j];
        const float mm = lean_quad<L, NACC, 0>(accq, rscale[j], csq, shq, false, rqdummy, 0.f, relu, lo, wq);
        vmax = mok[j] ? fmaxf(vmax, mm) : vmax;
        const int rt = (wp * WP + j) * 16 + frow;
#pragma unroll
        for (int l = 0; l < L; ++l)
          *reinterpret_cast<unsigned*>(lds + T2OFF + (((ch >> 6) * L + l) * BP + rt) * 64 +
                                       16 * (((ch >> 4) & 3) ^ swz<64>(frow)) + 4 * (lane >> 4)) = wq[l];
      }
    }
    if (__any(vmax > qmax) && lane == 0) atomicMax(a.overflow, 1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- phase 2: conv3 over the t2 image, four chunks of BC output channels ------------------
  const auto w3rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(ta.codes3), 0, ta.cout3 * BC, 0x00020000);
  const float rscale3 = ta.range2 * a.inv_qmax;
  const float inv3 = ta.yq_inv3;
  const float rsq3 = ta.res_scale * inv3;
  const float lo3 = ta.relu3 ? 0.f : -qmax;
  const bool relu3 = ta.relu3 != 0;
  const bool do_off3 = ta.has_offset3 != 0;
  const v4i qrs4 = make_rsrc(ta.yq, (long long)L * oplane);
  const bool nt = __builtin_amdgcn_readfirstlane(ta.nt_store3) != 0;
  float vmax3 = 0.f;
  // weight fragment i of K step k3 of chunk n3: 16 B of row n3 + chan-block, bytes 64 k3 + 16 (lane >> 4)
  auto load_w3 = [&](v4i (&fw)[WC], int n3, int k3) {
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const int row = n3 + (wc * WC + i) * 16 + frow;
      fw[i] = __builtin_bit_cast(
          v4i, __builtin_amdgcn_raw_buffer_load_b128(w3rs, (unsigned)(row * BC + 64 * k3 + 16 * (lane >> 4)), 0u, 0));
    }
  };
  const int rd3 = frow * 64 + 16 * ((lane >> 4) ^ swz<64>(frow));
  v4i fwa[WC], fwb[WC];
  load_w3(fwa, 0, 0);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int n3 = c * BC;
#pragma unroll
    for (int s = 0; s < NACC; ++s)
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j) acc[s][i][j] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int j = 0; j < WP; ++j) rs[l][j] = 0;
#pragma unroll
    for (int k3 = 0; k3 < KS3; ++k3) {
      v4i(&fw)[WC] = ((c * KS3 + k3) & 1) ? fwb : fwa;
      v4i(&fwn)[WC] = ((c * KS3 + k3) & 1) ? fwa : fwb;
      if (k3 + 1 < KS3) load_w3(fwn, n3, k3 + 1);
      else if (c + 1 < NCH) load_w3(fwn, n3 + BC, 0);
      v4i fa[L][WP];
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int j = 0; j < WP; ++j)
          fa[l][j] = *reinterpret_cast<const v4i*>(lds + T2OFF + ((k3 * L + l) * BP + (wp * WP + j) * 16) * 64 + rd3);
      if (do_off3) pix_sums(fa);
      mma(fw, fa);
    }
    // epilogue 2: residual + bn3 + relu -> output codes (lean), 16-B transposed stores
    if (do_off3) offset_fix(ta.w_off3, n3);
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < WP; ++j)
#pragma unroll
        for (int l = 0; l < L; ++l) {
          unsigned w0 = rq[4 * q][j][l], w1 = rq[4 * q + 1][j][l], w2 = rq[4 * q + 2][j][l], w3 = rq[4 * q + 3][j][l];
          transpose4(w0, w1, w2, w3);
          rq[4 * q][j][l] = w0;
          rq[4 * q + 1][j][l] = w1;
          rq[4 * q + 2][j][l] = w2;
          rq[4 * q + 3][j][l] = w3;
        }
    unsigned wq[WC][WP][L];
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const float4 cs = *reinterpret_cast<const float4*>(ta.col_scale3 + n3 + chan[i]);
      const float4 csh = *reinterpret_cast<const float4*>(ta.col_shift3 + n3 + chan[i]);
      const float csq[4] = {cs.x * inv3, cs.y * inv3, cs.z * inv3, cs.w * inv3};
      const float shq[4] = {csh.x * inv3, csh.y * inv3, csh.z * inv3, csh.w * inv3};
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        int rqv[4];
        decode4<L>(rq[i][j], rqv);
        v4i accq[NACC];
#pragma unroll
        for (int s = 0; s < NACC; ++s) accq[s] = acc[s][i][j];
        const float m = lean_quad<L, NACC, 0>(accq, mok[j] ? rscale3 : 0.f, csq, shq, true, rqv, rsq3, relu3, lo3,
                                              wq[i][j]);
        vmax3 = mok[j] ? fmaxf(vmax3, m) : vmax3;
      }
    }
    if (c + 1 < NCH) load_res(n3 + BC);  // the next chunk's residual, in flight under these stores
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < WP; ++j)
#pragma unroll
        for (int l = 0; l < L; ++l) {
          unsigned w0 = wq[4 * q][j][l], w1 = wq[4 * q + 1][j][l], w2 = wq[4 * q + 2][j][l], w3 = wq[4 * q + 3][j][l];
          transpose4(w0, w1, w2, w3);
          store_limbs16(v4u{w0, w1, w2, w3}, qrs4, qoff_of(n3, q, j),
                        __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane)), nt);
        }
  }
  if (__any(vmax3 > qmax) && lane == 0) atomicMax(a.overflow, 1);
}

// ------------------------------------------------------------------------------------------
struct TailCfg {
  int wavesc, wavesp, wc, wp, bk;
};
constexpr TailCfg kTail[] = {
    // (configs whose live registers exceed 256 at 3 limbs — WC * WP >= 8 — spill; not built)
    {1, 4, 4, 1, 64},   // 0:  64 ch x  64 px (cmid 64)
    {1, 8, 4, 1, 64},   // 1:  64 ch x 128 px, 8 waves
    {2, 2, 4, 1, 64},   // 2: 128 ch x  32 px (cmid 128)
    {2, 2, 4, 1, 128},  // 3: 128 ch x  32 px, 128-B K steps
    {2, 4, 4, 1, 64},   // 4: 128 ch x  64 px, 8 waves
    {2, 4, 4, 1, 128},  // 5: 128 ch x  64 px, 8 waves, 128-B K steps
    {4, 1, 4, 1, 64},   // 6: 256 ch x  16 px (cmid 256)
    {4, 1, 4, 1, 128},  // 7: 256 ch x  16 px, 128-B K steps
    {4, 2, 4, 1, 64},   // 8: 256 ch x  32 px, 8 waves
    {8, 1, 4, 1, 64},   // 9: 512 ch x  16 px, 8 waves (cmid 512)
};
constexpr int kNumTail = sizeof(kTail) / sizeof(kTail[0]);

static int tail_lds_bytes(const TailCfg& c, int limbs) {
  const int bc = 16 * c.wc * c.wavesc, bp = 16 * c.wp * c.wavesp;
  return 2 * (bc + limbs * bp) * c.bk + limbs * bp * bc;
}

static bool tail_supported(int cfg, int cmid, int cout3, int cin, int limbs) {
  if (cfg < 0 || cfg >= kNumTail || (limbs != 2 && limbs != 3)) return false;
  const TailCfg& c = kTail[cfg];
  const int bc = 16 * c.wc * c.wavesc;
  if (bc != cmid || cout3 != 4 * cmid || cin % c.bk != 0 || cmid % 64 != 0) return false;
  const int accs = limbs * c.wc * c.wp * 4;
  if (accs > 128) return false;
  return tail_lds_bytes(c, limbs) <= 160 * 1024;
}

template <int L, int WAVES_C, int WAVES_P, int WC, int WP, int BK>
static int launch_tail_one(const TailArgs& ta, hipStream_t stream) {
  constexpr int BP = 16 * WP * WAVES_P, BC = 16 * WC * WAVES_C;
  constexpr int LDSB = 2 * (BC + L * BP) * BK + L * BP * BC;
  if constexpr (L * WC * WP * 4 > 128 || LDSB > 160 * 1024) {
    return fail(SMPQ_E_INVALID, "smpq_bottleneck_tail_q: tile config too large for these limbs");
  } else {
    const long blocks = ((long)ta.a.M + BP - 1) / BP;
    auto k = qconv_tail_kernel<L, WAVES_C, WAVES_P, WC, WP, BK>;
    static const hipError_t attr = [&] {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDSB);
      if (e != hipSuccess) (void)hipGetLastError();
      return e;
    }();
    if (attr != hipSuccess) return check_hip(attr, "qconv_tail_kernel LDS attribute");
    hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(64 * WAVES_C * WAVES_P), LDSB, stream, ta);
    return check_hip(hipGetLastError(), "qconv_tail_kernel launch");
  }
}

template <int L>
static int launch_tail(int cfg, const TailArgs& ta, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_tail_one<L, 1, 4, 4, 1, 64>(ta, s);
    case 1: return launch_tail_one<L, 1, 8, 4, 1, 64>(ta, s);
    case 2: return launch_tail_one<L, 2, 2, 4, 1, 64>(ta, s);
    case 3: return launch_tail_one<L, 2, 2, 4, 1, 128>(ta, s);
    case 4: return launch_tail_one<L, 2, 4, 4, 1, 64>(ta, s);
    case 5: return launch_tail_one<L, 2, 4, 4, 1, 128>(ta, s);
    case 6: return launch_tail_one<L, 4, 1, 4, 1, 64>(ta, s);
    case 7: return launch_tail_one<L, 4, 1, 4, 1, 128>(ta, s);
    case 8: return launch_tail_one<L, 4, 2, 4, 1, 64>(ta, s);
    case 9: return launch_tail_one<L, 8, 1, 4, 1, 64>(ta, s);
    default: return fail(SMPQ_E_INVALID, "smpq_bottleneck_tail_q: bad tile config");
  }
}

}  // namespace smpq

using namespace smpq;

extern "C" int smpq_bottleneck_tail_num_configs(void) { return kNumTail; }

extern "C" int smpq_bottleneck_tail_supported(int cfg, int cmid, int cout3, int kh, int kw, int limbs) {
  (void)kh;
  (void)kw;
  return tail_supported(cfg, cmid, cout3, cmid, limbs) ? 1 : 0;
}

extern "C" int smpq_bottleneck_tail_q(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cmid,
                                      const int8_t* codes2, const int32_t* offset2, int kh, int kw, int stride,
                                      int pad, const float* col_scale2, const float* col_shift2, int relu2,
                                      float range2, const int8_t* codes3, const int32_t* offset3, int cout3,
                                      const float* col_scale3, const float* col_shift3, const int8_t* residual_q,
                                      float residual_range, int relu3, int limbs, int8_t* yq, float yq_range,
                                      int32_t* overflow, int tile_cfg, smpq_stream_t stream) {
  if (!xq || !x_absmax || !codes2 || !col_scale2 || !col_shift2 || !codes3 || !col_scale3 || !col_shift3 ||
      !residual_q || !yq || !overflow)
    return fail(SMPQ_E_INVALID, "smpq_bottleneck_tail_q: null pointer");
  if (!(range2 > 0.f) || !(yq_range > 0.f) || !(residual_range > 0.f))
    return fail(SMPQ_E_INVALID, "smpq_bottleneck_tail_q: ranges must be positive");
  if (n <= 0 || h <= 0 || w <= 0 || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0)
    return fail(SMPQ_E_SHAPE, "smpq_bottleneck_tail_q: bad shape");
  if (!tail_supported(tile_cfg, cmid, cout3, cmid, limbs))
    return fail(SMPQ_E_INVALID, "smpq_bottleneck_tail_q: tile config does not take this shape (cmid " +
                                    std::to_string(cmid) + ", cout3 " + std::to_string(cout3) + ", limbs " +
                                    std::to_string(limbs) + ")");
  const float qm = limbs == 2 ? 32512.f : 8323072.f;
  TailArgs ta = {};
  ConvArgs& a = ta.a;
  a.xq = xq;
  a.plane = (long long)n * h * w * cmid;
  a.x_absmax = x_absmax;
  a.codes = codes2;
  a.w_off = offset2;
  a.col_scale = col_scale2;
  a.col_shift = col_shift2;
  a.yq_inv = qm / range2;
  a.overflow = overflow;
  a.n = n;
  a.h = h;
  a.w = w;
  a.cin = cmid;
  a.cout = cmid;
  a.kh = kh;
  a.kw = kw;
  a.stride = stride;
  a.pad = pad;
  a.ho = (h + 2 * pad - kh) / stride + 1;
  a.wo = (w + 2 * pad - kw) / stride + 1;
  if (a.ho <= 0 || a.wo <= 0) return fail(SMPQ_E_SHAPE, "smpq_bottleneck_tail_q: empty output");
  const long M = (long)n * a.ho * a.wo;
  const long long lim = 0x7fffff00LL;
  if ((long long)limbs * a.plane > lim || (long long)limbs * M * cout3 > lim || (long long)cout3 * cmid > lim)
    return fail(SMPQ_E_SHAPE, "smpq_bottleneck_tail_q: planes must stay below 2 GiB");
  a.M = (int)M;
  a.K = kh * kw * cmid;
  a.cchunks = cmid / kKStep;
  a.ksteps = kh * kw * a.cchunks;
  a.wplane = (long long)cmid * a.K;
  a.relu = relu2 ? 1 : 0;
  a.has_offset = offset2 ? 1 : 0;
  a.inv_qmax = 1.f / qm;
  fast_div_init(a.ho * a.wo, a.hw_mul, a.hw_shr);
  fast_div_init(a.wo, a.wo_mul, a.wo_shr);
  ta.codes3 = codes3;
  ta.w_off3 = offset3;
  ta.col_scale3 = col_scale3;
  ta.col_shift3 = col_shift3;
  ta.res_q = residual_q;
  ta.res_scale = residual_range / qm;  // as smpq_conv2d_fwd_q computes it
  ta.yq = yq;
  ta.yq_inv3 = qm / yq_range;
  ta.range2 = range2;
  ta.cout3 = cout3;
  ta.relu3 = relu3 ? 1 : 0;
  ta.has_offset3 = offset3 ? 1 : 0;
  {
    static const long long nt_min = [] {
      const char* e = getenv("SMPQ_NT_MIN_MB");
      return (e ? atoll(e) : 64LL) << 20;
    }();
    ta.nt_store3 = ((long long)limbs * M * cout3 >= nt_min) ? 1 : 0;
  }
  hipStream_t s = (hipStream_t)stream;
  return limbs == 2 ? launch_tail<2>(tile_cfg, ta, s) : launch_tail<3>(tile_cfg, ta, s);
}
