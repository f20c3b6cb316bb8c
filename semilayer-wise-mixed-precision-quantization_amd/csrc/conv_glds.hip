// Quantized convolution forward for gfx950, LDS-DMA staged (cin % 64 == 0).
//
// Same contract and bitwise-identical results as qconv_kernel (conv.hip): an implicit GEMM on
// v_mfma_i32_16x16x64_i8 over int8 limb planes, replacing nn.Conv2d on the fake-quantized weight
// + eval BatchNorm + ReLU + residual add of resnet.py:55-68 / 97-116. What differs is how the
// operands reach the matrix cores and how outputs leave:
//
//  * Roles: the MFMA A operand is the WEIGHT tile (rows = output channels), B is the ACTIVATION
//    tile (cols = output pixels). The accumulator layout (row = 4*(lane>>4) + reg, col = lane&15)
//    then gives every lane 4 consecutive channels of one pixel: NHWC outputs, residuals and the
//    next layer's limb planes move as whole dwords / float4s straight from registers, with no LDS
//    round trip in the epilogue.
//  * Staging: every operand piece (16 rows x 64 B of one limb = one MFMA fragment block) arrives
//    by one `buffer_load_dwordx4 ... lds` wave-instruction (LDS-DMA): no VGPR staging, no
//    ds_write. Out-of-range offsets (conv zero padding, rows past M / cout) read as zeros through
//    the buffer descriptor's range check, so the loader is branch-free.
//  * LDS image: 64-B rows, no padding; the 16-B chunk c of row r sits at chunk c ^ ((4 - (r>>2)) & 3)
//    (the DMA writes lane-linearly, so the permutation is applied to each lane's SOURCE address).
//    That makes both the DMA writes and the ds_read_b128 fragment reads bank-conflict-free for
//    the b128 lane groups of gfx950.
//  * Two LDS stages: the DMA of K step k+1 is issued right after the fragments of step k are read
//    into registers and runs under step k's MFMAs; one s_barrier per K step.
//  * Tile order: block ids are remapped so that consecutive tiles (all channel tiles of one pixel
//    tile, then the neighbouring pixel tiles that share the 3x3 halo) run on the same XCD and
//    share its L2 (dispatch assigns block b to XCD b % 8).
#include "conv_common.h"

namespace smpq {

namespace {

constexpr unsigned kOOB = 0x80000000u;  // a buffer offset past every range we build (< 2^31 B)

__device__ __forceinline__ v4i make_rsrc(const void* base, long long bytes) {
  const unsigned long long b = reinterpret_cast<unsigned long long>(base);
  v4i r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
  r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));  // stride 0
  r.z = __builtin_amdgcn_readfirstlane((int)(unsigned)bytes);
  r.w = 0x00020000;
  return r;
}

// One 1-KiB piece: lane i's 16 bytes at rsrc[voff + soff] -> LDS [lds + 16 i, +16).
__device__ __forceinline__ void dma16(unsigned lds, v4i rsrc, unsigned voff, unsigned soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds), "s"(soff)
      : "memory");
}

__device__ __forceinline__ int swz(int row) { return (4 - (row >> 2)) & 3; }

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)reinterpret_cast<unsigned long long>(p);
}

// Balanced base-256 digit LIMB of q is byte LIMB of the returned int: d0 = (int8)q,
// d1 = (int8)((q + 0x80) >> 8), d2 = (q + 0x8080) >> 16 (the carries of the balanced split).
template <int LIMB>
__device__ __forceinline__ int digit_src(int q) {
  if constexpr (LIMB == 0) return q;
  else if constexpr (LIMB == 1) return q + 0x80;
  else return q + 0x8080;
}

// bytes k of four ints -> one dword
__device__ __forceinline__ unsigned pack_bytes(int b0, int b1, int b2, int b3, int k) {
  // v_perm_b32: selector byte values 0..3 pick bytes of the second operand, 4..7 of the first
  const unsigned sel_lo = (unsigned)k | ((unsigned)(k + 4) << 8) | 0x0c0c0000u;
  const unsigned lo = __builtin_amdgcn_perm((unsigned)b1, (unsigned)b0, sel_lo);
  const unsigned hi = __builtin_amdgcn_perm((unsigned)b3, (unsigned)b2, sel_lo);
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

}  // namespace

template <int L, int LW, int WAVES_C, int WAVES_P, int WC, int WP, int MINW>
__global__ __launch_bounds__(64 * WAVES_C * WAVES_P, MINW) void qconv_glds_kernel(ConvArgs a) {
  constexpr int NW = WAVES_C * WAVES_P;
  constexpr int BC = 16 * WC * WAVES_C;  // channels per block tile
  constexpr int BP = 16 * WP * WAVES_P;  // pixels per block tile
  constexpr int SMIN = (L + LW - 4) > 0 ? (L + LW - 4) : 0;
  constexpr int NACC = L + LW - 1 - SMIN;
  constexpr int WPIECES = LW * (BC / 16);
  constexpr int APIECES = L * (BP / 16);
  constexpr int NPIECE = WPIECES + APIECES;
  constexpr int STAGE = NPIECE * 1024;
  constexpr int WSLOTS = (WPIECES + NW - 1) / NW;
  constexpr int ASLOTS = (APIECES + NW - 1) / NW;
  __shared__ __attribute__((aligned(1024))) int8_t lds[2 * STAGE];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wc = wave / WAVES_P, wp = wave % WAVES_P;

  // ---- XCD-aware tile order ----------------------------------------------------------------
  const int ntc = (a.cout + BC - 1) / BC;
  const int total = (int)gridDim.x;
  const int full = total & ~7;
  int t = blockIdx.x;
  if (t < full) t = (t & 7) * (full >> 3) + (t >> 3);
  const int m0 = (t / ntc) * BP;
  const int n0 = (t % ntc) * BC;
  const int hw_out = a.ho * a.wo;

  const v4i wrs = make_rsrc(a.codes, (long long)LW * a.wplane);
  const v4i xrs = make_rsrc(a.xq, (long long)L * a.plane);

  // ---- per-lane source offsets of this wave's DMA pieces -------------------------------------
  // piece row = lane >> 2, physical chunk = lane & 3 -> logical K chunk (lane & 3) ^ swz(row)
  const int prow = lane >> 2;
  const int pchunk = (lane & 3) ^ swz(prow);
  unsigned wsrc[WSLOTS];
#pragma unroll
  for (int s = 0; s < WSLOTS; ++s) {
    const int p = wave + NW * s;  // weight piece: limb p / (BC/16), block p % (BC/16)
    const int lw = p / (BC / 16), bi = p % (BC / 16);
    const int row = n0 + 16 * bi + prow;
    wsrc[s] = (p < WPIECES && row < a.cout)
                  ? (unsigned)((long long)lw * a.wplane + (long long)row * a.K + 16 * pchunk)
                  : kOOB;
  }
  int apix[ASLOTS], aih[ASLOTS], aiw[ASLOTS];
#pragma unroll
  for (int s = 0; s < ASLOTS; ++s) {
    const int p = wave + NW * s;  // activation piece: limb p / (BP/16), block p % (BP/16)
    const int bj = p % (BP / 16);
    const int m = m0 + 16 * bj + prow;
    if (p < APIECES && m < a.M) {
      const int img = m / hw_out;
      const int rem = m - img * hw_out;
      const int oh = rem / a.wo, ow = rem - (rem / a.wo) * a.wo;
      aih[s] = oh * a.stride - a.pad;
      aiw[s] = ow * a.stride - a.pad;
      apix[s] = ((img * a.h + aih[s]) * a.w + aiw[s]) * a.cin + 16 * pchunk;
    } else {
      aih[s] = -(1 << 28);  // never inside the image
      aiw[s] = 0;
      apix[s] = 0;
    }
  }
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));

  // K position of step ks: tap (kr, kc), channel chunk c0 (scalar, advanced incrementally)
  auto issue = [&](int buf, int kr, int kc, int c0, int ks) {
    const unsigned sb = lds0 + buf * STAGE;
#pragma unroll
    for (int s = 0; s < WSLOTS; ++s) {
      const int p = wave + NW * s;
      if (p < WPIECES) dma16(sb + p * 1024, wrs, wsrc[s], __builtin_amdgcn_readfirstlane(ks * kKStep));
    }
    const int tapoff = (kr * a.w + kc) * a.cin + c0;
#pragma unroll
    for (int s = 0; s < ASLOTS; ++s) {
      const int p = wave + NW * s;
      if (p < APIECES) {
        const int l = p / (BP / 16);
        const bool ok = (unsigned)(aih[s] + kr) < (unsigned)a.h && (unsigned)(aiw[s] + kc) < (unsigned)a.w;
        const unsigned voff = ok ? (unsigned)(apix[s] + tapoff) : kOOB;
        dma16(sb + (WPIECES + p) * 1024, xrs, voff,
              __builtin_amdgcn_readfirstlane((unsigned)((long long)l * a.plane)));
      }
    }
  };

  v4i acc[NACC][WC][WP];
#pragma unroll
  for (int s = 0; s < NACC; ++s)
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) acc[s][i][j] = v4i{0, 0, 0, 0};
  const bool do_off = (LW == 1) && a.has_offset;
  int rs[L][WP];  // per-lane partial pixel sums of activation codes (LW == 1 offset correction)
#pragma unroll
  for (int l = 0; l < L; ++l)
#pragma unroll
    for (int j = 0; j < WP; ++j) rs[l][j] = 0;

  // fragment read offset inside a piece (same for every piece)
  const int frow = lane & 15;
  const int rd = frow * 64 + 16 * ((lane >> 4) ^ swz(frow));

  int kr = 0, kc = 0, c0 = 0;
  issue(0, 0, 0, 0, 0);
  for (int ks = 0; ks < a.ksteps; ++ks) {
    const int buf = ks & 1;
    // this wave's DMA of step ks has landed and its reads of step ks-1 are done; after the
    // barrier every wave's are, so stage ks is readable and stage ks-1 may be refilled
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int8_t* sb = lds + buf * STAGE;
    v4i wf[LW][WC], af[L][WP];
#pragma unroll
    for (int lw = 0; lw < LW; ++lw)
#pragma unroll
      for (int i = 0; i < WC; ++i)
        wf[lw][i] = *reinterpret_cast<const v4i*>(sb + (lw * (BC / 16) + wc * WC + i) * 1024 + rd);
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int j = 0; j < WP; ++j)
        af[l][j] = *reinterpret_cast<const v4i*>(sb + (WPIECES + l * (BP / 16) + wp * WP + j) * 1024 + rd);
    // advance the K position and start the next step's DMA into the other stage
    c0 += kKStep;
    if (c0 == a.cin) {
      c0 = 0;
      if (++kc == a.kw) {
        kc = 0;
        ++kr;
      }
    }
    if (ks + 1 < a.ksteps) issue(buf ^ 1, kr, kc, c0, ks + 1);
    if (do_off) {
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          int s = rs[l][j];
          s = __builtin_amdgcn_sdot4(af[l][j].x, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(af[l][j].y, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(af[l][j].z, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(af[l][j].w, 0x01010101, s, false);
          rs[l][j] = s;
        }
    }
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int lw = 0; lw < LW; ++lw) {
        if (l + lw < SMIN) continue;  // compile-time: skipped low-digit product
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j)
            acc[l + lw - SMIN][i][j] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(wf[lw][i], af[l][j], acc[l + lw - SMIN][i][j], 0, 0, 0);
      }
  }

  // ---- epilogue: straight from the accumulators --------------------------------------------
  // lane: channels ch(i) + r (r = 0..3) of pixel m(j)
  if (do_off) {
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        int s = rs[l][j];
        s += __shfl_xor(s, 16, kWave);
        s += __shfl_xor(s, 32, kWave);
        rs[l][j] = s;
      }
  }
  int mrow[WP];
  float rscale[WP];
  bool mok[WP];
#pragma unroll
  for (int j = 0; j < WP; ++j) {
    const int m = m0 + (wp * WP + j) * 16 + frow;
    mok[j] = m < a.M;
    mrow[j] = mok[j] ? m : 0;
    rscale[j] = mok[j] ? a.x_absmax[m / hw_out] * a.inv_qmax : 0.f;
  }
  int chan[WC];
  bool cok[WC];
  float4 cs[WC], csh[WC];
  int4 coff[WC];
#pragma unroll
  for (int i = 0; i < WC; ++i) {
    chan[i] = n0 + (wc * WC + i) * 16 + 4 * (lane >> 4);
    cok[i] = chan[i] < a.cout;  // cout % 16 == 0: the 4 channels are valid together
    const int c = cok[i] ? chan[i] : 0;
    cs[i] = *reinterpret_cast<const float4*>(a.col_scale + c);
    csh[i] = *reinterpret_cast<const float4*>(a.col_shift + c);
    coff[i] = do_off ? *reinterpret_cast<const int4*>(a.w_off + c) : int4{0, 0, 0, 0};
  }

  // residual: all loads issued before any use
  const long long oplane = (long long)a.M * a.cout;
  int rq[WC][WP][L];
  float4 rf[WC][WP];
  if (a.res_q) {
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.res_q), 0, (int)(L * oplane),
                                                       0x00020000);
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        const unsigned off = (mok[j] && cok[i]) ? (unsigned)(mrow[j] * a.cout + chan[i]) : kOOB;
#pragma unroll
        for (int l = 0; l < L; ++l)
          rq[i][j][l] = (int)__builtin_amdgcn_raw_buffer_load_b32(rrs, off, (unsigned)((long long)l * oplane), 0);
      }
  } else if (a.residual) {
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.residual), 0, (int)(4 * oplane),
                                                       0x00020000);
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        const unsigned off = (mok[j] && cok[i]) ? (unsigned)(4 * (mrow[j] * a.cout + chan[i])) : kOOB;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rrs, off, 0, 0);
        rf[i][j] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                               __uint_as_float(v[3]));
      }
  }

  constexpr float qmax = act_qmax<L>();
  float vmax = 0.f;  // max |y| over this lane's valid outputs (static-range overflow test)
  float pmax[WP];    // per-pixel max |y| (dynamic per-image range)
#pragma unroll
  for (int j = 0; j < WP; ++j) pmax[j] = 0.f;
#pragma unroll
  for (int i = 0; i < WC; ++i) {
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const bool ok = mok[j] && cok[i];
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int rsum[L];
#pragma unroll
        for (int l = 0; l < L; ++l) rsum[l] = rs[l][j];
        const int co = r == 0 ? coff[i].x : (r == 1 ? coff[i].y : (r == 2 ? coff[i].z : coff[i].w));
        float v = 0.f;
        float limbw = SMIN == 0 ? 1.f : (SMIN == 1 ? 256.f : 65536.f);
#pragma unroll
        for (int s = 0; s < NACC; ++s) {
          int tq = acc[s][i][j][r];
          if (SMIN == 0 && s < L && do_off) tq += co * rsum[s];
          v = __fmaf_rn((float)tq, limbw, v);
          limbw *= 256.f;
        }
        const float csr = r == 0 ? cs[i].x : (r == 1 ? cs[i].y : (r == 2 ? cs[i].z : cs[i].w));
        const float shr = r == 0 ? csh[i].x : (r == 1 ? csh[i].y : (r == 2 ? csh[i].z : csh[i].w));
        float out = affine(v, rscale[j], csr, shr);
        if (a.res_q) {
          int q = 0;
#pragma unroll
          for (int l = L - 1; l >= 0; --l) q = q * 256 + __builtin_amdgcn_sbfe(rq[i][j][l], 8 * r, 8);
          out = __fadd_rn(out, __fmul_rn(a.res_scale, (float)q));
        } else if (a.residual) {
          const float rv = r == 0 ? rf[i][j].x : (r == 1 ? rf[i][j].y : (r == 2 ? rf[i][j].z : rf[i][j].w));
          out = __fadd_rn(out, rv);
        }
        if (a.relu) out = fmaxf(out, 0.f);
        o[r] = out;
      }
      if (ok) {
        const float am = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3])));
        pmax[j] = fmaxf(pmax[j], am);
        vmax = fmaxf(vmax, am);
      }
      const long long oidx = (long long)mrow[j] * a.cout + chan[i];
      if (a.y && ok) *reinterpret_cast<float4*>(a.y + oidx) = make_float4(o[0], o[1], o[2], o[3]);
      if (a.yq && ok) {
        int q[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = (int)fminf(fmaxf(rintf(__fmul_rn(o[r], a.yq_inv)), -qmax), qmax);
        unsigned wd[L];
        if constexpr (L >= 1) wd[0] = pack_bytes(q[0], q[1], q[2], q[3], 0);
        if constexpr (L >= 2)
          wd[1] = pack_bytes(digit_src<1>(q[0]), digit_src<1>(q[1]), digit_src<1>(q[2]), digit_src<1>(q[3]), 1);
        if constexpr (L >= 3)
          wd[2] = pack_bytes(digit_src<2>(q[0]), digit_src<2>(q[1]), digit_src<2>(q[2]), digit_src<2>(q[3]), 2);
#pragma unroll
        for (int l = 0; l < L; ++l) *reinterpret_cast<unsigned*>(a.yq + l * oplane + oidx) = wd[l];
      }
    }
  }
  if (a.yq) {
    const bool ovf = rintf(__fmul_rn(vmax, a.yq_inv)) > qmax;
    if (__any(ovf) && lane == 0) atomicMax(a.overflow, 1);
  }
  if (a.y_absmax) {
    // per pixel: reduce over the 4 lane groups holding its channels
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      pmax[j] = fmaxf(pmax[j], __shfl_xor(pmax[j], 16, kWave));
      pmax[j] = fmaxf(pmax[j], __shfl_xor(pmax[j], 32, kWave));
    }
    const int mfirst = m0 + wp * WP * 16;
    const int mlast = min(mfirst + WP * 16, a.M) - 1;
    if (mfirst <= mlast) {
      const int img_lo = mfirst / hw_out, img_hi = mlast / hw_out;
      if (img_lo == img_hi) {
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < WP; ++j) v = fmaxf(v, pmax[j]);
        v = wave_max(v);
        if (lane == 0 && v > 0.f) atomic_max_nonneg(&a.y_absmax[img_lo], v);
      } else if (lane < 16) {
#pragma unroll
        for (int j = 0; j < WP; ++j)
          if (mok[j] && pmax[j] > 0.f) atomic_max_nonneg(&a.y_absmax[mrow[j] / hw_out], pmax[j]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
struct GldsCfg {
  int wavesc, wavesp, wc, wp;
};
constexpr GldsCfg kGlds[] = {
    {2, 2, 2, 2},  // 0:  64 ch x  64 px, 256 threads
    {2, 2, 2, 4},  // 1:  64 ch x 128 px
    {2, 2, 4, 2},  // 2: 128 ch x  64 px
    {1, 4, 4, 1},  // 3:  64 ch x  64 px (each wave all 64 channels of 16 px)
    {1, 4, 4, 2},  // 4:  64 ch x 128 px
    {4, 1, 2, 4},  // 5: 128 ch x  64 px (each wave 32 ch x all 64 px)
    {2, 2, 4, 4},  // 6: 128 ch x 128 px (<= 2 accumulator sets)
};
constexpr int kNumGlds = sizeof(kGlds) / sizeof(kGlds[0]);

int glds_num_cfgs() { return kNumGlds; }

void glds_cfg_info(int cfg, int* bm, int* bn, int* threads) {
  const GldsCfg& c = kGlds[cfg];
  *bm = 16 * c.wp * c.wavesp;  // pixels (GEMM rows)
  *bn = 16 * c.wc * c.wavesc;  // channels
  *threads = 64 * c.wavesc * c.wavesp;
}

template <int L, int LW, int WAVES_C, int WAVES_P, int WC, int WP>
static int launch_one(const ConvArgs& a, hipStream_t stream) {
  constexpr int SMIN = (L + LW - 4) > 0 ? (L + LW - 4) : 0;
  if constexpr ((L + LW - 1 - SMIN) * WC * WP * 4 > 128) {
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: tile config too large for these limb counts");
  } else {
    constexpr int BC = 16 * WC * WAVES_C, BP = 16 * WP * WAVES_P;
    const long mt = (a.M + BP - 1) / BP;
    const long nt = (a.cout + BC - 1) / BC;
    if (mt * nt > 0x7fffffffL) return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: grid too large");
    hipLaunchKernelGGL((qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, 2>), dim3((unsigned)(mt * nt)),
                       dim3(64 * WAVES_C * WAVES_P), 0, stream, a);
    return check_hip(hipGetLastError(), "qconv_glds_kernel launch");
  }
}

template <int L, int LW>
static int launch_cfg(int cfg, const ConvArgs& a, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_one<L, LW, 2, 2, 2, 2>(a, s);
    case 1: return launch_one<L, LW, 2, 2, 2, 4>(a, s);
    case 2: return launch_one<L, LW, 2, 2, 4, 2>(a, s);
    case 3: return launch_one<L, LW, 1, 4, 4, 1>(a, s);
    case 4: return launch_one<L, LW, 1, 4, 4, 2>(a, s);
    case 5: return launch_one<L, LW, 4, 1, 2, 4>(a, s);
    case 6: return launch_one<L, LW, 2, 2, 4, 4>(a, s);
    default: return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: bad tile config");
  }
}

int launch_glds(int cfg, int limbs, int wlimbs, const ConvArgs& a, hipStream_t s) {
  // operand and output planes are addressed with 32-bit buffer offsets below kOOB
  const long long lim = 0x7fffff00LL;
  if (a.cin % kKStep != 0 || a.cout % 16 != 0 || (long long)limbs * a.plane > lim ||
      (long long)wlimbs * a.wplane > lim || (long long)limbs * a.M * a.cout > lim ||
      (a.residual && 4LL * a.M * a.cout > lim))
    return fail(SMPQ_E_INVALID,
                "smpq_conv2d_fwd: LDS-DMA tile configs need cin % 64 == 0, cout % 16 == 0 and planes < 2 GiB");
  if (wlimbs == 1) {
    switch (limbs) {
      case 1: return launch_cfg<1, 1>(cfg, a, s);
      case 2: return launch_cfg<2, 1>(cfg, a, s);
      default: return launch_cfg<3, 1>(cfg, a, s);
    }
  }
  if (wlimbs == 3) return launch_cfg<3, 3>(cfg, a, s);
  switch (limbs) {
    case 1: return launch_cfg<1, 2>(cfg, a, s);
    case 2: return launch_cfg<2, 2>(cfg, a, s);
    default: return launch_cfg<3, 2>(cfg, a, s);
  }
}

}  // namespace smpq
