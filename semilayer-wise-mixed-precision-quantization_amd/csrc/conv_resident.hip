// Weight-stationary 1x1 conv tiles for gfx950 (round 6; tile kind SMPQ_TILE_RESIDENT1X1): the
// 1x1 convs with ONE 64-wide K step and 256 output channels whose epilogue only emits the next
// conv's limb planes — in the R50 forward the downsample of layer1[0] (resnet.py:188-192: conv1x1
// 64 -> 256 + BN, 24-bit fixed-point weights, 6 MFMA passes) — where the LDS-DMA kernel spends most
// of its staging on the weights: a 128 x 32 tile re-stages 24 KB of weight limbs for 6 KB of
// activations, 50,176 times per 256 images.
//
// Here a persistent workgroup (4 waves, wave w = output channels 64 w .. 64 w + 63) loads every
// weight limb ONCE, straight into VGPRs (LW x 4 A fragments per wave: each lane's 16 bytes are one
// buffer load), and walks pixel tiles of BP pixels (tile b, b + grid, b + 2 grid, ...): the activation tile of
// tile t + 1 is DMA'd into the other of two LDS stages while tile t's MFMAs and epilogue run; the
// epilogue is the lean static-range epilogue of the LDS-DMA kernel (lean_quad: limb recombination,
// folded BN, optional ReLU, rounding, clamp, digit encode), staged in LDS as a [L][BP][256] tile and
// copied out as whole 256-B pixel rows. Integer accumulation is exact and the epilogue is the same
// function, so the outputs and the overflow flag are bitwise those of every other tile config
// (tests/test_gpu_resident.py).
#include "conv_common.h"
#include "lds_dma.h"

namespace smpq {

namespace {

struct ResCfg {
  int bp;  // pixels per tile (16 x WP)
};
constexpr ResCfg kRes[] = {{32}, {16}};
constexpr int kNumRes = sizeof(kRes) / sizeof(kRes[0]);
constexpr int kResCout = 256;  // output channels (all of them per workgroup: 4 waves x 64)
constexpr int kResThreads = 256;

// MINW: workgroups per CU the register budget is compiled for (one wave per SIMD each)
template <int L, int LW, int WP, bool RELU, int MINW>
__global__ __launch_bounds__(kResThreads, MINW) void qconv_resident_kernel(ConvArgs a, int ntiles) {
  constexpr int SMIN = (L + LW - 4) > 0 ? (L + LW - 4) : 0;
  constexpr int NACC = L + LW - 1 - SMIN;
  constexpr int WC = 4;                       // 16-channel blocks per wave
  constexpr int BP = 16 * WP;                 // pixels per tile
  constexpr int ASTAGE = L * BP * 64;         // activation tile bytes
  constexpr int APIECES = L * BP / 16;        // 1-KiB DMA pieces per activation tile
  constexpr int OTILE = L * BP * kResCout;    // staged output tile bytes
  constexpr float qmax = act_qmax<L>();
  extern __shared__ __attribute__((aligned(1024))) int8_t lds[];  // 2 activation stages + the output tile
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15;
  const int rd = frow * 64 + 16 * ((lane >> 4) ^ swz<64>(frow));  // fragment read offset in a 16-row block
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  int8_t* const astage = lds;
  int8_t* const otile = lds + 2 * ASTAGE;

  // ---- the weight limbs -> VGPRs once: A fragment (lw, i) of lane (g, p) = the 16 bytes of K chunk
  // g of output channel 16 (4 wave + i) + p (row-major [LW][256][64] = the K-major layout at K 64)
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.codes), 0, (int)(LW * a.wplane), 0x00020000);
  v4i wa[LW][WC];
#pragma unroll
  for (int lw = 0; lw < LW; ++lw)
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const v4u v = __builtin_amdgcn_raw_buffer_load_b128(
          wrs, (unsigned)(((wave * WC + i) * 16 + frow) * 64 + 16 * (lane >> 4)), (unsigned)(lw * a.wplane), 0);
      wa[lw][i] = v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
    }
  const int prow = lane >> 2;                        // row inside a 1-KiB DMA piece
  const int pchunk = (lane & 3) ^ swz<64>(prow);     // logical K chunk this lane fetches
  // per-lane activation source: pixel m's 64 channels (1x1, any stride) of limb l
  const v4i xrs = make_rsrc(a.xq, (long long)L * a.plane);
  const int hw_out = a.ho * a.wo;
  auto act_src = [&](int m) -> unsigned {  // byte offset of pixel m's channel chunk pchunk in plane 0
    if (m >= a.M) return kOOB;
    const int img = fast_div(m, a.hw_mul, a.hw_shr);
    const int rem = m - img * hw_out;
    const int oh = fast_div(rem, a.wo_mul, a.wo_shr), ow = rem - oh * a.wo;
    return (unsigned)(((img * a.h + oh * a.stride) * a.w + ow * a.stride) * 64 + 16 * pchunk);
  };
  auto issue_acts = [&](int t, int stage) {  // this wave's pieces of tile t's activation tile
    for (int p = wave; p < APIECES; p += 4) {
      const int l = p / (BP / 16), rb = (p % (BP / 16)) * 16;
      const unsigned src = act_src(t * BP + rb + prow);
      dma16(lds0 + stage * ASTAGE + p * 1024, xrs, src,
            __builtin_amdgcn_readfirstlane((unsigned)((long long)l * a.plane)));
    }
  };
  int t = blockIdx.x;
  if (t < ntiles) issue_acts(t, 0);

  // ---- epilogue constants of this lane's channels -----------------------------------------------
  const float inv = a.yq_inv;
  float csq[WC][4], shq[WC][4];
#pragma unroll
  for (int i = 0; i < WC; ++i) {
    const int c = (wave * WC + i) * 16 + 4 * (lane >> 4);
    const float4 cs = *reinterpret_cast<const float4*>(a.col_scale + c);
    const float4 csh = *reinterpret_cast<const float4*>(a.col_shift + c);
    csq[i][0] = cs.x * inv, csq[i][1] = cs.y * inv, csq[i][2] = cs.z * inv, csq[i][3] = cs.w * inv;
    shq[i][0] = csh.x * inv, shq[i][1] = csh.y * inv, shq[i][2] = csh.z * inv, shq[i][3] = csh.w * inv;
  }
  const float lo = RELU ? 0.f : -qmax;
  const long long oplane = (long long)a.M * kResCout;
  const v4i qrs4 = make_rsrc(a.yq, (long long)L * oplane);
  const bool nt = __builtin_amdgcn_readfirstlane(a.nt_store) != 0;
  float vmax = 0.f;

  int stage = 0;
  for (; t < ntiles; t += gridDim.x) {
    const int m0 = t * BP;
    // tile t's activations have landed (this wave's pieces; the barrier: every wave's), and every
    // wave is past the previous tile's copy-out, so the output tile may be rewritten below
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    v4i fb[L][WP];
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int j = 0; j < WP; ++j)
        fb[l][j] = *reinterpret_cast<const v4i*>(astage + stage * ASTAGE + (l * BP + j * 16) * 64 + rd);
    if (t + (int)gridDim.x < ntiles) issue_acts(t + gridDim.x, stage ^ 1);  // under this tile's work
    v4i acc[NACC][WC][WP];
#pragma unroll
    for (int s = 0; s < NACC; ++s)
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j) acc[s][i][j] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int lw = 0; lw < LW; ++lw) {
        if (l + lw < SMIN) continue;  // compile-time: skipped low-digit product (as the LDS-DMA kernel)
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j)
            acc[l + lw - SMIN][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wa[lw][i], fb[l][j], acc[l + lw - SMIN][i][j], 0, 0, 0);
      }
    // lean epilogue -> the [L][BP][256] output tile in LDS (row = pixel, 16-B chunk c of a row at
    // c ^ swze<256>(row & 15): conflict-free, as the LDS-DMA kernel's staged tiles)
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const int m = m0 + j * 16 + frow;
      const float rscale = m < a.M ? a.x_absmax[fast_div(m, a.hw_mul, a.hw_shr)] * a.inv_qmax : 0.f;
#pragma unroll
      for (int i = 0; i < WC; ++i) {
        v4i accq[NACC];
#pragma unroll
        for (int s = 0; s < NACC; ++s) accq[s] = acc[s][i][j];
        unsigned wq[L];
        const float mm = lean_quad<L, NACC, SMIN>(accq, rscale, csq[i], shq[i], false, nullptr, 0.f, RELU, lo, wq);
        vmax = m < a.M ? fmaxf(vmax, mm) : vmax;
        const int rt = j * 16 + frow, cc = wave * WC + i;
#pragma unroll
        for (int l = 0; l < L; ++l)
          *reinterpret_cast<unsigned*>(otile + l * BP * kResCout + rt * kResCout + 16 * (cc ^ swze<kResCout>(frow)) +
                                       4 * (lane >> 4)) = wq[l];
      }
    }
    __syncthreads();
    // copy-out: whole 256-B pixel rows, 16 B per lane
    constexpr int ITEMS = OTILE / 16;
#pragma unroll
    for (int k = 0; k < (ITEMS + kResThreads - 1) / kResThreads; ++k) {
      const int it = threadIdx.x + kResThreads * k;
      if (ITEMS % kResThreads == 0 || it < ITEMS) {
        const int l = it / (BP * 16), rem = it - l * (BP * 16);
        const int rt = rem >> 4, c = rem & 15;
        const v4i v = *reinterpret_cast<const v4i*>(otile + l * BP * kResCout + rt * kResCout +
                                                     16 * (c ^ swze<kResCout>(rt & 15)));
        const unsigned off = m0 + rt < a.M ? (unsigned)((long long)(m0 + rt) * kResCout + 16 * c) : kOOB;
        store_limbs16(v4u{(unsigned)v.x, (unsigned)v.y, (unsigned)v.z, (unsigned)v.w}, qrs4, off,
                      __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane)), nt);
      }
    }
    stage ^= 1;
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

template <int L, int LW, int WP, bool RELU>
int launch_res_one(const ConvArgs& a, hipStream_t s) {
  constexpr int BP = 16 * WP;
  constexpr int lds_bytes = 2 * L * BP * 64 + L * BP * kResCout;
  // the register budget (one wave per SIMD per workgroup): 3 workgroups per CU where the
  // accumulators allow it (<= 168 VGPRs), else 2
  constexpr int MINW = (L + LW - 1 - ((L + LW - 4) > 0 ? (L + LW - 4) : 0)) * 4 * WP * 4 <= 48 ? 3 : 2;
  static_assert(MINW * lds_bytes <= 160 * 1024, "LDS per CU");
  auto k = qconv_resident_kernel<L, LW, WP, RELU, MINW>;
  static const hipError_t attr = [&] {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
  }();
  if (attr != hipSuccess) return check_hip(attr, "qconv_resident_kernel LDS attribute");
  const long long ntiles = ((long long)a.M + BP - 1) / BP;
  if (ntiles > 0x7fffffffLL) return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: grid too large");
  // persistent: as many workgroups as fit the CUs at once, at most one per tile
  long long blocks = (long long)device_cus_res() * MINW;
  if (blocks > ntiles) blocks = ntiles;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(kResThreads), lds_bytes, s, a, (int)ntiles);
  return check_hip(hipGetLastError(), "qconv_resident_kernel launch");
}

template <int L, int LW, bool RELU>
int launch_res_l(int cfg, const ConvArgs& a, hipStream_t s) {
  return kRes[cfg].bp == 16 ? launch_res_one<L, LW, 1, RELU>(a, s) : launch_res_one<L, LW, 2, RELU>(a, s);
}

}  // namespace

int resident_num_cfgs() { return kNumRes; }

void resident_cfg_info(int cfg, int* bm, int* bn, int* threads) {
  *bm = kRes[cfg].bp;
  *bn = kResCout;
  *threads = kResThreads;
}

// What tile_supported can see; the launcher also needs pad 0, no weight offsets and the
// static-range limb-plane epilogue without a residual (yq set; y, y_absmax, residual, residual_q NULL).
bool resident_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs) {
  if (cfg < 0 || cfg >= kNumRes) return false;
  return kh == 1 && kw == 1 && cin == 64 && cout == kResCout && limbs == 3 && (wlimbs == 1 || wlimbs == 3);
}

int launch_resident(int cfg, int limbs, int wlimbs, const ConvArgs& a, hipStream_t s) {
  if (!resident_supported(cfg, a.cin, a.cout, a.kh, a.kw, limbs, wlimbs) || a.pad != 0 || a.s2d)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tiles take 1x1 / pad 0 convs with cin 64, cout 256, "
                                "3 activation limbs and 1 or 3 weight limbs");
  if (!a.yq || a.y || a.residual || a.res_q || a.y_absmax || a.has_offset)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: resident tiles run the static-range limb-plane epilogue without "
                                "a residual or weight offsets only");
  if (wlimbs == 3) return a.relu ? launch_res_l<3, 3, true>(cfg, a, s) : launch_res_l<3, 3, false>(cfg, a, s);
  return a.relu ? launch_res_l<3, 1, true>(cfg, a, s) : launch_res_l<3, 1, false>(cfg, a, s);
}

}  // namespace smpq
