// Halo-patch 3x3 quantized conv (stride 1, pad 1) for gfx950: the static-range ("lean") forward of
// the quantized conv2 of BasicBlock / Bottleneck (resnet.py:22-25, 55-68, 97-116), bitwise equal to
// qconv_glds_kernel (conv_glds_kernel.h) on the same inputs.
//
// Why a second kernel for the 3x3 convs: the implicit GEMM stages the activation operand once per
// TAP — every input pixel crosses L2 -> LDS nine times (3 limbs each), and for the 64- and
// 128-channel 3x3 convs of the early layers that operand traffic, not the matrix cores, bounds
// the kernel (tools/batch_scaling.py). Here a block owns TH x TW output pixels of one
// image and 64 output channels; per 64-channel input chunk it stages
//   * the (TH + 2) x (TW + 2) input patch of every activation limb ONCE (LDS-DMA, 64 B per pixel),
//   * the chunk's weights of all nine taps ([tap][64 couts][64 B], from the K-major codes),
// and runs the nine taps out of LDS: tap (kr, kc) of pixel (r, c) is patch pixel (r + kr, c + kc),
// so a lane's B-fragment address is a per-lane base plus a compile-time offset per tap and limb.
// Operand bytes per output pixel and chunk fall from 9 * L * 64 to about (TH+2)(TW+2)/(TH*TW) * L * 64.
//
//  * Fragments: pixel fragment f of the block = tile pixels 16 f .. 16 f + 15 in row-major tile
//    order (2 rows x 8 columns at TW = 8, 4 x 4 at TW = 4); the MFMA is v_mfma_i32_16x16x64_i8 with
//    A = weights (16 couts x 64 K), B = activations (64 K x 16 pixels) as in qconv_glds_kernel, so
//    a lane ends with 4 consecutive output channels of one pixel and the epilogue is that kernel's.
//  * LDS patch image: pixel (pr, pc) of limb l at l * PH * PW * 64 + (pr * PW + pc) * 64, its 16-B
//    chunk c stored at c ^ 2 * (pr & 1): with the gfx950 ds_read_b128 lane groups this is
//    conflict-free for every tap of 2 x 8 and 4 x 4 fragments (checked exhaustively by
//    tools/halo_conflicts.py), and the row parity of a tap only flips the XOR, so each lane keeps
//    two bases (even / odd kr). The weight image is the implicit-GEMM kernel's (swz<64>).
//  * Stages: NST = 1 refills the single stage after a barrier per chunk (two blocks per CU overlap
//    each other's loads); NST = 2 prefetches chunk k + 1 during chunk k.
#include <type_traits>

#include "lds_dma.h"

namespace smpq {

struct HaloCfg {
  int th, tw, nwv, wpf, nst;  // tile rows x cols, waves, pixel fragments per wave, LDS stages
};
// tile = th x tw pixels of one image x 64 output channels; ceil(th * tw / 16) == nwv * wpf
constexpr HaloCfg kHalo[] = {
    {8, 8, 4, 1, 1},    // 0: 64 px   (56^2; 28^2 with a partial column tile)
    {16, 8, 8, 1, 1},   // 1: 128 px, 8 waves
    {16, 8, 4, 2, 1},   // 2: 128 px, 4 waves x 2 fragments
    {28, 4, 7, 1, 1},   // 3: 112 px  (28^2: whole columns of 4)
    {14, 4, 4, 1, 1},   // 4: 56 px   (28^2)
    {8, 8, 4, 1, 2},    // 5: as 0, chunk k + 1 prefetched
    {28, 4, 7, 1, 2},   // 6: as 3, prefetched
    {16, 8, 4, 2, 2},   // 7: as 2, prefetched
    {7, 14, 7, 1, 1},   // 8: 98 px   (14^2: half an image)
    {7, 14, 7, 1, 2},   // 9: as 8, prefetched
};
constexpr int kNumHalo = sizeof(kHalo) / sizeof(kHalo[0]);

namespace {

constexpr int kHaloWB = 9 * 64 * 64;  // weight image per stage: [tap][64 couts][64 B]

// the residual tile staged in LDS (RES): [L][16 ceil(px / 16)][64] limb bytes
__host__ __device__ constexpr int halo_res_bytes(int L, int th, int tw) { return L * ((th * tw + 15) / 16) * 1024; }
__host__ __device__ constexpr int halo_patch_bytes(int L, int th, int tw) {
  return (L * (th + 2) * (tw + 2) * 64 + 1023) / 1024 * 1024;  // whole DMA pieces
}

template <int L, int TH, int TW, int NWV, int WPF, int NST, bool OFF, bool RES>
__global__ __launch_bounds__(64 * NWV) void qconv_halo_kernel(ConvArgs a, int nct, int ntw, int tiles_img) {
  constexpr int PH = TH + 2, PW = TW + 2;
  constexpr int NPIX = TH * TW;
  constexpr int NF = NWV * WPF;
  static_assert(NF * 16 >= NPIX && NF * 16 < NPIX + 16, "fragments cover the tile");
  constexpr int PLIMB = PH * PW * 64;
  constexpr int PB = halo_patch_bytes(L, TH, TW);
  constexpr int STAGE = kHaloWB + PB;
  constexpr int PPIECE = PB / 1024;       // patch pieces; + 9 taps x 4 blocks of 16 couts of weights
  constexpr int WSL = (36 + NWV - 1) / NWV, PSL = (PPIECE + NWV - 1) / NWV;
  extern __shared__ __attribute__((aligned(1024))) int8_t lds[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < NWV);
  const int frow = lane & 15, grp = lane >> 4;

  // ---- tile: XCD-aware order (consecutive logical tiles share an XCD's L2: the channel tiles of
  // one patch, then the neighbouring patches whose halos overlap) ------------------------------
  const int total = gridDim.x, bid = blockIdx.x;
  const int full = total & ~7;
  int t = bid;
  if (t < full) t = (t & 7) * (full >> 3) + (t >> 3);
  const int ct = t % nct, s = t / nct;
  const int img = s / tiles_img, rem = s - img * tiles_img;
  const int tr = rem / ntw, tc = rem - tr * ntw;
  const int oh0 = tr * TH, ow0 = tc * TW;
  const int nch = a.cin / 64;

  const v4i wrs = make_rsrc(a.codes, a.wplane);
  const v4i xrs = make_rsrc(a.xq, (long long)L * a.plane);

  // ---- per-lane DMA sources (fixed over the chunks; the chunk moves the scalar offset) ---------
  // weight piece p = wave + NWV k (< 36): tap p / 4, couts 16 (p % 4) .. +15 of this channel tile;
  // patch piece q = wave + NWV k (< PPIECE): LDS bytes [1024 q, +1024) of the [L][PH][PW][64]
  // image, i.e. pixels 16 q .. 16 q + 15 (4 lanes per pixel). Patch coordinates advance
  // incrementally from piece to piece (no division per piece); offsets are 32-bit (every operand
  // plane is below 2 GiB, glds_planes_ok).
  unsigned wsrc[WSL], psrc[PSL];
  {
    const int row = lane >> 2;
    const int lc = (lane & 3) ^ swz<64>(row);
    const unsigned rowoff = a.w_kmajor ? (unsigned)((ct * 64 + row) * 64 + 16 * lc)
                                       : (unsigned)((ct * 64 + row) * a.K + 16 * lc);
    const unsigned tapstride = a.w_kmajor ? (unsigned)(nch * a.cout * 64) : (unsigned)a.cin;
    const unsigned blkstride = a.w_kmajor ? 16u * 64u : 16u * (unsigned)a.K;
#pragma unroll
    for (int k = 0; k < WSL; ++k) {
      const int p = wave + NWV * k;
      wsrc[k] = p < 36 ? rowoff + (unsigned)(p >> 2) * tapstride + (unsigned)(p & 3) * blkstride : kOOB;
    }
  }
  {
    constexpr int D = 16 * NWV;                     // pixels between a wave's consecutive pieces
    constexpr int DL = D / (PH * PW), DR = (D % (PH * PW)) / PW, DC = D % PW;
    int P = 16 * wave + (lane >> 2);                // this lane's pixel in the wave's first piece
    int l = P / (PH * PW);
    int pr = (P - l * (PH * PW)) / PW;
    int pc = P - l * (PH * PW) - pr * PW;
    const int c16 = 16 * (lane & 3);
    const int wcin = a.w * a.cin;
    const int q0 = ((img * a.h + oh0 - 1) * a.w + ow0 - 1) * a.cin;  // patch pixel (0, 0); may be < 0
    const int h1 = a.h - oh0 + 1, w1 = a.w - ow0 + 1;               // pr < h1 <=> ih < h
    const unsigned plane = (unsigned)a.plane;
#pragma unroll
    for (int k = 0; k < PSL; ++k) {
      const int q = wave + NWV * k;
      const bool ok = q < PPIECE && l < L && pr >= 1 - oh0 && pr < h1 && pc >= 1 - ow0 && pc < w1;
      psrc[k] = ok ? (unsigned)l * plane + (unsigned)(q0 + pr * wcin + pc * a.cin + (c16 ^ (32 * (pr & 1)))) : kOOB;
      pc += DC;
      pr += DR;
      if (pc >= PW) {
        pc -= PW;
        ++pr;
      }
      l += DL;
      if (pr >= PH) {
        pr -= PH;
        ++l;
      }
    }
  }
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  const unsigned wchunk = __builtin_amdgcn_readfirstlane(a.w_kmajor ? (unsigned)(a.cout * 64) : 64u);
  auto issue = [&](int cc, int stage) {
    const unsigned sb = lds0 + stage * STAGE;
#pragma unroll
    for (int k = 0; k < WSL; ++k)
      if (wave + NWV * k < 36)
        dma16(sb + (wave + NWV * k) * 1024, wrs, wsrc[k], __builtin_amdgcn_readfirstlane((unsigned)cc * wchunk));
#pragma unroll
    for (int k = 0; k < PSL; ++k)
      if (wave + NWV * k < PPIECE)
        dma16(sb + kHaloWB + (wave + NWV * k) * 1024, xrs, psrc[k], __builtin_amdgcn_readfirstlane((unsigned)cc * 64u));
  };

  // ---- per-lane fragment bases --------------------------------------------------------------
  const int wrd = frow * 64 + 16 * (grp ^ swz<64>(frow));  // A: + tap * 4096 + i * 1024
  int bpar[WPF][2];  // B: + l * PLIMB + (kr * PW + kc) * 64; [1] for odd kr
  int pr0[WPF], pc0[WPF];
#pragma unroll
  for (int j = 0; j < WPF; ++j) {
    const int pt = 16 * (wave * WPF + j) + frow;
    const int r = pt < NPIX ? pt / TW : 0, c = pt < NPIX ? pt - (pt / TW) * TW : 0;
    pr0[j] = pt < NPIX ? r : -1;
    pc0[j] = c;
#pragma unroll
    for (int par = 0; par < 2; ++par) bpar[j][par] = kHaloWB + (r * PW + c) * 64 + 16 * (grp ^ (2 * ((r + par) & 1)));
  }

  // RES: the limb-plane residual (BasicBlock conv2: + identity, then ReLU) — each lane's 4-channel
  // words of its pixels, loaded now and decoded in the epilogue (latency under the K loop)
  const long long oplane = (long long)a.M * a.cout;
  unsigned qoff[WPF];
#pragma unroll
  for (int j = 0; j < WPF; ++j) {
    const int oh = oh0 + pr0[j], ow = ow0 + pc0[j];
    const bool ok = pr0[j] >= 0 && oh < a.ho && ow < a.wo;
    qoff[j] = ok ? (unsigned)(((long long)(img * a.ho + oh) * a.wo + ow) * a.cout + ct * 64 + 16 * grp) : kOOB;
  }
  // the residual tile by LDS-DMA (whole 64-B pixel rows; when it fits beside the stages), else
  // each lane's 4-channel words by buffer loads
  constexpr int RPP = (NPIX + 15) / 16;  // 16-pixel pieces per limb
  constexpr bool RES_LDS = RES && NST * (kHaloWB + PB) + halo_res_bytes(L, TH, TW) <= 160 * 1024;
  const unsigned resoff = (unsigned)((nch < NST ? nch : NST) * STAGE);
  unsigned rqw[RES ? 4 : 1][WPF][RES ? L : 1];
  if constexpr (RES_LDS) {
    const v4i rrs = make_rsrc(a.res_q, (long long)L * oplane);
    const unsigned lds0r = __builtin_amdgcn_readfirstlane(lds_addr(lds));
#pragma unroll
    for (int k = 0; k < (L * RPP + NWV - 1) / NWV; ++k) {
      const int q = wave + NWV * k;
      if (q < L * RPP) {
        const int l = q / RPP, pt = (q - l * RPP) * 16 + (lane >> 2);
        const int oh = oh0 + pt / TW, ow = ow0 + pt % TW;
        const bool ok = pt < NPIX && oh < a.ho && ow < a.wo;
        const unsigned src = ok ? (unsigned)(((long long)(img * a.ho + oh) * a.wo + ow) * a.cout + ct * 64 + 16 * (lane & 3))
                                : kOOB;
        dma16(lds0r + resoff + (unsigned)q * 1024u, rrs, src, __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane)));
      }
    }
  } else if constexpr (RES) {
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.res_q), 0, (int)(L * oplane), 0x00020000);
#pragma unroll
    for (int j = 0; j < WPF; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // channels ct * 64 + 16 i + 4 grp .. + 3 of pixel j (qoff[j] points at block grp's 16)
        const unsigned ro = qoff[j] != kOOB ? qoff[j] - 16u * (unsigned)grp + 16u * (unsigned)i + 4u * (unsigned)grp : kOOB;
#pragma unroll
        for (int l = 0; l < L; ++l)
          rqw[i][j][l] = (unsigned)__builtin_amdgcn_raw_buffer_load_b32(rrs, ro, (unsigned)((long long)l * oplane), 0);
      }
  }

  v4i acc[L][4][WPF];  // set by the first chunk's first tap (an MFMA with a zero C operand)
  constexpr bool do_off = OFF;  // weight offsets (compile-time: no merged paths in the epilogue)
  int rs[L][WPF];
#pragma unroll
  for (int l = 0; l < L; ++l)
#pragma unroll
    for (int j = 0; j < WPF; ++j) rs[l][j] = 0;

  auto compute = [&](const int8_t* sb, auto first) {
#pragma unroll
    for (int kr = 0; kr < 3; ++kr)
#pragma unroll
      for (int kc = 0; kc < 3; ++kc) {
        const int tap = kr * 3 + kc;
        v4i fa[4], fb[L][WPF];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const v4i*>(sb + wrd + tap * 4096 + i * 1024);
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
          for (int j = 0; j < WPF; ++j)
            fb[l][j] = *reinterpret_cast<const v4i*>(sb + bpar[j][kr & 1] + l * PLIMB + (kr * PW + kc) * 64);
        if constexpr (do_off) {
#pragma unroll
          for (int l = 0; l < L; ++l)
#pragma unroll
            for (int j = 0; j < WPF; ++j) {
              int sacc = rs[l][j];
              sacc = __builtin_amdgcn_sdot4(fb[l][j].x, 0x01010101, sacc, false);
              sacc = __builtin_amdgcn_sdot4(fb[l][j].y, 0x01010101, sacc, false);
              sacc = __builtin_amdgcn_sdot4(fb[l][j].z, 0x01010101, sacc, false);
              sacc = __builtin_amdgcn_sdot4(fb[l][j].w, 0x01010101, sacc, false);
              rs[l][j] = sacc;
            }
        }
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < WPF; ++j)
              acc[l][i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                  fa[i], fb[l][j], (decltype(first)::value && tap == 0) ? v4i{0, 0, 0, 0} : acc[l][i][j], 0, 0, 0);
      }
  };

  using First = std::integral_constant<bool, true>;
  using Later = std::integral_constant<bool, false>;
  if constexpr (NST == 1) {
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    compute(lds, First{});
    for (int cc = 1; cc < nch; ++cc) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the last chunk
      __builtin_amdgcn_s_barrier();                        // ... and every other wave's
      asm volatile("" ::: "memory");
      issue(cc, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      compute(lds, Later{});
    }
  } else {
    // at the top of chunk cc: this wave's DMA of chunk cc has landed (chunk cc + 1 is not issued
    // yet) and its reads of chunk cc - 1 are done; after the barrier every wave's are, so stage
    // cc % 2 is readable and the other stage (chunk cc - 1's) may be refilled
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (nch > 1) issue(1, 1);
    compute(lds, First{});
    for (int cc = 1; cc < nch; ++cc) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (cc + 1 < nch) issue(cc + 1, (cc + 1) & 1);
      compute(lds + (cc & 1) * STAGE, Later{});
    }
  }

  // ---- epilogue: the implicit-GEMM kernel's lean static-range epilogue ------------------------
  if constexpr (do_off) {
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int j = 0; j < WPF; ++j) {
        int sacc = rs[l][j];
        sacc += __shfl_xor(sacc, 16, kWave);
        sacc += __shfl_xor(sacc, 32, kWave);
        rs[l][j] = sacc;
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int4 coff = *reinterpret_cast<const int4*>(a.w_off + ct * 64 + 16 * i + 4 * grp);
      const int cor[4] = {coff.x, coff.y, coff.z, coff.w};
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int j = 0; j < WPF; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[l][i][j][r] += __mul24(cor[r], rs[l][j]);
    }
  }
  constexpr float qmax = act_qmax<L>();
  const float rscale = a.x_absmax[img] * a.inv_qmax;
  const float inv = a.yq_inv;
  constexpr float lo = 0.f;  // ReLU (compile-time: the 3x3 convs of the ResNets; the launcher checks)
  constexpr bool relu = true;
  unsigned wq[4][WPF][L];
  float vmax = 0.f;
  const float rsq = RES ? a.res_scale * inv : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = ct * 64 + 16 * i + 4 * grp;
    const float4 cs = *reinterpret_cast<const float4*>(a.col_scale + c);
    const float4 csh = *reinterpret_cast<const float4*>(a.col_shift + c);
    const float csq[4] = {cs.x * inv, cs.y * inv, cs.z * inv, cs.w * inv};
    const float shq[4] = {csh.x * inv, csh.y * inv, csh.z * inv, csh.w * inv};
#pragma unroll
    for (int j = 0; j < WPF; ++j) {
      v4i accq[L];
#pragma unroll
      for (int l = 0; l < L; ++l) accq[l] = acc[l][i][j];
      int rqv[4] = {0, 0, 0, 0};
      if constexpr (RES_LDS) {
        // landed before the first chunk's barrier (the first vmcnt(0) covers this wave's DMA)
        const int pt = 16 * (wave * WPF + j) + frow;
        unsigned rw[L];
#pragma unroll
        for (int l = 0; l < L; ++l)
          rw[l] = *reinterpret_cast<const unsigned*>(lds + resoff + l * RPP * 1024 + pt * 64 + 16 * i + 4 * grp);
        decode4<L>(rw, rqv);
      } else if constexpr (RES) {
        decode4<L>(rqw[i][j], rqv);
      }
      const float m = lean_quad<L, L, 0>(accq, rscale, csq, shq, RES, rqv, rsq, relu, lo, wq[i][j]);
      vmax = qoff[j] != kOOB ? fmaxf(vmax, m) : vmax;
    }
  }
  const v4i qrs4 = make_rsrc(a.yq, (long long)L * oplane);
  const bool nt = __builtin_amdgcn_readfirstlane(a.nt_store) != 0;
#pragma unroll
  for (int j = 0; j < WPF; ++j)
#pragma unroll
    for (int l = 0; l < L; ++l) {
      unsigned w0 = wq[0][j][l], w1 = wq[1][j][l], w2 = wq[2][j][l], w3 = wq[3][j][l];
      transpose4(w0, w1, w2, w3);  // lane group g: the 16 channels of block g of its pixel
      store_limbs16(v4u{w0, w1, w2, w3}, qrs4, qoff[j], __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane)),
                    nt);
    }
  if (__any(vmax > qmax) && lane == 0) atomicMax(a.overflow, 1);
}

template <int L, int TH, int TW, int NWV, int WPF, int NST>
int launch_halo_one(const ConvArgs& a, hipStream_t stream) {
  const int nth = (a.ho + TH - 1) / TH, ntw = (a.wo + TW - 1) / TW, nct = a.cout / 64;
  const long long blocks = (long long)a.n * nth * ntw * nct;
  if (blocks > 0x7fffffffLL) return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: grid too large");
  constexpr int stage = kHaloWB + halo_patch_bytes(L, TH, TW);
  const int nch = a.cin / 64;
  constexpr int kResB = halo_res_bytes(L, TH, TW);
  constexpr bool kResLds = NST * stage + kResB <= 160 * 1024;  // the kernel's RES_LDS
  const int lds_bytes = (nch < NST ? nch : NST) * stage + (a.res_q && kResLds ? kResB : 0);
  constexpr int kMax = NST * stage + (kResLds ? kResB : 0);
  static_assert(NST * stage <= 160 * 1024, "LDS per CU");
  using KFn = decltype(&qconv_halo_kernel<L, TH, TW, NWV, WPF, NST, false, false>);
  // [offsets][residual]
  static const KFn fns[4] = {qconv_halo_kernel<L, TH, TW, NWV, WPF, NST, false, false>,
                             qconv_halo_kernel<L, TH, TW, NWV, WPF, NST, false, true>,
                             qconv_halo_kernel<L, TH, TW, NWV, WPF, NST, true, false>,
                             qconv_halo_kernel<L, TH, TW, NWV, WPF, NST, true, true>};
  static hipError_t attrs[4];
  static const bool attrs_set = [] {
    for (int i = 0; i < 4; ++i) {
      attrs[i] = hipFuncSetAttribute(reinterpret_cast<const void*>(fns[i]), hipFuncAttributeMaxDynamicSharedMemorySize, kMax);
      if (attrs[i] != hipSuccess) (void)hipGetLastError();
    }
    return true;
  }();
  (void)attrs_set;
  const int vi = (a.has_offset != 0 ? 2 : 0) + (a.res_q ? 1 : 0);
  if (attrs[vi] != hipSuccess) return check_hip(attrs[vi], "qconv_halo_kernel LDS attribute");
  hipLaunchKernelGGL(fns[vi], dim3((unsigned)blocks), dim3(64 * NWV), lds_bytes, stream, a, nct, ntw, nth * ntw);
  return check_hip(hipGetLastError(), "qconv_halo_kernel launch");
}

template <int L>
int launch_halo_l(int cfg, const ConvArgs& a, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_halo_one<L, 8, 8, 4, 1, 1>(a, s);
    case 1: return launch_halo_one<L, 16, 8, 8, 1, 1>(a, s);
    case 2: return launch_halo_one<L, 16, 8, 4, 2, 1>(a, s);
    case 3: return launch_halo_one<L, 28, 4, 7, 1, 1>(a, s);
    case 4: return launch_halo_one<L, 14, 4, 4, 1, 1>(a, s);
    case 5: return launch_halo_one<L, 8, 8, 4, 1, 2>(a, s);
    case 6: return launch_halo_one<L, 28, 4, 7, 1, 2>(a, s);
    case 7: return launch_halo_one<L, 16, 8, 4, 2, 2>(a, s);
    case 8: return launch_halo_one<L, 7, 14, 7, 1, 1>(a, s);
    case 9: return launch_halo_one<L, 7, 14, 7, 1, 2>(a, s);
    default: return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: bad halo tile config");
  }
}

}  // namespace

int halo_num_cfgs() { return kNumHalo; }

void halo_cfg_info(int cfg, int* bm, int* bn, int* threads) {
  const HaloCfg& c = kHalo[cfg];
  *bm = c.th * c.tw;  // pixels
  *bn = 64;           // channels
  *threads = 64 * c.nwv;
}

// What tile_supported can see: the kernel also needs stride 1, pad 1 and the static-range lean
// epilogue (limb-plane output only), which the launcher checks.
bool halo_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs) {
  (void)cfg;
  return kh == 3 && kw == 3 && cin % 64 == 0 && cout % 64 == 0 && wlimbs == 1 && limbs >= 2;
}

int launch_halo(int cfg, int limbs, int wlimbs, const ConvArgs& a, hipStream_t s) {
  if (cfg < 0 || cfg >= kNumHalo) return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: bad halo tile config");
  if (!halo_supported(cfg, a.cin, a.cout, a.kh, a.kw, limbs, wlimbs) || a.stride != 1 || a.pad != 1 || a.s2d)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: halo tiles take 3x3 / stride 1 / pad 1 convs with cin % 64 == 0, "
                                "cout % 64 == 0 and one weight limb");
  if (!a.yq || a.y || a.residual || a.y_absmax || !a.relu)
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: halo tiles run the static-range limb-plane epilogue with ReLU "
                                "(and optionally a limb-plane residual) only");
  switch (limbs) {
    case 2: return launch_halo_l<2>(cfg, a, s);
    case 3: return launch_halo_l<3>(cfg, a, s);
    default: return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: halo tiles need 2 or 3 activation limbs");
  }
}

}  // namespace smpq
