// Fused stem for gfx950: conv1 7x7/2/3 + bn1 + ReLU + maxpool 3x3/2/1 (resnet.py:143-147, run in
// that order by ResNet.forward, resnet.py:206-209) in ONE launch, static-range mode. Input: the
// space-to-depth limb planes of image_quantize_s2d ([L][n][h/2][w/2][16], channel
// (dy*2+dx)*4 + c); weights: pack_weights_s2d codes [LW][64][256] (K = [tap row][tap col][16]).
// Output: the POOLED activation's limb planes [L][n][h/4][w/4][64] — the 112x112x64 conv output
// never leaves the CU.
//
// Results are bitwise identical to smpq_stem_conv_s2d_q (static range) followed by
// smpq_maxpool_limbs: the same int32 accumulators, the same limb recombination and lean epilogue
// (lean_codes_v: one rounding sequence for every kernel; the general formula for one limb), and
// the max of codes == the code of the max: the epilogue is monotone in the recombined value per
// channel, so the kernel pools that value (sign-flipped where the channel's scale is negative)
// and runs the epilogue once per pooled output (round 5).
//
// Why a separate kernel: the generic LDS-DMA conv spends ~450 us on the stem at B=256 (each
// 64-pixel tile re-reads 48 KiB of weight limbs and a 16x im2col expansion of its input from L2,
// for only 4 K steps), and the 616 MB conv output is written and read back by the pool (~200 us).
// Here one workgroup walks down one image (or a band of it) row by row:
//  * The weight limbs of a wave's 16 output channels live in VGPRs for the whole kernel (LW x 4
//    tap rows fragments), never re-read.
//  * Input rows stream through an 8-row LDS ring by LDS-DMA (2 new rows per step, issued a whole
//    step ahead). A conv row's B fragment for tap row ty is 16 consecutive 16-B pixels of one
//    input row (lane (g, p) reads pixel p + g: tap column g), so fragments are read straight from
//    the row image — no im2col copy; the 16-B reads of a lane group hit distinct bank groups.
//  * 8 waves = 2 row parities x 4 channel blocks. Step k computes conv rows 2k-1 (parity 0) and
//    2k (parity 1), 7 pixel fragments (112 columns) each. A conv row's recombined values are
//    max-pooled horizontally in registers (DPP row shifts: lane p takes p-1, p, p+1; lane 0's left
//    neighbour is lane 15 of the previous fragment), parity 1 hands its row to parity 0 through
//    LDS, and parity 0 completes pooled row k-1 = max(rows 2k-3 (kept from the last step), 2k-2,
//    2k-1), runs the epilogue on it, encodes it and stores it.
// Every conv row is computed once per band (plus one shared boundary row per extra band).
#include "conv_common.h"
#include "lds_dma.h"

namespace smpq {

namespace {

// Diagnostic builds only (tools/ablate_build.sh STEM=1, -DSMPQ_SP_DIAG=N; results are wrong with any
// bit set): 1 no MFMA, 2 no epilogue, 4 no operand reads from LDS, 8 phase timestamps of workgroup 0
// (s_memtime / s_memrealtime, written over the start of the output).
#ifndef SMPQ_SP_DIAG
#define SMPQ_SP_DIAG 0
#endif
constexpr int kSpDiag = SMPQ_SP_DIAG;

constexpr int kSpF = 7;            // 16-pixel column fragments per conv row (conv width <= 112)
constexpr int kSpRing = 8;         // input rows in LDS: row R lives in slot R & 7
constexpr int kSpRowB = 2048;      // bytes per (slot, limb) row: 128 16-B pixels, input column x at x + 2
constexpr int kSpThreads = 512;    // 8 waves: 2 row parities x 4 blocks of 16 output channels
constexpr int kSpSlot = 4 * kSpF * 8 * 4 * 16;  // one horizontally pooled row: [cb][f][8 cols][g][4 x i32]

struct StemPoolArgs {
  const int8_t* xq;       // [L][n][hi][wi][16] space-to-depth limb planes
  long long plane;        // n * hi * wi * 16
  const float* x_absmax;  // [n] per-image input range
  const int8_t* codes;    // [LW][64][256] weight limb planes
  long long wplane;       // 64 * 256
  const float* col_scale;
  const float* col_shift;
  int8_t* yq;             // [L][n][hp][wp][64] pooled output limb planes
  long long oplane;       // n * hp * wp * 64
  float yq_inv;           // QMAX / range of the output quantizer
  float inv_qmax;         // 1 / QMAX of the input code
  int32_t* overflow;
  int n, hi, wi;          // input (space-to-depth) = conv output geometry
  int hp, wp;             // pooled geometry (hi / 2, wi / 2)
  int nseg;               // bands of pooled rows per image (one workgroup each)
};

// DPP moves inside 16-lane rows (lane p = pixel p of a fragment)
__device__ __forceinline__ int dpp_from_left(int v) {  // lane p <- lane p - 1 (row_shr:1)
  return __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ int dpp_from_right(int v) {  // lane p <- lane p + 1 (row_shl:1)
  return __builtin_amdgcn_mov_dpp(v, 0x101, 0xf, 0xf, true);
}
__device__ __forceinline__ int dpp_rotate(int v) {  // lane p <- lane (p - 1) mod 16 (row_ror:1)
  return __builtin_amdgcn_mov_dpp(v, 0x121, 0xf, 0xf, false);
}

}  // namespace

template <int L, int LW>
__global__ __launch_bounds__(kSpThreads, 1) void qconv_stem_pool_kernel(StemPoolArgs a) {
  constexpr int SMIN = (L + LW - 4) > 0 ? (L + LW - 4) : 0;
  constexpr int NACC = L + LW - 1 - SMIN;
  constexpr int RING = kSpRing * L * kSpRowB;
  constexpr float qmax = act_qmax<L>();
  extern __shared__ __attribute__((aligned(1024))) int8_t lds[];
  int8_t* const hslots = lds + RING;  // 4 column-pooled row slots (2 even rows, 2 odd rows), then the weights

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int par = wave >> 2, cb = wave & 3;
  const int p = lane & 15, g = lane >> 4;
  const int img = blockIdx.x / a.nseg;
  const int seg = blockIdx.x - img * a.nseg;
  const int i_lo = seg * a.hp / a.nseg, i_hi = (seg + 1) * a.hp / a.nseg;  // pooled rows [i_lo, i_hi)

  // zero the ring (its padding columns stay zero: the DMA only writes columns 2 .. wi + 1)
  for (int o = threadIdx.x * 16; o < RING; o += kSpThreads * 16) *reinterpret_cast<v4i*>(lds + o) = v4i{0, 0, 0, 0};

  // weight limbs -> LDS once: [lw][tap row][64 channels][64 B], 16-B chunk c of channel row ch at
  // c ^ swz<64>(ch & 15) (conflict-free fragment reads: lanes (g, p) read rows p, chunk g)
  int8_t* const wl = hslots + 4 * kSpSlot;
  for (int t = threadIdx.x; t < LW * 4 * 64 * 4; t += kSpThreads) {
    const int c = t & 3, ch = (t >> 2) & 63, ty = (t >> 8) & 3, lw = t >> 10;
    const v4i v = *reinterpret_cast<const v4i*>(a.codes + lw * a.wplane + ch * 256 + 64 * ty + 16 * c);
    *reinterpret_cast<v4i*>(wl + ((lw * 4 + ty) * 64 + ch) * 64 + 16 * (c ^ swz<64>(ch & 15))) = v;
  }
  const int8_t* const wrow = wl + (16 * cb + p) * 64 + 16 * (g ^ swz<64>(p));  // + (lw * 4 + ty) * 4096
  const float inv = a.yq_inv;
  float csq[4], shq[4];
  {
    const float4 cs = *reinterpret_cast<const float4*>(a.col_scale + 16 * cb + 4 * g);
    const float4 csh = *reinterpret_cast<const float4*>(a.col_shift + 16 * cb + 4 * g);
    const float f = L >= 2 ? inv : 1.f;
    csq[0] = cs.x * f, csq[1] = cs.y * f, csq[2] = cs.z * f, csq[3] = cs.w * f;
    shq[0] = csh.x * f, shq[1] = csh.y * f, shq[2] = csh.z * f, shq[3] = csh.w * f;
  }
  const float rscale = a.x_absmax[img] * a.inv_qmax;
  // channels whose epilogue decreases with v (rscale > 0): their windows pool the minimum of v
  bool neg[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) neg[r] = csq[r] < 0.f;

  const v4i xrs = make_rsrc(a.xq, (long long)L * a.plane);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  // input rows R0 .. R0 + nrows - 1 (all limbs) into their ring slots; parity-1 waves only,
  // row-limb q by wave 4 + q % 4; rows outside the image read as zeros (buffer range check)
  auto load_rows = [&](int R0, int nrows) {
    for (int q = cb; q < nrows * L; q += 4) {
      const int R = R0 + q / L, l = q - (q / L) * L;
      const unsigned dst = lds0 + (unsigned)((((R + 8) & 7) * L + l) * kSpRowB + 32);
      const bool rok = (unsigned)R < (unsigned)a.hi;
      const unsigned src = rok ? (unsigned)((long long)l * a.plane + (long long)(img * a.hi + R) * a.wi * 16) : 0u;
      if (lane < a.wi) dma16(dst, xrs, rok ? src + 16u * lane : kOOB, 0u);
      if (lane + 64 < a.wi) dma16(dst + 1024u, xrs, rok ? src + 1024u + 16u * lane : kOOB, 0u);
    }
  };
  __syncthreads();  // ring zeroed before any DMA lands in it; weights in place
  if (par == 1) {
    load_rows(2 * i_lo - 3, 5);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  const auto yrs = __builtin_amdgcn_make_buffer_rsrc(a.yq, 0, (int)(L * a.oplane), 0x00020000);
  const unsigned hoff = (unsigned)((cb * kSpF * 8 + (p >> 1)) * 4 + g) * 16;  // + f * 512: this lane's slot entry
  float m = 0.f;  // largest rounded output code of this wave (overflow test)

  // ---- one conv row: 4 tap rows x L limbs = 4L groups of 7 B fragments, each read one group ahead
  // of its MFMAs (double buffer; sched_barrier keeps the reads where they are issued)
  v4i acc[NACC][kSpF];
  auto conv_row = [&](int r) {
#pragma unroll
    for (int s = 0; s < NACC; ++s)
#pragma unroll
      for (int f = 0; f < kSpF; ++f) acc[s][f] = v4i{0, 0, 0, 0};
    constexpr int NG = 4 * L;
    v4i buf[2][kSpF];  // B fragments of groups gi (in use) and gi + 1 (landing)
    v4i wa[2][LW];     // A fragments of tap rows ty (in use) and ty + 1 (landing)
    auto load_group = [&](int gi) {
      const int ty = gi / L, l = L - 1 - gi % L;  // limbs high to low: the groups with most MFMAs first
      const int R = r + ty - 2;
      const int8_t* rowp = lds + (((R + 8) & 7) * L + l) * kSpRowB + 16 * (p + g);
#pragma unroll
      for (int f = 0; f < kSpF; ++f)
        buf[gi & 1][f] = (kSpDiag & 4) ? v4i{lane, f, gi, r} : *reinterpret_cast<const v4i*>(rowp + 256 * f);
      if (gi % L == 0) {
#pragma unroll
        for (int lw = 0; lw < LW; ++lw)
          wa[ty & 1][lw] = (kSpDiag & 4) ? v4i{lane, lw, ty, 1} : *reinterpret_cast<const v4i*>(wrow + (lw * 4 + ty) * 4096);
      }
    };
    load_group(0);
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      if (gi + 1 < NG) load_group(gi + 1);
      __builtin_amdgcn_sched_barrier(0);
      const int ty = gi / L, l = L - 1 - gi % L;
#pragma unroll
      for (int lw = 0; lw < LW; ++lw) {
        if (l + lw < SMIN || (kSpDiag & 1)) continue;  // compile-time: skipped low-digit product
#pragma unroll
        for (int f = 0; f < kSpF; ++f)
          acc[l + lw - SMIN][f] =
              __builtin_amdgcn_mfma_i32_16x16x64_i8(wa[ty & 1][lw], buf[gi & 1][f], acc[l + lw - SMIN][f], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // ---- the row in acc, pooled before its epilogue (round 5). The epilogue (limb recombination v,
  // z = fma(v, rscale * cs, sh), ReLU / rounding / clamp) is monotone in v for every channel —
  // non-decreasing where rscale * cs >= 0, non-increasing where it is < 0 — so the max of a 3 x 3
  // window's codes is the code of the window's max of u = (cs < 0 ? -v : v): pool u (in fp32, exact),
  // then run the epilogue once per POOLED output instead of once per conv output (a quarter of the
  // work; it was the longer half of every step, MI355X_MICROARCH 'an MFMA holds its SIMD's vector
  // issue for 8 of 16 cycles'). The codes, their maximum for the overflow test and so the output
  // are bitwise those of the per-output epilogue (every conv output lies in some pooled window;
  // padding is -inf, which a window's valid outputs always beat). Here: u of pixel 16 f + p,
  // channels 16 cb + 4 g + 0..3, then the 3-wide max across columns: even lane p of fragment f
  // holds pooled column 8 f + p / 2.
  auto urow = [&](float (*hu)[4]) {
    if constexpr ((kSpDiag & 2) != 0) {
#pragma unroll
      for (int f = 0; f < kSpF; ++f)
#pragma unroll
        for (int c = 0; c < 4; ++c) hu[f][c] = (float)(acc[0][f][c] ^ acc[NACC - 1][f][c]);
      return;
    }
    constexpr float w0 = SMIN == 0 ? 1.f : (SMIN == 1 ? 256.f : 65536.f);
    float u[kSpF][4];
#pragma unroll
    for (int f = 0; f < kSpF; ++f) {
      const bool ok = 16 * f + p < a.wi;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = (float)acc[0][f][r];  // the recombination of lean_codes
        if (SMIN != 0) v = v * w0;
#pragma unroll
        for (int t = 1; t < NACC; ++t) v = __fmaf_rn((float)acc[t][f][r], w0 * (float)(1 << (8 * t)), v);
        u[f][r] = ok ? (neg[r] ? -v : v) : -INFINITY;
      }
    }
#pragma unroll
    for (int f = 0; f < kSpF; ++f)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float prev = f == 0 ? -INFINITY : __int_as_float(dpp_rotate(__float_as_int(u[f - 1][c])));  // lane 0
        const float left = p == 0 ? prev : __int_as_float(dpp_from_left(__float_as_int(u[f][c])));
        hu[f][c] = fmaxf(fmaxf(left, u[f][c]), __int_as_float(dpp_from_right(__float_as_int(u[f][c]))));
      }
  };
  // the epilogue of one pooled u (4 channels): the codes and the largest rounded code
  auto codes_of = [&](const float* um, int* q) {
    float vs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) vs[r] = neg[r] ? -um[r] : um[r];
    if constexpr (L >= 2) {
      return lean_codes_v<L>(vs, rscale, csq, shq, false, nullptr, 0.f, true, 0.f, q);
    } else {
      float mm = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // one limb: the general epilogue (smpq_stem_conv_s2d_q)
        const float y = fmaxf(__fmaf_rn(vs[r], rscale * csq[r], shq[r]), 0.f);
        const float zr = rintf(y * inv);
        mm = fmaxf(mm, zr);
        q[r] = (int)fminf(fmaxf(zr, -qmax), qmax);
      }
      return mm;
    }
  };

  // Step k = two half-steps, each ended by a barrier. In each half one wave of every SIMD issues
  // MFMAs while the other runs VALU code:
  //   parity 0: half 0 convolves row 2k - 1; half 1 stores pooled row k - 2, then runs the
  //             epilogue of row 2k - 1 (-> column-pooled row H[2k-1] in slot 2 + (k & 1));
  //   parity 1: half 0 issues the DMA of input rows 2k + 2, 2k + 3 (for step k + 1) and runs the
  //             epilogue of row 2k - 2 (-> H[2k-2] in slot k & 1); half 1 convolves row 2k.
  // A wave's accumulators live across the barrier between its MFMA half and its VALU half.
  // Pooled row i = max(H[2i-1], H[2i], H[2i+1]) is complete after step i + 1 and stored in step
  // i + 2 (before that step's epilogue reuses the slot of H[2i-1]). Input rows: step k reads rows
  // 2k-3 .. 2k+1; the DMA of step k writes the slots of rows 2k-6, 2k-5 (last read in step k - 1)
  // and lands before the barrier that ends step k.
  auto put_row = [&](int slot, const float (*hu)[4]) {
    if ((p & 1) == 0) {
      int8_t* sp = hslots + slot * kSpSlot + hoff;
#pragma unroll
      for (int f = 0; f < kSpF; ++f)
        *reinterpret_cast<v4i*>(sp + 512 * f) = v4i{__float_as_int(hu[f][0]), __float_as_int(hu[f][1]),
                                                   __float_as_int(hu[f][2]), __float_as_int(hu[f][3])};
    }
  };
  auto stamp = [&](int k, int e) {  // diagnostic: [wave][step < 16][event < 8] x (clock, realtime)
    if constexpr ((kSpDiag & 8) != 0) {
      const long long t = (long long)__builtin_amdgcn_s_memtime(), rt = (long long)__builtin_amdgcn_s_memrealtime();
      if (blockIdx.x == 0 && lane == 0 && k - i_lo < 16) {
        long long* d = reinterpret_cast<long long*>(a.yq) + ((wave * 16 + (k - i_lo)) * 8 + e) * 2;
        d[0] = t;
        d[1] = rt;
      }
    }
  };
  for (int k = i_lo; k <= i_hi + 1; ++k) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      stamp(k, 4 * half);
      const int row = par == 0 ? 2 * k - 1 : 2 * k;
      const bool row_ok = par == 0 ? (k <= i_hi && row >= 0) : k < i_hi;
      if (half == par) {
        if (row_ok) conv_row(row);
      } else if (par == 0) {
        if (k >= i_lo + 2 && (p & 1) == 0) {
          const int i = k - 2;
          const int8_t* se = hslots + ((k - 1) & 1) * kSpSlot + hoff;        // H[2i]
          const int8_t* s0 = hslots + (2 + ((k - 2) & 1)) * kSpSlot + hoff;  // H[2i-1]
          const int8_t* s1 = hslots + (2 + ((k - 1) & 1)) * kSpSlot + hoff;  // H[2i+1]
#pragma unroll
          for (int f = 0; f < kSpF; ++f) {
            const v4i he = *reinterpret_cast<const v4i*>(se + 512 * f);
            const v4i h0 = *reinterpret_cast<const v4i*>(s0 + 512 * f);
            const v4i h1 = *reinterpret_cast<const v4i*>(s1 + 512 * f);
            const int pc = 8 * f + (p >> 1);
            float um[4];
#pragma unroll
            for (int c = 0; c < 4; ++c)
              um[c] = fmaxf(fmaxf(__int_as_float(he[c]), __int_as_float(h0[c])), __int_as_float(h1[c]));
            int pooled[4];
            const float mm = codes_of(um, pooled);
            m = pc < a.wp ? fmaxf(m, mm) : m;
            unsigned wq[L];
            encode4<L>(pooled, wq);
            if (pc < a.wp && !(kSpDiag & 8)) {  // (the diagnostic stamps own the output buffer)
              const unsigned off = (unsigned)(((img * a.hp + i) * a.wp + pc) * 64 + 16 * cb + 4 * g);
#pragma unroll
              for (int l = 0; l < L; ++l)
                __builtin_amdgcn_raw_buffer_store_b32(wq[l], yrs, off, (unsigned)((long long)l * a.oplane), 0);
            }
          }
        }
        if (k <= i_hi) {
          float hu[kSpF][4];
          if (row >= 0) {
            urow(hu);
          } else {
#pragma unroll
            for (int f = 0; f < kSpF; ++f)
#pragma unroll
              for (int c = 0; c < 4; ++c) hu[f][c] = -INFINITY;  // conv row -1: the pool's padding
          }
          put_row(2 + (k & 1), hu);
        }
      } else {
        if (k < i_hi) load_rows(2 * k + 2, 2);
        stamp(k, 1);
        if (k >= i_lo + 1 && k <= i_hi) {  // row 2k - 2, convolved in step k - 1
          float hu[kSpF][4];
          urow(hu);
          put_row(k & 1, hu);
        }
      }
      stamp(k, 4 * half + 2);
      if (par == 1 && half == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // step k + 1's rows
      stamp(k, 4 * half + 3);
      __syncthreads();
    }
  }
  if (__any(m > qmax) && lane == 0) atomicMax(a.overflow, 1);
}

template <int L, int LW>
static int launch_stem_pool(const StemPoolArgs& a, unsigned blocks, hipStream_t s) {
  constexpr int lds_bytes = kSpRing * L * kSpRowB + 4 * kSpSlot + LW * 4 * 64 * 64;
  static const hipError_t attr = [] {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(qconv_stem_pool_kernel<L, LW>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
  }();
  if (attr != hipSuccess) return check_hip(attr, "qconv_stem_pool_kernel LDS attribute");
  auto kern = qconv_stem_pool_kernel<L, LW>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kSpThreads), lds_bytes, s, a);
  return check_hip(hipGetLastError(), "qconv_stem_pool_kernel launch");
}

static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cus[dev] = c;
  }
  return cus[dev];
}

}  // namespace smpq

using namespace smpq;

extern "C" int smpq_stem_pool_supported(int n, int h, int w, int cout, int limbs, int wlimbs) {
  if (n <= 0 || cout != 64 || h < 4 || w < 4 || (h % 4) != 0 || (w % 4) != 0 || w / 2 > 16 * kSpF) return 0;
  if (!((limbs == 3 && wlimbs == 3) || (limbs == 2 && wlimbs == 2) || (limbs == 1 && wlimbs == 2))) return 0;
  const long long plane = (long long)n * (h / 2) * (w / 2) * 16, oplane = (long long)n * (h / 4) * (w / 4) * 64;
  return (limbs * plane <= 0x7fffff00LL && limbs * oplane <= 0x7fffff00LL) ? 1 : 0;
}

extern "C" int smpq_stem_pool_s2d_q(const int8_t* xq, const float* x_absmax, int n, int h, int w,
                                    const int8_t* codes, int wlimbs, int cout, const float* col_scale,
                                    const float* col_shift, int limbs, int8_t* yq, float yq_range,
                                    int32_t* overflow, smpq_stream_t stream) {
  if (!xq || !x_absmax || !codes || !col_scale || !col_shift || !yq || !overflow)
    return fail(SMPQ_E_INVALID, "smpq_stem_pool_s2d_q: null pointer");
  if (!(yq_range > 0.f)) return fail(SMPQ_E_INVALID, "smpq_stem_pool_s2d_q: the output range must be positive");
  if (!smpq_stem_pool_supported(n, h, w, cout, limbs, wlimbs))
    return fail(SMPQ_E_SHAPE,
                "smpq_stem_pool_s2d_q: needs cout 64, h and w multiples of 4, w <= 224, (limbs, wlimbs) in "
                "{(3, 3), (2, 2), (1, 2)}");
  StemPoolArgs a = {};
  a.xq = xq;
  a.x_absmax = x_absmax;
  a.codes = codes;
  a.col_scale = col_scale;
  a.col_shift = col_shift;
  a.yq = yq;
  a.overflow = overflow;
  a.n = n;
  a.hi = h / 2;
  a.wi = w / 2;
  a.hp = a.hi / 2;
  a.wp = a.wi / 2;
  a.plane = (long long)n * a.hi * a.wi * 16;
  a.oplane = (long long)n * a.hp * a.wp * 64;
  a.wplane = 64LL * 256;
  const float qmax = limbs == 1 ? 127.f : (limbs == 2 ? 32512.f : 8323072.f);
  a.yq_inv = qmax / yq_range;
  a.inv_qmax = 1.f / qmax;
  // enough workgroups to give every CU one (a band of pooled rows per workgroup)
  const int cus = device_cus();
  int nseg = (cus + n - 1) / n;
  nseg = nseg < 1 ? 1 : (nseg > a.hp ? a.hp : nseg);
  a.nseg = nseg;
  if ((long long)n * nseg > 0x7fffffffLL) return fail(SMPQ_E_SHAPE, "smpq_stem_pool_s2d_q: grid too large");
  const unsigned blocks = (unsigned)(n * nseg);
  hipStream_t s = (hipStream_t)stream;
  if (limbs == 3) return launch_stem_pool<3, 3>(a, blocks, s);
  if (limbs == 2) return launch_stem_pool<2, 2>(a, blocks, s);
  return launch_stem_pool<1, 2>(a, blocks, s);
}
