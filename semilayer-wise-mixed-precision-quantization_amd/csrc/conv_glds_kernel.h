// The LDS-DMA quantized-conv kernel template (qconv_glds_kernel), its tile-configuration table and
// the per-(limbs, weight limbs) launch switch. Included by conv_glds.hip (dispatch, stem tiles)
// and by conv_glds_inst.hip, which instantiates launch_cfg<L, LW> once per translation unit so
// that the seven (L, LW) families compile in parallel.
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
#pragma once

#include "conv_common.h"
#include "lds_dma.h"

namespace smpq {

namespace {

// Diagnostic builds only (tools/ablate_glds.sh compiles separate libraries with -DSMPQ_DIAG_ABLATE=N;
// results are wrong with any bit set): 1 no residual loads, 2 no limb-plane stores, 4 no operand
// DMA, 8 no MFMA, 16 no epilogue.
#ifndef SMPQ_DIAG_ABLATE
#define SMPQ_DIAG_ABLATE 0
#endif
constexpr int kAblate = SMPQ_DIAG_ABLATE;

}  // namespace

// Diagnostic builds only (tools/stamp_bench.hip, -DSMPQ_STAMPS): lane 0 of every wave records the
// shader clock (s_memtime) at fixed points of the block's life into smpq_stamps (32 slots per
// wave, vector stores); the product library never defines SMPQ_STAMPS.
#ifdef SMPQ_STAMPS
__device__ unsigned long long* smpq_stamps;
// The stamp buffer's address is read once per wave (stamp_base, at kernel start), and each stamp is
// a plain global store issued without waiting: a per-stamp load of the pointer would make every
// stamp wait (vmcnt) for the previous stamp's store to complete, ~2-3k cycles each.
#define SMPQ_STAMP(slot)                                                                                    \
  do {                                                                                                      \
    if (lane == 0) {                                                                                        \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                         \
      unsigned long long* p_ = stamp_base + (slot);                                                         \
      asm volatile("global_store_dwordx2 %0, %1, off\n\ts_nop 1" ::"v"(p_), "v"(t_) : "memory");            \
    }                                                                                                       \
  } while (0)
#else
#define SMPQ_STAMP(slot) \
  do {                   \
  } while (0)
#endif

// S2D: the space-to-depth stem. The image is stored as 16-channel pixels ([2x2 block][4 ch]) and
// the 7x7/2 conv is a 4x4/1 conv over them (pad 2, zero taps where the 8x8 extension falls
// outside 7x7); a 64-B K step is one tap row: lane chunk c = the 16 channels of tap column c.
// NST LDS stages: the DMA of K step k + NST - 1 is in flight while step k computes.
// BK: K bytes per stage and row. 64 = one MFMA K; 128 (cin % 128 == 0) = two, and every DMA piece
// is then 8 whole 128-B lines instead of 16 half lines (half the TA/TD work per byte).
// LEAN (0: the general epilogue; 1: lean, ReLU and residual decided at run time; 2: lean with
// ReLU, no residual — conv1 / conv2; 3: lean with ReLU and a limb-plane residual — conv3; 4: lean
// without ReLU or residual — the downsample convs): the
// static-range epilogue that only emits the next conv's limb planes (no fp32 output, no
// fp32 residual, no per-image maxima): the output quantizer's 1/step is folded into the column
// scale / shift and the residual scale, ReLU and the code clamp are one v_med3, and overflow is
// tracked on the rounded codes — about half the VALU work of the general epilogue per output.
// The body of one block (block `bid` of `total` blocks of this conv); `lds` = the dynamic LDS.
// OFF: weight offsets may be present (a.has_offset decides at run time); instantiated without them
// the offset sums and their correction compile away (a runtime-false branch still cost the
// epilogue ~50 register moves per wave to merge the two paths' accumulators).
template <int L, int LW, int WAVES_C, int WAVES_P, int WC, int WP, int MINW, bool S2D, int NST, int BK,
          int LEAN = 0, bool PIPE = false, bool OFF = true>
__device__ __forceinline__ void qconv_glds_body(ConvArgs a, int bid, int total, int8_t* lds) {
  static_assert(BK == 64 || BK == 128, "BK");
  static_assert(!S2D || BK == 64, "the s2d stem uses 64-B K steps");
  constexpr int NW = WAVES_C * WAVES_P;
  constexpr int BC = 16 * WC * WAVES_C;  // channels per block tile
  constexpr int BP = 16 * WP * WAVES_P;  // pixels per block tile
  constexpr int SMIN = (L + LW - 4) > 0 ? (L + LW - 4) : 0;
  constexpr int NACC = L + LW - 1 - SMIN;
  constexpr int KH = BK / 64;      // MFMA K steps per stage
  constexpr int RPP = 1024 / BK;   // rows per 1-KiB DMA piece
  constexpr int CPR = BK / 16;     // 16-B chunks per row
  constexpr int WPIECES = LW * (BC / RPP);
  constexpr int APIECES = L * (BP / RPP);
  constexpr int NPIECE = WPIECES + APIECES;
  constexpr int STAGE = NPIECE * 1024;
  constexpr int WSLOTS = (WPIECES + NW - 1) / NW;
  constexpr int ASLOTS = (APIECES + NW - 1) / NW;
  // Epilogue limb-plane tiles in LDS (configs with 4k channel blocks per wave): the residual's
  // tile arrives by DMA at kernel start (whole lines, overlapped with the K loop); the output's is
  // staged in the operand area and copied out row-major (whole lines when BC >= 128 or BC == cout)
  constexpr bool TRT = (WC % 4) == 0;
  constexpr int TILEB = L * BP * BC;
  if constexpr ((kAblate & 32) != 0) {  // diagnostic: static-range epilogue only
    a.y = nullptr;
    a.residual = nullptr;
    a.y_absmax = nullptr;
  }

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef SMPQ_STAMPS
  unsigned long long* const stamp_base = smpq_stamps + ((size_t)bid * NW + wave) * 32;
#endif
  SMPQ_STAMP(0);
  __builtin_assume(wave >= 0 && wave < NW);
  const int wc = wave / WAVES_P, wp = wave % WAVES_P;

  // ---- XCD-aware tile order ----------------------------------------------------------------
  const int ntc = (a.cout + BC - 1) / BC;
  const int full = total & ~7;
  int t = bid;
  if (t < full) t = (t & 7) * (full >> 3) + (t >> 3);
  const int tq = fast_div(t, a.ntc_mul, a.ntc_shr);  // t / ntc
  const int m0 = tq * BP;
  const int n0 = (t - tq * ntc) * BC;
  const int hw_out = a.ho * a.wo;

  const v4i wrs = make_rsrc(a.codes, (long long)LW * a.wplane);
  const v4i xrs = make_rsrc(a.xq, (long long)L * a.plane);

  // ---- per-lane source offsets of this wave's DMA pieces -------------------------------------
  // piece row = lane / CPR, physical chunk = lane % CPR -> logical K chunk (lane % CPR) ^ swz(row),
  // row = the row inside its 16-row MFMA block (the fragment reads' index; with BK = 128 a piece
  // is half a block, so odd pieces start at row 8)
  const int prow = lane / CPR;
  auto pchunk_of = [&](int q) { return (lane % CPR) ^ swz<BK>((RPP * q + prow) & 15); };
  unsigned wsrc[WSLOTS];
#pragma unroll
  for (int s = 0; s < WSLOTS; ++s) {
    const int p = wave + NW * s;  // weight piece: limb p / (BC/RPP), rows RPP * (p % (BC/RPP)) + ...
    const int lw = p / (BC / RPP), bi = p % (BC / RPP);
    const int row = n0 + RPP * bi + prow;
    // logical 16-B chunk lc of the row's BK-wide K slice: row-major [LW][cout][K] at row * K + 16 lc;
    // K-major [LW][K/64][cout][64] at (lc / 4) 64-B slices of cout rows further, row * 64 + 16 (lc % 4)
    const int lc = pchunk_of(bi);
    const long long woff = a.w_kmajor ? (long long)(lc >> 2) * a.cout * 64 + (long long)row * 64 + 16 * (lc & 3)
                                      : (long long)row * a.K + 16 * lc;
    wsrc[s] = (p < WPIECES && row < a.cout) ? (unsigned)((long long)lw * a.wplane + woff) : kOOB;
  }
  int apix[ASLOTS], aih[ASLOTS], aiw[ASLOTS];
#pragma unroll
  for (int s = 0; s < ASLOTS; ++s) {
    const int p = wave + NW * s;  // activation piece: limb p / (BP/RPP), rows RPP * (p % (BP/RPP)) + ...
    const int bj = p % (BP / RPP);
    const int m = m0 + RPP * bj + prow;
    const int pchunk = pchunk_of(bj);
    if (p < APIECES && m < a.M) {
      const int img = fast_div(m, a.hw_mul, a.hw_shr);
      const int rem = m - img * hw_out;
      const int oh = fast_div(rem, a.wo_mul, a.wo_shr), ow = rem - oh * a.wo;
      if constexpr (S2D) {
        aih[s] = oh - a.pad;
        aiw[s] = ow - a.pad + pchunk;  // this lane's tap column, fixed over the K steps
        apix[s] = ((img * a.h + aih[s]) * a.w + aiw[s]) * 16;
        if ((unsigned)aiw[s] >= (unsigned)a.w) aih[s] = -(1 << 28);
      } else {
        aih[s] = oh * a.stride - a.pad;
        aiw[s] = ow * a.stride - a.pad;
        apix[s] = ((img * a.h + aih[s]) * a.w + aiw[s]) * a.cin + 16 * pchunk;
      }
    } else {
      aih[s] = -(1 << 28);  // never inside the image
      aiw[s] = 0;
      apix[s] = 0;
    }
  }
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));

  // K position of step ks: tap (kr, kc), channel chunk c0 (scalar, advanced incrementally)
  // bytes between the weight slices of consecutive K steps (row-major: BK along the row; K-major:
  // BK / 64 slices of cout rows)
  const unsigned wstep = __builtin_amdgcn_readfirstlane(a.w_kmajor ? (unsigned)(BK * a.cout) : (unsigned)BK);
  auto issue = [&](int buf, int kr, int kc, int c0, int ks) {
    const unsigned sb = lds0 + buf * STAGE;
#pragma unroll
    for (int s = 0; s < WSLOTS; ++s) {
      const int p = wave + NW * s;
      if (p < WPIECES && !(kAblate & 4)) dma16(sb + p * 1024, wrs, wsrc[s], __builtin_amdgcn_readfirstlane(ks * wstep));
    }
    const int tapoff = (kr * a.w + kc) * a.cin + c0;
#pragma unroll
    for (int s = 0; s < ASLOTS; ++s) {
      const int p = wave + NW * s;
      if (p < APIECES && !(kAblate & 4)) {
        const int l = p / (BP / RPP);
        unsigned voff;
        if constexpr (S2D) {
          const bool ok = (unsigned)(aih[s] + ks) < (unsigned)a.h;
          voff = ok ? (unsigned)(apix[s] + ks * a.w * 16) : kOOB;
        } else {
          const bool ok = (unsigned)(aih[s] + kr) < (unsigned)a.h && (unsigned)(aiw[s] + kc) < (unsigned)a.w;
          voff = ok ? (unsigned)(apix[s] + tapoff) : kOOB;
        }
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
  const bool do_off = OFF && (LW == 1) && a.has_offset;
  int rs[L][WP];  // per-lane partial pixel sums of activation codes (LW == 1 offset correction)
#pragma unroll
  for (int l = 0; l < L; ++l)
#pragma unroll
    for (int j = 0; j < WP; ++j) rs[l][j] = 0;

  // fragment read offset inside a 16-row block of a [rows][BK] region, per MFMA K step h
  const int frow = lane & 15;
  int rd[KH];
#pragma unroll
  for (int h = 0; h < KH; ++h) rd[h] = frow * BK + 16 * ((4 * h + (lane >> 4)) ^ swz<BK>(frow));
  const int nsteps = a.ksteps / KH;  // a.ksteps counts 64-wide K steps

  // Output coordinates of this lane: channels chan[i] + 0..3 of pixel mrow[j]; ooff = element
  // offset in an NHWC plane, or kOOB (then buffer loads read 0 and buffer stores are dropped).
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
  for (int i = 0; i < WC; ++i) chan[i] = n0 + (wc * WC + i) * 16 + 4 * (lane >> 4);
  unsigned ooff[WC][WP];
#pragma unroll
  for (int i = 0; i < WC; ++i)
#pragma unroll
    for (int j = 0; j < WP; ++j)  // cout % 16 == 0: the 4 channels are valid together
      ooff[i][j] = (mok[j] && chan[i] < a.cout) ? (unsigned)(mrow[j] * a.cout + chan[i]) : kOOB;
  const long long oplane = (long long)a.M * a.cout;
  // With 4k channel blocks per wave the limb planes move as 16-B pieces: after a lane-group
  // transpose (transpose4) lane group g owns the 16 channels of block 4q + g of its pixel. When the
  // tile's rows are whole lines (BC >= 128, or BC == cout: the tile is one contiguous run) they go
  // through LDS tiles (residual by DMA, output staged and copied out row-major); otherwise each
  // wave-instruction moves 64 contiguous bytes of 16 pixel rows straight from registers.
  constexpr bool TR = TRT;
  constexpr int NQ = TR ? WC / 4 : 1;
  const bool lines = (kAblate & 32) ? BC >= 128 : (BC >= 128 || BC == a.cout);
  // limb-plane residual (compile-time in the LEAN 2 / 3 variants: no merged paths in the epilogue)
  const bool has_rq = LEAN == 3 || (LEAN != 2 && LEAN != 4 && a.res_q != nullptr);
  const bool stage_res = TR && has_rq && lines, stage_out = TR && a.yq && lines;
  unsigned qoff[NQ][WP];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const int c16 = n0 + (wc * WC + 4 * q + (lane >> 4)) * 16;
      qoff[q][j] = (TR && mok[j] && c16 < a.cout) ? (unsigned)(mrow[j] * a.cout + c16) : kOOB;
    }

  // residual limb planes: issued now, consumed in the epilogue (latency hidden behind the K loop)
  int rq[WC][WP][L];
  const int nst_eff = nsteps < NST ? nsteps : NST;
  const int resoff = (stage_out && TILEB > nst_eff * STAGE) ? TILEB : nst_eff * STAGE;  // LDS layout
  if constexpr (TR) {
    if (has_rq && !stage_res) {
      const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.res_q), 0, (int)(L * oplane),
                                                         0x00020000);
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int j = 0; j < WP; ++j)
#pragma unroll
          for (int l = 0; l < L; ++l) {
            const v4u v = (kAblate & 1) ? v4u{qoff[q][j], 0u, 0u, 0u}
                                        : __builtin_amdgcn_raw_buffer_load_b128(rrs, qoff[q][j],
                                                                                (unsigned)((long long)l * oplane), 0);
#pragma unroll
            for (int c = 0; c < 4; ++c) rq[4 * q + c][j][l] = (int)v[c];
          }
    } else if (has_rq) {
      // the [L][BP][BC] tile by LDS-DMA: piece = 1024 / BC rows of BC bytes
      constexpr int RROWS = 1024 / BC, RCPR = BC / 16, RPL = BP * BC / 1024, RPIECES = L * RPL;
      const v4i rrs = make_rsrc(a.res_q, (long long)L * oplane);
      const int rrow = lane / RCPR, rpc = lane % RCPR;
#pragma unroll
      for (int s = 0; s < (RPIECES + NW - 1) / NW; ++s) {
        const int pi = wave + NW * s;
        if (pi < RPIECES && !(kAblate & 1)) {
          const int l = pi / RPL, rt = (pi % RPL) * RROWS + rrow;
          const int lc = rpc ^ swze<BC>(rt & 15);
          const bool ok = m0 + rt < a.M && n0 + 16 * lc < a.cout;
          const unsigned voff = ok ? (unsigned)((long long)l * oplane + (long long)(m0 + rt) * a.cout + n0 + 16 * lc)
                                   : kOOB;
          dma16(lds0 + resoff + pi * 1024, rrs, voff, 0u);
        }
      }
    }
  } else if (has_rq) {
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.res_q), 0, (int)(L * oplane),
                                                       0x00020000);
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j)
#pragma unroll
        for (int l = 0; l < L; ++l)
          rq[i][j][l] = (kAblate & 1) ? (int)ooff[i][j]
                                      : (int)__builtin_amdgcn_raw_buffer_load_b32(rrs, ooff[i][j],
                                                                                  (unsigned)((long long)l * oplane), 0);
  }

  // DMA pieces this wave issues per K step (wave-uniform): the counted vmcnt below. When the
  // pieces divide evenly over the waves the count is a compile-time constant (PPW) and so are the
  // steady-state waits.
  constexpr bool kUniform = (WPIECES % NW) == 0 && (APIECES % NW) == 0;
  constexpr int PPW = (WPIECES + APIECES) / NW;
  int ppw = 0;
#pragma unroll
  for (int s = 0; s < WSLOTS; ++s) ppw += (wave + NW * s < WPIECES) ? 1 : 0;
#pragma unroll
  for (int s = 0; s < ASLOTS; ++s) ppw += (wave + NW * s < APIECES) ? 1 : 0;
  if constexpr (kUniform) ppw = PPW;

  int kr = 0, kc = 0, c0 = 0;  // K position of the next step to issue
  auto advance = [&]() {
    c0 += BK;
    if (c0 == a.cin) {
      c0 = 0;
      if (++kc == a.kw) {
        kc = 0;
        ++kr;
      }
    }
  };
  int nissued = 0, wbuf = 0, rbuf = 0;
  // fragments of one MFMA K step of a stage
  struct Frags {
    v4i w[LW][WC], a[L][WP];
  };
  auto read_frags = [&](Frags& f, const int8_t* sb, int h) {
#pragma unroll
    for (int lw = 0; lw < LW; ++lw)
#pragma unroll
      for (int i = 0; i < WC; ++i)
        f.w[lw][i] = *reinterpret_cast<const v4i*>(sb + (lw * BC + (wc * WC + i) * 16) * BK + rd[h]);
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int j = 0; j < WP; ++j)
        f.a[l][j] = *reinterpret_cast<const v4i*>(sb + WPIECES * 1024 + (l * BP + (wp * WP + j) * 16) * BK + rd[h]);
  };
  auto mma = [&](const Frags& f) {
    if (do_off) {
#pragma unroll
      for (int l = 0; l < L; ++l)
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          int s = rs[l][j];
          s = __builtin_amdgcn_sdot4(f.a[l][j].x, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(f.a[l][j].y, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(f.a[l][j].z, 0x01010101, s, false);
          s = __builtin_amdgcn_sdot4(f.a[l][j].w, 0x01010101, s, false);
          rs[l][j] = s;
        }
    }
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int lw = 0; lw < LW; ++lw) {
        if (l + lw < SMIN || (kAblate & 8)) continue;  // compile-time: skipped low-digit product
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j)
            acc[l + lw - SMIN][i][j] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(f.w[lw][i], f.a[l][j], acc[l + lw - SMIN][i][j], 0, 0, 0);
      }
  };
  auto issue_next = [&]() {
    if (nissued < nsteps) {
      issue(wbuf, kr, kc, c0, nissued);
      advance();
      ++nissued;
      wbuf = wbuf + 1 == NST ? 0 : wbuf + 1;
    }
  };
  // wait until this wave's DMA of step `ready` has landed (younger steps may still fly)
  auto wait_step = [&](int ready) {
    const int d = nissued - ready - 1;  // steps issued after it
    if (kUniform && d == NST - 1) {
      wait_vm<PPW * (NST - 1)>();
    } else if (kUniform && d == NST - 2) {
      wait_vm<PPW * (NST - 2)>();
    } else {
      wait_vmcnt(d * ppw);
    }
  };

  if constexpr (PIPE) {
    // Register-pipelined K loop (two fragment register sets): after the barrier that certifies
    // stage ks + 1 (every wave's DMA of it landed, every wave's reads of stage ks done — waited
    // before the barrier), the first fragments of step ks + 1 are read while step ks's MFMAs run
    // from registers, and the DMA of step ks + NST refills stage ks. The MFMAs never wait on LDS.
    // KH == 1: the two sets alternate between steps; KH == 2: set X holds the first MFMA K step of
    // a stage, set Y the second (read from the same stage before X's MFMAs).
#pragma unroll
    for (int st = 0; st < NST; ++st)
      if (st < nsteps) issue_next();
    Frags fx, fy;
    wait_step(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int8_t* sb = lds;
    read_frags(fx, sb, 0);
    rbuf = 1 == NST ? 0 : 1;
    auto next_stage = [&](int ks, Frags& f) {  // barrier for stage ks + 1, read its first fragments
      wait_step(ks + 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      sb = lds + rbuf * STAGE;
      rbuf = rbuf + 1 == NST ? 0 : rbuf + 1;
      read_frags(f, sb, 0);
      issue_next();  // into the stage of step ks
    };
    if constexpr (KH == 1) {
      auto step = [&](int ks, Frags& cur, Frags& nxt) {
        if (ks + 1 < nsteps) next_stage(ks, nxt);
        mma(cur);
      };
      for (int ks = 0; ks < nsteps; ks += 2) {
        step(ks, fx, fy);
        if (ks + 1 < nsteps) step(ks + 1, fy, fx);
      }
    } else {
      static_assert(KH == 2, "KH");
      for (int ks = 0; ks < nsteps; ++ks) {
        read_frags(fy, sb, 1);
        mma(fx);
        if (ks + 1 < nsteps) next_stage(ks, fx);
        mma(fy);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else {
#pragma unroll
    for (int st = 0; st < NST - 1; ++st)
      if (st < nsteps) issue_next();
    SMPQ_STAMP(1);
    for (int ks = 0; ks < nsteps; ++ks) {
      // this wave's DMA of step ks has landed (the younger steps' may still fly) and its reads of
      // step ks-1 are done; after the barrier every wave's are, so stage ks is readable and the
      // stage of step ks-1 may be refilled
      if constexpr (NST == 2) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      } else {
        wait_step(ks);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (ks < 16) SMPQ_STAMP(2 + ks);
      const int8_t* sb = lds + rbuf * STAGE;
      rbuf = rbuf + 1 == NST ? 0 : rbuf + 1;
      // fragments of MFMA K step h of this stage (the DMA below writes the other stage, so the
      // second half may be read after the first half's MFMAs: half the fragment registers live)
      Frags f;
      read_frags(f, sb, 0);
#ifdef SMPQ_STAMPS
      if (ks == 6) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        SMPQ_STAMP(18);
      }
#endif
      issue_next();  // the DMA of step ks + NST - 1 into the stage step ks - 1 used
      if (ks == 6) SMPQ_STAMP(19);
      mma(f);
#ifdef SMPQ_STAMPS
      if (ks == 6) {
        int keep = acc[0][0][0].x;
        asm volatile("v_mov_b32 %0, %0" : "+v"(keep));  // after the MFMAs have retired
        SMPQ_STAMP(20);
        acc[0][0][0].x = keep;
      }
#endif
#pragma unroll
      for (int h = 1; h < KH; ++h) {
        read_frags(f, sb, h);
        mma(f);
      }
    }
  }

  SMPQ_STAMP(21);
  if constexpr ((kAblate & 16) != 0) {  // diagnostic: no epilogue at all (keep the MFMAs live)
    int keep = 0;
#pragma unroll
    for (int q = 0; q < NACC; ++q)
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j) keep ^= acc[q][i][j].x ^ acc[q][i][j].w;
    if (keep == 0x7654321) a.overflow[0] = keep;
    return;
  }
  // ---- epilogue: straight from the accumulators, in phases (uniform branches per phase) -----
  // accumulator-layout dword (channels 4g..4g+3 of block wc * WC + i, pixel row of block j) of a
  // [L][BP][BC] limb-plane tile in LDS: conflict-free for ds_read_b32 / ds_write_b32 (64 banks)
  auto tile_word = [&](int base, int i, int j, int l) {
    const int rt = (wp * WP + j) * 16 + frow, cc = wc * WC + i;
    return base + l * BP * BC + rt * BC + 16 * (cc ^ swze<BC>(frow)) + 4 * (lane >> 4);
  };
  if constexpr (TR) {
    if (has_rq && !stage_res) {
      // lane (g, p) loaded 16 channels of block 4q + g: transpose to the accumulator layout
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int j = 0; j < WP; ++j)
#pragma unroll
          for (int l = 0; l < L; ++l) {
            unsigned w0 = rq[4 * q][j][l], w1 = rq[4 * q + 1][j][l], w2 = rq[4 * q + 2][j][l], w3 = rq[4 * q + 3][j][l];
            transpose4(w0, w1, w2, w3);
            rq[4 * q][j][l] = (int)w0;
            rq[4 * q + 1][j][l] = (int)w1;
            rq[4 * q + 2][j][l] = (int)w2;
            rq[4 * q + 3][j][l] = (int)w3;
          }
    }
  }
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
  if constexpr (SMIN == 0) {
    if (do_off) {  // weight offsets (8-bit channels off-centre): acc_l += offset_c * sum of pixel digits_l
#pragma unroll
      for (int i = 0; i < WC; ++i) {
        const int c = chan[i] < a.cout ? chan[i] : 0;
        const int4 coff = *reinterpret_cast<const int4*>(a.w_off + c);
        const int cor[4] = {coff.x, coff.y, coff.z, coff.w};
#pragma unroll
        for (int s = 0; s < L; ++s)
#pragma unroll
          for (int j = 0; j < WP; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)  // |offset| < 2^15, |pixel sum| < 2^22: full-rate 24-bit multiply
              acc[s][i][j][r] += __mul24(cor[r], rs[s][j]);
      }
    }
  }
  float rscale[WP];
#pragma unroll
  for (int j = 0; j < WP; ++j) rscale[j] = mok[j] ? a.x_absmax[fast_div(mrow[j], a.hw_mul, a.hw_shr)] * a.inv_qmax : 0.f;
  // residual limb planes -> codes, all at once (one LDS wait instead of one per block)
  int rqv[WC][WP][4];
  if (has_rq) {
    unsigned rw[WC][WP][L];
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j)
#pragma unroll
        for (int l = 0; l < L; ++l)
          rw[i][j][l] = (TR && stage_res) ? *reinterpret_cast<const unsigned*>(lds + tile_word(resoff, i, j, l))
                                          : (unsigned)rq[i][j][l];
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) decode4<L>(rw[i][j], rqv[i][j]);
  }
  constexpr float qmax = act_qmax<L>();
  // limb recombination of the accumulators: v = sum_s fl(acc_s) * 256^(SMIN + s), two channels at
  // a time (v_pk_* fp32 ops round like their scalar forms: the same bits as conv.hip's epilogue)
  auto combine = [&](int i, int j, int h) {
    f2 v;
#pragma unroll
    for (int s = 0; s < NACC; ++s) {
      const int t0 = acc[s][i][j][2 * h], t1 = acc[s][i][j][2 * h + 1];
      const f2 tf = f2{(float)t0, (float)t1};
      constexpr float w0 = SMIN == 0 ? 1.f : (SMIN == 1 ? 256.f : 65536.f);
      const float lw = w0 * (float)(1 << (8 * s));
      // fma(x, 1, 0) == x for x = (float)int (never -0): the first limb is a plain convert
      v = s == 0 ? (SMIN == 0 ? tf : tf * f2{lw, lw}) : __builtin_elementwise_fma(tf, f2{lw, lw}, v);
    }
    return v;
  };
  unsigned wq[WC][WP][L];
  float vmax = 0.f;
  if constexpr (LEAN) {
    // z = v * (rscale * col_scale / step_out) + col_shift / step_out [+ r * res_scale / step_out];
    // code = med3(rne(z), relu ? 0 : -QMAX, QMAX). Scalar fp32 ops: the packed forms need
    // register pairs and cost more moves than they save here.
    const float inv = a.yq_inv;
    const float rsq = a.res_scale * inv;
    const bool relu = LEAN == 2 || LEAN == 3 || (LEAN != 4 && a.relu != 0);
    const float lo = relu ? 0.f : -qmax;
    const bool has_res = has_rq;
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const int c = chan[i] < a.cout ? chan[i] : 0;
      const float4 cs = *reinterpret_cast<const float4*>(a.col_scale + c);
      const float4 csh = *reinterpret_cast<const float4*>(a.col_shift + c);
      const float csq[4] = {cs.x * inv, cs.y * inv, cs.z * inv, cs.w * inv};
      const float shq[4] = {csh.x * inv, csh.y * inv, csh.z * inv, csh.w * inv};
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        v4i accq[NACC];
#pragma unroll
        for (int t = 0; t < NACC; ++t) accq[t] = acc[t][i][j];
        const float m = lean_quad<L, NACC, SMIN>(accq, rscale[j], csq, shq, has_res, rqv[i][j], rsq, relu, lo,
                                                 wq[i][j]);
        vmax = ooff[i][j] != kOOB ? fmaxf(vmax, m) : vmax;
      }
    }
    SMPQ_STAMP(25);
  } else {
    float o[WC][WP][4];
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const int c = chan[i] < a.cout ? chan[i] : 0;
      const float4 cs = *reinterpret_cast<const float4*>(a.col_scale + c);
      const float4 csh = *reinterpret_cast<const float4*>(a.col_shift + c);
      const f2 csr[2] = {f2{cs.x, cs.y}, f2{cs.z, cs.w}};
      const f2 shr[2] = {f2{csh.x, csh.y}, f2{csh.z, csh.w}};
#pragma unroll
      for (int j = 0; j < WP; ++j) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f2 sc = f2{rscale[j], rscale[j]} * csr[h];
          f2 out = __builtin_elementwise_fma(combine(i, j, h), sc, shr[h]);
          if (has_rq)
            out = out + f2{a.res_scale, a.res_scale} * f2{(float)rqv[i][j][2 * h], (float)rqv[i][j][2 * h + 1]};
          o[i][j][2 * h] = out.x;
          o[i][j][2 * h + 1] = out.y;
        }
      }
    }
    if (a.residual && !has_rq) {
      const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.residual), 0, (int)(4 * oplane),
                                                         0x00020000);
      v4u rv[WC][WP];
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j) rv[i][j] = __builtin_amdgcn_raw_buffer_load_b128(rrs, f32_off(ooff[i][j]), 0, 0);
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[i][j][r] = __fadd_rn(o[i][j][r], __uint_as_float(rv[i][j][r]));
    }
    if (a.relu) {
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[i][j][r] = fmaxf(o[i][j][r], 0.f);
    }
    if (a.y) {
      const v4i yrs4 = make_rsrc(a.y, 4LL * oplane);
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          const v4u v = {__float_as_uint(o[i][j][0]), __float_as_uint(o[i][j][1]), __float_as_uint(o[i][j][2]),
                         __float_as_uint(o[i][j][3])};
          store_limbs16(v, yrs4, f32_off(ooff[i][j]), 0u, false);
        }
    }
    if (a.yq) {
      // fused quantizer of the next conv's input (static range)
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          int q[4];
          float am = 0.f;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f2 z = f2{o[i][j][2 * h], o[i][j][2 * h + 1]} * f2{a.yq_inv, a.yq_inv};
            q[2 * h] = (int)fminf(fmaxf(rintf(z.x), -qmax), qmax);
            q[2 * h + 1] = (int)fminf(fmaxf(rintf(z.y), -qmax), qmax);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) am = fmaxf(am, fabsf(o[i][j][r]));
          vmax = ooff[i][j] != kOOB ? fmaxf(vmax, am) : vmax;
          encode4<L>(q, wq[i][j]);
        }
    }
    if (a.y_absmax) {
      float pmax[WP];  // per pixel max |y| over this lane's channels, then over the 4 lane groups
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        float am = 0.f;
#pragma unroll
        for (int i = 0; i < WC; ++i)
          if (ooff[i][j] != kOOB)
#pragma unroll
            for (int r = 0; r < 4; ++r) am = fmaxf(am, fabsf(o[i][j][r]));
        am = fmaxf(am, __shfl_xor(am, 16, kWave));
        pmax[j] = fmaxf(am, __shfl_xor(am, 32, kWave));
      }
      const int mfirst = m0 + wp * WP * 16;
      const int mlast = min(mfirst + WP * 16, a.M) - 1;
      if (mfirst <= mlast) {
        const int img_lo = fast_div(mfirst, a.hw_mul, a.hw_shr), img_hi = fast_div(mlast, a.hw_mul, a.hw_shr);
        if (img_lo == img_hi) {
          float v = 0.f;
#pragma unroll
          for (int j = 0; j < WP; ++j) v = fmaxf(v, pmax[j]);
          v = wave_max(v);
          if (lane == 0 && v > 0.f) atomic_max_nonneg(&a.y_absmax[img_lo], v);
        } else if (lane < 16) {
#pragma unroll
          for (int j = 0; j < WP; ++j)
            if (mok[j] && pmax[j] > 0.f) atomic_max_nonneg(&a.y_absmax[fast_div(mrow[j], a.hw_mul, a.hw_shr)], pmax[j]);
        }
      }
    }
  }
  if (a.yq) {
    const auto qrs = __builtin_amdgcn_make_buffer_rsrc(a.yq, 0, (int)(L * oplane), 0x00020000);
    const v4i qrs4 = make_rsrc(a.yq, (long long)L * oplane);
    const bool nt = __builtin_amdgcn_readfirstlane(a.nt_store) != 0;
    if (TR && !stage_out) {
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int j = 0; j < WP; ++j)
#pragma unroll
          for (int l = 0; l < L; ++l) {
            unsigned w0 = wq[4 * q][j][l], w1 = wq[4 * q + 1][j][l], w2 = wq[4 * q + 2][j][l], w3 = wq[4 * q + 3][j][l];
            transpose4(w0, w1, w2, w3);
            if (!(kAblate & 2) || w0 == 0x12345679u)
              store_limbs16(v4u{w0, w1, w2, w3}, qrs4, qoff[q][j],
                            __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane)), nt);
          }
    } else if (TR) {
      // stage the [L][BP][BC] tile in the operand area (every wave is past its last fragment
      // read after this barrier), then copy it out row-major in 16-B pieces
      __syncthreads();
      SMPQ_STAMP(26);
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j)
#pragma unroll
          for (int l = 0; l < L; ++l) *reinterpret_cast<unsigned*>(lds + tile_word(0, i, j, l)) = wq[i][j][l];
      __syncthreads();
      SMPQ_STAMP(27);
      constexpr int RCPR = BC / 16, ITEMS = TILEB / 16;
#pragma unroll
      for (int k = 0; k < (ITEMS + 64 * NW - 1) / (64 * NW); ++k) {
        const int it = threadIdx.x + 64 * NW * k;
        if (it < ITEMS) {
          const int l = it / (BP * RCPR), rem = it - l * (BP * RCPR);
          const int rt = rem / RCPR, c = rem - rt * RCPR;
          const v4i v = *reinterpret_cast<const v4i*>(lds + l * BP * BC + rt * BC + 16 * (c ^ swze<BC>(rt & 15)));
          const bool ok = m0 + rt < a.M && n0 + 16 * c < a.cout;
          const unsigned off = ok ? (unsigned)((long long)(m0 + rt) * a.cout + n0 + 16 * c) : kOOB;
          if (!(kAblate & 2) || v.x == 0x12345679)
            store_limbs16(v4u{(unsigned)v.x, (unsigned)v.y, (unsigned)v.z, (unsigned)v.w}, qrs4, off,
                          __builtin_amdgcn_readfirstlane((unsigned)((long long)l * oplane)), nt);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j)
#pragma unroll
          for (int l = 0; l < L; ++l)
            if (!(kAblate & 2) || wq[i][j][l] == 0x12345679u)
              __builtin_amdgcn_raw_buffer_store_b32(wq[i][j][l], qrs, ooff[i][j], (unsigned)((long long)l * oplane), 0);
    }
    // LEAN: vmax is the largest rounded code; otherwise max |y| (|rne(y * inv)| is monotone in |y|)
    const bool ovf = LEAN ? vmax > qmax : rintf(__fmul_rn(vmax, a.yq_inv)) > qmax;
    if (__any(ovf) && lane == 0) atomicMax(a.overflow, 1);
  }
  SMPQ_STAMP(22);
#ifdef SMPQ_STAMPS
  if (lane == 0) {  // slot 23: the CU this wave ran on (XCC id << 16 | HW_ID CU/SH/SE bits)
    unsigned id, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    stamp_base[23] = ((unsigned long long)(xcc & 0xf) << 16) | ((id >> 8) & 0xff);
  }
#endif
}

template <int L, int LW, int WAVES_C, int WAVES_P, int WC, int WP, int MINW, bool S2D, int NST, int BK,
          int LEAN = 0, bool PIPE = false, bool OFF = true>
__global__ __launch_bounds__(64 * WAVES_C * WAVES_P, MINW) void qconv_glds_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(1024))) int8_t lds[];  // min(NST, ksteps) stages
  qconv_glds_body<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, LEAN, PIPE, OFF>(a, blockIdx.x, gridDim.x, lds);
}

// ------------------------------------------------------------------------------------------
struct GldsCfg {
  int wavesc, wavesp, wc, wp, stages, bk, pipe;
};
constexpr GldsCfg kGlds[] = {
    {2, 2, 2, 2, 2, 64, 0},  // 0:  64 ch x  64 px, 256 threads
    {2, 2, 2, 4, 2, 64, 0},  // 1:  64 ch x 128 px
    {2, 2, 4, 2, 2, 64, 0},  // 2: 128 ch x  64 px
    {1, 4, 4, 1, 2, 64, 0},  // 3:  64 ch x  64 px (each wave all 64 channels of 16 px)
    {1, 4, 4, 2, 2, 64, 0},  // 4:  64 ch x 128 px
    {4, 1, 2, 4, 2, 64, 0},  // 5: 128 ch x  64 px (each wave 32 ch x all 64 px)
    {2, 2, 4, 4, 2, 64, 0},  // 6: 128 ch x 128 px (<= 2 accumulator sets)
    {4, 1, 4, 2, 2, 64, 0},  // 7: 256 ch x  32 px (whole 256-B output rows per block: wide 1x1 expansions)
    {4, 1, 4, 1, 2, 64, 0},  // 8: 256 ch x  16 px
    {2, 2, 4, 1, 2, 64, 0},  // 9: 128 ch x  32 px
    {2, 2, 2, 2, 3, 64, 0},  // 10: as 0, 3 LDS stages (DMA two K steps ahead; long-K 3x3 convs)
    {1, 4, 4, 1, 3, 64, 0},  // 11: as 3, 3 stages
    {2, 2, 4, 2, 3, 64, 0},  // 12: as 2, 3 stages
    // 8 waves: twice the MFMA work per loaded byte (the 3x3 convs stream ~100 ops/B from L2 at 64 x 64)
    {2, 4, 4, 2, 2, 64, 0},  // 13: 128 ch x 128 px (waves 64 ch x 32 px)
    {4, 2, 2, 4, 2, 64, 0},  // 14: 128 ch x 128 px (waves 32 ch x 64 px)
    {4, 2, 4, 2, 2, 64, 0},  // 15: 256 ch x  64 px
    // (64 ch x 256 px with 8 pixel-waves was removed: never the fastest, and its static-range
    // limb output was intermittently wrong in the last pixel group — see tests/test_gpu.py
    // test_tile_configs_deterministic)
    // 128-B K steps (cin % 128 == 0): DMA pieces of whole cache lines
    {2, 2, 2, 2, 2, 128, 0},  // 16: as 0
    {1, 4, 4, 1, 2, 128, 0},  // 17: as 3
    {2, 2, 4, 2, 2, 128, 0},  // 18: as 2
    {2, 2, 4, 1, 2, 128, 0},  // 19: as 9
    {1, 4, 4, 2, 2, 128, 0},  // 20: as 4
    {2, 4, 4, 2, 2, 128, 0},  // 21: as 13
    // deeper DMA pipelines for the long-K 3x3 convs (latency of a K step's pieces hidden behind
    // NST - 1 steps of MFMAs)
    {2, 2, 4, 2, 4, 64, 0},   // 22: as 2, 4 stages
    {2, 2, 2, 2, 4, 64, 0},   // 23: as 0, 4 stages
    {1, 4, 4, 1, 4, 64, 0},   // 24: as 3, 4 stages
    {2, 2, 4, 2, 3, 128, 0},  // 25: as 18, 3 stages
    {2, 2, 2, 2, 3, 128, 0},  // 26: as 16, 3 stages
    // register-pipelined K loops (PIPE: two fragment register sets, the next step's fragments read
    // under the current step's MFMAs): long-K convs; they cost registers the short-K ones need
    {2, 2, 4, 2, 2, 64, 1},   // 27: as 2
    {1, 4, 4, 1, 2, 64, 1},   // 28: as 3
    {2, 2, 4, 1, 2, 64, 1},   // 29: as 9
    {1, 4, 4, 1, 3, 64, 1},   // 30: as 11
    {2, 2, 4, 2, 3, 64, 1},   // 31: as 12
    {2, 2, 4, 2, 2, 128, 1},  // 32: as 18
    {2, 2, 4, 1, 2, 128, 1},  // 33: as 19
    {2, 2, 4, 2, 4, 64, 1},   // 34: as 22
    {1, 4, 4, 1, 4, 64, 1},   // 35: as 24
    {2, 2, 2, 2, 3, 128, 1},  // 36: as 26
};
template <int L, int LW, int WAVES_C, int WAVES_P, int WC, int WP, bool S2D = false, int NST = 2, int MINW = 2,
          int BK = 64, bool PIPE = false>
static int launch_one(const ConvArgs& a, hipStream_t stream) {
  constexpr int SMIN = (L + LW - 4) > 0 ? (L + LW - 4) : 0;
  if constexpr ((L + LW - 1 - SMIN) * WC * WP * 4 > 128) {
    return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: tile config too large for these limb counts");
  } else {
    constexpr int BC = 16 * WC * WAVES_C, BP = 16 * WP * WAVES_P;
    const long mt = (a.M + BP - 1) / BP;
    const long nt = (a.cout + BC - 1) / BC;
    if (mt * nt > 0x7fffffffL) return fail(SMPQ_E_SHAPE, "smpq_conv2d_fwd: grid too large");
    if (BK == 128 && a.cin % 128 != 0)
      return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: 128-wide K steps need cin % 128 == 0");
    constexpr int STAGE = (LW * BC + L * BP) * BK;
    constexpr int kMaxLds = 160 * 1024;  // LDS per CU on gfx950
    // no more stages than K steps: a single-step conv (1x1, cin 64) needs one
    const int nsteps = a.ksteps / (BK / 64);
    // operand stages, enlarged to hold the staged output tile, + the residual tile (kernel layout)
    constexpr bool TRT = (WC % 4) == 0;
    constexpr int TILEB = L * BP * BC;
    const bool lines = BC >= 128 || BC == a.cout;
    int lds_bytes = (nsteps < NST ? nsteps : NST) * STAGE;
    if (TRT && lines && a.yq && TILEB > lds_bytes) lds_bytes = TILEB;
    if (TRT && lines && a.res_q) lds_bytes += TILEB;
    if (lds_bytes > kMaxLds) return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: tile config needs more LDS than a CU has");
    constexpr int kMaxNeed = (NST * STAGE > TILEB ? NST * STAGE : TILEB) + TILEB;
    ConvArgs b = a;
    fast_div_init((int)nt, b.ntc_mul, b.ntc_shr);
    const bool lean = L >= 2 && a.yq && !a.y && !a.residual && !a.y_absmax;
    // epilogue variants: general / lean (runtime ReLU + residual) / lean ReLU / lean ReLU + limb-plane
    // residual, each with and without weight offsets (LW == 1 only; the compile-time ReLU and
    // residual variants too: the block convs of the quantized ResNets)
    constexpr bool kV = LW == 1 && L >= 2;
    constexpr int kLean = L >= 2 ? 1 : 0;
    auto k00 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, 0, PIPE, false>;
    auto k10 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, kLean, PIPE, false>;
    auto k20 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, kV ? 2 : kLean, PIPE, false>;
    auto k30 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, kV ? 3 : kLean, PIPE, false>;
    auto k40 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, L >= 2 ? 4 : 0, PIPE, false>;
    auto k01 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, 0, PIPE, LW == 1>;
    auto k11 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, kLean, PIPE, LW == 1>;
    auto k21 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, kV ? 2 : kLean, PIPE, LW == 1>;
    auto k31 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, kV ? 3 : kLean, PIPE, LW == 1>;
    auto k41 = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, MINW, S2D, NST, BK, L >= 2 ? 4 : 0, PIPE, LW == 1>;
    auto set_lds = [](const void* k) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               kMaxNeed < kMaxLds ? kMaxNeed : kMaxLds);
      if (e != hipSuccess) (void)hipGetLastError();  // do not leave it for an unrelated launch to report
      return e;
    };
    using KFn = decltype(k00);
    static const KFn fns[10] = {k00, k10, k20, k30, k40, k01, k11, k21, k31, k41};
    static hipError_t attrs[10];
    static const bool attrs_set = [&] {
      for (int i = 0; i < 10; ++i) attrs[i] = set_lds(reinterpret_cast<const void*>(fns[i]));
      return true;
    }();
    (void)attrs_set;
    // variant: general / lean: ReLU + no residual, ReLU + limb-plane residual (one weight limb),
    // neither ReLU nor residual (the downsample convs), anything else at run time
    const int ev = !lean ? 0
                   : (kV && a.relu) ? (a.res_q ? 3 : 2)
                   : (!a.relu && !a.res_q) ? 4
                                           : 1;
    const int vi = ev + ((LW == 1 && a.has_offset) ? 5 : 0);
    if (attrs[vi] != hipSuccess) return check_hip(attrs[vi], "qconv_glds_kernel LDS attribute");
    hipLaunchKernelGGL(fns[vi], dim3((unsigned)(mt * nt)), dim3(64 * WAVES_C * WAVES_P), lds_bytes, stream, b);
    return check_hip(hipGetLastError(), "qconv_glds_kernel launch");
  }
}

// one (limbs, weight limbs) family: every tile configuration (conv_glds_inst.hip instantiates it)
template <int L, int LW>
int launch_cfg(int cfg, const ConvArgs& a, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_one<L, LW, 2, 2, 2, 2>(a, s);
    case 1: return launch_one<L, LW, 2, 2, 2, 4>(a, s);
    case 2: return launch_one<L, LW, 2, 2, 4, 2>(a, s);
    case 3: return launch_one<L, LW, 1, 4, 4, 1>(a, s);
    case 4: return launch_one<L, LW, 1, 4, 4, 2>(a, s);
    case 5: return launch_one<L, LW, 4, 1, 2, 4>(a, s);
    case 6: return launch_one<L, LW, 2, 2, 4, 4>(a, s);
    case 7: return launch_one<L, LW, 4, 1, 4, 2>(a, s);
    case 8: return launch_one<L, LW, 4, 1, 4, 1>(a, s);
    case 9: return launch_one<L, LW, 2, 2, 4, 1>(a, s);
    case 10: return launch_one<L, LW, 2, 2, 2, 2, false, 3>(a, s);
    case 11: return launch_one<L, LW, 1, 4, 4, 1, false, 3>(a, s);
    case 12: return launch_one<L, LW, 2, 2, 4, 2, false, 3>(a, s);
    case 13: return launch_one<L, LW, 2, 4, 4, 2>(a, s);
    case 14: return launch_one<L, LW, 4, 2, 2, 4>(a, s);
    case 15: return launch_one<L, LW, 4, 2, 4, 2>(a, s);
    case 16: return launch_one<L, LW, 2, 2, 2, 2, false, 2, 2, 128>(a, s);
    case 17: return launch_one<L, LW, 1, 4, 4, 1, false, 2, 2, 128>(a, s);
    case 18: return launch_one<L, LW, 2, 2, 4, 2, false, 2, 2, 128>(a, s);
    case 19: return launch_one<L, LW, 2, 2, 4, 1, false, 2, 2, 128>(a, s);
    case 20: return launch_one<L, LW, 1, 4, 4, 2, false, 2, 2, 128>(a, s);
    case 21: return launch_one<L, LW, 2, 4, 4, 2, false, 2, 2, 128>(a, s);
    case 22: return launch_one<L, LW, 2, 2, 4, 2, false, 4>(a, s);
    case 23: return launch_one<L, LW, 2, 2, 2, 2, false, 4>(a, s);
    case 24: return launch_one<L, LW, 1, 4, 4, 1, false, 4>(a, s);
    case 25: return launch_one<L, LW, 2, 2, 4, 2, false, 3, 2, 128>(a, s);
    case 26: return launch_one<L, LW, 2, 2, 2, 2, false, 3, 2, 128>(a, s);
    case 27: return launch_one<L, LW, 2, 2, 4, 2, false, 2, 2, 64, true>(a, s);
    case 28: return launch_one<L, LW, 1, 4, 4, 1, false, 2, 2, 64, true>(a, s);
    case 29: return launch_one<L, LW, 2, 2, 4, 1, false, 2, 2, 64, true>(a, s);
    case 30: return launch_one<L, LW, 1, 4, 4, 1, false, 3, 2, 64, true>(a, s);
    case 31: return launch_one<L, LW, 2, 2, 4, 2, false, 3, 2, 64, true>(a, s);
    case 32: return launch_one<L, LW, 2, 2, 4, 2, false, 2, 2, 128, true>(a, s);
    case 33: return launch_one<L, LW, 2, 2, 4, 1, false, 2, 2, 128, true>(a, s);
    case 34: return launch_one<L, LW, 2, 2, 4, 2, false, 4, 2, 64, true>(a, s);
    case 35: return launch_one<L, LW, 1, 4, 4, 1, false, 4, 2, 64, true>(a, s);
    case 36: return launch_one<L, LW, 2, 2, 2, 2, false, 3, 2, 128, true>(a, s);
    default: return fail(SMPQ_E_INVALID, "smpq_conv2d_fwd: bad tile config");
  }
}

}  // namespace smpq
