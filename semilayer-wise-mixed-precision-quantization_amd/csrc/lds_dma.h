// LDS-DMA staging helpers shared by the LDS-DMA conv kernels (conv_glds.hip, conv_stream.hip):
// buffer resources, one-KiB DMA pieces into swizzled LDS images, hazard-padded inline-asm stores,
// the lane-group transpose of the 16-B limb-plane epilogue. Not part of the public ABI.
#pragma once

#include "conv_common.h"

namespace smpq {
namespace {

constexpr unsigned kOOB = 0x80000000u;  // a buffer offset past every range we build (< 2^31 B)
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// Inline-asm VMEM instructions are invisible to the compiler's hazard recognizer, so they carry
// their own wait states on both sides:
//  * before: 5 (s_nop 4) — a VALU write of an SGPR (v_readfirstlane / v_readlane, e.g. an SGPR
//    restored from a VGPR lane under SGPR pressure) needs 5 wait states before a VMEM instruction
//    reads it as soffset / resource (observed: a limb-plane store whose soffset came from a
//    v_readlane one instruction earlier wrote its plane at a stale offset);
//  * after (stores): 2 (s_nop 1) — a VMEM store of more than 8 bytes must not have its data VGPRs
//    overwritten by the very next instruction (observed: dword 0 of a limb-plane store replaced by
//    the register's next value when a v_mov to it directly followed the store).
// 16-B store with the default (temporal) or the non-temporal cache policy (gfx950 CPol nt); nt is
// wave-uniform.
__device__ __forceinline__ void store_limbs16(v4u v, v4i rs, unsigned off, unsigned soff, bool nt) {
  if (nt)
    asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, %3 offen nt\n\ts_nop 1" ::"v"(v), "v"(off), "s"(rs),
                 "s"(soff)
                 : "memory");
  else
    asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, %3 offen\n\ts_nop 1" ::"v"(v), "v"(off), "s"(rs),
                 "s"(soff)
                 : "memory");
}

// byte offset of an fp32 element offset (kOOB stays out of range: 4 * kOOB would wrap to 0)
__device__ __forceinline__ unsigned f32_off(unsigned e) { return e == kOOB ? kOOB : 4u * e; }

__device__ __forceinline__ v4i make_rsrc(const void* base, long long bytes) {
  const unsigned long long b = reinterpret_cast<unsigned long long>(base);
  v4i r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
  r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));  // stride 0
  r.z = __builtin_amdgcn_readfirstlane((int)(unsigned)bytes);
  r.w = 0x00020000;
  return r;
}

// One 1-KiB piece: lane i's 16 bytes at rsrc[voff + soff] -> LDS [lds + 16 i, +16). The leading
// s_nop 1, the two s_movs and the s_nop 0 give the 5 wait states a VALU-written soffset / resource SGPR needs
// (see store_limbs16); the s_nop 0 separates the M0 write from the LDS DMA.
__device__ __forceinline__ void dma16(unsigned lds, v4i rsrc, unsigned voff, unsigned soff) {
  unsigned keep;
  asm volatile(
      "s_nop 1\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds), "s"(soff)
      : "memory");
}

// LDS image of a [rows][BK] operand region: the 16-B chunk c of row r is stored at c ^ swz<BK>(r).
// Conflict-free for the DMA's lane-linear writes and for ds_read_b128 fragment reads (16 rows,
// 16 B each, gfx950 b128 lane groups): BK = 64 rows are 4 chunks, BK = 128 rows are 8 chunks.
template <int BK>
__device__ __forceinline__ int swz(int row) {
  if constexpr (BK == 64) return (4 - (row >> 2)) & 3;
  else return (row >> 1) & 7;
}

// LDS image of a [pixels][BCT] limb-plane tile of the epilogue (BCT = 64 / 128 / 256 output
// channels): chunk c of tile row r at c ^ swze<BCT>(r & 15). Lane (g, p) of the transposed epilogue
// reads/writes row p, chunk 4k + g — the same lane pattern as the MFMA fragment reads, so the same
// XOR rules keep ds_read_b128 / ds_write_b128 and the row-major copy-out conflict-free.
template <int BCT>
__device__ __forceinline__ int swze(int r16) {
  if constexpr (BCT == 64) return (4 - (r16 >> 2)) & 3;
  else if constexpr (BCT == 128) return (r16 >> 1) & 7;
  else return r16 & 15;
}

// 4 x 4 transpose of (lane group g = lane >> 4, register c): afterwards group g register c holds
// what group c register g held. v_permlane32_swap exchanges the upper half of its first operand
// with the lower half of its second, v_permlane16_swap the odd rows of the first with the even
// rows of the second.
__device__ __forceinline__ void transpose4(unsigned& w0, unsigned& w1, unsigned& w2, unsigned& w3) {
  const auto a = __builtin_amdgcn_permlane32_swap(w0, w2, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(w1, w3, false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
  const auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
  w0 = c[0];
  w1 = c[1];
  w2 = d[0];
  w3 = d[1];
}

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

typedef float f2 __attribute__((ext_vector_type(2)));

// Lean static epilogue of one accumulator quad (channels 4g..4g+3 of one pixel): the limb
// accumulators recombined in fp32 (v = sum_s fl(acc_s) * 256^(SMIN + s)), then
// z = v * (rscale * csq) + shq [+ r * rsq] with csq / shq / rsq the column scale / shift / residual
// scale already multiplied by 1 / (output step), code = med3(rne(z), lo, QMAX) (lo = 0 for ReLU).
// Returns the largest rounded |z| (the overflow test: > QMAX), writes the codes' limb dwords. Both
// LDS-DMA kernels use it, so their static-range outputs agree bit for bit.
// lean_codes: the same, returning the clamped codes themselves (the fused stem + max pool pools
// them before encoding).
// lean_codes_v: the same from the recombined v (the limb-outer K loop folds its limbs itself).
template <int L>
__device__ __forceinline__ float lean_codes_v(const float* vs, float rscale, const float* csq, const float* shq,
                                              bool has_res, const int* rqv, float rsq, bool relu, float lo, int* q) {
  constexpr float qmax = act_qmax<L>();
  float m = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float z = __fmaf_rn(vs[r], rscale * csq[r], shq[r]);
    if (has_res) z = __fmaf_rn((float)rqv[r], rsq, z);
    const float zr = rintf(z);
    m = fmaxf(m, relu ? zr : fabsf(zr));
    q[r] = (int)__builtin_amdgcn_fmed3f(zr, lo, qmax);
  }
  return m;
}

template <int L, int NACC, int SMIN>
__device__ __forceinline__ float lean_codes(const v4i* accs, float rscale, const float* csq, const float* shq,
                                            bool has_res, const int* rqv, float rsq, bool relu, float lo, int* q) {
  constexpr float w0 = SMIN == 0 ? 1.f : (SMIN == 1 ? 256.f : 65536.f);
  float vs[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = (float)accs[0][r];
    if (SMIN != 0) v = v * w0;
#pragma unroll
    for (int t = 1; t < NACC; ++t) v = __fmaf_rn((float)accs[t][r], w0 * (float)(1 << (8 * t)), v);
    vs[r] = v;
  }
  return lean_codes_v<L>(vs, rscale, csq, shq, has_res, rqv, rsq, relu, lo, q);
}

template <int L, int NACC, int SMIN>
__device__ __forceinline__ float lean_quad(const v4i* accs, float rscale, const float* csq, const float* shq,
                                           bool has_res, const int* rqv, float rsq, bool relu, float lo,
                                           unsigned* wq) {
  int q[4];
  const float m = lean_codes<L, NACC, SMIN>(accs, rscale, csq, shq, has_res, rqv, rsq, relu, lo, q);
  encode4<L>(q, wq);
  return m;
}

}  // namespace

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be a constant)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define SMPQ_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    SMPQ_VMW(1) SMPQ_VMW(2) SMPQ_VMW(3) SMPQ_VMW(4) SMPQ_VMW(5) SMPQ_VMW(6) SMPQ_VMW(7) SMPQ_VMW(8)
    SMPQ_VMW(9) SMPQ_VMW(10) SMPQ_VMW(11) SMPQ_VMW(12) SMPQ_VMW(13) SMPQ_VMW(14) SMPQ_VMW(15) SMPQ_VMW(16)
    SMPQ_VMW(17) SMPQ_VMW(18) SMPQ_VMW(19) SMPQ_VMW(20) SMPQ_VMW(21) SMPQ_VMW(22) SMPQ_VMW(23) SMPQ_VMW(24)
    SMPQ_VMW(25) SMPQ_VMW(26) SMPQ_VMW(27) SMPQ_VMW(28) SMPQ_VMW(29) SMPQ_VMW(30) SMPQ_VMW(31) SMPQ_VMW(32)
#undef SMPQ_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}


}  // namespace smpq
