// Where does a K step of the LDS-DMA conv kernel spend its cycles? Diagnostic harness: compiles ONE
// qconv_glds_kernel instance with -DSMPQ_STAMPS (shader-clock stamps at fixed points, see
// conv_glds.hip) and runs it on a synthetic R50 shape (operand values random: timing only).
//
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSMPQ_STAMPS -DSMPQ_KERNEL_ONLY \
//   -I semilayer-wise-mixed-precision-quantization_amd/csrc tools/stamp_bench.hip -o tools/bin/stamp_bench
// ./tools/bin/stamp_bench [cin cout k hw [bk [stride]]]   (default: 3x3 256->256 at 14x14, B = 256, BK 64)
// Without -DSMPQ_STAMPS it only times the launch (add -DSB_LW=3 for the downsample's weight limbs,
// -DSMPQ_DIAG_ABLATE=N for conv_glds.hip's diagnostic ablations).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "conv_glds_kernel.h"

using namespace smpq;

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                       \
    }                                                                 \
  } while (0)

template <int BK>
int run(int argc, char** argv) {
  const int n = 256, cin = argc > 1 ? atoi(argv[1]) : 256, cout = argc > 2 ? atoi(argv[2]) : 256,
            k = argc > 3 ? atoi(argv[3]) : 3, hw = argc > 4 ? atoi(argv[4]) : 14,
            stride = argc > 6 ? atoi(argv[6]) : 1;
#ifndef SB_LW
#define SB_LW 1
#endif
  constexpr int L = 3, LW = SB_LW, WAVES_C = 2, WAVES_P = 2, WC = 4, WP = 2, NST = 2, NW = 4;
  constexpr int BC = 16 * WC * WAVES_C, BP = 16 * WP * WAVES_P, STAGE = (LW * BC + L * BP) * BK;
  ConvArgs a{};
  a.n = n; a.h = hw; a.w = hw; a.cin = cin; a.cout = cout; a.kh = k; a.kw = k; a.stride = stride; a.pad = k / 2;
  a.ho = (hw + 2 * a.pad - k) / stride + 1; a.wo = a.ho; a.M = n * a.ho * a.wo; a.K = k * k * cin; a.cchunks = cin / 64; a.ksteps = k * k * a.cchunks;
  a.plane = (long long)n * hw * hw * cin; a.wplane = (long long)cout * a.K;
  a.relu = 1; a.inv_qmax = 1.f / 8323072.f; a.yq_inv = 8323072.f / 1000.f;
  fast_div_init(a.ho * a.wo, a.hw_mul, a.hw_shr);
  fast_div_init(a.wo, a.wo_mul, a.wo_shr);
  const int mt = (a.M + BP - 1) / BP, nt = (cout + BC - 1) / BC, blocks = mt * nt;
  fast_div_init(nt, a.ntc_mul, a.ntc_shr);
  int8_t *xq, *codes, *yq;
  float *amax, *cs, *sh;
  int32_t* ovf;
  unsigned long long* st;
  CK(hipMalloc(&xq, L * a.plane));
  CK(hipMalloc(&codes, LW * a.wplane));
  CK(hipMalloc(&yq, (size_t)L * a.M * cout));
  CK(hipMalloc(&amax, n * 4));
  CK(hipMalloc(&cs, cout * 4));
  CK(hipMalloc(&sh, cout * 4));
  CK(hipMalloc(&ovf, 4));
  CK(hipMalloc(&st, (size_t)blocks * NW * 32 * 8));
  {
    std::vector<int8_t> hx(L * a.plane), hw8(LW * a.wplane);
    for (auto& v : hx) v = (int8_t)(rand() % 256 - 128);
    for (auto& v : hw8) v = (int8_t)(rand() % 64 - 32);
    std::vector<float> one(std::max(n, cout), 1e-3f);
    CK(hipMemcpy(xq, hx.data(), hx.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(codes, hw8.data(), hw8.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(amax, one.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(cs, one.data(), cout * 4, hipMemcpyHostToDevice));
    CK(hipMemset(sh, 0, cout * 4));
    CK(hipMemset(ovf, 0, 4));
    CK(hipMemset(st, 0, (size_t)blocks * NW * 32 * 8));
  }
  a.xq = xq; a.x_absmax = amax; a.codes = codes; a.col_scale = cs; a.col_shift = sh; a.yq = yq; a.overflow = ovf;
#ifdef SMPQ_STAMPS
  CK(hipMemcpyToSymbol(HIP_SYMBOL(smpq_stamps), &st, sizeof(st)));
#else
  printf("{\"shape\": \"%dx%d/%d %d->%d at %d^2, B=%d, BK=%d, LW=%d, ablate=%d\", \"kernel_us\": ", k, k, stride, cin, cout,
         hw, n, BK, LW, SMPQ_DIAG_ABLATE);
#endif
  auto kern = qconv_glds_kernel<L, LW, WAVES_C, WAVES_P, WC, WP, 2, false, NST, BK, 1, false>;
  const int nsteps = a.ksteps / (BK / 64);
  constexpr int TILEB = L * BP * BC;  // the staged output tile (WC % 4 == 0 and BC >= 128: lines)
  const int lds = std::max(std::min(nsteps, NST) * STAGE, TILEB);
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * NW), lds, 0, a);
  CK(hipEventRecord(e0));
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * NW), lds, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
#ifndef SMPQ_STAMPS
  printf("%.1f}\n", ms * 1e3);
  return 0;
#endif
  std::vector<unsigned long long> h((size_t)blocks * NW * 32);
  CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  // per wave: prologue (0->1), per K step (barrier to barrier, steps 1..14), step 6 split
  // (barrier -> fragments in registers -> DMA issued -> MFMAs retired -> next barrier), K loop end
  // -> epilogue end; medians over all waves
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
  };
  std::vector<double> pro, step, rd, iss, mf, rest, epi, life, skew, wait0, kloop, e_comp, e_sync, e_stage, e_out;
  for (int b = 0; b < blocks; ++b) {
    unsigned long long bar6[NW];
    for (int w = 0; w < NW; ++w) {
      const unsigned long long* t = &h[((size_t)b * NW + w) * 32];
      pro.push_back((double)(t[1] - t[0]));
      const int last = std::min(nsteps, 16) - 1;
      if (last >= 2) step.push_back((double)(t[2 + last] - t[3]) / (last - 1));
      if (nsteps > 7) {
        rd.push_back((double)(t[18] - t[8]));
        iss.push_back((double)(t[19] - t[18]));
        mf.push_back((double)(t[20] - t[19]));
        rest.push_back((double)(t[9] - t[20]));
      }
      wait0.push_back((double)(t[2] - t[1]));
      kloop.push_back((double)(t[21] - t[2]));
      epi.push_back((double)(t[22] - t[21]));
      if (t[25]) e_comp.push_back((double)(t[25] - t[21]));
      if (t[26] && t[25]) e_sync.push_back((double)(t[26] - t[25]));
      if (t[27] && t[26]) e_stage.push_back((double)(t[27] - t[26]));
      if (t[27]) e_out.push_back((double)(t[22] - t[27]));
      life.push_back((double)(t[22] - t[0]));
      bar6[w] = t[8];
    }
    unsigned long long lo = bar6[0], hi = bar6[0];
    for (int w = 1; w < NW; ++w) lo = std::min(lo, bar6[w]), hi = std::max(hi, bar6[w]);
    skew.push_back((double)(hi - lo));
  }
  // residency: per CU (slot 23), the most blocks alive at one instant and the mean over the kernel
  double conc_sum = 0;
  int conc_max = 0, ncu = 0;
  {
    std::vector<std::vector<std::pair<unsigned long long, int>>> ev(1 << 20);
    std::vector<int> used;
    for (int b = 0; b < blocks; ++b) {
      const unsigned long long* t = &h[(size_t)b * NW * 32];
      const unsigned cu = (unsigned)t[23] & 0xfffff;
      if (ev[cu].empty()) used.push_back((int)cu);
      ev[cu].push_back({t[0], 1});
      ev[cu].push_back({t[22], -1});
    }
    for (int cu : used) {
      auto& e = ev[cu];
      std::sort(e.begin(), e.end());
      int cur = 0;
      unsigned long long busy = 0, area = 0, prev = e.front().first;
      for (auto& x : e) {
        if (cur > 0) busy += x.first - prev, area += (x.first - prev) * cur;
        cur += x.second;
        prev = x.first;
        conc_max = std::max(conc_max, cur);
      }
      conc_sum += busy ? (double)area / busy : 0;
      ++ncu;
    }
  }
  printf("{\"cus_seen\": %d, \"max_blocks_per_cu\": %d, \"mean_blocks_per_cu_while_busy\": %.2f}\n", ncu, conc_max,
         ncu ? conc_sum / ncu : 0.0);
  printf("{\"shape\": \"%dx%d %d->%d at %d^2, B=%d, BK=%d\", \"blocks\": %d, \"ksteps\": %d, \"kernel_us\": %.1f, "
         "\"median_cycles\": {\"prologue\": %.0f, \"per_k_step\": %.0f, \"step6_barrier_to_frags\": %.0f, "
         "\"step6_dma_issue\": %.0f, \"step6_mfma_issue_to_retire\": %.0f, \"step6_to_next_barrier\": %.0f, "
         "\"epilogue\": %.0f, \"block_life\": %.0f, \"barrier_exit_skew\": %.0f, \"first_dma_wait\": %.0f, "
         "\"k_loop_after_first_barrier\": %.0f, \"epi_loads_and_math\": %.0f, \"epi_first_sync\": %.0f, "
         "\"epi_lds_stage\": %.0f, \"epi_copy_out_and_flag\": %.0f}}\n",
         k, k, cin, cout, hw, n, BK, blocks, nsteps, ms * 1e3, med(pro), med(step), med(rd), med(iss), med(mf),
         med(rest), med(epi), med(life), med(skew), med(wait0), med(kloop), med(e_comp), med(e_sync), med(e_stage),
         med(e_out));
  return 0;
}

int main(int argc, char** argv) { return (argc > 5 && atoi(argv[5]) == 128) ? run<128>(argc, argv) : run<64>(argc, argv); }
