// Quantized convolution forward for gfx950, LDS-DMA staged (cin % 64 == 0): tile-configuration
// queries and dispatch. The kernel itself (qconv_glds_kernel) and the design notes are in
// conv_glds_kernel.h; launch_cfg<L, LW> is instantiated per (L, LW) in conv_glds_inst.hip.
#include "conv_glds_kernel.h"

namespace smpq {

#define SMPQ_GLDS_FAMILY(L, LW) extern template int launch_cfg<L, LW>(int, const ConvArgs&, hipStream_t);
SMPQ_GLDS_FAMILY(1, 1)
SMPQ_GLDS_FAMILY(2, 1)
SMPQ_GLDS_FAMILY(3, 1)
SMPQ_GLDS_FAMILY(1, 2)
SMPQ_GLDS_FAMILY(2, 2)
SMPQ_GLDS_FAMILY(3, 2)
SMPQ_GLDS_FAMILY(3, 3)
#undef SMPQ_GLDS_FAMILY

constexpr int kNumGlds = sizeof(kGlds) / sizeof(kGlds[0]);

int glds_num_cfgs() { return kNumGlds + halo_num_cfgs() + resident_num_cfgs(); }

// numbering: LDS-DMA configs, then halo configs, then the weight-stationary 1x1 configs
static int res_base() { return kNumGlds + halo_num_cfgs(); }

bool glds_is_halo(int cfg) { return cfg >= kNumGlds && cfg < res_base(); }

bool glds_is_resident(int cfg) { return cfg >= res_base(); }

int glds_cfg_bk(int cfg) { return cfg >= kNumGlds ? 64 : kGlds[cfg].bk; }

// Same rules as launch_one / launch_glds (accumulator budget, K-step width, LDS per CU).
bool glds_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs) {
  if (cfg >= res_base()) return resident_supported(cfg - res_base(), cin, cout, kh, kw, limbs, wlimbs);
  if (cfg >= kNumGlds) return halo_supported(cfg - kNumGlds, cin, cout, kh, kw, limbs, wlimbs);
  const GldsCfg& c = kGlds[cfg];
  if (cin % 64 != 0 || cout % 16 != 0 || (c.bk == 128 && cin % 128 != 0)) return false;
  if (wlimbs == 3 && limbs != 3) return false;
  const int smin = limbs + wlimbs - 4 > 0 ? limbs + wlimbs - 4 : 0;
  const int accs = (limbs + wlimbs - 1 - smin) * c.wc * c.wp * 4;
  if (accs > 128 || (accs == 128 && limbs > 1)) return false;  // (128 at 2 activation limbs spills)
  const int bc = 16 * c.wc * c.wavesc, bp = 16 * c.wp * c.wavesp;
  const int stage = (wlimbs * bc + limbs * bp) * c.bk;
  const int nsteps = kh * kw * cin / c.bk;
  int lds = (nsteps < c.stages ? nsteps : c.stages) * stage;
  if (c.wc % 4 == 0) {  // worst case: staged output tile + residual tile (static-range epilogue)
    const int tile = limbs * bp * bc;
    lds = (lds > tile ? lds : tile) + tile;
  }
  return lds <= 160 * 1024;
}

static bool glds_planes_ok(const ConvArgs& a, int limbs, int wlimbs) {
  const long long lim = 0x7fffff00LL;  // operand and output planes use 32-bit buffer offsets
  return (long long)limbs * a.plane <= lim && (long long)wlimbs * a.wplane <= lim &&
         (long long)limbs * a.M * a.cout <= lim && !((a.residual || a.y) && 4LL * a.M * a.cout > lim);
}

// Built-in tile when the caller passes -1 (the Python layer autotunes per shape instead): a
// general 128 x 64 tile (64 x 64 for cout <= 64), else the first configuration that takes the
// shape; -1 when no LDS-DMA configuration does.
int glds_default_cfg(const ConvArgs& a, int limbs, int wlimbs) {
  if (a.s2d || a.cin % kKStep != 0 || a.cout % 16 != 0 || !glds_planes_ok(a, limbs, wlimbs)) return -1;
  const int first = a.cout <= 64 ? 3 : 2;
  if (glds_supported(first, a.cin, a.cout, a.kh, a.kw, limbs, wlimbs)) return first;
  for (int c = 0; c < kNumGlds; ++c)  // (never a halo tile: those need the lean epilogue)
    if (glds_supported(c, a.cin, a.cout, a.kh, a.kw, limbs, wlimbs)) return c;
  return -1;
}

void glds_cfg_info(int cfg, int* bm, int* bn, int* threads) {
  if (cfg >= res_base()) return resident_cfg_info(cfg - res_base(), bm, bn, threads);
  if (cfg >= kNumGlds) return halo_cfg_info(cfg - kNumGlds, bm, bn, threads);
  const GldsCfg& c = kGlds[cfg];
  *bm = 16 * c.wp * c.wavesp;  // pixels (GEMM rows)
  *bn = 16 * c.wc * c.wavesc;  // channels
  *threads = 64 * c.wavesc * c.wavesp;
}

// The stem (cout 64): tiles of 64 output channels only, fixed-point weights (LW = max(2, L)).
template <int L, int LW>
static int launch_s2d(int cfg, const ConvArgs& a, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_one<L, LW, 2, 2, 2, 2, true>(a, s);
    case 1: return launch_one<L, LW, 2, 2, 2, 4, true>(a, s);
    case 3: return launch_one<L, LW, 1, 4, 4, 1, true>(a, s);
    case 4: return launch_one<L, LW, 1, 4, 4, 2, true>(a, s);
    default: return fail(SMPQ_E_INVALID, "smpq_stem_conv_s2d_q: tile config not built for the stem");
  }
}

int launch_glds(int cfg, int limbs, int wlimbs, const ConvArgs& a, hipStream_t s) {
  // operand and output planes are addressed with 32-bit buffer offsets below kOOB
  if ((!a.s2d && a.cin % kKStep != 0) || a.cout % 16 != 0 || !glds_planes_ok(a, limbs, wlimbs))
    return fail(SMPQ_E_INVALID,
                "smpq_conv2d_fwd: LDS-DMA tile configs need cin % 64 == 0, cout % 16 == 0 and planes < 2 GiB");
  if (cfg >= res_base()) return launch_resident(cfg - res_base(), limbs, wlimbs, a, s);
  if (cfg >= kNumGlds) return launch_halo(cfg - kNumGlds, limbs, wlimbs, a, s);
  if (a.s2d) {
    if (wlimbs == 2 && limbs == 1) return launch_s2d<1, 2>(cfg, a, s);
    if (wlimbs == 2 && limbs == 2) return launch_s2d<2, 2>(cfg, a, s);
    if (wlimbs == 3 && limbs == 3) return launch_s2d<3, 3>(cfg, a, s);
    return fail(SMPQ_E_INVALID, "smpq_stem_conv_s2d_q: weight limbs must be max(2, limbs)");
  }
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
