// One (activation limbs, weight limbs) family of the LDS-DMA conv kernel: every tile configuration
// of launch_cfg<SMPQ_INST_L, SMPQ_INST_LW>. __graft_entry__.build() compiles this file once per
// family (-DSMPQ_INST_L=.. -DSMPQ_INST_LW=..), in parallel.
#include "conv_glds_kernel.h"

namespace smpq {
template int launch_cfg<SMPQ_INST_L, SMPQ_INST_LW>(int, const ConvArgs&, hipStream_t);
}  // namespace smpq
