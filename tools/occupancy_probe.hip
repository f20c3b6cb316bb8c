// Occupancy of an LDS-DMA conv block as a function of its dynamic LDS: what the runtime reports
// (hipOccupancyMaxActiveBlocksPerMultiprocessor) and what the hardware does (blocks seen resident
// on one CU at once, from HW_ID + s_memtime stamps of a grid of 8 x 256 long-running blocks).
//   hipcc --offload-arch=gfx950 -O3 tools/occupancy_probe.hip -o tools/bin/occupancy_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256, 2) void k_hold(unsigned long long* t0, unsigned long long* t1, unsigned* cu,
                                                 int spin) {
  extern __shared__ int lds[];
  lds[threadIdx.x] = threadIdx.x;
  const unsigned long long s = __builtin_amdgcn_s_memtime();
  unsigned long long now = s;
  while (now - s < (unsigned long long)spin) now = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    // CU id within the XCD: HW_ID[11:8] = CU, [13:12] = SH, [15:14] = SE
    t0[blockIdx.x] = s;
    t1[blockIdx.x] = now;
    cu[blockIdx.x] = ((xcc & 0xf) << 16) | ((id >> 8) & 0xff);
  }
  if (lds[(threadIdx.x + 1) & 255] == -1) t0[0] = 0;
}

int main() {
  const int nb = 256 * 8;
  unsigned long long *t0, *t1;
  unsigned* cu;
  if (hipMalloc(&t0, nb * 8) || hipMalloc(&t1, nb * 8) || hipMalloc(&cu, nb * 4)) return 1;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_hold), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  printf("{\"probe\": \"blocks of 256 threads resident per CU vs dynamic LDS\", \"rows\": [");
  bool first = true;
  for (int lds : {40960, 65536, 73728, 77824, 79872, 80896, 81408, 81920}) {
    int occ = -1;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_hold, 256, lds);
    hipLaunchKernelGGL(k_hold, dim3(nb), dim3(256), lds, 0, t0, t1, cu, 200000);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<unsigned long long> a(nb), b(nb);
    std::vector<unsigned> c(nb);
    (void)hipMemcpy(a.data(), t0, nb * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(b.data(), t1, nb * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(c.data(), cu, nb * 4, hipMemcpyDeviceToHost);
    // max number of blocks of one CU whose [t0, t1] intervals overlap a common instant
    int best = 0;
    for (int i = 0; i < nb; ++i) {
      int n = 0;
      for (int j = 0; j < nb; ++j)
        if (c[j] == c[i] && a[j] <= a[i] && b[j] > a[i]) ++n;
      best = std::max(best, n);
    }
    printf("%s{\"lds\": %d, \"api_blocks_per_cu\": %d, \"seen_blocks_per_cu\": %d}", first ? "" : ", ", lds, occ, best);
    first = false;
  }
  printf("]}\n");
  return 0;
}
