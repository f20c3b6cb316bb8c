// Does the limb-plane layout cost HBM bandwidth? A copy-like kernel with the traffic mix of the
// 1x1 64->256 residual expansion at 56^2 (B=256, L=3): per output pixel it reads 64 input bytes x
// 3 limbs + 256 residual bytes x 3 limbs and writes 256 bytes x 3 limbs, either from / to three
// separate limb planes per tensor ([L][pixels][C], the library's layout: 9 concurrent streams) or
// from / to limb-interleaved rows ([pixels][L][C]: 3 streams). 16-B accesses, grid-stride, no
// compute (bytes are xor-folded so the loads are live). Diagnostics only.
//
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_bench.hip -o tools/bin/stream_bench
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

// one thread = 16 output bytes of one limb of one pixel row chunk; PLANAR: limb l of element e at
// l * plane + e, else at (e / C) * 3C + l * C + e % C
template <bool PLANAR>
__global__ __launch_bounds__(256) void mix_kernel(const v4i* __restrict__ x, const v4i* __restrict__ r,
                                                  v4i* __restrict__ y, long long pix, int cin, int cout) {
  const long long cvec = cout / 16, xvec = cin / 16;   // 16-B vectors per pixel row
  const long long total = pix * cvec;                  // output vectors per limb
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < total;
       v += (long long)gridDim.x * blockDim.x) {
    const long long p = v / cvec, q = v - p * cvec;
#pragma unroll
    for (int l = 0; l < 3; ++l) {
      const long long yo = PLANAR ? l * total + v : p * 3 * cvec + l * cvec + q;
      v4i a = r[yo];
      if (q < xvec) {  // the input row (64 B at cin 64) read by the first lanes of the pixel
        const long long xo = PLANAR ? l * pix * xvec + p * xvec + q : p * 3 * xvec + l * xvec + q;
        a ^= x[xo];
      }
      y[yo] = a;
    }
  }
}

int main() {
  const long long pix = 256LL * 56 * 56;
  const int cin = 64, cout = 256;
  const size_t xb = 3 * pix * cin, rb = 3 * pix * cout;
  v4i *x, *r, *y;
  CK(hipMalloc(&x, xb));
  CK(hipMalloc(&r, rb));
  CK(hipMalloc(&y, rb));
  CK(hipMemset(x, 1, xb));
  CK(hipMemset(r, 2, rb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)xb + 2.0 * rb;
  for (int planar = 1; planar >= 0; --planar) {
    for (int grid : {1024, 2048, 4096, 8192}) {
      auto k = planar ? mix_kernel<true> : mix_kernel<false>;
      for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, x, r, y, pix, cin, cout);
      CK(hipEventRecord(e0));
      for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, x, r, y, pix, cin, cout);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 10;
      printf("{\"layout\": \"%s\", \"grid\": %d, \"us\": %.1f, \"TB_s\": %.2f}\n", planar ? "limb planes" : "limb-interleaved",
             grid, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
