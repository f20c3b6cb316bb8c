// Diagnostic only (tools/timeline_probe.py; never part of libsmpq): a one-lane kernel that stores
// the 100 MHz constant clock (s_memrealtime) into buf[idx] with a VECTOR store. Launched on the
// current stream around every conv of a forward (also inside a captured graph, where each stamp
// becomes a node of the chain), it gives the replayed graph's per-kernel timeline without a profiler.
#include <hip/hip_runtime.h>

__global__ void stamp_kernel(unsigned long long* buf, int idx) {
  if (threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    unsigned long long* p = buf + idx;
    asm volatile("global_store_dwordx2 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(t) : "memory");
  }
}

extern "C" int stamp_launch(void* buf, int idx, void* stream) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)buf, idx);
  return (int)hipGetLastError();
}
