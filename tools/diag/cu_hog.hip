// Diagnostic kernel, not part of any training step (kept out of the production _hq_kernels library): the
// CU-occupying spin kernel of the GEMM tile-schedule contention test (tests/test_gemm_sched_gpu.py,
// tools/gemm_contention_bench.py).  Built into tools/diag/_hq_diag.so by csrc/build.py build_diag(), loaded
// with ctypes (tools/diag/__init__.py).
#include <hip/hip_runtime.h>

namespace {

// 96 KiB of LDS keeps it alone on its CU, as a GEMM workgroup would need that CU's whole LDS;
// s_memrealtime is the 100 MHz constant clock.
__global__ __launch_bounds__(256) void cu_hog_kernel(long ticks) {
  extern __shared__ char hog_lds[];
  const long t0 = (long)__builtin_amdgcn_s_memrealtime();
  while ((long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 1023) hog_lds[0] = 0;   // never true: keeps the LDS allocation
}

}  // namespace

extern "C" int hq_cu_hog(int blocks, int usec, void* stream) {
  constexpr int lds = 96 * 1024;
  static bool init = [] {
    (void)hipFuncSetAttribute((const void*)cu_hog_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    return true;
  }();
  (void)init;
  hipLaunchKernelGGL(cu_hog_kernel, dim3(blocks), dim3(256), lds, static_cast<hipStream_t>(stream), (long)usec * 100);
  return (int)hipGetLastError();
}
