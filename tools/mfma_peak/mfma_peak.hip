// MFMA throughput ceiling on this part: back-to-back independent bf16 MFMAs, no memory traffic, no
// barriers.  Tells apart "the GEMM pipeline leaves MFMA cycles idle" from "the matrix cores run at a
// lower clock under sustained load" when reading the GEMM kernels' PF/s.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_peak tools/mfma_peak/mfma_peak.hip && /tmp/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int SHAPE>
__global__ __launch_bounds__(256) void peak(float* out, int iters) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 1e-3f + i); b[i] = (__bf16)(i * 1e-3f); }
  if constexpr (SHAPE == 16) {
    // eight named accumulators (an array let hipcc rotate overlapping AGPR ranges between iterations,
    // chaining the MFMAs)
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
    for (int it = 0; it < iters; ++it) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c3, 0, 0, 0);
      c4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c4, 0, 0, 0);
      c5 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c5, 0, 0, 0);
      c6 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c6, 0, 0, 0);
      c7 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c7, 0, 0, 0);
    }
    const f32x4 t = ((c0 + c1) + (c2 + c3)) + ((c4 + c5) + (c6 + c7));
    const float s = t[0] + t[1] + t[2] + t[3];
    if (s == 1.2345f) out[threadIdx.x] = s;
  } else if constexpr (SHAPE == 17) {
    // 16x16x32 through inline asm: eight independent accumulators hipcc cannot rotate (the builtin form above
    // compiles to accvgpr moves between the MFMAs)
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
    for (int it = 0; it < iters; ++it) {
      asm volatile(
          "v_mfma_f32_16x16x32_bf16 %0, %8, %9, %0\n\t"
          "v_mfma_f32_16x16x32_bf16 %1, %8, %9, %1\n\t"
          "v_mfma_f32_16x16x32_bf16 %2, %8, %9, %2\n\t"
          "v_mfma_f32_16x16x32_bf16 %3, %8, %9, %3\n\t"
          "v_mfma_f32_16x16x32_bf16 %4, %8, %9, %4\n\t"
          "v_mfma_f32_16x16x32_bf16 %5, %8, %9, %5\n\t"
          "v_mfma_f32_16x16x32_bf16 %6, %8, %9, %6\n\t"
          "v_mfma_f32_16x16x32_bf16 %7, %8, %9, %7"
          : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
          : "v"(a), "v"(b));
    }
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    const f32x4 t = ((c0 + c1) + (c2 + c3)) + ((c4 + c5) + (c6 + c7));
    const float s = t[0] + t[1] + t[2] + t[3];
    if (s == 1.2345f) out[threadIdx.x] = s;
  } else {
    f32x16 c[4];
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 16; ++r) c[j][r] = 0.f;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[j], 0, 0, 0);
    float s = 0.f;
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 16; ++r) s += c[j][r];
    if (s == 1.2345f) out[threadIdx.x] = s;
  }
}

template <int SHAPE>
void run(int waves_per_simd) {
  float* out;
  (void)hipMalloc(&out, 4096);
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = ncu * waves_per_simd;   // 4 waves per block = one per SIMD
  const int iters = 20000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(peak<SHAPE>, dim3(blocks), dim3(256), 0, 0, out, 100);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(peak<SHAPE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double per = SHAPE != 32 ? 16.0 * 16 * 32 * 2 * 8 : 32.0 * 32 * 16 * 2 * 4;   // flop per wave-iteration
  const double flop = per * iters * blocks * 4;
  printf("mfma %s  waves/SIMD %d  %.3f ms  %.0f TFLOP/s\n", SHAPE == 16 ? "16x16x32" : SHAPE == 17 ? "16x16x32 asm" : "32x32x16", waves_per_simd, ms, flop / ms / 1e9);
  (void)hipFree(out);
}

int main() {
  for (int w : {1, 2, 4}) run<16>(w);
  for (int w : {1, 2, 4}) run<17>(w);
  for (int w : {1, 2, 4}) run<32>(w);
  return 0;
}
