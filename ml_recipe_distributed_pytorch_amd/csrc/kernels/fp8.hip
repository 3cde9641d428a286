// OCP fp8 (e4m3fn) quantisation passes for --precision fp8 (the standalone form: the training step's fp8
// inputs are written by their producers under delayed scaling; the GEMMs are gemm_fp8.hip's own block-scaled
// MFMA kernels).  Current (just-in-time) per-tensor scaling, with no host synchronisation:
//   hq_amax_bf16 : amax = max |x|                          (grid-wide max via float-as-uint atomics)
//   hq_fp8_quant : y = sat(x · 448 / amax) → e4m3fn,  scale = amax / 448 (the dequant factor the fp8 GEMM
//                  multiplies back in), both read from / written to device memory.
// v_cvt_pk_fp8_f32 converts two f32 to OCP e4m3 on gfx950; inputs are clamped to ±448 first so an
// out-of-range value saturates instead of becoming NaN (e4m3fn has no infinity).
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr float kFp8Max = 448.f;

__global__ __launch_bounds__(256) void amax_kernel(const uint16_t* __restrict__ x, size_t n8, unsigned* __restrict__ amax) {
  float m = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    float f[8];
    hq_unpack8(reinterpret_cast<const uint4*>(x)[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(f[k]));
  }
  m = hq_wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(amax, __float_as_uint(m));  // non-negative floats order like their bit patterns
  }
}

__global__ __launch_bounds__(256) void fp8_quant_kernel(const uint16_t* __restrict__ x, uint2* __restrict__ y, size_t n8,
                                                        const unsigned* __restrict__ amax, float* __restrict__ scale) {
  const float a = fmaxf(__uint_as_float(*amax), 1e-12f);
  const float inv = kFp8Max / a;
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale = a / kFp8Max;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    float f[8];
    hq_unpack8(reinterpret_cast<const uint4*>(x)[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = fminf(fmaxf(f[k] * inv, -kFp8Max), kFp8Max);
    uint32_t lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
    uint32_t hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
    y[i] = make_uint2(lo, hi);
  }
}

int grid_for(size_t n8) { return (int)std::min<size_t>((n8 + 255) / 256, 256 * 8); }

// bf16 gelu' -> the 8-bit code with the very encoder the fp8 FFN1 epilogue uses (hq_gd_encode8): for a bf16 gelu'
// that must meet the fp8 FFN2 dgrad (ops.gelud_encode)
__global__ __launch_bounds__(256) void gelud_encode8_kernel(const uint4* __restrict__ g, uint2* __restrict__ q, size_t n8) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float f[8];
    hq_unpack8(g[i], f);
    q[i] = hq_gd_encode8(f);
  }
}

}  // namespace

void hq_gelud_encode8(const uint16_t* g, uint8_t* q, size_t n, hipStream_t s) {
  const size_t n8 = n / 8;
  const int grid = std::max(1, (int)std::min<size_t>((n8 + 255) / 256, 4096));
  hipLaunchKernelGGL(gelud_encode8_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint4*>(g),
                     reinterpret_cast<uint2*>(q), n8);
}

void hq_amax_bf16(const uint16_t* x, size_t n, unsigned* amax, hipStream_t s) {
  hq_zero_f32(reinterpret_cast<float*>(amax), 1, s);   // own kernel: no runtime memset node under graph capture
  const size_t n8 = n / 8;
  if (n8) hipLaunchKernelGGL(amax_kernel, dim3(grid_for(n8)), dim3(256), 0, s, x, n8, amax);
}

void hq_fp8_quant(const uint16_t* x, uint8_t* y, size_t n, const unsigned* amax, float* scale, hipStream_t s) {
  const size_t n8 = n / 8;
  hipLaunchKernelGGL(fp8_quant_kernel, dim3(grid_for(n8 ? n8 : 1)), dim3(256), 0, s, x, reinterpret_cast<uint2*>(y), n8,
                     amax, scale);
}
