// Batched transpose of 64×64 tiles (bf16 or fp8 bytes): refreshes the transposed working copies Wᵀ of
// the encoder projection weights after every optimizer step, so that every dgrad (dy·W) runs as an NT GEMM on
// K-contiguous operands.  One launch covers all weights (a host-built tile table); each 256-thread
// block moves one tile through LDS with 16-B global loads and stores.
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

// 16 elements per thread in and out: 64 rows × 4 threads × 16 = one 64×64 tile per 256-thread block.
// T = uint16_t (bf16 Wᵀ) or uint8_t (the fp8 e4m3 Wᵀ of the --precision fp8 dgrad GEMMs: the bytes of
// the already-quantised forward copy, so both copies share one dequant scale).
template <typename T>
__global__ __launch_bounds__(256) void transpose_tiles_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                              const int* __restrict__ tiles) {
  constexpr int PAD = 16 / sizeof(T);
  __shared__ T t[64][64 + PAD];
  const int* e = tiles + blockIdx.x * 6;
  const int src_off = e[0], dst_off = e[1], rows = e[2], cols = e[3], r0 = e[4], c0 = e[5];
  const int r = threadIdx.x >> 2, seg = (threadIdx.x & 3) * 16;
  typedef __attribute__((ext_vector_type(16 * sizeof(T) / 4))) uint32_t vec;
  union U { vec v; T x[16]; };
  U in;
  in.v = *reinterpret_cast<const vec*>(src + src_off + (size_t)(r0 + r) * cols + c0 + seg);
#pragma unroll
  for (int i = 0; i < 16; ++i) t[r][seg + i] = in.x[i];
  __syncthreads();
  // dst row = source column c0 + r, dst columns = source rows r0 + seg .. r0 + seg + 15
  U out;
#pragma unroll
  for (int i = 0; i < 16; ++i) out.x[i] = t[seg + i][r];
  *reinterpret_cast<vec*>(dst + dst_off + (size_t)(c0 + r) * rows + r0 + seg) = out.v;
}

}  // namespace

void hq_transpose_tiles(const uint16_t* src, uint16_t* dst, const int* tiles, int ntiles, hipStream_t s) {
  if (ntiles > 0) hipLaunchKernelGGL(transpose_tiles_kernel<uint16_t>, dim3(ntiles), dim3(256), 0, s, src, dst, tiles);
}

void hq_transpose_tiles8(const uint8_t* src, uint8_t* dst, const int* tiles, int ntiles, hipStream_t s) {
  if (ntiles > 0) hipLaunchKernelGGL(transpose_tiles_kernel<uint8_t>, dim3(ntiles), dim3(256), 0, s, src, dst, tiles);
}
