// Batched bf16 transpose of 64×64 tiles: refreshes the transposed working copies Wᵀ of the encoder
// projection weights after every optimizer step, so that every dgrad (dy·W) runs as an NT GEMM on
// K-contiguous operands.  One launch covers all weights (a host-built tile table); each 256-thread
// block moves one tile through LDS with 16-B global loads and stores.
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

__global__ __launch_bounds__(256) void transpose_tiles_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                              const int* __restrict__ tiles) {
  __shared__ uint16_t t[64][72];
  const int* e = tiles + blockIdx.x * 6;
  const int src_off = e[0], dst_off = e[1], rows = e[2], cols = e[3], r0 = e[4], c0 = e[5];
  const int r = threadIdx.x >> 2, seg = (threadIdx.x & 3) * 16;
  const uint16_t* s = src + src_off + (size_t)(r0 + r) * cols + c0 + seg;
  const uint4 a = *reinterpret_cast<const uint4*>(s);
  const uint4 b = *reinterpret_cast<const uint4*>(s + 8);
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    t[r][seg + 2 * i] = (uint16_t)(w[i] & 0xFFFFu);
    t[r][seg + 2 * i + 1] = (uint16_t)(w[i] >> 16);
  }
  __syncthreads();
  // dst row = source column c0 + r, dst columns = source rows r0 + seg .. r0 + seg + 15
  uint32_t o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (uint32_t)t[seg + 2 * i][r] | ((uint32_t)t[seg + 2 * i + 1][r] << 16);
  uint16_t* d = dst + dst_off + (size_t)(c0 + r) * rows + r0 + seg;
  *reinterpret_cast<uint4*>(d) = make_uint4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<uint4*>(d + 8) = make_uint4(o[4], o[5], o[6], o[7]);
}

}  // namespace

void hq_transpose_tiles(const uint16_t* src, uint16_t* dst, const int* tiles, int ntiles, hipStream_t s) {
  if (ntiles > 0) hipLaunchKernelGGL(transpose_tiles_kernel, dim3(ntiles), dim3(256), 0, s, src, dst, tiles);
}
