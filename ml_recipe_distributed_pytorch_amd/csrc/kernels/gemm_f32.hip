// Exact-fp32 GEMM on the gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32) for --precision fp32
// (the reference's apex_level None / O0 mode: fp32 everywhere, /root/reference/modules/model/trainer/trainer.py:23-32,
// 128-133, 200-204).  The bf16 path never runs here; this kernel carries every GEMM-shaped FLOP of the fp32 mode:
// the encoder projections (forward, dgrad, weight gradient) and the attention's batched QKᵀ / PV products and their
// backward.
//
//   C[i, j] = alpha · Σ_k A(i, k) · B(j, k)  (+ bias[j])  (+ R[i, j])
//
// with strided operands A(i, k) = A[i·sa_i + k·sa_k] and B(j, k) = B[j·sb_j + k·sb_k], one of the two strides of each
// operand being 1 (A_K / B_K: the k stride is 1), so every layout the fp32 mode needs is a view, never a copy:
//   forward x·Wᵀ           A_K B_K      dgrad dy·W        A_K !B_K      weight grad dyᵀ·x    !A_K !B_K
// and the attention products through a two-level batch index z = outer·nb_in + inner (strides per operand).
//
// * 128 × 128 block tile, BK = 16, 256 threads = 4 waves as 2 × 2, each wave 64 × 64 = 2 × 2 MFMA 32×32 tiles
//   (64 accumulator VGPRs).  The MFMA operands are one f32 VGPR per lane: lane l reads A[i = l & 31][k = l >> 5]
//   and B[k = l >> 5][j = l & 31] — LDS holds both tiles k-major ([BK][128]), so the 32 lanes of a half-wave
//   read 32 consecutive words (conflict-free ds_read_b32).
// * Global → LDS by register staging (the k-contiguous operand is transposed in the write), double-buffered:
//   tile t+1's loads are issued before tile t's MFMAs, written to the other LDS buffer after them.
// * Numerics: each MFMA is a k-ordered f32 fma chain (exact f32 products, one rounding each, CDNA4 guide §3),
//   so the result matches an fp32 reference to ~1e-7·Σ|a·b|.
// * Split-K (ksplit > 1, unbatched): split s sums k-tiles [s·nk/ksplit, (s+1)·nk/ksplit) into fp32 slab ws[s];
//   gemm_f32_reduce_kernel folds the slabs in order (deterministic) and applies the epilogue.
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int TB = 128;      // block tile (rows = cols)
constexpr int BKF = 16;      // k per LDS stage
constexpr int LDS_ROW = TB;  // floats per k-row of a staged tile

struct F32Args {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  const float* R;
  float* ws;
  int M, N, K, ldc, ldr, nb_in, ksplit;
  long long sa_i, sa_k, sb_j, sb_k;
  long long ba_out, ba_in, bb_out, bb_in, bc_out, bc_in;
  float alpha;
};

// the [BKF][TB] k-major stage of one operand: rows r0.. of the operand (i or j), k-tile starting at k0
template <bool KC>
__device__ __forceinline__ void load_stage(const float* __restrict__ X, long long s_r, long long s_k, int rows, int K,
                                           int r0, int k0, int tid, float4 (&reg)[2]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (KC) {                    // k contiguous: a float4 = 4 k of one row
      const int r = tid & 127, kq = (tid >> 7) + 2 * q;
      const int gr = r0 + r, gk = k0 + kq * 4;
      if (gr < rows && gk < K) v = *reinterpret_cast<const float4*>(X + gr * s_r + gk);
    } else {                               // row contiguous: a float4 = 4 rows of one k
      const int rq = tid & 31, kk = (tid >> 5) + 8 * q;
      const int gr = r0 + rq * 4, gk = k0 + kk;
      if (gr < rows && gk < K) v = *reinterpret_cast<const float4*>(X + gr + gk * s_k);
    }
    reg[q] = v;
  }
}

template <bool KC>
__device__ __forceinline__ void store_stage(float* __restrict__ lds, int tid, const float4 (&reg)[2]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if constexpr (KC) {
      const int r = tid & 127, kq = (tid >> 7) + 2 * q;
      lds[(kq * 4 + 0) * LDS_ROW + r] = reg[q].x;
      lds[(kq * 4 + 1) * LDS_ROW + r] = reg[q].y;
      lds[(kq * 4 + 2) * LDS_ROW + r] = reg[q].z;
      lds[(kq * 4 + 3) * LDS_ROW + r] = reg[q].w;
    } else {
      const int rq = tid & 31, kk = (tid >> 5) + 8 * q;
      *reinterpret_cast<float4*>(lds + kk * LDS_ROW + rq * 4) = reg[q];
    }
  }
}

template <bool A_K, bool B_K>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(F32Args a) {
  __shared__ __attribute__((aligned(16))) float smem[2][2][BKF * LDS_ROW];   // [buf][A|B][k][row]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (a.N + TB - 1) / TB;
  const int tile = blockIdx.x;
  const int m0 = (tile / tiles_n) * TB, n0 = (tile % tiles_n) * TB;
  const int split = blockIdx.y;
  const int z = blockIdx.z, zo = z / a.nb_in, zi = z - zo * a.nb_in;
  const float* A = a.A + zo * a.ba_out + zi * a.ba_in;
  const float* B = a.B + zo * a.bb_out + zi * a.bb_in;
  const int nk = (a.K + BKF - 1) / BKF;
  const int kt0 = split * nk / a.ksplit, kt1 = (split + 1) * nk / a.ksplit;

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float4 ra[2], rb[2];
  if (kt0 < kt1) {
    load_stage<A_K>(A, a.sa_i, a.sa_k, a.M, a.K, m0, kt0 * BKF, tid, ra);
    load_stage<B_K>(B, a.sb_j, a.sb_k, a.N, a.K, n0, kt0 * BKF, tid, rb);
    store_stage<A_K>(smem[0][0], tid, ra);
    store_stage<B_K>(smem[0][1], tid, rb);
  }
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      load_stage<A_K>(A, a.sa_i, a.sa_k, a.M, a.K, m0, (kt + 1) * BKF, tid, ra);
      load_stage<B_K>(B, a.sb_j, a.sb_k, a.N, a.K, n0, (kt + 1) * BKF, tid, rb);
    }
    const float* As = smem[buf][0];
    const float* Bs = smem[buf][1];
#pragma unroll
    for (int ks = 0; ks < BKF; ks += 2) {
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = As[(ks + lk) * LDS_ROW + wm * 64 + i * 32 + li];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[(ks + lk) * LDS_ROW + wn * 64 + j * 32 + li];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_stage<A_K>(smem[buf ^ 1][0], tid, ra);
      store_stage<B_K>(smem[buf ^ 1][1], tid, rb);
    }
    __syncthreads();
  }

  // C/D map of the 32×32 MFMA: col = lane & 31, row = (r & 3) + 8·(r >> 2) + 4·(lane >> 5)
  const int col_l = lane & 31, row_h = 4 * (lane >> 5);
  HQ_DASSERT(split < a.ksplit && m0 < a.M && n0 < a.N);
  if (a.ksplit > 1) {
    HQ_DASSERT(a.ws != nullptr);
    float* slab = a.ws + (long long)split * a.M * a.N;   // slab `split` of the [ksplit][M][N] workspace
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int gj = n0 + wn * 64 + j * 32 + col_l;
        if (gj >= a.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int gi = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + row_h;
          if (gi < a.M) {
            HQ_DASSERT(gj < a.N);
            slab[(long long)gi * a.N + gj] = acc[i][j][r];
          }
        }
      }
    return;
  }
  float* C = a.C + zo * a.bc_out + zi * a.bc_in;
  const float* R = a.R ? a.R + zo * a.bc_out + zi * a.bc_in : nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gj = n0 + wn * 64 + j * 32 + col_l;
      if (gj >= a.N) continue;
      const float bj = a.bias ? a.bias[gj] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gi = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + row_h;
        if (gi >= a.M) continue;
        float v = a.alpha * acc[i][j][r] + bj;
        HQ_DASSERT(gj < a.N && gj < a.ldc && (R == nullptr || gj < a.ldr));
        if (R) v += R[(long long)gi * a.ldr + gj];
        C[(long long)gi * a.ldc + gj] = v;
      }
    }
}

__global__ __launch_bounds__(256) void gemm_f32_reduce_kernel(const float* __restrict__ ws, int ksplit, float* __restrict__ C,
                                                              const float* __restrict__ bias, const float* __restrict__ R,
                                                              int M, int N, int ldc, int ldr, float alpha) {
  const long long n = (long long)M * N;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < ksplit; ++k) s += ws[k * n + e];   // slab order: deterministic
    const int i = (int)(e / N), j = (int)(e - (long long)i * N);
    float v = alpha * s + (bias ? bias[j] : 0.f);
    if (R) v += R[(long long)i * ldr + j];
    C[(long long)i * ldc + j] = v;
  }
}

}  // namespace

int hq_gemm_f32_splits(int M, int N, int K, int batch) {
  // enough workgroups to fill 256 CUs at 2 per CU when the output alone cannot (the weight gradients:
  // dW[768, 768] is 36 tiles over K = 98304 tokens); each split keeps >= 64 k-tiles
  const int tiles = ((M + TB - 1) / TB) * ((N + TB - 1) / TB) * batch;
  if (batch > 1 || tiles >= 256) return 1;
  const int nk = (K + BKF - 1) / BKF;
  int s = (512 + tiles - 1) / tiles;
  s = std::min(s, std::max(1, nk / 64));
  return std::max(1, std::min(s, 64));
}

void hq_gemm_f32(const float* A, const float* B, float* C, const float* bias, const float* R, float* ws, int M, int N,
                 int K, long long sa_i, long long sa_k, long long sb_j, long long sb_k, int ldc, int ldr, int batch,
                 int nb_in, long long ba_out, long long ba_in, long long bb_out, long long bb_in, long long bc_out,
                 long long bc_in, float alpha, int ksplit, hipStream_t s) {
  F32Args a{A, B, C, bias, R, ws, M, N, K, ldc, ldr, nb_in, ksplit, sa_i, sa_k, sb_j, sb_k,
            ba_out, ba_in, bb_out, bb_in, bc_out, bc_in, alpha};
  const int tiles = ((M + TB - 1) / TB) * ((N + TB - 1) / TB);
  dim3 grid(tiles, ksplit, batch);
  const bool ak = sa_k == 1, bk = sb_k == 1;
  if (ak && bk) gemm_f32_kernel<true, true><<<grid, 256, 0, s>>>(a);
  else if (ak) gemm_f32_kernel<true, false><<<grid, 256, 0, s>>>(a);
  else if (bk) gemm_f32_kernel<false, true><<<grid, 256, 0, s>>>(a);
  else gemm_f32_kernel<false, false><<<grid, 256, 0, s>>>(a);
  if (ksplit > 1) {
    const long long n = (long long)M * N;
    const int blocks = (int)std::min<long long>((n + 255) / 256, 2048);
    gemm_f32_reduce_kernel<<<blocks, 256, 0, s>>>(ws, ksplit, C, bias, R, M, N, ldc, ldr, alpha);
  }
}
