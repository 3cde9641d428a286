// bf16 "NT" GEMM, two workgroups per CU:  C[M,N] = A[M,K] · B[N,K]ᵀ (+ fused epilogue)
//
// Why a second design next to gemm.hip's 8-wave 256² kernels: those run ONE workgroup per CU, so every
// tile's epilogue — bias/GELU/GELU' math on the VALU, the aux-operand loads and 128 KB of stores — runs
// while the CU's matrix cores sit idle (FFN1 + GELU' at 0.77 PF/s, profiles/r2_gemm_epilogue).  Here a
// workgroup is 4 waves with a BM × BN tile (2 × 2 waves, each (BM/2) × (BN/2)) and ≤ 80 KB of LDS, so two
// of them share each CU (one wave of each per SIMD, ≤ 256 VGPRs each): while one runs its epilogue the
// other's MFMAs keep the SIMD's matrix pipe busy, and their K-loop barriers interleave the same way.
//
// * BK = 32 per stage: one 64-B LDS row per operand row; a 3-deep ring (issue stage t+2 right after the
//   barrier that retires stage t), ONE barrier per stage, counted vmcnt (never 0 in the loop), raw
//   s_barrier (a __syncthreads fence would drain the LDS-DMA in flight), one __shared__ array.
// * Operands reach LDS by buffer_load … lds (16 B per lane, wave-uniform LDS base + 16·lane): the bank
//   swizzle chunk' = chunk ^ g(row) is applied to the per-lane SOURCE address and undone on the
//   ds_read_b128 fragment read (playbook rule 21).  g(row) = (row>>2)&3 for v_mfma_f32_32x32x16_bf16
//   (lane l reads row l&31, chunk l>>5), (-(row>>2))&3 for v_mfma_f32_16x16x32_bf16 (row l&15, chunk
//   l>>4): with 64-B rows both spread each 16-lane ds_read_b128 group over all 16 slots of the bank row.
// * Swapped operands (the weight fragment is the MFMA's A input), so the accumulator is Cᵀ: a lane owns
//   one output row and 4 consecutive output columns per register group.
// * Epilogue: acc (+ bias) → bf16 tile in LDS (the ring's bytes, 8-B writes, conflict-free row stride
//   2·BN + 8), barrier, then 64-column slabs read back as 16-B row pieces (8 lanes per row → 128-B
//   segments per row), the elementwise epilogue, 16-B global stores; DMUL/DGELU column sums reduce over
//   the slab's rows in registers, across waves through LDS, into part[M/BM][N].
// * M tail: the A descriptor's num_records ends at row M, so rows past it stage as zeros and are never
//   stored.  N % BN == 0 and K % 32 == 0 are the host's contract.
// * BM = BN = 192 tiles the BERT-base shapes at M = 98 304 tokens (512 × {4, 12, 16} tiles for N = 768,
//   2304, 3072) into whole rounds of the 512 workgroup slots: no half-empty last wave.
// * XCD-aware bijective block remap; tiles walk M-major within an XCD (A row panel + all of B in its L2).
#include <algorithm>
#include <mutex>

#include "hq_common.h"
#include "hq_kernels.h"

namespace {
namespace hq_nt4 {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int kThreads = 256;
constexpr int BK = 32;
constexpr int NST = 3;

template <int MF>
__device__ __forceinline__ int swz(int row) {
  if constexpr (MF == 32) return (row >> 2) & 3;
  else return (-(row >> 2)) & 3;
}

template <int BM, int BN, int MF>
struct Geo {
  static constexpr int WM = BM / 2, WN = BN / 2;             // wave tile
  static constexpr int FM = WM / MF, FN = WN / MF;           // fragments per wave along m / n
  static constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int RING = NST * STAGE;
  static constexpr int RS = BN * 2 + 8;                      // epilogue staging row stride (bytes)
  static constexpr int TILE = BM * RS;
  static constexpr int SCR = 4 * 64 * 4;                     // column-sum scratch [4 waves][64] f32
  static constexpr int LDS = RING > TILE + SCR ? RING : TILE + SCR;
  static constexpr int A_IPW = BM / 64;                      // LDS-DMA instructions per wave per stage
  static constexpr int B_IPW = BN / 64;                      // (one instruction = 16 rows of 64 B)
  static constexpr int LOADS = A_IPW + B_IPW;
  static_assert(WM % MF == 0 && WN % MF == 0 && BM % 64 == 0 && BN % 64 == 0, "tile");
  static_assert(LDS <= 80 * 1024, "two workgroups per CU");
};

template <int MF> struct AccT;
template <> struct AccT<32> { typedef f32x16_t type; };
template <> struct AccT<16> { typedef f32x4_t type; };

// one MFMA of the chosen shape (a template, not an overload set: an overloaded __device__ call inside the
// kernel's lambdas fails overload resolution in hipcc's host pass and silently drops the launch stub)
template <int MF, typename T>
__device__ __forceinline__ T mfma(const bf16x8_t& a, const bf16x8_t& b, const T& c) {
  if constexpr (MF == 32) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int EPI, int BM, int BN, int MF>
__global__ __launch_bounds__(kThreads, 2) void gemm_nt4_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                               uint16_t* __restrict__ C, const float* __restrict__ bias,
                                                               uint16_t* __restrict__ P, const uint16_t* __restrict__ R,
                                                               float* __restrict__ part, int M, int N, int K, int lda,
                                                               int ldb, int ldc, HqDropArg dr, int stagger) {
  using G = Geo<BM, BN, MF>;
  using acc_t = typename AccT<MF>::type;
  constexpr int NACC = MF == 32 ? 16 : 4;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const uint32_t key = EPI == HQ_EPI_BDR ? dr.kd.get() : 0u;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int nwg = gridDim.x, bid = blockIdx.x;
  // experiment: start the second workgroup of each CU (first dispatch round only) `stagger` × 8128 cycles
  // late, so the two co-resident workgroups run their epilogues out of phase
  if (stagger > 0 && bid >= 256 && bid < 512)
    for (int i = 0; i < stagger; ++i) __builtin_amdgcn_s_sleep(127);
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_n = N / BN;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int rows_a = min(BM, M - m0);
  const int nt = K / BK;
  HQ_DASSERT(rows_a > 0 && n0 + BN <= N && K % BK == 0);

  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * lda), (short)0, rows_a * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(B + (size_t)n0 * ldb), (short)0, BN * ldb * 2, 0x00020000);
  // wave w stages panel rows w·(BM/4) + 16i + lane/4 (A) and w·(BN/4) + 16i + lane/4 (B); the LDS image is
  // lane-linear (row = 16-row block + lane/4, slot lane&3), the SOURCE chunk is the swizzled one
  // (fixed-size arrays: a template-dependent bound on these makes hipcc's host pass reject the buffer-load
  // builtin's voffset operand and silently drop the kernel's launch stub)
  static_assert(G::A_IPW <= 4 && G::B_IPW <= 4, "voffset arrays");
  int voA[4], voB[4];
#pragma unroll
  for (int i = 0; i < G::A_IPW; ++i) {
    const int row = wave * (BM / 4) + i * 16 + (lane >> 2);
    voA[i] = (row * lda + (((lane & 3) ^ swz<MF>(row)) << 3)) * 2;
  }
#pragma unroll
  for (int i = 0; i < G::B_IPW; ++i) {
    const int row = wave * (BN / 4) + i * 16 + (lane >> 2);
    voB[i] = (row * ldb + (((lane & 3) ^ swz<MF>(row)) << 3)) * 2;
  }
  auto stage = [&](int t, int buf) {
    char* sa = smem + buf * G::STAGE + wave * (BM / 4) * 64;
    char* sb = smem + buf * G::STAGE + G::A_BYTES + wave * (BN / 4) * 64;
    const int ko = t * BK * 2;
#pragma unroll
    for (int i = 0; i < G::A_IPW; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(sa + i * 1024), 16, voA[i], ko, 0, 0);
#pragma unroll
    for (int i = 0; i < G::B_IPW; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(sb + i * 1024), 16, voB[i], ko, 0, 0);
  };

  // fragment read offsets (bytes within a stage's panel); the swizzle term depends on the lane only,
  // because every fragment base row is a multiple of 16 (the swizzle reads row bits 2-3)
  constexpr int KSTEPS = MF == 32 ? 2 : 1;
  const int fr = MF == 32 ? (lane & 31) : (lane & 15);
  int offA[KSTEPS], offB[KSTEPS];
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int ch = MF == 32 ? 2 * ks + (lane >> 5) : (lane >> 4);
    offA[ks] = (wm * G::WM + fr) * 64 + ((ch ^ swz<MF>(fr)) << 4);
    offB[ks] = (wn * G::WN + fr) * 64 + ((ch ^ swz<MF>(fr)) << 4);
  }

  acc_t acc[G::FN][G::FM];
#pragma unroll
  for (int j = 0; j < G::FN; ++j)
#pragma unroll
    for (int i = 0; i < G::FM; ++i)
#pragma unroll
      for (int e = 0; e < NACC; ++e) acc[j][i][e] = 0.f;

  // all of the stage's fragments are read up front (both k-steps of the 32x32x16 form, distinct registers),
  // so the second k-step's LDS latency hides under the first k-step's MFMAs
  auto compute = [&](int buf) {
    const char* pa = smem + buf * G::STAGE;
    const char* pb = pa + G::A_BYTES;
    bf16x8_t fa[KSTEPS][G::FM], fb[KSTEPS][G::FN];
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
#pragma unroll
      for (int j = 0; j < G::FN; ++j) fb[ks][j] = *reinterpret_cast<const bf16x8_t*>(pb + offB[ks] + j * MF * 64);
#pragma unroll
      for (int i = 0; i < G::FM; ++i) fa[ks][i] = *reinterpret_cast<const bf16x8_t*>(pa + offA[ks] + i * MF * 64);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
      for (int j = 0; j < G::FN; ++j)
#pragma unroll
        for (int i = 0; i < G::FM; ++i) acc[j][i] = mfma<MF>(fb[ks][j], fa[ks][i], acc[j][i]);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- K loop: 3-stage ring, one barrier per stage.  At the top of iteration t the wave's outstanding
  // DMA is stage t (older) and stage t+1: vmcnt(LOADS) retires stage t.  The barrier then (RAW) publishes
  // every wave's stage-t bytes and (WAR) proves every wave finished reading stage t-1, whose buffer
  // (t+2) % 3 is refilled right after it.
  stage(0, 0);
  if (nt > 1) stage(1, 1);
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(G::LOADS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (t + 2 < nt) stage(t + 2, (t + 2) % NST);
    compute(t % NST);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();   // every wave is done with the ring: its bytes become the epilogue tile

  // ---- epilogue phase 1: acc (+ bias) → bf16 tile [BM][RS] in LDS
  constexpr bool kBias = EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD || EPI == HQ_EPI_BDR || EPI == 8;
#pragma unroll
  for (int j = 0; j < G::FN; ++j) {
#pragma unroll
    for (int g = 0; g < NACC / 4; ++g) {
      const int nl = MF == 32 ? wn * G::WN + j * 32 + 8 * g + 4 * (lane >> 5) : wn * G::WN + j * 16 + 4 * (lane >> 4);
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (kBias) bv = *reinterpret_cast<const float4*>(bias + n0 + nl);
#pragma unroll
      for (int i = 0; i < G::FM; ++i) {
        const int ml = wm * G::WM + i * MF + fr;
        float v[4] = {acc[j][i][4 * g], acc[j][i][4 * g + 1], acc[j][i][4 * g + 2], acc[j][i][4 * g + 3]};
        if constexpr (kBias) { v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w; }
        *reinterpret_cast<uint2*>(smem + ml * G::RS + nl * 2) = hq_pack4(v);
      }
    }
  }
  __syncthreads();

  // ---- phase 2: 64-column slabs, 8 lanes per row (16 B each), 32 rows per pass
  constexpr bool kAux = EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL || EPI == HQ_EPI_RESID || EPI == HQ_EPI_BDR;
  constexpr bool kColsum = EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL;
  constexpr int PASSES = BM / 32;
  const int ch = tid & 7, rr = tid >> 3;
  float* scr = reinterpret_cast<float*>(smem + G::TILE);
#pragma unroll 1
  for (int s = 0; s < BN / 64; ++s) {
    const int col = s * 64 + ch * 8;
    uint4 aux[kAux ? PASSES : 1];
    if constexpr (kAux) {
      const uint16_t* src = (EPI == HQ_EPI_RESID || EPI == HQ_EPI_BDR) ? R : P;
#pragma unroll
      for (int p = 0; p < PASSES; ++p) {
        const int gm = m0 + p * 32 + rr;
        aux[p] = gm < M ? *reinterpret_cast<const uint4*>(src + (size_t)gm * ldc + n0 + col) : make_uint4(0, 0, 0, 0);
      }
    }
    float csum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
#pragma unroll
    for (int p = 0; p < PASSES; ++p) {
      const int row = p * 32 + rr, gm = m0 + row;
      uint4 piece = *reinterpret_cast<const uint4*>(smem + row * G::RS + col * 2);
      if (gm >= M) continue;
      const size_t goff = (size_t)gm * ldc + n0 + col;
      if constexpr (EPI == HQ_EPI_GELU) {
        *reinterpret_cast<uint4*>(P + goff) = piece;   // pre-activation, kept for the backward
        float x[8];
        hq_unpack8(piece, x);
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = hq_gelu(x[e]);
        piece = hq_pack8(x);
      } else if constexpr (EPI == HQ_EPI_GELUD) {
        float x[8], gr[8];
        hq_unpack8(piece, x);
        hq_gelu_grad8(x, gr);   // gr = gelu'(x), x = gelu(x)
        *reinterpret_cast<uint4*>(P + goff) = hq_pack8(gr);
        piece = hq_pack8(x);
      } else if constexpr (EPI == 8) {   // experiment: GELUD with the 3-term erf
        float x[8], gr[8];
        hq_unpack8(piece, x);
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float xv = x[e]; gr[e] = hq_gelu_grad(xv); x[e] = hq_gelu(xv); }
        *reinterpret_cast<uint4*>(P + goff) = hq_pack8(gr);
        piece = hq_pack8(x);
      } else if constexpr (EPI == HQ_EPI_DMUL || EPI == HQ_EPI_DGELU) {
        float d[8], a[8];
        hq_unpack8(piece, d);
        hq_unpack8(aux[p], a);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          d[e] *= (EPI == HQ_EPI_DMUL ? a[e] : hq_gelu_grad(a[e]));
          csum[e] += d[e];
        }
        piece = hq_pack8(d);
      } else if constexpr (EPI == HQ_EPI_RESID) {
        float d[8], a[8];
        hq_unpack8(piece, d);
        hq_unpack8(aux[p], a);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] += a[e];
        piece = hq_pack8(d);
      } else if constexpr (EPI == HQ_EPI_BDR) {
        piece = hq_epi_bdr8(piece, aux[p], (uint32_t)goff, dr, key);
      }
      *reinterpret_cast<uint4*>(C + goff) = piece;
    }
    if constexpr (kColsum) {
      // lanes with equal ch (= lane & 7) hold the same 8 columns: reduce over the wave's 8 rows-groups,
      // then over the 4 waves through LDS
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) csum[e] += __shfl_xor(csum[e], o, 64);
      if (lane < 8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) scr[wave * 64 + lane * 8 + e] = csum[e];
      }
      __syncthreads();
      if (tid < 64) part[(size_t)tm * N + n0 + s * 64 + tid] = scr[tid] + scr[64 + tid] + scr[128 + tid] + scr[192 + tid];
      __syncthreads();
    }
  }
}


// ---------------------------------------------------------------------------------------- host side
int g_stagger = 0;   // experiment knob (hq_gemm_nt4_set_stagger)

template <int EPI, int BM, int BN, int MF>
void launch_one(const uint16_t* A, const uint16_t* B, uint16_t* C, const float* bias, uint16_t* P, const uint16_t* R,
                float* part, int M, int N, int K, int lda, int ldb, int ldc, hipStream_t s, const HqDropArg& dr) {
  using G = Geo<BM, BN, MF>;
  static bool init = [] {
    (void)hipFuncSetAttribute((const void*)gemm_nt4_kernel<EPI, BM, BN, MF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              G::LDS);
    return true;
  }();
  (void)init;
  const int grid = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL((gemm_nt4_kernel<EPI, BM, BN, MF>), dim3(grid), dim3(kThreads), G::LDS, s, A, B, C, bias, P, R, part, M,
                     N, K, lda, ldb, ldc, dr, g_stagger);
}

template <int BM, int BN, int MF>
void launch_shape(int epi, const uint16_t* A, const uint16_t* B, uint16_t* C, const float* bias, uint16_t* P,
                  const uint16_t* R, float* part, int M, int N, int K, int lda, int ldb, int ldc, hipStream_t s,
                  const HqDropArg& dr) {
  switch (epi) {
    case HQ_EPI_NONE: launch_one<HQ_EPI_NONE, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case HQ_EPI_BIAS: launch_one<HQ_EPI_BIAS, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case HQ_EPI_GELU: launch_one<HQ_EPI_GELU, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case HQ_EPI_DGELU: launch_one<HQ_EPI_DGELU, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case HQ_EPI_RESID: launch_one<HQ_EPI_RESID, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case HQ_EPI_GELUD: launch_one<HQ_EPI_GELUD, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case HQ_EPI_DMUL: launch_one<HQ_EPI_DMUL, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case HQ_EPI_BDR: launch_one<HQ_EPI_BDR, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case 8: launch_one<8, BM, BN, MF>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
  }
}

}  // namespace hq_nt4
}  // namespace

// Shape families of the two-workgroups-per-CU kernel: 0 = 192×192 (32x32x16 MFMA), 1 = 192×192 (16x16x32),
// 2 = 256×128 (32x32x16), 3 = 192×128 (32x32x16).  Returns the tile's BM (rows of the column-partial
// buffer = ceil(M / BM)), 0 if N does not tile.
void hq_gemm_nt4_set_stagger(int v) { hq_nt4::g_stagger = v; }

int hq_gemm_nt4_bm(int family, int N) {
  static const int bm[4] = {192, 192, 256, 192}, bn[4] = {192, 192, 128, 128};
  if (family < 0 || family > 3 || N % bn[family]) return 0;
  return bm[family];
}

void hq_gemm_nt4(int family, const uint16_t* A, const uint16_t* B, uint16_t* C, const float* bias, uint16_t* P,
                 const uint16_t* R, float* part, int M, int N, int K, int lda, int ldb, int ldc, int epi, hipStream_t s,
                 const HqDropArg& dr) {
  switch (family) {
    case 0: hq_nt4::launch_shape<192, 192, 32>(epi, A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case 1: hq_nt4::launch_shape<192, 192, 16>(epi, A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case 2: hq_nt4::launch_shape<256, 128, 32>(epi, A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
    case 3: hq_nt4::launch_shape<192, 128, 32>(epi, A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, s, dr); break;
  }
}
