// Weight-gradient GEMM ("TN") for gfx950:  part[s] = Aᵀ·B over the s-th token range, i.e.
//   dW[N, K] = Σ_t dy[t, n] · x[t, k]      A = dy [T, N], B = x [T, K], both token-major row-major,
// split-K over the T tokens into S fp32 partial slabs, then hq_splitk_reduce adds the slabs into the
// fp32 grad arena (optionally accumulating).  Replaces hipBLASLt's batched split-K wgrad.
//
// Same pipeline as gemm.hip's v2 NT kernel (256×256 output tile, 64-token K-tiles, 8 waves as
// 2 (N) × 4 (K) ping-ponging wave groups, four phases per K-tile, one 16 KiB half-panel of LDS-DMA
// per phase with three halves in flight under a counted vmcnt(6), buffer_load … lds with the K-tile
// advance in the scalar offset).  What differs is the operand layout: a half-panel is a
// [64 tokens][128 columns] slab (256-B rows) copied straight from the token-major tensor, and the
// MFMA fragments — which need 8 consecutive TOKENS of one column per lane — come from pairs of
// ds_read_b64_tr_b16 hardware-transposed reads (CDNA4 playbook T10).
// LDS bank conflicts: a transposed read's 32-lane half touches 8 token rows × 32 B of one column
// block; with 256-B rows those all hit the same banks, so each row's 32-B chunks are XOR-swizzled by
//   f(t) = (t & 3) | ((t >> 3) & 1) << 2
// (8 distinct values across the 8 rows → conflict-free).  The DMA image is lane-linear, so the
// swizzle is applied on the per-lane SOURCE chunk and undone on the read (playbook rule 21).
//
// fp8 variant (gemm_tn8_kernel, --precision fp8): dy in e5m2 and x in e4m3, both token-major bytes as their
// producers wrote them, on v_mfma_scale_f32_16x16x128_f8f6f4.  One MFMA consumes 128 tokens, so a K-tile is
// 128 tokens and a half-panel [128 tokens][128 columns] = 16 KiB — the same bytes, DMA instructions, phase
// table and waits as the bf16 kernel; the fragments (32 consecutive tokens of one column per lane) come
// from four ds_read_b64_tr_b8 per operand (8 tokens each), conflict-free under the row swizzle
//   f8(t) = ((t >> 1) & 3) | ((t >> 5) & 1) << 2   (16-B chunks of 128-B rows; tools/fp8_lab/tr8_probe.hip).
//
// Optional fused bias gradient (bf16 kernel only, BIAS): db[n] = Σ_t dy[t, n] is dyᵀ·1, so the first column-tile's
// blocks run, in their k-column-0 waves, one extra MFMA per dy fragment against a constant ones
// fragment (12.5 % more MFMAs in a third of the waves of a third of the blocks) and write fp32 partials
// [S][N] that the same reduce kernel folds in — replacing a separate 450 MB column-sum pass.
#include <algorithm>
#include <type_traits>
#include <utility>
#include <cstdlib>

#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int BT = 64;          // tokens per K-tile
constexpr int kThreads = 512;
constexpr int HALF = BT * 256;  // [64 tokens][128 bf16] = 16 KiB
constexpr int STAGE = 4 * HALF; // A0 A1 B0 B1

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int tswz(int t) { return (t & 3) | (((t >> 3) & 1) << 2); }
// f(integral_constant<int, n>) for n = 0 … N-1, fully unrolled in order
template <typename F, int... n>
__device__ __forceinline__ void unroll_n(F&& f, std::integer_sequence<int, n...>) { (f(std::integral_constant<int, n>{}), ...); }

// Fragment of 8 consecutive tokens (ks·32 + 8g … +7) of column `cblk`·16 + (lane & 15) from a half
// image at LDS byte address `img`.  `roff` = (8g + q)·256 + 8p and `sw` = f(8g + q) are per-lane
// constants (q = (lane>>2)&3, p = lane&3, g = lane>>4): the transposed read's lane 4q+p addresses
// row q, columns 4p..4p+3.  Inline asm, not the builtin: hipcc (ROCm 7.2) treats the builtin as
// aliasing the in-flight LDS-DMA and drains vmcnt(0) before every fragment read, which would
// serialise the pipeline; the consumer (mma) waits lgkmcnt(0) + sched_barrier itself.
__device__ __forceinline__ bf16x8_t trfrag(uint32_t img, int roff, int sw, int cblk, int ks) {
  const uint32_t a = img + roff + ((cblk ^ sw) << 5) + ks * (32 * 256);
  typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
  u32x2 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(hi) : "v"(a) : "memory");
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
  const u32x4 u = {lo[0], lo[1], hi[0], hi[1]};
  return __builtin_bit_cast(bf16x8_t, u);
}

template <int ABL, bool BIAS>
__global__ __launch_bounds__(kThreads, 1) void gemm_tn_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                              float* __restrict__ part, float* __restrict__ bpart, int T,
                                                              int N, int K, int S, int tiles_k) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);

  // bijective XCD remap; consecutive ids on an XCD = the same token range (split) over neighbouring
  // output tiles, so co-resident blocks share their dy / x slabs through that XCD's L2
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tiles = nwg / S;
  const int split = id / tiles, tile = id % tiles;
  const int n0 = (tile / tiles_k) * 256, k0 = (tile % tiles_k) * 256;
  const int nkt = (T + BT - 1) / BT;      // a partial last K-tile (T % 64 != 0) stages zero rows
  const int kt0 = (int)((long)split * nkt / S), kt1 = (int)((long)(split + 1) * nkt / S);
  const int nt = kt1 - kt0;
  const int rows = min(nt * BT, T - kt0 * BT);  // tokens of this split that exist: the descriptors end there
  // N, K multiples of 128: a last tile may stick out by 128 columns.  Its DMA reads the next row's bytes
  // (or zeros past the descriptor's end) into the unused columns, which only feed outputs that are never
  // stored: each output (n, k) depends on column n of dy and column k of x alone.
  HQ_DASSERT(n0 + 128 <= N && k0 + 128 <= K && nt >= 2 && rows > 0);

  const uint16_t* Ab = A + (size_t)kt0 * BT * N + n0;
  const uint16_t* Bb = B + (size_t)kt0 * BT * K + k0;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, rows * N * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, rows * K * 2, 0x00020000);

  // staging: wave w moves rows (2w + i)·4 … +3 of a half (1 KiB per instruction, lane-linear:
  // lane L → row +L/16, 16-B slot L%16), loading the source chunk that the swizzle places there
  int voA[2], voB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 4 + (lane >> 4);
    const int pos = lane & 15;
    const int c16 = ((((pos >> 1) ^ tswz(row))) << 1) | (pos & 1);
    voA[i] = (row * N + c16 * 8) * 2;
    voB[i] = (row * K + c16 * 8) * 2;
  }
  auto stage = [&](const __amdgpu_buffer_rsrc_t& rs, const int (&vo)[2], int ld, int half, int t, char* img) {
    if constexpr ((ABL & 1) != 0) return;
    char* dst = img + wave_u * 2048;
    const int so = half * 256 + t * BT * ld * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 1024), 16, vo[i], so, 0, 0);
  };
  auto stA = [&](int half, int t) { stage(rA, voA, N, half, t, smem + (t & 1) * STAGE + half * HALF); };
  auto stB = [&](int half, int t) { stage(rB, voB, K, half, t, smem + (t & 1) * STAGE + (2 + half) * HALF); };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // bias: only the k-column-0 waves (wn == 0) of the first column tile; block/wave-uniform flag
  const bool do_bias = BIAS && (k0 == 0) && (__builtin_amdgcn_readfirstlane(wn) == 0);
  f32x4_t bacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bacc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;

  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int roff = (8 * g + qq) * 256 + 8 * pp;
  const int sw = tswz(8 * g + qq);
  bf16x8_t af[2][4], bf0[2][2], bf1[2][2];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto readA = [&](int t, int mh) {
    if constexpr ((ABL & 2) != 0) { if (t > 0) return; }
    const uint32_t img = lds0 + (t & 1) * STAGE + mh * HALF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = trfrag(img, roff, sw, wm * 4 + i, ks);
  };
  auto readB = [&](int t, int nh, bf16x8_t (&bf)[2][2]) {
    if constexpr ((ABL & 2) != 0) { if (t > 0) return; }
    const uint32_t img = lds0 + (t & 1) * STAGE + (2 + nh) * HALF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[ks][j] = trfrag(img, roff, sw, wn * 2 + j, ks);
  };
  auto mma = [&](int mh, int nh, const bf16x8_t (&bf)[2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);   // keep the MFMAs below the wait (playbook rule 18)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mh * 4 + i][nh * 2 + j] = mfma16(bf[ks][j], af[ks][i], acc[mh * 4 + i][nh * 2 + j]);
    if constexpr (BIAS) {
      if (do_bias && nh == mh) {   // once per A-half: P0 (0,0) and P2 (1,1)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) bacc[mh * 4 + i] = mfma16(ones, af[ks][i], bacc[mh * 4 + i]);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue (always real loads): tile 0 A0 B0 B1 A1, tile 1 A0 B0 B1; retire tile 0
  {
    auto pro = [&](const __amdgpu_buffer_rsrc_t& rs, const int (&vo)[2], int ld, int half, int t, char* img) {
      char* dst = img + wave_u * 2048;
      const int so = half * 256 + t * BT * ld * 2;
#pragma unroll
      for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 1024), 16, vo[i], so, 0, 0);
    };
    pro(rA, voA, N, 0, 0, smem + 0 * HALF);
    pro(rB, voB, K, 0, 0, smem + 2 * HALF);
    pro(rB, voB, K, 1, 0, smem + 3 * HALF);
    pro(rA, voA, N, 1, 0, smem + 1 * HALF);
    pro(rA, voA, N, 0, 1, smem + STAGE + 0 * HALF);
    pro(rB, voB, K, 0, 1, smem + STAGE + 2 * HALF);
    pro(rB, voB, K, 1, 1, smem + STAGE + 3 * HALF);
  }
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  bar();

  // two phases of 32 MFMAs per K-tile (schedule, waits and hazard argument: gemm.hip, gemm_nt3_kernel):
  //   P01: reads B(0) A(0) B(1), stages A1 of t+1 | (0,0) (0,1);   P23: reads A(1), stages A0 B0 B1 of t+2 | (1,1) (1,0)
  auto ktile = [&](int t) {
    const bool more1 = t + 1 < nt, more2 = t + 2 < nt;
    // A1(t): younger are P23(t-1)'s three halves when it staged K-tile t+1 (the prologue's K-tile 1 at t = 0)
    if (t == 0 || more1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    readB(t, 0, bf0);
    readA(t, 0);
    readB(t, 1, bf1);
    if (more1) stA(1, t + 1);
    bar();
    mma(0, 0, bf0);
    mma(0, 1, bf1);
    bar();
    // A0 B0 B1 of t+1 (read by both wave rows in their next P01): younger is this P01's A1 stage.  Both rows
    // wait (gemm.hip, gemm_nt3_kernel P23: each half's rows come from all 8 waves)
    if (more1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    readA(t, 1);
    if (more2) { stA(0, t + 2); stB(0, t + 2); stB(1, t + 2); }
    bar();
    mma(1, 1, bf1);
    mma(1, 0, bf0);
    bar();
  };
  if (__builtin_amdgcn_readfirstlane(wm) == 0) {
    for (int t = 0; t < nt; ++t) ktile(t);
    bar();
  } else {
    bar();
    for (int t = 0; t < nt; ++t) ktile(t);
  }

  // epilogue: fp32 slab, straight from the accumulators (lane: output row n, 4 consecutive k)
  float* out = part + (size_t)split * N * K;
  const int fr = lane & 15, fq = lane >> 4;
  const bool n_full = n0 + 256 <= N, k_full = k0 + 256 <= K;   // block-uniform: a 128-column edge tile
#pragma unroll
  for (int I = 0; I < 8; ++I) {
    const int row = n0 + (I >> 2) * 128 + wm * 64 + (I & 3) * 16 + fr;
    if (!n_full && (I >> 2) == 1) continue;
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      if (!k_full && (J >> 1) == 1) continue;
      const int col = k0 + (J >> 1) * 128 + wn * 32 + (J & 1) * 16 + fq * 4;
      *reinterpret_cast<float4*>(out + (size_t)row * K + col) = make_float4(acc[I][J][0], acc[I][J][1], acc[I][J][2], acc[I][J][3]);
    }
  }
  if constexpr (BIAS) {
    // every accumulator register of bacc holds the column sum of output row n = lane & 15 (+ subtile)
    if (do_bias && fq == 0) {
#pragma unroll
      for (int I = 0; I < 8; ++I)
        if (n_full || (I >> 2) == 0) bpart[(size_t)split * N + n0 + (I >> 2) * 128 + wm * 64 + (I & 3) * 16 + fr] = bacc[I][0];
    }
  }
}

// ------------------------------------------------------------------ lockstep form (no bias)
// gemm_tn_kernel alternates its two wave rows (one row's MFMAs under the other's fragment reads), so at any
// time ONE wave per SIMD issues MFMAs, and a K-tile has four barriers.  Here all 8 waves run in lockstep, BOTH
// waves of a SIMD issue MFMAs all the time, and each wave hides its own fragment reads with two register
// sets: a K-tile is two sub-steps of 32 tokens (ks 0, ks 1), each with its operands in one set (A0 A1: 16
// VGPRs each, B0 B1: 8), and a sub-step first issues the 24 reads of the NEXT sub-step into the other set,
// then its own 32 MFMAs — every read has a whole sub-step to land.  One barrier per K-tile, at the start of
// ks 1: lgkmcnt(0) (every read of this K-tile's buffer has returned) + vmcnt(0) (this wave's share of K-tile
// t+1 has landed) → barrier → K-tile t+2 is staged into this K-tile's buffer and K-tile t+1's ks-0 operands
// are read.  Per accumulator the MFMAs run in gemm_tn_kernel's K order (ks 0, ks 1 per K-tile): bitwise equal.
template <int LAB>   // lab switches (results wrong): bit 0 no vmcnt wait, bit 1 no fragment reads in the loop
__global__ __launch_bounds__(kThreads, 1) void gemm_tn2_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                               float* __restrict__ part, int T, int N, int K, int S,
                                                               int tiles_k) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tiles = nwg / S;
  const int split = id / tiles, tile = id % tiles;
  const int n0 = (tile / tiles_k) * 256, k0 = (tile % tiles_k) * 256;
  const int nkt = (T + BT - 1) / BT;
  const int kt0 = (int)((long)split * nkt / S), kt1 = (int)((long)(split + 1) * nkt / S);
  const int nt = kt1 - kt0;
  const int rows = min(nt * BT, T - kt0 * BT);
  HQ_DASSERT(n0 + 128 <= N && k0 + 128 <= K && nt >= 2 && rows > 0);

  const uint16_t* Ab = A + (size_t)kt0 * BT * N + n0;
  const uint16_t* Bb = B + (size_t)kt0 * BT * K + k0;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, rows * N * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, rows * K * 2, 0x00020000);
  int voA[2], voB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 4 + (lane >> 4);
    const int pos = lane & 15;
    const int c16 = ((((pos >> 1) ^ tswz(row))) << 1) | (pos & 1);
    voA[i] = (row * N + c16 * 8) * 2;
    voB[i] = (row * K + c16 * 8) * 2;
  }
  auto stage = [&](const __amdgpu_buffer_rsrc_t& rs, const int (&vo)[2], int ld, int half, int t, char* img) {
    char* dst = img + wave_u * 2048;
    const int so = half * 256 + t * BT * ld * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 1024), 16, vo[i], so, 0, 0);
  };
  auto stage_all = [&](int t) {   // 8 DMA instructions per wave
    char* img = smem + (t & 1) * STAGE;
    stage(rA, voA, N, 0, t, img);
    stage(rA, voA, N, 1, t, img + HALF);
    stage(rB, voB, K, 0, t, img + 2 * HALF);
    stage(rB, voB, K, 1, t, img + 3 * HALF);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int roff = (8 * g + qq) * 256 + 8 * pp;
  const int sw = tswz(8 * g + qq);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // per-lane read bases of this K-tile's stage (cA, cB) and of the next one's (nA, nB), swapped every K-tile:
  // half, ks and second-read offsets are compile-time and go in the instruction's 16-bit offset field
  uint32_t cA[4], cB[2], nA[4], nB[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    cA[i] = lds0 + roff + (((wm * 4 + i) ^ sw) << 5);
    nA[i] = cA[i] + STAGE;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    cB[j] = lds0 + roff + (((wn * 2 + j) ^ sw) << 5);
    nB[j] = cB[j] + STAGE;
  }
  bf16x8_t fa[2][2][4], fb[2][2][2];   // [set][half][fragment]
  auto frag = [&](uint32_t base, auto off_c) {
    constexpr int OFF = decltype(off_c)::value;
    typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
    u32x2 lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(base), "i"(OFF) : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(base), "i"(OFF + 1024) : "memory");
    typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
    const u32x4 u = {lo[0], lo[1], hi[0], hi[1]};
    return __builtin_bit_cast(bf16x8_t, u);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // one of the 8 DMA instructions of K-tile t: A half 0/1, B half 0/1, two 1-KiB rows blocks each
  auto stage_one = [&](auto pc_c, int t) {
    constexpr int PC = decltype(pc_c)::value, W = PC >> 1, I = PC & 1;
    char* dst = smem + (t & 1) * STAGE + W * HALF + wave_u * 2048 + I * 1024;
    if constexpr (W < 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)dst, 16, voA[I], (W & 1) * 256 + t * BT * N * 2, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)dst, 16, voB[I], (W & 1) * 256 + t * BT * K * 2, 0, 0);
  };
  // fragment f (0 … 11) of a set: A0[0..3] B0[0..1] A1[0..3] B1[0..1] — the order in which the previous
  // sub-step last read the registers it overwrites (its MFMAs run (mh, nh, i, j) with mh outermost)
  auto read_frag = [&](auto q_c, auto f_c, const uint32_t (&ba)[4], const uint32_t (&bb)[2], auto ks_c) {
    constexpr int Q = decltype(q_c)::value, f = decltype(f_c)::value, KO = decltype(ks_c)::value * 32 * 256;
    if constexpr (f < 4) fa[Q][0][f] = frag(ba[f], std::integral_constant<int, KO>{});
    else if constexpr (f < 6) fb[Q][0][f - 4] = frag(bb[f - 4], std::integral_constant<int, 2 * HALF + KO>{});
    else if constexpr (f < 10) fa[Q][1][f - 6] = frag(ba[f - 6], std::integral_constant<int, HALF + KO>{});
    else fb[Q][1][f - 10] = frag(bb[f - 10], std::integral_constant<int, 3 * HALF + KO>{});
  };
  // one sub-step: the 32 MFMAs of set P with the next sub-step's 12 fragments (24 ds_reads) into the other set
  // after MFMAs 1, 3, …, 23 (hipcc spreads the pairs to one read per MFMA) and, with DMA, K-tile tdma's 8 staging
  // instructions after MFMAs 2, 6, …, 30 — so that neither wave of a SIMD stalls its MFMA issue on an LDS or DMA
  // burst.  (Measured slower: the 24 reads in one burst before the MFMAs; a second barrier mid-sub-step that
  // let the next K-tile's DMA land later, with the reads packed into the second half.)
  auto substep = [&](auto p_c, auto dma_c, const uint32_t (&ba)[4], const uint32_t (&bb)[2], auto rks_c, int tdma) {
    constexpr int P = decltype(p_c)::value, Q = 1 - P;
    __builtin_amdgcn_sched_barrier(0);
    unroll_n([&](auto n_c) {
      constexpr int n = decltype(n_c)::value;
      constexpr int mh = n >> 4, nh = (n >> 3) & 1, ii = (n >> 1) & 3, jj = n & 1;
      acc[mh * 4 + ii][nh * 2 + jj] = mfma16(fb[P][nh][jj], fa[P][mh][ii], acc[mh * 4 + ii][nh * 2 + jj]);
      if constexpr ((n & 1) && (n >> 1) < 12) read_frag(std::integral_constant<int, Q>{}, std::integral_constant<int, (n >> 1)>{}, ba, bb, rks_c);
      if constexpr (decltype(dma_c)::value && (n & 3) == 2) stage_one(std::integral_constant<int, (n >> 2)>{}, tdma);
      __builtin_amdgcn_sched_barrier(0);
    }, std::make_integer_sequence<int, 32>{});
  };

  // prologue: K-tiles 0 and 1 staged; K-tile 0's ks-0 fragments into set 0
  stage_all(0);
  stage_all(1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  bar();
  unroll_n([&](auto f_c) { read_frag(I0{}, f_c, cA, cB, I0{}); }, std::make_integer_sequence<int, 12>{});
  // Every K-tile stages K-tile t+2 and reads ahead unconditionally: past the split's last K-tile the DMA
  // reads zeros (outside the buffer descriptor) into the consumed buffer and the reads fetch an idle image —
  // a conditional would make hipcc hold two values of a register set across a branch.
  for (int t = 0; t < nt; ++t) {
    // ks 0 (set 0), reading ks 1 of this K-tile into set 1
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    substep(I0{}, std::false_type{}, cA, cB, I1{}, 0);
    // ks 1 (set 1): sync, then K-tile t+2's staging and K-tile t+1's ks 0 (into set 0) under the MFMAs
    if constexpr (LAB & 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(0)" ::: "memory");
    bar();
    substep(I1{}, std::true_type{}, nA, nB, I0{}, t + 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) { const uint32_t x = cA[i]; cA[i] = nA[i]; nA[i] = x; }
#pragma unroll
    for (int j = 0; j < 2; ++j) { const uint32_t x = cB[j]; cB[j] = nB[j]; nB[j] = x; }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");   // the trailing zero stages / reads

  // epilogue: fp32 slab, straight from the accumulators (as gemm_tn_kernel)
  float* out = part + (size_t)split * N * K;
  const int fr = lane & 15, fq = lane >> 4;
  const bool n_full = n0 + 256 <= N, k_full = k0 + 256 <= K;
#pragma unroll
  for (int I = 0; I < 8; ++I) {
    const int row = n0 + (I >> 2) * 128 + wm * 64 + (I & 3) * 16 + fr;
    if (!n_full && (I >> 2) == 1) continue;
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      if (!k_full && (J >> 1) == 1) continue;
      const int col = k0 + (J >> 1) * 128 + wn * 32 + (J & 1) * 16 + fq * 4;
      HQ_DASSERT(split < S && row < N && col + 4 <= K);
      *reinterpret_cast<float4*>(out + (size_t)row * K + col) = make_float4(acc[I][J][0], acc[I][J][1], acc[I][J][2], acc[I][J][3]);
    }
  }
}

// ------------------------------------------------------------------ fp8 (e5m2 dy × e4m3 x)
typedef __attribute__((ext_vector_type(8))) int i32x8;
constexpr int BT8 = 128;   // tokens (bytes) per K-tile

__device__ __forceinline__ int tswz8(int t) { return ((t >> 1) & 3) | (((t >> 5) & 1) << 2); }

// w: the x fragment (e4m3, format 0); g: the dy fragment (e5m2, format 1); unit e8m0 block scales
__device__ __forceinline__ f32x4_t mfma_tn8(const i32x8& w, const i32x8& g, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(w, g, c, 0, 1, 0, 127, 0, 127);
}

// 32 consecutive tokens (32·G … +31, G = lane >> 4) of column cblk·16 + (lane & 15) from a half image at
// LDS byte address `img`: four transposed reads of 8 tokens each (rows +0, +8, +16, +24 → offsets 1 KiB
// apart).  `roff` = (32G + q)·128 + 8p and `sw` = f8(32G + q) are lane constants (q = (lane>>1)&7,
// p = lane&1: lane 2q + p of a 16-lane group addresses row q, bytes 8p … 8p+7 of the column block).
__device__ __forceinline__ i32x8 trfrag8(uint32_t img, int roff, int sw, int cblk) {
  const uint32_t a = img + roff + ((cblk ^ sw) << 4);
  typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
  u32x2 r0, r1, r2, r3;
  asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(r0) : "v"(a) : "memory");
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:1024" : "=v"(r1) : "v"(a) : "memory");
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:2048" : "=v"(r2) : "v"(a) : "memory");
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:3072" : "=v"(r3) : "v"(a) : "memory");
  i32x8 v;
  v[0] = (int)r0[0]; v[1] = (int)r0[1]; v[2] = (int)r1[0]; v[3] = (int)r1[1];
  v[4] = (int)r2[0]; v[5] = (int)r2[1]; v[6] = (int)r3[0]; v[7] = (int)r3[1];
  return v;
}

// No fused bias variant: its 40 extra VGPRs (bias accumulators + a ones fragment) spill at 256; the fp8
// step runs the one wgrad with a bias (QKV) in bf16.
__global__ __launch_bounds__(kThreads, 1) void gemm_tn8_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                               float* __restrict__ part, const float* __restrict__ sa,
                                                               const float* __restrict__ sb, int T, int N, int K, int S,
                                                               int tiles_k) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tiles = nwg / S;
  const int split = id / tiles, tile = id % tiles;
  const int n0 = (tile / tiles_k) * 256, k0 = (tile % tiles_k) * 256;
  const int nkt = (T + BT8 - 1) / BT8;
  const int kt0 = (int)((long)split * nkt / S), kt1 = (int)((long)(split + 1) * nkt / S);
  const int nt = kt1 - kt0;
  const int rows = min(nt * BT8, T - kt0 * BT8);
  HQ_DASSERT(n0 + 128 <= N && k0 + 128 <= K && nt >= 2 && rows > 0);

  const uint8_t* Ab = A + (size_t)kt0 * BT8 * N + n0;
  const uint8_t* Bb = B + (size_t)kt0 * BT8 * K + k0;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, rows * N, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, rows * K, 0x00020000);

  // staging: wave w moves rows (2w + i)·8 … +7 of a half (1 KiB per instruction, lane-linear: lane L → row
  // +L/8, 16-B slot L%8), loading the source chunk that the swizzle places there
  int voA[2], voB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3);
    const int c16 = (lane & 7) ^ tswz8(row);
    voA[i] = row * N + c16 * 16;
    voB[i] = row * K + c16 * 16;
  }
  auto dma = [&](const __amdgpu_buffer_rsrc_t& rs, const int (&vo)[2], int ld, int half, int t, char* img) {
    char* dst = img + wave_u * 2048;
    const int so = half * 128 + t * BT8 * ld;
#pragma unroll
    for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 1024), 16, vo[i], so, 0, 0);
  };
  auto stA = [&](int half, int t) { dma(rA, voA, N, half, t, smem + (t & 1) * STAGE + half * HALF); };
  auto stB = [&](int half, int t) { dma(rB, voB, K, half, t, smem + (t & 1) * STAGE + (2 + half) * HALF); };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int G = lane >> 4, qq = (lane >> 1) & 7, pp = lane & 1;
  const int roff = (32 * G + qq) * 128 + 8 * pp;
  const int sw = tswz8(32 * G + qq);
  i32x8 af[4], bf0[2], bf1[2];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto readA = [&](int t, int mh) {
    const uint32_t img = lds0 + (t & 1) * STAGE + mh * HALF;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = trfrag8(img, roff, sw, wm * 4 + i);
  };
  auto readB = [&](int t, int nh, i32x8 (&bf)[2]) {
    const uint32_t img = lds0 + (t & 1) * STAGE + (2 + nh) * HALF;
#pragma unroll
    for (int j = 0; j < 2; ++j) bf[j] = trfrag8(img, roff, sw, wn * 2 + j);
  };
  auto mma = [&](int mh, int nh, const i32x8 (&bf)[2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[mh * 4 + i][nh * 2 + j] = mfma_tn8(bf[j], af[i], acc[mh * 4 + i][nh * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue, schedule and waits: identical to gemm_tn_kernel (2 DMA instructions per wave per half)
  stA(0, 0); stB(0, 0); stB(1, 0); stA(1, 0); stA(0, 1); stB(0, 1); stB(1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  bar();
  auto ktile = [&](int t) {
    const bool more1 = t + 1 < nt, more2 = t + 2 < nt;
    if (t == 0 || more1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    readB(t, 0, bf0);
    readA(t, 0);
    readB(t, 1, bf1);
    if (more1) stA(1, t + 1);
    bar();
    mma(0, 0, bf0);
    mma(0, 1, bf1);
    bar();
    // both wave rows (gemm.hip, gemm_nt3_kernel P23)
    if (more1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    readA(t, 1);
    if (more2) { stA(0, t + 2); stB(0, t + 2); stB(1, t + 2); }
    bar();
    mma(1, 1, bf1);
    mma(1, 0, bf0);
    bar();
  };
  if (__builtin_amdgcn_readfirstlane(wm) == 0) {
    for (int t = 0; t < nt; ++t) ktile(t);
    bar();
  } else {
    bar();
    for (int t = 0; t < nt; ++t) ktile(t);
  }

  // epilogue: fp32 slab of the dequantised product
  const float dq = sa[0] * sb[0];
  float* out = part + (size_t)split * N * K;
  const int fr = lane & 15, fq = lane >> 4;
  const bool n_full = n0 + 256 <= N, k_full = k0 + 256 <= K;
#pragma unroll
  for (int I = 0; I < 8; ++I) {
    const int row = n0 + (I >> 2) * 128 + wm * 64 + (I & 3) * 16 + fr;
    if (!n_full && (I >> 2) == 1) continue;
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      if (!k_full && (J >> 1) == 1) continue;
      const int col = k0 + (J >> 1) * 128 + wn * 32 + (J & 1) * 16 + fq * 4;
      *reinterpret_cast<float4*>(out + (size_t)row * K + col) =
          make_float4(acc[I][J][0] * dq, acc[I][J][1] * dq, acc[I][J][2] * dq, acc[I][J][3] * dq);
    }
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float4* __restrict__ part, int S, size_t n4,
                                                            float4* __restrict__ out, int accumulate) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 a = accumulate ? out[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    int s = 0;
    for (; s + 4 <= S; s += 4) {
      const float4 p0 = part[(size_t)s * n4 + i], p1 = part[(size_t)(s + 1) * n4 + i];
      const float4 p2 = part[(size_t)(s + 2) * n4 + i], p3 = part[(size_t)(s + 3) * n4 + i];
      a.x += (p0.x + p1.x) + (p2.x + p3.x);
      a.y += (p0.y + p1.y) + (p2.y + p3.y);
      a.z += (p0.z + p1.z) + (p2.z + p3.z);
      a.w += (p0.w + p1.w) + (p2.w + p3.w);
    }
    for (; s < S; ++s) {
      const float4 p = part[(size_t)s * n4 + i];
      a.x += p.x; a.y += p.y; a.z += p.z; a.w += p.w;
    }
    out[i] = a;
  }
}

}  // namespace

int hq_gemm_tn_splits(int T, int N, int K) {
  if (T <= 0 || N % 128 || K % 128 || N < 128 || K < 128) return 0;
  if ((size_t)T * N * 2 >= (1ull << 31) || (size_t)T * K * 2 >= (1ull << 31)) return 0;
  const int tiles = ((N + 255) / 256) * ((K + 255) / 256);
  int S = 256 / tiles;                     // one full round of the 256 CUs
  if (S < 1) S = 1;
  const int nkt = (T + BT - 1) / BT;
  // K-tiles per block kept (prologue amortised): 4 (micro-batch 2 x 512: 388 -> 400 samples/s vs 8, batch
  // 64 neutral; batch 256 never splits that far)
  constexpr int min_kt = 4;
  while (S > 1 && nkt / S < min_kt) --S;
  if (nkt < 2) return 0;
  return S;
}

// bias-free weight gradients: 0 = auto — gemm_tn2_kernel (lockstep) for N >= 2304 at K <= 768, where it measured
// 5 % faster inside the training step (the FFN1 weight gradient; profiles/r5_tn_lockstep), gemm_tn_kernel
// (alternating wave rows) elsewhere (the out-projection's was 11 % slower lockstep, FFN2's even); 1 = always
// lockstep, 5 = always alternating rows; 2-4 lockstep lab builds (tests, tools/tn_variant_bench.py)
int g_tn_variant = 0;
void hq_gemm_tn_set_variant(int v) { g_tn_variant = v; }

void hq_gemm_tn(const uint16_t* A, const uint16_t* B, float* part, float* out, float* bpart, float* bout, int T, int N, int K,
                int S, bool accumulate, hipStream_t s) {
  constexpr size_t lds = 2 * STAGE;
  static bool init = [] {
    (void)hipFuncSetAttribute((const void*)gemm_tn_kernel<0, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)gemm_tn_kernel<0, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)gemm_tn2_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)gemm_tn2_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)gemm_tn2_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)gemm_tn2_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return true;
  }();
  (void)init;
  const int tiles_k = (K + 255) / 256, tiles = ((N + 255) / 256) * tiles_k;
  if (bout)
    hipLaunchKernelGGL((gemm_tn_kernel<0, true>), dim3(tiles * S), dim3(kThreads), lds, s, A, B, part, bpart, T, N, K, S,
                       tiles_k);
  else if ((g_tn_variant >= 1 && g_tn_variant <= 4) || (g_tn_variant == 0 && N >= 2304 && K <= 768)) {
    auto k2 = g_tn_variant <= 1 ? gemm_tn2_kernel<0> : g_tn_variant == 2 ? gemm_tn2_kernel<1>
            : g_tn_variant == 3 ? gemm_tn2_kernel<2> : gemm_tn2_kernel<3>;
    hipLaunchKernelGGL(k2, dim3(tiles * S), dim3(kThreads), lds, s, A, B, part, T, N, K, S, tiles_k);
  }
  else
    hipLaunchKernelGGL((gemm_tn_kernel<0, false>), dim3(tiles * S), dim3(kThreads), lds, s, A, B, part, bpart, T, N, K, S,
                       tiles_k);
  const size_t n4 = (size_t)N * K / 4;
  const int grid = (int)std::min<size_t>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, s, (const float4*)part, S, n4, (float4*)out,
                     accumulate ? 1 : 0);
  if (bout)
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((N / 4 + 255) / 256), dim3(256), 0, s, (const float4*)bpart, S,
                       (size_t)N / 4, (float4*)bout, accumulate ? 1 : 0);
}

int hq_gemm_tn8_splits(int T, int N, int K) {
  if (T <= 0 || N % 128 || K % 128 || N < 128 || K < 128) return 0;
  if ((size_t)T * N >= (1ull << 31) || (size_t)T * K >= (1ull << 31)) return 0;
  const int tiles = ((N + 255) / 256) * ((K + 255) / 256);
  int S = 256 / tiles;
  if (S < 1) S = 1;
  const int nkt = (T + BT8 - 1) / BT8;
  while (S > 1 && nkt / S < 4) --S;
  if (nkt < 2) return 0;
  return S;
}

void hq_gemm_tn8(const uint8_t* A, const uint8_t* B, const float* sa, const float* sb, float* part, float* out, int T,
                 int N, int K, int S, bool accumulate, hipStream_t s) {
  constexpr size_t lds = 2 * STAGE;
  static bool init = [] {
    (void)hipFuncSetAttribute((const void*)gemm_tn8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return true;
  }();
  (void)init;
  const int tiles_k = (K + 255) / 256, tiles = ((N + 255) / 256) * tiles_k;
  hipLaunchKernelGGL(gemm_tn8_kernel, dim3(tiles * S), dim3(kThreads), lds, s, A, B, part, sa, sb, T, N, K, S, tiles_k);
  const size_t n4 = (size_t)N * K / 4;
  const int grid = (int)std::min<size_t>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, s, (const float4*)part, S, n4, (float4*)out,
                     accumulate ? 1 : 0);
}
