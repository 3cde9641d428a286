// OCP fp8 (e4m3fn) "NT" GEMM for the --precision fp8 forward projections on gfx950:
//   C[M,N] = (A8[M,K] · B8[N,K]ᵀ) · sa · sb (+ epilogue),  A8/B8 e4m3, sa/sb per-tensor dequant scales.
//
// The pipeline is gemm.hip's v2 (256×256 output tile, 8 ping-ponging waves, four phases per K-tile,
// one 16 KiB half-panel of buffer_load…lds per phase under a counted vmcnt(6)) with the byte-identical
// LDS image: a K-tile is 128 fp8 = 128 B per row, exactly the bf16 kernel's 64 × 2 B rows.  What
// changes is the matrix core: v_mfma_scale_f32_16x16x128_f8f6f4 (block-scaled MX form, unit e8m0
// scales) consumes a whole 128-deep K-tile per instruction at twice the bf16 FLOP rate, so per LDS
// byte the MFMA time equals the bf16 kernel's while each K-tile carries twice the K — half the
// K-tiles, half the load traffic.  Per-tensor scales are applied once in the epilogue.
//
// Fragment map (probed with exact integer data, tools/fp8_lab/mfma_probe.hip): lane l holds
// A[row l&15][32·(l>>4) … +31] and B[col l&15][same k] — 32 contiguous bytes = two swizzled 16-B
// LDS slots (2·fq, 2·fq+1); C/D is the standard 16×16 map.
//
// Epilogues, forward (A = e4m3 activations): EPI_BIAS (QKV / out-proj / FFN2) and EPI_GELUD (FFN1:
// act = gelu(pre), P = gelu'(pre)); Q8 additionally writes act as e4m3 for the next fp8 GEMM.
// Backward dgrad (A = e5m2 activation gradient, B = e4m3 Wᵀ): EPI_NONE (FFN1 / out-proj dgrad), EPI_RESID
// (QKV dgrad + the residual gradient, read through P) and EPI_DMUL (FFN2 dgrad: dpre = (dy·W) ⊙ P with P = the stored gelu', plus per-tile column sums of dpre
// for the FFN1 bias gradient); Q8 on DMUL writes dpre as e5m2 for the FFN1 dgrad.  The e5m2 range
// (±57344) is what gradients need; the mixed-format MFMA takes the operand formats as immediates.
// Every Q8 output is under DELAYED scaling: the scale is derived from the previous step's amax (slot
// (phase+2)%3 of the 4-float state), this step's amax accumulates into slot `phase`, slot (phase+1)%3
// is cleared for the step after, and the scale used is stored in state[3] for the consumer GEMM's
// dequantisation.  No host synchronisation anywhere.
#include <algorithm>
#include <cstdio>
#include <vector>

#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 128;  // BK in fp8 elements (= bytes)
constexpr int kThreads = 512;
constexpr float kFp8Max = 448.f;
constexpr float kMargin = 2.f;               // delayed-scaling headroom over last step's amax

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) int i32x8;

// w: the weight fragment (always e4m3, format code 0); x: the activation fragment, e4m3 (0) in the
// forward or e5m2 (1) for the backward's gradients.  Unit e8m0 block scales (127).
template <int FX>
__device__ __forceinline__ f32x4_t mfma_fp8(const i32x8& w, const i32x8& x, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(w, x, c, 0, FX, 0, 127, 0, 127);
}

// 16-B chunk swizzle of the 128-B LDS rows: chunk ^= f8row(row).  With the bf16 kernels' (row >> 1) & 7 the
// fragment reads below were 2-way bank-conflicted (PMC: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.50): in
// each 16-lane group of a ds_read_b128 (lanes {0–3,12–15,20–27}, {4–11,16–19,28–31}, …) rows 2j / 2j+1 of
// fq = 0 and rows of fq = 1 land on the same chunks.  j ^ ((j & 2) << 1), j = (row >> 1) & 7, gives the
// eight rows of each parity in a group eight distinct chunks for every slot pair (2fq, 2fq+1).
__device__ __forceinline__ int f8row(int row) {
  const int j = (row >> 1) & 7;
  return j ^ ((j & 2) << 1);
}

// 32-byte fragment (k = 32·fq … +31) of LDS row `row`: slots 2fq and 2fq+1, source swizzle undone.
// Inline asm: with plain loads hipcc (ROCm 7.2) drained vmcnt(0) before these reads in this kernel (it
// could not rule out aliasing with the in-flight LDS-DMA); mma() waits lgkmcnt(0) + sched_barrier.
__device__ __forceinline__ i32x8 frag32(uint32_t panel, int row, int fq) {
  const int sw = f8row(row);
  const uint32_t a0 = panel + row * 128 + (((2 * fq) ^ sw) << 4);
  const uint32_t a1 = panel + row * 128 + (((2 * fq + 1) ^ sw) << 4);
  typedef __attribute__((ext_vector_type(4))) int i32x4;
  i32x4 lo, hi;
  asm volatile("ds_read_b128 %0, %1" : "=v"(lo) : "v"(a0) : "memory");
  asm volatile("ds_read_b128 %0, %1" : "=v"(hi) : "v"(a1) : "memory");
  i32x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

__device__ __forceinline__ float delayed_scale(const float* st, int phase) {
  static_assert(kMargin == 2.f && kFp8Max == kHqFp8Max, "one delayed-scaling rule (hq_common.h)");
  return hq_fp8_delayed_scale(st, phase);   // first step: unit scale
}

constexpr bool grad_epi(int epi) { return epi == HQ_EPI_NONE || epi == HQ_EPI_DMUL || epi == HQ_EPI_RESID; }

// One 8-column bf16 piece of the dequantised (+bias) tile through the epilogue `EPI` and out to global
// memory at element offset goff: RESID adds the residual, DMUL multiplies by gelu' (column sums into csum)
// and with Q8 writes the e5m2 copy, GELUD writes gelu' to P and act (Q8: also e4m3).  `aux` is the piece of
// P (DMUL: gelu', RESID: residual) loaded ahead.  WC = false skips the bf16 output (GELUD / DMUL with Q8, once
// every consumer reads the fp8 copy) — a template flag: a runtime test around the 16 unrolled stores made hipcc
// spill the DMUL epilogue.
// the epilogue operand piece at element offset goff: 8 bf16 (RESID's residual, bf16 DMUL's gelu') or, for the
// fp8 DMUL (Q8), the 8-byte gelu' code the fp8 FFN1 forward stored (hq_gd_encode8)
template <int EPI, bool Q8>
__device__ __forceinline__ uint4 load_aux(const uint16_t* __restrict__ P, size_t goff) {
  if constexpr (EPI == HQ_EPI_DMUL && Q8) {
    const uint2 c = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(P) + goff);
    return make_uint4(c.x, c.y, 0u, 0u);
  } else {
    return *reinterpret_cast<const uint4*>(P + goff);
  }
}

template <int EPI, bool Q8, bool WC, bool GD8>
__device__ __forceinline__ void epi_piece(uint4 piece, const uint4& aux, size_t goff, uint16_t* __restrict__ C,
                                          uint16_t* __restrict__ P, uint8_t* __restrict__ C8, float inv8, float& amax,
                                          float (&csum)[8]) {
  if constexpr (EPI == HQ_EPI_RESID) {
    float d[8], rr[8];
    hq_unpack8(piece, d);
    hq_unpack8(aux, rr);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] += rr[e];
    piece = hq_pack8(d);
  } else if constexpr (EPI == HQ_EPI_DMUL) {
    // no fma contraction of d·gd into the column sum: hipcc contracted it in one kernel form and not the
    // other, and the per-tile / persistent partials must agree bit for bit
#pragma clang fp contract(off)
    float d[8], gd[8];
    hq_unpack8(piece, d);
    if constexpr (Q8) hq_gd_decode8(make_uint2(aux.x, aux.y), gd);   // the fp8 forward's 8-bit gelu' code
    else hq_unpack8(aux, gd);
#pragma unroll
    for (int e = 0; e < 8; ++e) { d[e] *= gd[e]; csum[e] += d[e]; }
    piece = hq_pack8(d);
    if constexpr (Q8) {   // e5m2 dpre for the FFN1 dgrad, from the bf16-rounded values the bf16 copy holds
      hq_unpack8(piece, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(d[e]));
      *reinterpret_cast<uint2*>(C8 + goff) = make_uint2(hq_pack_bf8x4(d, inv8), hq_pack_bf8x4(d + 4, inv8));
    }
  } else if constexpr (EPI == HQ_EPI_GELUD) {
    float x[8], g[8];
    hq_unpack8(piece, x);
    hq_gelu_grad8(x, g);   // g = gelu'(x), x = gelu(x)
    // GD8: the 8-bit gelu' code, only when the fp8 FFN2 dgrad will read it; else gelu' in bf16
    if constexpr (GD8) *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(P) + goff) = hq_gd_encode8(g);
    else *reinterpret_cast<uint4*>(P + goff) = hq_pack8(g);
    piece = hq_pack8(x);
    if constexpr (Q8) {
      float f[8];
      hq_unpack8(piece, f);   // quantise the bf16-rounded act, exactly what the bf16 copy holds
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(f[e]));
      *reinterpret_cast<uint2*>(C8 + goff) = make_uint2(hq_pack_fp8x4(f, inv8), hq_pack_fp8x4(f + 4, inv8));
    }
  }
  if constexpr (WC) *reinterpret_cast<uint4*>(C + goff) = piece;
}

template <int EPI, bool Q8, bool WC, bool GD8>
__global__ __launch_bounds__(kThreads, 1) void gemm_fp8_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                               uint16_t* __restrict__ C, const float* __restrict__ bias,
                                                               uint16_t* __restrict__ P, const float* __restrict__ sa,
                                                               const float* __restrict__ sb, uint8_t* __restrict__ C8,
                                                               const float* __restrict__ q8, float* __restrict__ part8,
                                                               float* __restrict__ part, int phase, int M, int N, int K,
                                                               int lda, int ldb, int ldc) {
  constexpr int FX = grad_epi(EPI) ? 1 : 0;   // A operand: e5m2 gradient (backward) or e4m3 activation
  constexpr int PANEL = 256 * 128, STAGE = 2 * PANEL;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_n = N / BN;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  HQ_DASSERT(m0 + BM <= M && n0 + BN <= N && K % BK == 0 && K >= 2 * BK);
  const uint8_t* Ab = A + (size_t)m0 * lda;
  const uint8_t* Bb = B + (size_t)n0 * ldb;
  const int nt = K / BK;
  if constexpr (Q8) hq_fp8_publish_scale(q8, phase, EPI == HQ_EPI_DMUL ? kHqBf8Max : kHqFp8Max);

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, BM * lda, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, BN * ldb, 0x00020000);
  int voA[2], voB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + (lane >> 3);
    const int src_slot = (lane & 7) ^ f8row(row);
    voA[i] = row * lda + src_slot * 16;
    voB[i] = row * ldb + src_slot * 16;
  }
  auto half = [&](const __amdgpu_buffer_rsrc_t& rs, const int (&vo)[2], int ld, int h, int t, char* panel) {
    char* dst = panel + (h * 128 + wave_u * 16) * 128;
    const int so = h * 128 * ld + t * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 8 * 128), 16, vo[i], so, 0, 0);
  };
  auto stA = [&](int h, int t) { half(rA, voA, lda, h, t, smem + (t & 1) * STAGE); };
  auto stB = [&](int h, int t) { half(rB, voB, ldb, h, t, smem + (t & 1) * STAGE + PANEL); };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  i32x8 af[4], bf0[2], bf1[2];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto readA = [&](int t, int mh) {
    const uint32_t pa = lds0 + (t & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag32(pa, mh * 128 + wm * 64 + i * 16 + fr, fq);
  };
  auto readB = [&](int t, int nh, i32x8 (&bf)[2]) {
    const uint32_t pb = lds0 + (t & 1) * STAGE + PANEL;
#pragma unroll
    for (int j = 0; j < 2; ++j) bf[j] = frag32(pb, wn * 64 + nh * 32 + j * 16 + fr, fq);
  };
  auto mma = [&](int mh, int nh, const i32x8 (&bf)[2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);   // keep the MFMAs below the wait (playbook rule 18)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[mh * 4 + i][nh * 2 + j] = mfma_fp8<FX>(bf[j], af[i], acc[mh * 4 + i][nh * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  stA(0, 0); stB(0, 0); stB(1, 0); stA(1, 0); stA(0, 1); stB(0, 1); stB(1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  bar();
  // two 32-MFMA phases per K-tile; stage / wait table and hazard argument: gemm.hip, gemm_nt3_kernel
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

  // ---- epilogue: acc · (sa·sb) (+bias) -> bf16 staging (as gemm.hip v2), then row-coalesced pieces
  const float dq = sa[0] * sb[0];
  constexpr int WN = 64, RS = WN * 2 + 16;
  constexpr bool kBias = EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELUD;
  char* wreg = smem + wave * (128 * RS);
#pragma unroll
  for (int J = 0; J < 4; ++J) {
    const int nh = J >> 1, j = J & 1;
    const int lc = nh * 32 + j * 16 + fq * 4;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (kBias) bv = *reinterpret_cast<const float4*>(bias + n0 + wn * 64 + nh * 32 + j * 16 + fq * 4);
#pragma unroll
    for (int I = 0; I < 8; ++I) {
      float v[4] = {fmaf(acc[I][J][0], dq, bv.x), fmaf(acc[I][J][1], dq, bv.y), fmaf(acc[I][J][2], dq, bv.z),
                    fmaf(acc[I][J][3], dq, bv.w)};
      *reinterpret_cast<uint2*>(wreg + (I * 16 + fr) * RS + lc * 2) = hq_pack4(v);
    }
  }
  float s8 = 1.f, inv8 = 1.f, amax = 0.f;
  if constexpr (Q8) {
    s8 = hq_fp8_delayed_scale(q8, phase, EPI == HQ_EPI_DMUL ? kHqBf8Max : kHqFp8Max);
    inv8 = 1.f / s8;
  }
  constexpr int SEGS = WN / 8, ROWS_PER_IT = 64 / SEGS, NIT = 128 / ROWS_PER_IT;
  const int seg = lane % SEGS, rsub = lane / SEGS;
  const int gcol = n0 + wn * 64 + seg * 8;   // full 128-B lines per store (gemm.hip gemm_nt3_kernel)
  auto grow_of = [&](int it) {
    const int lr = it * ROWS_PER_IT + rsub;
    return m0 + (lr >> 6) * 128 + wm * 64 + (lr & 63);
  };
  // DMUL's gelu' / RESID's residual (both via P): all 16 pieces of this lane issued at once (one exposed
  // HBM latency, gemm.hip v2)
  constexpr bool kAux = EPI == HQ_EPI_DMUL || EPI == HQ_EPI_RESID;
  uint4 aux[kAux ? NIT : 1];
  float csum[8];
  if constexpr (kAux) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) aux[it] = load_aux<EPI, Q8>(P, (size_t)grow_of(it) * ldc + gcol);
  }
  if constexpr (EPI == HQ_EPI_DMUL) {
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  }
  auto piece_out = [&](int it) {
    const int lr = it * ROWS_PER_IT + rsub;
    const uint4 piece = *reinterpret_cast<const uint4*>(wreg + lr * RS + seg * 16);
    epi_piece<EPI, Q8, WC, GD8>(piece, aux[kAux ? it : 0], (size_t)grow_of(it) * ldc + gcol, C, P, C8, inv8, amax, csum);
  };
  if constexpr (kAux) {   // fully unrolled: aux[] must stay in registers
#pragma unroll
    for (int it = 0; it < NIT; ++it) piece_out(it);
  } else {
#pragma unroll 4
    for (int it = 0; it < NIT; ++it) piece_out(it);
  }
  if constexpr (Q8) {   // this wave's amax -> its own partial slot (hq_fp8_amax_fold reduces them)
    amax = hq_wave_max(amax);
    if (lane == 0) part8[blockIdx.x * (kThreads / 64) + wave] = amax;
  }
  if constexpr (EPI == HQ_EPI_DMUL) {   // column sums of dpre over this tile's 256 rows -> part[tm][n]
#pragma unroll
    for (int e = 0; e < 8; ++e)
      for (int o = SEGS; o < 64; o <<= 1) csum[e] += __shfl_xor(csum[e], o, 64);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [2][BN] by tile column, one row per wm
    if (rsub == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wm * BN + (gcol - n0) + e] = csum[e];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += kThreads) part[(size_t)tm * N + n0 + c] = red[c] + red[BN + c];
  }
}

// ------------------------------------------------------------------ persistent form (gemm.hip v3)
// At K = 768 a 256² fp8 tile is only 6 K-tiles, so v2's per-tile fixed cost (workgroup launch, the
// prologue's first HBM round trip, the epilogue's drain) is about half of it.  This form keeps ONE workgroup
// per CU walking tiles (tile = id, id + grid, …) and runs the LDS-DMA pipeline across the tile seam exactly
// as gemm.hip's gemm_nt3_kernel (same LDS plan, phase table and counted waits — the fp8 K-tile has the bf16
// one's byte geometry): the next tile's K-tile 0 is staged during this tile's last two K-tiles, its K-tile-1
// first halves after the epilogue, which borrows the last K-tile's buffer (two 64-row rounds per wave).
// The epilogue's vm ops per lane (E) are counted into the next tile's first waits.  Amax partials: one per
// wave, accumulated over the wave's tiles and written at the end.
template <int EPI, bool Q8, bool WC>
struct P8Epi {   // vm ops per lane per tile: C (WC), P (GELUD), C8 (Q8) stores, aux loads (DMUL / RESID)
  static constexpr bool kAux = EPI == HQ_EPI_DMUL || EPI == HQ_EPI_RESID;
  static constexpr int kStores = (WC ? 16 : 0) + (EPI == HQ_EPI_GELUD ? 16 : 0) + (Q8 ? 16 : 0);
  static constexpr int E = kStores + (kAux ? 16 : 0);
  static_assert(6 + E <= 63, "vmcnt field");
};

template <int EPI, bool Q8, bool WC, bool GD8>
__global__ __launch_bounds__(kThreads, 1) void gemm_fp8p_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                                uint16_t* __restrict__ C, const float* __restrict__ bias,
                                                                uint16_t* __restrict__ P, const float* __restrict__ sa,
                                                                const float* __restrict__ sb, uint8_t* __restrict__ C8,
                                                                const float* __restrict__ q8, float* __restrict__ part8,
                                                                float* __restrict__ part, int phase, int M, int N, int K) {
  constexpr int FX = grad_epi(EPI) ? 1 : 0;
  constexpr int PANEL = 256 * 128, STAGE = 2 * PANEL;
  constexpr int WN = 64, RS = WN * 2 + 16;
  constexpr int REGION = 64 * RS;            // one wave's 64-row staging round (9216 B)
  constexpr int SPARE = 2 * STAGE;           // past both stage buffers: wave 7's region, then csum scratch
  constexpr int E = P8Epi<EPI, Q8, WC>::E;
  constexpr bool kAux = P8Epi<EPI, Q8, WC>::kAux;
  static_assert(7 * REGION <= STAGE && SPARE + REGION + 2 * BN * 4 <= 160 * 1024, "LDS plan");
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_n = N / BN, ntiles = (M / BM) * tiles_n;
  const int nt = K / BK;
  const int lda = K, ldb = K, ldc = N;
  HQ_DASSERT(K % BK == 0 && nt >= 2 && N % BN == 0 && M % BM == 0);

  int voA[2], voB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + (lane >> 3);
    const int src_slot = (lane & 7) ^ f8row(row);
    voA[i] = row * lda + src_slot * 16;
    voB[i] = row * ldb + src_slot * 16;
  }
  auto rsrc_a = [&](int tile) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)(tile / tiles_n) * BM * lda), (short)0, BM * lda, 0x00020000);
  };
  auto rsrc_b = [&](int tile) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(B + (size_t)(tile % tiles_n) * BN * ldb), (short)0, BN * ldb, 0x00020000);
  };
  auto stA = [&](__amdgpu_buffer_rsrc_t rs, int half, int kt, int buf) {
    char* dst = smem + buf * STAGE + (half * 128 + wave_u * 16) * 128;
    const int so = half * 128 * lda + kt * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 8 * 128), 16, voA[i], so, 0, 0);
  };
  auto stB = [&](__amdgpu_buffer_rsrc_t rs, int half, int kt, int buf) {
    char* dst = smem + buf * STAGE + PANEL + (half * 128 + wave_u * 16) * 128;
    const int so = half * 128 * ldb + kt * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 8 * 128), 16, voB[i], so, 0, 0);
  };

  f32x4_t acc[8][4];
  const int fr = lane & 15, fq = lane >> 4;
  i32x8 af[4], bf0[2], bf1[2];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto readA = [&](int buf, int mh) {
    const uint32_t pa = lds0 + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag32(pa, mh * 128 + wm * 64 + i * 16 + fr, fq);
  };
  auto readB = [&](int buf, int nh, i32x8 (&bf)[2]) {
    const uint32_t pb = lds0 + buf * STAGE + PANEL;
#pragma unroll
    for (int j = 0; j < 2; ++j) bf[j] = frag32(pb, wn * 64 + nh * 32 + j * 16 + fr, fq);
  };
  auto mma = [&](int mh, int nh, const i32x8 (&bf)[2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[mh * 4 + i][nh * 2 + j] = mfma_fp8<FX>(bf[j], af[i], acc[mh * 4 + i][nh * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  const float dq = sa[0] * sb[0];
  float inv8 = 1.f, amax = 0.f;
  if constexpr (Q8) {
    hq_fp8_publish_scale(q8, phase, EPI == HQ_EPI_DMUL ? kHqBf8Max : kHqFp8Max);
    inv8 = 1.f / hq_fp8_delayed_scale(q8, phase, EPI == HQ_EPI_DMUL ? kHqBf8Max : kHqFp8Max);
  }

  int tile = id;
  HQ_DASSERT(tile < ntiles);   // the host launches min(tiles, CUs) workgroups
  int next = tile + nwg;
  __amdgpu_buffer_rsrc_t ca = rsrc_a(tile), cb = rsrc_b(tile);
  int p0 = 0;
  stA(ca, 0, 0, 0); stB(cb, 0, 0, 0); stB(cb, 1, 0, 0); stA(ca, 1, 0, 0);
  stA(ca, 0, 1, 1); stB(cb, 0, 1, 1); stB(cb, 1, 1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  bar();
  bool first = true;

  for (;;) {
    const bool last = next >= ntiles;
    const __amdgpu_buffer_rsrc_t na = rsrc_a(last ? tile : next), nb = rsrc_b(last ? tile : next);
    const int tm = tile / tiles_n, tn = tile % tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // two 32-MFMA phases per K-tile; stage / wait table and hazard argument: gemm.hip gemm_nt3_kernel
    auto ktile = [&](int t) {
      const bool more1 = t + 1 < nt || !last;
      const bool more2 = t + 2 < nt || (t + 2 == nt && !last);
      const bool prev2 = t + 1 < nt || (t + 1 == nt && !last);
      const int b0 = (p0 + t) & 1, b1 = b0 ^ 1;
      const bool x1 = t + 1 >= nt, x2 = t + 2 >= nt;
      const __amdgpu_buffer_rsrc_t a1 = x1 ? na : ca;
      const __amdgpu_buffer_rsrc_t a2 = x2 ? na : ca, b2r = x2 ? nb : cb;
      const int k1 = x1 ? t + 1 - nt : t + 1, k2 = x2 ? t + 2 - nt : t + 2;
      if (t == 0 && !first) {
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + E) : "memory");
      } else if (t == 0 || prev2) {
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      readB(b0, 0, bf0);
      readA(b0, 0);
      readB(b0, 1, bf1);
      if (more1) stA(a1, 1, k1, b1);
      bar();
      mma(0, 0, bf0);
      mma(0, 1, bf1);
      bar();
      // both wave rows (gemm.hip, gemm_nt3_kernel P23); at t = 0 of a following unit the epilogue's E vm ops
      // are younger too
      if (t == 0 && !first) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 + E) : "memory");
      else if (more1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      readA(b0, 1);
      if (more2) { stA(a2, 0, k2, b0); stB(b2r, 0, k2, b0); stB(b2r, 1, k2, b0); }
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
    const int bl = (p0 + nt - 1) & 1;
    char* wreg = wave < 7 ? smem + bl * STAGE + wave * REGION : smem + SPARE;

    // ---- epilogue, 64 local rows per round (acc · sa·sb (+bias) -> bf16 staging -> epi_piece)
    constexpr int SEGS = WN / 8, ROWS_PER_IT = 64 / SEGS;
    constexpr bool kBias = EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELUD;
    const int seg = lane % SEGS, rsub = lane / SEGS;
    const int gcol = n0 + wn * 64 + seg * 8;   // full 128-B lines per store (gemm.hip gemm_nt3_kernel)
    float csum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
#pragma unroll
    for (int rnd = 0; rnd < 2; ++rnd) {
#pragma unroll
      for (int J = 0; J < 4; ++J) {
        const int nh = J >> 1, j = J & 1;
        const int lc = nh * 32 + j * 16 + fq * 4;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (kBias) bv = *reinterpret_cast<const float4*>(bias + n0 + wn * 64 + nh * 32 + j * 16 + fq * 4);
#pragma unroll
        for (int I = 0; I < 4; ++I) {
          const f32x4_t& a = acc[rnd * 4 + I][J];
          float v[4] = {fmaf(a[0], dq, bv.x), fmaf(a[1], dq, bv.y), fmaf(a[2], dq, bv.z), fmaf(a[3], dq, bv.w)};
          *reinterpret_cast<uint2*>(wreg + (I * 16 + fr) * RS + lc * 2) = hq_pack4(v);
        }
      }
      auto goff_of = [&](int it) {   // it: 0..7 within this round
        const int lr = it * ROWS_PER_IT + rsub;
        return (size_t)(m0 + rnd * 128 + wm * 64 + lr) * ldc + gcol;
      };
      // aux pieces in batches of AB: all 8 at once (one exposed latency) spills the Q8 DMUL epilogue here
      constexpr int AB = (EPI == HQ_EPI_DMUL && Q8) ? 4 : 8;
#pragma unroll
      for (int h = 0; h < 8; h += AB) {
        uint4 aux[kAux ? AB : 1];
        if constexpr (kAux) {
#pragma unroll
          for (int it = 0; it < AB; ++it) aux[it] = load_aux<EPI, Q8>(P, goff_of(h + it));
        }
#pragma unroll
        for (int it = 0; it < AB; ++it) {
          const int lr = (h + it) * ROWS_PER_IT + rsub;
          const uint4 piece = *reinterpret_cast<const uint4*>(wreg + lr * RS + seg * 16);
          epi_piece<EPI, Q8, WC, GD8>(piece, aux[kAux ? it : 0], goff_of(h + it), C, P, C8, inv8, amax, csum);
        }
      }
    }
    if constexpr (EPI == HQ_EPI_DMUL) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        for (int o = SEGS; o < 64; o <<= 1) csum[e] += __shfl_xor(csum[e], o, 64);
      float* red = reinterpret_cast<float*>(smem + SPARE + REGION);  // [2][BN], by tile column
      if (rsub == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red[wm * BN + (gcol - n0) + e] = csum[e];
      }
      bar();
      for (int c = tid; c < BN; c += kThreads) part[(size_t)tm * N + n0 + c] = red[c] + red[BN + c];
    }
    if (last) break;
    // every wave has read its staging rounds out of buffer bl: stage the next tile's K-tile-1 halves there
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    stA(na, 0, 1, bl); stB(nb, 0, 1, bl); stB(nb, 1, 1, bl);
    tile = next;
    next = tile + nwg;
    ca = na;
    cb = nb;
    p0 = (p0 + nt) & 1;
    first = false;
  }
  if constexpr (Q8) {   // this wave's amax over all its tiles -> its partial slot
    amax = hq_wave_max(amax);
    if (lane == 0) part8[blockIdx.x * (kThreads / 64) + wave] = amax;
  }
}

constexpr size_t lds_bytes() {
  const size_t stage = 2 * (size_t)(2 * 256 * 128);
  const size_t epi = 8 * 128 * (size_t)(64 * 2 + 16);
  return stage > epi ? stage : epi;
}

// 0 = auto, 2 = always v2, 3 = always persistent (A/B, tests).  Auto = persistent, except the Q8 DMUL
// epilogue, whose e5m2 copy pushes the persistent kernel past 256 VGPRs (spills: 486 vs 408 µs as v2);
// persistent elsewhere measured 1.01-1.15x v2 on the b256 step shapes (tools/fp8_lab/fp8_variant_bench.py,
// profiles/r3_fp8_bwd).
int g_fp8_variant = 0;

template <int EPI, bool Q8, bool WC = true, bool GD8 = Q8>
void launch(const uint8_t* A, const uint8_t* B, uint16_t* C, const float* bias, uint16_t* P, const float* sa,
            const float* sb, uint8_t* C8, float* q8, float* part, int phase, int M, int N, int K, hipStream_t s) {
  const bool persist = g_fp8_variant == 3 || (g_fp8_variant == 0 && !(EPI == HQ_EPI_DMUL && Q8));
  if (persist) {
    constexpr size_t lds = 2 * (size_t)(2 * 256 * 128) + 64 * (64 * 2 + 16) + 2 * BN * 4;
    static int ncu = [] {
      int dev = 0, n = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipFuncSetAttribute((const void*)gemm_fp8p_kernel<EPI, Q8, WC, GD8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      return n > 0 ? n : 256;
    }();
    const int tiles = (M / BM) * (N / BN);
    const int nwg = std::min(tiles, ncu);   // every workgroup has at least one tile
    float* part8 = Q8 ? hq_fp8_amax_parts((size_t)nwg * (kThreads / 64), q8, s) : nullptr;
    hipLaunchKernelGGL((gemm_fp8p_kernel<EPI, Q8, WC, GD8>), dim3(nwg), dim3(kThreads), lds, s, A, B, C, bias, P, sa, sb, C8, q8,
                       part8, part, phase, M, N, K);
    if (Q8) hq_fp8_amax_fold(part8, nwg * (kThreads / 64), q8, phase, s, EPI == HQ_EPI_DMUL ? kHqBf8Max : kHqFp8Max);
    return;
  }
  constexpr size_t lds = lds_bytes();
  static bool init = [] {
    (void)hipFuncSetAttribute((const void*)gemm_fp8_kernel<EPI, Q8, WC, GD8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return true;
  }();
  (void)init;
  const int grid = (M / BM) * (N / BN);
  float* part8 = Q8 ? hq_fp8_amax_parts((size_t)grid * (kThreads / 64), q8, s) : nullptr;
  hipLaunchKernelGGL((gemm_fp8_kernel<EPI, Q8, WC, GD8>), dim3(grid), dim3(kThreads), lds, s, A, B, C, bias, P, sa, sb,
                     C8, q8, part8, part, phase, M, N, K, K, K, N);
  if (Q8) hq_fp8_amax_fold(part8, grid * (kThreads / 64), q8, phase, s, EPI == HQ_EPI_DMUL ? kHqBf8Max : kHqFp8Max);
}

// ------------------------------------------------------------------ delayed-scaling quantiser
// y = e4m3(x / s), s = 2·amax_prev/448 from state slot (phase+2)%3 (unit when unset); this call's amax
// into slot `phase`, slot (phase+1)%3 cleared, s stored in state[3].  One read of x instead of the
// current-scaling path's two.
__global__ __launch_bounds__(256) void quant_delayed_kernel(const uint16_t* __restrict__ x, uint2* __restrict__ y, size_t n8,
                                                            const float* __restrict__ q8, float* __restrict__ part,
                                                            int phase) {
  hq_fp8_publish_scale(q8, phase);
  const float s = delayed_scale(q8, phase);
  const float inv = 1.f / s;
  float m = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    float f[8];
    hq_unpack8(reinterpret_cast<const uint4*>(x)[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m = fmaxf(m, fabsf(f[k]));
      f[k] = fminf(fmaxf(f[k] * inv, -kFp8Max), kFp8Max);
    }
    uint32_t lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
    uint32_t hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
    y[i] = make_uint2(lo, hi);
  }
  m = hq_wave_max(m);
  if ((threadIdx.x & 63) == 0) part[blockIdx.x * 4 + (threadIdx.x >> 6)] = m;
}

// Every weight of the model in ONE launch (ParamStore.view_fp8 after each optimizer step): segment g is
// x[xo, xo + 8·n8) -> y[yo, …) under its own state states[g]; a block handles kQmBlk8 8-element groups
// of one segment (segment g owns blocks blk[g] … blk[g+1]-1).  Same math as quant_delayed_kernel; the
// per-block amax only reaches the atomic when it beats the slot's current value (monotonic, so a stale
// read costs at most a redundant atomic) — 48 launches of ~13 µs each become one bandwidth-bound pass.
constexpr int kQmBlk8 = 256 * 8;
__global__ __launch_bounds__(256) void quant_delayed_multi_kernel(const uint16_t* __restrict__ x, uint8_t* __restrict__ y,
                                                                  const long long* __restrict__ seg, int nseg,
                                                                  const float* __restrict__ states,
                                                                  float* __restrict__ part, int phase) {
  int g = 0;
  while (g + 1 < nseg && (long long)blockIdx.x >= seg[4 * (g + 1) + 3]) ++g;   // uniform scan, nseg <= ~100
  const long long xo = seg[4 * g], yo = seg[4 * g + 1], n8 = seg[4 * g + 2], b0 = seg[4 * g + 3];
  const float* q8 = states + 4 * g;
  const float s = delayed_scale(q8, phase);
  const float inv = 1.f / s;
  const uint4* xs = reinterpret_cast<const uint4*>(x + xo);
  uint2* ys = reinterpret_cast<uint2*>(y + yo);
  const long long i0 = ((long long)blockIdx.x - b0) * kQmBlk8;
  const long long i1 = i0 + kQmBlk8 < n8 ? i0 + kQmBlk8 : n8;
  float m = 0.f;
  for (long long i = i0 + threadIdx.x; i < i1; i += 256) {
    float f[8];
    hq_unpack8(xs[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m = fmaxf(m, fabsf(f[k]));
      f[k] = fminf(fmaxf(f[k] * inv, -kFp8Max), kFp8Max);
    }
    uint32_t lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
    uint32_t hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
    ys[i] = make_uint2(lo, hi);
  }
  m = hq_wave_max(m);
  if ((threadIdx.x & 63) == 0) part[blockIdx.x * 4 + (threadIdx.x >> 6)] = m;
}

// ------------------------------------------------------------------ amax fold
// The fp8 producers (LN forward, attention ctx store, FFN1 epilogue, the quantisers) write one amax per
// wave into a scratch array instead of atomics on the state word: tens of thousands of same-address
// atomics serialise in one L2 channel (measured: 36.9 K per-wave atomics turned a 236 µs attention
// forward into 967 µs).  This single-block kernel then folds the partials into slot `phase`, clears slot
// (phase+1)%3 and stores the scale the producer used in state[3] — segment g of a multi-segment call
// (blockIdx.x = g) folds partials [4·blk[g], 4·blk[g+1]).
__device__ __forceinline__ void amax_fold_segment(const float* __restrict__ part, long long i0, long long i1,
                                                  float* __restrict__ q8, int phase, float fmax) {
  // partial counts are multiples of 4 (4 or 8 waves per producer block): float4 loads, 4 in flight
  const float4* p4 = reinterpret_cast<const float4*>(part);
  const long long j0 = i0 >> 2, j1 = i1 >> 2;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
  long long j = j0 + threadIdx.x;
  for (; j + 3 * 1024 < j1; j += 4 * 1024) {
    const float4 v0 = p4[j], v1 = p4[j + 1024], v2 = p4[j + 2048], v3 = p4[j + 3072];
    a.x = fmaxf(fmaxf(a.x, v0.x), v1.x); a.y = fmaxf(fmaxf(a.y, v0.y), v1.y);
    a.z = fmaxf(fmaxf(a.z, v0.z), v1.z); a.w = fmaxf(fmaxf(a.w, v0.w), v1.w);
    c.x = fmaxf(fmaxf(c.x, v2.x), v3.x); c.y = fmaxf(fmaxf(c.y, v2.y), v3.y);
    c.z = fmaxf(fmaxf(c.z, v2.z), v3.z); c.w = fmaxf(fmaxf(c.w, v2.w), v3.w);
  }
  for (; j < j1; j += 1024) {
    const float4 v = p4[j];
    a.x = fmaxf(a.x, v.x); a.y = fmaxf(a.y, v.y); a.z = fmaxf(a.z, v.z); a.w = fmaxf(a.w, v.w);
  }
  float m = fmaxf(fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)), fmaxf(fmaxf(c.x, c.y), fmaxf(c.z, c.w)));
  m = hq_wave_max(m);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < 16; ++w) m = fmaxf(m, red[w]);   // m = red[0] here (thread 0's wave)
    unsigned* st = reinterpret_cast<unsigned*>(q8);
    const float s = hq_fp8_delayed_scale(q8, phase, fmax);   // 448 (e4m3) or 57344 (e5m2 gradients)
    st[phase] = __float_as_uint(fmaxf(__uint_as_float(st[phase]), m));
    st[(phase + 1) % 3] = 0u;   // cleared for the step after next's accumulation
    q8[3] = s;                  // dequant scale of this step's e4m3 output
  }
}

__global__ __launch_bounds__(1024) void amax_fold_kernel(const float* __restrict__ part, const long long* __restrict__ seg,
                                                         int nseg, long long nblk, int n, float* __restrict__ states,
                                                         int phase, float fmax) {
  const int g = blockIdx.x;
  long long i0 = 0, i1 = n;
  if (seg != nullptr) {
    i0 = 4 * seg[4 * g + 3];
    i1 = 4 * (g + 1 < nseg ? seg[4 * (g + 1) + 3] : nblk);
  }
  amax_fold_segment(part, i0, i1, states + 4 * g, phase, fmax);
}

// Deferred folds (hq_fp8_fold_defer): up to kFoldBatch sites' folds in ONE launch, block g = site g — the ~97
// per-site single-block launches of an fp8 training step (~5 µs each, mostly launch and drain) become a handful.
struct FoldSeg {
  const float* part;
  float* q8;
  int n, phase;
  float fmax;
  int pad;
};
constexpr int kFoldBatch = 32;
struct FoldBatch {
  FoldSeg s[kFoldBatch];
};
__global__ __launch_bounds__(1024) void amax_fold_batch_kernel(FoldBatch b) {
  const FoldSeg& g = b.s[blockIdx.x];
  amax_fold_segment(g.part, 0, g.n, g.q8, g.phase, g.fmax);
}

// Per-device deferral state: partial slots come from one arena, bump-allocated and reset when the pending folds are
// launched, so every pending site keeps its own partials until its fold has read them.
struct FoldDefer {
  bool on = false;
  float* arena = nullptr;
  size_t cap = 0, used = 0;
  hipStream_t stream = nullptr;
  std::vector<FoldSeg> pending;
};
constexpr size_t kFoldArena = size_t(8) << 20;   // floats (32 MiB): a BERT-large step's partials with room to spare
FoldDefer& fold_defer() {
  static std::vector<FoldDefer> st;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if ((int)st.size() <= dev) st.resize(dev + 1);
  return st[dev];
}

void fold_flush(FoldDefer& d) {
  for (size_t i = 0; i < d.pending.size(); i += kFoldBatch) {
    FoldBatch b{};
    const int n = (int)std::min<size_t>(kFoldBatch, d.pending.size() - i);
    for (int j = 0; j < n; ++j) b.s[j] = d.pending[i + j];
    hipLaunchKernelGGL(amax_fold_batch_kernel, dim3(n), dim3(1024), 0, d.stream, b);
  }
  d.pending.clear();
  d.used = 0;   // stream order: the folds above read the arena before any later producer on d.stream writes it
}

}  // namespace

long long hq_fp8_quant_multi_blocks(long long n8) { return (n8 + kQmBlk8 - 1) / kQmBlk8; }

void hq_fp8_quant_delayed_multi(const uint16_t* x, uint8_t* y, const long long* seg, int nseg, long long blocks,
                                float* states, int phase, hipStream_t s) {
  if (blocks <= 0 || nseg <= 0) return;
  float* part = hq_fp8_amax_parts((size_t)blocks * 4);
  hipLaunchKernelGGL(quant_delayed_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, y, seg, nseg, states, part,
                     phase);
  hipLaunchKernelGGL(amax_fold_kernel, dim3(nseg), dim3(1024), 0, s, part, seg, nseg, blocks, 0, states, phase, kFp8Max);
}

float* hq_fp8_amax_parts(size_t n, const float* q8, hipStream_t s) {
  FoldDefer& d = fold_defer();
  if (d.on && q8 != nullptr) {
    // a site whose previous production still has a pending fold (its next scale reads that fold's slot), or a
    // producer on another stream (unordered against the pending folds' partials): launch the pending folds first
    bool flush = !d.pending.empty() && s != d.stream;
    for (const FoldSeg& g : d.pending) flush = flush || g.q8 == q8;
    const size_t n4 = (n + 3) & ~size_t(3);
    if (flush || d.used + n4 > d.cap) fold_flush(d);
    if (n4 <= d.cap) {
      float* p = d.arena + d.used;
      d.used += n4;
      d.stream = s;
      return p;
    }
  }
  // immediate mode: per-device scratch, grown on demand and never freed while kernels may still read it (the old
  // block is kept: a grow happens a handful of times per process).  Producers and their fold share one stream.
  static std::vector<std::pair<float*, size_t>> bufs;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if ((int)bufs.size() <= dev) bufs.resize(dev + 1, {nullptr, 0});
  auto& b = bufs[dev];
  if (b.second < n) {
    const size_t cap = std::max<size_t>(n, 1 << 18);
    float* p = nullptr;
    if (hipMalloc(&p, cap * sizeof(float)) != hipSuccess) { fprintf(stderr, "hq_fp8_amax_parts: hipMalloc failed\n"); abort(); }
    b = {p, cap};
  }
  return b.first;
}

void hq_fp8_amax_fold(const float* part, int n, float* q8, int phase, hipStream_t s, float fmax) {
  if (n % 4 != 0) { fprintf(stderr, "hq_fp8_amax_fold: %d partials (must be a multiple of 4)\n", n); abort(); }
  FoldDefer& d = fold_defer();
  if (d.on && part >= d.arena && part < d.arena + d.cap && s == d.stream) {
    d.pending.push_back(FoldSeg{part, q8, n, phase, fmax, 0});
    return;
  }
  hipLaunchKernelGGL(amax_fold_kernel, dim3(1), dim3(1024), 0, s, part, nullptr, 1, 0LL, n, q8, phase, fmax);
}

void hq_fp8_fold_flush() { fold_flush(fold_defer()); }

int hq_fp8_fold_defer(int on) {
  FoldDefer& d = fold_defer();
  if (!on) {
    fold_flush(d);
    d.on = false;
    return 0;
  }
  if (d.arena == nullptr) {   // allocated once, outside any graph capture (the first deferred step is eager)
    if (hipMalloc(&d.arena, kFoldArena * sizeof(float)) != hipSuccess) {
      fprintf(stderr, "hq_fp8_fold_defer: hipMalloc failed\n");
      abort();
    }
    d.cap = kFoldArena;
  }
  d.on = true;
  return 0;
}

int hq_fp8_fold_pending() { return (int)fold_defer().pending.size(); }

void hq_gemm_fp8_set_variant(int v) { g_fp8_variant = v; }

int hq_gemm_fp8_supported(int M, int N, int K) {
  return (M % BM == 0 && N % BN == 0 && K % BK == 0 && K >= 2 * BK && (size_t)BM * K < (1ull << 31) &&
          (size_t)BN * K < (1ull << 31)) ? 1 : 0;
}

void hq_gemm_fp8(const uint8_t* A, const uint8_t* B, uint16_t* C, const float* bias, uint16_t* P, const float* sa,
                 const float* sb, uint8_t* C8, float* q8, int phase, int M, int N, int K, int epi, hipStream_t s,
                 float* part, int gd8) {
  switch (epi) {
    case HQ_EPI_GELUD:
      // gd8 = 0: gelu' in bf16 beside the e4m3 act (the FFN2 dgrad runs in bf16 and would otherwise decode the code)
      if (C8 && C && !gd8) launch<HQ_EPI_GELUD, true, true, false>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s);
      else if (C8 && C) launch<HQ_EPI_GELUD, true>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s);
      else if (C8) launch<HQ_EPI_GELUD, true, false>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s);
      else launch<HQ_EPI_GELUD, false>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s);
      break;
    case HQ_EPI_DMUL:
      if (C8 && C) launch<HQ_EPI_DMUL, true>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s);
      else if (C8) launch<HQ_EPI_DMUL, true, false>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s);
      else launch<HQ_EPI_DMUL, false>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s);
      break;
    case HQ_EPI_NONE: launch<HQ_EPI_NONE, false>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s); break;
    case HQ_EPI_RESID: launch<HQ_EPI_RESID, false>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s); break;
    default: launch<HQ_EPI_BIAS, false>(A, B, C, bias, P, sa, sb, C8, q8, part, phase, M, N, K, s); break;
  }
}

void hq_fp8_quant_delayed(const uint16_t* x, uint8_t* y, size_t n, float* q8, int phase, hipStream_t s) {
  const size_t n8 = n / 8;
  const int grid = std::max(1, (int)std::min<size_t>((n8 + 255) / 256, 256 * 8));
  float* part = hq_fp8_amax_parts((size_t)grid * 4, q8, s);
  hipLaunchKernelGGL(quant_delayed_kernel, dim3(grid), dim3(256), 0, s, x, reinterpret_cast<uint2*>(y), n8, q8, part,
                     phase);
  hq_fp8_amax_fold(part, grid * 4, q8, phase, s);
}
