// bf16 "NT" GEMM for gfx950 with fused epilogues:  C[M,N] = A[M,K] · B[N,K]ᵀ  (+ epilogue)
//
// Both operands are K-contiguous row-major — the layout of every BERT projection in the forward
// (x · Wᵀ) and, with the transposed bf16 weight copy kept by the ParamStore, of every dgrad
// (dy · W = dy · (Wᵀ)ᵀ).  Epilogues fuse what used to be separate HBM passes:
//   EPI_NONE   C = acc
//   EPI_BIAS   C = acc + bias[n]
//   EPI_GELU   P = acc + bias[n] (stored, needed by backward),  C = gelu_erf(P)
//   EPI_DGELU  C = acc · gelu'(P[m,n])  and per-block column sums of C (the bias gradient of the
//              producing Linear) into part[M/BM][N]  — replaces the separate gelu_bwd pass
//   EPI_RESID  C = acc + R[m,n]  (residual-gradient add of dgrad)
//   EPI_GELUD  as EPI_GELU but P receives gelu'(pre) instead of pre: the forward already evaluates
//              Φ and φ, so the derivative costs one FMA here and saves the backward ~15 VALU/element
//   EPI_DMUL   C = acc · P[m,n] (P = stored gelu') + column partials — the backward of EPI_GELUD
//
// Structure (CDNA4 playbook §5):
// * 256×BN block tile, BK = 64, 512 threads = 8 waves as 2 (M) × 4 (N); a wave owns 128 × BN/4.
// * Operands reach LDS by LDS-DMA (global_load_lds, 16 B per lane): the image is lane-linear, so the
//   bank-conflict XOR swizzle is applied to the per-lane global SOURCE address and undone on the
//   ds_read_b128 fragment read (rule 21).  Rows are 128 B; slot' = slot ^ ((row >> 1) & 7) makes the
//   16-lane fragment reads of 16 rows hit all 64 banks once.
// * Double-buffered ring: tile t+1 is issued before tile t is consumed; a COUNTED s_waitcnt vmcnt
//   (never 0 inside the loop) retires tile t, then a raw s_barrier (no __syncthreads: its fence would
//   drain the DMA in flight).  One __shared__ array for everything (trap 4a).
// * mfma_f32_16x16x32_bf16 with the operands SWAPPED (B fragment as the MFMA's A input) so the
//   accumulator holds Cᵀ: each lane owns 4 consecutive n of one m → 8-byte row-contiguous stores,
//   a float4 of bias per lane, and the column (bias-grad) sums reduce over lanes.
// * XCD-aware bijective block remap: each XCD walks a contiguous range of tiles in M-major order,
//   so the tiles that share an A row-panel share that XCD's L2.
#include <mutex>
#include <type_traits>
#include <vector>

#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int BM = 256;
constexpr int BK = 64;
constexpr int kThreads = 512;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float gelu_erf(float x) { return hq_gelu(x); }
__device__ __forceinline__ float gelu_grad(float x) { return hq_gelu_grad(x); }

// Issue the LDS-DMA of one [ROWS × 64] bf16 panel (rows of 128 B) into lds (+ byte offset).
// Each wave-instruction moves 8 rows (64 lanes × 16 B); this wave handles `n_instr` of them
// starting at panel row `row0`.
template <int N_INSTR>
__device__ __forceinline__ void stage_panel(const uint16_t* __restrict__ g, int ld, int row0, int k0, char* lds_base,
                                            int lane) {
  const int r_in = lane >> 3;          // 0..7 row within the 8-row piece
  const int slot = lane & 7;           // 16-B slot in the 128-B LDS row (lane-linear destination)
#pragma unroll
  for (int i = 0; i < N_INSTR; ++i) {
    const int row = row0 + i * 8 + r_in;
    const int src_slot = slot ^ ((row >> 1) & 7);
    const uint16_t* src = g + (size_t)row * ld + k0 + src_slot * 8;
    char* dst = lds_base + (size_t)(row0 + i * 8) * 128;  // wave-uniform; lane L lands at dst + 16 L
    __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)dst, 16, 0, 0);
  }
}

// 16-B fragment read of LDS row `row`, k-slot `slot` (8 bf16 = 16 B), undoing the source swizzle.
__device__ __forceinline__ bf16x8_t frag(const char* panel, int row, int slot) {
  const int off = row * 128 + ((slot ^ ((row >> 1) & 7)) << 4);
  return *reinterpret_cast<const bf16x8_t*>(panel + off);
}

template <int EPI, int BN>
__global__ __launch_bounds__(kThreads, 1) void gemm_nt_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                              uint16_t* __restrict__ C, const float* __restrict__ bias,
                                                              uint16_t* __restrict__ P, const uint16_t* __restrict__ R,
                                                              float* __restrict__ part, int M, int N, int K, int lda,
                                                              int ldb, int ldc, HqDropArg dr) {
  const uint32_t key = EPI == HQ_EPI_BDR ? dr.kd.get() : 0u;   // EPI_BDR dropout key (device seed word under graphs)
  constexpr int WN = BN / 4;            // columns per wave
  constexpr int NJ = WN / 16;           // 16-wide n subtiles per wave
  constexpr int MI = 8;                 // 16-high m subtiles per wave (128 rows)
  constexpr int A_BYTES = BM * 128;     // one A panel (256 × 64 bf16)
  constexpr int B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;

  // ---- bijective XCD remap of the linear block id, then M-major tile order within an XCD
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_n = N / BN;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  HQ_DASSERT(m0 + BM <= M && n0 + BN <= N && K % BK == 0);

  const uint16_t* Ab = A + (size_t)m0 * lda;
  const uint16_t* Bb = B + (size_t)n0 * ldb;
  const int nt = K / BK;

  // staging split: A panel = 32 pieces of 8 rows (4 per wave); B panel = BN/8 pieces (BN/64 per wave)
  constexpr int A_INSTR = BM / 8 / 8;
  constexpr int B_INSTR = BN / 8 / 8;
  constexpr int LOADS_PER_TILE = A_INSTR + B_INSTR;

  f32x4_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int t, int buf) {
    char* base = smem + buf * STAGE;
    stage_panel<A_INSTR>(Ab, lda, wave * (BM / 8), t * BK, base, lane);
    stage_panel<B_INSTR>(Bb, ldb, wave * (BN / 8), t * BK, base + A_BYTES, lane);
  };

  const int fr = lane & 15;           // fragment row within a 16-row subtile
  const int fq = lane >> 4;           // k-slot quarter (8 bf16 each) within a 32-wide k step
  bf16x8_t bf[NJ], af[MI];
  auto read_frags = [&](int t, int ks) {   // R phase: this wave's fragments of k-step ks of tile t
    const char* pa = smem + (t & 1) * STAGE;
    const char* pb = pa + A_BYTES;
#pragma unroll
    for (int j = 0; j < NJ; ++j) bf[j] = frag(pb, wn * WN + j * 16 + fr, ks * 4 + fq);
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = frag(pa, wm * 128 + i * 16 + fr, ks * 4 + fq);
  };
  auto mfma_block = [&]() {               // M phase
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() { __builtin_amdgcn_s_barrier(); };
  auto drain = []() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  // Two wave groups (wm = 0: waves 0-3, wm = 1: waves 4-7; a SIMD hosts one wave of each) run the
  // same R/M phase sequence offset by one workgroup barrier, so on every SIMD one wave reads its
  // LDS fragments while the other issues MFMAs.  Group 1 starts with an extra barrier, group 0 ends
  // with one.  Barrier k of group 0 pairs with barrier k of group 1 (one phase later in its program):
  //   RAW: every wave drains its LDS-DMA of tile t before the barrier that precedes the first read of
  //   tile t by either group; WAR: a tile-(t+1) DMA into buffer (t+1)&1 is issued only after the
  //   barrier that follows the other group's last read of tile t-1.
  stage(0, 0);
  drain();
  bar();
  if (__builtin_amdgcn_readfirstlane(wm) == 0) {
    for (int t = 0; t < nt; ++t) {
      if (t + 1 < nt) stage(t + 1, (t + 1) & 1);
      read_frags(t, 0);
      bar();
      mfma_block();
      bar();
      read_frags(t, 1);
      bar();
      mfma_block();
      drain();
      bar();
    }
    bar();
  } else {
    bar();
    for (int t = 0; t < nt; ++t) {
      if (t + 1 < nt) stage(t + 1, (t + 1) & 1);
      read_frags(t, 0);
      bar();
      mfma_block();
      bar();
      read_frags(t, 1);
      drain();
      bar();
      mfma_block();
      bar();
    }
  }
  (void)LOADS_PER_TILE;

  // ---- epilogue, phase 1: acc (+bias) -> bf16 into this wave's private LDS region [128][WN]
  // (row stride WN*2+16 B keeps the 16-row ds_write_b64 groups at most 2-way and rows 16-B aligned).
  // The last loop barrier guarantees every wave is done reading the A/B panels.
  constexpr int RS = WN * 2 + 16;
  char* wreg = smem + wave * (128 * RS);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nl = j * 16 + fq * 4;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD || EPI == HQ_EPI_BDR) bv = *reinterpret_cast<const float4*>(bias + n0 + wn * WN + nl);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float v[4] = {acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w};
      *reinterpret_cast<uint2*>(wreg + (i * 16 + fr) * RS + nl * 2) = hq_pack4(v);
    }
  }
  // ---- phase 2: row-coalesced 16-B pieces (8 columns) -> epilogue math -> 16-B global stores
  constexpr int SEGS = WN / 8;                  // 16-B pieces per row of the wave tile
  constexpr int ROWS_PER_IT = 64 / SEGS;
  const int seg = lane % SEGS, rsub = lane / SEGS;
  const int mb = m0 + wm * 128, nb = n0 + wn * WN + seg * 8;
  float csum[8];
  if constexpr (EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL) {
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  }
#pragma unroll 4
  for (int it = 0; it < 128 / ROWS_PER_IT; ++it) {
    const int row = it * ROWS_PER_IT + rsub;
    uint4 piece = *reinterpret_cast<const uint4*>(wreg + row * RS + seg * 16);
    const size_t goff = (size_t)(mb + row) * ldc + nb;
    if constexpr (EPI == HQ_EPI_GELU) {
      *reinterpret_cast<uint4*>(P + goff) = piece;   // pre-activation (bf16), kept for backward
      float x[8];
      hq_unpack8(piece, x);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = gelu_erf(x[e]);
      piece = hq_pack8(x);
    } else if constexpr (EPI == HQ_EPI_GELUD) {
      float x[8], g[8];
      hq_unpack8(piece, x);
      hq_gelu_grad8(x, g);   // g = gelu'(x), x = gelu(x)
      *reinterpret_cast<uint4*>(P + goff) = hq_pack8(g);
      piece = hq_pack8(x);
    } else if constexpr (EPI == HQ_EPI_DMUL) {
      float d[8], gd[8];
      hq_unpack8(piece, d);
      hq_unpack8(*reinterpret_cast<const uint4*>(P + goff), gd);
#pragma unroll
      for (int e = 0; e < 8; ++e) { d[e] *= gd[e]; csum[e] += d[e]; }
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_DGELU) {
      float d[8], pr[8];
      hq_unpack8(piece, d);
      hq_unpack8(*reinterpret_cast<const uint4*>(P + goff), pr);
#pragma unroll
      for (int e = 0; e < 8; ++e) { d[e] *= gelu_grad(pr[e]); csum[e] += d[e]; }
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_RESID) {
      float d[8], rr[8];
      hq_unpack8(piece, d);
      hq_unpack8(*reinterpret_cast<const uint4*>(R + goff), rr);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] += rr[e];
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_BDR) {
      piece = hq_epi_bdr8(piece, *reinterpret_cast<const uint4*>(R + goff), (uint32_t)goff, dr, key);
    }
    *reinterpret_cast<uint4*>(C + goff) = piece;
  }
  if constexpr (EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL) {
    // column sums: lanes with equal `seg` hold the same 8 columns -> xor-reduce over rsub, then the
    // two M-waves through LDS (after everyone is done with its staging region)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      for (int o = SEGS; o < 64; o <<= 1) csum[e] += __shfl_xor(csum[e], o, 64);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [2][BN]
    if (rsub == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wm * BN + wn * WN + seg * 8 + e] = csum[e];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += kThreads) part[(size_t)tm * N + n0 + c] = red[c] + red[BN + c];
  }
}


// ============================================================================================
// vS — 128×128 tiles for the shapes the 256-row kernels do not cover well: M % 256 != 0 (dynamically
// padded NQ batches, the reference micro-batch of 2 × 512 tokens) and grids that fill the 256 CUs
// poorly with 256² tiles (batch 64: N = 768 gives 288 tiles = 1.1 waves).  4 waves (2 M × 2 N, 64×64
// each), two 32 KiB LDS-DMA stages (buffer_load … lds, same source swizzle as the big kernels), so two
// workgroups share a CU.  The M tail costs nothing extra: the A descriptor's num_records ends at row M,
// the out-of-range rows stage as zeros, and the epilogue stores only rows < M.  Same epilogues as v1;
// DGELU / DMUL column partials are per 128-row block (part has ceil(M/128) rows).
// Split-K (ksplit > 1, EPI none / bias / resid only): for grids far below one workgroup per CU with a long
// K (the reference micro-batch of 2 × 512 tokens: 48 tiles of N = 768 at K = 3072 / 2304), workgroup
// id / tiles sums K-tiles [split·nt/ksplit, (split+1)·nt/ksplit) into fp32 slab ws[split] and
// splitk_epi_kernel folds the slabs in order (deterministic) and applies the epilogue.
template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nts_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                          uint16_t* __restrict__ C, const float* __restrict__ bias,
                                                          uint16_t* __restrict__ P, const uint16_t* __restrict__ R,
                                                          float* __restrict__ part, int M, int N, int K, int lda, int ldb,
                                                          int ldc, int ksplit, float* __restrict__ ws, HqDropArg dr) {
  const uint32_t key = EPI == HQ_EPI_BDR ? dr.kd.get() : 0u;   // EPI_BDR dropout key (device seed word under graphs)
  constexpr int SB = 128;                  // tile rows = tile cols
  constexpr int PANEL = SB * 128;          // one operand panel: 128 rows × 64 bf16
  constexpr int STAGE = 2 * PANEL;
  constexpr int RS = 64 * 2 + 16;          // epilogue staging row stride (bytes)
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave >> 1, wn = wave & 1;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles = nwg / ksplit;
  const int split = id / tiles, tile = id - split * tiles;
  const int tiles_n = N / SB;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * SB, n0 = tn * SB;
  const int rows_a = min(SB, M - m0);
  const int nk = K / BK, kt0 = split * nk / ksplit, nt = (split + 1) * nk / ksplit - kt0;
  HQ_DASSERT(rows_a > 0 && n0 + SB <= N && K % BK == 0 && nt > 0 && (ksplit == 1 || EPI == HQ_EPI_NONE ||
             EPI == HQ_EPI_BIAS || EPI == HQ_EPI_RESID));

  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * lda), (short)0, rows_a * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(B + (size_t)n0 * ldb), (short)0, SB * ldb * 2, 0x00020000);
  int voA[4], voB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 32 + i * 8 + (lane >> 3);
    const int src_slot = (lane & 7) ^ ((row >> 1) & 7);
    voA[i] = (row * lda + src_slot * 8) * 2;
    voB[i] = (row * ldb + src_slot * 8) * 2;
  }
  auto stage = [&](int t, int buf) {
    char* base = smem + buf * STAGE + wave_u * 32 * 128;
    const int ko = (kt0 + t) * BK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(base + i * 8 * 128), 16, voA[i], ko, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(base + PANEL + i * 8 * 128), 16, voB[i], ko, 0, 0);
  };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  stage(0, 0);
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) {
      stage(t + 1, (t + 1) & 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // this wave's 8 pieces of stage t landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();                                               // ... and every other wave's
    const char* pa = smem + (t & 1) * STAGE;
    const char* pb = pa + PANEL;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[4], bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = frag(pb, wn * 64 + j * 16 + fr, ks * 4 + fq);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag(pa, wm * 64 + i * 16 + fr, ks * 4 + fq);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();                                               // WAR: stage t+2 reuses this buffer
  }

  if (ksplit > 1) {   // fp32 slab of this split: lane holds C[m][n … n+3] (swapped-operand accumulator)
    float* slab = ws + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4_t& a = acc[i][j];
        *reinterpret_cast<float4*>(slab + (size_t)m * N + n0 + wn * 64 + j * 16 + fq * 4) =
            make_float4(a[0], a[1], a[2], a[3]);
      }
    }
    return;
  }

  // ---- epilogue: acc (+bias) -> bf16 in this wave's LDS region [64][64], then row-coalesced 16-B pieces
  char* wreg = smem + wave * 64 * RS;
  constexpr bool kBias = EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD || EPI == HQ_EPI_BDR;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nl = j * 16 + fq * 4;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (kBias) bv = *reinterpret_cast<const float4*>(bias + n0 + wn * 64 + nl);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4] = {acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w};
      *reinterpret_cast<uint2*>(wreg + (i * 16 + fr) * RS + nl * 2) = hq_pack4(v);
    }
  }
  constexpr int SEGS = 8, ROWS_PER_IT = 64 / SEGS;
  const int seg = lane % SEGS, rsub = lane / SEGS;
  const int gcol = n0 + wn * 64 + seg * 8;
  float csum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) csum[e] = 0.f;
#pragma unroll 2
  for (int it = 0; it < 64 / ROWS_PER_IT; ++it) {
    const int row = it * ROWS_PER_IT + rsub;
    const int grow = m0 + wm * 64 + row;
    if (grow >= M) continue;
    uint4 piece = *reinterpret_cast<const uint4*>(wreg + row * RS + seg * 16);
    const size_t goff = (size_t)grow * ldc + gcol;
    if constexpr (EPI == HQ_EPI_GELU) {
      *reinterpret_cast<uint4*>(P + goff) = piece;
      float x[8];
      hq_unpack8(piece, x);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = gelu_erf(x[e]);
      piece = hq_pack8(x);
    } else if constexpr (EPI == HQ_EPI_GELUD) {
      float x[8], g[8];
      hq_unpack8(piece, x);
      hq_gelu_grad8(x, g);   // g = gelu'(x), x = gelu(x)
      *reinterpret_cast<uint4*>(P + goff) = hq_pack8(g);
      piece = hq_pack8(x);
    } else if constexpr (EPI == HQ_EPI_DMUL) {
      float d[8], gd[8];
      hq_unpack8(piece, d);
      hq_unpack8(*reinterpret_cast<const uint4*>(P + goff), gd);
#pragma unroll
      for (int e = 0; e < 8; ++e) { d[e] *= gd[e]; csum[e] += d[e]; }
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_DGELU) {
      float d[8], pr[8];
      hq_unpack8(piece, d);
      hq_unpack8(*reinterpret_cast<const uint4*>(P + goff), pr);
#pragma unroll
      for (int e = 0; e < 8; ++e) { d[e] *= gelu_grad(pr[e]); csum[e] += d[e]; }
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_RESID) {
      float d[8], rr[8];
      hq_unpack8(piece, d);
      hq_unpack8(*reinterpret_cast<const uint4*>(R + goff), rr);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] += rr[e];
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_BDR) {
      piece = hq_epi_bdr8(piece, *reinterpret_cast<const uint4*>(R + goff), (uint32_t)goff, dr, key);
    }
    *reinterpret_cast<uint4*>(C + goff) = piece;
  }
  if constexpr (EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      for (int o = SEGS; o < 64; o <<= 1) csum[e] += __shfl_xor(csum[e], o, 64);
    float* red = reinterpret_cast<float*>(smem + 4 * 64 * RS);  // [2][128], past the staging regions
    if (rsub == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wm * SB + wn * 64 + seg * 8 + e] = csum[e];
    }
    __syncthreads();
    if (tid < SB) part[(size_t)tm * N + n0 + tid] = red[tid] + red[SB + tid];
  }
}

// C[m, n] = epi(Σ_s ws[s][m][n]) for the split-K vS path: slabs summed in split order (deterministic).
template <int EPI>
__global__ __launch_bounds__(256) void splitk_epi_kernel(const float* __restrict__ ws, int ksplit, uint16_t* __restrict__ C,
                                                         const float* __restrict__ bias, const uint16_t* __restrict__ R,
                                                         int M, int N, int ldc) {
  const size_t n8 = (size_t)M * N / 8;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    const size_t e = i * 8;
    const int m = (int)(e / N), n = (int)(e - (size_t)m * N);
    float v[8];
    const float4* w0 = reinterpret_cast<const float4*>(ws + e);
    float4 a = w0[0], b = w0[1];
    for (int s = 1; s < ksplit; ++s) {
      const float4* ws_s = reinterpret_cast<const float4*>(ws + (size_t)s * M * N + e);
      const float4 c = ws_s[0], d = ws_s[1];
      a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
      b.x += d.x; b.y += d.y; b.z += d.z; b.w += d.w;
    }
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    if constexpr (EPI == HQ_EPI_BIAS) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + n), b1 = *reinterpret_cast<const float4*>(bias + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    } else if constexpr (EPI == HQ_EPI_RESID) {
      float rr[8];
      hq_unpack8(*reinterpret_cast<const uint4*>(R + (size_t)m * ldc + n), rr);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += rr[k];
    }
    *reinterpret_cast<uint4*>(C + (size_t)m * ldc + n) = hq_pack8(v);
  }
}

// ============================================================================================
// v2 — deep LDS-DMA pipeline (CDNA4 playbook §5 "8-phase" structure, re-derived for this tile).
//
// Same 256×256×64 tile, 8 waves, swizzle and swapped-operand MFMA as v1, but the K-tile is split
// into FOUR phases of 16 MFMAs per wave and the staging into four 16 KiB "halves" (128 rows of
// the A or B panel, 2 LDS-DMA instructions per thread), ONE half issued per phase, so three
// halves stay in flight across every barrier (counted vmcnt(6), never 0 in the steady state)
// instead of v1's whole-tile issue + vmcnt(0) drain per K-tile.
//
// Wave (wm, wn) owns four 64×32 quadrants (mh, nh): rows mh·128 + wm·64 + [0,64),
// cols nh·128 + wn·32 + [0,32) — so quadrant (mh, nh) reads exactly A-half mh and B-half nh.
//   phase  quadrant  LDS reads (ds_read_b128)   stage issued          wait (vmcnt 6) retires
//   P0     (0,0)     A0 (8) + B0 (4)            B1(t+1)               B1(t)
//   P1     (0,1)     B1 (4)                     A1(t+1)               A1(t)
//   P2     (1,1)     A1 (8)                     A0(t+2)               —
//   P3     (1,0)     — (B0 kept in registers)   B0(t+2)               A0(t+1), B0(t+1)
// Hazards (two wave groups staggered by one barrier, two barriers per phase): a slot is
// restaged ≥ 2 phases after its last read (WAR) and read ≥ 1 phase after the wait that retires
// it (RAW); the table satisfies both (3/3/2/3 phases and 4-5 phases of load latency hiding).
// Tail tiles skip the stages past the end and use the exact smaller vmcnt.
// ABL (tools/gemm_lab only; production = 0): bit0 skip the in-loop LDS-DMA stages, bit1 skip the
// in-loop fragment reads, bit2 run both wave groups in lockstep (no stagger barrier), bit3 stage
// with buffer_load … lds (SRD + precomputed per-lane offsets) instead of global_load_lds, bit4
// grouped tile order (8 row panels × all column panels per group).
template <int EPI, int ABL = 0>
__global__ __launch_bounds__(kThreads, 1) void gemm_nt2_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                               uint16_t* __restrict__ C, const float* __restrict__ bias,
                                                               uint16_t* __restrict__ P, const uint16_t* __restrict__ R,
                                                               float* __restrict__ part, int M, int N, int K, int lda,
                                                               int ldb, int ldc, HqDropArg dr) {
  const uint32_t key = EPI == HQ_EPI_BDR ? dr.kd.get() : 0u;   // EPI_BDR dropout key (device seed word under graphs)
  constexpr int BN = 256;
  constexpr int PANEL = 256 * 128;      // one A or B panel (256 rows × 64 bf16)
  constexpr int HALF = 128 * 128;       // 128 rows of a panel
  constexpr int STAGE = 2 * PANEL;      // A panel then B panel
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int tiles_n = N / BN;
  // Half-tile tail (as v3's; production buffer-load form, ungrouped order only): the host launches rt blocks
  // more than there are tiles when the last wave of tiles would be at most half full; blocks F … nwg-1,
  // dispatched last, run the last rt tiles as 2·rt 128-row halves.
  constexpr bool kHalfOK = !(EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL) && (ABL & 8) != 0 && (ABL & 16) == 0;
  const int ntiles = (M / BM) * tiles_n;
  const int rt = kHalfOK ? nwg - ntiles : 0;
  const int F = nwg - 2 * rt;                    // full-tile blocks (= ntiles - rt)
  const bool half = rt > 0 && bid >= F;
  const int nfull = rt > 0 ? F : nwg;
  const int xcd = bid & 7, q = nfull >> 3, r = nfull & 7;
  const int tile = half ? F + ((bid - F) >> 1) : (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int tm = tile / tiles_n, tn = tile % tiles_n;
  if constexpr ((ABL & 16) != 0) {
    constexpr int GM = 8;
    const int tiles_m = M / BM, per = GM * tiles_n;
    const int first = (tile / per) * GM, gsz = min(tiles_m - first, GM), in = tile % per;
    tm = first + in % gsz;
    tn = in / gsz;
  }
  const int m0 = tm * BM + (half ? ((bid - F) & 1) * 128 : 0), n0 = tn * BN;
  HQ_DASSERT(m0 + (half ? 128 : BM) <= M && n0 + BN <= N && K % BK == 0 && K >= 2 * BK);

  const uint16_t* Ab = A + (size_t)m0 * lda;
  const uint16_t* Bb = B + (size_t)n0 * ldb;
  const int nt = K / BK;

  // one half = 16 pieces of 8 rows; wave w stages rows w·16 .. w·16+15 of it (2 instructions)
  auto stage_half = [&](const uint16_t* g, int ld, int half, int t, char* panel) {
    stage_panel<2>(g, ld, half * 128 + wave * 16, t * BK, panel, lane);
  };
  // buffer-load staging: SRDs over the block's A / B row panels; the per-lane byte offsets of the two
  // 8-row pieces a wave stages are the same for every half and K-tile (the swizzle depends on row
  // bits 1..3 only), so the K-tile and half advance lives in the scalar soffset.
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  // (a last half tile's panel ends at row M: its unread second 128 rows load as zeros)
  __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, min(BM, M - m0) * lda * 2, 0x00020000);
  __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, BN * ldb * 2, 0x00020000);
  int voA[2], voB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + (lane >> 3);
    const int src_slot = (lane & 7) ^ ((row >> 1) & 7);
    voA[i] = (row * lda + src_slot * 8) * 2;
    voB[i] = (row * ldb + src_slot * 8) * 2;
  }
  auto buf_half = [&](__amdgpu_buffer_rsrc_t rs, const int (&vo)[2], int ld, int half, int t, char* panel) {
    char* dst = panel + (half * 128 + wave_u * 16) * 128;
    const int so = half * 128 * ld * 2 + t * BK * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 8 * 128), 16, vo[i], so, 0, 0);
  };
  auto stA = [&](int half, int t) {
    if constexpr ((ABL & 1) != 0) return;
    if constexpr ((ABL & 8) != 0) buf_half(rA, voA, lda, half, t, smem + (t & 1) * STAGE);
    else stage_half(Ab, lda, half, t, smem + (t & 1) * STAGE);
  };
  auto stB = [&](int half, int t) {
    if constexpr ((ABL & 1) != 0) return;
    if constexpr ((ABL & 8) != 0) buf_half(rB, voB, ldb, half, t, smem + (t & 1) * STAGE + PANEL);
    else stage_half(Bb, ldb, half, t, smem + (t & 1) * STAGE + PANEL);
  };

  f32x4_t acc[8][4];   // [mh·4 + i][nh·2 + j]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  bf16x8_t af[2][4];        // [ks][i] of the current m-half
  bf16x8_t bf0[2][2], bf1[2][2];   // [ks][j] of n-half 0 / 1
  auto readA = [&](int t, int mh) {
    if constexpr ((ABL & 2) != 0) { if (t > 0) return; }
    const char* pa = smem + (t & 1) * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag(pa, mh * 128 + wm * 64 + i * 16 + fr, ks * 4 + fq);
  };
  auto readB = [&](int t, int nh, bf16x8_t (&bf)[2][2]) {
    if constexpr ((ABL & 2) != 0) { if (t > 0) return; }
    const char* pb = smem + (t & 1) * STAGE + PANEL;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[ks][j] = frag(pb, wn * 64 + nh * 32 + j * 16 + fr, ks * 4 + fq);
  };
  auto mma = [&](int mh, int nh, const bf16x8_t (&bf)[2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mh * 4 + i][nh * 2 + j] = mfma16(bf[ks][j], af[ks][i], acc[mh * 4 + i][nh * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue: tile 0 (A0 B0 B1 A1) and the first two halves of tile 1; retire A0(0), B0(0).  Always real
  // loads (also in the no-load ablation); the buffer form reads a last half tile's panel end as zeros.
  auto proA = [&](int half, int t) {
    if constexpr ((ABL & 8) != 0) buf_half(rA, voA, lda, half, t, smem + (t & 1) * STAGE);
    else stage_half(Ab, lda, half, t, smem + (t & 1) * STAGE);
  };
  auto proB = [&](int half, int t) {
    if constexpr ((ABL & 8) != 0) buf_half(rB, voB, ldb, half, t, smem + (t & 1) * STAGE + PANEL);
    else stage_half(Bb, ldb, half, t, smem + (t & 1) * STAGE + PANEL);
  };
  proA(0, 0); proB(0, 0); proB(1, 0); proA(1, 0);
  proA(0, 1); proB(0, 1); proB(1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  bar();

  // One K-tile = 2 phases of 32 MFMAs (stage / wait table and hazard argument: gemm_nt3_kernel below);
  // `G1` = the staggered group (one barrier behind).
  auto ktile = [&](int t) {
    const bool more1 = t + 1 < nt, more2 = t + 2 < nt;
    // P01 (0,0) (0,1): A1 of K-tile t; younger: the previous P23's three halves (the prologue's at t = 0)
    if (t == 0 || more1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    readB(t, 0, bf0);
    readA(t, 0);
    readB(t, 1, bf1);
    if (more1) stA(1, t + 1);
    bar();
    mma(0, 0, bf0);
    mma(0, 1, bf1);
    bar();
    // P23 (1,1) (1,0): K-tile t+1's A0 B0 B1, read by BOTH wave rows in their next P01 (rows of a half come from
    // all 8 waves); younger: this P01's A1.  Both rows wait here, two barriers ahead of the reads.
    if (more1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!half) readA(t, 1);
    if (more2) { stA(0, t + 2); stB(0, t + 2); stB(1, t + 2); }
    bar();
    if (!half) {
      mma(1, 1, bf1);
      mma(1, 0, bf0);
    }
    bar();
  };
  if (ABL & 4) {
    for (int t = 0; t < nt; ++t) ktile(t);
  } else if (__builtin_amdgcn_readfirstlane(wm) == 0) {
    for (int t = 0; t < nt; ++t) ktile(t);
    bar();
  } else {
    bar();
    for (int t = 0; t < nt; ++t) ktile(t);
  }

  // ---- epilogue (as v1, with the quadrant → tile mapping): acc (+bias) -> bf16 into this wave's
  // private LDS region [128 local rows][64 local cols], local row lr = mh·64 + i·16 + ..,
  // local col lc = nh·32 + j·16 + ..; then row-coalesced 16-B pieces -> epilogue math -> global.
  constexpr int WN = 64;
  constexpr int RS = WN * 2 + 16;
  constexpr int SEGS = WN / 8;                  // 8 pieces of 16 B per local row
  constexpr int ROWS_PER_IT = 64 / SEGS;        // 8
  constexpr int NIT = 128 / ROWS_PER_IT;        // 16 row-coalesced pieces per lane
  constexpr bool kReadsAux = EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL || EPI == HQ_EPI_RESID || EPI == HQ_EPI_BDR;
  const int seg = lane % SEGS, rsub = lane / SEGS;
  const int gcol = n0 + wn * 64 + seg * 8;   // full 128-B lines per store (see gemm_nt3_kernel)
  auto grow_of = [&](int it) {
    const int lr = it * ROWS_PER_IT + rsub;
    return m0 + (lr >> 6) * 128 + wm * 64 + (lr & 63);
  };
  char* wreg = smem + wave * (128 * RS);
  constexpr bool kBias = EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD || EPI == HQ_EPI_BDR;
#pragma unroll
  for (int J = 0; J < 4; ++J) {
    const int nh = J >> 1, j = J & 1;
    const int lc = nh * 32 + j * 16 + fq * 4;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (kBias) bv = *reinterpret_cast<const float4*>(bias + n0 + wn * 64 + nh * 32 + j * 16 + fq * 4);
#pragma unroll
    for (int I = 0; I < 8; ++I) {
      float v[4] = {acc[I][J][0], acc[I][J][1], acc[I][J][2], acc[I][J][3]};
      if constexpr (kBias) { v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w; }  // no "+0" canonicalise adds
      *reinterpret_cast<uint2*>(wreg + (I * 16 + fr) * RS + lc * 2) = hq_pack4(v);
    }
  }
  // The epilogue's second operand (P = stored pre / gelu', R = residual) comes from HBM: issue all 16
  // pieces of this lane at once so ONE load latency is exposed instead of one per few pieces inside the
  // store loop (64 VGPRs; the accumulators are dead now).  Issued after the staging writes: hipcc
  // drains vmcnt(0) before the first LDS write (the main loop's LDS-DMA shares the counter).
  // a half tile has local rows 0..63 only (it < NIT / 2)
  uint4 aux[kReadsAux ? NIT : 1];
  if constexpr (kReadsAux) {
    const uint16_t* src = (EPI == HQ_EPI_RESID || EPI == HQ_EPI_BDR) ? R : P;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {   // a half tile re-reads its rows for the unused pieces (no per-load branch)
      const int itl = half ? (it & (NIT / 2 - 1)) : it;
      aux[it] = *reinterpret_cast<const uint4*>(src + (size_t)grow_of(itl) * ldc + gcol);
    }
  }
  float csum[8];
  if constexpr (EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL) {
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    if (half && it >= NIT / 2) continue;
    const int lr = it * ROWS_PER_IT + rsub;
    uint4 piece = *reinterpret_cast<const uint4*>(wreg + lr * RS + seg * 16);
    const size_t goff = (size_t)grow_of(it) * ldc + gcol;
    if constexpr (EPI == HQ_EPI_GELU) {
      *reinterpret_cast<uint4*>(P + goff) = piece;
      float x[8];
      hq_unpack8(piece, x);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = gelu_erf(x[e]);
      piece = hq_pack8(x);
    } else if constexpr (EPI == HQ_EPI_GELUD) {
      float x[8], g[8];
      hq_unpack8(piece, x);
      hq_gelu_grad8(x, g);   // g = gelu'(x), x = gelu(x)
      *reinterpret_cast<uint4*>(P + goff) = hq_pack8(g);
      piece = hq_pack8(x);
    } else if constexpr (EPI == HQ_EPI_DMUL) {
      float d[8], gd[8];
      hq_unpack8(piece, d);
      hq_unpack8(aux[it], gd);
#pragma unroll
      for (int e = 0; e < 8; ++e) { d[e] *= gd[e]; csum[e] += d[e]; }
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_DGELU) {
      float d[8], pr[8];
      hq_unpack8(piece, d);
      hq_unpack8(aux[it], pr);
#pragma unroll
      for (int e = 0; e < 8; ++e) { d[e] *= gelu_grad(pr[e]); csum[e] += d[e]; }
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_RESID) {
      float d[8], rr[8];
      hq_unpack8(piece, d);
      hq_unpack8(aux[it], rr);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] += rr[e];
      piece = hq_pack8(d);
    } else if constexpr (EPI == HQ_EPI_BDR) {
      piece = hq_epi_bdr8(piece, aux[it], (uint32_t)goff, dr, key);
    }
    *reinterpret_cast<uint4*>(C + goff) = piece;
  }
  if constexpr (EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      for (int o = SEGS; o < 64; o <<= 1) csum[e] += __shfl_xor(csum[e], o, 64);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [2][BN], indexed by tile column
    if (rsub == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wm * BN + (gcol - n0) + e] = csum[e];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += kThreads) part[(size_t)tm * N + n0 + c] = red[c] + red[BN + c];
  }
}

// ================================================================================ v3: persistent
// v2's per-tile fixed cost (WG launch, the prologue's first HBM round trip, the epilogue's drain) is
// ~11k cycles per 256² tile — a third of a K = 768 tile (profiles/s3_prof: the same 464 GFLOP run
// 1.03 PF/s as 4608 K=768 tiles, 1.20 PF/s as 1152 K=3072 tiles).  v3 keeps ONE workgroup per CU
// walking tiles (tile = id, id + grid, …) and runs the LDS-DMA pipeline straight across the tile seam:
// K-tile 0 of the next tile is staged during the last two K-tiles of this one (exactly the loads the
// steady state would issue for t+1 / t+2), so its data lands under the last MFMA phases and the
// epilogue, and the next tile's K-tile-1 A0 / B0 / B1 halves go into the last K-tile's buffer as soon as
// every wave has read it, ahead of the epilogue.
//
// Epilogue LDS: the 128 local rows of each wave are staged in four 32-row rounds through a 4.5 KB region
// per wave — waves 0-2 in the A1 half of the last K-tile's buffer (the next tile stages its K-tile-1 A1 there
// only in its first phase), waves 3-4 past both buffers, waves 5-7 past the bias.  The epilogue's global
// loads/stores (E per lane, EPI-dependent, issued after the next tile's K-tile-1 halves) are counted into
// the first K-tile's vmcnt waits.  Raw barriers only (a __syncthreads fence would drain
// the in-flight DMA).
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// HQ_EPI_DIAG (lab builds only, never in the production library): bit 0 = the persistent kernel's epilogue issues no
// global stores (data kept live), bit 1 = GELUD skips the GELU math — isolates store cost from VALU cost.
#ifndef HQ_EPI_DIAG
#define HQ_EPI_DIAG 0
#endif
// Cache policy of the persistent kernel's epilogue stores (gfx950 CPol bits: 1 = sc0, 2 = nt, 16 = sc1).  NTS
// kernels store with nt | sc1 — streamed past the caches: at K = 768 the output is a third of the kernel's work in
// bytes and its default-policy write-back holds the next tiles' LDS-DMA operand loads up (the stores retire, in
// vmcnt order, ahead of them); nt | sc1 made the K = 768 NONE / BIAS / GELU / GELUD GEMMs 6-11 % faster on one box
// (profiles/r5_epi_diag/aux*.log), while the K = 2304 / 3072 shapes and the epilogues that load an operand (DMUL /
// RESID) lost 0-3 %.  HQ_EPI_STORE_AUX (lab builds) forces the bits for every variant.
#ifndef HQ_EPI_STORE_AUX
#define HQ_EPI_STORE_AUX 0
#endif
template <int EPI>
struct NT3Epi {
  static constexpr int kStores = (HQ_EPI_DIAG & 1) ? 0 : 16 * (1 + (EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD ? 1 : 0));
  static constexpr int kLoads = (EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL || EPI == HQ_EPI_RESID || EPI == HQ_EPI_BDR) ? 16 : 0;
  static constexpr int E = kStores + kLoads;   // vm ops per lane (the part store of waves 0-3 is not counted: a
};                                             // smaller count only waits longer)

// DYN: the per-XCD ticket schedule is compiled in (a launch with sched == nullptr runs the static one either
// way).  The static-only build (DYN = false, the single-GPU default) has no ticket atomic, whose pending return
// makes hipcc drain vmcnt(0) — the next tile's in-flight K-tile-0 DMA — at every tile's epilogue.
template <int EPI, bool DYN, bool NTS>
__global__ __launch_bounds__(kThreads, 1) void gemm_nt3_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                               uint16_t* __restrict__ C, const float* __restrict__ bias,
                                                               uint16_t* __restrict__ P, const uint16_t* __restrict__ R,
                                                               float* __restrict__ part, int M, int N, int K, int lda,
                                                               int ldb, int ldc, int stagger, unsigned* __restrict__ sched,
                                                               HqDropArg dr) {
  const uint32_t key = EPI == HQ_EPI_BDR ? dr.kd.get() : 0u;   // EPI_BDR dropout key (device seed word under graphs)
  constexpr int BN = 256;
  constexpr int PANEL = 256 * 128;
  constexpr int STAGE = 2 * PANEL;
  constexpr int WN = 64;
  constexpr int RS = WN * 2 + 16;
  constexpr int REGION = 64 * RS;            // one wave's 64-row staging round (9216 B)
  constexpr int SPARE = 2 * STAGE;           // past both stage buffers: wave 7's region, then csum scratch
  constexpr int E = NT3Epi<EPI>::E;
  constexpr int TICKET = SPARE + REGION + 2 * BN * 4;   // LDS word: the tile after `next` (dynamic schedule)
  constexpr int BIASL = TICKET + 16;                    // the unit's 256 fp32 bias values (1 KiB, LDS-DMA by wave 0)
  // epilogue staging: 32-row rounds, QREG bytes per wave — waves 0-2 in the A1 half of the last K-tile's
  // buffer, 3-4 in SPARE, 5-7 past the bias — so that the buffer's other three halves take the next tile's
  // K-tile 1 BEFORE the epilogue's stores (vmcnt retires in issue order: K-tile 1 issued after the stores
  // could not be waited for before they drained, which the first K-tile's counted waits then did)
  constexpr int QREG = 32 * RS;
  constexpr int TAIL = BIASL + 1024;
  static_assert(3 * QREG <= PANEL / 2 && 2 * QREG <= REGION && TAIL + 3 * QREG <= 160 * 1024, "LDS plan");
  constexpr bool kBiasE = EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD || EPI == HQ_EPI_BDR;
  const bool ht_on = (stagger >> 16) & 1;   // kHalfTail
  const bool quarter_on = (stagger >> 17) & 1;
  stagger &= 0xFF;
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_n = N / BN, ntiles = (M / BM) * tiles_n;
  // The epilogue's bias comes through LDS: wave 0 stages a unit's 256 values with one LDS-DMA instruction at the
  // unit's start (retired by the K-loop's counted waits, made visible by its barriers), and the epilogue reads
  // them with inline-asm ds_reads — a global load there would wait (vmcnt, in issue order) for the next tile's
  // K-tile-0 DMA still in flight, and a builtin LDS read makes hipcc drain vmcnt(0) for the same reason.
  auto stage_bias = [&](int n0u) {
    if constexpr (kBiasE) {
      if (__builtin_amdgcn_readfirstlane(wave) == 0) {
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)bias, (short)0, N * 4, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(smem + BIASL), 16, lane * 16, n0u * 4, 0, 0);
      }
    }
  };

  const int nt = K / BK;
  HQ_DASSERT(K % BK == 0 && nt >= 2 && N % BN == 0 && M % BM == 0);
  // Half-tile tail: when the last wave of tiles is at most half full (rtail = ntiles % nwg tiles on nwg
  // workgroups), its rtail tiles run as 2·rtail 128-row "half tiles", one per workgroup, so that wave costs about
  // half a tile's time instead of a whole one (at B = 256 every N = 768 GEMM has 4.5 waves of tiles).  Work
  // units: 0 … F-1 the full tiles, F … F+2·rtail-1 the halves (unit F + 2h + e = rows e·128 … of tile F + h).  A
  // half tile keeps the full tile's load / barrier / wait sequence (its second 128 A rows are staged and
  // never read) and skips the m-half-1 MFMA phases, fragment reads and epilogue round.  Column partials
  // (DGELU / DMUL) are per 256-row block, so those epilogues never split.
  constexpr bool kHalfOK = !(EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL);
  const int rtail = ntiles % nwg;
  const bool halftail = kHalfOK && ht_on && rtail > 0 && 2 * rtail <= nwg;
  const int F = halftail ? ntiles - rtail : ntiles;
  const int nunits = halftail ? F + 2 * rtail : ntiles;
  auto unit_m0 = [&](int u) {
    return u < F ? (u / tiles_n) * BM : ((F + ((u - F) >> 1)) / tiles_n) * BM + ((u - F) & 1) * 128;
  };
  auto unit_n0 = [&](int u) { return (u < F ? u : F + ((u - F) >> 1)) % tiles_n * BN; };

  int voA[2], voB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 16 + i * 8 + (lane >> 3);
    const int src_slot = (lane & 7) ^ ((row >> 1) & 7);
    voA[i] = (row * lda + src_slot * 8) * 2;
    voB[i] = (row * ldb + src_slot * 8) * 2;
  }
  // buffer descriptors over a unit's A row panel / B column panel (a last half tile's panel ends at row M:
  // its unread second 128 rows load as zeros)
  auto rsrc_a = [&](int u) {
    const int m0 = unit_m0(u);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * lda), (short)0, min(BM, M - m0) * lda * 2,
                                             0x00020000);
  };
  auto rsrc_b = [&](int u) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(B + (size_t)unit_n0(u) * ldb), (short)0, BN * ldb * 2, 0x00020000);
  };
  // one 16 KiB half (128 rows × 64 bf16) of K-tile `kt` into LDS buffer `buf`
  auto stA = [&](__amdgpu_buffer_rsrc_t rs, int half, int kt, int buf) {
    char* dst = smem + buf * STAGE + (half * 128 + wave_u * 16) * 128;
    const int so = half * 128 * lda * 2 + kt * BK * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 8 * 128), 16, voA[i], so, 0, 0);
  };
  auto stB = [&](__amdgpu_buffer_rsrc_t rs, int half, int kt, int buf) {
    char* dst = smem + buf * STAGE + PANEL + (half * 128 + wave_u * 16) * 128;
    const int so = half * 128 * ldb * 2 + kt * BK * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + i * 8 * 128), 16, voB[i], so, 0, 0);
  };

  f32x4_t acc[8][4];
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8_t af[2][4];
  bf16x8_t bf0[2][2], bf1[2][2];
  auto readA = [&](int buf, int mh) {
    const char* pa = smem + buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag(pa, mh * 128 + wm * 64 + i * 16 + fr, ks * 4 + fq);
  };
  auto readB = [&](int buf, int nh, bf16x8_t (&bf)[2][2]) {
    const char* pb = smem + buf * STAGE + PANEL;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[ks][j] = frag(pb, wn * 64 + nh * 32 + j * 16 + fr, ks * 4 + fq);
  };
  auto mma = [&](int mh, int nh, const bf16x8_t (&bf)[2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mh * 4 + i][nh * 2 + j] = mfma16(bf[ks][j], af[ks][i], acc[mh * 4 + i][nh * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // Tile schedule.  Static: tile id, id + nwg, id + 2·nwg, …  — the blocks of one XCD (x = bid & 7, the
  // cnt_x workgroups with ids base_x … base_x + cnt_x - 1) walk, round after round, the same contiguous
  // run of cnt_x tiles, so their A row panels stay in that XCD's L2.  Dynamic (sched != null) keeps that
  // per-XCD sequence, tile(s) = (s / cnt_x)·nwg + base_x + s % cnt_x, but hands out its entries s ≥ 2·cnt_x
  // by tickets from the XCD's own counter (sched[32·x]); the first two (s = j, cnt_x + j) stay static, as the
  // pipeline stages the next tile's K-tile 0 during this tile's last K-tiles, so `next` must be known when
  // this tile starts.  A workgroup dispatched late — its CU held by another stream's kernel, e.g. the RCCL
  // all-reduce overlapped with the backward — then delays only its first two tiles instead of its whole
  // 1/nwg share (tools/gemm_contention_bench.py).  The ticket is drawn by thread 0 early in the tile
  // (a per-lane address keeps hipcc's atomic optimizer — whose readfirstlane would wait for the return on
  // the spot — out of it) and published through LDS after the K-loop, where hipcc drains vmcnt anyway.
  // Every workgroup bumps sched[256] on exit; the last one zeroes the counters for the next launch on this
  // stream (stream order: the next launch starts after this one has drained, graph replays included).
  int tile = id;                // a work unit (see the half-tile tail above)
  HQ_DASSERT(tile < nunits);     // the host launches min(tiles, CUs) workgroups, so every one has a tile
  if (tile >= nunits) return;   // (unreachable; an early exit would skip the exit count that re-zeroes sched)
  int next = tile + nwg;
  const int cnt_x = q + (xcd < r ? 1 : 0), base_x = id - (bid >> 3);
  if constexpr (!DYN) sched = nullptr;
  unsigned* tix = sched ? sched + 32 * xcd : nullptr;
  // Phase offset for half of each XCD's workgroups (stagger × 8128 cycles): the tile seams of all CUs
  // otherwise coincide, and every epilogue's stores / aux loads hit HBM in one chip-wide burst that the
  // next K-tile's counted wait (vmcnt counts stores too) then stalls on.
  // bit 17 of the flag word: four groups (offsets 0, 1, 2, 3 × stagger) instead of two (0, stagger)
  const int sgroup = quarter_on ? ((bid >> 3) & 3) : ((bid >> 3) & 1);
  for (int i = 0; i < stagger * sgroup; ++i) __builtin_amdgcn_s_sleep(127);
  __amdgpu_buffer_rsrc_t ca = rsrc_a(tile), cb = rsrc_b(tile);
  int p0 = 0;                   // LDS buffer of this tile's K-tile 0
  // prologue of the first tile: K-tile 0 (A0 B0 B1 A1) and K-tile 1's A0 B0 B1 (its A1 is staged in K-tile 0)
  stage_bias(unit_n0(tile));   // oldest op of wave 0: retired by the wait below
  stA(ca, 0, 0, 0); stB(cb, 0, 0, 0); stB(cb, 1, 0, 0); stA(ca, 1, 0, 0);
  stA(ca, 0, 1, 1); stB(cb, 0, 1, 1); stB(cb, 1, 1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  bar();
  bool first = true;
  bool prev_half = false;       // the previous unit was a half tile: its epilogue issued E / 2 vm ops

  for (;;) {
    const bool last = next >= nunits;
    const bool half = __builtin_amdgcn_readfirstlane(tile >= F ? 1 : 0) != 0;
    unsigned ticket = 0;
    const bool draw = DYN && sched && !last;
    // drawn in phase P1 of K-tile 0, after that phase's stage: the counted vmcnt(6) of K-tile 1's P1 (6 newer
    // loads by then) retires it about a K-tile later, so its round trip never stalls a wait (issued at the
    // tile top it was the OLDEST op under K-tile 0's first wait and cost ~1-3 % per GEMM)
    auto draw_ticket = [&]() {
      if (tid == 0) {
        unsigned zero;
        asm volatile("v_mov_b32 %0, 0" : "=v"(zero));   // opaque per-lane offset (see above)
        ticket = __hip_atomic_fetch_add(tix + zero, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    };
    const __amdgpu_buffer_rsrc_t na = rsrc_a(last ? tile : next), nb = rsrc_b(last ? tile : next);
    const int m0 = unit_m0(tile), n0 = unit_n0(tile);
    const int tm = m0 / BM;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // One K-tile = 2 phases of 32 MFMAs per wave, each a (fragment reads + stage | barrier | MFMAs | barrier)
    // pair; the two wave rows (wm) run one barrier apart, so one row's MFMAs cover the other's reads:
    //   P01: reads B(nh 0), A(mh 0), B(nh 1); stages A1 of K-tile t+1   | MFMAs (0,0) (0,1)
    //   P23: reads A(mh 1); stages A0, B0, B1 of K-tile t+2              | MFMAs (1,1) (1,0)
    // Every half is staged by all 8 waves (16 rows each) and read 4-6 barrier intervals later; each wave's
    // counted wait retires its own rows at least one barrier before ANY wave reads them.  A half is
    // re-staged only after both rows have read it (A1 of buffer b1 two intervals after its last read, the
    // others one).  Past this tile's end the stages come from the next tile's K-tile 0 (t+1 == nt,
    // t+2 == nt); its K-tile-1 A0 B0 B1 (t+2 == nt+1) go into buffer bl right after the last K-tile.
    auto ktile = [&](int t) {
      const bool more1 = t + 1 < nt || !last;                    // P01 stages A1 of K-tile t+1
      const bool more2 = t + 2 < nt || (t + 2 == nt && !last);    // P23 stages K-tile t+2 (A0 B0 B1)
      const bool prev2 = t + 1 < nt || (t + 1 == nt && !last);    // P23 of K-tile t-1 staged K-tile t+1
      const int b0 = (p0 + t) & 1, b1 = b0 ^ 1;
      const bool x1 = t + 1 >= nt, x2 = t + 2 >= nt;        // the "ahead" halves belong to the next tile
      const __amdgpu_buffer_rsrc_t a1 = x1 ? na : ca;
      const __amdgpu_buffer_rsrc_t a2 = x2 ? na : ca, b2r = x2 ? nb : cb;
      const int k1 = x1 ? t + 1 - nt : t + 1, k2 = x2 ? t + 2 - nt : t + 2;
      // P01: A1 of K-tile t (staged in P01 of t-1; younger: P23(t-1)'s 3 halves, or at t = 0 the K-tile-1
      // halves and the epilogue's E vm ops); K-tile t's A0 B0 B1 were retired by P23(t-1)'s wait
      // HQ_EPI_DIAG bit 3 (timing lab only, results WRONG): no vmcnt wait in K-tiles 1-7 of a following unit, i.e.
      // what the mainloop would cost if the previous epilogue's stores never held up the DMA waits
      // bit 4: no vmcnt wait in ANY K-tile of a following unit (pure issue timing, results wrong)
      const bool relax = ((HQ_EPI_DIAG & 8) && !first && t >= 1 && t < 8) || ((HQ_EPI_DIAG & 16) && !first);
      if (relax) {
      } else if (t == 0 && !first) {
        if (prev_half) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + E / 2) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + E) : "memory");
      } else if (t == 0 || prev2) {
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      readB(b0, 0, bf0);
      readA(b0, 0);
      readB(b0, 1, bf1);
      if (more1) stA(a1, 1, k1, b1);
      if (t == 0 && draw) draw_ticket();
      bar();
      mma(0, 0, bf0);
      mma(0, 1, bf1);
      bar();
      // P23: K-tile t+1's A0 B0 B1 (read by both wave rows in their next P01) — younger: this P01's A1 and,
      // at t = 0 of a following unit, the previous unit's epilogue (E vm ops, E / 2 after a half tile), which was
      // issued after K-tile 1.  BOTH rows wait: each half's rows are staged by all 8 waves, so a wave of row 0
      // reads rows of the other row-0 waves, whose P01 wait is in the same barrier interval as that read (round
      // 4's schedule let row 0 skip this wait and relied on the DMA landing within the 6 intervals since issue).
      if (relax) {
      } else if (t == 0 && !first) {
        if (prev_half) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 + E / 2) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 + E) : "memory");
      } else if (more1) {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (!half) readA(b0, 1);
      if (more2) { stA(a2, 0, k2, b0); stB(b2r, 0, k2, b0); stB(b2r, 1, k2, b0); }
      bar();
      if (!half) {
        mma(1, 1, bf1);
        mma(1, 0, bf0);
      }
      bar();
    };
    if (__builtin_amdgcn_readfirstlane(wm) == 0) {
      for (int t = 0; t < nt; ++t) ktile(t);
      bar();
    } else {
      bar();
      for (int t = 0; t < nt; ++t) ktile(t);
    }
    // every wave has passed its last MFMA phase: the buffer of the last K-tile is free
    if (draw && tid == 0)
      *reinterpret_cast<unsigned*>(smem + TICKET) = 2u * (unsigned)cnt_x + ticket;   // sequence index s
    const int bl = (p0 + nt - 1) & 1;
    char* wreg = wave < 3 ? smem + bl * STAGE + PANEL / 2 + wave * QREG
                          : (wave < 5 ? smem + SPARE + (wave - 3) * QREG : smem + TAIL + (wave - 5) * QREG);
    // every wave is past its last read of buffer bl: the next tile's K-tile-1 A0 / B0 / B1 halves go there now,
    // ahead of the epilogue's loads and stores (its A1 half holds waves 0-2's staging; P01 of K-tile 0 stages it)
    if (!last) { stA(na, 0, 1, bl); stB(nb, 0, 1, bl); stB(nb, 1, 1, bl); }

    // ---- epilogue (v2's math), 32 local rows per round (4 rounds, 2 in a half tile).  Ordered so that no round
    // waits for an earlier round's stores (vmcnt counts loads and stores in issue order): the bias and ALL the
    // epilogue operands (aux: 16 pieces per lane, 64 VGPRs — the fragment registers are dead) are loaded before
    // the first store, and the staging writes are inline-asm ds_writes, which hipcc does not fence with vmcnt(0)
    // as it does a builtin LDS store while LDS-DMA may be in flight.  Nothing targets a wave's staging region by
    // DMA during the epilogue, and LDS executes a wave's ds operations in order, so a round's writes cannot
    // overtake the previous round's reads.
    constexpr int SEGS = WN / 8, ROWS_PER_IT = 64 / SEGS;
    constexpr bool kReadsAux = EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL || EPI == HQ_EPI_RESID || EPI == HQ_EPI_BDR;
    constexpr bool kBias = EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD || EPI == HQ_EPI_BDR;
    const int seg = lane % SEGS, rsub = lane / SEGS;
    // wave column wn owns the 64 contiguous tile columns wn·64 … +63 (B fragments nh·32 + j·16 inside it), so each
    // store instruction writes 8 rows × one full 128-B line — the earlier wn·32 + {0, 128} map wrote two 64-B half
    // lines per row, each line split between two waves: −2…−3 % on every K = 768 GEMM, +1.45 % step
    // (profiles/r6_lines)
    const int gcol = n0 + wn * 64 + seg * 8;
    const uint32_t wreg_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)wreg;
    // round q: rows (q >> 1)·128 + wm·64 + (q & 1)·32 + it·8 + rsub of the tile (it: 0..3 within the round)
    auto goff_of = [&](int q, int it) {
      return (size_t)(m0 + (q >> 1) * 128 + wm * 64 + (q & 1) * 32 + it * ROWS_PER_IT + rsub) * ldc + gcol;
    };
    // epilogue global traffic through buffer descriptors over the unit's rows: ONE per-lane offset register
    // (row rsub of the wave's 64-row block, column gcol) and a wave-uniform scalar offset per piece, instead
    // of a 64-bit address per piece (16 pieces × 2 VGPRs spilled once both rounds' operands are prefetched)
    const int rows_u = half ? 128 : BM;
    auto rsrc_of = [&](const uint16_t* base) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (size_t)m0 * ldc), (short)0, rows_u * ldc * 2, 0x00020000);
    };
    const int vo_lane = ((wm * 64 + rsub) * ldc + gcol) * 2;
    auto so_of = [&](int q, int it) { return ((q >> 1) * 128 + (q & 1) * 32 + it * ROWS_PER_IT) * ldc * 2; };
    auto bload = [&](__amdgpu_buffer_rsrc_t r, int rnd, int it) {
#if HQ_EPI_DIAG & 64
      // bit 6 (timing lab only, results WRONG): every operand load reads the tile's first 8 rows (L2-resident):
      // what the epilogue would cost if the operand never came from HBM
      const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, vo_lane & 0xFFFF, 0, 0);
#else
      const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, vo_lane, so_of(rnd, it), 0);
#endif
      return make_uint4(v.x, v.y, v.z, v.w);
    };
    // STORE-DATA HOLD.  A dwordx4 store can read its data VGPRs well after it issued when the wave has a
    // queue of stores (and LDS-DMA) in flight: measured on MI355X, the GELU epilogue's P store (its data
    // overwritten by the GELU math 5 instructions later — hipcc pads 1-2 wait states) wrote the NEW value into
    // dword 0 of 16-lane groups 1 and 3 (~3e-5 of the elements, varying run to run).  So every store's data
    // stays live (an empty asm use) until the NEXT piece's stores have issued, and each round ends with a
    // 64-wait-state pad that holds the last piece (and, for BIAS's back-to-back stores, every piece).
    auto bstore = [&](__amdgpu_buffer_rsrc_t r, int rnd, int it, const uint4& d) {
      const u32x4_t v = {d.x, d.y, d.z, d.w};
#if HQ_EPI_DIAG & 1
      asm volatile("" :: "v"(v));
#elif HQ_EPI_DIAG & 32
      // bit 5: every store goes to the tile's first 8 rows (L2-resident): issue cost without the HBM write traffic
      __builtin_amdgcn_raw_buffer_store_b128(v, r, vo_lane & 0xFFFF, 0, 0);
#else
      __builtin_amdgcn_raw_buffer_store_b128(v, r, vo_lane, so_of(rnd, it), HQ_EPI_STORE_AUX | (NTS ? 18 : 0));
#endif
      return v;
    };
    float csum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
    // NR = 2 row halves (full tile) or 1 (half tile), a compile-time count: with a runtime `half` test hipcc
    // sinks the later rounds' operand loads into the branch, i.e. behind the first round's stores
    auto epilogue = [&](auto nr_c) {
      constexpr int NR = decltype(nr_c)::value;
      // BDR keeps per-round operand loads (both rounds' 64 VGPRs spill beside its dropout hash)
      constexpr bool kAll = kReadsAux && EPI != HQ_EPI_BDR;
      f32x4_t bvs[4] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f},
                        f32x4_t{0.f, 0.f, 0.f, 0.f}};
      if constexpr (kBias) {   // J = 0..3 at byte offsets 0, 64, 128, 192 (cols +0, +16, +32, +48); one statement
        const uint32_t bias_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(smem + BIASL);
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
                     "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(bvs[0]), "=&v"(bvs[1]), "=&v"(bvs[2]), "=&v"(bvs[3])
                     : "v"(bias_lds + (uint32_t)((wn * 64 + fq * 4) * 4))
                     : "memory");
      }
      const __amdgpu_buffer_rsrc_t rC = rsrc_of(C);
      const __amdgpu_buffer_rsrc_t rP = rsrc_of(P ? P : C);
      const __amdgpu_buffer_rsrc_t rA = (EPI == HQ_EPI_RESID || EPI == HQ_EPI_BDR) ? rsrc_of(R) : rP;   // aux source
      constexpr int NQ = 2 * NR;   // 32-row rounds
      uint4 aux[kReadsAux ? (kAll ? 8 * NR : 4) : 1];
      // per round: stage (inline-asm ds_writes: no vmcnt fence), read its 4 pieces back, math, stores; the
      // second row half's operands are loaded after the first round's staging, still before its first store
      uint4 pieces[NQ][4];
      // acc (+bias) → bf16 pairs for every round up front: the 128 accumulator VGPRs die here (64 hold the packed
      // tile), which is what lets both rounds' operands and a round of pieces stay in registers without spilling
      u32x2_t pk[NR][16];
#pragma unroll
      for (int rnd = 0; rnd < NR; ++rnd)
#pragma unroll
        for (int J = 0; J < 4; ++J) {
          const f32x4_t bv = bvs[J];
#pragma unroll
          for (int I = 0; I < 4; ++I) {
            const f32x4_t& a = acc[rnd * 4 + I][J];
            float v[4] = {a[0], a[1], a[2], a[3]};
            if constexpr (kBias) { v[0] += bv[0]; v[1] += bv[1]; v[2] += bv[2]; v[3] += bv[3]; }
            const uint2 q = hq_pack4(v);
            pk[rnd][J * 4 + I] = u32x2_t{q.x, q.y};
          }
        }
      __builtin_amdgcn_sched_barrier(0);   // packed now, not sunk to the staging (the fp32 accumulators die)
      if constexpr (kAll) {   // the first row half's operands now (their latency hides under the staging) ...
#pragma unroll
        for (int it = 0; it < 8; ++it) aux[it] = bload(rA, it >> 2, it & 3);
      }
      auto stage_round = [&](int q) {   // rows (q & 1)·32 … +31 of row half q >> 1: 16-row blocks I = 2·(q & 1) + i
        const int rnd = q >> 1, sub = q & 1;
#pragma unroll
        for (int J = 0; J < 4; ++J) {
          const int nh = J >> 1, j = J & 1;
          const int lc = nh * 32 + j * 16 + fq * 4;
#pragma unroll
          for (int i = 0; i < 2; ++i)
            asm volatile("ds_write_b64 %0, %1" :: "v"(wreg_lds + (uint32_t)((i * 16 + fr) * RS + lc * 2)),
                         "v"(pk[rnd][J * 4 + 2 * sub + i]) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (!kReadsAux) {
          // inline asm: a builtin LDS read would make hipcc drain vmcnt(0), i.e. wait for the next tile's
          // K-tile DMA (epilogues with operand loads wait for those, which are younger, anyway).  The reads and
          // their lgkmcnt wait are ONE asm statement: the outputs are defined only when it completes (with
          // separate statements hipcc may copy an output register before the data has returned).
          static_assert(ROWS_PER_IT * RS == 1152, "ds_read offsets below");
          u32x4_t v0, v1, v2, v3;
          asm volatile(
              "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1152\n\tds_read_b128 %2, %4 offset:2304\n\t"
              "ds_read_b128 %3, %4 offset:3456\n\ts_waitcnt lgkmcnt(0)"
              : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
              : "v"(wreg_lds + (uint32_t)(rsub * RS + seg * 16))
              : "memory");
          const u32x4_t vv[4] = {v0, v1, v2, v3};
#pragma unroll
          for (int it = 0; it < 4; ++it) pieces[q][it] = make_uint4(vv[it].x, vv[it].y, vv[it].z, vv[it].w);
        } else {
#pragma unroll
          for (int it = 0; it < 4; ++it)
            pieces[q][it] = *reinterpret_cast<const uint4*>(wreg + (it * ROWS_PER_IT + rsub) * RS + seg * 16);
        }
      };
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q > 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous round's piece reads returned
        stage_round(q);
        if constexpr (kAll && NR > 1) {
          if (q == 0) {   // the second row half's operands: after the first staging, before its stores
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int it = 0; it < 8; ++it) aux[8 + it] = bload(rA, 2 + (it >> 2), it & 3);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if constexpr (kReadsAux && !kAll) {
#pragma unroll
          for (int it = 0; it < 4; ++it) aux[it] = bload(rA, q, it);
        }
        constexpr bool kTwo = EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD;   // P and C stores per piece
        u32x4_t holdP = {0u, 0u, 0u, 0u}, holdC = holdP;                    // the previous piece's store data
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          uint4 piece = pieces[q][it];
          const size_t goff = goff_of(q, it);
          const uint4 ax = aux[kAll ? q * 4 + it : (kReadsAux ? it : 0)];
          u32x4_t sP = holdP;
          if constexpr (EPI == HQ_EPI_GELU) {
            sP = bstore(rP, q, it, piece);
            float x[8];
            hq_unpack8(piece, x);
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = gelu_erf(x[e]);
            piece = hq_pack8(x);
          } else if constexpr (EPI == HQ_EPI_GELUD) {
            float x[8], g[8];
            hq_unpack8(piece, x);
#if HQ_EPI_DIAG & 2
            for (int e = 0; e < 8; ++e) g[e] = x[e];
#else
            hq_gelu_grad8(x, g);   // g = gelu'(x), x = gelu(x)
#endif
            sP = bstore(rP, q, it, hq_pack8(g));
            piece = hq_pack8(x);
          } else if constexpr (EPI == HQ_EPI_DMUL) {
            float d[8], gd[8];
            hq_unpack8(piece, d);
            hq_unpack8(ax, gd);
#pragma unroll
            for (int e = 0; e < 8; ++e) { d[e] *= gd[e]; csum[e] += d[e]; }
            piece = hq_pack8(d);
          } else if constexpr (EPI == HQ_EPI_DGELU) {
            float d[8], pr[8];
            hq_unpack8(piece, d);
            hq_unpack8(ax, pr);
#pragma unroll
            for (int e = 0; e < 8; ++e) { d[e] *= gelu_grad(pr[e]); csum[e] += d[e]; }
            piece = hq_pack8(d);
          } else if constexpr (EPI == HQ_EPI_RESID) {
            float d[8], rr[8];
            hq_unpack8(piece, d);
            hq_unpack8(ax, rr);
#pragma unroll
            for (int e = 0; e < 8; ++e) d[e] += rr[e];
            piece = hq_pack8(d);
          } else if constexpr (EPI == HQ_EPI_BDR) {
            piece = hq_epi_bdr8(piece, ax, (uint32_t)goff, dr, key);
          }
          const u32x4_t sC = bstore(rC, q, it, piece);
          if (it > 0) {
            if constexpr (kTwo) asm volatile("" :: "v"(holdP), "v"(holdC));
            else asm volatile("" :: "v"(holdC));
          }
          holdP = sP;
          holdC = sC;
          // column-partial epilogues: one piece at a time (hipcc otherwise computes every piece's products
          // ahead of the serial csum chain and spills them)
          if constexpr (EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL) __builtin_amdgcn_sched_barrier(0);
        }
        // round end: 64 wait states with the last stores' data held (BIAS stores back to back: all 4 pieces)
#define HQ_PAD64 "s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15"
        if constexpr (EPI == HQ_EPI_BIAS) {
          auto u = [&](int i) { const uint4& w = pieces[q][i]; return u32x4_t{w.x, w.y, w.z, w.w}; };
          asm volatile(HQ_PAD64 :: "v"(u(0)), "v"(u(1)), "v"(u(2)), "v"(u(3)));
        } else if constexpr (kTwo) {
          asm volatile(HQ_PAD64 :: "v"(holdP), "v"(holdC));
        } else {
          asm volatile(HQ_PAD64 :: "v"(holdC));
        }
#undef HQ_PAD64
      }
    };
    if constexpr (!kHalfOK) epilogue(std::integral_constant<int, 2>{});   // column partials: never a half tile
    else if (half) epilogue(std::integral_constant<int, 1>{});
    else epilogue(std::integral_constant<int, 2>{});
    if constexpr (EPI == HQ_EPI_DGELU || EPI == HQ_EPI_DMUL) {
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
    // every wave has read the bias (and its staging rounds): stage the next unit's bias (an extra, younger op of
    // wave 0 only: its counted waits wait longer)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    stage_bias(unit_n0(next));
    int after = next + nwg;
    if (sched) {
      const unsigned sx = *reinterpret_cast<const unsigned*>(smem + TICKET);
      const long t = (long)(sx / (unsigned)cnt_x) * nwg + base_x + (long)(sx % (unsigned)cnt_x);
      after = t < nunits ? (int)t : nunits;
    }
    prev_half = half;
    tile = next;
    next = __builtin_amdgcn_readfirstlane(after);
    ca = na;
    cb = nb;
    p0 = (p0 + nt) & 1;
    first = false;
  }
  if (sched && tid == 0) {
    if (__hip_atomic_fetch_add(sched + 256, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nwg - 1) {
      for (int x = 0; x < 8; ++x) __hip_atomic_store(sched + 32 * x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sched + 256, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// 0 = auto (v3 for K <= 2304, else v2), 1 = force v1, 2 = force v2, 3 = force v3, 4 = force vS; set only by
// the tests / lab tools through gemm_set_variant (no environment knob)
int g_gemm_variant = 0;
// v3 flag word (gemm_set_stagger, tests / lab tools only): start offset of odd workgroups per XCD in units of
// s_sleep(127) (bits 0-7, 0 in production); bit 16 (kHalfTail): a last, at most half-full wave of tiles runs
// as 128-row half tiles (on)
constexpr int kHalfTail = 1 << 16;
int g_gemm_stagger = kHalfTail;

// default static: uncontended the dynamic schedule costs ~0.9 % of the step (profiles/r2_sched); GradReducer
// switches it on when an all-reduce overlaps the backward (world > 1); HQ_GEMM_SCHED overrides either way
// epilogue store cache policy of the persistent kernel (see HQ_EPI_STORE_AUX): 1 = streamed stores for the
// operand-free epilogues at K <= 768 (production), 0 = default policy everywhere, 2 = streamed at any K (A/B only)
int g_store_policy = 1;

int g_gemm_sched = [] {
  const char* e = getenv("HQ_GEMM_SCHED");
  return e ? atoi(e) : 0;
}();

// Per (device, stream) slot of the v3 ticket schedule: 8 per-XCD ticket counters and the exit counter,
// each on its own 128-B line (words 32·x, 256), carved from one 64-slot block per device that is
// allocated and zeroed on the first use (an eager call: no allocation inside a graph capture once the
// step has run once).  Stream order serialises the launches that share a slot.
constexpr size_t kSchedWords = 9 * 32;
struct SchedPool { unsigned* base = nullptr; std::vector<hipStream_t> streams; };
std::mutex g_sched_mu;

// the current device's pool, allocated and zeroed on first use (caller holds g_sched_mu)
SchedPool* sched_pool_locked() {
  static std::vector<SchedPool> pools;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if ((int)pools.size() <= dev) pools.resize(dev + 1);
  SchedPool& p = pools[dev];
  if (!p.base) {
    void* q = nullptr;
    if (hipMalloc(&q, 64 * kSchedWords * sizeof(unsigned)) != hipSuccess ||
        hipMemset(q, 0, 64 * kSchedWords * sizeof(unsigned)) != hipSuccess) {
      fprintf(stderr, "nt3 tile schedule: slot allocation failed, static schedule\n");
      g_gemm_sched = 0;
      return nullptr;
    }
    p.base = static_cast<unsigned*>(q);
  }
  return &p;
}

unsigned* nt3_sched_slot(hipStream_t s) {
  std::lock_guard<std::mutex> lock(g_sched_mu);
  SchedPool* p = sched_pool_locked();
  if (!p) return nullptr;
  for (size_t i = 0; i < p->streams.size(); ++i)
    if (p->streams[i] == s) return p->base + kSchedWords * i;
  if (p->streams.size() >= 64) return nullptr;   // more streams than slots: static schedule on the rest
  p->streams.push_back(s);
  return p->base + kSchedWords * (p->streams.size() - 1);
}

int nts_num_cus() {
  static int ncu = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return ncu;
}

// vS split-K factor: only epilogues without column partials / GELU, grids below half a workgroup per CU,
// and at least 8 K-tiles per split; HQ_GEMM_SPLITK=0 disables (A/B), N > 1 forces up to N.
int g_nts_splitk = [] {
  const char* e = getenv("HQ_GEMM_SPLITK");
  return e ? atoi(e) : -1;
}();
template <int EPI>
int nts_ksplit(int tiles, int nk) {
  if (!(EPI == HQ_EPI_NONE || EPI == HQ_EPI_BIAS || EPI == HQ_EPI_RESID) || g_nts_splitk == 0) return 1;
  int ks = g_nts_splitk > 1 ? g_nts_splitk : (2 * tiles <= nts_num_cus() ? 2 * nts_num_cus() / tiles : 1);
  ks = std::min(ks, std::min(4, nk / 8));
  return ks > 1 ? ks : 1;
}

constexpr size_t epi_lds(int bn) {
  const size_t stage = 2 * (size_t)(BM * 128 + bn * 128);
  const size_t epi = 8 * 128 * (size_t)(bn / 4 * 2 + 16);
  return stage > epi ? stage : epi;
}

template <int EPI>
void launch_epi(const uint16_t* A, const uint16_t* B, uint16_t* C, const float* bias, uint16_t* P, const uint16_t* R,
                float* part, int M, int N, int K, int lda, int ldb, int ldc, int bn, hipStream_t s, const HqDropArg& dr,
                float* ws) {
  if (bn == 1) {   // vS: 128×128 tiles, M tail
    constexpr size_t lds = 2 * 2 * 128 * 128;
    static bool init = [] {
      (void)hipFuncSetAttribute((const void*)gemm_nts_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      return true;
    }();
    (void)init;
    const int grid_s = ((M + 127) / 128) * (N / 128);
    int ks = nts_ksplit<EPI>(grid_s, K / BK);
    if (ks > 1 && !ws) {   // no workspace from the caller: run unsplit rather than share a scratch buffer
      ks = 1;
    }
    hipLaunchKernelGGL((gemm_nts_kernel<EPI>), dim3(grid_s * ks), dim3(256), lds, s, A, B, C, bias, P, R, part, M, N, K,
                       lda, ldb, ldc, ks, ws, dr);
    if (ks > 1) {
      const size_t n8 = (size_t)M * N / 8;
      const int g = (int)std::min<size_t>((n8 + 255) / 256, 2048);
      hipLaunchKernelGGL((splitk_epi_kernel<EPI == HQ_EPI_BIAS ? HQ_EPI_BIAS : EPI == HQ_EPI_RESID ? HQ_EPI_RESID
                                                                                                   : HQ_EPI_NONE>),
                         dim3(g), dim3(256), 0, s, ws, ks, C, bias, R, M, N, ldc);
    }
    return;
  }
  const int grid = (M / BM) * (N / bn);
  const bool srd_ok = (size_t)BM * lda * 2 < (1ull << 31) && (size_t)256 * ldb * 2 < (1ull << 31);
  // v3 (persistent, pipelined across tiles) where the per-tile fixed cost matters: K <= 2304 (+2-6 % at
  // K = 768 / 2304 on the b256 shapes, -1-3 % at K = 3072: tools/gemm_nt3_check.py, profiles/s3_gemm_v3)
  // (and at any K when the half-tile tail applies: at K = 3072 v3 + tail beat v2 + tail by 0.2-2.8 % on two
  // boxes, profiles/r3_halftail)
  const int ncu_t = nts_num_cus(), rt_t = grid % ncu_t;
  const bool tail_t = (g_gemm_stagger & kHalfTail) && EPI != HQ_EPI_DGELU && EPI != HQ_EPI_DMUL && rt_t > 0 &&
                      2 * rt_t <= ncu_t && grid > ncu_t;
  const bool v3_auto = g_gemm_variant == 0 && (K <= 2304 || tail_t);
  if (bn == 256 && (g_gemm_variant == 3 || v3_auto) && K >= 2 * BK && srd_ok) {
    constexpr size_t lds = 2 * 2 * 256 * 128 + 64 * 144 + 2 * 256 * 4 + 16 + 1024 + 3 * 32 * 144;
    static int ncu = [] {
      int dev = 0, n = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      for (const void* f : {(const void*)gemm_nt3_kernel<EPI, false, false>, (const void*)gemm_nt3_kernel<EPI, true, false>,
                            (const void*)gemm_nt3_kernel<EPI, false, true>, (const void*)gemm_nt3_kernel<EPI, true, true>})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      return n > 0 ? n : 256;
    }();
    const int nwg = std::min(grid, ncu);
    unsigned* sched = (g_gemm_sched && grid > 2 * nwg) ? nt3_sched_slot(s) : nullptr;
    // streamed (nt | sc1) epilogue stores: epilogues without an operand load, K <= 768 (g_store_policy 1), or at any K
    // (2, A/B only), or never (0)
    constexpr bool kNoAux = EPI == HQ_EPI_NONE || EPI == HQ_EPI_BIAS || EPI == HQ_EPI_GELU || EPI == HQ_EPI_GELUD;
    const bool nts = kNoAux && (g_store_policy == 2 || (g_store_policy == 1 && K <= 768));
    auto go = [&](auto kern, unsigned* sc) {
      hipLaunchKernelGGL(kern, dim3(nwg), dim3(kThreads), lds, s, A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc,
                         g_gemm_stagger, sc, dr);
    };
    if (sched) {
      if (nts) go(gemm_nt3_kernel<EPI, true, true>, sched); else go(gemm_nt3_kernel<EPI, true, false>, sched);
    } else {
      if (nts) go(gemm_nt3_kernel<EPI, false, true>, nullptr); else go(gemm_nt3_kernel<EPI, false, false>, nullptr);
    }
  } else if (bn == 256 && (g_gemm_variant == 0 || g_gemm_variant == 2 || g_gemm_variant == 3) && K >= 2 * BK && srd_ok) {
    // production v2: buffer_load…lds staging (+8-12 % over global_load_lds on the BERT shapes,
    // tools/gemm_lab); grouped 8-row-panel tile order only for wide N (+15 % at 8192², neutral at
    // N <= 3072 where an XCD's co-resident tiles already share few panels).
    constexpr size_t lds = epi_lds(256);
    static bool init = [] {
      (void)hipFuncSetAttribute((const void*)gemm_nt2_kernel<EPI, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      (void)hipFuncSetAttribute((const void*)gemm_nt2_kernel<EPI, 24>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      return true;
    }();
    (void)init;
    if (N / 256 >= 16) {
      hipLaunchKernelGGL((gemm_nt2_kernel<EPI, 24>), dim3(grid), dim3(kThreads), lds, s, A, B, C, bias, P, R, part, M, N, K,
                         lda, ldb, ldc, dr);
    } else {
      // half-tile tail: rt more blocks, the last 2·rt of them halves of the last rt tiles
      const int ncu = nts_num_cus(), rt = grid % ncu;
      const bool ht = (g_gemm_stagger & kHalfTail) && EPI != HQ_EPI_DGELU && EPI != HQ_EPI_DMUL && rt > 0 &&
                      2 * rt <= ncu && grid > ncu;
      hipLaunchKernelGGL((gemm_nt2_kernel<EPI, 8>), dim3(ht ? grid + rt : grid), dim3(kThreads), lds, s, A, B, C, bias, P,
                         R, part, M, N, K, lda, ldb, ldc, dr);
    }
  } else if (bn == 256) {
    constexpr size_t lds = epi_lds(256);
    static bool init = [] {
      (void)hipFuncSetAttribute((const void*)gemm_nt_kernel<EPI, 256>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      return true;
    }();
    (void)init;
    hipLaunchKernelGGL((gemm_nt_kernel<EPI, 256>), dim3(grid), dim3(kThreads), lds, s, A, B, C, bias, P, R, part, M, N, K,
                       lda, ldb, ldc, dr);
  } else {
    constexpr size_t lds = epi_lds(128);
    static bool init = [] {
      (void)hipFuncSetAttribute((const void*)gemm_nt_kernel<EPI, 128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      return true;
    }();
    (void)init;
    hipLaunchKernelGGL((gemm_nt_kernel<EPI, 128>), dim3(grid), dim3(kThreads), lds, s, A, B, C, bias, P, R, part, M, N, K,
                       lda, ldb, ldc, dr);
  }
}

}  // namespace

void hq_gemm_set_variant(int v) { g_gemm_variant = v; }
void hq_gemm_set_store_policy(int v) { g_store_policy = v; }
void hq_gemm_set_stagger(int v) { g_gemm_stagger = v; }
int hq_gemm_get_sched() { return g_gemm_sched; }
void hq_gemm_set_sched(int v) {
  g_gemm_sched = v;
  if (v) {   // allocate the slots now, eagerly: a first GEMM inside a graph capture must not hipMalloc
    std::lock_guard<std::mutex> lock(g_sched_mu);
    (void)sched_pool_locked();
  }
}

// Kernel family for a shape: 256 / 128 = the 256-row kernels with that block width, 1 = vS (128² tiles),
// 0 = unsupported.  Variants 1-3 force the 256-row kernels where they apply, 4 forces vS; auto takes the
// 256-row kernels when M % 256 == 0 and their grid fills >= 80 % of the CUs' last wave, else vS.
int hq_gemm_nt_supported(int M, int N, int K) {
  if (M <= 0 || K % BK || K < BK || N % 128) return 0;
  const int big = (M % BM == 0) ? (N % 256 == 0 ? 256 : 128) : 0;
  if (g_gemm_variant == 4 || !big) return 1;
  if (g_gemm_variant != 0) return big;
  static int ncu = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const long tiles = (long)(M / BM) * (N / big);
  const long waves = (tiles + ncu - 1) / ncu;
  return tiles * 5 >= waves * ncu * 4 ? big : 1;
}

int hq_gemm_nt_part_rows(int M, int N, int K) {
  const int k = hq_gemm_nt_supported(M, N, K);
  return k == 1 ? (M + 127) / 128 : M / BM;
}

size_t hq_gemm_nt_ws_floats(int M, int N, int K, int epi) {
  if (hq_gemm_nt_supported(M, N, K) != 1) return 0;   // split-K exists on the 128² (vS) kernel only
  const int grid_s = ((M + 127) / 128) * (N / 128);
  int ks = 1;
  switch (epi) {
    case HQ_EPI_NONE: ks = nts_ksplit<HQ_EPI_NONE>(grid_s, K / BK); break;
    case HQ_EPI_BIAS: ks = nts_ksplit<HQ_EPI_BIAS>(grid_s, K / BK); break;
    case HQ_EPI_RESID: ks = nts_ksplit<HQ_EPI_RESID>(grid_s, K / BK); break;
    default: ks = 1;
  }
  return ks > 1 ? (size_t)ks * M * N : 0;
}

void hq_gemm_nt(const uint16_t* A, const uint16_t* B, uint16_t* C, const float* bias, uint16_t* P, const uint16_t* R,
                float* part, int M, int N, int K, int lda, int ldb, int ldc, int epi, int bn, hipStream_t s, float drop_p,
                uint32_t drop_seed, uint32_t drop_opid, float* ws) {
  HqDropArg dr{hq_drop_key(drop_seed, drop_opid), 0u, 1.f};
  if (epi == HQ_EPI_BDR && drop_p > 0.f) {
    dr.thr = hq_threshold(drop_p);
    dr.ks = hq_keep_scale(dr.thr);
  }
  switch (epi) {
    case HQ_EPI_NONE: launch_epi<HQ_EPI_NONE>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, bn, s, dr, ws); break;
    case HQ_EPI_BIAS: launch_epi<HQ_EPI_BIAS>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, bn, s, dr, ws); break;
    case HQ_EPI_GELU: launch_epi<HQ_EPI_GELU>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, bn, s, dr, ws); break;
    case HQ_EPI_DGELU: launch_epi<HQ_EPI_DGELU>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, bn, s, dr, ws); break;
    case HQ_EPI_RESID: launch_epi<HQ_EPI_RESID>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, bn, s, dr, ws); break;
    case HQ_EPI_GELUD: launch_epi<HQ_EPI_GELUD>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, bn, s, dr, ws); break;
    case HQ_EPI_DMUL: launch_epi<HQ_EPI_DMUL>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, bn, s, dr, ws); break;
    case HQ_EPI_BDR: launch_epi<HQ_EPI_BDR>(A, B, C, bias, P, R, part, M, N, K, lda, ldb, ldc, bn, s, dr, ws); break;
  }
}
