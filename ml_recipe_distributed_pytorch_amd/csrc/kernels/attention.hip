// Flash attention for BERT (head_dim 64, L <= 512, additive key mask, fused dropout) on gfx950.
//
// Input is the packed QKV GEMM output [T, 3H] (token-major; head h of Q/K/V at column
// {0,H,2H} + 64h), so no head-split transpose is ever materialised; ctx is written straight in
// [T, H] and the backward writes dQ/dK/dV straight into packed dQKV [T, 3H].
//
// Structure (v2, "whole head per workgroup"): at BERT lengths a head's K and V (L·64·2 B each,
// 96 KB at L=384) fit in LDS, so one workgroup of NWB waves loads them ONCE with every thread
// issuing its 16-B loads up front (a single exposed HBM latency), one barrier, and then every
// wave streams its 32 queries (fwd / dQ) or 32 keys (dK/dV) over the whole sequence with NO
// further barriers.  (v1 staged 64-key tiles with two barriers each and no prefetch: 3-4x slower.)
//
// MFMA: v_mfma_f32_32x32x16_bf16 (32x32 tile, K=16, wave64).  Orientation keeps every softmax
// statistic lane-local:
//   fwd : Sᵀ = K·Qᵀ (query on the lane); Oᵀ += Vᵀ·Pᵀ with Pᵀ fed from the accumulator registers as
//         the B operand (cdna_hip_programming.md §3) and Vᵀ via ds_read_b64_tr_b16 (T10).
//         Online softmax rescales O only when some lane's running max grew (exact: α=1 otherwise).
//   dQ  : Sᵀ, dPᵀ = V·dOᵀ (query on the lane); dQᵀ += Kᵀ·dSᵀ.  Also computes δ = rowsum(dO·O).
//   dKdV: S = Q·Kᵀ, dP = dO·Vᵀ (key on the lane); dVᵀ += dOᵀ·Pd, dKᵀ += Qᵀ·dS.
// Dropout: the forward draws keep bits from the counter hash (hq_common.h, element index
// ((b·nh+h)·L+q)·L+k, bit-identical to ops/rng.py) and stores them as one 16-bit word per lane per
// 32×32 subtile (14 MB per BERT-base layer at B=64); the backward kernels read the bits instead of
// re-hashing (dKdV gathers its key's bits with ds_bpermute).
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int D = 64;  // head dim
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

__device__ __forceinline__ f32x16_t mfma32(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// LDS images are [rows][64] bf16 (128-B rows) with the 16-B chunk index XOR-swizzled by
//   f(row) = ((row>>1)&1)<<2 | ((row>>3)&3)
// found by exhaustive search (tools/lds_swizzle_search.py) to make BOTH access patterns bank-conflict
// free: ds_read_b128 row reads (16 rows of a lane group, one chunk) and ds_read_b64_tr_b16 reads
// (4 rows × 64 B per 32-lane half).  Unswizzled the row reads are 8-way conflicted (T2).
__device__ __forceinline__ int swz(int row) { return (((row >> 1) & 1) << 2) | ((row >> 3) & 3); }
__device__ __forceinline__ int lds_off(int row, int col) {  // element offset of (row, col)
  return row * D + ((((col >> 3) ^ swz(row)) << 3) | (col & 7));
}

__device__ __forceinline__ bf16x8_t lds_row8(const uint16_t* tile, int row, int col) {
  return *reinterpret_cast<const bf16x8_t*>(tile + lds_off(row, col));
}

// swz(row) only depends on row bits 1..4, so every offset inside a 32-row subtile is a lane constant:
// precompute them once (12 VGPRs) instead of re-deriving the XOR per access in VALU-bound loops.
struct LdsOffsets {
  int row[4];        // ds_read_b128 row reads: row (lane&31), chunk 16s + 8hh
  int tr[2][2][2];   // ds_read_b64_tr_b16: [s][dblk][lo/hi]
  __device__ __forceinline__ void init(int lane) {
    const int hh = lane >> 5;
#pragma unroll
    for (int s = 0; s < 4; ++s) row[s] = lds_off(lane & 31, 16 * s + 8 * hh);
    const int g = lane >> 4, i = lane & 15;
    const int th = g >> 1, dsub = g & 1;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const int r = 16 * s + 4 * th + (i >> 2);
        const int c = d * 32 + 16 * dsub + 4 * (i & 3);
        tr[s][d][0] = lds_off(r, c);
        tr[s][d][1] = lds_off(r + 8, c);
      }
  }
};

__device__ __forceinline__ bf16x8_t row8(const uint16_t* tile, int row0, const LdsOffsets& o, int s) {
  return *reinterpret_cast<const bf16x8_t*>(tile + row0 * D + o.row[s]);
}

__device__ __forceinline__ bf16x8_t tr8(const uint16_t* tile, int row0, const LdsOffsets& o, int s, int dblk) {
  const uint16_t* t = tile + row0 * D;
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(t + o.tr[s][dblk][0]));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(t + o.tr[s][dblk][1]));
  bf16x8_t out;
  out[0] = lo[0]; out[1] = lo[1]; out[2] = lo[2]; out[3] = lo[3];
  out[4] = hi[0]; out[5] = hi[1]; out[6] = hi[2]; out[7] = hi[3];
  return out;
}

// A operand "Xᵀ" of a 32x32x16 MFMA from a row-major [rows][64] LDS image: lane supplies
// X[row(s,hh,j)][d], d = dblk*32 + (lane&31), row = row0 + 16s + 4hh + (j&3) + 8(j>>2) (the k order
// of an accumulator-fed B operand).
__device__ __forceinline__ bf16x8_t lds_tr8(const uint16_t* tile, int row0, int s, int dblk, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int hh = g >> 1, dsub = g & 1;
  const int r = row0 + 16 * s + 4 * hh + (i >> 2);
  const int c = dblk * 32 + 16 * dsub + 4 * (i & 3);
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(tile + lds_off(r, c)));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(tile + lds_off(r + 8, c)));
  bf16x8_t out;
  out[0] = lo[0]; out[1] = lo[1]; out[2] = lo[2]; out[3] = lo[3];
  out[4] = hi[0]; out[5] = hi[1]; out[6] = hi[2]; out[7] = hi[3];
  return out;
}

__device__ __forceinline__ bf16x8_t pack_b(const float* v, int s) {
  const uint32_t w0 = hq_pack2(v[8 * s + 0], v[8 * s + 1]), w1 = hq_pack2(v[8 * s + 2], v[8 * s + 3]);
  const uint32_t w2 = hq_pack2(v[8 * s + 4], v[8 * s + 5]), w3 = hq_pack2(v[8 * s + 6], v[8 * s + 7]);
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
  u32x4 u = {w0, w1, w2, w3};
  return __builtin_bit_cast(bf16x8_t, u);
}

// Q fragment pre-multiplied by c = softmax_scale·log2(e) (rounded to bf16): the score MFMA then
// yields log2-domain scores directly, and its accumulator is initialised with the per-key mask bias
// (and, in the backward, minus the per-query LSE), so no per-element scale/bias/LSE VALU remains.
// The forward and both backward kernels use the identical rounded Q·c, so P is recomputed exactly.
__device__ __forceinline__ bf16x8_t prescale8(const bf16x8_t& q, float c) {
  float f[8];
  hq_unpack8(__builtin_bit_cast(uint4, q), f);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] *= c;
  return __builtin_bit_cast(bf16x8_t, hq_pack8(f));
}

__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// One 64-column output row per lane pair from two transposed 32x32 accumulators (the O / dQ / dK / dV
// layout: lane q and q+32 hold the two 4-column halves of each 8-column group) as 16-B stores (playbook
// T21): one permlane32 swap per pair of groups hands lane q the 8 columns of the even group and lane q+32
// those of the odd one — 4 dwordx4 stores per lane instead of 8 dwordx2 (the store tail is issue-bound).
__device__ __forceinline__ void store_row64(uint16_t* out, const f32x16_t (&a)[2], float mul, int hh) {
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      const float va[4] = {a[d][4 * g] * mul, a[d][4 * g + 1] * mul, a[d][4 * g + 2] * mul, a[d][4 * g + 3] * mul};
      const float vb[4] = {a[d][4 * g + 4] * mul, a[d][4 * g + 5] * mul, a[d][4 * g + 6] * mul, a[d][4 * g + 7] * mul};
      const uint2 A = hq_pack4(va), B = hq_pack4(vb);
      // swap(vdst = A, src = B): lanes 32-63 of A trade with lanes 0-31 of B, so lane q now holds
      // [own A | partner's A] = group g and lane q+32 [partner's B | own B] = group g+1
      const auto r0 = __builtin_amdgcn_permlane32_swap(A.x, B.x, false, false);
      const auto r1 = __builtin_amdgcn_permlane32_swap(A.y, B.y, false, false);
      *reinterpret_cast<uint4*>(out + d * 32 + 8 * g + 8 * hh) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
    }
}

// A wave's 32 output rows × 64 bf16 (the same two transposed accumulators as store_row64, × mul per lane) as
// FULL 128-B lines: lane (q, hh) holds a[d][4G + j] of row q, column d·32 + 8G + 4hh + j; it writes those as
// 8-B pieces into a private 4 KiB LDS region (row r's 16-B chunk c at c ^ (r & 7): conflict-free reads), reads
// back 16 B of row (l >> 3) + 8i, chunk l & 7, and each store instruction writes 8 rows × one whole line.
// store_row64's pieces cover a quarter line per row and instruction (the GEMMs measured half-line stores
// 2-3 % slower than whole lines, profiles/r6_lines).  Rows >= nvalid are not stored.  `lds` must be free of
// other waves' traffic; the region is reused at once by the same wave (its LDS operations run in order).
__device__ __forceinline__ void store_tile64_lines(uint16_t* out0, size_t ld, int nvalid, const f32x16_t (&a)[2],
                                                   float mul, int lane, char* lds) {
  const int q = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int G = 0; G < 4; ++G) {
      const float v[4] = {a[d][4 * G] * mul, a[d][4 * G + 1] * mul, a[d][4 * G + 2] * mul, a[d][4 * G + 3] * mul};
      const int c = d * 4 + G;
      *reinterpret_cast<uint2*>(lds + q * 128 + ((c ^ (q & 7)) << 4) + hh * 8) = hq_pack4(v);
    }
  const int c = lane & 7, r0 = lane >> 3;
  uint4 w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = *reinterpret_cast<const uint4*>(lds + (r0 + 8 * i) * 128 + ((c ^ r0) << 4));
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (r0 + 8 * i < nvalid) *reinterpret_cast<uint4*>(out0 + (size_t)(r0 + 8 * i) * ld + c * 8) = w[i];
}

// store_row64 plus the same 8 bf16-rounded values per lane as e4m3 (x·inv8) at out8 (same element
// offsets, one byte each); returns this lane's |max| for the delayed-scaling amax.
__device__ __forceinline__ float store_row64_q8(uint16_t* out, uint8_t* out8, const f32x16_t (&a)[2], float mul,
                                                float inv8, int hh) {
  float amax = 0.f;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      const float va[4] = {a[d][4 * g] * mul, a[d][4 * g + 1] * mul, a[d][4 * g + 2] * mul, a[d][4 * g + 3] * mul};
      const float vb[4] = {a[d][4 * g + 4] * mul, a[d][4 * g + 5] * mul, a[d][4 * g + 6] * mul, a[d][4 * g + 7] * mul};
      const uint2 A = hq_pack4(va), B = hq_pack4(vb);
      const auto r0 = __builtin_amdgcn_permlane32_swap(A.x, B.x, false, false);
      const auto r1 = __builtin_amdgcn_permlane32_swap(A.y, B.y, false, false);
      const uint4 w = make_uint4(r0[0], r1[0], r0[1], r1[1]);
      const int col = d * 32 + 8 * g + 8 * hh;
      *reinterpret_cast<uint4*>(out + col) = w;
      float f[8];
      hq_unpack8(w, f);   // quantise the bf16-rounded ctx, exactly what the bf16 copy holds
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(f[e]));
      *reinterpret_cast<uint2*>(out8 + col) = make_uint2(hq_pack_fp8x4(f, inv8), hq_pack_fp8x4(f + 4, inv8));
    }
  return amax;
}

// store_row64 plus an e5m2 copy (x·inv8) at out8 for the backward's dQ / dK / dV (the fp8 QKV dgrad's
// input), quantised from the fp32 values (one rounding; the bf16 copy is rounded separately): the four
// fp8 bytes of each 4-column half are packed BEFORE the permlane32 swap, so one swap of one dword places
// them like the bf16 words.  Saturation (only needed when this step's amax outgrew the delayed scale's 64×
// headroom) runs as a wave-uniform branch.  Returns this lane's |max| for the amax.
__device__ __forceinline__ uint32_t bf8x4_raw(float a, float b, float c, float d) {
  const uint32_t w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
}
template <bool WB = true>   // WB = false: the e5m2 copy only (no bf16 output)
__device__ __forceinline__ float store_row64_e5(uint16_t* out, uint8_t* out8, const f32x16_t (&a)[2], float mul,
                                                float inv8, int hh) {
  float amax = 0.f;   // of the scaled values (|x·mul| = |x|·|mul|)
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; r += 2) amax = fmaxf(amax, fmaxf(fabsf(a[d][r]), fabsf(a[d][r + 1])));
  amax *= fabsf(mul);
  // rare: this step's amax outgrew the scale's 64× headroom — the fp8 copy saturates to ±57344 (e5m2 would
  // overflow to inf); the bf16 copy is unaffected
  const bool sat = __any(amax * inv8 >= kHqBf8Max);
  const float lim = kHqBf8Max / inv8;
  auto q = [&](float x) { return (sat ? fminf(fmaxf(x, -lim), lim) : x) * inv8; };
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      const float va[4] = {a[d][4 * g] * mul, a[d][4 * g + 1] * mul, a[d][4 * g + 2] * mul, a[d][4 * g + 3] * mul};
      const float vb[4] = {a[d][4 * g + 4] * mul, a[d][4 * g + 5] * mul, a[d][4 * g + 6] * mul, a[d][4 * g + 7] * mul};
      const int col = d * 32 + 8 * g + 8 * hh;
      if constexpr (WB) {
        const uint2 A = hq_pack4(va), B = hq_pack4(vb);
        const auto r0 = __builtin_amdgcn_permlane32_swap(A.x, B.x, false, false);
        const auto r1 = __builtin_amdgcn_permlane32_swap(A.y, B.y, false, false);
        *reinterpret_cast<uint4*>(out + col) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
      }
      const uint32_t A8 = bf8x4_raw(q(va[0]), q(va[1]), q(va[2]), q(va[3]));
      const uint32_t B8 = bf8x4_raw(q(vb[0]), q(vb[1]), q(vb[2]), q(vb[3]));
      const auto r8 = __builtin_amdgcn_permlane32_swap(A8, B8, false, false);
      *reinterpret_cast<uint2*>(out8 + col) = make_uint2(r8[0], r8[1]);
    }
  return amax;
}

// --precision fp8, calibrated: the QKV bias gradient Σ_t dQKV[t, :] as per-wave column partials (the
// fp8 QKV weight gradient has no fused bias).  Column sums of one 32-column half of a transposed 32x32
// accumulator over the 32 lanes of each wave half (the wave's 32 tokens), as a reduce-scatter butterfly on
// VALU lane exchanges only (no LDS): lane bit 4 with v_permlane16_swap (one swap hands each 16-lane row the
// other row's half, so keep + partner = both results summed), then DPP row_ror:8 (bit 3), row_half_mirror
// (lane ^ 7: decides bit 2), quad_perm (lane ^ 2), and a final lane ^ 1 add.  Lanes l and l^1 end with the
// sum of accumulator row r = (l >> 1) & 15.  Invalid lanes (tokens past L) contribute 0.
__device__ __forceinline__ float dpp_f(float x, int ctrl_sel) {
  const int v = __float_as_int(x);
  int r;
  switch (ctrl_sel) {   // compile-time after inlining
    case 0: r = __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false); break;   // row_ror:8  (lane ^ 8)
    case 1: r = __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false); break;   // row_half_mirror (^ 7)
    case 2: r = __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false); break;    // quad_perm 2,3,0,1 (^ 2)
    default: r = __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false); break;   // quad_perm 1,0,3,2 (^ 1)
  }
  return __int_as_float(r);
}
// lanes in the (compile-time) EXEC-shaped `mask` take a, the others b: one v_cndmask_b32 on an SGPR-pair constant.
// Written as asm because hipcc rewrites the butterfly's `up ? v[i] : v[i + k]` (up = a lane bit) into a
// lane-dependent array index and lowers every such read to a 16-way v_cmp / v_cndmask chain (profiled: the
// MODE 2 dK/dV epilogue was 2,500 VALU + 750 s_nop per wave, +83 µs per layer at B = 256, L = 384)
__device__ __forceinline__ float lane_sel(uint64_t mask, float a, float b) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(mask));
  return r;
}
__device__ __forceinline__ float colsum16(const f32x16_t& a, float mul, bool valid, int lane) {
  (void)lane;
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = valid ? a[r] * mul : 0.f;
  // bit 4: rows 0/1 (and 2/3) of 16 lanes trade halves; afterwards both hold keep + partner's
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 8]), false, false);
    v[i] = __uint_as_float(t[0]) + __uint_as_float(t[1]);
  }
  // bits 3, 2, 1: keep the half selected by the lane bit, add the partner's copy of it
#pragma unroll
  for (int lvl = 0; lvl < 3; ++lvl) {
    const int k = 4 >> lvl;
    // lanes with bit (8 >> lvl) set: 0xFF00…, 0xF0F0…, 0xCCCC…
    const uint64_t up = lvl == 0 ? 0xFF00FF00FF00FF00ull : lvl == 1 ? 0xF0F0F0F0F0F0F0F0ull : 0xCCCCCCCCCCCCCCCCull;
#pragma unroll
    for (int i = 0; i < k; ++i) {
      const float send = lane_sel(up, v[i], v[i + k]);
      const float keep = lane_sel(up, v[i + k], v[i]);
      v[i] = keep + dpp_f(send, lvl);
    }
  }
  return v[0] + dpp_f(v[0], 3);
}
// both halves of a row-of-64 accumulator pair -> row `dst` (64 floats: column d·32 + acc_row(r, hh))
__device__ __forceinline__ void colsum_row64(float* dst, const f32x16_t (&a)[2], float mul, bool valid, int lane,
                                             int hh) {
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const float sum = colsum16(a[d], mul, valid, lane);
    if ((lane & 1) == 0) dst[d * 32 + acc_row((lane >> 1) & 15, hh)] = sum;
  }
}


// Packed-f32 pair (v_pk_add/mul/fma_f32 on gfx950: two lanes' worth of f32 work per VALU issue).
typedef float f2_t __attribute__((ext_vector_type(2)));

// x if bit `pos` of w is set, else +0: v_bfe_i32 sign-extends the bit to an all-ones / all-zero word and one
// v_and_b32 applies it (2 VALU per element instead of a bit test, a compare and a select)
__device__ __forceinline__ float keep_and(float x, uint32_t w, int pos) {
  return __uint_as_float(__float_as_uint(x) & (uint32_t)__builtin_amdgcn_sbfe((int)w, (unsigned)pos, 1u));
}
// bit of the forward's 16-bit keep word that holds element r of a lane's 16 (even elements in the low byte,
// odd in the high: the forward builds them as packed-pair flags, see attn_fwd_ring_kernel)
__host__ __device__ constexpr int kbit(int r) { return ((r & 1) << 3) | (r >> 1); }
typedef uint16_t u16x2_t __attribute__((ext_vector_type(2)));

// lane ^ 32 exchange without LDS: v_permlane32_swap hands each half the other half's value.
__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// max over the 16 accumulator registers as a v_max3 chain
__device__ __forceinline__ float max16(const f32x16_t& a) {
  float m = fmaxf(fmaxf(a[0], a[1]), a[2]);
#pragma unroll
  for (int r = 3; r < 15; r += 2) m = fmaxf(fmaxf(m, a[r]), a[r + 1]);
  return fmaxf(m, a[15]);
}

// Both head matrices of a kernel's prologue in ONE load phase: every thread issues all its 16-B loads
// of A and of B before the first LDS store, so the workgroup pays a single exposed HBM latency instead
// of one per matrix (with one workgroup per CU nothing else hides the prologue).
template <int NT, bool SCALE_A = false>
__device__ __forceinline__ void load_heads2(uint16_t* dstA, const uint16_t* srcA, size_t ldA, uint16_t* dstB,
                                            const uint16_t* srcB, size_t ldB, int L, int Lp, float c = 1.f) {
  constexpr int kMax = 8;
  uint4 ba[kMax], bb[kMax];
  const int n = Lp * 8;
#pragma unroll
  for (int i = 0; i < kMax; ++i) {
    const int t = threadIdx.x + i * NT;
    ba[i] = make_uint4(0, 0, 0, 0);
    bb[i] = make_uint4(0, 0, 0, 0);
    if (t < n && (t >> 3) < L) {
      ba[i] = *reinterpret_cast<const uint4*>(srcA + (size_t)(t >> 3) * ldA + (t & 7) * 8);
      bb[i] = *reinterpret_cast<const uint4*>(srcB + (size_t)(t >> 3) * ldB + (t & 7) * 8);
    }
  }
#pragma unroll
  for (int i = 0; i < kMax; ++i) {
    const int t = threadIdx.x + i * NT;
    if (t < n) {
      uint4 v = ba[i];
      if constexpr (SCALE_A) {
        float f[8];
        hq_unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= c;
        v = hq_pack8(f);
      }
      *reinterpret_cast<uint4*>(dstA + lds_off(t >> 3, (t & 7) * 8)) = v;
      *reinterpret_cast<uint4*>(dstB + lds_off(t >> 3, (t & 7) * 8)) = bb[i];
    }
  }
}

// ============================================================================ forward v3: LDS-DMA ring
// The whole-head design above keeps K and V of a head resident (96 KB at L=384), so only ONE workgroup
// fits a CU and its load prologue and store epilogue never overlap compute: measured 151 of 285 µs at
// B=256 (profiles/s3_prof/attn_lab.txt).  v3 instead:
// * a workgroup is 4 waves × 32 queries of one head; the head's K and V stream through an RNS-slot LDS
//   ring of 32-key tiles by LDS-DMA (global_load_lds, 1 KiB per wave-instruction, source-swizzled so the
//   lane-linear image is the conflict-free lds_off layout), RAHEAD tiles ahead of the consumer, with a
//   COUNTED vmcnt + raw s_barrier per tile — three workgroups per CU, so one's loads overlap the others'
//   MFMAs;
// * blockIdx is remapped so the query blocks of one head are consecutive on ONE XCD (they run together
//   and read K/V through the same L2);
// * the key-mask bias and the running row max ride in a 5th MFMA per tile: K' = [K | b_hi, b_lo, 1, 0…]
//   and Q' = [Q·c | 1, 1, −m, 0…] (bf16; b_hi + b_lo = bias·log2e to ~16 bits, m kept bf16-exact), so
//   S' = c·QKᵀ + bias − m leaves the MFMA ready for exp2 — no accumulator init, no subtraction in VALU;
// * no per-tile max and no rescale: m is the first tile's row max (a lower bound of the row max, so
//   P ≤ 2^(rowmax − m) and l ≥ 1); bf16/fp32 relative precision does not depend on magnitude, and a
//   workgroup with a row whose l exceeds 2^64 recomputes its rows on an in-kernel slow path (per-tile max
//   + rescale, per-wave LDS staging) after the fast loop.  LSE = m + log2 l.
constexpr int RW = 4;                    // waves per workgroup
constexpr int RQ = RW * 32;              // queries per workgroup
// ring slots: RAHEAD + 2 (tiles kt … kt+RAHEAD in flight plus one being drained); the Q staging block of
// the prologue aliases slots RAHEAD, RAHEAD+1, which are first restaged after the first barrier
constexpr int RTILE = 32 * D * 2;        // bytes of one 32-key tile of K (or V)
typedef __attribute__((address_space(1))) void ag_void;
typedef __attribute__((address_space(3))) void al_void;

__device__ __forceinline__ uint16_t bf16_rne(float f) { return (uint16_t)(hq_pack2(f, 0.f) & 0xFFFFu); }
// the key bias (log2 domain) exactly as the forward's 5th MFMA adds it: bf16 hi + bf16 lo
__device__ __forceinline__ float bias_l2(float kb) {
  const float x = kb * LOG2E;
  const float hi = hq_bf2f(bf16_rne(x));
  return hi + hq_bf2f(bf16_rne(x - hi));
}

// LDS-DMA of 8 rows × 128 B (rows row0..row0+7 of `src`, ld elements apart) into a lane-linear
// [rows][64] image at `dst` (wave-uniform); the source chunk is pre-swizzled so the image is lds_off().
// Inline asm on purpose (cdna_hip_programming.md §5.7): with the builtin, hipcc treats the DMA as a
// pending LDS write and drains it (vmcnt(0)) before every later ds_read_b64_tr_b16 — which would wait
// for the tiles being prefetched.  Completion is counted by hand (vmcnt(N) + barrier per tile).
__device__ __forceinline__ void dma_piece(const uint16_t* g, char* dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(al_void*)dst);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}
// element offset of this lane's 16 B inside an 8-row piece starting at image row row0 (source-swizzled)
__device__ __forceinline__ int dma_lane_off(int row0, size_t ld, int lane) {
  const int r = row0 + (lane >> 3);
  return (lane >> 3) * (int)ld + (((lane & 7) ^ swz(r)) << 3);
}
__device__ __forceinline__ void dma_rows8(const uint16_t* src, size_t ld, int row0, int rows_valid, char* dst,
                                          int lane) {
  const int r = row0 + (lane >> 3);
  const int rs = r < rows_valid ? r : rows_valid - 1;   // clamp: padded keys are masked by bias = -inf
  dma_piece(src + (size_t)rs * ld + (((lane & 7) ^ swz(r)) << 3), dst + row0 * 128);
}

// `vmcnt(n)` with a value that constant-folds once the tile loop is unrolled
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
  }
}

template <bool DROP, bool EVEN, int NT, int RAHEAD>
__global__ __launch_bounds__(RW * 64, 4) void attn_fwd_ring_kernel(const uint16_t* __restrict__ qkv,
                                                                   const float* __restrict__ key_bias,
                                                                   uint16_t* __restrict__ ctx, float* __restrict__ lse,
                                                                   uint16_t* __restrict__ mbits, int L, int nh,
                                                                   int n_qb, float c_scale, HqDropKey kd_,
                                                                   uint32_t thr, float kscale, int force_slow,
                                                                   uint8_t* __restrict__ ctx8,
                                                                   const float* __restrict__ q8,
                                                                   float* __restrict__ part8, int phase) {
  const uint32_t key = kd_.get();
  if (ctx8 != nullptr) hq_fp8_publish_scale(q8, phase);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Lp = NT > 0 ? NT * 32 : (L + 31) & ~31, n32 = Lp >> 5;
  constexpr int RNS = RAHEAD + 2;
  static_assert(RAHEAD >= 2 && RAHEAD <= 4, "ring depth (>= RW slots: per-wave slow-path / store regions)");
  char* ring = reinterpret_cast<char*>(smem);                       // [RNS][K 4 KB | V 4 KB]
  char* sQ = ring + RAHEAD * 2 * RTILE;                             // [RQ][64] bf16 = ring slots RAHEAD, +1
  uint2* sA = reinterpret_cast<uint2*>(ring + RNS * 2 * RTILE);     // [Lp]: (pk(b_hi, b_lo), pk(1, 0))
  // XCD-aware block order (bijective): blocks b, b+8, … share an XCD; give each XCD a contiguous run of
  // (head, query-block) pairs with the query block fastest, so a head's blocks are co-resident on one L2
  const int nblk = gridDim.x, ob = blockIdx.x, xcd = ob & 7, qq = nblk >> 3, rr = nblk & 7;
  const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (ob >> 3);
  const int bh = lin / n_qb, qb = lin - bh * n_qb;
  const int b = bh / nh, h = bh - b * nh;
  const int H = nh * D, ld = 3 * H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, hh = lane >> 5;
  const int qs = qb * RW + wave;                       // this wave's 32-query subtile (of the head)
  const int qi = qs * 32 + (lane & 31);
  const bool active = qs * 32 < L;                     // waves past L (last block) only help with DMA
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  HQ_DASSERT(L > 0 && L <= 512 && (NT == 0 || L == NT * 32) && bh < nblk / n_qb);

  // ---- prologue: Q block (this wave's 8 row-pieces... 32 rows = 4 pieces) + the first RAHEAD tiles
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r0 = wave * 32 + p * 8;                  // row within the workgroup's 128 queries
    const int rows = L - qb * RQ;                      // valid query rows of this block
    dma_rows8(base + (size_t)qb * RQ * ld, ld, r0, rows > 0 ? rows : 1, sQ, lane);
  }
  const int kv_off = dma_lane_off(wave * 8, ld, lane) + wave * 8 * ld;
  auto stage = [&](int kt) {                           // tile kt → slot kt % RNS: this wave's K and V piece
    char* slot = ring + (kt % RNS) * 2 * RTILE;
    const uint16_t* kb = base + H + (size_t)kt * 32 * ld;   // wave-uniform
    if (EVEN || kt * 32 + 32 <= L) {
      dma_piece(kb + kv_off, slot + wave * 8 * 128);
      dma_piece(kb + H + kv_off, slot + RTILE + wave * 8 * 128);
    } else {
      dma_rows8(kb, ld, wave * 8, L - kt * 32, slot, lane);
      dma_rows8(kb + H, ld, wave * 8, L - kt * 32, slot + RTILE, lane);
    }
  };
#pragma unroll
  for (int t = 0; t < RAHEAD; ++t)
    if (t < n32) stage(t);
  // keys past L get a FINITE −1e30 (exp2 → 0): the hh = 1 lanes read these same words as k-dims 8..15,
  // which meet zeros in Q' — finite × 0 = 0, where −inf × 0 would be NaN
  for (int t = threadIdx.x; t < Lp; t += RW * 64) {
    const float bl = t < L ? key_bias[(size_t)b * L + t] * LOG2E : -1e30f;
    const uint16_t hi = bf16_rne(bl);
    const uint16_t lo = t < L ? bf16_rne(bl - hq_bf2f(hi)) : 0;
    sA[t] = make_uint2((uint32_t)hi | ((uint32_t)lo << 16), 0x3F80u);  // (b_hi, b_lo, 1.0, 0)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  LdsOffsets lo_;
  lo_.init(lane);
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const bf16x8_t raw = *reinterpret_cast<const bf16x8_t*>(sQ + 2 * (wave * 32 * D + lo_.row[s]));
    qf[s] = prescale8(raw, c_scale);
  }
  const uint2* aug_src = sA + (lane & 31);               // hh = 1 lanes: meets zeros in Q' (k-dims 8..15)
  float m_b = 0.f;                                        // bf16-exact running max (log2 domain)
  const uint32_t qaug_w0 = hh ? 0u : 0x3F803F80u;         // (1, 1) against (b_hi, b_lo)
  uint32_t qaug_w = 0u;                                   // (−m, 0) against (1, 0); −0 until the first tile
  f32x16_t o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  f2_t l2 = {0.f, 0.f};
  const uint32_t row_idx = ((uint32_t)bh * L + (uint32_t)min(qi, L - 1)) * (uint32_t)L;
  uint16_t* my_bits = mbits + (((size_t)bh * n32 + qs) * n32) * 64 + lane;
  const f32x16_t zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool stores = DROP && active;

  // tile kt landed.  Iteration j issues stage(j + RAHEAD) (2 pieces, if it exists) then bits(j); tile kt
  // was staged in iteration kt − RAHEAD, so younger than it are the RAHEAD bit stores of iterations
  // kt − RAHEAD … kt − 1 and the stages of iterations kt − RAHEAD + 1 … kt − 1 that exist (prologue tiles
  // kt < RAHEAD were drained before the loop: any count is safe for them)
  auto wait_tile = [&](int kt, bool with_stores) {
    const int later = kt + RAHEAD - 1 < n32 ? RAHEAD - 1 : n32 - 1 - kt;
    wait_vm((with_stores ? RAHEAD : 0) + 2 * (later > 0 ? later : 0));
  };
  constexpr int UNR = NT > 0 ? NT : 1;
  if (!active) {  // waves past L (last query block): their share of the DMA and every barrier, nothing else
#pragma unroll UNR
    for (int kt = 0; kt < n32; ++kt) {
      wait_tile(kt, false);
      __builtin_amdgcn_s_barrier();
      if (kt + RAHEAD < n32) stage(kt + RAHEAD);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    (void)__syncthreads_or(0);                         // the workgroup's slow-path vote (below)
    if (ctx8 != nullptr && lane == 0) part8[blockIdx.x * RW + wave] = 0.f;   // its (empty) amax partial
    return;
  }
  // Branch-free tile loop: a per-tile rescale branch makes hipcc copy the 32 O registers across the join
  // (43 v_mov_b64 per tile measured).  m stays the first tile's row max, so every P ≤ 2^(rowmax − m); a
  // workgroup with a row whose l outgrew 2^64 redoes its rows on the slow path after the loop (never
  // triggered by BERT activations; a left-padded row with a fully masked first tile is the realistic case).
#pragma unroll UNR
  for (int kt = 0; kt < n32; ++kt) {
    wait_tile(kt, DROP);
    __builtin_amdgcn_s_barrier();
    if (kt + RAHEAD < n32) stage(kt + RAHEAD);         // its slot was last read two barriers ago
    const char* sK = ring + (kt % RNS) * 2 * RTILE;
    const uint16_t* tK = reinterpret_cast<const uint16_t*>(sK);
    const uint16_t* tV = reinterpret_cast<const uint16_t*>(sK + RTILE);
    bf16x8_t kf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) kf[s] = row8(tK, 0, lo_, s);
    const uint2 aw = aug_src[kt * 32];
    typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
    const bf16x8_t ka = __builtin_bit_cast(bf16x8_t, u32x4{aw.x, aw.y, 0u, 0u});
    const bf16x8_t qa = __builtin_bit_cast(bf16x8_t, u32x4{qaug_w0, qaug_w, 0u, 0u});
    f32x16_t acc = mfma32(kf[0], qf[0], zero16);
#pragma unroll
    for (int s = 1; s < 4; ++s) acc = mfma32(kf[s], qf[s], acc);
    acc = mfma32(ka, qa, acc);                          // + bias_k − m_q
    float sc[16];
    if (kt == 0) {                                      // first tile: the row max over the full tile
      const float mx = xor32_max(max16(acc));
      m_b = hq_bf2f(bf16_rne(mx == -INFINITY ? 0.f : mx));
      qaug_w = hh ? 0u : (uint32_t)bf16_rne(-m_b);
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = __builtin_amdgcn_exp2f(acc[r] - m_b);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = __builtin_amdgcn_exp2f(acc[r]);
    }
    {  // the softmax denominator counts every key (dropout only thins P·V); pairwise tree, not a chain
      const f2_t a0 = f2_t{sc[0], sc[1]} + f2_t{sc[2], sc[3]}, a1 = f2_t{sc[4], sc[5]} + f2_t{sc[6], sc[7]};
      const f2_t a2 = f2_t{sc[8], sc[9]} + f2_t{sc[10], sc[11]}, a3 = f2_t{sc[12], sc[13]} + f2_t{sc[14], sc[15]};
      l2 += (a0 + a1) + (a2 + a3);
    }
    // dropout on the PACKED bf16 P: element pair p = (2p, 2p + 1) is one bf16x2 word of pack_b and one
    // 32-bit hash (low half → element 2p).  Packed u16 saturating ops turn the hash halves into keep flags
    // (z = sat(thr − h) is 0 iff kept; sat(1 − z) is the flag) and the flags into a per-half AND mask —
    // 5 VALU per pair instead of two compares, two f32 selects and a bit insert per element.
    uint32_t km[8];
    if constexpr (DROP) {
      uint32_t kb = 0;   // keep flags: element 2p at bit p, element 2p + 1 at bit 16 + p
      if constexpr (EVEN) {
        uint32_t pk = (((row_idx >> 1) + (uint32_t)kt * 16u) ^ key) ^ (2u * (uint32_t)hh);
        pk ^= pk >> 16;                                   // hq_mix24's first xorshift, once per tile
        const u16x2_t thr2 = {(uint16_t)thr, (uint16_t)thr}, one2 = {1, 1}, zero2 = {0, 0};
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int ip = 0; ip < 2; ++ip) {
            const uint32_t hsh = hq_mix24_post(pk ^ (uint32_t)(4 * g + ip));   // = hq_mix24(pair ^ key)
            const int p = 2 * g + ip;
            const u16x2_t z = __builtin_elementwise_sub_sat(thr2, __builtin_bit_cast(u16x2_t, hsh));
            const u16x2_t kf = __builtin_elementwise_sub_sat(one2, z);
            km[p] = __builtin_bit_cast(uint32_t, zero2 - kf);
            kb |= __builtin_bit_cast(uint32_t, kf) << p;
          }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t idx0 = row_idx + kt * 32 + 8 * g + 4 * hh;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * g + i;
            kb |= (uint32_t)hq_keep(idx0 + i, key, thr) << ((r >> 1) + 16 * (r & 1));
          }
        }
#pragma unroll
        for (int p = 0; p < 8; ++p)
          km[p] = ((kb >> p) & 1u ? 0xFFFFu : 0u) | ((kb >> (16 + p)) & 1u ? 0xFFFF0000u : 0u);
      }
      // stored word: element r at bit kbit(r) (bytes 0 and 2 of kb)
      my_bits[(size_t)kt * 64] = (uint16_t)((kb & 0xFFu) | ((kb >> 8) & 0xFF00u));
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t pb = pack_b(sc, s);
      if constexpr (DROP) {
        typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
        u32x4 u = __builtin_bit_cast(u32x4, pb);
        u &= u32x4{km[4 * s], km[4 * s + 1], km[4 * s + 2], km[4 * s + 3]};
        pb = __builtin_bit_cast(bf16x8_t, u);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) o[d] = mfma32(tr8(tV, 0, lo_, s, d), pb, o[d]);
    }
  }
  float l_tot = xor32_sum(l2.x + l2.y);
  // slow-path vote: any row of the workgroup whose l left [1, 2^64) (P could have overflowed) — or every
  // workgroup when force_slow (tests) — recomputes with a per-tile max and rescale.  The ring is idle now
  // (every tile consumed; only bit stores may be in flight), so each wave stages K/V in a private 8 KB of it.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (__syncthreads_or(force_slow || (qi < L && !(l_tot < 0x1p64f)))) {
    uint16_t* pK = reinterpret_cast<uint16_t*>(ring + wave * 2 * RTILE);
    uint16_t* pV = pK + 32 * D;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
    l2 = f2_t{0.f, 0.f};
    float m_run = -INFINITY;
    const uint16_t* kbase = base + H;
    for (int kt = 0; kt < n32; ++kt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // private staging: plain loads, ds_write; LDS is in order per wave
        const int r = i * 8 + (lane >> 3), c = (lane & 7) * 8;
        const int kr = min(kt * 32 + r, L - 1);
        const uint4 kv = *reinterpret_cast<const uint4*>(kbase + (size_t)kr * ld + c);
        const uint4 vv = *reinterpret_cast<const uint4*>(kbase + H + (size_t)kr * ld + c);
        *reinterpret_cast<uint4*>(pK + lds_off(r, c)) = kv;
        *reinterpret_cast<uint4*>(pV + lds_off(r, c)) = vv;
      }
      bf16x8_t kf[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) kf[s] = row8(pK, 0, lo_, s);
      const uint2 aw = aug_src[kt * 32];
      typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
      const bf16x8_t ka = __builtin_bit_cast(bf16x8_t, u32x4{aw.x, aw.y, 0u, 0u});
      const bf16x8_t qa = __builtin_bit_cast(bf16x8_t, u32x4{qaug_w0, 0u, 0u, 0u});  // m = 0: exact scores
      f32x16_t acc = mfma32(kf[0], qf[0], zero16);
#pragma unroll
      for (int s = 1; s < 4; ++s) acc = mfma32(kf[s], qf[s], acc);
      acc = mfma32(ka, qa, acc);
      const float m_new = fmaxf(m_run, xor32_max(max16(acc)));
      const float ms = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run - ms);
      m_run = m_new;
      l2 *= f2_t{alpha, alpha};
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
      float sc[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sc[r] = __builtin_amdgcn_exp2f(acc[r] - ms);
        l2.x += sc[r];
      }
      if constexpr (DROP) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t idx0 = row_idx + kt * 32 + 8 * g + 4 * hh;
#pragma unroll
          for (int i = 0; i < 4; ++i) sc[4 * g + i] = hq_keep(idx0 + i, key, thr) ? sc[4 * g + i] : 0.f;
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t pb = pack_b(sc, s);
#pragma unroll
        for (int d = 0; d < 2; ++d) o[d] = mfma32(tr8(pV, 0, lo_, s, d), pb, o[d]);
      }
    }
    m_b = m_run == -INFINITY ? 0.f : m_run;
    l_tot = xor32_sum(l2.x + l2.y);
  }
  const float inv = (DROP ? kscale : 1.f) / l_tot;
  if (ctx8 != nullptr) {   // --precision fp8: ctx also in e4m3 for the out-projection (delayed scaling)
    const float s8 = hq_fp8_delayed_scale(q8, phase);
    float amax = 0.f;
    if (qi < L) {
      const size_t row = ((size_t)b * L + qi) * H + h * D;
      amax = store_row64_q8(ctx + row, ctx8 + row, o, inv, 1.f / s8, hh);
      if (hh == 0) lse[(size_t)bh * L + qi] = (m_b + __builtin_amdgcn_logf(l_tot)) * LN2;
    }
    amax = hq_wave_max(amax);   // -> this wave's partial slot, folded by hq_fp8_amax_fold (no atomics)
    if (lane == 0) part8[blockIdx.x * RW + wave] = amax;
    return;
  }
  // ctx as whole 128-B lines through this wave's slow-path region of the ring (every tile was consumed before
  // the vote's barrier, and no other wave touches this region)
  store_tile64_lines(ctx + ((size_t)b * L + qs * 32) * H + h * D, H, L - qs * 32, o, inv, lane,
                     ring + wave * 2 * RTILE);
  if (qi < L && hh == 0) lse[(size_t)bh * L + qi] = (m_b + __builtin_amdgcn_logf(l_tot)) * LN2;  // v_log_f32 = log2
}

// ============================================================================ backward v3
// Same ideas as the ring forward, for the two backward kernels (dQ first — it also produces δ — then
// dK/dV, which reads δ):
// * dQ: 4-wave workgroups of 32 queries each; K and V tiles stream through the LDS-DMA ring; Q·c, dO
//   and the dropout words of the wave's rows are loaded before the ring starts; bias and −LSE ride in the
//   5th MFMA (A' = [K | b_hi, b_lo, 1, 1, 1], B' = [Q·c | 1, 1, −l_hi, −l_mid, −l_lo]: LSE to ~24 bits).
// * dK/dV: ONE pass (S, dP, dV, dK per tile: 17 MFMAs instead of the two-pass 20) in 4-wave workgroups
//   of 32 keys each; Q·c, dO, LSE and δ of each 32-query tile are register-staged into a 2-slot LDS
//   ring (issue the loads before the tile's MFMAs, write after: T14) — Q must be prescaled on its way
//   into LDS to reproduce the forward's rounded Q·c, which an LDS-DMA cannot do.
__device__ __forceinline__ void split3(float x, uint16_t& hi, uint16_t& mid, uint16_t& lo) {
  hi = bf16_rne(x);
  const float r = x - hq_bf2f(hi);
  mid = bf16_rne(r);
  lo = bf16_rne(r - hq_bf2f(mid));
}

// MODE 0: bf16 dQKV; 1: bf16 + e5m2 copy (fp8 backward, calibrating); 2: e5m2 only + column partials of the
// QKV bias gradient into bpart [B·n32][3H] (fp8 backward, calibrated: every consumer reads the e5m2 copy)
template <bool DROP, int NT, int RAHEAD, int MODE = 0>
__global__ __launch_bounds__(RW * 64, MODE == 0 && NT > 0 ? 4 : 3) void attn_bwd_dq_ring_kernel(
    const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ dctx, const uint16_t* __restrict__ ctx,
    const float* __restrict__ lse, const float* __restrict__ key_bias, const uint16_t* __restrict__ mbits,
    float* __restrict__ delta, uint16_t* __restrict__ dqkv, int L, int nh, int n_qb, float c_scale, float scale,
    float kscale, uint8_t* __restrict__ dqkv8, const float* __restrict__ q8, float* __restrict__ part8, int phase,
    float* __restrict__ bpart) {
  constexpr bool Q8 = MODE > 0;
  if constexpr (Q8) hq_fp8_publish_scale(q8, phase, kHqBf8Max);   // dQKV's state (dK/dV share it)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int RNS = RAHEAD + 2;
  const int Lp = NT > 0 ? NT * 32 : (L + 31) & ~31, n32 = Lp >> 5;
  char* ring = reinterpret_cast<char*>(smem);                       // [RNS][K 4 KB | V 4 KB]
  uint32_t* sA = reinterpret_cast<uint32_t*>(ring + RNS * 2 * RTILE);  // [Lp] A' word 0 (b_hi,b_lo); 1-3 constant
  uint16_t* sM = reinterpret_cast<uint16_t*>(sA + Lp);              // [RW][n32][64] dropout words
  const int nblk = gridDim.x, ob = blockIdx.x, xcd = ob & 7, qq = nblk >> 3, rr = nblk & 7;
  const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (ob >> 3);
  const int bh = lin / n_qb, qb = lin - bh * n_qb;
  const int b = bh / nh, h = bh - b * nh;
  const int H = nh * D, ld = 3 * H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, hh = lane >> 5;
  const int qs = qb * RW + wave;
  const int qi = qs * 32 + (lane & 31);
  const bool active = qs * 32 < L;
  const bool qok = qi < L;
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  HQ_DASSERT(L > 0 && L <= 512 && (NT == 0 || L == NT * 32));

  // ---- prologue (plain loads, issued before any LDS-DMA): Q·c, dO, δ = rowsum(dO·O), −LSE words, bits
  const int qr = qok ? qi : L - 1;
  const size_t orow = ((size_t)b * L + qr) * H + h * D;
  bf16x8_t qf[4], of[4];
  float dpart = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = prescale8(*reinterpret_cast<const bf16x8_t*>(base + (size_t)qr * ld + 16 * s + 8 * hh), c_scale);
    of[s] = *reinterpret_cast<const bf16x8_t*>(dctx + orow + 16 * s + 8 * hh);
    float x[8], y[8];
    hq_unpack8(__builtin_bit_cast(uint4, of[s]), x);
    hq_unpack8(*reinterpret_cast<const uint4*>(ctx + orow + 16 * s + 8 * hh), y);
#pragma unroll
    for (int j = 0; j < 8; ++j) dpart += x[j] * y[j];
  }
  const float dlt = xor32_sum(dpart);  // δ over all 64 dims (lanes q and q+32 hold 32 each)
  if (active && qok && hh == 0) delta[(size_t)bh * L + qi] = dlt;
  const float lq = lse[(size_t)bh * L + qr] * LOG2E;
  uint16_t lh, lm, ll;
  split3(-lq, lh, lm, ll);
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
  const u32x4 qaw = hh ? u32x4{0u, 0u, 0u, 0u}
                       : u32x4{0x3F803F80u, (uint32_t)lh | ((uint32_t)lm << 16), (uint32_t)ll, 0u};
  const bf16x8_t qa = __builtin_bit_cast(bf16x8_t, qaw);
  if constexpr (DROP) {
    constexpr int kMaxT = 16;
    uint16_t mw[kMaxT];
    const uint16_t* gbits = mbits + (((size_t)bh * n32 + qs) * n32) * 64 + lane;
#pragma unroll
    for (int t = 0; t < kMaxT; ++t)
      if (active && t < n32) mw[t] = gbits[(size_t)t * 64];
#pragma unroll
    for (int t = 0; t < kMaxT; ++t)
      if (active && t < n32) sM[(wave * n32 + t) * 64 + lane] = mw[t];
  }
  for (int t = threadIdx.x; t < Lp; t += RW * 64) {  // finite −1e30 past L: see the forward
    const float bl = t < L ? key_bias[(size_t)b * L + t] * LOG2E : -1e30f;
    const uint16_t hi = bf16_rne(bl);
    const uint16_t lo = t < L ? bf16_rne(bl - hq_bf2f(hi)) : 0;
    sA[t] = (uint32_t)hi | ((uint32_t)lo << 16);
  }
  const int kv_off = dma_lane_off(wave * 8, ld, lane) + wave * 8 * ld;
  auto stage = [&](int kt) {
    char* slot = ring + (kt % RNS) * 2 * RTILE;
    const uint16_t* kb = base + H + (size_t)kt * 32 * ld;
    if (NT > 0 || kt * 32 + 32 <= L) {
      dma_piece(kb + kv_off, slot + wave * 8 * 128);
      dma_piece(kb + H + kv_off, slot + RTILE + wave * 8 * 128);
    } else {
      dma_rows8(kb, ld, wave * 8, L - kt * 32, slot, lane);
      dma_rows8(kb + H, ld, wave * 8, L - kt * 32, slot + RTILE, lane);
    }
  };
#pragma unroll
  for (int t = 0; t < RAHEAD; ++t)
    if (t < n32) stage(t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  auto wait_tile = [&](int kt) {  // only the two DMA pieces of each later staged tile are younger
    const int later = kt + RAHEAD - 1 < n32 ? RAHEAD - 1 : n32 - 1 - kt;
    wait_vm(2 * (later > 0 ? later : 0));
  };
  constexpr int UNR = NT > 0 ? NT : 1;
  if (!active) {
#pragma unroll UNR
    for (int kt = 0; kt < n32; ++kt) {
      wait_tile(kt);
      __builtin_amdgcn_s_barrier();
      if (kt + RAHEAD < n32) stage(kt + RAHEAD);
    }
    if (Q8 && lane == 0) part8[blockIdx.x * RW + wave] = 0.f;   // its (empty) amax partial
    return;
  }
  LdsOffsets lo_;
  lo_.init(lane);
  const uint32_t* aug_src = sA + (lane & 31);
  const uint16_t* my_bits = sM + wave * n32 * 64 + lane;
  const f32x16_t zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x16_t dq[2] = {zero16, zero16};
  const f2_t dl2 = {dlt, dlt};
#pragma unroll UNR
  for (int kt = 0; kt < n32; ++kt) {
    wait_tile(kt);
    __builtin_amdgcn_s_barrier();
    if (kt + RAHEAD < n32) stage(kt + RAHEAD);
    const char* sK = ring + (kt % RNS) * 2 * RTILE;
    const uint16_t* tK = reinterpret_cast<const uint16_t*>(sK);
    const uint16_t* tV = reinterpret_cast<const uint16_t*>(sK + RTILE);
    const bf16x8_t ka = __builtin_bit_cast(bf16x8_t, u32x4{aug_src[kt * 32], 0x3F803F80u, 0x3F80u, 0u});
    // without dropout the MFMA groups run at s_setprio 1 (backward −9 % at p = 0, profiles/r6_attn_prio_not_adopted;
    // with dropout it gains nothing, and dK/dV and the forward lose with it)
    if constexpr (!DROP) __builtin_amdgcn_s_setprio(1);
    f32x16_t s_acc = mfma32(row8(tK, 0, lo_, 0), qf[0], zero16);
#pragma unroll
    for (int s = 1; s < 4; ++s) s_acc = mfma32(row8(tK, 0, lo_, s), qf[s], s_acc);
    s_acc = mfma32(ka, qa, s_acc);                      // S' = c·q·k + bias − lse (log2 domain)
    f32x16_t p_acc = mfma32(row8(tV, 0, lo_, 0), of[0], zero16);
#pragma unroll
    for (int s = 1; s < 4; ++s) p_acc = mfma32(row8(tV, 0, lo_, s), of[s], p_acc);
    if constexpr (!DROP) __builtin_amdgcn_s_setprio(0);
    uint32_t bits = 0xFFFFu;
    f2_t ksc = {1.f, 1.f};
    if constexpr (DROP) {
      bits = (uint32_t)my_bits[kt * 64];
      ksc = f2_t{kscale, kscale};
    }
    float ds[16];
#pragma unroll
    for (int r = 0; r < 16; r += 2) {  // dS = P·(dP·mask·ksc − δ): mask as an all-ones/zero AND (v_bfe_i32)
      const f2_t P = {__builtin_amdgcn_exp2f(s_acc[r]), __builtin_amdgcn_exp2f(s_acc[r + 1])};
      f2_t dp = {p_acc[r], p_acc[r + 1]};
      if constexpr (DROP) dp = f2_t{keep_and(dp.x, bits, kbit(r)), keep_and(dp.y, bits, kbit(r + 1))};
      const f2_t v = (dp * ksc - dl2) * P;
      ds[r] = v.x; ds[r + 1] = v.y;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8_t sb = pack_b(ds, s);
      if constexpr (!DROP) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int d = 0; d < 2; ++d) dq[d] = mfma32(tr8(tK, 0, lo_, s, d), sb, dq[d]);
      if constexpr (!DROP) __builtin_amdgcn_s_setprio(0);
    }
  }
  const size_t orow_q = ((size_t)b * L + qi) * ld + h * D;
  if constexpr (Q8) {   // --precision fp8: dQ also as e5m2 for the QKV dgrad (delayed scaling)
    const float inv8 = 1.f / hq_fp8_delayed_scale(q8, phase, kHqBf8Max);
    float amax = qok ? store_row64_e5<MODE == 1>(dqkv + orow_q, dqkv8 + orow_q, dq, scale, inv8, hh) : 0.f;
    amax = hq_wave_max(amax);
    if (lane == 0) part8[blockIdx.x * RW + wave] = amax;
    if constexpr (MODE == 2) colsum_row64(bpart + ((size_t)b * n32 + qs) * 3 * H + h * D, dq, scale, qok, lane, hh);
    return;
  }
  // (dQ keeps the quarter-line store_row64: the staged whole-line form pushed this 128-VGPR loop into 43 spills)
  if (qok) store_row64(dqkv + orow_q, dq, scale, hh);
}

// dK/dV: keys on the lanes.  Per 32-query tile: S = Q'·Kᵀ (+ aug: −LSE, bias), dP = dO·Vᵀ, then
// dVᵀ += dOᵀ·(P∘mask) and dKᵀ += Q'ᵀ·dS with P/dS fed from the accumulators (no LDS round trip).
template <bool DROP, int NT, int MODE = 0>   // MODE: as attn_bwd_dq_ring_kernel
__global__ __launch_bounds__(RW * 64, 2) void attn_bwd_dkdv_ring_kernel(
    const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ dctx, const float* __restrict__ lse,
    const float* __restrict__ delta, const float* __restrict__ key_bias, const uint16_t* __restrict__ mbits,
    uint16_t* __restrict__ dqkv, int L, int nh, int n_kb, float c_scale, float scale, float kscale,
    uint8_t* __restrict__ dqkv8, const float* __restrict__ q8, float* __restrict__ part8, int phase,
    float* __restrict__ bpart) {
  constexpr bool Q8 = MODE > 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // slot: Q' [32][64] 4 KB | dO [32][64] 4 KB | A' words [32] uint4 512 B | δ [32] f32 128 B | bits [RW][64] u16
  constexpr int SLOT = 2 * RTILE + 512 + 128 + RW * 128;
  static_assert(2 * SLOT >= RW * 4096, "dK/dV store staging: 4 KiB per wave in the two slots");
  const int Lp = NT > 0 ? NT * 32 : (L + 31) & ~31, n32 = Lp >> 5;
  const int nblk = gridDim.x, ob = blockIdx.x, xcd = ob & 7, qq = nblk >> 3, rr = nblk & 7;
  const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (ob >> 3);
  const int bh = lin / n_kb, kbk = lin - bh * n_kb;
  const int b = bh / nh, h = bh - b * nh;
  const int H = nh * D, ld = 3 * H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, hh = lane >> 5;
  const int tid = threadIdx.x;
  const int ks_idx = kbk * RW + wave;                  // this wave's 32-key subtile
  const int kj = ks_idx * 32 + (lane & 31);
  const bool active = ks_idx * 32 < L;
  const bool kok = kj < L;
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  HQ_DASSERT(L > 0 && L <= 512 && (NT == 0 || L == NT * 32));

  // per-wave key fragments (B operands of S and dP) and the B' words (1,1,1,b_hi | b_lo,0,…)
  const int kr = kok ? kj : L - 1;
  bf16x8_t kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8_t*>(base + (size_t)kr * ld + H + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const bf16x8_t*>(base + (size_t)kr * ld + 2 * H + 16 * s + 8 * hh);
  }
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
  bf16x8_t kaug;
  {
    const float bl = kok ? key_bias[(size_t)b * L + kj] * LOG2E : -1e30f;
    const uint16_t bhi = bf16_rne(bl), blo = kok ? bf16_rne(bl - hq_bf2f(bhi)) : 0;
    const u32x4 w = hh ? u32x4{0u, 0u, 0u, 0u}
                       : u32x4{0x3F803F80u, 0x3F80u | ((uint32_t)bhi << 16), (uint32_t)blo, 0u};
    kaug = __builtin_bit_cast(bf16x8_t, w);
  }
  // register staging of query tile t: thread tid → row tid>>3, 16-B chunk tid&7 of Q and dO; threads
  // 0..31 the A' words (−l_hi,−l_mid | −l_lo,1 | 1,0 | 0) of query tid, 32..63 δ; each wave its bit words.
  // Three tiles in flight in registers (HBM latency under load ≈ 2-3 tile bodies); two LDS slots.
  const int srow = tid >> 3, schunk = tid & 7;
  struct Stage {
    uint4 q, o;
    float l;
    uint16_t bits;
  };
  auto issue = [&](int t, Stage& st) {
    const int q = min(t * 32 + srow, L - 1);
    st.q = *reinterpret_cast<const uint4*>(base + (size_t)q * ld + schunk * 8);
    st.o = *reinterpret_cast<const uint4*>(dctx + ((size_t)b * L + q) * H + h * D + schunk * 8);
    // every thread issues every load (wave 0's lse/δ values are the ones committed; the other waves load
    // them redundantly): exec-masked loads would make hipcc's vmcnt counting assume they were skipped and
    // wait for a tile too many
    {
      const int qq2 = min(t * 32 + (lane & 31), L - 1);
      st.l = (lane < 32 ? lse : delta)[(size_t)bh * L + qq2];
      if (t * 32 + (lane & 31) >= L) st.l = lane < 32 ? 1e30f : 0.f;  // queries past L: P = 0 (finite: split3)
    }
    st.bits = 0;
    if constexpr (DROP) st.bits = mbits[(((size_t)bh * n32 + t) * n32 + min(ks_idx, n32 - 1)) * 64 + lane];
  };
  auto slot_of = [&](int t) { return (t & 1) * SLOT; };
  auto commit = [&](int t, const Stage& st) {
    char* slot = reinterpret_cast<char*>(smem) + slot_of(t);
    uint16_t* sq = reinterpret_cast<uint16_t*>(slot);
    uint16_t* so = sq + 32 * D;
    float f[8];
    hq_unpack8(st.q, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= c_scale;       // Q·c rounded exactly as the forward's prescale8
    *reinterpret_cast<uint4*>(sq + lds_off(srow, schunk * 8)) = hq_pack8(f);
    *reinterpret_cast<uint4*>(so + lds_off(srow, schunk * 8)) = st.o;
    if (tid < 32) {
      uint16_t lh, lm, ll;
      split3(-st.l * LOG2E, lh, lm, ll);
      reinterpret_cast<uint4*>(slot + 2 * RTILE)[tid] =
          make_uint4((uint32_t)lh | ((uint32_t)lm << 16), (uint32_t)ll | (0x3F80u << 16), 0x3F80u, 0u);
    } else if (tid < 64) {
      reinterpret_cast<float*>(slot + 2 * RTILE + 512)[tid - 32] = st.l;
    }
    if constexpr (DROP) reinterpret_cast<uint16_t*>(slot + 2 * RTILE + 640)[wave * 64 + lane] = st.bits;
  };
  LdsOffsets lo_;
  lo_.init(lane);
  const f32x16_t zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x16_t dv[2] = {zero16, zero16}, dk[2] = {zero16, zero16};
  const int krel = lane & 31;
  const int hh_f = (krel >> 2) & 1;
  const int r_f = kbit((krel & 3) + 4 * (krel >> 3));   // bit position in the forward's keep word
  const float ksc = DROP ? kscale : 1.f;
  const f2_t ksc2 = {ksc, ksc};
  // S = Q'·Kᵀ (+ bias_k − lse_q through the A'/B' words) and dP = dO·Vᵀ of tile t.  All eight operand reads are
  // issued before the first MFMA (sched_barrier): left to itself hipcc reads each operand just before its
  // MFMA and waits lgkmcnt(0) there, exposing the LDS latency once per MFMA.
  auto scores = [&](int t, f32x16_t& s_acc, f32x16_t& p_acc) {
    const char* slot = reinterpret_cast<const char*>(smem) + slot_of(t);
    const uint16_t* tq = reinterpret_cast<const uint16_t*>(slot);
    const uint16_t* to = tq + 32 * D;
    bf16x8_t fq[4], fo[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      fq[s] = row8(tq, 0, lo_, s);
      fo[s] = row8(to, 0, lo_, s);
    }
    const uint4 aw = reinterpret_cast<const uint4*>(slot + 2 * RTILE)[hh ? 0 : krel];
    __builtin_amdgcn_sched_barrier(0);
    const bf16x8_t qa = hh ? bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0} : __builtin_bit_cast(bf16x8_t, u32x4{aw.x, aw.y, aw.z, aw.w});
    s_acc = mfma32(fq[0], kf[0], zero16);
    p_acc = mfma32(fo[0], vf[0], zero16);
#pragma unroll
    for (int s = 1; s < 4; ++s) {
      s_acc = mfma32(fq[s], kf[s], s_acc);
      p_acc = mfma32(fo[s], vf[s], p_acc);
    }
    s_acc = mfma32(qa, kaug, s_acc);                   // + bias_k − lse_q
  };
  // P, dS of tile t from its accumulators, then dVᵀ += dOᵀ·(P∘mask), dKᵀ += Q'ᵀ·dS
  auto grads = [&](int t, const f32x16_t& s_acc, const f32x16_t& p_acc) {
    const char* slot = reinterpret_cast<const char*>(smem) + slot_of(t);
    const uint16_t* tq = reinterpret_cast<const uint16_t*>(slot);
    const uint16_t* to = tq + 32 * D;
    // mask: the forward word of fwd-lane l' = q + 32·hh' holds bit r' for key acc_row(r', hh'); this lane
    // (key krel) needs, for query rows acc_row(r, hh) = 8g + 4hh + i, bit r_f of the words of fwd-lanes
    // 8g + 4hh + i + 32·hh_f: four consecutive words per g, one 8-byte LDS read per g
    const uint16_t* wsrc = reinterpret_cast<const uint16_t*>(slot + 2 * RTILE + 640) + wave * 64 + 4 * hh + 32 * hh_f;
    const float* sdl = reinterpret_cast<const float*>(slot + 2 * RTILE + 512);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      // this half's dV / dK operands read ahead of the exp / mask VALU that produces the other operand
      bf16x8_t ov[2], oq[2];
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        ov[d] = tr8(to, 0, lo_, s, d);
        oq[d] = tr8(tq, 0, lo_, s, d);
      }
      __builtin_amdgcn_sched_barrier(0);
      float pd[8], dsv[8];
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        const int g = 2 * s + gg;
        const float4 d4 = *reinterpret_cast<const float4*>(sdl + 8 * g + 4 * hh);
        const f2_t dl[2] = {f2_t{d4.x, d4.y}, f2_t{d4.z, d4.w}};
        float P[4], dp[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          P[i] = __builtin_amdgcn_exp2f(s_acc[4 * g + i]);
          dp[i] = p_acc[4 * g + i];
        }
        // keep bits as AND masks: pd = P·mask (kscale is applied once, at the dV store), dS = P·(dP·mask·ksc − δ)
        float pm[4] = {P[0], P[1], P[2], P[3]};
        if constexpr (DROP) {
          const uint64_t w = *reinterpret_cast<const uint64_t*>(wsrc + 8 * g);
          const uint32_t wl = (uint32_t)w, wh = (uint32_t)(w >> 32);
          const int pos[4] = {r_f, r_f + 16, r_f, r_f + 16};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            pm[i] = keep_and(P[i], i < 2 ? wl : wh, pos[i]);
            dp[i] = keep_and(dp[i], i < 2 ? wl : wh, pos[i]);
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f2_t Pj = {P[2 * j], P[2 * j + 1]}, dpj = {dp[2 * j], dp[2 * j + 1]};
          const f2_t v = (dpj * ksc2 - dl[j]) * Pj;
          pd[4 * gg + 2 * j] = pm[2 * j];
          pd[4 * gg + 2 * j + 1] = pm[2 * j + 1];
          dsv[4 * gg + 2 * j] = v.x;
          dsv[4 * gg + 2 * j + 1] = v.y;
        }
      }
      const bf16x8_t pb = pack_b(pd, 0), sb = pack_b(dsv, 0);
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        dv[d] = mfma32(ov[d], pb, dv[d]);
        dk[d] = mfma32(oq[d], sb, dk[d]);
      }
    }
  };
  // Tile t lives in register set st[t % 3] (compile-time index in the unrolled NT > 0 loop: a rotation by
  // copies would make hipcc wait for the NEWER tile's loads before each copy); the rolled NT = 0 loop
  // rotates by copies (one tile less lookahead).
  Stage st[3];
  issue(0, st[0]);
  if (n32 > 1) issue(1, st[1]);
  if (n32 > 2) issue(2, st[2]);
  constexpr int UNR = NT > 0 ? NT : 1;
  {
    commit(0, st[0]);
    __syncthreads();
    if constexpr (NT > 0) {
      if (n32 > 3) issue(3, st[0]);
    } else {
      st[0] = st[1];
      st[1] = st[2];
      if (n32 > 3) issue(3, st[2]);
    }
#pragma unroll UNR
    for (int t = 0; t < n32; ++t) {
      if constexpr (NT > 0) {
        // tile t+1 into the other slot BEFORE this tile's work, so its LDS writes overlap the MFMA chains: that
        // slot's last reader (tile t-1) finished before the previous barrier
        if (t + 1 < n32) {
          commit(t + 1, st[(t + 1) % 3]);
          if (t + 4 < n32) issue(t + 4, st[(t + 1) % 3]);
        }
      }
      if (active) {
        f32x16_t s_acc, p_acc;
        scores(t, s_acc, p_acc);
        grads(t, s_acc, p_acc);
      }
      if (t + 1 < n32) {                                  // the other slot: last read before this barrier
        if constexpr (NT > 0) {
          __syncthreads();
        } else {
          commit(t + 1, st[0]);
          __syncthreads();
          st[0] = st[1];
          st[1] = st[2];
          if (t + 4 < n32) issue(t + 4, st[2]);
        }
      }
    }
  }
  const size_t orow_k = ((size_t)b * L + kj) * ld + h * D;
  if constexpr (Q8) {   // dK, dV also as e5m2; partial slots after the dQ kernel's
    const float inv8 = 1.f / hq_fp8_delayed_scale(q8, phase, kHqBf8Max);
    float amax = 0.f;
    if (active && kok) {
      amax = store_row64_e5<MODE == 1>(dqkv + orow_k + 2 * H, dqkv8 + orow_k + 2 * H, dv, ksc, inv8, hh);
      amax = fmaxf(amax, store_row64_e5<MODE == 1>(dqkv + orow_k + H, dqkv8 + orow_k + H, dk, LN2, inv8, hh));
    }
    amax = hq_wave_max(amax);
    if (lane == 0) part8[(gridDim.x + blockIdx.x) * RW + wave] = amax;
    if constexpr (MODE == 2) {
      if (active) {   // every key subtile < n32 is active (L ≤ 32·n32): each partial row is written once
        float* row = bpart + ((size_t)b * n32 + ks_idx) * 3 * H + h * D;
        colsum_row64(row + 2 * H, dv, ksc, kok, lane, hh);
        colsum_row64(row + H, dk, LN2, kok, lane, hh);
      }
    }
    return;
  }
  // dV, dK as whole 128-B lines: every wave is past its last slot read after this barrier; 4 KiB per wave
  __syncthreads();
  if (active) {
    uint16_t* out = dqkv + ((size_t)b * L + ks_idx * 32) * ld + h * D;
    char* reg = reinterpret_cast<char*>(smem) + wave * 4096;
    store_tile64_lines(out + 2 * H, ld, L - ks_idx * 32, dv, ksc, lane, reg);   // pd carried the mask only
    store_tile64_lines(out + H, ld, L - ks_idx * 32, dk, LN2, lane, reg);       // Q' = c·Q, c = scale·log2e
  }
  (void)orow_k;
}

}  // namespace

size_t hq_attn_mask_bytes(int B, int L, int nh) {
  const size_t n32 = (size_t)(L + 31) / 32;
  return (size_t)B * nh * n32 * n32 * 64 * sizeof(uint16_t);
}


// HQ_ATTN_FORCE_SLOW=1 / attn_set_force_slow(1): every workgroup of the ring forward takes its slow path
// (tests only: the rare rescale branch gets its own coverage, kernel playbook rule 26)
static int g_attn_force_slow = [] {
  const char* e = getenv("HQ_ATTN_FORCE_SLOW");
  return e && atoi(e) ? 1 : 0;
}();
void hq_attn_set_force_slow(int v) { g_attn_force_slow = v ? 1 : 0; }

void hq_attn_fwd(const uint16_t* qkv, const float* key_bias, uint16_t* ctx, float* lse, uint16_t* mbits, int B, int L,
                 int nh, int dh, float p, uint32_t seed, uint32_t opid, float scale, hipStream_t s, uint8_t* ctx8,
                 float* q8, int phase) {
  if (dh != D || L > 512) { fprintf(stderr, "hq_attn_fwd: head_dim %d / L %d unsupported\n", dh, L); abort(); }
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey key = hq_drop_key(seed, opid);
  const int Lp = (L + 31) & ~31;
  {
    const int n_qb = (L + RQ - 1) / RQ;
    const int force_slow = g_attn_force_slow;
    constexpr int ahead = 2;   // K/V tiles in flight (4-deep measured slower: profiles/r2_attn)
    const size_t lds = (size_t)4 * 2 * RTILE + Lp * sizeof(uint2);
    const int nparts = B * nh * n_qb * RW;
    float* part8 = ctx8 ? hq_fp8_amax_parts((size_t)nparts, q8, s) : nullptr;
    auto run = [&](auto cn) {
      constexpr int NT = decltype(cn)::value;
      auto launch1 = [&](auto kern) {
        static bool attr =
            (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) == hipSuccess);
        (void)attr;
        hipLaunchKernelGGL(kern, dim3(B * nh * n_qb), dim3(RW * 64), lds, s, qkv, key_bias, ctx, lse,
                           thr ? mbits : nullptr, L, nh, n_qb, scale * LOG2E, key, thr, hq_keep_scale(thr), force_slow,
                           ctx8, q8, part8, phase);
      };
      (void)ahead;
      // EVEN (L % 32 == 0) also selects the unclamped DMA addressing: never pass it for a ragged L
      // (NT > 0 implies L = 32·NT, so the ragged variants exist only for the rolled NT = 0 loop)
      if constexpr (NT > 0) {
        if (!thr) launch1(attn_fwd_ring_kernel<false, true, NT, 2>);
        else launch1(attn_fwd_ring_kernel<true, true, NT, 2>);
      } else {
        if (!thr && (L & 31) == 0) launch1(attn_fwd_ring_kernel<false, true, 0, 2>);
        else if (!thr) launch1(attn_fwd_ring_kernel<false, false, 0, 2>);
        else if ((L & 31) == 0) launch1(attn_fwd_ring_kernel<true, true, 0, 2>);
        else launch1(attn_fwd_ring_kernel<true, false, 0, 2>);
      }
    };
    if (L == 384) run(std::integral_constant<int, 12>{});
    else if (L == 512) run(std::integral_constant<int, 16>{});
    else if (L == 256) run(std::integral_constant<int, 8>{});
    else if (L == 128) run(std::integral_constant<int, 4>{});
    else run(std::integral_constant<int, 0>{});
    if (ctx8) hq_fp8_amax_fold(part8, nparts, q8, phase, s);
  }
}

void hq_attn_bwd(const uint16_t* dctx, const uint16_t* qkv, const uint16_t* ctx, const float* lse, const float* key_bias,
                 const uint16_t* mbits, uint16_t* dqkv, float* delta, int B, int L, int nh, int dh, float p,
                 float scale, bool deterministic, hipStream_t s, uint8_t* dqkv8, float* q8, int phase, float* bpart) {
  if (dh != D || L > 512) { fprintf(stderr, "hq_attn_bwd: head_dim %d / L %d unsupported\n", dh, L); abort(); }
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const float ks = hq_keep_scale(thr);
  const uint16_t* bits = thr ? mbits : nullptr;
  const int Lp = (L + 31) & ~31, n32 = Lp / 32;
  (void)deterministic;   // both backward kernels are deterministic (no atomics)
  {
    const int nb = (L + RQ - 1) / RQ;                 // 128-row blocks (queries for dQ, keys for dK/dV)
    // ring depth: 2 tiles ahead on the bf16 path (39.5 KB of LDS per workgroup at L = 384 with dropout, so
    // 4 workgroups — 4 waves per SIMD — share a CU), 3 on the fp8 paths (their e5m2 epilogues need > 128 VGPRs)
    constexpr int AH = 2, AH8 = 3;
    const size_t lds_dq = (size_t)((dqkv8 ? AH8 : AH) + 2) * 2 * RTILE + Lp * sizeof(uint32_t) +
                          (bits ? (size_t)RW * n32 * 128 : 0);
    const size_t lds_kv = 2 * (size_t)(2 * RTILE + 512 + 128 + RW * 128);
    // dQ and dK/dV grids are the same size: partials [dQ waves | dK/dV waves], one fold after both
    const int nparts = B * nh * nb * RW;
    float* part8 = dqkv8 ? hq_fp8_amax_parts((size_t)2 * nparts, q8, s) : nullptr;
    auto run = [&](auto cn) {
      constexpr int NT = decltype(cn)::value;
      auto launch = [&](auto kdq, auto kkv) {
        static bool attr =
            (hipFuncSetAttribute((const void*)kdq, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) == hipSuccess);
        (void)attr;
        hipLaunchKernelGGL(kdq, dim3(B * nh * nb), dim3(RW * 64), lds_dq, s, qkv, dctx, ctx, lse, key_bias, bits, delta,
                           dqkv, L, nh, nb, scale * LOG2E, scale, ks, dqkv8, q8, part8, phase, bpart);
        hipLaunchKernelGGL(kkv, dim3(B * nh * nb), dim3(RW * 64), lds_kv, s, qkv, dctx, lse, delta, key_bias, bits, dqkv,
                           L, nh, nb, scale * LOG2E, scale, ks, dqkv8, q8, part8, phase, bpart);
      };
      if (dqkv8 && bpart) {   // --precision fp8, calibrated: e5m2 + bias partials, no bf16
        if (bits) launch(attn_bwd_dq_ring_kernel<true, NT, AH8, 2>, attn_bwd_dkdv_ring_kernel<true, NT, 2>);
        else launch(attn_bwd_dq_ring_kernel<false, NT, AH8, 2>, attn_bwd_dkdv_ring_kernel<false, NT, 2>);
      } else if (dqkv8) {   // --precision fp8: the e5m2-writing variants
        if (bits) launch(attn_bwd_dq_ring_kernel<true, NT, AH8, 1>, attn_bwd_dkdv_ring_kernel<true, NT, 1>);
        else launch(attn_bwd_dq_ring_kernel<false, NT, AH8, 1>, attn_bwd_dkdv_ring_kernel<false, NT, 1>);
      } else {
        if (bits) launch(attn_bwd_dq_ring_kernel<true, NT, AH>, attn_bwd_dkdv_ring_kernel<true, NT>);
        else launch(attn_bwd_dq_ring_kernel<false, NT, AH>, attn_bwd_dkdv_ring_kernel<false, NT>);
      }
    };
    if (L == 384) run(std::integral_constant<int, 12>{});
    else if (L == 512) run(std::integral_constant<int, 16>{});
    else if (L == 256) run(std::integral_constant<int, 8>{});
    else if (L == 128) run(std::integral_constant<int, 4>{});
    else run(std::integral_constant<int, 0>{});
    if (dqkv8) hq_fp8_amax_fold(part8, 2 * nparts, q8, phase, s, kHqBf8Max);
  }
}
