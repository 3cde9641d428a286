// Flash attention for BERT (head_dim 64, L <= 512, additive key mask, fused dropout) on gfx950.
//
// Input is the packed QKV GEMM output [T, 3H] (token-major; head h of Q/K/V at column
// {0,H,2H} + 64h), so no head-split transpose is ever materialised; output ctx is written
// straight in [T, H] and the backward writes dQ/dK/dV straight into packed dQKV [T, 3H].
//
// MFMA: v_mfma_f32_32x32x16_bf16 (32x32 tile, K=16, wave64).  Per wave 32 queries (fwd / dQ)
// or 32 keys (dK/dV).  Orientation is chosen so every softmax statistic is lane-local:
//   fwd : Sᵀ = K·Qᵀ (query on the lane) → online softmax needs one cross-half exchange per tile;
//         Oᵀ += Vᵀ·Pᵀ takes Pᵀ straight from the accumulator registers as the B operand
//         (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand") and Vᵀ from
//         LDS via ds_read_b64_tr_b16 (T10).
//   dKdV: S = Q·Kᵀ (key on the lane); dVᵀ += dOᵀ·Pd and dKᵀ += Qᵀ·dS with Pd/dS from registers.
//   dQ  : Sᵀ = K·Qᵀ (query on the lane); dQᵀ += Kᵀ·dSᵀ.
// Two backward kernels (dK/dV per key block, dQ per query block) instead of dQ float atomics:
// deterministic, and at L<=512 the recomputed QKᵀ/dOVᵀ is cheaper than 1.3 TB/s atomics.
// Dropout on P uses the counter hash of hq_common.h with element index ((b·nh+h)·L+q)·L+k.
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int D = 64;          // head dim
constexpr int KT = 64;         // keys per LDS tile (fwd, dQ)
constexpr int QT = 64;         // queries per LDS tile (dK/dV)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

__device__ __forceinline__ f32x16_t mfma32(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// 16-byte LDS row read: 8 bf16 at tile[row][col..col+7] (row stride D elements)
__device__ __forceinline__ bf16x8_t lds_row8(const uint16_t* tile, int row, int col) {
  return *reinterpret_cast<const bf16x8_t*>(tile + row * D + col);
}

// A operand "Xᵀ" of a 32x32x16 MFMA from a row-major [rows][64] LDS tile, k-step s of a 32-row
// subtile starting at row0: lane supplies X[row(s,hh,j)][d] with d = dblk*32 + (lane&31) and
// row(s,hh,j) = row0 + 16s + 4hh + (j&3) + 8(j>>2)  (the k order of an accumulator-fed B operand).
__device__ __forceinline__ bf16x8_t lds_tr8(const uint16_t* tile, int row0, int s, int dblk, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int hh = g >> 1, dsub = g & 1;
  const int r = row0 + 16 * s + 4 * hh + (i >> 2);
  const int c = dblk * 32 + 16 * dsub + 4 * (i & 3);
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(tile + r * D + c));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(tile + (r + 8) * D + c));
  bf16x8_t out;
  out[0] = lo[0]; out[1] = lo[1]; out[2] = lo[2]; out[3] = lo[3];
  out[4] = hi[0]; out[5] = hi[1]; out[6] = hi[2]; out[7] = hi[3];
  return out;
}

// accumulator registers 8s..8s+7 → bf16 B fragment
__device__ __forceinline__ bf16x8_t pack_b(const float* v, int s) {
  bf16x8_t out;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (short)hq_f2bf(v[8 * s + j]);
  return out;
}

// row (within a 32-row MFMA tile) of accumulator register r for lane-half hh
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// cooperative global→LDS copy of a [64][64] bf16 tile: rows row0.. of a [*, ld] matrix (zero past nrows)
__device__ __forceinline__ void stage_tile(uint16_t* lds, const uint16_t* src, size_t ld, int row0, int nrows) {
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int t = threadIdx.x + pass * 256;
    const int row = t >> 3, chunk = t & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row0 + row < nrows) v = *reinterpret_cast<const uint4*>(src + (size_t)(row0 + row) * ld + chunk * 8);
    *reinterpret_cast<uint4*>(lds + row * D + chunk * 8) = v;
  }
}

// ============================================================================ forward
__global__ __launch_bounds__(256) void attn_fwd_kernel(const uint16_t* __restrict__ qkv, const float* __restrict__ key_bias,
                                                       uint16_t* __restrict__ ctx, float* __restrict__ lse, int L, int nh,
                                                       float c_scale, uint32_t key, uint32_t thr, float kscale) {
  __shared__ __attribute__((aligned(16))) uint16_t sK[KT * D];
  __shared__ __attribute__((aligned(16))) uint16_t sV[KT * D];
  __shared__ __attribute__((aligned(16))) float sB[KT];
  const int H = nh * D, ld = 3 * H;
  const int bh = blockIdx.y, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int hh = lane >> 5;
  const int qi = blockIdx.x * 128 + wave * 32 + (lane & 31);
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;

  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = (qi < L) ? *reinterpret_cast<const bf16x8_t*>(base + (size_t)qi * ld + 16 * s + 8 * hh) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x16_t o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const uint32_t row_idx = ((uint32_t)bh * L + (uint32_t)min(qi, L - 1)) * (uint32_t)L;
  const bool pair_ok = ((L & 1) == 0);

  for (int k0 = 0; k0 < L; k0 += KT) {
    stage_tile(sK, base + H, ld, k0, L);
    stage_tile(sV, base + 2 * H, ld, k0, L);
    if (threadIdx.x < KT) {
      const int kk = k0 + threadIdx.x;
      sB[threadIdx.x] = kk < L ? key_bias[(size_t)b * L + kk] * LOG2E : -INFINITY;
    }
    __syncthreads();
    float sc[2][16];
    float mx = -INFINITY;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x16_t acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma32(lds_row8(sK, sub * 32 + (lane & 31), 16 * s + 8 * hh), qf[s], acc);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bb = *reinterpret_cast<const float4*>(sB + sub * 32 + 8 * g + 4 * hh);
        sc[sub][4 * g + 0] = acc[4 * g + 0] * c_scale + bb.x;
        sc[sub][4 * g + 1] = acc[4 * g + 1] * c_scale + bb.y;
        sc[sub][4 * g + 2] = acc[4 * g + 2] * c_scale + bb.z;
        sc[sub][4 * g + 3] = acc[4 * g + 3] * c_scale + bb.w;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[sub][r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float rs = 0.f;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sc[sub][r] = exp2f(sc[sub][r] - m_new);
        rs += sc[sub][r];
      }
    l_run = l_run * alpha + rs;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
    if (thr) {
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t idx0 = row_idx + k0 + sub * 32 + 8 * g + 4 * hh;
          float mk[4];
          if (pair_ok) {
            hq_keep4(idx0, key, thr, kscale, mk);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) mk[i] = hq_keep(idx0 + i, key, thr) ? kscale : 0.f;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) sc[sub][4 * g + i] *= mk[i];
        }
    }
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t pb = pack_b(sc[sub], s);
#pragma unroll
        for (int d = 0; d < 2; ++d) o[d] = mfma32(lds_tr8(sV, sub * 32, s, d, lane), pb, o[d]);
      }
    __syncthreads();
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.f / l_tot;
  if (qi < L) {
    uint16_t* out = ctx + ((size_t)b * L + qi) * H + h * D;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v4[4] = {o[d][4 * g] * inv, o[d][4 * g + 1] * inv, o[d][4 * g + 2] * inv, o[d][4 * g + 3] * inv};
        *reinterpret_cast<uint2*>(out + d * 32 + 8 * g + 4 * hh) = hq_pack4(v4);
      }
    if (hh == 0) lse[(size_t)bh * L + qi] = (m_run + log2f(l_tot)) * LN2;
  }
}

// ============================================================================ backward
// delta[bh][q] = Σ_d dO·O   (one thread per (token, head))
__global__ __launch_bounds__(256) void attn_delta_kernel(const uint16_t* __restrict__ dctx, const uint16_t* __restrict__ ctx,
                                                         float* __restrict__ delta, int T, int L, int nh) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= T * nh) return;
  const int t = i / nh, h = i % nh;
  const int H = nh * D;
  const uint4* a = reinterpret_cast<const uint4*>(dctx + (size_t)t * H + h * D);
  const uint4* c = reinterpret_cast<const uint4*>(ctx + (size_t)t * H + h * D);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float x[8], y[8];
    hq_unpack8(a[k], x);
    hq_unpack8(c[k], y);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * y[j];
  }
  const int b = t / L, q = t % L;
  delta[((size_t)b * nh + h) * L + q] = s;
}

// dK, dV for 128 keys per block (32 per wave), looping over all queries in 64-row LDS tiles
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ dctx,
                                                            const float* __restrict__ lse, const float* __restrict__ delta,
                                                            const float* __restrict__ key_bias, uint16_t* __restrict__ dqkv,
                                                            int L, int nh, float c_scale, float scale, uint32_t key,
                                                            uint32_t thr, float kscale) {
  __shared__ __attribute__((aligned(16))) uint16_t sQ[QT * D];
  __shared__ __attribute__((aligned(16))) uint16_t sO[QT * D];   // dO tile
  __shared__ __attribute__((aligned(16))) float sL[QT];           // lse·log2e (+inf past L)
  __shared__ __attribute__((aligned(16))) float sD[QT];           // delta
  const int H = nh * D, ld = 3 * H;
  const int bh = blockIdx.y, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int hh = lane >> 5;
  const int kj = blockIdx.x * 128 + wave * 32 + (lane & 31);  // this lane's key (S column)
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  const uint16_t* dbase = dctx + (size_t)b * L * H + h * D;

  bf16x8_t kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const bool ok = kj < L;
    kf[s] = ok ? *reinterpret_cast<const bf16x8_t*>(base + (size_t)kj * ld + H + 16 * s + 8 * hh) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    vf[s] = ok ? *reinterpret_cast<const bf16x8_t*>(base + (size_t)kj * ld + 2 * H + 16 * s + 8 * hh) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const float kb = kj < L ? key_bias[(size_t)b * L + kj] * LOG2E : -INFINITY;
  f32x16_t dv[2], dk[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dv[d][r] = 0.f; dk[d][r] = 0.f; }

  for (int q0 = 0; q0 < L; q0 += QT) {
    stage_tile(sQ, base, ld, q0, L);
    stage_tile(sO, dbase, H, q0, L);
    if (threadIdx.x < QT) {
      const int qq = q0 + threadIdx.x;
      sL[threadIdx.x] = qq < L ? lse[(size_t)bh * L + qq] * LOG2E : INFINITY;
      sD[threadIdx.x] = qq < L ? delta[(size_t)bh * L + qq] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x16_t s_acc, p_acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s_acc[r] = 0.f; p_acc[r] = 0.f; }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s_acc = mfma32(lds_row8(sQ, sub * 32 + (lane & 31), 16 * s + 8 * hh), kf[s], s_acc);
        p_acc = mfma32(lds_row8(sO, sub * 32 + (lane & 31), 16 * s + 8 * hh), vf[s], p_acc);
      }
      float pd[16], ds[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *reinterpret_cast<const float4*>(sL + sub * 32 + 8 * g + 4 * hh);
        const float4 d4 = *reinterpret_cast<const float4*>(sD + sub * 32 + 8 * g + 4 * hh);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        const float dlt[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          const float P = exp2f(s_acc[r] * c_scale + kb - lv[i]);
          float mk = 1.f;
          if (thr) {
            const int q = q0 + sub * 32 + acc_row(r, hh);
            const uint32_t idx = ((uint32_t)bh * L + (uint32_t)min(q, L - 1)) * (uint32_t)L + (uint32_t)min(kj, L - 1);
            mk = hq_keep(idx, key, thr) ? kscale : 0.f;
          }
          pd[r] = P * mk;
          ds[r] = P * (p_acc[r] * mk - dlt[i]);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t pb = pack_b(pd, s);
        const bf16x8_t sb = pack_b(ds, s);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = mfma32(lds_tr8(sO, sub * 32, s, d, lane), pb, dv[d]);
          dk[d] = mfma32(lds_tr8(sQ, sub * 32, s, d, lane), sb, dk[d]);
        }
      }
    }
    __syncthreads();
  }
  if (kj < L) {
    uint16_t* out = dqkv + ((size_t)b * L + kj) * ld + h * D;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float k4[4] = {dk[d][4 * g] * scale, dk[d][4 * g + 1] * scale, dk[d][4 * g + 2] * scale, dk[d][4 * g + 3] * scale};
        float v4[4] = {dv[d][4 * g], dv[d][4 * g + 1], dv[d][4 * g + 2], dv[d][4 * g + 3]};
        *reinterpret_cast<uint2*>(out + H + d * 32 + 8 * g + 4 * hh) = hq_pack4(k4);
        *reinterpret_cast<uint2*>(out + 2 * H + d * 32 + 8 * g + 4 * hh) = hq_pack4(v4);
      }
  }
}

// dQ for 128 queries per block (32 per wave), looping over all keys in 64-row LDS tiles
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ dctx,
                                                          const float* __restrict__ lse, const float* __restrict__ delta,
                                                          const float* __restrict__ key_bias, uint16_t* __restrict__ dqkv,
                                                          int L, int nh, float c_scale, float scale, uint32_t key,
                                                          uint32_t thr, float kscale) {
  __shared__ __attribute__((aligned(16))) uint16_t sK[KT * D];
  __shared__ __attribute__((aligned(16))) uint16_t sV[KT * D];
  __shared__ __attribute__((aligned(16))) float sB[KT];
  const int H = nh * D, ld = 3 * H;
  const int bh = blockIdx.y, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int hh = lane >> 5;
  const int qi = blockIdx.x * 128 + wave * 32 + (lane & 31);
  const bool qok = qi < L;
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  bf16x8_t qf[4], of[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = qok ? *reinterpret_cast<const bf16x8_t*>(base + (size_t)qi * ld + 16 * s + 8 * hh) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    of[s] = qok ? *reinterpret_cast<const bf16x8_t*>(dctx + ((size_t)b * L + qi) * H + h * D + 16 * s + 8 * hh)
                : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const float lq = qok ? lse[(size_t)bh * L + qi] * LOG2E : INFINITY;
  const float dq_delta = qok ? delta[(size_t)bh * L + qi] : 0.f;
  const uint32_t row_idx = ((uint32_t)bh * L + (uint32_t)min(qi, L - 1)) * (uint32_t)L;
  const bool pair_ok = ((L & 1) == 0);
  f32x16_t dq[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[d][r] = 0.f;

  for (int k0 = 0; k0 < L; k0 += KT) {
    stage_tile(sK, base + H, ld, k0, L);
    stage_tile(sV, base + 2 * H, ld, k0, L);
    if (threadIdx.x < KT) {
      const int kk = k0 + threadIdx.x;
      sB[threadIdx.x] = kk < L ? key_bias[(size_t)b * L + kk] * LOG2E : -INFINITY;
    }
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x16_t s_acc, p_acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s_acc[r] = 0.f; p_acc[r] = 0.f; }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s_acc = mfma32(lds_row8(sK, sub * 32 + (lane & 31), 16 * s + 8 * hh), qf[s], s_acc);
        p_acc = mfma32(lds_row8(sV, sub * 32 + (lane & 31), 16 * s + 8 * hh), of[s], p_acc);
      }
      float ds[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bb = *reinterpret_cast<const float4*>(sB + sub * 32 + 8 * g + 4 * hh);
        const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
        float mk[4] = {1.f, 1.f, 1.f, 1.f};
        if (thr) {
          const uint32_t idx0 = row_idx + k0 + sub * 32 + 8 * g + 4 * hh;
          if (pair_ok) {
            hq_keep4(idx0, key, thr, kscale, mk);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) mk[i] = hq_keep(idx0 + i, key, thr) ? kscale : 0.f;
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          const float P = exp2f(s_acc[r] * c_scale + bv[i] - lq);
          ds[r] = P * (p_acc[r] * mk[i] - dq_delta);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t sb = pack_b(ds, s);
#pragma unroll
        for (int d = 0; d < 2; ++d) dq[d] = mfma32(lds_tr8(sK, sub * 32, s, d, lane), sb, dq[d]);
      }
    }
    __syncthreads();
  }
  if (qok) {
    uint16_t* out = dqkv + ((size_t)b * L + qi) * ld + h * D;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v4[4] = {dq[d][4 * g] * scale, dq[d][4 * g + 1] * scale, dq[d][4 * g + 2] * scale, dq[d][4 * g + 3] * scale};
        *reinterpret_cast<uint2*>(out + d * 32 + 8 * g + 4 * hh) = hq_pack4(v4);
      }
  }
}

}  // namespace

void hq_attn_fwd(const uint16_t* qkv, const float* key_bias, uint16_t* ctx, float* lse, int B, int L, int nh, int dh,
                 float p, uint32_t seed, uint32_t opid, float scale, hipStream_t s) {
  if (dh != D) { fprintf(stderr, "hq_attn_fwd: head_dim %d unsupported (64 only)\n", dh); abort(); }
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const uint32_t key = hq_op_key(seed, opid);
  hipLaunchKernelGGL(attn_fwd_kernel, dim3((L + 127) / 128, B * nh), dim3(256), 0, s, qkv, key_bias, ctx, lse, L, nh,
                     scale * LOG2E, key, thr, hq_keep_scale(thr));
}

void hq_attn_bwd(const uint16_t* dctx, const uint16_t* qkv, const uint16_t* ctx, const float* lse, const float* key_bias,
                 uint16_t* dqkv, float* delta, int B, int L, int nh, int dh, float p, uint32_t seed, uint32_t opid,
                 float scale, hipStream_t s) {
  if (dh != D) { fprintf(stderr, "hq_attn_bwd: head_dim %d unsupported (64 only)\n", dh); abort(); }
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const uint32_t key = hq_op_key(seed, opid);
  const float ks = hq_keep_scale(thr);
  const int T = B * L;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((T * nh + 255) / 256), dim3(256), 0, s, dctx, ctx, delta, T, L, nh);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3((L + 127) / 128, B * nh), dim3(256), 0, s, qkv, dctx, lse, delta, key_bias,
                     dqkv, L, nh, scale * LOG2E, scale, key, thr, ks);
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((L + 127) / 128, B * nh), dim3(256), 0, s, qkv, dctx, lse, delta, key_bias,
                     dqkv, L, nh, scale * LOG2E, scale, key, thr, ks);
}
