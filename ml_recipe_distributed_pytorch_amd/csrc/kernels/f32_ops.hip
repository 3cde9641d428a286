// Native fp32 row-wise ops and flash attention for ``--precision fp32`` (the reference's Apex-off training mode,
// /root/reference/modules/model/trainer/trainer.py:23-32,128-133; --finetune forces it, modules/init.py:86-92).
//
// The fp32 step's GEMMs run on gemm_f32.hip (exact-f32 MFMA); everything else the encoder does per element or per
// row runs here instead of as ATen ops — fp32 in, fp32 out, fp32 statistics, dropout masks from the same counter
// hash as every other kernel (hq_keep, bit-identical to ops/rng.py), so the GPU fp32 model reproduces the CPU
// oracle (ops/reference.py) op for op:
//   f32_embed_fwd / _bwd   : 3 gathers + LayerNorm + dropout; backward with f32 atomics into the tables
//   f32_ln_fwd / _bwd      : z = dropout(a) + resid, y = LN(z); backward dz, da and γ / β / bias column partials
//   f32_gelu_fwd / _bwd    : erf GELU; backward with the producing Linear's bias-gradient column partials
//   f32_colsum             : column partials of a [T, N] matrix (the Linear bias gradients), then a fixed-order fold
//   f32_attn_fwd / _bwd    : flash attention (head_dim 64) — never holds a [B, nh, L, L] tensor: scores are
//                            recomputed per 32-key tile in registers (online softmax forward, LSE backward).
// Layout of the attention kernels: a quad of lanes owns one query (forward / dQ) or one key (dK / dV), lane q & 3
// holding head dims [16·(q & 3), +16); a dot product over the 64 dims is 16 FMAs per lane + a 2-step DPP quad sum,
// so every lane of the quad ends with the same score (no LDS exchange).
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int kW = 4;            // waves per block in the row kernels (one row per wave at a time)
constexpr int kRowsPerBlock = 64;  // column-partial kernels: rows summed per partial

__device__ __forceinline__ float quad_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // lane ^ 1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // lane ^ 2
  return v;
}

__device__ __forceinline__ float keep_mul(uint32_t idx, uint32_t key, uint32_t thr, float ks) {
  return thr ? (hq_keep(idx, key, thr) ? ks : 0.f) : 1.f;
}

// ---------------------------------------------------------------------------------------------- embedding
// one wave per row; lane l holds columns c·64 + l (coalesced 256-B rows); NC = ceil(H / 64) <= 16
template <int NC>
__global__ __launch_bounds__(256) void f32_embed_fwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ pids,
                                                            const int64_t* __restrict__ tids, const float* __restrict__ ww,
                                                            const float* __restrict__ wp, const float* __restrict__ wt,
                                                            const float* __restrict__ gamma, const float* __restrict__ beta,
                                                            float* __restrict__ y, float* __restrict__ mean,
                                                            float* __restrict__ rstd, int T, int H, float eps, int V, int P,
                                                            int NTY, HqDropKey kd, uint32_t thr, float ks) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * kW + (threadIdx.x >> 6);
  if (row >= T) return;
  const uint32_t key = kd.get();
  const int64_t id = ids[row], pid = pids[row], tid = tids[row];
  HQ_DASSERT(id >= 0 && id < V && pid >= 0 && pid < P && tid >= 0 && tid < NTY);
  float x[NC];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * 64 + lane;
    x[c] = col < H ? ww[id * H + col] + wp[pid * H + col] + wt[tid * H + col] : 0.f;
    s += x[c];
  }
  const float mu = hq_wave_sum(s) / H;
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c * 64 + lane < H) v += (x[c] - mu) * (x[c] - mu);
  const float rs = rsqrtf(hq_wave_sum(v) / H + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * 64 + lane;
    if (col < H) {
      const float o = (x[c] - mu) * rs * gamma[col] + beta[col];
      y[(size_t)row * H + col] = o * keep_mul((uint32_t)((size_t)row * H + col), key, thr, ks);
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

// rows [blockIdx.x·kRowsPerBlock, +kRowsPerBlock), one wave per row at a time; γ / β partials per block
template <int NC>
__global__ __launch_bounds__(256) void f32_embed_bwd_kernel(const float* __restrict__ dy, const int64_t* __restrict__ ids,
                                                            const int64_t* __restrict__ pids, const int64_t* __restrict__ tids,
                                                            const float* __restrict__ ww, const float* __restrict__ wp,
                                                            const float* __restrict__ wt, const float* __restrict__ gamma,
                                                            const float* __restrict__ mean, const float* __restrict__ rstd,
                                                            float* __restrict__ g_word, float* __restrict__ g_pos,
                                                            float* __restrict__ g_type, float* __restrict__ part, int T, int H,
                                                            int pad_word, int pad_pos, int V, int P, int NTY, HqDropKey kd,
                                                            uint32_t thr, float ks) {
  // γ | β | type-0 | type-1 partials per block (the type rows as partials when NTY <= 2: every row of the batch
  // hits one of two rows, which f32 atomics serialise)
  __shared__ float red[kW][4][NC * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t key = kd.get();
  const bool tpart = NTY <= 2;
  float ag[NC], ab[NC], at0[NC], at1[NC], gam[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    ag[c] = ab[c] = at0[c] = at1[c] = 0.f;
    gam[c] = c * 64 + lane < H ? gamma[c * 64 + lane] : 0.f;
  }
  const int r0 = blockIdx.x * kRowsPerBlock, r1 = min(T, r0 + kRowsPerBlock);
  for (int row = r0 + wave; row < r1; row += kW) {
    const int64_t id = ids[row], pid = pids[row], tid = tids[row];
    HQ_DASSERT(id >= 0 && id < V && pid >= 0 && pid < P && tid >= 0 && tid < NTY);
    const float mu = mean[row], rs = rstd[row];
    float xh[NC], g[NC], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * 64 + lane;
      if (col < H) {
        const float x = ww[id * H + col] + wp[pid * H + col] + wt[tid * H + col];
        xh[c] = (x - mu) * rs;
        g[c] = dy[(size_t)row * H + col] * keep_mul((uint32_t)((size_t)row * H + col), key, thr, ks);
      } else {
        xh[c] = g[c] = 0.f;
      }
      ag[c] += g[c] * xh[c];
      ab[c] += g[c];
      const float d = g[c] * gam[c];
      s1 += d;
      s2 += d * xh[c];
    }
    s1 = hq_wave_sum(s1) / H;
    s2 = hq_wave_sum(s2) / H;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * 64 + lane;
      if (col < H) {
        const float dx = rs * (g[c] * gam[c] - s1 - xh[c] * s2);
        if (id != pad_word) atomicAdd(g_word + id * H + col, dx);
        if (pid != pad_pos) atomicAdd(g_pos + pid * H + col, dx);
        if (!tpart) atomicAdd(g_type + tid * H + col, dx);
        at0[c] += tid == 0 ? dx : 0.f;
        at1[c] += tid == 1 ? dx : 0.f;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    red[wave][0][c * 64 + lane] = ag[c];
    red[wave][1][c * 64 + lane] = ab[c];
    red[wave][2][c * 64 + lane] = at0[c];
    red[wave][3][c * 64 + lane] = at1[c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * H; i += 256) {
    const int w = i / H, col = i - w * H;
    part[(size_t)blockIdx.x * 4 * H + i] = (red[0][w][col] + red[1][w][col]) + (red[2][w][col] + red[3][w][col]);
  }
}

// ---------------------------------------------------------------------------- residual + dropout + LayerNorm
template <int NC>
__global__ __launch_bounds__(256) void f32_ln_fwd_kernel(const float* __restrict__ a, const float* __restrict__ resid,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         float* __restrict__ y, float* __restrict__ z, float* __restrict__ mean,
                                                         float* __restrict__ rstd, int T, int H, float eps, HqDropKey kd,
                                                         uint32_t thr, float ks) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * kW + (threadIdx.x >> 6);
  if (row >= T) return;
  const uint32_t key = kd.get();
  float x[NC];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * 64 + lane;
    const size_t o = (size_t)row * H + col;
    x[c] = col < H ? a[o] * keep_mul((uint32_t)o, key, thr, ks) + resid[o] : 0.f;
    s += x[c];
  }
  const float mu = hq_wave_sum(s) / H;
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c * 64 + lane < H) v += (x[c] - mu) * (x[c] - mu);
  const float rs = rsqrtf(hq_wave_sum(v) / H + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * 64 + lane;
    if (col < H) {
      const size_t o = (size_t)row * H + col;
      z[o] = x[c];
      y[o] = (x[c] - mu) * rs * gamma[col] + beta[col];
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

// dz = LN backward of g = dy (+ dy2), da = dz·keep; partials [block][3H] = Σ g·x̂ | Σ g | Σ da.  beta != null: `z` is
// the forward output y and x̂ = (y − β)/γ (0 where γ = 0), ops/reference.py ln_bwd's FROMY form.
template <int NC>
__global__ __launch_bounds__(256) void f32_ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ dy2,
                                                         const float* __restrict__ z, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, float* __restrict__ dz,
                                                         float* __restrict__ da, float* __restrict__ part, int T, int H,
                                                         HqDropKey kd, uint32_t thr, float ks) {
  __shared__ float red[kW][3][NC * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t key = kd.get();
  float acc[3][NC], gam[NC], ig[NC], bb[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    acc[0][c] = acc[1][c] = acc[2][c] = 0.f;
    const int col = c * 64 + lane;
    gam[c] = col < H ? gamma[col] : 0.f;
    ig[c] = gam[c] != 0.f ? 1.f / gam[c] : 0.f;
    bb[c] = (beta != nullptr && col < H) ? beta[col] : 0.f;
  }
  const int r0 = blockIdx.x * kRowsPerBlock, r1 = min(T, r0 + kRowsPerBlock);
  for (int row = r0 + wave; row < r1; row += kW) {
    const float mu = mean[row], rs = rstd[row];
    float xh[NC], g[NC], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * 64 + lane;
      const size_t o = (size_t)row * H + col;
      if (col < H) {
        g[c] = dy[o] + (dy2 ? dy2[o] : 0.f);
        xh[c] = beta != nullptr ? z[o] * ig[c] - bb[c] * ig[c] : (z[o] - mu) * rs;
      } else {
        g[c] = xh[c] = 0.f;
      }
      acc[0][c] += g[c] * xh[c];
      acc[1][c] += g[c];
      const float d = g[c] * gam[c];
      s1 += d;
      s2 += d * xh[c];
    }
    s1 = hq_wave_sum(s1) / H;
    s2 = hq_wave_sum(s2) / H;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * 64 + lane;
      if (col < H) {
        const size_t o = (size_t)row * H + col;
        const float d = rs * (g[c] * gam[c] - s1 - xh[c] * s2);
        const float dd = d * keep_mul((uint32_t)o, key, thr, ks);
        dz[o] = d;
        da[o] = dd;
        acc[2][c] += dd;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int k = 0; k < 3; ++k) red[wave][k][c * 64 + lane] = acc[k][c];
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * H; i += 256) {
    const int k = i / H, col = i - k * H;
    part[(size_t)blockIdx.x * 3 * H + i] = (red[0][k][col] + red[1][k][col]) + (red[2][k][col] + red[3][k][col]);
  }
}

// ------------------------------------------------------------------------------------------------ GELU
constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

__global__ __launch_bounds__(256) void f32_gelu_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const float v = x[i];
    y[i] = 0.5f * v * (1.f + erff(v * kInvSqrt2));
  }
}

// d = dout·gelu'(x); column partials of d per kRowsPerBlock rows (thread = column: coalesced rows)
__global__ __launch_bounds__(256) void f32_gelu_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ x,
                                                           float* __restrict__ d, float* __restrict__ part, int T, int N) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= N) return;
  const int r0 = blockIdx.y * kRowsPerBlock, r1 = min(T, r0 + kRowsPerBlock);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) {
    const size_t o = (size_t)r * N + col;
    const float v = x[o];
    const float g = dout[o] * (0.5f * (1.f + erff(v * kInvSqrt2)) + v * expf(-0.5f * v * v) * kInvSqrt2Pi);
    d[o] = g;
    s += g;
  }
  if (part) part[(size_t)blockIdx.y * N + col] = s;
}

// column partials of x [T, N] per kRowsPerBlock rows
__global__ __launch_bounds__(256) void f32_colpart_kernel(const float* __restrict__ x, float* __restrict__ part, int T, int N) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= N) return;
  const int r0 = blockIdx.y * kRowsPerBlock, r1 = min(T, r0 + kRowsPerBlock);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += x[(size_t)r * N + col];
  part[(size_t)blockIdx.y * N + col] = s;
}

// Deterministic two-level fold of column partials part[nb][W] (nb ~ T / 64 rows, W up to 3·H): a single
// column-per-thread pass had W / 256 blocks (9 at W = 2304) each walking ~400 rows serially — 97 µs per fold.
// Level 1: blocks of (64 columns × one of kFoldS row slices), 4 waves each summing every 4th row of the slice,
// combined in LDS in a fixed order -> p2[kFoldS][W]; level 2: out[c] (+)= Σ_s p2[s][c] in slice order.
constexpr int kFoldS = 16;
__global__ __launch_bounds__(256) void f32_fold1_kernel(const float* __restrict__ part, int nb, int W,
                                                        float* __restrict__ p2) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, sl = blockIdx.y;
  const int b0 = nb * sl / kFoldS, b1 = nb * (sl + 1) / kFoldS;
  float s = 0.f;
  if (c < W)
    for (int b = b0 + wave; b < b1; b += 4) s += part[(size_t)b * W + c];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < W) p2[(size_t)sl * W + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}
__global__ __launch_bounds__(256) void f32_fold2_kernel(const float* __restrict__ p2, int W, int width, HqOuts outs,
                                                        int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= W) return;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kFoldS; ++k) s += p2[(size_t)k * W + i];
  float* dst = outs.p[i / width];
  if (dst == nullptr) return;
  const int c = i % width;
  dst[c] = accumulate ? dst[c] + s : s;
}

// ------------------------------------------------------------------------------------------- attention
// qkv [T, 3H] (q | k | v, head h at columns h·64 of each third), key_bias [B, L], z = b·nh + h.
constexpr int AD = 64;      // head dim
constexpr int AQ = 64;      // queries (forward / dQ) or keys (dK / dV) per block: 16 quads per wave × 4 waves
constexpr int AT = 32;      // keys (or queries) per LDS tile

__device__ __forceinline__ void load16(const float* __restrict__ p, float (&v)[16]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 t = reinterpret_cast<const float4*>(p)[i];
    v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
  }
}
__device__ __forceinline__ float dot16(const float (&a)[16], const float* __restrict__ b) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 t = reinterpret_cast<const float4*>(b)[i];
    s = fmaf(a[4 * i], t.x, s); s = fmaf(a[4 * i + 1], t.y, s); s = fmaf(a[4 * i + 2], t.z, s); s = fmaf(a[4 * i + 3], t.w, s);
  }
  return s;
}
__device__ __forceinline__ void axpy16(float (&y)[16], float a, const float* __restrict__ x) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 t = reinterpret_cast<const float4*>(x)[i];
    y[4 * i] = fmaf(a, t.x, y[4 * i]); y[4 * i + 1] = fmaf(a, t.y, y[4 * i + 1]);
    y[4 * i + 2] = fmaf(a, t.z, y[4 * i + 2]); y[4 * i + 3] = fmaf(a, t.w, y[4 * i + 3]);
  }
}

// stage rows [r0, r0 + AT) (clamped to L) of one head matrix (column offset `col`) into an [AT][AD] LDS tile;
// rows past L are zero
__device__ __forceinline__ void stage_rows(float* __restrict__ dst, const float* __restrict__ src, int ld, int col, int b,
                                           int L, int r0) {
  for (int i = threadIdx.x; i < AT * AD / 4; i += 256) {
    const int r = i / (AD / 4), c4 = i % (AD / 4);
    const int row = r0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < L) v = *reinterpret_cast<const float4*>(src + (size_t)(b * L + row) * ld + col + 4 * c4);
    reinterpret_cast<float4*>(dst)[i] = v;
  }
}

__global__ __launch_bounds__(256) void f32_attn_fwd_kernel(const float* __restrict__ qkv, const float* __restrict__ key_bias,
                                                           float* __restrict__ ctx, float* __restrict__ lse, int B, int L,
                                                           int nh, float scale, HqDropKey kd, uint32_t thr, float ks) {
  __shared__ __attribute__((aligned(16))) float Ks[AT * AD], Vs[AT * AD], Bs[AT];
  const int z = blockIdx.y, b = z / nh, h = z - b * nh;
  const int H = nh * AD, H3 = 3 * H;
  const int lane = threadIdx.x & 63, sub = lane & 3;
  const int q = blockIdx.x * AQ + (threadIdx.x >> 2);
  const bool qv = q < L;
  const uint32_t key = kd.get();
  float qr[16], o[16];
  if (qv) load16(qkv + (size_t)(b * L + q) * H3 + h * AD + 16 * sub, qr);
  else
#pragma unroll
    for (int i = 0; i < 16; ++i) qr[i] = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = 0.f;
  float m = -INFINITY, l = 0.f;
  const uint32_t rowidx = (uint32_t)(((size_t)z * L + (qv ? q : 0)) * L);
  for (int k0 = 0; k0 < L; k0 += AT) {
    __syncthreads();
    stage_rows(Ks, qkv, H3, H + h * AD, b, L, k0);
    stage_rows(Vs, qkv, H3, 2 * H + h * AD, b, L, k0);
    if (threadIdx.x < AT) Bs[threadIdx.x] = k0 + (int)threadIdx.x < L ? key_bias[b * L + k0 + threadIdx.x] : 0.f;
    __syncthreads();
    const int nk = min(AT, L - k0);
    float s[AT];
    float tmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < AT; ++j) {
      s[j] = j < nk ? quad_sum(dot16(qr, Ks + j * AD + 16 * sub)) * scale + Bs[j] : -INFINITY;
      tmax = fmaxf(tmax, s[j]);
    }
    const float mn = fmaxf(m, tmax);
    const float alpha = m == -INFINITY ? 0.f : expf(m - mn);
    l *= alpha;
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] *= alpha;
#pragma unroll
    for (int j = 0; j < AT; ++j) {
      if (j < nk) {
        const float p = expf(s[j] - mn);
        l += p;
        axpy16(o, p * keep_mul(rowidx + (uint32_t)(k0 + j), key, thr, ks), Vs + j * AD + 16 * sub);
      }
    }
    m = mn;
  }
  if (!qv) return;
  const float inv = 1.f / l;
  float* out = ctx + (size_t)(b * L + q) * H + h * AD + 16 * sub;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    reinterpret_cast<float4*>(out)[i] = make_float4(o[4 * i] * inv, o[4 * i + 1] * inv, o[4 * i + 2] * inv, o[4 * i + 3] * inv);
  if (sub == 0) lse[(size_t)z * L + q] = m + logf(l);
}

// dQ (and δ = rowsum(dO ∘ O) for the dK / dV kernel): a quad per query, keys streamed through LDS tiles.
// dS = P·(dP·keep − δ), dQ = scale·Σ_k dS·K_k (ops/reference.py attn_bwd).
__global__ __launch_bounds__(256) void f32_attn_dq_kernel(const float* __restrict__ dctx, const float* __restrict__ qkv,
                                                          const float* __restrict__ ctx, const float* __restrict__ lse,
                                                          const float* __restrict__ key_bias, float* __restrict__ dqkv,
                                                          float* __restrict__ delta, int B, int L, int nh, float scale,
                                                          HqDropKey kd, uint32_t thr, float ks) {
  __shared__ __attribute__((aligned(16))) float Ks[AT * AD], Vs[AT * AD], Bs[AT];
  const int z = blockIdx.y, b = z / nh, h = z - b * nh;
  const int H = nh * AD, H3 = 3 * H;
  const int lane = threadIdx.x & 63, sub = lane & 3;
  const int q = blockIdx.x * AQ + (threadIdx.x >> 2);
  const bool qv = q < L;
  const uint32_t key = kd.get();
  float qr[16], dor[16], dq[16];
  float dl = 0.f, ls = 0.f;
  if (qv) {
    load16(qkv + (size_t)(b * L + q) * H3 + h * AD + 16 * sub, qr);
    load16(dctx + (size_t)(b * L + q) * H + h * AD + 16 * sub, dor);
    float orr[16];
    load16(ctx + (size_t)(b * L + q) * H + h * AD + 16 * sub, orr);
    float d = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) d = fmaf(dor[i], orr[i], d);
    dl = quad_sum(d);
    ls = lse[(size_t)z * L + q];
    if (sub == 0) delta[(size_t)z * L + q] = dl;
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) qr[i] = dor[i] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) dq[i] = 0.f;
  const uint32_t rowidx = (uint32_t)(((size_t)z * L + (qv ? q : 0)) * L);
  for (int k0 = 0; k0 < L; k0 += AT) {
    __syncthreads();
    stage_rows(Ks, qkv, H3, H + h * AD, b, L, k0);
    stage_rows(Vs, qkv, H3, 2 * H + h * AD, b, L, k0);
    if (threadIdx.x < AT) Bs[threadIdx.x] = k0 + (int)threadIdx.x < L ? key_bias[b * L + k0 + threadIdx.x] : 0.f;
    __syncthreads();
    const int nk = min(AT, L - k0);
    for (int j = 0; j < nk; ++j) {
      const float s = quad_sum(dot16(qr, Ks + j * AD + 16 * sub)) * scale + Bs[j];
      const float p = expf(s - ls);
      const float dp = quad_sum(dot16(dor, Vs + j * AD + 16 * sub)) * keep_mul(rowidx + (uint32_t)(k0 + j), key, thr, ks);
      axpy16(dq, p * (dp - dl), Ks + j * AD + 16 * sub);
    }
  }
  if (!qv) return;
  float* out = dqkv + (size_t)(b * L + q) * H3 + h * AD + 16 * sub;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    reinterpret_cast<float4*>(out)[i] = make_float4(dq[4 * i] * scale, dq[4 * i + 1] * scale, dq[4 * i + 2] * scale,
                                                    dq[4 * i + 3] * scale);
}

// dK, dV: a quad per key, queries streamed through LDS tiles (Q, dO, LSE, δ).
__global__ __launch_bounds__(256) void f32_attn_dkdv_kernel(const float* __restrict__ dctx, const float* __restrict__ qkv,
                                                            const float* __restrict__ lse, const float* __restrict__ delta,
                                                            const float* __restrict__ key_bias, float* __restrict__ dqkv,
                                                            int B, int L, int nh, float scale, HqDropKey kd, uint32_t thr,
                                                            float ks) {
  __shared__ __attribute__((aligned(16))) float Qs[AT * AD], Os[AT * AD], Ls[AT], Ds[AT];
  const int z = blockIdx.y, b = z / nh, h = z - b * nh;
  const int H = nh * AD, H3 = 3 * H;
  const int lane = threadIdx.x & 63, sub = lane & 3;
  const int k = blockIdx.x * AQ + (threadIdx.x >> 2);
  const bool kv = k < L;
  const uint32_t key = kd.get();
  float kr[16], vr[16], dk[16], dv[16];
  float kb = 0.f;
  if (kv) {
    load16(qkv + (size_t)(b * L + k) * H3 + H + h * AD + 16 * sub, kr);
    load16(qkv + (size_t)(b * L + k) * H3 + 2 * H + h * AD + 16 * sub, vr);
    kb = key_bias[b * L + k];
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) kr[i] = vr[i] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) dk[i] = dv[i] = 0.f;
  for (int q0 = 0; q0 < L; q0 += AT) {
    __syncthreads();
    stage_rows(Qs, qkv, H3, h * AD, b, L, q0);
    stage_rows(Os, dctx, H, h * AD, b, L, q0);
    if (threadIdx.x < AT) {
      const bool ok = q0 + (int)threadIdx.x < L;
      Ls[threadIdx.x] = ok ? lse[(size_t)z * L + q0 + threadIdx.x] : 0.f;
      Ds[threadIdx.x] = ok ? delta[(size_t)z * L + q0 + threadIdx.x] : 0.f;
    }
    __syncthreads();
    const int nq = min(AT, L - q0);
    for (int j = 0; j < nq; ++j) {
      const float s = quad_sum(dot16(kr, Qs + j * AD + 16 * sub)) * scale + kb;
      const float p = expf(s - Ls[j]);
      const float km = keep_mul((uint32_t)(((size_t)z * L + q0 + j) * L + (kv ? k : 0)), key, thr, ks);
      axpy16(dv, p * km, Os + j * AD + 16 * sub);
      const float dp = quad_sum(dot16(vr, Os + j * AD + 16 * sub)) * km;
      axpy16(dk, p * (dp - Ds[j]), Qs + j * AD + 16 * sub);
    }
  }
  if (!kv) return;
  float* ok = dqkv + (size_t)(b * L + k) * H3 + H + h * AD + 16 * sub;
  float* ov = ok + H;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    reinterpret_cast<float4*>(ok)[i] = make_float4(dk[4 * i] * scale, dk[4 * i + 1] * scale, dk[4 * i + 2] * scale,
                                                   dk[4 * i + 3] * scale);
    reinterpret_cast<float4*>(ov)[i] = make_float4(dv[4 * i], dv[4 * i + 1], dv[4 * i + 2], dv[4 * i + 3]);
  }
}

template <typename F>
void dispatch_nc(int H, F&& f) {
  if (H <= 256) f(std::integral_constant<int, 4>{});
  else if (H <= 512) f(std::integral_constant<int, 8>{});
  else if (H <= 768) f(std::integral_constant<int, 12>{});
  else if (H <= 1024) f(std::integral_constant<int, 16>{});
  else { fprintf(stderr, "f32 row kernels: hidden size %d > 1024 unsupported\n", H); abort(); }
}

// part must have room for kFoldS more rows past its nb partial rows (the level-1 result lives there)
void fold(float* part, int nb, int width, int nout, HqOuts outs, bool accumulate, hipStream_t s) {
  const int W = width * nout;
  float* p2 = part + (size_t)nb * W;
  hipLaunchKernelGGL(f32_fold1_kernel, dim3((W + 63) / 64, kFoldS), dim3(256), 0, s, part, nb, W, p2);
  hipLaunchKernelGGL(f32_fold2_kernel, dim3((W + 255) / 256), dim3(256), 0, s, p2, W, width, outs, accumulate ? 1 : 0);
}

}  // namespace

int hq_f32_row_partials(int T) { return (T + kRowsPerBlock - 1) / kRowsPerBlock; }
int hq_f32_part_rows(int T) { return hq_f32_row_partials(T) + kFoldS; }

void hq_f32_embed_fwd(const int64_t* ids, const int64_t* pids, const int64_t* tids, const float* ww, const float* wp,
                      const float* wt, const float* gamma, const float* beta, float* y, float* mean, float* rstd, int T, int H,
                      float eps, float p, uint32_t seed, uint32_t opid, int V, int P, int NTY, hipStream_t s) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey kd = hq_drop_key(seed, opid);
  dispatch_nc(H, [&](auto nc) {
    hipLaunchKernelGGL(f32_embed_fwd_kernel<decltype(nc)::value>, dim3((T + kW - 1) / kW), dim3(256), 0, s, ids, pids, tids,
                       ww, wp, wt, gamma, beta, y, mean, rstd, T, H, eps, V, P, NTY, kd, thr, hq_keep_scale(thr));
  });
}

void hq_f32_embed_bwd(const float* dy, const int64_t* ids, const int64_t* pids, const int64_t* tids, const float* ww,
                      const float* wp, const float* wt, const float* gamma, const float* mean, const float* rstd,
                      float* g_word, float* g_pos, float* g_type, float* part, HqOuts outs, int T, int H, int pad_word,
                      int pad_pos, float p, uint32_t seed, uint32_t opid, bool accumulate, int V, int P, int NTY,
                      hipStream_t s) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey kd = hq_drop_key(seed, opid);
  const int nb = hq_f32_row_partials(T);
  dispatch_nc(H, [&](auto nc) {
    hipLaunchKernelGGL(f32_embed_bwd_kernel<decltype(nc)::value>, dim3(nb), dim3(256), 0, s, dy, ids, pids, tids, ww, wp, wt,
                       gamma, mean, rstd, g_word, g_pos, g_type, part, T, H, pad_word, pad_pos, V, P, NTY, kd, thr,
                       hq_keep_scale(thr));
  });
  fold(part, nb, H, 4, outs, accumulate, s);
}

void hq_f32_ln_fwd(const float* a, const float* resid, const float* gamma, const float* beta, float* y, float* z, float* mean,
                   float* rstd, int T, int H, float eps, float p, uint32_t seed, uint32_t opid, hipStream_t s) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey kd = hq_drop_key(seed, opid);
  dispatch_nc(H, [&](auto nc) {
    hipLaunchKernelGGL(f32_ln_fwd_kernel<decltype(nc)::value>, dim3((T + kW - 1) / kW), dim3(256), 0, s, a, resid, gamma,
                       beta, y, z, mean, rstd, T, H, eps, kd, thr, hq_keep_scale(thr));
  });
}

void hq_f32_ln_bwd(const float* dy, const float* dy2, const float* z, const float* gamma, const float* beta, const float* mean,
                   const float* rstd, float* dz, float* da, float* part, HqOuts outs, int T, int H, float p, uint32_t seed,
                   uint32_t opid, bool accumulate, hipStream_t s) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey kd = hq_drop_key(seed, opid);
  const int nb = hq_f32_row_partials(T);
  dispatch_nc(H, [&](auto nc) {
    hipLaunchKernelGGL(f32_ln_bwd_kernel<decltype(nc)::value>, dim3(nb), dim3(256), 0, s, dy, dy2, z, gamma, beta, mean, rstd,
                       dz, da, part, T, H, kd, thr, hq_keep_scale(thr));
  });
  fold(part, nb, H, 3, outs, accumulate, s);
}

void hq_f32_gelu_fwd(const float* x, float* y, size_t n, hipStream_t s) {
  const int grid = (int)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 8192));
  hipLaunchKernelGGL(f32_gelu_fwd_kernel, dim3(grid), dim3(256), 0, s, x, y, n);
}

void hq_f32_gelu_bwd(const float* dout, const float* x, float* d, float* part, float* g_bias, int T, int N, bool accumulate,
                     hipStream_t s) {
  const int nb = hq_f32_row_partials(T);
  hipLaunchKernelGGL(f32_gelu_bwd_kernel, dim3((N + 255) / 256, nb), dim3(256), 0, s, dout, x, d, g_bias ? part : nullptr, T,
                     N);
  if (g_bias) fold(part, nb, N, 1, HqOuts{{g_bias, nullptr, nullptr, nullptr}}, accumulate, s);
}

void hq_f32_colsum(const float* x, float* part, float* out, int T, int N, bool accumulate, hipStream_t s) {
  const int nb = hq_f32_row_partials(T);
  hipLaunchKernelGGL(f32_colpart_kernel, dim3((N + 255) / 256, nb), dim3(256), 0, s, x, part, T, N);
  fold(part, nb, N, 1, HqOuts{{out, nullptr, nullptr, nullptr}}, accumulate, s);
}

void hq_f32_attn_fwd(const float* qkv, const float* key_bias, float* ctx, float* lse, int B, int L, int nh, float p,
                     uint32_t seed, uint32_t opid, float scale, hipStream_t s) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey kd = hq_drop_key(seed, opid);
  hipLaunchKernelGGL(f32_attn_fwd_kernel, dim3((L + AQ - 1) / AQ, B * nh), dim3(256), 0, s, qkv, key_bias, ctx, lse, B, L, nh,
                     scale, kd, thr, hq_keep_scale(thr));
}

void hq_f32_attn_bwd(const float* dctx, const float* qkv, const float* ctx, const float* lse, const float* key_bias,
                     float* dqkv, float* delta, int B, int L, int nh, float p, uint32_t seed, uint32_t opid, float scale,
                     hipStream_t s) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey kd = hq_drop_key(seed, opid);
  const float kss = hq_keep_scale(thr);
  const dim3 grid((L + AQ - 1) / AQ, B * nh);
  hipLaunchKernelGGL(f32_attn_dq_kernel, grid, dim3(256), 0, s, dctx, qkv, ctx, lse, key_bias, dqkv, delta, B, L, nh, scale,
                     kd, thr, kss);
  hipLaunchKernelGGL(f32_attn_dkdv_kernel, grid, dim3(256), 0, s, dctx, qkv, lse, delta, key_bias, dqkv, B, L, nh, scale, kd,
                     thr, kss);
}
