// Row-wise fused kernels for the BERT encoder (gfx950, wave64).
//
//   ln_fwd   : z = dropout(a) + resid (rounded to bf16, as HF under autocast) ; y = LN(z)
//   ln_bwd   : dz = LN_bwd(dy [+ dy2]) ; da = dropout_bwd(dz) ; per-block partial Σ(g·x̂), Σg, Σda
//   embed_fwd: y = dropout(LN(word[id] + pos[pid] + type[tid]))
//   embed_bwd: recompute x̂, LN_bwd; word grads summed per id over the id-sorted rows (no atomics),
//              position grads summed per wave over the batch (position-major walk) into partial rows,
//              type/γ/β grads through deterministic partials
//   gelu_fwd / gelu_bwd(+bias grad partials), bias_grad partials, colsum finalize
//
// Layout: one wave per row; lane owns 4 consecutive columns per 256-column chunk (8-byte bf16
// vector access), NCH = ceil(H/256) chunks.  Column partial sums are reduced per block through
// LDS and finished by hq_colsum (one 1024-thread block per 64 columns), so every gradient is
// bitwise deterministic (position ids other than 0 … L-1 fall back to float atomics for the position rows).

#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int kRowsPerWave = 8;   // rows a wave walks in the backward kernels
constexpr int kWaves = 4;         // 256-thread blocks

// LayerNorm forward, RPW rows per wave.  RES = true: z = dropout(a) + resid (rounded to bf16, as HF under
// autocast; stored only when z != null — the backward recomputes x̂ from y) ; y = LN(z).  RES = false: y =
// LN(z) where z was already written by the producing GEMM's EPI_BDR epilogue (out-projection / FFN2).
// Each wave issues all its rows' loads before the first reduction: one row per wave was latency-bound
// (88.7 µs at T = 98304 with RES, 5.1 TB/s over its three streams; RPW = 2: 77.7 µs, 5.8 TB/s; RPW = 4
// 84.0 µs — profiles/r3_ln_rpw).
// Q8 (--precision fp8): y is also written as e4m3 under the delayed scale of the consuming GEMM's input
// state q8 (the next QKV / FFN1 projection reads it instead of a separate quantisation pass over y).  Each
// wave's amax goes to a partial slot that hq_fp8_amax_fold reduces (no same-address atomics: those
// serialise in one L2 channel — a per-block filtered atomic cost +27 µs at T = 98304, a per-wave one +97).
template <int NCH, int RPW, bool RES, bool Q8 = false>
__global__ __launch_bounds__(256) void ln_fwd_rows_kernel(const uint16_t* __restrict__ zin, const uint16_t* __restrict__ resid,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          uint16_t* __restrict__ y, uint16_t* __restrict__ z,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out, int T,
                                                          int H, float eps, HqDropKey kd_, uint32_t thr, float kscale,
                                                          uint8_t* __restrict__ y8, const float* __restrict__ q8,
                                                          float* __restrict__ part8, int phase) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float amax = 0.f, inv8 = 1.f;
  if constexpr (Q8) {
    hq_fp8_publish_scale(q8, phase);
    inv8 = 1.f / hq_fp8_delayed_scale(q8, phase);
  }
  const int row0 = (blockIdx.x * kWaves + wave) * RPW;
  uint2 ra[RPW][NCH], rr[RES ? RPW : 1][NCH];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      const bool ok = row0 + r < T && col < H;
      const size_t off = (size_t)(row0 + r) * H + col;
      ra[r][c] = ok ? *reinterpret_cast<const uint2*>(zin + off) : make_uint2(0u, 0u);
      if constexpr (RES) rr[r][c] = ok ? *reinterpret_cast<const uint2*>(resid + off) : make_uint2(0u, 0u);
    }
  float v[RPW][NCH][4];
  if constexpr (RES) {
    const uint32_t key = kd_.get();
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = c * 256 + lane * 4;
        const size_t off = (size_t)(row0 + r) * H + col;
        float fa[4], fr[4], m[4] = {1.f, 1.f, 1.f, 1.f};
        hq_unpack4(ra[r][c], fa);
        hq_unpack4(rr[r][c], fr);
        if (thr) hq_keep4((uint32_t)off, key, thr, kscale, m);
        float zz[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) zz[i] = fa[i] * m[i] + fr[i];
        const uint2 packed = hq_pack4(zz);
        if (z && row0 + r < T && col < H) *reinterpret_cast<uint2*>(z + off) = packed;
        hq_unpack4(packed, v[r][c]);   // statistics of the bf16-rounded z
      }
  } else {
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c) hq_unpack4(ra[r][c], v[r][c]);
  }
  float mean[RPW], rstd[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) sum += v[r][c][i];
    mean[r] = hq_wave_sum(sum) / H;
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      if (col < H) {
#pragma unroll
        for (int i = 0; i < 4; ++i) { const float d = v[r][c][i] - mean[r]; sq += d * d; }
      }
    }
    rstd[r] = rsqrtf(hq_wave_sum(sq) / H + eps);
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    if (col < H) {
      const float4 g = *reinterpret_cast<const float4*>(gamma + col);
      const float4 b = *reinterpret_cast<const float4*>(beta + col);
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        if (row0 + r < T) {
          float o[4] = {(v[r][c][0] - mean[r]) * rstd[r] * g.x + b.x, (v[r][c][1] - mean[r]) * rstd[r] * g.y + b.y,
                        (v[r][c][2] - mean[r]) * rstd[r] * g.z + b.z, (v[r][c][3] - mean[r]) * rstd[r] * g.w + b.w};
          const uint2 packed = hq_pack4(o);
          *reinterpret_cast<uint2*>(y + (size_t)(row0 + r) * H + col) = packed;
          if constexpr (Q8) {
            hq_unpack4(packed, o);   // quantise the bf16-rounded y, exactly what the bf16 copy holds
#pragma unroll
            for (int i = 0; i < 4; ++i) amax = fmaxf(amax, fabsf(o[i]));
            *reinterpret_cast<uint32_t*>(y8 + (size_t)(row0 + r) * H + col) = hq_pack_fp8x4(o, inv8);
          }
        }
      }
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < RPW; ++r)
      if (row0 + r < T) { mean_out[row0 + r] = mean[r]; rstd_out[row0 + r] = rstd[r]; }
  }
  if constexpr (Q8) {   // this wave's amax -> its own partial slot
    amax = hq_wave_max(amax);
    if (lane == 0) part8[blockIdx.x * kWaves + wave] = amax;
  }
}

// Reduce NQ per-lane column accumulators over the 4 waves of the block into part[block][q][H].
template <int NCH, int NQ>
__device__ __forceinline__ void block_partials(float (&acc)[NQ][NCH][4], float* lds, float* part, int H) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      if (col < H) *reinterpret_cast<float4*>(lds + wave * H + col) = make_float4(acc[q][c][0], acc[q][c][1], acc[q][c][2], acc[q][c][3]);
    }
    __syncthreads();
    for (int col = threadIdx.x; col < H; col += 256) {
      float s = lds[col] + lds[H + col] + lds[2 * H + col] + lds[3 * H + col];
      part[(((size_t)blockIdx.y * gridDim.x + blockIdx.x) * NQ + q) * H + col] = s;  // linear block id (2-D grids)
    }
    __syncthreads();
  }
}

// Rows of one wave are software-pipelined: the next row's dy/dy2/z loads are in flight while the
// current row is reduced and stored (the kernel is HBM-latency bound at 3 waves/SIMD otherwise).
template <int NCH>
__device__ __forceinline__ void ln_bwd_load(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ dy2,
                                            const uint16_t* __restrict__ z, size_t base, int lane, int H,
                                            uint2 (&vdy)[NCH], uint2 (&vdy2)[NCH], uint2 (&vz)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    if (col < H) {
      vdy[c] = *reinterpret_cast<const uint2*>(dy + base + col);
      vdy2[c] = dy2 ? *reinterpret_cast<const uint2*>(dy2 + base + col) : make_uint2(0u, 0u);
      vz[c] = *reinterpret_cast<const uint2*>(z + base + col);
    }
  }
}

// RPW rows per wave: 8 at large T (partials amortised), 2 for small token counts (T = 1024: 32 blocks of
// 8-row waves left most CUs idle and each wave latency-bound — see ln_rows_per_wave)
// FROMY ("memory-efficient" LayerNorm backward): the third input is the forward OUTPUT y instead of z, and
// x̂ = (y − β)/γ = y·(1/γ) − β/γ per column (one FMA) — the forward then never stores z (151 MB per LayerNorm at
// T = 98304), and rstd is the only row statistic read.  x̂ carries y's bf16 rounding scaled by 1/γ instead of
// z's.  A column with γ = 0 has no recoverable x̂ (set to 0): its own dz (via x̂·mean(g·γ·x̂)) and γ gradient are
// then wrong — the limit of every "memory-efficient" LayerNorm; HQ_LN_FROM_Y=0 keeps z for such models.
template <int NCH, int RPW = kRowsPerWave, bool Q8 = false, bool FROMY = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ dy2,
                                                     const uint16_t* __restrict__ z, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     uint16_t* __restrict__ dz_out, uint16_t* __restrict__ da_out,
                                                     float* __restrict__ part, int T, int H, HqDropKey kd_, uint32_t thr,
                                                     float kscale, uint8_t* __restrict__ da8, const float* __restrict__ q8,
                                                     float* __restrict__ part8, int phase, const float* __restrict__ beta) {
  const uint32_t key = kd_.get();
  // Q8 (--precision fp8 backward): da also as e5m2 under the delayed scale of the dgrad GEMM that consumes
  // it (state q8), so that GEMM runs on fp8 operands without a separate quantisation pass
  float inv8 = 1.f, amax8 = 0.f;
  if constexpr (Q8) {
    hq_fp8_publish_scale(q8, phase, kHqBf8Max);
    inv8 = 1.f / hq_fp8_delayed_scale(q8, phase, kHqBf8Max);
  }
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float acc[3][NCH][4];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[q][c][i] = 0.f;
  float gam[NCH][4], ig[FROMY ? NCH : 1][4], nb[FROMY ? NCH : 1][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    float4 g = col < H ? *reinterpret_cast<const float4*>(gamma + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    gam[c][0] = g.x; gam[c][1] = g.y; gam[c][2] = g.z; gam[c][3] = g.w;
    if constexpr (FROMY) {
      const float4 b = col < H ? *reinterpret_cast<const float4*>(beta + col) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float bb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ig[c][i] = gam[c][i] != 0.f ? 1.f / gam[c][i] : 0.f;
        nb[c][i] = -bb[i] * ig[c][i];
      }
    }
  }
  const int row0 = blockIdx.x * kWaves * RPW + wave;
  // loads run TWO rows ahead (c = this row, n = next, f = the one after): with one row in flight per
  // wave the kernel left ~15 % of the HBM bandwidth unused at its 4 waves/SIMD occupancy
  uint2 cdy[NCH], cdy2[NCH], cz[NCH], ndy[NCH], ndy2[NCH], nz[NCH];
  float cmu = 0.f, crs = 0.f, nmu = 0.f, nrs = 0.f;
  if (row0 < T) {
    ln_bwd_load<NCH>(dy, dy2, z, (size_t)row0 * H, lane, H, cdy, cdy2, cz);
    cmu = mean[row0];
    crs = rstd[row0];
  }
  if (RPW > 1 && row0 + kWaves < T) {
    ln_bwd_load<NCH>(dy, dy2, z, (size_t)(row0 + kWaves) * H, lane, H, ndy, ndy2, nz);
    nmu = mean[row0 + kWaves];
    nrs = rstd[row0 + kWaves];
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = row0 + r * kWaves;
    if (row < T) {
      const size_t base = (size_t)row * H;
      uint2 fdy[NCH], fdy2[NCH], fz[NCH];
      float fmu = 0.f, frs = 0.f;
      const int frow = row + 2 * kWaves;
      if (r + 2 < RPW && frow < T) {
        ln_bwd_load<NCH>(dy, dy2, z, (size_t)frow * H, lane, H, fdy, fdy2, fz);
        fmu = mean[frow];
        frs = rstd[frow];
      }
      float g[NCH][4], xh[NCH][4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = c * 256 + lane * 4;
        if (col < H) {
          float fz[4], f2[4];
          hq_unpack4(cdy[c], g[c]);
          hq_unpack4(cdy2[c], f2);
          hq_unpack4(cz[c], fz);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            g[c][i] += f2[i];
            if constexpr (FROMY) xh[c][i] = fmaf(fz[i], ig[c][i], nb[c][i]);
            else xh[c][i] = (fz[i] - cmu) * crs;
            acc[0][c][i] += g[c][i] * xh[c][i];
            acc[1][c][i] += g[c][i];
            const float dxh = g[c][i] * gam[c][i];
            s1 += dxh;
            s2 += dxh * xh[c][i];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) { g[c][i] = 0.f; xh[c][i] = 0.f; }
        }
      }
      s1 = hq_wave_sum(s1) / H;
      s2 = hq_wave_sum(s2) / H;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = c * 256 + lane * 4;
        if (col < H) {
          float dz[4], m[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
          for (int i = 0; i < 4; ++i) dz[i] = crs * (g[c][i] * gam[c][i] - s1 - xh[c][i] * s2);
          *reinterpret_cast<uint2*>(dz_out + base + col) = hq_pack4(dz);
          if (thr) hq_keep4((uint32_t)(base + col), key, thr, kscale, m);
          float da[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) { da[i] = dz[i] * m[i]; acc[2][c][i] += da[i]; }
          const uint2 da_bf = hq_pack4(da);
          // da_out == null (Q8 only, --precision fp8 once every consumer reads da8): no bf16 da
          if (!Q8 || da_out != nullptr) *reinterpret_cast<uint2*>(da_out + base + col) = da_bf;
          if constexpr (Q8) {   // from the bf16-rounded da, exactly what the bf16 copy holds
            float r[4];
            hq_unpack4(da_bf, r);
#pragma unroll
            for (int i = 0; i < 4; ++i) amax8 = fmaxf(amax8, fabsf(r[i]));
            *reinterpret_cast<uint32_t*>(da8 + base + col) = hq_pack_bf8x4(r, inv8);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        cdy[c] = ndy[c]; cdy2[c] = ndy2[c]; cz[c] = nz[c];
        ndy[c] = fdy[c]; ndy2[c] = fdy2[c]; nz[c] = fz[c];
      }
      cmu = nmu; crs = nrs;
      nmu = fmu; nrs = frs;
    }
  }
  if constexpr (Q8) {   // this wave's amax -> its own partial slot (hq_fp8_amax_fold reduces them)
    amax8 = hq_wave_max(amax8);
    if (lane == 0) part8[blockIdx.x * kWaves + wave] = amax8;
  }
  block_partials<NCH, 3>(acc, lds, part, H);
}

// QA span head (reference model.py:30,54-58: position_outputs = Linear(H, 2) over the sequence
// output): fwd logits[t] = (seq[t]·w0 + b0, seq[t]·w1 + b1) in fp32 straight from the bf16 sequence
// (no fp32 copy of the [T, H] activations); bwd dseq[t] = g[t,0]·w0 + g[t,1]·w1 (bf16) plus
// deterministic per-block partials of dW = Σ_t g[t]ᵀ·seq[t].
template <int NCH>
__global__ __launch_bounds__(256) void span_fwd_kernel(const uint16_t* __restrict__ seq, const float* __restrict__ w,
                                                       const float* __restrict__ bias, float* __restrict__ logits, int T,
                                                       int H) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * kWaves + wave;
  if (row >= T) return;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    if (col < H) {
      float x[4];
      hq_unpack4(*reinterpret_cast<const uint2*>(seq + (size_t)row * H + col), x);
      const float4 a = *reinterpret_cast<const float4*>(w + col);
      const float4 b = *reinterpret_cast<const float4*>(w + H + col);
      s0 += x[0] * a.x + x[1] * a.y + x[2] * a.z + x[3] * a.w;
      s1 += x[0] * b.x + x[1] * b.y + x[2] * b.z + x[3] * b.w;
    }
  }
  s0 = hq_wave_sum(s0);
  s1 = hq_wave_sum(s1);
  if (lane == 0) *reinterpret_cast<float2*>(logits + 2 * (size_t)row) = make_float2(s0 + bias[0], s1 + bias[1]);
}

template <int NCH>
__global__ __launch_bounds__(256) void span_bwd_kernel(const uint16_t* __restrict__ seq, const float* __restrict__ w,
                                                       const float* __restrict__ g, uint16_t* __restrict__ dseq,
                                                       float* __restrict__ part, int T, int H, int rpw) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float acc[2][NCH][4];
  float w0[NCH][4], w1[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    const float4 a = col < H ? *reinterpret_cast<const float4*>(w + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b = col < H ? *reinterpret_cast<const float4*>(w + H + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    w0[c][0] = a.x; w0[c][1] = a.y; w0[c][2] = a.z; w0[c][3] = a.w;
    w1[c][0] = b.x; w1[c][1] = b.y; w1[c][2] = b.z; w1[c][3] = b.w;
#pragma unroll
    for (int i = 0; i < 4; ++i) { acc[0][c][i] = 0.f; acc[1][c][i] = 0.f; }
  }
  const int row0 = blockIdx.x * kWaves * rpw;
  for (int r = 0; r < rpw; ++r) {
    const int row = row0 + r * kWaves + wave;
    if (row >= T) break;
    const float2 gg = *reinterpret_cast<const float2*>(g + 2 * (size_t)row);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      if (col < H) {
        float x[4], d[4];
        hq_unpack4(*reinterpret_cast<const uint2*>(seq + (size_t)row * H + col), x);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[0][c][i] += gg.x * x[i];
          acc[1][c][i] += gg.y * x[i];
          d[i] = gg.x * w0[c][i] + gg.y * w1[c][i];
        }
        *reinterpret_cast<uint2*>(dseq + (size_t)row * H + col) = hq_pack4(d);
      }
    }
  }
  block_partials<NCH, 2>(acc, lds, part, H);
}

template <int NCH>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ pids,
                                                        const int64_t* __restrict__ tids, const uint16_t* __restrict__ ww,
                                                        const uint16_t* __restrict__ wp, const uint16_t* __restrict__ wt,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        uint16_t* __restrict__ y, float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, int T, int H, float eps, HqDropKey kd_,
                                                        uint32_t thr, float kscale, int V, int P, int NTY) {
  const uint32_t key = kd_.get();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * kWaves + wave;
  if (row >= T) return;
  HQ_DASSERT(ids[row] >= 0 && ids[row] < V && pids[row] >= 0 && pids[row] < P && tids[row] >= 0 && tids[row] < NTY);
  const size_t rw = (size_t)ids[row] * H, rp = (size_t)pids[row] * H, rt = (size_t)tids[row] * H;
  float v[NCH][4];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    if (col < H) {
      float f1[4], f2[4], f3[4];
      hq_unpack4(*reinterpret_cast<const uint2*>(ww + rw + col), f1);
      hq_unpack4(*reinterpret_cast<const uint2*>(wp + rp + col), f2);
      hq_unpack4(*reinterpret_cast<const uint2*>(wt + rt + col), f3);
#pragma unroll
      for (int i = 0; i < 4; ++i) { v[c][i] = f1[i] + f2[i] + f3[i]; sum += v[c][i]; }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[c][i] = 0.f;
    }
  }
  const float mu = hq_wave_sum(sum) / H;
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
    if (c * 256 + lane * 4 < H)
#pragma unroll
      for (int i = 0; i < 4; ++i) { float d = v[c][i] - mu; sq += d * d; }
  const float rs = rsqrtf(hq_wave_sum(sq) / H + eps);
  const size_t base = (size_t)row * H;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    if (col < H) {
      const float4 g = *reinterpret_cast<const float4*>(gamma + col);
      const float4 b = *reinterpret_cast<const float4*>(beta + col);
      float m[4] = {1.f, 1.f, 1.f, 1.f};
      if (thr) hq_keep4((uint32_t)(base + col), key, thr, kscale, m);
      float o[4] = {((v[c][0] - mu) * rs * g.x + b.x) * m[0], ((v[c][1] - mu) * rs * g.y + b.y) * m[1],
                    ((v[c][2] - mu) * rs * g.z + b.z) * m[2], ((v[c][3] - mu) * rs * g.w + b.w) * m[3]};
      *reinterpret_cast<uint2*>(y + base + col) = hq_pack4(o);
    }
  }
  if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
}

// Deterministic embedding backward (no float atomics at the default position ids):
//   1. sort: the token rows by word id (hq_sort_ids: own LSD radix sort of (id, row) pairs — stable, so each
//      id's rows stay in token order);
//   2. embed_bwd_kernel (position-major): recompute x̂ and the LayerNorm backward per row; γ / β / type
//      gradients as per-block partials, the position gradient summed per wave over its kEmbNB batch rows and
//      stored as that wave's partial row [blockIdx.y][l] (folded by colsum in a fixed order);
//   3. embed_word_kernel (id-major): the same per-row recompute over the SORTED rows, kEmbCH per wave, summing
//      each id's run in registers; a run inside the chunk is stored straight into its gradient row, the
//      pieces of a run that crosses chunk boundaries go to two carry rows per chunk;
//   4. embed_carry_kernel: the chunk where a crossing run starts adds its pieces in chunk order.
// Every sum has a fixed order, so the result is bitwise reproducible (the round-4 kernel scattered 75 M f32
// atomics into the word gradients: 316 µs at T = 98304 and run-to-run different low bits).
// Position ids other than l (RoBERTa's l + 2, user-supplied ids) fall back to f32 atomics for those rows.
//
// part layout per block: [gamma | beta | type0 | type1] × H
//
// Position-major traversal: wave w of block (x, y) owns sequence position l = x·4 + w and walks the
// kEmbNB batch rows b = y·kEmbNB … (row = b·L + l).  The next row's dy / embedding rows / statistics are
// loaded while the current row is reduced (one dependent HBM round trip per row otherwise).
constexpr int kEmbNB = 16;       // batch rows per wave in the position pass (<= 64, as kEmbCH)
constexpr int kEmbCH = 16;       // sorted rows per wave in the word pass (<= 64: one row's metadata per lane)
constexpr int kEmbMaxL = 4096;   // position partials [T / L / kEmbNB][min(L, P)][H] only for real sequence layouts

template <int NCH>
struct EmbRow {
  int64_t id, pid, tid;
  float mu, rs;
  uint2 w[NCH], p[NCH], t[NCH], d[NCH];
};

// Row metadata of up to 64 rows, one row per lane (ids, position / type ids, LayerNorm statistics), loaded once
// up front: the per-row loop then reads them with v_readlane and issues only the row-data loads — no dependent
// index → row round trip inside the loop.
struct EmbMeta {
  int id, pid, tid;
  float mu, rs;
};
__device__ __forceinline__ EmbMeta emb_meta_load(int64_t row, bool ok, const int64_t* __restrict__ ids,
                                                 const int64_t* __restrict__ pids, const int64_t* __restrict__ tids,
                                                 const float* __restrict__ mean, const float* __restrict__ rstd) {
  EmbMeta m{0, 0, 0, 0.f, 0.f};
  if (ok) { m.id = (int)ids[row]; m.pid = (int)pids[row]; m.tid = (int)tids[row]; m.mu = mean[row]; m.rs = rstd[row]; }
  return m;
}
// row data of the row whose metadata lane k holds
template <int NCH>
__device__ __forceinline__ void emb_load_k(EmbRow<NCH>& r, const EmbMeta& m, int k, size_t row, const uint16_t* __restrict__ dy,
                                           const uint16_t* __restrict__ ww, const uint16_t* __restrict__ wp,
                                           const uint16_t* __restrict__ wt, int H, int lane) {
  r.id = __builtin_amdgcn_readlane(m.id, k);
  r.pid = __builtin_amdgcn_readlane(m.pid, k);
  r.tid = __builtin_amdgcn_readlane(m.tid, k);
  r.mu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m.mu), k));
  r.rs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m.rs), k));
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    if (col < H) {
      r.w[c] = *reinterpret_cast<const uint2*>(ww + (size_t)r.id * H + col);
      r.p[c] = *reinterpret_cast<const uint2*>(wp + (size_t)r.pid * H + col);
      r.t[c] = *reinterpret_cast<const uint2*>(wt + (size_t)r.tid * H + col);
      r.d[c] = *reinterpret_cast<const uint2*>(dy + row * H + col);
    }
  }
}

// One row's LayerNorm backward from the recomputed x̂: g = dropout-masked dy, x̂, and dx = ∂/∂(word+pos+type).
template <int NCH>
__device__ __forceinline__ void emb_row_grad(const EmbRow<NCH>& cur, size_t base, const float (&gam)[NCH][4],
                                             uint32_t key, uint32_t thr, float kscale, int H, int lane,
                                             float (&g)[NCH][4], float (&xh)[NCH][4], float (&dx)[NCH][4]) {
  const float mu = cur.mu, rs = cur.rs;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    if (col < H) {
      float f1[4], f2[4], f3[4], m[4] = {1.f, 1.f, 1.f, 1.f};
      hq_unpack4(cur.w[c], f1);
      hq_unpack4(cur.p[c], f2);
      hq_unpack4(cur.t[c], f3);
      hq_unpack4(cur.d[c], g[c]);
      if (thr) hq_keep4((uint32_t)(base + col), key, thr, kscale, m);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        g[c][i] *= m[i];
        xh[c][i] = (f1[i] + f2[i] + f3[i] - mu) * rs;
        const float dxh = g[c][i] * gam[c][i];
        s1 += dxh;
        s2 += dxh * xh[c][i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) { g[c][i] = 0.f; xh[c][i] = 0.f; }
    }
  }
  s1 = hq_wave_sum(s1) / H;
  s2 = hq_wave_sum(s2) / H;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) dx[c][i] = c * 256 + lane * 4 < H ? rs * (g[c][i] * gam[c][i] - s1 - xh[c][i] * s2) : 0.f;
}

template <int NCH>
__device__ __forceinline__ void emb_gamma(const float* __restrict__ gamma, int H, int lane, float (&gam)[NCH][4]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    const float4 g = col < H ? *reinterpret_cast<const float4*>(gamma + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    gam[c][0] = g.x; gam[c][1] = g.y; gam[c][2] = g.z; gam[c][3] = g.w;
  }
}

template <int NCH>
__global__ __launch_bounds__(256) void embed_bwd_kernel(
    const uint16_t* __restrict__ dy, const int64_t* __restrict__ ids, const int64_t* __restrict__ pids,
    const int64_t* __restrict__ tids, const uint16_t* __restrict__ ww, const uint16_t* __restrict__ wp,
    const uint16_t* __restrict__ wt, const float* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ rstd, float* __restrict__ g_pos, float* __restrict__ g_type, float* __restrict__ ppart,
    float* __restrict__ part, int T, int H, int n_types, int pad_pos, HqDropKey kd_, uint32_t thr, float kscale, int V,
    int P, int B, int L, int PL) {
  const uint32_t key = kd_.get();
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [4][H] block-partial scratch
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  float acc[4][NCH][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[q][c][i] = 0.f;
  float gam[NCH][4], pacc[NCH][4];
  emb_gamma<NCH>(gamma, H, lane, gam);
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) pacc[c][i] = 0.f;
  const int l = blockIdx.x * kWaves + wave;
  // this wave's position-partial row [blockIdx.y][l] (l < PL = min(L, P): pid == l needs l < P; ppart = null:
  // every position flush is atomic)
  float* prow = (ppart != nullptr && l < PL) ? ppart + ((size_t)blockIdx.y * PL + l) * H : nullptr;
  // the partial rows are [ceil(B / kEmbNB)][PL][H] with PL = min(L, P): row l exists only for l < PL (77ab202: the
  // flat layout, L = T > P, once wrote rows past the buffer)
  HQ_DASSERT(prow == nullptr || (l < PL && PL <= P && (int)blockIdx.y < (B + kEmbNB - 1) / kEmbNB));
  bool pstored = false;
  int pcur = -1;
  auto flush_pos = [&]() {
    if (pcur >= 0 && pcur != pad_pos) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = c * 256 + lane * 4;
        if (col < H) {
          if (prow != nullptr && pcur == l) {   // the default ids: the wave's own partial row, plain stores
            float4 v = make_float4(pacc[c][0], pacc[c][1], pacc[c][2], pacc[c][3]);
            if (pstored) {
              const float4 o = *reinterpret_cast<const float4*>(prow + col);
              v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
            }
            *reinterpret_cast<float4*>(prow + col) = v;
          } else {
            HQ_DASSERT(pcur >= 0 && pcur < P);
#pragma unroll
            for (int i = 0; i < 4; ++i) atomicAdd(g_pos + (size_t)pcur * H + col + i, pacc[c][i]);
          }
        }
      }
      if (prow != nullptr && pcur == l) pstored = true;
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) pacc[c][i] = 0.f;
  };
  const int b0 = blockIdx.y * kEmbNB, b1 = l < L ? min(B, b0 + kEmbNB) : b0;
  // rows two ahead in a ring of three (compile-time slots in the unrolled loop: a rotation by copies would wait
  // for the newest loads at every copy)
  const EmbMeta meta = emb_meta_load((int64_t)(b0 + lane) * L + l, lane < b1 - b0, ids, pids, tids, mean, rstd);
  EmbRow<NCH> cur, nxt;
  if (b0 < b1) emb_load_k<NCH>(nxt, meta, 0, (size_t)b0 * L + l, dy, ww, wp, wt, H, lane);
#pragma unroll 1
  for (int b = b0; b < b1; ++b) {
    const size_t row = (size_t)b * L + l;
    cur = nxt;
    if (b + 1 < b1) emb_load_k<NCH>(nxt, meta, b + 1 - b0, row + L, dy, ww, wp, wt, H, lane);
    const int64_t pid = cur.pid, tid = cur.tid;
    HQ_DASSERT(cur.id >= 0 && cur.id < V && pid >= 0 && pid < P && tid >= 0 && tid < n_types);
    float g[NCH][4], xh[NCH][4], dx[NCH][4];
    emb_row_grad<NCH>(cur, row * H, gam, key, thr, kscale, H, lane, g, xh, dx);
    if ((int)pid != pcur) {  // wave-uniform: the running position sum belongs to another position
      flush_pos();
      pcur = (int)pid;
    }
    const bool t1 = (tid & 1) != 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      if (col < H) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[0][c][i] += g[c][i] * xh[c][i];
          acc[1][c][i] += g[c][i];
          pacc[c][i] += dx[c][i];
        }
        if (n_types <= 2) {  // static indices only: acc[2 + (tid & 1)] put the whole array in scratch memory
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc[2][c][i] += t1 ? 0.f : dx[c][i];
            acc[3][c][i] += t1 ? dx[c][i] : 0.f;
          }
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) atomicAdd(g_type + (size_t)tid * H + col + i, dx[c][i]);
        }
      }
    }
  }
  flush_pos();
  if (prow != nullptr && !pstored) {   // no row at position l in this batch slice: a zero partial
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      if (col < H) *reinterpret_cast<float4*>(prow + col) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();
  block_partials<NCH, 4>(acc, lds, part, H);
}

// ---- own stable LSD radix sort of the (word id, row) pairs: 8-bit digits, ceil(bits / 8) passes -------------
// Each pass is a stable counting sort over 256 bins in tiles of kSortTile rows:
//   sort_hist_kernel (first pass only): per-tile digit counts -> hist[digit][tile] (LDS integer atomics);
//   sort_scan_kernel: one block, exclusive scan of hist in (digit, tile) order -> every tile's start per digit;
//                     also zeroes the next pass's histogram;
//   sort_scatter_kernel: each wave ranks its 64-row batches by digit with 8 ballots (the lanes holding the same
//                     digit, in lane order), batch counts are scanned per digit in LDS, and every row goes to
//                     tile start + earlier batches + rank — stable, so each id's rows keep token order.  It also
//                     counts the NEXT pass's digits of the tile each row lands in (integer atomics).
// Integer counts and fixed ranks: the output is the same permutation every run (no float, no order race).
constexpr int kSortTile = 1024;   // 256 threads × 4 batches of 64

__global__ __launch_bounds__(256) void sort_hist_kernel(const int64_t* __restrict__ ids, int T, int* __restrict__ hist,
                                                        int ntiles) {
  __shared__ int cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const int t0 = blockIdx.x * kSortTile;
  for (int i = threadIdx.x; i < kSortTile; i += 256)
    if (t0 + i < T) atomicAdd(&cnt[(int)ids[t0 + i] & 255], 1);
  __syncthreads();
  hist[threadIdx.x * ntiles + blockIdx.x] = cnt[threadIdx.x];
}

// Exclusive scan of the (digit, tile) histogram by one block: coalesced 16 K-entry chunks through LDS (a thread's
// contiguous run read straight from global memory was latency-bound: 35 µs), each thread scans 16 consecutive
// entries, the 1024 run totals are scanned wave by wave, a running carry links the chunks.
__global__ __launch_bounds__(1024) void sort_scan_kernel(int* __restrict__ hist, int n, int* __restrict__ next_hist) {
  constexpr int kPer = 16, kChunk = 1024 * kPer;
  __shared__ int buf[kChunk];
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int carry = 0;
  for (int base = 0; base < n; base += kChunk) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = base + k * 1024 + tid;
      buf[k * 1024 + tid] = i < n ? hist[i] : 0;
    }
    __syncthreads();
    int v[kPer], run = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) { v[k] = buf[tid * kPer + k]; run += v[k]; }
    int incl = run;   // inclusive scan of the run totals within the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int before = carry;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    int total = carry;
    for (int w = 0; w < 16; ++w) total += wsum[w];
    int ex = before + incl - run;
#pragma unroll
    for (int k = 0; k < kPer; ++k) { buf[tid * kPer + k] = ex; ex += v[k]; }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = base + k * 1024 + tid;
      if (i < n) hist[i] = buf[k * 1024 + tid];
    }
    carry = total;
    __syncthreads();
  }
  if (next_hist)
    for (int i = tid; i < n; i += 1024) next_hist[i] = 0;
}

__global__ __launch_bounds__(256) void sort_scatter_kernel(const int64_t* __restrict__ ids, const int32_t* __restrict__ kin,
                                                           const int32_t* __restrict__ vin, int32_t* __restrict__ kout,
                                                           int32_t* __restrict__ vout, const int* __restrict__ start,
                                                           int* __restrict__ next_hist, int T, int shift, int ntiles) {
  __shared__ int bcnt[16][256];   // [batch][digit]: rows of the digit in the batch, then their exclusive prefix
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 16 * 256; i += 256) (&bcnt[0][0])[i] = 0;
  __syncthreads();
  const int t0 = blockIdx.x * kSortTile;
  const uint64_t lt = (1ull << lane) - 1ull;
  int key[4], val[4], dig[4], rank[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = wave * 4 + j;            // batch q covers tile rows q·64 … q·64 + 63 (tile order)
    const int i = t0 + q * 64 + lane;
    const bool ok = i < T;
    key[j] = ok ? (kin ? kin[i] : (int)ids[i]) : 0;
    val[j] = ok ? (vin ? vin[i] : i) : 0;
    dig[j] = (key[j] >> shift) & 255;
    uint64_t peers = __ballot(ok);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const bool on = (dig[j] >> bit) & 1;
      const uint64_t m = __ballot(on);
      peers &= on ? m : ~m;
    }
    rank[j] = __popcll(peers & lt);
    if (ok && rank[j] == 0) bcnt[q][dig[j]] = __popcll(peers);   // the digit's first lane writes the batch count
    if (!ok) rank[j] = -1;
  }
  __syncthreads();
  {   // per digit (one per thread): exclusive prefix over the 16 batches, in batch order
    int run = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = bcnt[q][tid];
      bcnt[q][tid] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (rank[j] < 0) continue;
    const int q = wave * 4 + j;
    const int pos = start[dig[j] * ntiles + blockIdx.x] + bcnt[q][dig[j]] + rank[j];
    HQ_DASSERT(pos >= 0 && pos < T);
    kout[pos] = key[j];
    vout[pos] = val[j];
    if (next_hist) atomicAdd(&next_hist[((key[j] >> (shift + 8)) & 255) * ntiles + pos / kSortTile], 1);
  }
}

// Word gradients over the id-sorted rows.  Wave c owns sorted positions [c·kEmbCH, …); the run of one id is
// summed in token order.  Run kinds: inside the chunk → stored into g_word[id] (fresh: =, accumulate: +=);
// the chunk's FIRST run when it continues from chunk c-1 → carry slot 0 of c; the chunk's LAST run when it
// continues into chunk c+1 and began in this chunk → carry slot 1 of c (a run covering the whole chunk from
// both sides is slot 0).  embed_carry_kernel completes the crossing runs.  Padding ids get no gradient.
template <int NCH>
__global__ __launch_bounds__(256) void embed_word_kernel(
    const int32_t* __restrict__ skeys, const int32_t* __restrict__ srows, const uint16_t* __restrict__ dy,
    const int64_t* __restrict__ ids, const int64_t* __restrict__ pids, const int64_t* __restrict__ tids,
    const uint16_t* __restrict__ ww, const uint16_t* __restrict__ wp, const uint16_t* __restrict__ wt,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ rstd,
    float* __restrict__ g_word, float* __restrict__ carry, int T, int H, int pad_word, int accumulate, HqDropKey kd_,
    uint32_t thr, float kscale, int V) {
  const uint32_t key = kd_.get();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int c = blockIdx.x * kWaves + wave;
  const int j0 = c * kEmbCH;
  if (j0 >= T) return;
  const int j1 = min(T, j0 + kEmbCH);
  float gam[NCH][4], acc[NCH][4];
  emb_gamma<NCH>(gamma, H, lane, gam);
#pragma unroll
  for (int q = 0; q < NCH; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[q][i] = 0.f;
  const int first = __builtin_amdgcn_readfirstlane(skeys[j0]);
  const bool head_cont = c > 0 && __builtin_amdgcn_readfirstlane(skeys[j0 - 1]) == first;
  const int after = j1 < T ? __builtin_amdgcn_readfirstlane(skeys[j1]) : -1;
  auto flush = [&](int id, int kind) {   // kind 0: carry slot 0, 1: carry slot 1, 2: the gradient row
    if (id != pad_word) {
      // a gradient row of a real id, or carry slot (c, kind) of the [chunks][2][H] carry buffer
      HQ_DASSERT(kind == 2 ? (id >= 0 && id < V) : (kind >= 0 && kind < 2 && c * kEmbCH < T));
      float* dst = kind == 2 ? g_word + (size_t)id * H : carry + ((size_t)c * 2 + kind) * H;
#pragma unroll
      for (int q = 0; q < NCH; ++q) {
        const int col = q * 256 + lane * 4;
        if (col < H) {
          float4 v = make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]);
          if (kind == 2 && accumulate) {
            const float4 o = *reinterpret_cast<const float4*>(dst + col);
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *reinterpret_cast<float4*>(dst + col) = v;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NCH; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[q][i] = 0.f;
  };
  int seg = first;
  bool seg_first = true;
  // the chunk's sorted rows and their metadata, one per lane (kEmbCH <= 64)
  const int myrow = lane < j1 - j0 ? srows[j0 + lane] : 0;
  const EmbMeta meta = emb_meta_load(myrow, lane < j1 - j0, ids, pids, tids, mean, rstd);
  EmbRow<NCH> cur, nxt;
  emb_load_k<NCH>(nxt, meta, 0, (size_t)__builtin_amdgcn_readlane(myrow, 0), dy, ww, wp, wt, H, lane);
#pragma unroll 1
  for (int j = j0; j < j1; ++j) {
    const size_t row = (size_t)__builtin_amdgcn_readlane(myrow, j - j0);
    cur = nxt;
    if (j + 1 < j1)
      emb_load_k<NCH>(nxt, meta, j + 1 - j0, (size_t)__builtin_amdgcn_readlane(myrow, j + 1 - j0), dy, ww, wp, wt, H, lane);
    const int id = (int)cur.id;
    HQ_DASSERT(id >= 0 && id < V && row < (size_t)T);
    if (id != seg) {
      flush(seg, seg_first && head_cont ? 0 : 2);
      seg = id;
      seg_first = false;
    }
    float g[NCH][4], xh[NCH][4], dx[NCH][4];
    emb_row_grad<NCH>(cur, row * H, gam, key, thr, kscale, H, lane, g, xh, dx);
#pragma unroll
    for (int q = 0; q < NCH; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[q][i] += dx[q][i];
  }
  const bool from_prev = seg_first && head_cont;
  flush(seg, from_prev ? 0 : (after == seg ? 1 : 2));
}

// Runs that cross chunk boundaries: the chunk holding a run's start piece (carry slot 1) adds the following
// chunks' slot-0 pieces in chunk order and stores the gradient row.
template <int NCH>
__global__ __launch_bounds__(256) void embed_carry_kernel(const int32_t* __restrict__ skeys, const float* __restrict__ carry,
                                                          float* __restrict__ g_word, int T, int H, int pad_word,
                                                          int accumulate, int V) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int c = blockIdx.x * kWaves + wave;
  const int j0 = c * kEmbCH;
  if (j0 >= T) return;
  const int j1 = min(T, j0 + kEmbCH);
  const int last = __builtin_amdgcn_readfirstlane(skeys[j1 - 1]);
  if (j1 >= T || skeys[j1] != last || last == pad_word) return;                  // the last run ends here
  if (skeys[j0] == last && c > 0 && skeys[j0 - 1] == last) return;               // ... or began before
  // end of the run: the first sorted position past j1 whose key differs, by a 64-ary search over the sorted keys
  int lo = j1, hi = T;   // skeys[lo] == last; the end lies in (lo, hi]
  while (hi - lo > 1) {
    const int step = (hi - lo + 63) / 64;
    const int q = lo + lane * step;
    const bool in = q < hi && skeys[q] == last;
    const uint64_t m = __ballot(in);   // a prefix of the lanes (sorted keys)
    const int k = 63 - __builtin_clzll(m);
    lo = lo + k * step;
    hi = min(hi, lo + step);
  }
  const int ce = (hi - 1) / kEmbCH;   // the last chunk holding rows of the run: pieces of chunks c+1 … ce
  HQ_DASSERT(last >= 0 && last < V && hi <= T && ce * kEmbCH < T && ce > c);
  float acc[NCH][4];
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int col = q * 256 + lane * 4;
    const float4 v = col < H ? *reinterpret_cast<const float4*>(carry + ((size_t)c * 2 + 1) * H + col)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    acc[q][0] = v.x; acc[q][1] = v.y; acc[q][2] = v.z; acc[q][3] = v.w;
  }
  for (int cc = c + 1; cc <= ce; cc += 8) {   // 8 pieces in flight, added in chunk order
    float4 v[8][NCH];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int q = 0; q < NCH; ++q) {
        const int col = q * 256 + lane * 4;
        v[u][q] = (cc + u <= ce && col < H) ? *reinterpret_cast<const float4*>(carry + ((size_t)(cc + u) * 2) * H + col)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (cc + u <= ce)
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
          acc[q][0] += v[u][q].x; acc[q][1] += v[u][q].y; acc[q][2] += v[u][q].z; acc[q][3] += v[u][q].w;
        }
  }
  float* dst = g_word + (size_t)last * H;
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int col = q * 256 + lane * 4;
    if (col < H) {
      float4 v = make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]);
      if (accumulate) {
        const float4 o = *reinterpret_cast<const float4*>(dst + col);
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
      }
      *reinterpret_cast<float4*>(dst + col) = v;
    }
  }
}

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const uint16_t* __restrict__ pre, uint16_t* __restrict__ out, size_t n8) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float x[8], o[8];
    hq_unpack8(reinterpret_cast<const uint4*>(pre)[i], x);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = hq_gelu(x[k]);
    reinterpret_cast<uint4*>(out)[i] = hq_pack8(o);
  }
}

// dpre = dout * gelu'(pre); per-block column partials of dpre.  Block: 256 threads × 8 columns =
// 2048-column tile, kRowsBlock rows.  grid = (ceil(N/2048), ceil(T/kRowsBlock)).
constexpr int kRowsBlock = 32;
__global__ __launch_bounds__(256) void gelu_bwd_kernel(const uint16_t* __restrict__ dout, const uint16_t* __restrict__ pre,
                                                       uint16_t* __restrict__ dpre, float* __restrict__ part, int T, int N) {
  const int col = (blockIdx.x * 256 + threadIdx.x) * 8;
  const int r0 = blockIdx.y * kRowsBlock;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (col < N) {
    for (int r = r0; r < min(T, r0 + kRowsBlock); ++r) {
      const size_t off = (size_t)r * N + col;
      float d[8], x[8], o[8];
      hq_unpack8(*reinterpret_cast<const uint4*>(dout + off), d);
      hq_unpack8(*reinterpret_cast<const uint4*>(pre + off), x);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float cdf, pdf;
        hq_normal_cdf_pdf(x[k], cdf, pdf);
        o[k] = d[k] * (cdf + x[k] * pdf);
        acc[k] += o[k];
      }
      *reinterpret_cast<uint4*>(dpre + off) = hq_pack8(o);
    }
    float* dst = part + (size_t)blockIdx.y * N + col;
    *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

__global__ __launch_bounds__(256) void colpart_kernel(const uint16_t* __restrict__ x, float* __restrict__ part, int T, int N) {
  const int col = (blockIdx.x * 256 + threadIdx.x) * 8;
  const int r0 = blockIdx.y * kRowsBlock;
  if (col >= N) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = r0; r < min(T, r0 + kRowsBlock); ++r) {
    float d[8];
    hq_unpack8(*reinterpret_cast<const uint4*>(x + (size_t)r * N + col), d);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += d[k];
  }
  float* dst = part + (size_t)blockIdx.y * N + col;
  *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// out[q*H + c] (+)= Σ_p part[p][q][c]   for the columns named by (Q, H): part is [P][Q*H].
// One 1024-thread block per 64 columns; 16 waves stride over the logical rows p < P, which live at
// physical rows p·Pphys/P (Pphys == P: all rows; otherwise the chunk heads of colsum_chunk_kernel).
// LDS combine.  Deterministic.
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ part, int P, int N, HqOuts outs, int Hq,
                                                      int accumulate, int Pphys) {
  __shared__ float red[16][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < N) {
    if (Pphys == P) {
      int p = wave;
      for (; p + 48 < P; p += 64) {
        s += part[(size_t)p * N + col] + part[(size_t)(p + 16) * N + col] + part[(size_t)(p + 32) * N + col] +
             part[(size_t)(p + 48) * N + col];
      }
      for (; p < P; p += 16) s += part[(size_t)p * N + col];
    } else {
      for (int p = wave; p < P; p += 16) s += part[(size_t)((long)p * Pphys / P) * N + col];
    }
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    float* out = outs.p[col / Hq];
    if (out) {
      const int c = col % Hq;
      out[c] = accumulate ? out[c] + t : t;
    }
  }
}

// First pass for tall partial matrices: block (x, c) sums rows [c·P/C, (c+1)·P/C) of its 64 columns
// and writes the sum over the chunk's FIRST row (a row only this block reads), so the pass needs no
// scratch and stays deterministic; colsum_kernel then folds the C chunk heads.  The single-pass
// kernel ran only N/64 blocks (36 for a 2304-column LayerNorm partial of 3072 rows: ~20 µs).
__global__ __launch_bounds__(1024) void colsum_chunk_kernel(float* __restrict__ part, int P, int N, int C) {
  __shared__ float red[16][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = blockIdx.x * 64 + lane;
  const int r0 = (int)((long)blockIdx.y * P / C), r1 = (int)((long)(blockIdx.y + 1) * P / C);
  float s = 0.f;
  if (col < N)
    for (int p = r0 + wave; p < r1; p += 16) s += part[(size_t)p * N + col];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    part[(size_t)r0 * N + col] = t;
  }
}

// The same first pass with 16-B loads: block (x, c) = 4 waves over 256 columns (a float4 per lane) and rows
// [c·P/C, (c+1)·P/C); each wave walks every 4th row with 4 loads in flight, the block folds its 4 waves in LDS in
// wave order.  The 64-column form issued 4-B loads (256 B per wave instruction, one row at a time): 9.7 µs for a
// 28 MB LayerNorm partial (2.9 TB/s).  Needs N % 4 == 0 and 16-B-aligned rows.
__global__ __launch_bounds__(256) void colsum_chunk4_kernel(float* __restrict__ part, int P, int N, int C) {
  __shared__ float4 red[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c4 = blockIdx.x * 64 + lane;                       // float4 column index
  const int n4 = N >> 2;
  const int r0 = (int)((long)blockIdx.y * P / C), r1 = (int)((long)(blockIdx.y + 1) * P / C);
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  if (c4 < n4) {
    int p = r0 + wave;
    for (; p + 12 < r1; p += 16) {   // 4 rows in flight, two accumulators (fixed association per wave)
      const float4 v0 = p4[(size_t)p * n4 + c4], v1 = p4[(size_t)(p + 4) * n4 + c4];
      const float4 v2 = p4[(size_t)(p + 8) * n4 + c4], v3 = p4[(size_t)(p + 12) * n4 + c4];
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      b.x += v1.x; b.y += v1.y; b.z += v1.z; b.w += v1.w;
      a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
      b.x += v3.x; b.y += v3.y; b.z += v3.z; b.w += v3.w;
    }
    for (; p < r1; p += 4) {
      const float4 v = p4[(size_t)p * n4 + c4];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[wave][lane] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  __syncthreads();
  if (wave == 0 && c4 < n4) {
    float4 t = red[0][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) { const float4 v = red[w][lane]; t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w; }
    reinterpret_cast<float4*>(part)[(size_t)r0 * n4 + c4] = t;
  }
}

template <typename F>
void dispatch_nch(int H, F&& f) {
  const int nch = (H + 255) / 256;
  switch (nch) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    case 6: f(std::integral_constant<int, 6>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    default: fprintf(stderr, "hq: unsupported hidden size %d\n", H); abort();
  }
}

void colsum(const float* part, int P, int N, HqOuts outs, int Hq, bool accumulate, hipStream_t s) {
  const int C = P >= 128 ? std::min(32, P / 32) : P;
  if (C < P) {
    if (N % 4 == 0 && reinterpret_cast<uintptr_t>(part) % 16 == 0)
      hipLaunchKernelGGL(colsum_chunk4_kernel, dim3((N / 4 + 63) / 64, C), dim3(256), 0, s, const_cast<float*>(part), P, N,
                         C);
    else
      hipLaunchKernelGGL(colsum_chunk_kernel, dim3((N + 63) / 64, C), dim3(1024), 0, s, const_cast<float*>(part), P, N, C);
  }
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64), dim3(1024), 0, s, part, C, N, outs, Hq, accumulate ? 1 : 0, P);
}

}  // namespace

// Zero-fill of a gradient buffer (the embedding backward's fresh g_word / g_pos): an own grid-stride kernel with
// 16-B stores instead of hipMemsetAsync, so the step's graph holds kernel nodes only (a runtime memset node
// is the one kind of node the rest of the step never uses) and the step trace names every kernel.
// p[0, head) and the last `tail` (< 4 each) are the unaligned ends, [head, head + 4·n4) the 16-B-aligned body
__global__ __launch_bounds__(256) void zero_f32_kernel(float* __restrict__ p, int head, size_t n4, int tail) {
  float4* body = reinterpret_cast<float4*>(p + head);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) body[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (blockIdx.x == 0) {
    if ((int)threadIdx.x < head) p[threadIdx.x] = 0.f;
    if ((int)threadIdx.x < tail) p[head + 4 * n4 + threadIdx.x] = 0.f;
  }
}

// ================================================================================== launchers
namespace {
const uint32_t* g_seed_ptr = nullptr;
}
void hq_set_dropout_seed_ptr(const uint32_t* p) { g_seed_ptr = p; }
void hq_zero_f32(float* p, size_t n, hipStream_t s) {
  if (n == 0) return;
  const size_t mis = (reinterpret_cast<uintptr_t>(p) / sizeof(float)) % 4;   // p is 4-B aligned (f32 tensor)
  const int head = (int)std::min<size_t>(n, mis ? 4 - mis : 0);
  const size_t n4 = (n - head) / 4;
  const int tail = (int)(n - head - 4 * n4);
  const size_t blocks = (n4 + 255) / 256;
  const int grid = (int)(blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks));
  hipLaunchKernelGGL(zero_f32_kernel, dim3(grid), dim3(256), 0, s, p, head, n4, tail);
}
HqDropKey hq_drop_key(uint32_t seed, uint32_t opid) { return HqDropKey{hq_op_key(seed, opid), opid, g_seed_ptr}; }

void hq_ln_fwd(const uint16_t* a, const uint16_t* resid, const float* gamma, const float* beta, uint16_t* y, uint16_t* z,
               float* mean, float* rstd, int T, int H, float eps, float p, uint32_t seed, uint32_t opid, hipStream_t s,
               uint8_t* y8, float* q8, int phase) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey key = hq_drop_key(seed, opid);
  const float ks = hq_keep_scale(thr);
  constexpr int rpw = 2;   // rows per wave (1 / 2 / 4 measured: profiles/r3_ln_rpw)
  const int grid = (T + kWaves * rpw - 1) / (kWaves * rpw);
  float* part8 = y8 ? hq_fp8_amax_parts((size_t)grid * kWaves, q8, s) : nullptr;
  dispatch_nch(H, [&](auto nch) {
    constexpr int C = decltype(nch)::value;
    auto go = [&](auto R, auto res, auto q) {
      hipLaunchKernelGGL((ln_fwd_rows_kernel<C, decltype(R)::value, decltype(res)::value, decltype(q)::value>),
                         dim3(grid), dim3(256), 0, s, a, resid, gamma, beta, y, z, mean, rstd, T, H, eps, key, thr, ks,
                         y8, q8, part8, phase);
    };
    auto by_rows = [&](auto res, auto q) {
      if (rpw == 1) go(std::integral_constant<int, 1>{}, res, q);
      else if (rpw == 4) go(std::integral_constant<int, 4>{}, res, q);
      else go(std::integral_constant<int, 2>{}, res, q);
    };
    // resid == null: a = z from an EPI_BDR GEMM epilogue
    if (y8) { if (resid) by_rows(std::true_type{}, std::true_type{}); else by_rows(std::false_type{}, std::true_type{}); }
    else if (resid) by_rows(std::true_type{}, std::false_type{});
    else by_rows(std::false_type{}, std::false_type{});
  });
  if (y8) hq_fp8_amax_fold(part8, grid * kWaves, q8, phase, s);
}

static int ln_rows_per_wave(int T) { return T >= 16384 ? kRowsPerWave : 2; }
int hq_ln_bwd_partials(int T) {
  const int rpw = ln_rows_per_wave(T);
  return (T + kWaves * rpw - 1) / (kWaves * rpw);
}
int hq_embed_bwd_partials(int T, int L) {
  if (L <= 0 || T % L) L = T;
  return ((L + kWaves - 1) / kWaves) * ((T / L + kEmbNB - 1) / kEmbNB);
}

void hq_ln_bwd(const uint16_t* dy, const uint16_t* dy2, const uint16_t* z, const float* gamma, const float* mean,
               const float* rstd, uint16_t* dz, uint16_t* da, float* part, HqOuts outs, int T, int H, float p,
               uint32_t seed, uint32_t opid, bool accumulate, hipStream_t s, uint8_t* da8, float* q8, int phase,
               const float* beta) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey key = hq_drop_key(seed, opid);
  const float ks = hq_keep_scale(thr);
  const int nb = hq_ln_bwd_partials(T);
  float* part8 = da8 ? hq_fp8_amax_parts((size_t)nb * kWaves, q8, s) : nullptr;
  dispatch_nch(H, [&](auto nch) {
    constexpr int C = decltype(nch)::value;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 4 * H * sizeof(float), s, dy, dy2, z, gamma, mean, rstd, dz, da, part,
                         T, H, key, thr, ks, da8, q8, part8, phase, beta);
    };
    // beta != null: `z` is the forward output y (FROMY)
    if (ln_rows_per_wave(T) == kRowsPerWave) {
      if (da8) { if (beta) go(ln_bwd_kernel<C, kRowsPerWave, true, true>); else go(ln_bwd_kernel<C, kRowsPerWave, true, false>); }
      else { if (beta) go(ln_bwd_kernel<C, kRowsPerWave, false, true>); else go(ln_bwd_kernel<C, kRowsPerWave, false, false>); }
    } else {
      if (da8) { if (beta) go(ln_bwd_kernel<C, 2, true, true>); else go(ln_bwd_kernel<C, 2, true, false>); }
      else { if (beta) go(ln_bwd_kernel<C, 2, false, true>); else go(ln_bwd_kernel<C, 2, false, false>); }
    }
  });
  if (da8) hq_fp8_amax_fold(part8, nb * kWaves, q8, phase, s, kHqBf8Max);
  colsum(part, nb, 3 * H, outs, H, accumulate, s);
}

void hq_embed_fwd(const int64_t* ids, const int64_t* pids, const int64_t* tids, const uint16_t* ww, const uint16_t* wp,
                  const uint16_t* wt, const float* gamma, const float* beta, uint16_t* y, float* mean, float* rstd, int T,
                  int H, float eps, float p, uint32_t seed, uint32_t opid, int V, int P, int NTY, hipStream_t s) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey key = hq_drop_key(seed, opid);
  const float ks = hq_keep_scale(thr);
  dispatch_nch(H, [&](auto nch) {
    hipLaunchKernelGGL(embed_fwd_kernel<decltype(nch)::value>, dim3((T + kWaves - 1) / kWaves), dim3(256), 0, s, ids,
                       pids, tids, ww, wp, wt, gamma, beta, y, mean, rstd, T, H, eps, key, thr, ks, V, P, NTY);
  });
}

static int emb_sort_bits(int V) { return V > 1 ? 32 - __builtin_clz((unsigned)(V - 1)) : 1; }
static int emb_sort_passes(int V) { return (emb_sort_bits(V) + 7) / 8; }
static int emb_sort_tiles(int T) { return (T + kSortTile - 1) / kSortTile; }

size_t hq_sort_ids_bytes(int T, int V) { return (size_t)emb_sort_passes(V) * 256 * emb_sort_tiles(T) * sizeof(int); }

// Stable sort of (ids[t], t) by id (sort_*_kernel): sorted ids -> skeys, their rows -> srows; keys / rows are the
// ping-pong buffers of the odd passes (all [T]); hist: hq_sort_ids_bytes(T, V) bytes.  Passes alternate so that
// the last one lands in (skeys, srows).
void hq_sort_ids(const int64_t* ids, int T, int V, int32_t* keys, int32_t* rows, int32_t* skeys, int32_t* srows,
                 void* hist_buf, size_t hist_bytes, hipStream_t s) {
  const int np = emb_sort_passes(V), nt = emb_sort_tiles(T);
  if (T <= 0) return;
  if (hist_bytes < hq_sort_ids_bytes(T, V)) {
    fprintf(stderr, "hq_sort_ids: histogram scratch too small (%zu < %zu)\n", hist_bytes, hq_sort_ids_bytes(T, V));
    abort();
  }
  int* hist = reinterpret_cast<int*>(hist_buf);
  hipLaunchKernelGGL(sort_hist_kernel, dim3(nt), dim3(256), 0, s, ids, T, hist, nt);
  const int32_t *kin = nullptr, *vin = nullptr;
  for (int p = 0; p < np; ++p) {
    int* h = hist + (size_t)p * 256 * nt;
    int* hn = p + 1 < np ? h + 256 * nt : nullptr;
    const bool to_final = (np - 1 - p) % 2 == 0;
    int32_t* kout = to_final ? skeys : keys;
    int32_t* vout = to_final ? srows : rows;
    hipLaunchKernelGGL(sort_scan_kernel, dim3(1), dim3(1024), 0, s, h, 256 * nt, hn);
    hipLaunchKernelGGL(sort_scatter_kernel, dim3(nt), dim3(256), 0, s, ids, kin, vin, kout, vout, h, hn, T, 8 * p, nt);
    kin = kout;
    vin = vout;
  }
}

HqEmbScratchSizes hq_embed_bwd_scratch(int T, int V, int L, int P) {
  HqEmbScratchSizes z{};
  z.sort_bytes = hq_sort_ids_bytes(T, V);   // one [256][tiles] digit histogram per radix pass
  z.chunks = (T + kEmbCH - 1) / kEmbCH;
  if (L <= 0 || T % L) L = T;
  // partial rows exist for the positions l < min(L, P) only: a row whose pid == l needs l < P
  z.pos_rows = L <= kEmbMaxL ? ((T / L + kEmbNB - 1) / kEmbNB) * std::min(L, P) : 0;
  return z;
}

void hq_embed_bwd(const uint16_t* dy, const int64_t* ids, const int64_t* pids, const int64_t* tids, const uint16_t* ww,
                  const uint16_t* wp, const uint16_t* wt, const float* gamma, const float* mean, const float* rstd,
                  float* g_word, float* g_pos, float* g_type, float* part, HqOuts outs, int T, int H,
                  int n_types, int pad_word, int pad_pos, float p, uint32_t seed, uint32_t opid, bool accumulate,
                  int V, int P, int L, const HqEmbScratch& sc, hipStream_t s) {
  const uint32_t thr = p > 0.f ? hq_threshold(p) : 0u;
  const HqDropKey key = hq_drop_key(seed, opid);
  const float ks = hq_keep_scale(thr);
  if (L <= 0 || T % L) L = T;  // rows are b·L + l; any other layout is one "sequence" of T positions
  const int B = T / L;
  const dim3 grid((L + kWaves - 1) / kWaves, (B + kEmbNB - 1) / kEmbNB);
  const int nb = hq_embed_bwd_partials(T, L);
  const HqEmbScratchSizes z = hq_embed_bwd_scratch(T, V, L, P);
  const int PL = std::min(L, P);   // position-partial rows per batch slice
  float* ppart = z.pos_rows > 0 ? sc.ppart : nullptr;
  // (id, row) sort: the own stable radix sort, so every id's rows stay in token order
  hq_sort_ids(ids, T, V, sc.keys, sc.rows, sc.skeys, sc.srows, sc.sort_tmp, sc.sort_bytes, s);
  const int nwb = (z.chunks + kWaves - 1) / kWaves;
  dispatch_nch(H, [&](auto nch) {
    constexpr int C = decltype(nch)::value;
    hipLaunchKernelGGL(embed_bwd_kernel<C>, grid, dim3(256), 4 * H * sizeof(float), s, dy, ids, pids, tids, ww, wp, wt,
                       gamma, mean, rstd, g_pos, g_type, ppart, part, T, H, n_types, pad_pos, key, thr, ks, V, P, B, L,
                       PL);
    hipLaunchKernelGGL(embed_word_kernel<C>, dim3(nwb), dim3(256), 0, s, sc.skeys, sc.srows, dy, ids, pids, tids, ww,
                       wp, wt, gamma, mean, rstd, g_word, sc.carry, T, H, pad_word, accumulate ? 1 : 0, key, thr, ks, V);
    hipLaunchKernelGGL(embed_carry_kernel<C>, dim3(nwb), dim3(256), 0, s, sc.skeys, sc.carry, g_word, T, H, pad_word,
                       accumulate ? 1 : 0, V);
  });
  // outs: gamma, beta, type0, type1 (type rows only when n_types <= 2)
  colsum(part, nb, 4 * H, outs, H, accumulate, s);
  // position partials [B / kEmbNB][min(L, P)][H] -> rows 0 … min(L, P)-1 of g_pos, on top of its zeroed (or
  // accumulated) rows and the atomic flushes of non-default position ids
  if (ppart) colsum(ppart, (B + kEmbNB - 1) / kEmbNB, PL * H, HqOuts{{g_pos, nullptr, nullptr, nullptr}}, PL * H, true, s);
}

// LayerNorm-from-y guard (models/bert.py _ln_flags): LayerNorm i may recompute x̂ from its bf16 output iff every
// column has γ != 0 and |β| <= ratio·|γ|.  One block per LayerNorm over the fp32 master arena (γ at goff[i], β at
// boff[i]); flags[i] = 1 / 0.  Replaces a stack / abs / compare / and / all chain of ATen kernels.
__global__ __launch_bounds__(256) void ln_guard_kernel(const float* __restrict__ master, const int64_t* __restrict__ goff,
                                                       const int64_t* __restrict__ boff, int H, float ratio,
                                                       uint8_t* __restrict__ flags) {
  const float* g = master + goff[blockIdx.x];
  const float* b = master + boff[blockIdx.x];
  int bad = 0;
  for (int c = threadIdx.x; c < H; c += 256) {
    const float ag = fabsf(g[c]), ab = fabsf(b[c]);
    bad |= !(ag > 0.f && ab <= ratio * ag);
  }
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) flags[blockIdx.x] = bad ? 0 : 1;
}

// Additive attention key bias from the collated bool mask (HF: (1 - mask)·-10000): 0 for a real key, -10000 for
// padding.  Replaces a cast / rsub / mul chain of ATen kernels at the start of every forward.
__global__ __launch_bounds__(256) void key_bias_kernel(const uint8_t* __restrict__ mask, float* __restrict__ kb, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) kb[i] = mask[i] ? 0.f : -10000.f;
}

void hq_key_bias(const uint8_t* mask, float* kb, int n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(key_bias_kernel, dim3((n + 255) / 256), dim3(256), 0, s, mask, kb, n);
}

void hq_ln_guard(const float* master, const int64_t* goff, const int64_t* boff, int n, int H, float ratio, uint8_t* flags,
                 hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(ln_guard_kernel, dim3(n), dim3(256), 0, s, master, goff, boff, H, ratio, flags);
}

void hq_gelu_fwd(const uint16_t* pre, uint16_t* out, size_t n, hipStream_t s) {
  const size_t n8 = n / 8;
  const int grid = (int)std::min<size_t>((n8 + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(grid), dim3(256), 0, s, pre, out, n8);
}

int hq_rowblock_partials(int T) { return (T + kRowsBlock - 1) / kRowsBlock; }

void hq_gelu_bwd(const uint16_t* dout, const uint16_t* pre, uint16_t* dpre, float* part, HqOuts outs, int T, int N,
                 bool accumulate, hipStream_t s) {
  const int nb = hq_rowblock_partials(T);
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3((N + 2047) / 2048, nb), dim3(256), 0, s, dout, pre, dpre, part, T, N);
  if (outs.p[0]) colsum(part, nb, N, outs, N, accumulate, s);
}

void hq_bias_grad(const uint16_t* dy, float* part, HqOuts outs, int T, int N, bool accumulate, hipStream_t s) {
  const int nb = hq_rowblock_partials(T);
  hipLaunchKernelGGL(colpart_kernel, dim3((N + 2047) / 2048, nb), dim3(256), 0, s, dy, part, T, N);
  colsum(part, nb, N, outs, N, accumulate, s);
}

void hq_colsum(const float* part, int P, int N, float* out, bool accumulate, hipStream_t s) {
  colsum(part, P, N, HqOuts{{out, nullptr, nullptr, nullptr}}, N, accumulate, s);
}

void hq_colsum_outs(const float* part, int P, int N, HqOuts outs, int Hq, bool accumulate, hipStream_t s) {
  colsum(part, P, N, outs, Hq, accumulate, s);
}

void hq_span_fwd(const uint16_t* seq, const float* w, const float* b, float* logits, int T, int H, hipStream_t s) {
  dispatch_nch(H, [&](auto nch) {
    hipLaunchKernelGGL(span_fwd_kernel<decltype(nch)::value>, dim3((T + kWaves - 1) / kWaves), dim3(256), 0, s, seq, w, b,
                       logits, T, H);
  });
}

void hq_span_bwd(const uint16_t* seq, const float* w, const float* g, uint16_t* dseq, float* part, float* dw, int T,
                 int H, bool accumulate, hipStream_t s) {
  const int nb = hq_ln_bwd_partials(T);
  dispatch_nch(H, [&](auto nch) {
    hipLaunchKernelGGL(span_bwd_kernel<decltype(nch)::value>, dim3(nb), dim3(256), 4 * H * sizeof(float), s, seq, w, g,
                       dseq, part, T, H, ln_rows_per_wave(T));
  });
  colsum(part, nb, 2 * H, HqOuts{{dw, dw + H, nullptr, nullptr}}, H, accumulate, s);
}
