// Fused QA heads + losses (gfx950, wave64): the pooler, the four reference heads and the five QA
// losses of one micro-batch in THREE launches (forward, loss, backward) plus the column-sum of the
// span weight-gradient partials, replacing ~70 small ATen launches (pooler slice/cast/addmm/tanh,
// dropout, 3 Linear+Sigmoid, 2 CE + 2 MSE + the class loss, weighted sum, their backward and the
// per-parameter grad memsets).
//
// Reference semantics (modules/model/model/model.py:27-41,54-73; loss.py:5-106; init.py:18-40):
//   pooled  = tanh(seq[:,0] · Wpᵀ + bp)                      (HF BertPooler)
//   start/end logits = seq · Wspᵀ + bsp                       (position_outputs, Linear(H,2))
//   cls     = dropout(pooled) · Wcᵀ + bc                      (classifier = Dropout + Linear(H,NL))
//   reg_s/e = sigmoid(pooled · w_{s,e} + b_{s,e})              (reg_start / reg_end)
//   loss    = w0·CE(start, ignore -1) + w1·CE(end, ignore -1) + w2·MSE(reg_s) + w3·MSE(reg_e)
//             + w4·{CE(weights, ignore -100) | focal NLL (ignore -1) | label-smoothing KL (batchmean)}
// Everything is fp32 on the fp32 master weights (the encoder output is read as bf16).
//
// Work split:
//   fwd : blocks [0, npool)  pooled tiles (32 samples × 64 outputs, K staged through LDS), epilogue
//                            tanh + per-tile partial dot products of the small heads; the LAST pooled
//                            block to finish (agent-scope ticket) folds the partials → cls / reg;
//         blocks [npool, …)  kSpanFwdRPW sequence rows per wave: span logits.
//   loss: blocks [0, nrow)   one wave per sample: online log-sum-exp over L for start AND end
//                            (float2 rows), CE value + gradient (softmax − onehot)·w/n written in place;
//         block nrow         class + regression losses and gradients for all samples;
//         last arriver       folds the per-block sums in a fixed order → losses[6] (deterministic).
//   bwd : dpre = dL/d(pooler pre-activation) is recomputed wherever needed (NL+2 FMAs + one hash)
//         instead of being materialised; roles by block id:
//         R1  dx tiles   dseq[b, 0, :] = dpre[b] · Wp + span part        (32 samples × 64 columns)
//         R2  dWp tiles  dWp[k, i] = Σ_b dpre[b, k] · x[b, i]            (64 × 64, deterministic)
//         R3  small grads dbp, dWc, dw_reg (+ the head biases in block 0)
//         R4  span rows  dseq = g·Wsp (rows other than CLS) + dW/db partials → hq_colsum
// The loss gradient is computed for d(total) = 1; the backward multiplies by the autograd incoming
// scalar `gscale` (device pointer, e.g. 1/batch_split), so no host sync and no extra scale launch.
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

constexpr int kHS = 16;      // row stride of dheads / head partials: [0, NL) class logits, 8 / 9 = reg start / end
constexpr int kMaxNL = 8;
constexpr int kSpanRPW = 16; // span rows per wave in the backward (64 rows per block)
constexpr int kSpanFwdRPW = 8;  // span rows per wave in the forward: all loads issued before the dot products
                                // (one row per wave was latency-bound at the pooled path's LDS occupancy:
                                // 102 µs for 151 MB at T = 98304)

__device__ __forceinline__ float keep_mult(uint32_t idx, uint32_t key, uint32_t thr, float ks) {
  return thr ? (hq_keep(idx, key, thr) ? ks : 0.f) : 1.f;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// Agent-scope ticket (the in-launch split-K hand-off recipe): every block publishes its plain stores
// with one release, the last arriver acquires and resets the counter.  Returns true in ALL threads of
// the last-arriving block.  `flag` is a word inside the block's single LDS array.
__device__ bool last_arriver(unsigned* cnt, unsigned nblocks, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == nblocks - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// The sequence (encoder output) and its gradient are bf16 (the bf16 / fp8 step) or fp32 (--precision fp32): TS is
// the element type; every load widens to fp32 and the head math is fp32 either way.
template <typename TS> struct SeqRaw4 { using type = uint2; };    // 4 elements as loaded
template <> struct SeqRaw4<float> { using type = float4; };
template <typename TS>
__device__ __forceinline__ typename SeqRaw4<TS>::type ld_raw4(const void* base, size_t off) {
  return *reinterpret_cast<const typename SeqRaw4<TS>::type*>(static_cast<const TS*>(base) + off);
}
__device__ __forceinline__ void raw_to_f4(const uint2& r, float* x) { hq_unpack4(r, x); }
__device__ __forceinline__ void raw_to_f4(const float4& r, float* x) { x[0] = r.x; x[1] = r.y; x[2] = r.z; x[3] = r.w; }
template <typename TS>
__device__ __forceinline__ void ld8f(const void* base, size_t off, float* f) {
  if constexpr (std::is_same<TS, float>::value) {
    const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(base) + off);
    const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(base) + off + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else {
    hq_unpack8(*reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(base) + off), f);
  }
}
template <typename TS>
__device__ __forceinline__ float ld1f(const void* base, size_t off) {
  if constexpr (std::is_same<TS, float>::value) return static_cast<const float*>(base)[off];
  else return hq_bf2f(static_cast<const uint16_t*>(base)[off]);
}
template <typename TS>
__device__ __forceinline__ void st1f(void* base, size_t off, float v) {
  if constexpr (std::is_same<TS, float>::value) static_cast<float*>(base)[off] = v;
  else static_cast<uint16_t*>(base)[off] = hq_f2bf(v);
}
template <typename TS>
__device__ __forceinline__ void st4f(void* base, size_t off, const float* d) {
  if constexpr (std::is_same<TS, float>::value)
    *reinterpret_cast<float4*>(static_cast<float*>(base) + off) = make_float4(d[0], d[1], d[2], d[3]);
  else
    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(base) + off) = hq_pack4(d);
}

// =============================================================================================== fwd
struct FwdArgs {
  const void* seq;
  const float *wp, *bp, *wc, *bc, *wrs, *brs, *wre, *bre, *wsp, *bsp;
  float *logits, *pooled, *cls, *reg, *hpart;  // hpart [H/64][B][kHS] scratch
  unsigned* cnt;
  int B, L, H, NL, T, npool;
  HqDropKey kd;
  uint32_t thr;
  float ks;
};

template <int NCH, typename TS>
__global__ __launch_bounds__(256) void qa_heads_fwd_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t key = a.kd.get();
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int H = a.H;
  if ((int)blockIdx.x >= a.npool) {  // ---------------------------------------------- span rows
    const int row0 = (((int)blockIdx.x - a.npool) * 4 + wv) * kSpanFwdRPW;
    if (row0 >= a.T) return;
    typename SeqRaw4<TS>::type raw[kSpanFwdRPW][NCH];
#pragma unroll
    for (int r = 0; r < kSpanFwdRPW; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = c * 256 + lane * 4;
        raw[r][c] = row0 + r < a.T && col < H ? ld_raw4<TS>(a.seq, (size_t)(row0 + r) * H + col)
                                              : typename SeqRaw4<TS>::type{};
      }
    float4 u[NCH], v[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      u[c] = col < H ? *reinterpret_cast<const float4*>(a.wsp + col) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[c] = col < H ? *reinterpret_cast<const float4*>(a.wsp + H + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int r = 0; r < kSpanFwdRPW; ++r) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        float x[4];
        raw_to_f4(raw[r][c], x);
        s0 += x[0] * u[c].x + x[1] * u[c].y + x[2] * u[c].z + x[3] * u[c].w;
        s1 += x[0] * v[c].x + x[1] * v[c].y + x[2] * v[c].z + x[3] * v[c].w;
      }
      s0 = hq_wave_sum(s0);
      s1 = hq_wave_sum(s1);
      if (lane == 0 && row0 + r < a.T)
        *reinterpret_cast<float2*>(a.logits + 2 * (size_t)(row0 + r)) = make_float2(s0 + a.bsp[0], s1 + a.bsp[1]);
    }
    return;
  }
  // ---------------------------------------------------------------------------- pooled tile
  float* xs = lds;             // [32][64]  CLS rows, k chunk
  float* ws = lds + 32 * 64;   // [64][65]  Wp rows j, k chunk (padded: conflict-free column reads)
  const int nj = H / 64;
  const int sb = blockIdx.x / nj, jb = blockIdx.x % nj;
  float acc[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) acc[s] = 0.f;
  // the next K chunk's global loads are issued before this chunk's FMAs (register double buffer); with the parallel
  // partial fold below the kernel went 103.4 -> 86.6 µs at B = 256, L = 384 (profiles/r6_s3_heads)
  const int xs_s = tid >> 3, xs_k = (tid & 7) * 8, xs_b = sb * 32 + xs_s;
  float f[8];
  float4 wq[4];
  auto load_chunk = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = 0.f;
    if (xs_b < a.B) ld8f<TS>(a.seq, (size_t)xs_b * a.L * H + k0 + xs_k, f);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * 256, r = idx >> 4, c4 = (idx & 15) * 4;
      wq[q] = *reinterpret_cast<const float4*>(a.wp + (size_t)(jb * 64 + r) * H + k0 + c4);
    }
  };
  load_chunk(0);
  for (int k0 = 0; k0 < H; k0 += 64) {
    *reinterpret_cast<float4*>(xs + xs_s * 64 + xs_k) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(xs + xs_s * 64 + xs_k + 4) = make_float4(f[4], f[5], f[6], f[7]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * 256, r = idx >> 4, c4 = (idx & 15) * 4;
      float* d = ws + r * 65 + c4;
      d[0] = wq[q].x; d[1] = wq[q].y; d[2] = wq[q].z; d[3] = wq[q].w;
    }
    __syncthreads();
    if (k0 + 64 < H) load_chunk(k0 + 64);
#pragma unroll 4
    for (int kk = 0; kk < 64; kk += 4) {
      const float w0 = ws[lane * 65 + kk], w1 = ws[lane * 65 + kk + 1], w2 = ws[lane * 65 + kk + 2],
                  w3 = ws[lane * 65 + kk + 3];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const float4 x = *reinterpret_cast<const float4*>(xs + (wv * 8 + s) * 64 + kk);
        acc[s] = fmaf(x.x, w0, fmaf(x.y, w1, fmaf(x.z, w2, fmaf(x.w, w3, acc[s]))));
      }
    }
    __syncthreads();
  }
  const int j = jb * 64 + lane;
  const float bj = a.bp[j];
  float wcj[kMaxNL];
#pragma unroll
  for (int c = 0; c < kMaxNL; ++c) wcj[c] = c < a.NL ? a.wc[(size_t)c * H + j] : 0.f;
  const float wsj = a.wrs[j], wej = a.wre[j];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int b = sb * 32 + wv * 8 + s;
    if (b >= a.B) break;  // wave-uniform
    const float pv = tanhf(acc[s] + bj);
    a.pooled[(size_t)b * H + j] = pv;
    const float pm = pv * keep_mult((uint32_t)((size_t)b * H + j), key, a.thr, a.ks);
    float* hp = a.hpart + ((size_t)jb * a.B + b) * kHS;
#pragma unroll
    for (int c = 0; c < kMaxNL; ++c) {
      if (c < a.NL) {
        const float v = hq_wave_sum(pm * wcj[c]);
        if (lane == 0) hp[c] = v;
      }
    }
    const float vs = hq_wave_sum(pv * wsj), ve = hq_wave_sum(pv * wej);
    if (lane == 0) { hp[8] = vs; hp[9] = ve; }
  }
  if (!last_arriver(a.cnt, (unsigned)a.npool, reinterpret_cast<int*>(lds))) return;
  const int nout = a.NL + 2;
  for (int idx = tid; idx < a.B * nout; idx += 256) {
    const int b = idx / nout, c = idx % nout;
    const int col = c < a.NL ? c : 8 + (c - a.NL);
    // every partial's load in flight at once (nj <= 4·NCH), then the sum in the same q order (bitwise the old result):
    // the loop of dependent load → add steps was 12 L2 round trips per output, 7 outputs per thread, in ONE block
    float v[4 * NCH];
#pragma unroll
    for (int q = 0; q < 4 * NCH; ++q) v[q] = q < nj ? a.hpart[((size_t)q * a.B + b) * kHS + col] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 4 * NCH; ++q)
      if (q < nj) s += v[q];
    if (c < a.NL) a.cls[(size_t)b * a.NL + c] = s + a.bc[c];
    else if (c == a.NL) a.reg[2 * b] = sigmoidf_(s + a.brs[0]);
    else a.reg[2 * b + 1] = sigmoidf_(s + a.bre[0]);
  }
}

// ============================================================================================== loss
struct LossArgs {
  const float *logits, *cls, *reg;
  const int64_t *t_start, *t_end, *t_cls;
  const float *t_rs, *t_re, *lw;
  float *dlog, *dheads, *losses, *part;  // part [nrow + 1][4]
  unsigned* cnt;
  const int* seg_len;   // [nseg] span length of each segment (its micro-batch's own padded length) or null
  int B, L, NL, kind, ignore_cls, nrow, nseg;
  float w0, w1, w2, w3, w4, alpha, gamma, conf, fill;
};

enum { kLossCE = 0, kLossFocal = 1, kLossSmooth = 2 };

// Segments (exact-objective micro-batch merge): the batch is nseg equal, contiguous segments, each one of the
// reference's micro-batches.  Every loss term is normalised inside its segment (span CE over the segment's
// valid spans and over its own span length, class CE / focal over its valid targets, KL batchmean and MSE over
// its samples) and the terms are averaged over the segments — the reference's mean of per-micro-batch means
// (trainer.py:197-204).  nseg = 1 is the plain batch.
__device__ __forceinline__ int seg_span_len(const LossArgs& a, int s) {
  return a.seg_len ? min(max(a.seg_len[s], 1), a.L) : a.L;
}

__device__ __forceinline__ int span_valid_count(const int64_t* t, int lo, int n, int L, int lane) {
  float c = 0.f;
  for (int i = lane; i < n; i += 64) {
    const int64_t v = t[lo + i];
    c += (v >= 0 && v < L) ? 1.f : 0.f;
  }
  return (int)hq_wave_sum(c);
}

__device__ __forceinline__ bool cls_valid(const LossArgs& a, int64_t t) {
  if (t < 0 || t >= a.NL) return false;
  if (a.kind == kLossCE) return t != a.ignore_cls;
  if (a.kind == kLossFocal) return t != -1;
  return true;
}

__global__ __launch_bounds__(256) void qa_loss_kernel(LossArgs a) {
  __shared__ float red[4 * 256 + 8];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int B = a.B, L = a.L;
  const int bs = B / a.nseg;                         // samples per segment
  const float inv_seg = 1.f / (float)a.nseg;
  if ((int)blockIdx.x < a.nrow) {  // -------------------------------------- span CE, one wave per sample
    const int b = blockIdx.x * 4 + wv;
    float nll_s = 0.f, nll_e = 0.f;
    if (b < B) {
      const int sg = b / bs, lo = sg * bs, Ls = seg_span_len(a, sg);
      const int ns = span_valid_count(a.t_start, lo, bs, Ls, lane), ne = span_valid_count(a.t_end, lo, bs, Ls, lane);
      const float2* row = reinterpret_cast<const float2*>(a.logits) + (size_t)b * L;
      float ms = -INFINITY, me = -INFINITY, ss = 0.f, se = 0.f;
      for (int j = lane; j < Ls; j += 64) {
        const float2 z = row[j];
        if (z.x > ms) { ss = ss * expf(ms - z.x) + 1.f; ms = z.x; } else { ss += expf(z.x - ms); }
        if (z.y > me) { se = se * expf(me - z.y) + 1.f; me = z.y; } else { se += expf(z.y - me); }
      }
      const float Ms = hq_wave_max(ms), Me = hq_wave_max(me);
      const float Ss = hq_wave_sum(ms == -INFINITY ? 0.f : ss * expf(ms - Ms));
      const float Se = hq_wave_sum(me == -INFINITY ? 0.f : se * expf(me - Me));
      const float lse_s = Ms + logf(Ss), lse_e = Me + logf(Se);
      const int64_t ts = a.t_start[b], te = a.t_end[b];
      const bool vs = ts >= 0 && ts < Ls, ve = te >= 0 && te < Ls;
      // per-sample terms already normalised by the segment's valid count and the segment count; a segment
      // with no valid span is 0/0 = NaN in torch's CE (ignore_index) — its first sample carries that NaN
      const float cs = inv_seg / (float)ns, ce = inv_seg / (float)ne;
      if (vs) nll_s = (lse_s - row[ts].x) * cs;
      if (ve) nll_e = (lse_e - row[te].y) * ce;
      if (b == lo && ns == 0) nll_s = NAN;
      if (b == lo && ne == 0) nll_e = NAN;
      const float gs = vs ? a.w0 * cs : 0.f, ge = ve ? a.w1 * ce : 0.f;
      float2* drow = reinterpret_cast<float2*>(a.dlog) + (size_t)b * L;
      for (int j = lane; j < L; j += 64) {
        float2 d = make_float2(0.f, 0.f);   // positions past the segment's own length are not in its softmax
        if (j < Ls) {
          const float2 z = row[j];
          d.x = gs * (expf(z.x - lse_s) - (j == ts ? 1.f : 0.f));
          d.y = ge * (expf(z.y - lse_e) - (j == te ? 1.f : 0.f));
        }
        drow[j] = d;
      }
    }
    if (lane == 0) { red[2 * wv] = nll_s; red[2 * wv + 1] = nll_e; }
    __syncthreads();
    if (tid == 0) {
      float* p = a.part + (size_t)blockIdx.x * 4;
      p[0] = ((red[0] + red[2]) + red[4]) + red[6];
      p[1] = ((red[1] + red[3]) + red[5]) + red[7];
    }
  } else {  // ------------------------------------------------------- class + regression block
    // pass 1: class-loss normaliser (CE: Σ weights of valid targets; focal: #valid; smooth: B) of the whole
    // batch; with segments each sample recomputes its own segment's (bs targets) in pass 2
    float den = 0.f;
    for (int b = tid; b < B; b += 256) {
      const int64_t t = a.t_cls[b];
      if (a.kind != kLossSmooth && cls_valid(a, t)) den += (a.kind == kLossCE && a.lw) ? a.lw[t] : 1.f;
    }
    den = hq_wave_sum(den);
    if (lane == 0) red[wv] = den;
    __syncthreads();
    den = a.kind == kLossSmooth ? (float)B : ((red[0] + red[1]) + red[2]) + red[3];
    __syncthreads();
    // pass 2: per-sample losses and gradients w.r.t. the predictions
    float lc = 0.f, lrs = 0.f, lre = 0.f;
    const float invB = 1.f / (float)B;
    for (int b = tid; b < B; b += 256) {
      float den_s = den;   // this sample's segment normaliser (× nseg below)
      if (a.nseg > 1 && a.kind != kLossSmooth) {
        den_s = 0.f;
        for (int i = (b / bs) * bs, e = i + bs; i < e; ++i) {
          const int64_t ti = a.t_cls[i];
          if (cls_valid(a, ti)) den_s += (a.kind == kLossCE && a.lw) ? a.lw[ti] : 1.f;
        }
      }
      const float inv_den = a.kind == kLossSmooth ? invB : inv_seg / den_s;
      if (a.kind != kLossSmooth && b % bs == 0 && den_s == 0.f) lc = NAN;   // torch: mean over no targets
      float z[kMaxNL], dz[kMaxNL];
      float m = -INFINITY;
#pragma unroll
      for (int c = 0; c < kMaxNL; ++c) {
        z[c] = c < a.NL ? a.cls[(size_t)b * a.NL + c] : -INFINITY;
        m = fmaxf(m, z[c]);
      }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < kMaxNL; ++c) se += c < a.NL ? expf(z[c] - m) : 0.f;
      const float lse = m + logf(se);
      const int64_t t = a.t_cls[b];
#pragma unroll
      for (int c = 0; c < kMaxNL; ++c) dz[c] = 0.f;
      if (a.kind == kLossSmooth) {
        if (t >= 0 && t < a.NL) {
          float S = 0.f;
#pragma unroll
          for (int c = 0; c < kMaxNL; ++c) {
            if (c < a.NL) {
              const float dist = c == t ? a.conf : a.fill;
              S += dist;
              if (dist > 0.f) lc += dist * (logf(dist) - (z[c] - lse)) * invB;
            }
          }
#pragma unroll
          for (int c = 0; c < kMaxNL; ++c)
            if (c < a.NL) dz[c] = a.w4 * (S * expf(z[c] - lse) - (c == t ? a.conf : a.fill)) * invB;
        }
      } else if (cls_valid(a, t)) {
        float zt = 0.f;  // z[t] without a dynamically indexed register array
#pragma unroll
        for (int c = 0; c < kMaxNL; ++c) zt = c == t ? z[c] : zt;
        const float lp = zt - lse;
        if (a.kind == kLossCE) {
          const float wt = a.lw ? a.lw[t] : 1.f;
          lc += wt * -lp * inv_den;
          const float g = a.w4 * wt * inv_den;
#pragma unroll
          for (int c = 0; c < kMaxNL; ++c)
            if (c < a.NL) dz[c] = g * (expf(z[c] - lse) - (c == t ? 1.f : 0.f));
        } else {  // focal: loss_b = -α(1-p)^γ·log p
          const float pt = expf(lp), omp = 1.f - pt;
          const float powg = powf(omp, a.gamma);
          lc += -a.alpha * powg * lp * inv_den;
          const float d2 = omp > 0.f ? a.gamma * powf(omp, a.gamma - 1.f) * pt * lp : 0.f;
          const float gl = -a.alpha * (powg - d2) * inv_den * a.w4;  // d loss / d log p_t
#pragma unroll
          for (int c = 0; c < kMaxNL; ++c)
            if (c < a.NL) dz[c] = gl * ((c == t ? 1.f : 0.f) - expf(z[c] - lse));
        }
      }
      float* dh = a.dheads + (size_t)b * kHS;
#pragma unroll
      for (int c = 0; c < kMaxNL; ++c)
        if (c < a.NL) dh[c] = dz[c];
      const float d0 = a.reg[2 * b] - a.t_rs[b], d1 = a.reg[2 * b + 1] - a.t_re[b];
      lrs += d0 * d0;
      lre += d1 * d1;
      dh[8] = a.w2 * 2.f * d0 * invB;
      dh[9] = a.w3 * 2.f * d1 * invB;
    }
    lc = hq_wave_sum(lc); lrs = hq_wave_sum(lrs); lre = hq_wave_sum(lre);
    if (lane == 0) { red[4 * wv] = lc; red[4 * wv + 1] = lrs; red[4 * wv + 2] = lre; }
    __syncthreads();
    if (tid == 0) {
      float* p = a.part + (size_t)blockIdx.x * 4;
#pragma unroll
      for (int q = 0; q < 3; ++q) p[q] = ((red[q] + red[4 + q]) + red[8 + q]) + red[12 + q];
      p[3] = den;
    }
  }
  if (!last_arriver(a.cnt, (unsigned)(a.nrow + 1), reinterpret_cast<int*>(red + 4 * 256))) return;
  if (wv != 0) return;
  float ss = 0.f, se = 0.f;   // the per-sample terms arrive normalised (segment count, valid count)
  for (int r = lane; r < a.nrow; r += 64) { ss += a.part[(size_t)r * 4]; se += a.part[(size_t)r * 4 + 1]; }
  ss = hq_wave_sum(ss);
  se = hq_wave_sum(se);
  if (lane == 0) {
    const float* pc = a.part + (size_t)a.nrow * 4;
    const float l0 = ss, l1 = se;   // NaN when a segment has every span target ignored (torch's 0/0)
    const float l2 = pc[1] / (float)B, l3 = pc[2] / (float)B;
    const float l4 = pc[0];
    a.losses[0] = l0; a.losses[1] = l1; a.losses[2] = l2; a.losses[3] = l3; a.losses[4] = l4;
    a.losses[5] = a.w0 * l0 + a.w1 * l1 + a.w2 * l2 + a.w3 * l3 + a.w4 * l4;
  }
}

// =============================================================================================== bwd
struct BwdArgs {
  const void* seq;
  const float *dlog, *dheads, *gscale, *pooled, *reg;
  const float *wp, *wc, *wrs, *wre, *wsp;
  void* dseq;
  float* span_part;  // [nspan][2H + 2]
  float *gwp, *gbp, *gwc, *gbc, *gwrs, *gbrs, *gwre, *gbre;
  int B, L, H, NL, T, acc;
  int nA, nW, nS;
  HqDropKey kd;
  uint32_t thr;
  float ks;
  float* dpre;   // [B][H] dL/d(pooler pre-activation), written by qa_dpre_kernel before the backward (or null: recomputed)
};

// per-sample backward scalars: [0, NL) gs·dcls, 8 / 9 = gs·dreg·σ'(pre) for start / end
__device__ __forceinline__ float sample_scalar(const BwdArgs& a, int b, int c, float gs) {
  if (c < a.NL) return gs * a.dheads[(size_t)b * kHS + c];
  if (c == 8 || c == 9) {
    const float r = a.reg[2 * b + (c - 8)];
    return gs * a.dheads[(size_t)b * kHS + c] * r * (1.f - r);
  }
  return 0.f;
}

// dL/d(pooler pre-activation)[b, k] from the per-sample scalars sc[kHS]
__device__ __forceinline__ float dpre_at(const BwdArgs& a, uint32_t key, int b, int k, const float* sc) {
  float d = 0.f;
  for (int c = 0; c < a.NL; ++c) d = fmaf(sc[c], a.wc[(size_t)c * a.H + k], d);
  d *= keep_mult((uint32_t)((size_t)b * a.H + k), key, a.thr, a.ks);
  d = fmaf(sc[8], a.wrs[k], fmaf(sc[9], a.wre[k], d));
  const float pv = a.pooled[(size_t)b * a.H + k];
  return d * (1.f - pv * pv);
}

__device__ __forceinline__ void put(float* p, float v, int acc) { *p = acc ? *p + v : v; }

// dpre [B][H] once per backward: the dx tiles (R1, 12 column blocks per sample block) and the dWp tiles (R2, 12 row
// blocks per k block) each recomputed it for every element they read — the same dpre_at call, so the same bits
__global__ __launch_bounds__(256) void qa_dpre_kernel(BwdArgs a) {
  const uint32_t key = a.kd.get();
  const float gs = a.gscale ? *a.gscale : 1.f;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)a.B * a.H) return;
  const int b = (int)(i / a.H), k = (int)(i % a.H);
  float sc[kHS];
#pragma unroll
  for (int c = 0; c < kHS; ++c) sc[c] = sample_scalar(a, b, c, gs);
  a.dpre[i] = dpre_at(a, key, b, k, sc);
}

template <int NCH, typename TS>
__global__ __launch_bounds__(256) void qa_heads_bwd_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t key = a.kd.get();
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int H = a.H, B = a.B, nj = H / 64;
  const float gs = a.gscale ? *a.gscale : 1.f;
  int blk = blockIdx.x;
  if (blk < a.nA) {  // ------------------------------------------------ R1: dx of the CLS rows
    float* scs = lds;            // [32][kHS]
    float* dp = lds + 32 * kHS;  // [32][64]
    float* wt = dp + 32 * 64;    // [64][64]  Wp rows k, columns i
    const int sb = blk / nj, ib = blk % nj;
    for (int idx = tid; idx < 32 * kHS; idx += 256) {
      const int s = idx / kHS, c = idx % kHS, b = sb * 32 + s;
      scs[idx] = b < B ? sample_scalar(a, b, c, gs) : 0.f;
    }
    __syncthreads();
    float acc[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = 0.f;
    for (int k0 = 0; k0 < H; k0 += 64) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int s = wv + 4 * q, b = sb * 32 + s;
        dp[s * 64 + lane] = b >= B ? 0.f
                            : a.dpre ? a.dpre[(size_t)b * H + k0 + lane] : dpre_at(a, key, b, k0 + lane, scs + s * kHS);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = tid + q * 256, r = idx >> 4, c4 = (idx & 15) * 4;
        *reinterpret_cast<float4*>(wt + r * 64 + c4) =
            *reinterpret_cast<const float4*>(a.wp + (size_t)(k0 + r) * H + ib * 64 + c4);
      }
      __syncthreads();
#pragma unroll 4
      for (int kk = 0; kk < 64; kk += 4) {
        const float w0 = wt[kk * 64 + lane], w1 = wt[(kk + 1) * 64 + lane], w2 = wt[(kk + 2) * 64 + lane],
                    w3 = wt[(kk + 3) * 64 + lane];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const float4 d = *reinterpret_cast<const float4*>(dp + (wv * 8 + s) * 64 + kk);
          acc[s] = fmaf(d.x, w0, fmaf(d.y, w1, fmaf(d.z, w2, fmaf(d.w, w3, acc[s]))));
        }
      }
      __syncthreads();
    }
    const int i = ib * 64 + lane;
    const float u0 = a.wsp[i], u1 = a.wsp[H + i];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int b = sb * 32 + wv * 8 + s;
      if (b >= B) break;
      const size_t row = (size_t)b * a.L;
      const float2 g = *reinterpret_cast<const float2*>(a.dlog + 2 * row);
      st1f<TS>(a.dseq, row * H + i, acc[s] + gs * (g.x * u0 + g.y * u1));
    }
    return;
  }
  blk -= a.nA;
  if (blk < a.nW) {  // ------------------------------------------------- R2: dWp tiles
    if (!a.gwp) return;
    float* scs = lds;            // [32][kHS]
    float* dp = lds + 32 * kHS;  // [32][64]  dpre[b][k]
    float* xs = dp + 32 * 64;    // [32][64]  x[b][i]
    const int kb = blk / nj, ib = blk % nj;
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
    for (int b0 = 0; b0 < B; b0 += 32) {
      for (int idx = tid; idx < 32 * kHS; idx += 256) {
        const int s = idx / kHS, c = idx % kHS, b = b0 + s;
        scs[idx] = b < B ? sample_scalar(a, b, c, gs) : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int s = wv + 4 * q, b = b0 + s;
        dp[s * 64 + lane] = b >= B ? 0.f
                            : a.dpre ? a.dpre[(size_t)b * H + kb * 64 + lane]
                                     : dpre_at(a, key, b, kb * 64 + lane, scs + s * kHS);
        xs[s * 64 + lane] = b < B ? ld1f<TS>(a.seq, (size_t)b * a.L * H + ib * 64 + lane) : 0.f;
      }
      __syncthreads();
#pragma unroll 4
      for (int s = 0; s < 32; ++s) {
        const float x = xs[s * 64 + lane];
#pragma unroll
        for (int j = 0; j < 16; j += 4) {
          const float4 d = *reinterpret_cast<const float4*>(dp + s * 64 + wv * 16 + j);
          acc[j] = fmaf(d.x, x, acc[j]);
          acc[j + 1] = fmaf(d.y, x, acc[j + 1]);
          acc[j + 2] = fmaf(d.z, x, acc[j + 2]);
          acc[j + 3] = fmaf(d.w, x, acc[j + 3]);
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) put(a.gwp + (size_t)(kb * 64 + wv * 16 + j) * H + ib * 64 + lane, acc[j], a.acc);
    return;
  }
  blk -= a.nW;
  if (blk < a.nS) {  // ------------------------------------------------ R3: dbp, dWc, dw_reg (+ biases)
    constexpr int NA = kMaxNL + 3;  // dbp, dWc[NL], dw_rs, dw_re
    float* red = lds;               // [4][64][NA]
    const int k = blk * 64 + lane;
    float wck[kMaxNL];
#pragma unroll
    for (int c = 0; c < kMaxNL; ++c) wck[c] = c < a.NL ? a.wc[(size_t)c * H + k] : 0.f;
    const float wsk = a.wrs[k], wek = a.wre[k];
    float ac[NA];
#pragma unroll
    for (int q = 0; q < NA; ++q) ac[q] = 0.f;
    for (int b = wv; b < B; b += 4) {
      float sc[kMaxNL];
#pragma unroll
      for (int c = 0; c < kMaxNL; ++c) sc[c] = c < a.NL ? gs * a.dheads[(size_t)b * kHS + c] : 0.f;
      const float s8 = sample_scalar(a, b, 8, gs), s9 = sample_scalar(a, b, 9, gs);
      const float pv = a.pooled[(size_t)b * H + k];
      const float m = keep_mult((uint32_t)((size_t)b * H + k), key, a.thr, a.ks);
      float d = 0.f;
#pragma unroll
      for (int c = 0; c < kMaxNL; ++c) d = fmaf(sc[c], wck[c], d);
      ac[0] += fmaf(d, m, fmaf(s8, wsk, s9 * wek)) * (1.f - pv * pv);
      const float pm = pv * m;
#pragma unroll
      for (int c = 0; c < kMaxNL; ++c) ac[1 + c] = fmaf(sc[c], pm, ac[1 + c]);
      ac[1 + kMaxNL] = fmaf(s8, pv, ac[1 + kMaxNL]);
      ac[2 + kMaxNL] = fmaf(s9, pv, ac[2 + kMaxNL]);
    }
#pragma unroll
    for (int q = 0; q < NA; ++q) red[(wv * 64 + lane) * NA + q] = ac[q];
    __syncthreads();
    if (wv == 0) {
      float t[NA];
#pragma unroll
      for (int q = 0; q < NA; ++q)
        t[q] = ((red[lane * NA + q] + red[(64 + lane) * NA + q]) + red[(128 + lane) * NA + q]) + red[(192 + lane) * NA + q];
      if (a.gbp) put(a.gbp + k, t[0], a.acc);
      if (a.gwc)
        for (int c = 0; c < a.NL; ++c) put(a.gwc + (size_t)c * H + k, t[1 + c], a.acc);
      if (a.gwrs) put(a.gwrs + k, t[1 + kMaxNL], a.acc);
      if (a.gwre) put(a.gwre + k, t[2 + kMaxNL], a.acc);
    }
    if (blk == 0) {  // head biases: Σ_b of the per-sample scalars
      __syncthreads();
      float bs[kMaxNL + 2];
#pragma unroll
      for (int c = 0; c < kMaxNL + 2; ++c) bs[c] = 0.f;
      for (int b = tid; b < B; b += 256) {
#pragma unroll
        for (int c = 0; c < kMaxNL; ++c) bs[c] += c < a.NL ? gs * a.dheads[(size_t)b * kHS + c] : 0.f;
        bs[kMaxNL] += sample_scalar(a, b, 8, gs);
        bs[kMaxNL + 1] += sample_scalar(a, b, 9, gs);
      }
#pragma unroll
      for (int c = 0; c < kMaxNL + 2; ++c) {
        const float v = hq_wave_sum(bs[c]);
        if (lane == 0) red[wv * (kMaxNL + 2) + c] = v;
      }
      __syncthreads();
      if (tid < kMaxNL + 2) {
        const float v = ((red[tid] + red[(kMaxNL + 2) + tid]) + red[2 * (kMaxNL + 2) + tid]) + red[3 * (kMaxNL + 2) + tid];
        if (tid < a.NL) { if (a.gbc) put(a.gbc + tid, v, a.acc); }
        else if (tid == kMaxNL) { if (a.gbrs) put(a.gbrs, v, a.acc); }
        else if (tid == kMaxNL + 1) { if (a.gbre) put(a.gbre, v, a.acc); }
      }
    }
    return;
  }
  blk -= a.nS;  // -------------------------------------------------------- R4: span rows
  float w0[NCH][4], w1[NCH][4], acc[2][NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 256 + lane * 4;
    const float4 u = col < H ? *reinterpret_cast<const float4*>(a.wsp + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 v = col < H ? *reinterpret_cast<const float4*>(a.wsp + H + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    w0[c][0] = u.x; w0[c][1] = u.y; w0[c][2] = u.z; w0[c][3] = u.w;
    w1[c][0] = v.x; w1[c][1] = v.y; w1[c][2] = v.z; w1[c][3] = v.w;
#pragma unroll
    for (int i = 0; i < 4; ++i) { acc[0][c][i] = 0.f; acc[1][c][i] = 0.f; }
  }
  float gsum0 = 0.f, gsum1 = 0.f;
  const int row0 = blk * 4 * kSpanRPW;
#pragma unroll 2
  for (int r = 0; r < kSpanRPW; ++r) {
    const int row = row0 + r * 4 + wv;
    if (row >= a.T) break;
    float2 g = *reinterpret_cast<const float2*>(a.dlog + 2 * (size_t)row);
    g.x *= gs;
    g.y *= gs;
    gsum0 += g.x;
    gsum1 += g.y;
    const bool cls_row = row % a.L == 0;  // written (with the pooler part) by R1
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      if (col < H) {
        float x[4], d[4];
        raw_to_f4(ld_raw4<TS>(a.seq, (size_t)row * H + col), x);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[0][c][i] = fmaf(g.x, x[i], acc[0][c][i]);
          acc[1][c][i] = fmaf(g.y, x[i], acc[1][c][i]);
          d[i] = g.x * w0[c][i] + g.y * w1[c][i];
        }
        if (!cls_row) st4f<TS>(a.dseq, (size_t)row * H + col, d);
      }
    }
  }
  const int N = 2 * H + 2;
  float* st = lds;  // [4][N]
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      if (col < H)
        *reinterpret_cast<float4*>(st + wv * N + q * H + col) =
            make_float4(acc[q][c][0], acc[q][c][1], acc[q][c][2], acc[q][c][3]);
    }
  if (lane == 0) { st[wv * N + 2 * H] = gsum0; st[wv * N + 2 * H + 1] = gsum1; }
  __syncthreads();
  for (int col = tid; col < N; col += 256)
    a.span_part[(size_t)blk * N + col] = ((st[col] + st[N + col]) + st[2 * N + col]) + st[3 * N + col];
}

template <typename F>
void dispatch_nch(int H, F&& f) {
  switch ((H + 255) / 256) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    case 6: f(std::integral_constant<int, 6>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    default: fprintf(stderr, "hq heads: unsupported hidden size %d\n", H); abort();
  }
}

}  // namespace

// ================================================================================== launchers
size_t hq_qa_heads_fwd_scratch(int B, int H) { return (size_t)(H / 64) * B * kHS; }

void hq_qa_heads_fwd(const void* seq, const HqHeadWeights& w, float* logits, float* pooled, float* cls, float* reg,
                     float* hpart, unsigned* cnt, int B, int L, int H, int NL, float p, uint32_t seed, uint32_t opid,
                     hipStream_t s, bool seq_f32) {
  FwdArgs a;
  a.seq = seq;
  a.wp = w.wp; a.bp = w.bp; a.wc = w.wc; a.bc = w.bc; a.wrs = w.wrs; a.brs = w.brs; a.wre = w.wre; a.bre = w.bre;
  a.wsp = w.wsp; a.bsp = w.bsp;
  a.logits = logits; a.pooled = pooled; a.cls = cls; a.reg = reg; a.hpart = hpart; a.cnt = cnt;
  a.B = B; a.L = L; a.H = H; a.NL = NL; a.T = B * L;
  a.npool = ((B + 31) / 32) * (H / 64);
  a.thr = p > 0.f ? hq_threshold(p) : 0u;
  a.kd = hq_drop_key(seed, opid);
  a.ks = hq_keep_scale(a.thr);
  const int nspan = (a.T + 4 * kSpanFwdRPW - 1) / (4 * kSpanFwdRPW);
  const size_t lds = (32 * 64 + 64 * 65) * sizeof(float);
  dispatch_nch(H, [&](auto nch) {
    if (seq_f32)
      hipLaunchKernelGGL((qa_heads_fwd_kernel<decltype(nch)::value, float>), dim3(a.npool + nspan), dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL((qa_heads_fwd_kernel<decltype(nch)::value, uint16_t>), dim3(a.npool + nspan), dim3(256), lds, s,
                         a);
  });
}

int hq_qa_loss_partials(int B) { return (B + 3) / 4 + 1; }

void hq_qa_loss(const float* logits, const float* cls, const float* reg, const int64_t* t_start, const int64_t* t_end,
                const int64_t* t_cls, const float* t_rs, const float* t_re, const float* lw, float* dlog, float* dheads,
                float* losses, float* part, unsigned* cnt, int B, int L, int NL, const HqLossCfg& cfg, const int* seg_len,
                int nseg, hipStream_t s) {
  LossArgs a;
  a.seg_len = seg_len;
  a.nseg = nseg > 0 ? nseg : 1;
  a.logits = logits; a.cls = cls; a.reg = reg;
  a.t_start = t_start; a.t_end = t_end; a.t_cls = t_cls; a.t_rs = t_rs; a.t_re = t_re; a.lw = lw;
  a.dlog = dlog; a.dheads = dheads; a.losses = losses; a.part = part; a.cnt = cnt;
  a.B = B; a.L = L; a.NL = NL; a.kind = cfg.kind; a.ignore_cls = cfg.ignore_cls;
  a.nrow = (B + 3) / 4;
  a.w0 = cfg.w[0]; a.w1 = cfg.w[1]; a.w2 = cfg.w[2]; a.w3 = cfg.w[3]; a.w4 = cfg.w[4];
  a.alpha = cfg.alpha; a.gamma = cfg.gamma; a.conf = cfg.conf; a.fill = cfg.fill;
  hipLaunchKernelGGL(qa_loss_kernel, dim3(a.nrow + 1), dim3(256), 0, s, a);
}

int hq_qa_heads_bwd_span_blocks(int T) { return (T + 4 * kSpanRPW - 1) / (4 * kSpanRPW); }

void hq_qa_heads_bwd(const void* seq, const float* dlog, const float* dheads, const float* gscale, const float* pooled,
                     const float* reg, const HqHeadWeights& w, const HqHeadGrads& g, void* dseq, float* span_part,
                     int B, int L, int H, int NL, bool accumulate, float p, uint32_t seed, uint32_t opid, hipStream_t s,
                     bool seq_f32, float* dpre) {
  BwdArgs a;
  a.dpre = dpre;
  a.seq = seq; a.dlog = dlog; a.dheads = dheads; a.gscale = gscale; a.pooled = pooled; a.reg = reg;
  a.wp = w.wp; a.wc = w.wc; a.wrs = w.wrs; a.wre = w.wre; a.wsp = w.wsp;
  a.dseq = dseq; a.span_part = span_part;
  a.gwp = g.gwp; a.gbp = g.gbp; a.gwc = g.gwc; a.gbc = g.gbc; a.gwrs = g.gwrs; a.gbrs = g.gbrs; a.gwre = g.gwre;
  a.gbre = g.gbre;
  a.B = B; a.L = L; a.H = H; a.NL = NL; a.T = B * L; a.acc = accumulate ? 1 : 0;
  const int nj = H / 64;
  a.nA = ((B + 31) / 32) * nj;
  a.nW = nj * nj;
  a.nS = nj;
  a.thr = p > 0.f ? hq_threshold(p) : 0u;
  a.kd = hq_drop_key(seed, opid);
  a.ks = hq_keep_scale(a.thr);
  const int nspan = hq_qa_heads_bwd_span_blocks(a.T);
  size_t lds = (32 * kHS + 32 * 64 + 64 * 64) * sizeof(float);                     // R1
  lds = std::max(lds, (size_t)4 * 64 * (kMaxNL + 3) * sizeof(float));              // R3
  lds = std::max(lds, (size_t)4 * (2 * H + 2) * sizeof(float));                    // R4
  if (dpre) hipLaunchKernelGGL(qa_dpre_kernel, dim3((unsigned)(((size_t)B * H + 255) / 256)), dim3(256), 0, s, a);
  dispatch_nch(H, [&](auto nch) {
    if (seq_f32)
      hipLaunchKernelGGL((qa_heads_bwd_kernel<decltype(nch)::value, float>), dim3(a.nA + a.nW + a.nS + nspan), dim3(256),
                         lds, s, a);
    else
      hipLaunchKernelGGL((qa_heads_bwd_kernel<decltype(nch)::value, uint16_t>), dim3(a.nA + a.nW + a.nS + nspan),
                         dim3(256), lds, s, a);
  });
  hq_colsum_outs(span_part, nspan, 2 * H + 2, HqOuts{{g.gwsp, g.gwsp ? g.gwsp + H : nullptr, g.gbsp, nullptr}}, H,
                 accumulate, s);
}
