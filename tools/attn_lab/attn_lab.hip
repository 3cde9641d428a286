// Attention-forward lab: times the production forward against instrumented / restructured variants
// at one BERT shape (hipEvent timing, no torch).  Build + run: tools/attn_lab/run.sh
#include "../../ml_recipe_distributed_pytorch_amd/csrc/kernels/attention.hip"

#include <cmath>
#include <cstring>
#include <cstdio>
#include <vector>

namespace {

typedef float f2_t __attribute__((ext_vector_type(2)));

// single-matrix prologue loader (the production kernels now use load_heads2 for K and V together)
template <int NT>
__device__ __forceinline__ void load_head(uint16_t* dst, const uint16_t* src, size_t ld, int L, int Lp) {
  for (int t = threadIdx.x; t < Lp * 8; t += NT) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if ((t >> 3) < L) v = *reinterpret_cast<const uint4*>(src + (size_t)(t >> 3) * ld + (t & 7) * 8);
    *reinterpret_cast<uint4*>(dst + lds_off(t >> 3, (t & 7) * 8)) = v;
  }
}

// V1: prologue + epilogue only (what the loads cost with no compute).
template <int NWB>
__global__ __launch_bounds__(NWB * 64) void fwd_prologue_only(const uint16_t* __restrict__ qkv,
                                                                const float* __restrict__ key_bias,
                                                                uint16_t* __restrict__ ctx, float* __restrict__ lse,
                                                                int L, int nh, float c_scale) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Lp = (L + 31) & ~31;
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sV = sK + Lp * D;
  float* sB = reinterpret_cast<float*>(sV + Lp * D);
  const int H = nh * D, ld = 3 * H;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, hh = lane >> 5;
  const int qs = blockIdx.y * NWB + wave;
  const int qi = qs * 32 + (lane & 31);
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = (qi < L) ? prescale8(*reinterpret_cast<const bf16x8_t*>(base + (size_t)qi * ld + 16 * s + 8 * hh), c_scale)
                     : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  load_head<NWB * 64>(sK, base + H, ld, L, Lp);
  load_head<NWB * 64>(sV, base + 2 * H, ld, L, Lp);
  for (int t = threadIdx.x; t < Lp; t += NWB * 64) sB[t] = t < L ? key_bias[(size_t)b * L + t] * LOG2E : -INFINITY;
  __syncthreads();
  if (qi < L) {
    uint16_t* out = ctx + ((size_t)b * L + qi) * H + h * D;
    LdsOffsets lo_;
    lo_.init(lane);
    bf16x8_t x = row8(sK, (qs * 32) % Lp, lo_, 0);
    float v4[4] = {(float)qf[0][0] + (float)x[0], sB[lane], 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2*>(out + d * 32 + 8 * g + 4 * hh) = hq_pack4(v4);
    if (hh == 0) lse[(size_t)bh * L + qi] = 0.f;
  }
}

// V2: p = 0 forward with a compile-time tile count (fully unrolled: LDS offsets become immediates),
// packed-f32 subtract / row-sum / rescale and max3 trees.
template <int NWB, int NT>
__global__ __launch_bounds__(NWB * 64) void fwd_v2(const uint16_t* __restrict__ qkv, const float* __restrict__ key_bias,
                                                     uint16_t* __restrict__ ctx, float* __restrict__ lse, int L, int nh,
                                                     float c_scale) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int Lp = NT * 32;
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sV = sK + Lp * D;
  float* sB = reinterpret_cast<float*>(sV + Lp * D);
  const int H = nh * D, ld = 3 * H;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, hh = lane >> 5;
  const int qs = blockIdx.y * NWB + wave;
  const int qi = qs * 32 + (lane & 31);
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = (qi < L) ? prescale8(*reinterpret_cast<const bf16x8_t*>(base + (size_t)qi * ld + 16 * s + 8 * hh), c_scale)
                     : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  load_head<NWB * 64>(sK, base + H, ld, L, Lp);
  load_head<NWB * 64>(sV, base + 2 * H, ld, L, Lp);
  for (int t = threadIdx.x; t < Lp; t += NWB * 64) sB[t] = t < L ? key_bias[(size_t)b * L + t] * LOG2E : -INFINITY;
  __syncthreads();
  if (qs * 32 >= L) return;
  LdsOffsets lo_;
  lo_.init(lane);
  f32x16_t o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -INFINITY;
  f2_t l2 = {0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    f32x16_t acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bb = *reinterpret_cast<const float4*>(sB + kt * 32 + 8 * g + 4 * hh);
      acc[4 * g + 0] = bb.x; acc[4 * g + 1] = bb.y; acc[4 * g + 2] = bb.z; acc[4 * g + 3] = bb.w;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma32(row8(sK, kt * 32, lo_, s), qf[s], acc);
    float mx = fmaxf(fmaxf(acc[0], acc[1]), acc[2]);
    mx = fmaxf(fmaxf(mx, acc[3]), acc[4]);
    mx = fmaxf(fmaxf(mx, acc[5]), acc[6]);
    mx = fmaxf(fmaxf(mx, acc[7]), acc[8]);
    mx = fmaxf(fmaxf(mx, acc[9]), acc[10]);
    mx = fmaxf(fmaxf(mx, acc[11]), acc[12]);
    mx = fmaxf(fmaxf(mx, acc[13]), acc[14]);
    mx = fmaxf(mx, acc[15]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (__any(mx > m_run)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      m_run = m_new;
      const f2_t a2 = {alpha, alpha};
      l2 *= a2;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          f2_t v = {o[d][r], o[d][r + 1]};
          v *= a2;
          o[d][r] = v.x; o[d][r + 1] = v.y;
        }
    }
    float sc[16];
    const f2_t m2 = {m_run, m_run};
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      f2_t v = {acc[r], acc[r + 1]};
      v -= m2;
      sc[r] = __builtin_amdgcn_exp2f(v.x);
      sc[r + 1] = __builtin_amdgcn_exp2f(v.y);
      const f2_t e = {sc[r], sc[r + 1]};
      l2 += e;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8_t pb = pack_b(sc, s);
#pragma unroll
      for (int d = 0; d < 2; ++d) o[d] = mfma32(tr8(sV, kt * 32, lo_, s, d), pb, o[d]);
    }
  }
  const float l_run = l2.x + l2.y;
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
    if (hh == 0) lse[(size_t)bh * L + qi] = (m_run + __builtin_amdgcn_logf(l_tot)) * LN2;
  }
}

// LDS-DMA one [rows][64] bf16 head slice into the swizzled image: each wave-instruction moves 8 rows
// (1 KB, lane-linear destination); the swizzle is applied to the per-lane SOURCE chunk.
template <int NWB>
__device__ __forceinline__ void dma_head(uint16_t* dst, const uint16_t* src, int ld, int L, int Lp, int wave, int lane) {
  const int r_in = lane >> 3, slot = lane & 7;
  for (int r0 = wave * 8; r0 < Lp; r0 += NWB * 8) {
    const int row = r0 + r_in;
    const int chunk = slot ^ swz(row);
    const uint16_t* g = src + (size_t)min(row, L - 1) * ld + chunk * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)(dst + r0 * D), 16, 0, 0);
  }
}

// V3: v2 + single-latency prologue (Q loads, K/V LDS-DMA and the bias load all in flight together).
template <int NWB, int NT>
__global__ __launch_bounds__(NWB * 64) void fwd_v3(const uint16_t* __restrict__ qkv, const float* __restrict__ key_bias,
                                                     uint16_t* __restrict__ ctx, float* __restrict__ lse, int L, int nh,
                                                     float c_scale) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int Lp = NT * 32;
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sV = sK + Lp * D;
  float* sB = reinterpret_cast<float*>(sV + Lp * D);
  const int H = nh * D, ld = 3 * H;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, hh = lane >> 5;
  const int qs = blockIdx.y * NWB + wave;
  const int qi = qs * 32 + (lane & 31);
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  bf16x8_t qraw[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qraw[s] = *reinterpret_cast<const bf16x8_t*>(base + (size_t)min(qi, L - 1) * ld + 16 * s + 8 * hh);
  dma_head<NWB>(sK, base + H, ld, L, Lp, wave, lane);
  dma_head<NWB>(sV, base + 2 * H, ld, L, Lp, wave, lane);
  float kbv = 0.f;
  const int tb = threadIdx.x;
  if (tb < Lp) kbv = tb < L ? key_bias[(size_t)b * L + tb] : 0.f;
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
  if (tb < Lp) sB[tb] = tb < L ? kbv * LOG2E : -INFINITY;
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = prescale8(qraw[s], c_scale);
  __syncthreads();
  if (qs * 32 >= L) return;
  LdsOffsets lo_;
  lo_.init(lane);
  f32x16_t o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -INFINITY;
  f2_t l2 = {0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    f32x16_t acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bb = *reinterpret_cast<const float4*>(sB + kt * 32 + 8 * g + 4 * hh);
      acc[4 * g + 0] = bb.x; acc[4 * g + 1] = bb.y; acc[4 * g + 2] = bb.z; acc[4 * g + 3] = bb.w;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma32(row8(sK, kt * 32, lo_, s), qf[s], acc);
    float mx = fmaxf(fmaxf(acc[0], acc[1]), acc[2]);
    mx = fmaxf(fmaxf(mx, acc[3]), acc[4]);
    mx = fmaxf(fmaxf(mx, acc[5]), acc[6]);
    mx = fmaxf(fmaxf(mx, acc[7]), acc[8]);
    mx = fmaxf(fmaxf(mx, acc[9]), acc[10]);
    mx = fmaxf(fmaxf(mx, acc[11]), acc[12]);
    mx = fmaxf(fmaxf(mx, acc[13]), acc[14]);
    mx = fmaxf(mx, acc[15]);
    {
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    }
    if (__any(mx > m_run)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      m_run = m_new;
      const f2_t a2 = {alpha, alpha};
      l2 *= a2;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          f2_t v = {o[d][r], o[d][r + 1]};
          v *= a2;
          o[d][r] = v.x; o[d][r + 1] = v.y;
        }
    }
    float sc[16];
    const f2_t m2 = {m_run, m_run};
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      f2_t v = {acc[r], acc[r + 1]};
      v -= m2;
      sc[r] = __builtin_amdgcn_exp2f(v.x);
      sc[r + 1] = __builtin_amdgcn_exp2f(v.y);
      const f2_t e = {sc[r], sc[r + 1]};
      l2 += e;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8_t pb = pack_b(sc, s);
#pragma unroll
      for (int d = 0; d < 2; ++d) o[d] = mfma32(tr8(sV, kt * 32, lo_, s, d), pb, o[d]);
    }
  }
  const float l_run = l2.x + l2.y;
  float l_tot;
  {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
    l_tot = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
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
    if (hh == 0) lse[(size_t)bh * L + qi] = (m_run + __builtin_amdgcn_logf(l_tot)) * LN2;
  }
}

// V3 prologue only
template <int NWB, int NT>
__global__ __launch_bounds__(NWB * 64) void fwd_v3_prologue(const uint16_t* __restrict__ qkv, const float* __restrict__ key_bias,
                                                     uint16_t* __restrict__ ctx, float* __restrict__ lse, int L, int nh,
                                                     float c_scale) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int Lp = NT * 32;
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sV = sK + Lp * D;
  float* sB = reinterpret_cast<float*>(sV + Lp * D);
  const int H = nh * D, ld = 3 * H;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, hh = lane >> 5;
  const int qs = blockIdx.y * NWB + wave;
  const int qi = qs * 32 + (lane & 31);
  const uint16_t* base = qkv + (size_t)b * L * ld + h * D;
  bf16x8_t qraw[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qraw[s] = *reinterpret_cast<const bf16x8_t*>(base + (size_t)min(qi, L - 1) * ld + 16 * s + 8 * hh);
  dma_head<NWB>(sK, base + H, ld, L, Lp, wave, lane);
  dma_head<NWB>(sV, base + 2 * H, ld, L, Lp, wave, lane);
  float kbv = 0.f;
  const int tb = threadIdx.x;
  if (tb < Lp) kbv = tb < L ? key_bias[(size_t)b * L + tb] : 0.f;
  __builtin_amdgcn_s_waitcnt(0);
  if (tb < Lp) sB[tb] = tb < L ? kbv * LOG2E : -INFINITY;
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = prescale8(qraw[s], c_scale);
  __syncthreads();
  if (qi < L) {
    uint16_t* out = ctx + ((size_t)b * L + qi) * H + h * D;
    LdsOffsets lo_;
    lo_.init(lane);
    bf16x8_t x = row8(sK, (qs * 32) % Lp, lo_, 0);
    bf16x8_t y = row8(sV, (qs * 32) % Lp, lo_, 1);
    float v4[4] = {(float)qf[0][0] + (float)x[0] + (float)y[1], sB[lane], 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2*>(out + d * 32 + 8 * g + 4 * hh) = hq_pack4(v4);
    if (hh == 0) lse[(size_t)bh * L + qi] = 0.f;
  }
}

// V4: persistent workgroups (one per CU) walking heads; K/V live in an LDS image that is refilled
// chunk by chunk: once every wave has finished key tile kt-1 of head i (the barrier at the top of
// tile kt), that 32-row slot is re-filled by LDS-DMA with head i+1's rows, so the next head's loads
// hide behind this head's compute.  Waves 0-3 move K rows, waves 4-7 V rows (one 1-KB DMA each per
// step); the only waits are vmcnt(0) at the head boundary (everything then in flight is >= 1 tile old)
// and a counted wait before tile NT-1 for the slot refilled at the boundary.
template <int NWB, int NT, int UNR>
__global__ __launch_bounds__(NWB * 64) void fwd_v4(const uint16_t* __restrict__ qkv, const float* __restrict__ key_bias,
                                                     uint16_t* __restrict__ ctx, float* __restrict__ lse, int L, int nh,
                                                     int n_bh, float c_scale) {
  static_assert(NWB == NT && NT * 32 <= NWB * 64, "one wave per 32-query subtile, one bias thread per key");
  // requires L == NT * 32 (no ragged last tile)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int Lp = NT * 32;
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sV = sK + Lp * D;
  uint16_t* sQ = sV + Lp * D;                         // next head's Q rows (DMA), read at the boundary
  float* sB = reinterpret_cast<float*>(sQ + Lp * D);  // [2][Lp], by head parity
  const int H = nh * D, ld = 3 * H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, hh = lane >> 5;
  const int tid = threadIdx.x;
  const int qi = wave * 32 + (lane & 31);
  // LDS-DMA source offsets: the swizzle depends on row bits 1..4 only, so a lane's byte offset inside
  // any 32-row chunk is loop-invariant; the chunk base is wave-uniform (scalar address arithmetic).
  const int r_lane = (wave & 3) * 8 + (lane >> 3);
  const uint32_t off_kv = (uint32_t)(r_lane * ld + (((lane & 7) ^ swz(r_lane)) << 3)) * 2u;
  auto uniform_ptr = [](const uint16_t* p) -> const char* {
    const uint64_t u = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return (const char*)(((uint64_t)hi << 32) | lo);
  };
  auto dma_chunk = [&](int bh_, int kt) {
    if (wave < 8) {
      const int b_ = bh_ / nh, h_ = bh_ - b_ * nh;
      uint32_t step = (uint32_t)kt * 32u * (uint32_t)ld * 2u;
      asm volatile("" : "+s"(step));  // materialise here (keeps the unrolled loop from hoisting 11 pointers)
      const char* src = uniform_ptr(qkv + (size_t)b_ * L * ld + h_ * D + (wave < 4 ? H : 2 * H)) + step;
      uint16_t* dst = (wave < 4 ? sK : sV) + (kt * 32 + (wave & 3) * 8) * D;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + off_kv),
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  auto dma_q = [&](int bh_) {  // all Lp rows of Q: Lp/8/NWB 1-KB pieces per wave
    const int b_ = bh_ / nh, h_ = bh_ - b_ * nh;
#pragma unroll
    for (int i = 0; i < Lp / 8 / NWB; ++i) {
      const int r0 = (wave * (Lp / 8 / NWB) + i) * 8;
      const int row = r0 + (lane >> 3);
      const uint32_t off = (uint32_t)((lane >> 3) * ld + (((lane & 7) ^ swz(row)) << 3)) * 2u;
      const char* src = uniform_ptr(qkv + ((size_t)b_ * L + r0) * ld + h_ * D);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + off),
                                       (__attribute__((address_space(3))) void*)(sQ + r0 * D), 16, 0, 0);
    }
  };
  auto q_from_lds = [&](bf16x8_t* q) {  // this wave's 32 query rows, fragment layout of the score MFMA
    LdsOffsets lo;
    lo.init(lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) q[s] = prescale8(row8(sQ, wave * 32, lo, s), c_scale);
  };
  auto load_bias = [&](int bh_) -> float {
    const int b_ = bh_ / nh;
    return (tid < L) ? key_bias[(size_t)b_ * L + tid] : 0.f;
  };
  int bh = blockIdx.x;
  if (bh >= n_bh) return;
  bf16x8_t qf[4];
  dma_q(bh);
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) dma_chunk(bh, kt);
  float kbn = load_bias(bh);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (tid < Lp) sB[tid] = tid < L ? kbn * LOG2E : -INFINITY;
  __builtin_amdgcn_s_barrier();
  q_from_lds(qf);
  LdsOffsets lo_;
  lo_.init(lane);
  for (int it = 0;; ++it) {
    const int nbh = bh + gridDim.x;
    const bool has_next = nbh < n_bh;
    const float* sBc = sB + (it & 1) * Lp;
    f32x16_t o[2];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
    float m_run = -INFINITY;
    f2_t l2 = {0.f, 0.f};
#pragma unroll UNR
    for (int kt = 0; kt < NT; ++kt) {
      if (kt > 0) {
        if (kt == NT - 1) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");  // slot NT-1 (refilled at the boundary)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own reads of slot kt-1 retired before it is refilled
        __builtin_amdgcn_s_barrier();
        if (has_next) dma_chunk(nbh, kt - 1);
      }
      if (kt == NT / 2 && has_next) {
        dma_q(nbh);
        kbn = load_bias(nbh);
      }
      f32x16_t acc;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bb = *reinterpret_cast<const float4*>(sBc + kt * 32 + 8 * g + 4 * hh);
        acc[4 * g + 0] = bb.x; acc[4 * g + 1] = bb.y; acc[4 * g + 2] = bb.z; acc[4 * g + 3] = bb.w;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma32(row8(sK, kt * 32, lo_, s), qf[s], acc);
      float mx = fmaxf(fmaxf(acc[0], acc[1]), acc[2]);
      mx = fmaxf(fmaxf(mx, acc[3]), acc[4]);
      mx = fmaxf(fmaxf(mx, acc[5]), acc[6]);
      mx = fmaxf(fmaxf(mx, acc[7]), acc[8]);
      mx = fmaxf(fmaxf(mx, acc[9]), acc[10]);
      mx = fmaxf(fmaxf(mx, acc[11]), acc[12]);
      mx = fmaxf(fmaxf(mx, acc[13]), acc[14]);
      mx = fmaxf(mx, acc[15]);
      {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
      }
      if (__any(mx > m_run)) {
        const float m_new = fmaxf(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        const f2_t a2 = {alpha, alpha};
        l2 *= a2;
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            f2_t v = {o[d][r], o[d][r + 1]};
            v *= a2;
            o[d][r] = v.x; o[d][r + 1] = v.y;
          }
      }
      float sc[16];
      const f2_t m2 = {m_run, m_run};
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        f2_t v = {acc[r], acc[r + 1]};
        v -= m2;
        sc[r] = __builtin_amdgcn_exp2f(v.x);
        sc[r + 1] = __builtin_amdgcn_exp2f(v.y);
        const f2_t e = {sc[r], sc[r + 1]};
        l2 += e;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t pb = pack_b(sc, s);
#pragma unroll
        for (int d = 0; d < 2; ++d) o[d] = mfma32(tr8(sV, kt * 32, lo_, s, d), pb, o[d]);
      }
    }
    const float l_run = l2.x + l2.y;
    float l_tot;
    {
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
      l_tot = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    const float inv = 1.f / l_tot;
    {
      const int b_ = bh / nh, h_ = bh - b_ * nh;
      if (qi < L) {
        uint16_t* out = ctx + ((size_t)b_ * L + qi) * H + h_ * D;
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float v4[4] = {o[d][4 * g] * inv, o[d][4 * g + 1] * inv, o[d][4 * g + 2] * inv, o[d][4 * g + 3] * inv};
            *reinterpret_cast<uint2*>(out + d * 32 + 8 * g + 4 * hh) = hq_pack4(v4);
          }
        if (hh == 0) lse[(size_t)bh * L + qi] = (m_run + __builtin_amdgcn_logf(l_tot)) * LN2;
      }
    }
    if (!has_next) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // next head's slots 0..NT-2, its Q and bias
    if (tid < Lp) sB[((it + 1) & 1) * Lp + tid] = tid < L ? kbn * LOG2E : -INFINITY;
    __builtin_amdgcn_s_barrier();  // every wave is done with slot NT-1; next Q / bias visible
    q_from_lds(qf);
    dma_chunk(nbh, NT - 1);
    bh = nbh;
  }
}

// Lab probes: (a) the v2 loop with no global loads (LDS left as is), (b) the v3 prologue reading a
// head-major [B*nh][3][L][64] copy (each head's K/V/Q contiguous) instead of the packed [T,3H] rows.
template <int NWB, int NT>
__global__ __launch_bounds__(NWB * 64) void fwd_compute_only(uint16_t* __restrict__ ctx, float* __restrict__ lse, int L,
                                                               int nh) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int Lp = NT * 32;
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sV = sK + Lp * D;
  float* sB = reinterpret_cast<float*>(sV + Lp * D);
  const int H = nh * D;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, hh = lane >> 5;
  const int qi = wave * 32 + (lane & 31);
  for (int t = threadIdx.x; t < Lp * D; t += NWB * 64) { sK[t] = 0x3c00; sV[t] = 0x3c00; }
  for (int t = threadIdx.x; t < Lp; t += NWB * 64) sB[t] = 0.f;
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = bf16x8_t{(short)(lane + s), 1, 2, 3, 4, 5, 6, 7};
  __syncthreads();
  LdsOffsets lo_;
  lo_.init(lane);
  f32x16_t o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -INFINITY;
  f2_t l2 = {0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    f32x16_t acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bb = *reinterpret_cast<const float4*>(sB + kt * 32 + 8 * g + 4 * hh);
      acc[4 * g + 0] = bb.x; acc[4 * g + 1] = bb.y; acc[4 * g + 2] = bb.z; acc[4 * g + 3] = bb.w;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma32(row8(sK, kt * 32, lo_, s), qf[s], acc);
    float mx = fmaxf(fmaxf(acc[0], acc[1]), acc[2]);
    mx = fmaxf(fmaxf(mx, acc[3]), acc[4]);
    mx = fmaxf(fmaxf(mx, acc[5]), acc[6]);
    mx = fmaxf(fmaxf(mx, acc[7]), acc[8]);
    mx = fmaxf(fmaxf(mx, acc[9]), acc[10]);
    mx = fmaxf(fmaxf(mx, acc[11]), acc[12]);
    mx = fmaxf(fmaxf(mx, acc[13]), acc[14]);
    mx = fmaxf(mx, acc[15]);
    {
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    }
    if (__any(mx > m_run)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      m_run = m_new;
      const f2_t a2 = {alpha, alpha};
      l2 *= a2;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          f2_t v = {o[d][r], o[d][r + 1]};
          v *= a2;
          o[d][r] = v.x; o[d][r + 1] = v.y;
        }
    }
    float sc[16];
    const f2_t m2 = {m_run, m_run};
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      f2_t v = {acc[r], acc[r + 1]};
      v -= m2;
      sc[r] = __builtin_amdgcn_exp2f(v.x);
      sc[r + 1] = __builtin_amdgcn_exp2f(v.y);
      const f2_t e = {sc[r], sc[r + 1]};
      l2 += e;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8_t pb = pack_b(sc, s);
#pragma unroll
      for (int d = 0; d < 2; ++d) o[d] = mfma32(tr8(sV, kt * 32, lo_, s, d), pb, o[d]);
    }
  }
  const float l_tot = l2.x + l2.y;
  if (qi < L && o[0][0] + o[1][5] + l_tot == 1234.5f) ctx[(size_t)bh * 64 + lane] = 1;  // keep the work live
  if (qi < L && hh == 0 && m_run == 12345.f) lse[(size_t)bh * L + qi] = 0.f;
}

template <int NWB, int NT>
__global__ __launch_bounds__(NWB * 64) void fwd_prologue_headmajor(const uint16_t* __restrict__ hm,
                                                                     uint16_t* __restrict__ ctx, int L, int nh) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int Lp = NT * 32;
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sV = sK + Lp * D;
  const int H = nh * D;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, hh = lane >> 5;
  const int qi = wave * 32 + (lane & 31);
  const uint16_t* hq = hm + (size_t)bh * 3 * L * D;
  bf16x8_t qraw[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qraw[s] = *reinterpret_cast<const bf16x8_t*>(hq + (size_t)qi * D + 16 * s + 8 * hh);
  dma_head<NWB>(sK, hq + L * D, D, L, Lp, wave, lane);
  dma_head<NWB>(sV, hq + 2 * L * D, D, L, Lp, wave, lane);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  LdsOffsets lo_;
  lo_.init(lane);
  bf16x8_t x = row8(sK, wave * 32, lo_, 0);
  bf16x8_t y = row8(sV, wave * 32, lo_, 1);
  float v4[4] = {(float)qraw[0][0] + (float)x[0] + (float)y[1], 0.f, 0.f, 0.f};
  uint16_t* out = ctx + ((size_t)b * L + qi) * H + h * D;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2*>(out + d * 32 + 8 * g + 4 * hh) = hq_pack4(v4);
}

}  // namespace

static float bf2f(uint16_t u) {
  uint32_t x = (uint32_t)u << 16;
  float f;
  std::memcpy(&f, &x, 4);
  return f;
}

template <typename F>
static float time_it(F&& f, int iters = 20) {
  hipEvent_t a, b;
  HQ_CHECK(hipEventCreate(&a));
  HQ_CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  HQ_CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  HQ_CHECK(hipEventRecord(b));
  HQ_CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  HQ_CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256, L = 384, nh = 12, H = nh * D;
  const size_t T = (size_t)B * L;
  std::vector<uint16_t> hq(T * 3 * H);
  uint32_t st = 12345u;
  for (auto& x : hq) {
    st = st * 1664525u + 1013904223u;
    const float f = ((st >> 8) & 0xFFFF) / 32768.f - 1.f;
    uint32_t u;
    std::memcpy(&u, &f, 4);
    x = (uint16_t)(u >> 16);
  }
  uint16_t *qkv, *ctx0, *ctx1;
  float *kb, *lse0, *lse1;
  HQ_CHECK(hipMalloc(&qkv, hq.size() * 2));
  HQ_CHECK(hipMalloc(&ctx0, T * H * 2));
  HQ_CHECK(hipMalloc(&ctx1, T * H * 2));
  HQ_CHECK(hipMalloc(&kb, T * 4));
  HQ_CHECK(hipMalloc(&lse0, (size_t)B * nh * L * 4));
  HQ_CHECK(hipMalloc(&lse1, (size_t)B * nh * L * 4));
  HQ_CHECK(hipMemcpy(qkv, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
  HQ_CHECK(hipMemset(kb, 0, T * 4));
  const float scale = 0.125f;
  const int Lp = 384;
  const size_t lds = (size_t)Lp * D * 2 * 2 + Lp * sizeof(float);
  const double flops = 4.0 * B * nh * (double)L * L * D;
  auto report = [&](const char* name, float us) {
    printf("%-28s %8.1f us  %7.1f TF/s\n", name, us, flops / us / 1e6);
  };
  // baseline
  report("fwd prod p=0", time_it([&] { hq_attn_fwd(qkv, kb, ctx0, lse0, nullptr, B, L, nh, D, 0.f, 1, 1, scale, 0); }));

  {
    auto k = fwd_v2<12, 12>;
    HQ_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    report("v2 unrolled+pk p=0", time_it([&] {
             hipLaunchKernelGGL(k, dim3(B * nh, 1), dim3(768), lds, 0, qkv, kb, ctx1, lse1, L, nh, scale * LOG2E);
           }));
    HQ_CHECK(hipDeviceSynchronize());
    std::vector<uint16_t> a(T * H), b(T * H);
    HQ_CHECK(hipMemcpy(a.data(), ctx0, T * H * 2, hipMemcpyDeviceToHost));
    HQ_CHECK(hipMemcpy(b.data(), ctx1, T * H * 2, hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < a.size(); ++i) md = std::max(md, (double)fabsf(bf2f(a[i]) - bf2f(b[i])));
    printf("  v2 vs prod max|diff| = %.3g\n", md);
  }


  auto run_v4 = [&](auto k, const char* tag) {
    HQ_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const size_t lds4 = (size_t)Lp * D * 2 * 3 + 2 * Lp * sizeof(float);
    for (int g : {256, 512}) {
      char nm[64];
      snprintf(nm, sizeof nm, "v4 %s grid=%d", tag, g);
      HQ_CHECK(hipMemset(ctx1, 0, T * H * 2));
      report(nm, time_it([&] {
               hipLaunchKernelGGL(k, dim3(g), dim3(768), lds4, 0, qkv, kb, ctx1, lse1, L, nh, B * nh, scale * LOG2E);
             }));
      HQ_CHECK(hipDeviceSynchronize());
      std::vector<uint16_t> a(T * H), b(T * H);
      HQ_CHECK(hipMemcpy(a.data(), ctx0, T * H * 2, hipMemcpyDeviceToHost));
      HQ_CHECK(hipMemcpy(b.data(), ctx1, T * H * 2, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < a.size(); ++i) md = std::max(md, (double)fabsf(bf2f(a[i]) - bf2f(b[i])));
      printf("  v4 vs prod max|diff| = %.3g\n", md);
    }
  };


  {
    auto k1 = fwd_prologue_only<12>;
    HQ_CHECK(hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    report("prologue+epilogue only", time_it([&] {
             hipLaunchKernelGGL(k1, dim3(B * nh, 1), dim3(768), lds, 0, qkv, kb, ctx1, lse1, L, nh, scale * LOG2E);
           }));
    auto k3 = fwd_v3_prologue<12, 12>;
    HQ_CHECK(hipFuncSetAttribute((const void*)k3, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    report("v3 (DMA) prologue only", time_it([&] {
             hipLaunchKernelGGL(k3, dim3(B * nh, 1), dim3(768), lds, 0, qkv, kb, ctx1, lse1, L, nh, scale * LOG2E);
           }));
  }
  run_v4(fwd_v4<12, 12, 12>, "persistent");
  {
    auto k = fwd_v3<12, 12>;
    HQ_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    for (int rep = 0; rep < 2; ++rep) {
      report("v3 DMA prologue p=0", time_it([&] {
               hipLaunchKernelGGL(k, dim3(B * nh, 1), dim3(768), lds, 0, qkv, kb, ctx1, lse1, L, nh, scale * LOG2E);
             }));
      report("fwd prod p=0 (interleaved)",
             time_it([&] { hq_attn_fwd(qkv, kb, ctx0, lse0, nullptr, B, L, nh, D, 0.f, 1, 1, scale, 0); }));
    }
    HQ_CHECK(hipDeviceSynchronize());
    std::vector<uint16_t> a(T * H), b(T * H);
    HQ_CHECK(hipMemcpy(a.data(), ctx0, T * H * 2, hipMemcpyDeviceToHost));
    HQ_CHECK(hipMemcpy(b.data(), ctx1, T * H * 2, hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < a.size(); ++i) md = std::max(md, (double)fabsf(bf2f(a[i]) - bf2f(b[i])));
    printf("  v3 vs prod max|diff| = %.3g\n", md);
  }

  report("fwd prod p=0 (again)", time_it([&] { hq_attn_fwd(qkv, kb, ctx0, lse0, nullptr, B, L, nh, D, 0.f, 1, 1, scale, 0); }));
  report("fwd prod p=0.1", time_it([&] {
           static uint16_t* bits = nullptr;
           if (!bits) HQ_CHECK(hipMalloc(&bits, hq_attn_mask_bytes(B, L, nh)));
           hq_attn_fwd(qkv, kb, ctx0, lse0, bits, B, L, nh, D, 0.1f, 1, 1, scale, 0);
         }));
  return 0;
}
