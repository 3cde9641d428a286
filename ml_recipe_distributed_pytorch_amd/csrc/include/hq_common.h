// Shared device helpers for the gfx950 (CDNA4) kernels.
// - wave64 reductions (never 32-wide warp idioms)
// - bf16 <-> f32 packing for 8/16-byte vector access
// - the counter-hash dropout RNG, bit-identical to ml_recipe_distributed_pytorch_amd/ops/rng.py
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "hq_kernels.h"   // kHqGdLo / kHqGdStep

#define HQ_WAVE 64

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // MFMA A/B fragment (4 VGPRs)
typedef __attribute__((ext_vector_type(4))) short bf16x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;  // 32x32 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

// ------------------------------------------------------------------------------ bf16 helpers
typedef __bf16 hq_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float hq_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float hq_bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
// RNE f32 -> bf16.  A vector convert of a PAIR lowers to ONE v_cvt_pk_bf16_f32 on gfx950 (NaN-safe);
// converting the halves separately costs 4 instructions per pair.
__device__ __forceinline__ uint32_t hq_pack2(float lo, float hi) {
  hq_f32x2_t f = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, hq_bf16x2_t));
}
__device__ __forceinline__ uint16_t hq_f2bf(float f) { return (uint16_t)(hq_pack2(f, 0.f) & 0xFFFFu); }
__device__ __forceinline__ void hq_unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xFFFF0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xFFFF0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xFFFF0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xFFFF0000u);
}
__device__ __forceinline__ uint4 hq_pack8(const float* f) {
  return make_uint4(hq_pack2(f[0], f[1]), hq_pack2(f[2], f[3]), hq_pack2(f[4], f[5]), hq_pack2(f[6], f[7]));
}
__device__ __forceinline__ void hq_unpack4(const uint2& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xFFFF0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xFFFF0000u);
}
__device__ __forceinline__ uint2 hq_pack4(const float* f) {
  return make_uint2(hq_pack2(f[0], f[1]), hq_pack2(f[2], f[3]));
}

// ------------------------------------------------------------------------------ GELU (erf form)
// Normal CDF Φ(x) and pdf φ(x) sharing ONE exp: Abramowitz–Stegun 7.1.25 for erf(|x|/√2) (three terms,
// |erf err| < 2.5e-5 → |Φ err| < 1.3e-5, far below bf16 resolution; 1/√2 and ½ folded into the constants)
// with raw v_rcp / v_exp; the negative tail is computed as q directly (no 1 - (1 - q) cancellation).
__device__ __forceinline__ void hq_normal_cdf_pdf(float x, float& cdf, float& pdf) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.33267340f, fabsf(x), 1.f));     // p / √2
  const float poly = fmaf(fmaf(0.3739278f, t, -0.0479399f), t, 0.1740121f) * t;
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);       // e^{-x²/2}
  const float q = poly * e;                                                    // Φ(-|x|)
  cdf = x >= 0.f ? 1.f - q : q;
  pdf = 0.3989422804014327f * e;
}
__device__ __forceinline__ float hq_gelu(float x) {
  float c, d;
  hq_normal_cdf_pdf(x, c, d);
  return x * c;
}
__device__ __forceinline__ float hq_gelu_grad(float x) {
  float c, d;
  hq_normal_cdf_pdf(x, c, d);
  return fmaf(x, d, c);
}

// GELU and GELU' of 8 values (the GELUD GEMM epilogues) in packed fp32 (v_pk_mul_f32 / v_pk_fma_f32, two
// lanes' worth per instruction); only rcp / exp2 stay scalar.  Same operations in the same order as
// hq_normal_cdf_pdf + fmaf(x, pdf, cdf) / x·cdf, so the results are bitwise those of the scalar form.
typedef float hq_f2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ hq_f2_t hq_s2(float c) { return hq_f2_t{c, c}; }
__device__ __forceinline__ hq_f2_t hq_fma2(hq_f2_t a, hq_f2_t b, hq_f2_t c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ void hq_gelu_grad8(float* x, float* g) {
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const hq_f2_t v = {x[e], x[e + 1]};
    const hq_f2_t den = hq_fma2(hq_s2(0.33267340f), hq_f2_t{fabsf(v.x), fabsf(v.y)}, hq_s2(1.f));
    const hq_f2_t t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
    hq_f2_t p = hq_fma2(hq_s2(0.3739278f), t, hq_s2(-0.0479399f));
    p = hq_fma2(p, t, hq_s2(0.1740121f)) * t;
    const hq_f2_t ea = (v * v) * hq_s2(-0.72134752044448170f);
    const hq_f2_t ex = {__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
    const hq_f2_t q = p * ex;                                        // Φ(-|x|)
    const hq_f2_t omq = hq_s2(1.f) - q;
    const hq_f2_t cdf = {v.x >= 0.f ? omq.x : q.x, v.y >= 0.f ? omq.y : q.y};
    const hq_f2_t pdf = hq_s2(0.3989422804014327f) * ex;
    const hq_f2_t gr = hq_fma2(v, pdf, cdf);
    const hq_f2_t y = v * cdf;
    g[e] = gr.x; g[e + 1] = gr.y;
    x[e] = y.x; x[e + 1] = y.y;
  }
}

// ------------------------------------------------------------------------------ reductions
__device__ __forceinline__ float hq_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float hq_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ------------------------------------------------------------------------------ dropout RNG
// key = fmix32(seed ^ opid*0x9E3779B9) is computed on the host (hq_op_key) once per op.
__host__ __device__ __forceinline__ uint32_t hq_fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16; return h;
}
__host__ __device__ __forceinline__ uint32_t hq_op_key(uint32_t seed, uint32_t opid) {
  return hq_fmix32(seed ^ (opid * 0x9E3779B9u));
}
// Dropout stream of one op, passed by value to the kernels: the host-derived key, or — when a device seed
// word is registered (hq_set_dropout_seed_ptr: captured HIP graphs, whose replays must draw new masks
// without re-launching from the host) — the key derived in-kernel from *seedp.
struct HqDropKey {
  uint32_t key;
  uint32_t opid;
  const uint32_t* seedp;
  __device__ __forceinline__ uint32_t get() const { return seedp ? hq_op_key(*seedp, opid) : key; }
};
static inline uint32_t hq_threshold(float p) { return (uint32_t)__builtin_rintf(p * 65536.0f); }
static inline float hq_keep_scale(uint32_t thr) { return thr < 65536u ? 65536.0f / (float)(65536u - thr) : 0.f; }

// 32-bit hash covering the element pair (2i, 2i+1).  Built from full-rate v_mul_u32_u24 instead of
// fmix32's quarter-rate 32-bit multiplies (9 full-rate VALU per pair instead of ~18 slot-equivalents):
// the first xorshift folds the high byte into the low 24 bits before each 24-bit multiply.  Avalanche
// 0.4996-0.5003 per input bit, no detectable pair/stride correlation (ops/rng.py documents the test).
// hq_mix24 after its first xorshift.  For c < 2^16, hq_mix24(x ^ c) == hq_mix24_post((x ^ (x >> 16)) ^ c):
// a loop hashing x ^ c for several small c does the first xorshift once.
__device__ __forceinline__ uint32_t hq_mix24_post(uint32_t x) {
  x = __umul24(x, 0x9E3779u);
  x ^= x >> 15;
  x = __umul24(x, 0xC2B2AEu);
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hq_mix24(uint32_t x) {  // x = pair_index ^ key
  return hq_mix24_post(x ^ (x >> 16));
}
__device__ __forceinline__ uint32_t hq_pair_hash(uint32_t idx_even, uint32_t key) {
  uint32_t x = (idx_even >> 1) ^ key;
  x ^= x >> 16;
  x = __umul24(x, 0x9E3779u);
  x ^= x >> 15;
  x = __umul24(x, 0xC2B2AEu);
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool hq_keep(uint32_t idx, uint32_t key, uint32_t thr) {
  uint32_t h = hq_pair_hash(idx, key);
  uint32_t u = (h >> ((idx & 1u) * 16u)) & 0xFFFFu;
  return u >= thr;
}
// keep-multipliers (0 or scale) for 8 consecutive elements starting at an even index
__device__ __forceinline__ void hq_keep8(uint32_t idx0, uint32_t key, uint32_t thr, float scale, float* m) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t h = hq_pair_hash(idx0 + 2 * i, key);
    m[2 * i] = ((h & 0xFFFFu) >= thr) ? scale : 0.f;
    m[2 * i + 1] = ((h >> 16) >= thr) ? scale : 0.f;
  }
}

// GEMM epilogues: EPI_BDR dropout stream (unused by the other epilogues): key source, 16-bit keep threshold, keep scale
struct HqDropArg {
  HqDropKey kd;
  uint32_t thr;
  float ks;
};
// z = x·keep + r for 8 consecutive elements from flat index idx (even): ln_fwd's z, bit for bit
__device__ __forceinline__ uint4 hq_epi_bdr8(const uint4& piece, const uint4& r4, uint32_t idx, const HqDropArg& dr,
                                          uint32_t key) {
  float d[8], rr[8], m[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  hq_unpack8(piece, d);
  hq_unpack8(r4, rr);
  if (dr.thr) hq_keep8(idx, key, dr.thr, dr.ks, m);
#pragma unroll
  for (int e = 0; e < 8; ++e) d[e] = d[e] * m[e] + rr[e];
  return hq_pack8(d);
}

__device__ __forceinline__ void hq_keep4(uint32_t idx0, uint32_t key, uint32_t thr, float scale, float* m) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint32_t h = hq_pair_hash(idx0 + 2 * i, key);
    m[2 * i] = ((h & 0xFFFFu) >= thr) ? scale : 0.f;
    m[2 * i + 1] = ((h >> 16) >= thr) ? scale : 0.f;
  }
}

// ------------------------------------------------------------------------------ fp8 (OCP e4m3) delayed scaling
// 4-float state per quantisation site: slots 0-2 rotate as (this step's amax, next step's (cleared), last
// step's amax) by phase = step % 3; state[3] = the scale this step's e4m3 tensor was written with.
// s = margin·amax_prev / fmax (unit scale before the first amax exists), margin 2 for the e4m3 forward inputs
// and 64 for the e5m2 gradients: a gradient's amax moves by more than 2× from one step to the next (measured,
// profiles/r4_fp8_conv: 9 % of the gradient productions overflowed a 2× margin, by up to 37×), and e5m2's
// 30-binade exponent range affords the 5 binades that a 64× margin takes off its bottom.
constexpr float kHqFp8Max = 448.f;      // OCP e4m3 (forward activations / weights)
constexpr float kHqBf8Max = 57344.f;    // OCP e5m2 (backward activation gradients)

// --precision fp8: the FFN1 epilogue stores gelu'(pre) for the FFN2 dgrad as an 8-bit linear code over its exact
// range [−0.12890, 1.12890] (gelu'(∓√2)): q = rint((g − lo)·(1/step)) clamped to 0…255, g ≈ lo + q·step (absolute
// error ≤ step/2 = 0.0025).  The dgrad's product is quantised to e5m2 (relative error up to 12.5 %) right after,
// so bf16 precision on this operand bought nothing but 604 MB of extra traffic per FFN per step.
// (kHqGdLo, kHqGdStep: hq_kernels.h, shared with the host bindings)
__device__ __forceinline__ uint2 hq_gd_encode8(const float* g) {
  // q = (g − lo)/step as one FMA, then v_cvt_pk_u8_f32 (round to nearest, saturate to 0…255) packs it into its byte
  constexpr float inv = kHqGdInv, off = kHqGdOff;
  uint32_t w[2] = {0u, 0u};
#pragma unroll
  for (int e = 0; e < 8; ++e) w[e >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(fmaf(g[e], inv, off), e & 3, w[e >> 2]);
  return make_uint2(w[0], w[1]);
}
__device__ __forceinline__ void hq_gd_decode8(const uint2& c, float* g) {
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = fmaf((float)(((e < 4 ? c.x : c.y) >> (8 * (e & 3))) & 0xFFu), kHqGdStep, kHqGdLo);
}
constexpr float kHqFp8Margin = 2.f;
constexpr float kHqBf8Margin = 64.f;
__device__ __forceinline__ float hq_fp8_delayed_scale(const float* st, int phase, float fmax = kHqFp8Max) {
  const float prev = __uint_as_float(reinterpret_cast<const unsigned*>(st)[(phase + 2) % 3]);
  const float margin = fmax == kHqBf8Max ? kHqBf8Margin : kHqFp8Margin;
  return prev > 0.f ? prev * margin / fmax : 1.f;
}
// A producer publishes the dequant scale of its own fp8 output (state[3]) itself — one thread of block 0, at its
// start — so that its amax fold (hq_fp8_amax_fold) may run later, batched with the other sites' folds
// (hq_fp8_fold_defer); the fold writes the same value again.  Nothing in the producer reads state[3].
__device__ __forceinline__ void hq_fp8_publish_scale(const float* st, int phase, float fmax = kHqFp8Max) {
  if ((blockIdx.x | blockIdx.y | threadIdx.x) == 0) const_cast<float*>(st)[3] = hq_fp8_delayed_scale(st, phase, fmax);
}
// 4 values -> 4 e5m2 bytes (x·inv, saturated to ±57344)
__device__ __forceinline__ uint32_t hq_pack_bf8x4(const float* f, float inv) {
  float g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = fminf(fmaxf(f[i] * inv, -kHqBf8Max), kHqBf8Max);
  uint32_t w = __builtin_amdgcn_cvt_pk_bf8_f32(g[0], g[1], 0, false);
  return __builtin_amdgcn_cvt_pk_bf8_f32(g[2], g[3], w, true);
}
// 4 values -> 4 e4m3 bytes (x·inv, saturated to ±448)
__device__ __forceinline__ uint32_t hq_pack_fp8x4(const float* f, float inv) {
  float g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = fminf(fmaxf(f[i] * inv, -kHqFp8Max), kHqFp8Max);
  uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(g[0], g[1], 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(g[2], g[3], w, true);
}

// Device-side assertions for the debug build only (`python -m ...csrc.build --debug` defines
// HQ_DEBUG); the release build compiles them to nothing.  A failing assertion prints its site and
// traps, so the faulting kernel is named by the runtime instead of corrupting memory silently.
#ifdef HQ_DEBUG
#define HQ_DASSERT(cond)                                                                       \
  do {                                                                                         \
    if (!(cond)) {                                                                             \
      printf("HQ_DASSERT %s:%d block (%d,%d) thread %d: %s\n", __FILE__, __LINE__, (int)blockIdx.x, \
             (int)blockIdx.y, (int)threadIdx.x, #cond);                                        \
      __builtin_trap();                                                                        \
    }                                                                                          \
  } while (0)
#else
#define HQ_DASSERT(cond) ((void)0)
#endif

#define HQ_CHECK(x)                                                                       \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      abort();                                                                            \
    }                                                                                     \
  } while (0)
