// Fused optimizer kernels over the flat fp32 parameter / gradient arenas (gfx950).
//
// Replaces the reference's per-parameter optimizer + clip_grad_norm_ (≈8 elementwise kernels ×
// 199 params + 199 norm kernels) with:
//   hq_sq_norm_partials : one grid-stride pass over the whole grad arena (float4), per-block Σg²
//   hq_clip_coef        : single block, deterministic sum → ‖g‖ and min(1, max_norm/(‖g‖+1e-6)) ON DEVICE
//   hq_adamw / hq_adamod: one block per ≤8192-element chunk of a parameter segment; reads the
//                         clip coefficient from device memory (no host sync), updates m, v (, n),
//                         the fp32 master and writes the bf16 working copy in the same pass.
// HF AdamW semantics (reference init.py:137, correct_bias=False): decay applied AFTER the update.
// AdaMod semantics (reference modules/model/trainer/optim.py:76-98): decay BEFORE the update.
#include "hq_common.h"
#include "hq_kernels.h"

namespace {

__global__ __launch_bounds__(256) void sq_norm_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ partials) {
  __shared__ float red[4];
  float s = 0.f;
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) s += g[i] * g[i];
  s = hq_wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Σg² of one chunk of the grad arena per block: chunk c = [chunks[2c], +chunks[2c+1]) (starts 16-B aligned, sizes % 4 == 0,
// <= kNormChunk floats).  The chunk table cuts every readiness group of the arena into pieces, so a group's partials
// are the same numbers whether the full pass writes them after the backward or the gradient reducer's comm stream
// writes them right after that group's bucket all-reduce — the clip coefficient is bitwise the same either way.
__global__ __launch_bounds__(256) void sq_norm_chunks_kernel(const float* __restrict__ g, const int64_t* __restrict__ chunks,
                                                             int c0, float* __restrict__ partials) {
  __shared__ float red[4];
  const int c = c0 + blockIdx.x;
  const float4* p = reinterpret_cast<const float4*>(g + chunks[2 * c]);
  const int n4 = (int)(chunks[2 * c + 1] / 4);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = threadIdx.x;
  for (; i + 3 * 256 < n4; i += 4 * 256) {   // four independent loads in flight per thread
    const float4 a = p[i], b = p[i + 256], d = p[i + 512], e = p[i + 768];
    s0 += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
    s1 += b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w;
    s2 += d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
    s3 += e.x * e.x + e.y * e.y + e.z * e.z + e.w * e.w;
  }
  for (; i < n4; i += 256) {
    const float4 a = p[i];
    s0 += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
  }
  float s = hq_wave_sum((s0 + s1) + (s2 + s3));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[c] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void clip_coef_kernel(const float* __restrict__ partials, int nparts, float max_norm,
                                                        float* __restrict__ norm_out, float* __restrict__ coef_out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += partials[i];
  s = hq_wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]);
    norm_out[0] = norm;
    if (coef_out) coef_out[0] = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
  }
}

struct AdamWArgs {
  float beta1, beta2, eps, step_mult;
};

__device__ __forceinline__ void adamw_elem(float& p, float& m, float& v, float g, float lr, float wd, const AdamWArgs& a) {
  m = a.beta1 * m + (1.f - a.beta1) * g;
  v = a.beta2 * v + (1.f - a.beta2) * g * g;
  const float denom = sqrtf(v) + a.eps;
  p = p - (lr * a.step_mult) * (m / denom);
  if (wd > 0.f) p = p - (lr * wd) * p;
}

__device__ __forceinline__ void st_nt4(float* dst, const float4& v) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w}, reinterpret_cast<f4*>(dst));
}
__device__ __forceinline__ float4 ld_nt4(const float* src) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt2(uint16_t* dst, const uint2& v) {
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(u2{v.x, v.y}, reinterpret_cast<u2*>(dst));
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ master, uint16_t* __restrict__ compute,
                                                    const float* __restrict__ grad, float* __restrict__ exp_avg,
                                                    float* __restrict__ exp_avg_sq, const HqOptChunk* __restrict__ chunks,
                                                    HqOptGroups groups, AdamWArgs a, const float* __restrict__ clip) {
  const HqOptChunk c = chunks[blockIdx.x];
  const float lr = groups.lr[c.group], wd = groups.wd[c.group];
  const float cc = clip ? clip[0] : 1.f;
  const int64_t s0 = c.start;
  if ((s0 & 3) == 0) {
    const int n4 = c.numel / 4;
    // two float4 of each stream per thread per iteration, all eight loads issued before any math: the loop is
    // HBM-bound (16 B read ×4 + written ×3 + 8 B bf16 per 4 elements) and one quartet in flight per lane leaves
    // the memory pipe under-filled between iterations
    auto step4 = [&](int64_t o, float4& p, float4& m, float4& v, const float4& g) {
      adamw_elem(p.x, m.x, v.x, g.x * cc, lr, wd, a);
      adamw_elem(p.y, m.y, v.y, g.y * cc, lr, wd, a);
      adamw_elem(p.z, m.z, v.z, g.z * cc, lr, wd, a);
      adamw_elem(p.w, m.w, v.w, g.w * cc, lr, wd, a);
      // streaming (non-temporal) loads and stores: every state word is read and written once per step, so
      // nothing is gained by allocating it in L2
      st_nt4(master + o, p);
      st_nt4(exp_avg + o, m);
      st_nt4(exp_avg_sq + o, v);
      if (compute) {
        const float pf[4] = {p.x, p.y, p.z, p.w};
        st_nt2(compute + o, hq_pack4(pf));
      }
    };
    int i = threadIdx.x;
    for (; i + 256 < n4; i += 512) {
      const int64_t o0 = s0 + 4 * (int64_t)i, o1 = o0 + 4 * 256;
      float4 p0 = ld_nt4(master + o0), p1 = ld_nt4(master + o1);
      float4 m0 = ld_nt4(exp_avg + o0), m1 = ld_nt4(exp_avg + o1);
      float4 v0 = ld_nt4(exp_avg_sq + o0), v1 = ld_nt4(exp_avg_sq + o1);
      const float4 g0 = ld_nt4(grad + o0), g1 = ld_nt4(grad + o1);
      step4(o0, p0, m0, v0, g0);
      step4(o1, p1, m1, v1, g1);
    }
    for (; i < n4; i += 256) {
      const int64_t o = s0 + 4 * (int64_t)i;
      float4 p = *reinterpret_cast<float4*>(master + o);
      float4 m = *reinterpret_cast<float4*>(exp_avg + o);
      float4 v = *reinterpret_cast<float4*>(exp_avg_sq + o);
      const float4 g = *reinterpret_cast<const float4*>(grad + o);
      step4(o, p, m, v, g);
    }
    for (int i = n4 * 4 + threadIdx.x; i < c.numel; i += 256) {
      const int64_t o = s0 + i;
      adamw_elem(master[o], exp_avg[o], exp_avg_sq[o], grad[o] * cc, lr, wd, a);
      if (compute) compute[o] = hq_f2bf(master[o]);
    }
  } else {
    for (int i = threadIdx.x; i < c.numel; i += 256) {
      const int64_t o = s0 + i;
      adamw_elem(master[o], exp_avg[o], exp_avg_sq[o], grad[o] * cc, lr, wd, a);
      if (compute) compute[o] = hq_f2bf(master[o]);
    }
  }
}

struct AdaModArgs {
  float beta1, beta2, beta3, eps, base;  // base = bias-corrected step-size factor (times lr per group)
};

__global__ __launch_bounds__(256) void adamod_kernel(float* __restrict__ master, uint16_t* __restrict__ compute,
                                                     const float* __restrict__ grad, float* __restrict__ exp_avg,
                                                     float* __restrict__ exp_avg_sq, float* __restrict__ exp_avg_lr,
                                                     const HqOptChunk* __restrict__ chunks, HqOptGroups groups, AdaModArgs a,
                                                     const float* __restrict__ clip) {
  const HqOptChunk c = chunks[blockIdx.x];
  const float lr = groups.lr[c.group], wd = groups.wd[c.group];
  const float cc = clip ? clip[0] : 1.f;
  for (int i = threadIdx.x; i < c.numel; i += 256) {
    const int64_t o = c.start + i;
    const float g = grad[o] * cc;
    float m = a.beta1 * exp_avg[o] + (1.f - a.beta1) * g;
    float v = a.beta2 * exp_avg_sq[o] + (1.f - a.beta2) * g * g;
    const float denom = sqrtf(v) + a.eps;
    float p = master[o];
    if (wd != 0.f) p = p - (wd * lr) * p;
    float ss = (lr * a.base) / denom;
    const float n = a.beta3 * exp_avg_lr[o] + (1.f - a.beta3) * ss;
    ss = fminf(ss, n) * m;
    p = p - ss;
    exp_avg[o] = m;
    exp_avg_sq[o] = v;
    exp_avg_lr[o] = n;
    master[o] = p;
    if (compute) compute[o] = hq_f2bf(p);
  }
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                            int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(src)[i];
    const float f[4] = {v.x * scale, v.y * scale, v.z * scale, v.w * scale};
    reinterpret_cast<uint2*>(dst)[i] = hq_pack4(f);
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) dst[i] = hq_f2bf(src[i] * scale);
}

__global__ __launch_bounds__(256) void cast_bf16_f32_kernel(const uint16_t* __restrict__ src, float* __restrict__ dst,
                                                            int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float f[4];
    hq_unpack4(reinterpret_cast<const uint2*>(src)[i], f);
    reinterpret_cast<float4*>(dst)[i] = make_float4(f[0] * scale, f[1] * scale, f[2] * scale, f[3] * scale);
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) dst[i] = hq_bf2f(src[i]) * scale;
}

// Exact replica fingerprint of an fp32 arena: part p covers [p·n/P, (p+1)·n/P) and holds
//   Σ_i bits(x_i) · (2i + 1)   (mod 2^64, i = global element index)
// — integer wrap-around adds are associative, so the value does not depend on the summation order and equals the
// host-side numpy fingerprint (parallel/reducer.py) bit for bit.  Any flipped bit, sign, or swapped pair of words
// changes it.  Used after the timed region only (bench / trainer cross-rank weight equality check).
__global__ __launch_bounds__(256) void fingerprint_kernel(const uint32_t* __restrict__ x, int64_t n, int nparts,
                                                          uint64_t* __restrict__ out) {
  __shared__ uint64_t red[256];
  const int64_t lo = n * blockIdx.x / nparts, hi = n * (blockIdx.x + 1) / nparts;
  HQ_DASSERT(lo <= hi && hi <= n);
  uint64_t s = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) s += (uint64_t)x[i] * (2ull * (uint64_t)i + 1ull);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

int grid_for(int64_t n4) { return (int)std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 2048)); }

}  // namespace

void hq_fingerprint(const float* x, int64_t n, int nparts, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(fingerprint_kernel, dim3(nparts), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(x), n, nparts,
                     out);
}

void hq_sq_norm_partials(const float* g, int64_t n, float* partials, int nparts, hipStream_t s) {
  hipLaunchKernelGGL(sq_norm_kernel, dim3(nparts), dim3(256), 0, s, g, n, partials);
}

void hq_sq_norm_chunks(const float* g, const int64_t* chunks, int c0, int c1, float* partials, hipStream_t s) {
  if (c1 > c0) hipLaunchKernelGGL(sq_norm_chunks_kernel, dim3(c1 - c0), dim3(256), 0, s, g, chunks, c0, partials);
}

void hq_clip_coef(const float* partials, int nparts, float max_norm, float* norm_out, float* coef_out, hipStream_t s) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, s, partials, nparts, max_norm, norm_out, coef_out);
}

void hq_adamw(float* master, uint16_t* compute, const float* grad, float* m, float* v, const HqOptChunk* chunks, int nchunks,
              HqOptGroups groups, float beta1, float beta2, float eps, float step_size_mult, const float* clip_coef,
              hipStream_t s) {
  AdamWArgs a{beta1, beta2, eps, step_size_mult};
  hipLaunchKernelGGL(adamw_kernel, dim3(nchunks), dim3(256), 0, s, master, compute, grad, m, v, chunks, groups, a, clip_coef);
}

void hq_adamod(float* master, uint16_t* compute, const float* grad, float* m, float* v, float* n, const HqOptChunk* chunks,
               int nchunks, HqOptGroups groups, float beta1, float beta2, float beta3, float eps, float bias_corr,
               const float* clip_coef, hipStream_t s) {
  AdaModArgs a{beta1, beta2, beta3, eps, bias_corr};
  hipLaunchKernelGGL(adamod_kernel, dim3(nchunks), dim3(256), 0, s, master, compute, grad, m, v, n, chunks, groups, a,
                     clip_coef);
}

void hq_cast_f32_bf16(const float* src, uint16_t* dst, int64_t n, float scale, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n / 4)), dim3(256), 0, s, src, dst, n, scale);
}

void hq_cast_bf16_f32(const uint16_t* src, float* dst, int64_t n, float scale, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n / 4)), dim3(256), 0, s, src, dst, n, scale);
}
