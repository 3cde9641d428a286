// GEMM lab: a 4-wave, one-wave-per-SIMD NT mainloop (each wave owns 128×128 of a 256² tile, its
// accumulators in the AGPR half of a 512-register budget) against the production v3 kernel.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I ml_recipe_distributed_pytorch_amd/csrc/include \
//         tools/gemm_lab/nt5_lab.hip -o tools/gemm_lab/nt5_lab && tools/gemm_lab/nt5_lab
#include "../../ml_recipe_distributed_pytorch_amd/csrc/kernels/gemm.hip"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

namespace {

// BK = 32 K-steps, NST-deep LDS ring of [256 rows × 64 B] A and B panels (32 KiB per step).
// 64-B rows: the 16 lanes of a fragment read (16 rows, one 16-B slot) hit all 64 banks once under
// slot' = slot ^ ((row >> 2) & 3) (4 rows share a 256-B bank row).
__device__ __forceinline__ bf16x8_t frag64(const char* panel, int row, int slot) {
  return *reinterpret_cast<const bf16x8_t*>(panel + row * 64 + ((slot ^ ((row >> 2) & 3)) << 4));
}

// s_waitcnt immediate (gfx9 encoding) as a builtin, so hipcc's waitcnt pass sees the wait (an inline-asm
// wait is opaque to it: it then re-waits before the next step's MFMAs on reads it thinks still in flight)
constexpr int wcnt(int vm, int lgkm) { return (vm & 0xF) | ((vm >> 4) << 14) | (7 << 4) | ((lgkm & 0xF) << 8); }

// SCHED: 0 = compiler order, 1 = sched_group_barrier interleave (1 ds_read per 4 MFMAs, 1 DMA per 8)
template <int NST, int SCHED, int MF = 16>
__global__ __launch_bounds__(256, 1) void nt5_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                     uint16_t* __restrict__ C, int M, int N, int K) {
  constexpr int BK5 = 32;
  constexpr int PANEL = 256 * 64;
  constexpr int STG = 2 * PANEL;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_n = N / 256;
  const int m0 = (tile / tiles_n) * 256, n0 = (tile % tiles_n) * 256;
  const int nk = K / BK5;

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * K), (short)0, 256 * K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (size_t)n0 * K), (short)0, 256 * K * 2, 0x00020000);
  // wave w stages rows w·64 … w·64+63 of each panel: 4 instructions of 16 rows (lane L → row L/4, slot L%4)
  int vo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 64 + i * 16 + (lane >> 2);
    const int src_slot = (lane & 3) ^ ((row >> 2) & 3);
    vo[i] = (row * K + src_slot * 8) * 2;
  }
  auto stage = [&](int t) {
    char* pa = smem + (t % NST) * STG + wave_u * 64 * 64;
    const int so = t * BK5 * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(pa + i * 1024), 16, vo[i], so, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(pa + PANEL + i * 1024), 16, vo[i], so, 0, 0);
  };

  f32x4_t acc[8][8];
  f32x16_t acc32[4][4];
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc32[i][j] = f32x16_t{};
  }
  const int fr = lane & 15, fq = lane >> 4;
  const int r32 = lane & 31, h32 = lane >> 5;
  // MF 16: fragment i = 16-row block i; MF 32: fragment ks·4 + i = 32-row block i, k16 step ks
  bf16x8_t fa[2][8], fb[2][8];
  auto rd = [&](int t, int set) {
    const char* pa = smem + (t % NST) * STG;
    if constexpr (MF == 16) {
#pragma unroll
      for (int i = 0; i < 8; ++i) fb[set][i] = frag64(pa + PANEL, wn * 128 + i * 16 + fr, fq);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[set][i] = frag64(pa, wm * 128 + i * 16 + fr, fq);
    } else {
#pragma unroll
      for (int f = 0; f < 8; ++f) fb[set][f] = frag64(pa + PANEL, wn * 128 + (f & 3) * 32 + r32, (f >> 2) * 2 + h32);
#pragma unroll
      for (int f = 0; f < 8; ++f) fa[set][f] = frag64(pa, wm * 128 + (f & 3) * 32 + r32, (f >> 2) * 2 + h32);
    }
  };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue: steps 0 … NST-2 in flight, retire 0 and 1
#pragma unroll
  for (int t = 0; t < NST - 1; ++t) stage(t);
  __builtin_amdgcn_s_waitcnt(wcnt((NST - 3) * 8, 15));
  bar();
  rd(0, 0);
  __builtin_amdgcn_s_waitcnt(wcnt(63, 0));

  // GEN: steady state (stage and read unconditionally, vmcnt(8·(NST-3))) or the tail (runtime conditions)
  auto step = [&](auto GEN, int s, auto CUR) {
    constexpr int cur = decltype(CUR)::value;
    constexpr bool gen = decltype(GEN)::value;
    const bool st = gen ? s + NST - 1 < nk : true;
    if (st) stage(s + NST - 1);
    if (!gen || s + 1 < nk) rd(s + 1, cur ^ 1);
    if constexpr (MF == 16) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][j], fa[cur][i], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[cur][ks * 4 + j], fa[cur][ks * 4 + i], acc32[i][j], 0, 0, 0);
    }
    if constexpr (SCHED == 1) {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM (LDS-DMA)
        __builtin_amdgcn_sched_group_barrier(0x008, MF == 16 ? 4 : 2, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, MF == 16 ? 4 : 2, 0);   // MFMA
      }
    }
    if constexpr (!gen) {
      __builtin_amdgcn_s_waitcnt(wcnt((NST - 3) * 8, 0));
    } else {
      __builtin_amdgcn_s_waitcnt(wcnt(63, 0));
      if (s + 2 < nk) __builtin_amdgcn_s_waitcnt(wcnt(0, 15));   // tail: drain (tile s+2 is the last one staged)
    }
    bar();
  };
  using T0 = std::integral_constant<int, 0>;
  using T1 = std::integral_constant<int, 1>;
  using G0 = std::integral_constant<bool, false>;
  using G1 = std::integral_constant<bool, true>;
  int s = 0;
  for (; s + NST < nk; s += 2) {   // both steps of the pair stage a tile
    step(G0{}, s, T0{});
    step(G0{}, s + 1, T1{});
  }
  for (; s + 1 < nk; s += 2) {
    step(G1{}, s, T0{});
    step(G1{}, s + 1, T1{});
  }
  if (s < nk) step(G1{}, s, T0{});

  // lab epilogue: straight from the accumulators (lane: row m, 4 consecutive n)
  if constexpr (MF == 32) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x16_t& a = acc32[i][j];
          float v[4] = {a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]};
          *reinterpret_cast<uint2*>(C + (size_t)(m0 + wm * 128 + i * 32 + r32) * N + n0 + wn * 128 + j * 32 + g * 8 + h32 * 4) =
              hq_pack4(v);
        }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4_t& a = acc[i][j];
      float v[4] = {a[0], a[1], a[2], a[3]};
      *reinterpret_cast<uint2*>(C + (size_t)(m0 + wm * 128 + i * 16 + fr) * N + n0 + wn * 128 + j * 16 + fq * 4) = hq_pack4(v);
    }
}

__global__ void fill_rand(uint16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = hq_f2bf((h & 0xFFFFFF) / 8388608.0f - 1.0f);
  }
}

}  // namespace

HqDropKey hq_drop_key(uint32_t seed, uint32_t opid) { return HqDropKey{hq_op_key(seed, opid), opid, nullptr}; }

static float bf2f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }

int main() {
  const int shapes[][3] = {{98304, 2304, 768}, {98304, 768, 768}, {98304, 3072, 768}, {98304, 768, 3072}, {98304, 768, 2304}};
  constexpr size_t lds3 = 2 * 2 * 256 * 128 + 64 * 144 + 2 * 256 * 4 + 16;
  CK(hipFuncSetAttribute((const void*)gemm_nt3_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds3));
  typedef void (*K5)(const uint16_t*, const uint16_t*, uint16_t*, int, int, int);
  struct V5 { const char* name; K5 k; int lds; };
  const V5 v5s[] = {{"16 ring4", nt5_kernel<4, 0, 16>, 4 * 32768}, {"16 ring4 sgb", nt5_kernel<4, 1, 16>, 4 * 32768},
                    {"16 ring5", nt5_kernel<5, 0, 16>, 5 * 32768}, {"32 ring4", nt5_kernel<4, 0, 32>, 4 * 32768},
                    {"32 ring4 sgb", nt5_kernel<4, 1, 32>, 4 * 32768}, {"32 ring5", nt5_kernel<5, 0, 32>, 5 * 32768},
                    {"32 ring5 sgb", nt5_kernel<5, 1, 32>, 5 * 32768}};
  constexpr int NV5 = sizeof(v5s) / sizeof(v5s[0]);
  for (auto& v : v5s) CK(hipFuncSetAttribute((const void*)v.k, hipFuncAttributeMaxDynamicSharedMemorySize, v.lds));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  HqDropArg dr{hq_drop_key(0, 0), 0u, 1.f};
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    uint16_t *A, *B, *C0, *C1;
    CK(hipMalloc(&A, (size_t)M * K * 2)); CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C0, (size_t)M * N * 2)); CK(hipMalloc(&C1, (size_t)M * N * 2));
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, A, (size_t)M * K, 1u);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, B, (size_t)N * K, 2u);
    const int grid = (M / 256) * (N / 256);
    auto v3 = [&](uint16_t* C) {
      hipLaunchKernelGGL((gemm_nt3_kernel<0>), dim3(std::min(grid, ncu)), dim3(512), lds3, 0, A, B, C, nullptr, nullptr,
                         nullptr, nullptr, M, N, K, K, K, N, 0, nullptr, dr);
    };
    auto v5 = [&](int w, uint16_t* C) {
      hipLaunchKernelGGL(v5s[w].k, dim3(grid), dim3(256), v5s[w].lds, 0, A, B, C, M, N, K);
    };
    // correctness: every nt5 form against v3 (same math, different accumulation order: bf16 rounding only)
    v3(C0);
    CK(hipDeviceSynchronize());
    std::vector<uint16_t> h0((size_t)M * N), h1((size_t)M * N);
    CK(hipMemcpy(h0.data(), C0, h0.size() * 2, hipMemcpyDeviceToHost));
    for (int w = 0; w < NV5; ++w) {
      CK(hipMemset(C1, 0, (size_t)M * N * 2));
      v5(w, C1);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h1.data(), C1, h1.size() * 2, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (size_t i = 0; i < h0.size(); i += 7) {
        md = std::max(md, (double)fabsf(bf2f(h0[i]) - bf2f(h1[i])));
        mx = std::max(mx, (double)fabsf(bf2f(h0[i])));
      }
      printf("M=%d N=%d K=%d %-14s max|diff| %.4g (max|C| %.4g)\n", M, N, K, v5s[w].name, md, mx);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(NV5 + 1);
    for (int round = 0; round < 7; ++round)
      for (int w = 0; w <= NV5; ++w) {
        CK(hipEventRecord(e0));
        for (int it = 0; it < 5; ++it) (w == 0 ? v3(C0) : v5(w - 1, C1));
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[w].push_back(ms * 1000 / 5);
      }
    for (int w = 0; w <= NV5; ++w) {
      std::sort(t[w].begin(), t[w].end());
      const float us = t[w][t[w].size() / 2];
      printf("M=%d N=%d K=%d %-14s %8.1f us  %.3f PF/s\n", M, N, K, w ? v5s[w - 1].name : "v3 (prod)", us, 2.0 * M * N * K / us / 1e9);
    }
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C0)); CK(hipFree(C1));
  }
  return 0;
}
