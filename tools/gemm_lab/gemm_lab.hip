// Standalone GEMM lab: times the production NT kernels and ablated v2 builds on random bf16
// operands (interleaved rounds in one process, median).  Build + run:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I ml_recipe_distributed_pytorch_amd/csrc/include \
//         tools/gemm_lab/gemm_lab.hip -o tools/gemm_lab/gemm_lab && tools/gemm_lab/gemm_lab
#include "../../ml_recipe_distributed_pytorch_amd/csrc/kernels/gemm.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

__global__ void fill_rand(uint16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    float f = (h & 0xFFFFFF) / 8388608.0f - 1.0f;
    p[i] = hq_f2bf(f);
  }
}

HqDropKey hq_drop_key(uint32_t seed, uint32_t opid) { return HqDropKey{hq_op_key(seed, opid), opid, nullptr}; }

typedef void (*Kern)(const uint16_t*, const uint16_t*, uint16_t*, const float*, uint16_t*, const uint16_t*, float*, int,
                     int, int, int, int, int, HqDropArg);

struct Variant { const char* name; Kern k; };

int main(int argc, char** argv) {
  const int shapes[][3] = {{98304, 768, 3072}, {98304, 3072, 768}, {98304, 2304, 768}, {8192, 8192, 8192}};
  Variant vs[] = {
      {"v1", (Kern)gemm_nt_kernel<0, 256>},
      {"v2-glds", (Kern)gemm_nt2_kernel<0, 0>},
      {"v2 (prod)", (Kern)gemm_nt2_kernel<0, 8>},
      {"v2-noload", (Kern)gemm_nt2_kernel<0, 1>},
      {"v2-noread", (Kern)gemm_nt2_kernel<0, 2>},
      {"v2-noload-noread", (Kern)gemm_nt2_kernel<0, 3>},
      {"v2-lockstep", (Kern)gemm_nt2_kernel<0, 4>},
      {"v2-buf", (Kern)gemm_nt2_kernel<0, 8>},
      {"v2-group", (Kern)gemm_nt2_kernel<0, 16>},
      {"v2-buf-group", (Kern)gemm_nt2_kernel<0, 24>},
      {"v2-buf-noread", (Kern)gemm_nt2_kernel<0, 10>},
  };
  const int NV = sizeof(vs) / sizeof(vs[0]);
  const size_t lds = epi_lds(256);
  for (auto& v : vs) CK(hipFuncSetAttribute((const void*)v.k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    uint16_t *A, *B, *C;
    CK(hipMalloc(&A, (size_t)M * K * 2)); CK(hipMalloc(&B, (size_t)N * K * 2)); CK(hipMalloc(&C, (size_t)M * N * 2));
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, A, (size_t)M * K, 1u);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, B, (size_t)N * K, 2u);
    const int grid = (M / 256) * (N / 256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(NV);
    const int iters = 10;
    for (int round = 0; round < 5; ++round)
      for (int v = 0; v < NV; ++v) {
        hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(512), lds, 0, A, B, C, nullptr, nullptr, nullptr, nullptr, M, N, K, K, K, N, HqDropArg{});
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i)
          hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(512), lds, 0, A, B, C, nullptr, nullptr, nullptr, nullptr, M, N, K, K, K, N, HqDropArg{});
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1000.f / iters);
      }
    for (int v = 0; v < NV; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const float us = t[v][2];
      printf("M=%d N=%d K=%d %-18s %9.1f us %7.1f TF/s\n", M, N, K, vs[v].name, us, 2.0 * M * N * K / us / 1e6);
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C));
  }
  return 0;
}
