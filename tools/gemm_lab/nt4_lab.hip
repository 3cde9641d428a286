// GEMM lab: the production NT GEMM (gemm.hip: nt2 / nt3 / vS picked by hq_gemm_nt) against the
// two-workgroups-per-CU nt4 variants on the BERT-base b256 projection shapes, with their real epilogues,
// random bf16 operands.  Checks every variant against the production output, then times interleaved
// rounds in one process (median; cdna_hip_programming.md §5.4 rule 24).  Build + run:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I ml_recipe_distributed_pytorch_amd/csrc/include \
//         tools/gemm_lab/nt4_lab.hip -o tools/gemm_lab/nt4_lab && tools/gemm_lab/nt4_lab [M]
#include "../../ml_recipe_distributed_pytorch_amd/csrc/kernels/gemm.hip"
#include "nt4_kernel.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

__global__ void fill_rand(uint16_t* p, size_t n, uint32_t seed, float scale) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    float f = ((h & 0xFFFFFF) / 8388608.0f - 1.0f) * scale;
    p[i] = hq_f2bf(f);
  }
}
__global__ void fill_randf(float* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = ((h & 0xFFFF) / 32768.0f - 1.0f) * 0.1f;
  }
}

HqDropKey hq_drop_key(uint32_t seed, uint32_t opid) { return HqDropKey{hq_op_key(seed, opid), opid, nullptr}; }

static std::vector<float> to_host_bf16(const uint16_t* d, size_t n) {
  std::vector<uint16_t> h(n);
  CK(hipMemcpy(h.data(), d, n * 2, hipMemcpyDeviceToHost));
  std::vector<float> f(n);
  for (size_t i = 0; i < n; ++i) { uint32_t u = (uint32_t)h[i] << 16; memcpy(&f[i], &u, 4); }
  return f;
}
static double max_rel(const std::vector<float>& a, const std::vector<float>& b) {
  double md = 0, mr = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    md = std::max(md, (double)std::fabs(a[i] - b[i]));
    mr = std::max(mr, (double)std::fabs(b[i]));
  }
  return md / (mr > 0 ? mr : 1);
}

struct Case { const char* name; int N, K, epi; };

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 98304;
  const Case cases[] = {
      {"qkv_fwd+bias", 2304, 768, HQ_EPI_BIAS},   {"out_fwd+bias", 768, 768, HQ_EPI_BIAS},
      {"ffn1_fwd+geluD", 3072, 768, HQ_EPI_GELUD}, {"ffn2_fwd+bias", 768, 3072, HQ_EPI_BIAS},
      {"ffn2_dgrad*D", 3072, 768, HQ_EPI_DMUL},    {"ffn1_dgrad", 768, 3072, HQ_EPI_NONE},
      {"out_dgrad", 768, 768, HQ_EPI_NONE},        {"qkv_dgrad+res", 768, 2304, HQ_EPI_RESID},
  };
  const size_t maxMK = (size_t)M * 3072, maxNK = (size_t)3072 * 3072, maxMN = (size_t)M * 3072;
  uint16_t *A, *B, *C, *P, *R, *C2, *P2;
  float *bias, *part, *part2;
  CK(hipMalloc(&A, maxMK * 2)); CK(hipMalloc(&B, maxNK * 2));
  CK(hipMalloc(&C, maxMN * 2)); CK(hipMalloc(&C2, maxMN * 2));
  CK(hipMalloc(&P, maxMN * 2)); CK(hipMalloc(&P2, maxMN * 2)); CK(hipMalloc(&R, maxMN * 2));
  CK(hipMalloc(&bias, 3072 * 4)); CK(hipMalloc(&part, (size_t)(M / 64 + 8) * 3072 * 4));
  CK(hipMalloc(&part2, (size_t)(M / 64 + 8) * 3072 * 4));
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, A, maxMK, 1u, 1.0f);
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, B, maxNK, 2u, 0.05f);
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, R, maxMN, 3u, 1.0f);
  hipLaunchKernelGGL(fill_randf, dim3(16), dim3(256), 0, 0, bias, (size_t)3072, 4u);
  CK(hipDeviceSynchronize());
  const HqDropArg dr{hq_drop_key(1, 1), 0u, 1.f};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));

  for (const Case& c : cases) {
    const int N = c.N, K = c.K, epi = c.epi;
    const bool auxP = epi == HQ_EPI_DMUL;
    // DMUL reads P (the stored gelu'): give it random values in both runs
    if (auxP) {
      hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, P, (size_t)M * N, 5u, 1.0f);
      CK(hipMemcpy(P2, P, (size_t)M * N * 2, hipMemcpyDeviceToDevice));
    }
    struct V { std::string name; std::function<void(uint16_t*, uint16_t*, float*)> run; int bm; };
    std::vector<V> vs;
    const int bn_prod = hq_gemm_nt_supported(M, N, K);
    vs.push_back({"prod", [&](uint16_t* Co, uint16_t* Po, float* pa) {
                    hq_gemm_nt(A, B, Co, bias, Po, R, pa, M, N, K, K, K, N, epi, bn_prod, 0, 0.f, 0, 0);
                  }, bn_prod == 1 ? 128 : 256});
    const char* fam_names[2] = {"nt4 192² m32", "nt4 192² m16"};
    for (int f = 0; f < 2; ++f) {
      const int bm = hq_gemm_nt4_bm(f, N);
      if (!bm) continue;
      for (int st : {0, 1, 2}) {   // stagger in units of s_sleep(127) (~3.9 us)
        std::string nm = std::string(fam_names[f]) + " st" + std::to_string(st);
        vs.push_back({nm, [&, f, epi, st](uint16_t* Co, uint16_t* Po, float* pa) {
                        hq_gemm_nt4_set_stagger(st);
                        hq_gemm_nt4(f, A, B, Co, bias, Po, R, pa, M, N, K, K, K, N, epi, 0, dr);
                      }, bm});
        if (epi == HQ_EPI_GELUD)
          vs.push_back({nm + " fastgelu", [&, f, st](uint16_t* Co, uint16_t* Po, float* pa) {
                          hq_gemm_nt4_set_stagger(st);
                          hq_gemm_nt4(f, A, B, Co, bias, Po, R, pa, M, N, K, K, K, N, 8, 0, dr);
                        }, bm});
      }
    }

    // correctness vs prod
    vs[0].run(C, P, part);
    CK(hipDeviceSynchronize());
    std::vector<float> cref = to_host_bf16(C, (size_t)M * N), pref;
    if (epi == HQ_EPI_GELUD) pref = to_host_bf16(P, (size_t)M * N);
    std::vector<float> colref;
    auto colsum = [&](float* pa, int bm) {
      const int rows = (M + bm - 1) / bm;
      std::vector<float> h((size_t)rows * N), s(N, 0.f);
      CK(hipMemcpy(h.data(), pa, h.size() * 4, hipMemcpyDeviceToHost));
      for (int r = 0; r < rows; ++r)
        for (int n = 0; n < N; ++n) s[n] += h[(size_t)r * N + n];
      return s;
    };
    if (auxP) colref = colsum(part, vs[0].bm);
    for (size_t v = 1; v < vs.size(); ++v) {
      CK(hipMemset(C2, 0, (size_t)M * N * 2));
      vs[v].run(C2, P2, part2);
      CK(hipDeviceSynchronize());
      double ec = max_rel(to_host_bf16(C2, (size_t)M * N), cref);
      double ep = epi == HQ_EPI_GELUD ? max_rel(to_host_bf16(P2, (size_t)M * N), pref) : 0.0;
      double es = 0;
      if (auxP) {
        std::vector<float> s = colsum(part2, vs[v].bm);
        double md = 0, mr = 0;
        for (int n = 0; n < N; ++n) { md = std::max(md, (double)std::fabs(s[n] - colref[n])); mr = std::max(mr, (double)std::fabs(colref[n])); }
        es = md / mr;
      }
      printf("check %-16s %-16s C %.2e P %.2e colsum %.2e %s\n", c.name, vs[v].name.c_str(), ec, ep, es,
             (ec < 2e-2 && ep < 2e-2 && es < 2e-3) ? "ok" : "MISMATCH");
    }
    // timing
    std::vector<std::vector<float>> t(vs.size());
    const int iters = 8;
    for (int round = 0; round < 5; ++round)
      for (size_t v = 0; v < vs.size(); ++v) {
        vs[v].run(C2, P2, part2);
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) vs[v].run(C2, P2, part2);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1000.f / iters);
      }
    for (size_t v = 0; v < vs.size(); ++v) {
      std::sort(t[v].begin(), t[v].end());
      const float us = t[v][2];
      printf("time  %-16s M=%d N=%d K=%d %-16s %8.1f us %7.1f TF/s (min %.1f)\n", c.name, M, N, K, vs[v].name.c_str(), us,
             2.0 * M * N * K / us / 1e6, t[v][0]);
    }
    fflush(stdout);
  }
  return 0;
}
