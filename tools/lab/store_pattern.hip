// Lab: store throughput of the GEMM epilogue's row-piece patterns (no mainloop).  A persistent grid of 8-wave
// workgroups writes a [M, N] bf16 matrix tile by tile (256 x 256 tiles, 16 x dwordx4 per wave per tile, as the
// persistent NT GEMM's epilogue issues them), with three lane -> (row, column) maps:
//   0  nt3: a wave owns two 32-column strips 128 columns apart; a store instruction = 8 rows x 2 x 64 B
//   1  line: a store instruction = 8 rows x one full 128-B line (8 lanes per row)
//   2  wide: a store instruction = 2 rows x 512 B (32 lanes per row: 4 consecutive lines)
// Usage: store_pattern [M N grid_wgs]  (default 98304 3072 256).  Prints GB/s per pattern (median of 7).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int PAT>
__global__ __launch_bounds__(512, 1) void store_tiles(uint16_t* __restrict__ C, int M, int N) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_n = N / 256, ntiles = (M / 256) * tiles_n;
  uint4 v = make_uint4(lane, wave, blockIdx.x, 0x3f803f80u);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int m0 = (t / tiles_n) * 256, n0 = (t % tiles_n) * 256;
    // each wave stores 128 rows x 64 columns = 16 KB = 16 instructions of 1 KB
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      int row, col;
      if (PAT == 0) {          // nt3: seg = lane % 8 -> (seg >> 2) * 128 + wn * 32 + (seg & 3) * 8; 8 rows per instr
        const int seg = lane & 7, rsub = lane >> 3;
        row = m0 + wm * 128 + it * 8 + rsub;
        col = n0 + (seg >> 2) * 128 + wn * 32 + (seg & 3) * 8;
      } else if (PAT == 1) {   // full 128-B lines: wave owns 64 contiguous columns, 8 lanes per row
        const int seg = lane & 7, rsub = lane >> 3;
        row = m0 + wm * 128 + it * 8 + rsub;
        col = n0 + wn * 64 + seg * 8;
      } else {                 // 512-B rows: the wave stores rows of 256 columns, 32 lanes per row
        const int seg = lane & 31, rsub = lane >> 5;
        row = m0 + wm * 128 + wn * 32 + it * 2 + rsub;
        col = n0 + seg * 8;
      }
      v.w += 1;
      *reinterpret_cast<uint4*>(C + (size_t)row * N + col) = v;
    }
  }
}

// retirement latency: each wave stores its 16 KB per tile (nt3 map), then waits vmcnt(0); the cycles that wait
// takes (s_memtime) are summed per workgroup into lat[blockIdx.x] (wave 0's view)
__global__ __launch_bounds__(512, 1) void store_tiles_lat(uint16_t* __restrict__ C, int M, int N,
                                                          unsigned long long* __restrict__ lat) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_n = N / 256, ntiles = (M / 256) * tiles_n;
  uint4 v = make_uint4(lane, wave, blockIdx.x, 0x3f803f80u);
  unsigned long long tot = 0;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int m0 = (t / tiles_n) * 256, n0 = (t % tiles_n) * 256;
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int seg = lane & 7, rsub = lane >> 3;
      const int row = m0 + wm * 128 + it * 8 + rsub;
      const int col = n0 + (seg >> 2) * 128 + wn * 32 + (seg & 3) * 8;
      v.w += 1;
      *reinterpret_cast<uint4*>(C + (size_t)row * N + col) = v;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tot += __builtin_amdgcn_s_memtime() - t0;
  }
  if (threadIdx.x == 0) lat[blockIdx.x] = tot;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 98304;
  const int N = argc > 2 ? atoi(argv[2]) : 3072;
  const int grid = argc > 3 ? atoi(argv[3]) : 256;
  uint16_t* C = nullptr;
  CK(hipMalloc(&C, (size_t)M * N * 2));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](int pat) {
    if (pat == 0) store_tiles<0><<<grid, 512>>>(C, M, N);
    else if (pat == 1) store_tiles<1><<<grid, 512>>>(C, M, N);
    else store_tiles<2><<<grid, 512>>>(C, M, N);
  };
  for (int pat = 0; pat < 3; ++pat) run(pat);
  CK(hipDeviceSynchronize());
  const char* names[3] = {"nt3 (8 rows x 2 x 64 B)", "line (8 rows x 128 B)", "wide (2 rows x 512 B)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int pat = 0; pat < 3; ++pat) {
      std::vector<float> ts;
      for (int i = 0; i < 7; ++i) {
        CK(hipEventRecord(a));
        run(pat);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double bytes = (double)M * N * 2;
      printf("M=%d N=%d grid=%d %-26s %8.1f us  %7.1f GB/s\n", M, N, grid, names[pat], ts[3] * 1e3,
             bytes / (ts[3] * 1e-3) / 1e9);
    }
  {
    unsigned long long* lat = nullptr;
    CK(hipMalloc(&lat, grid * sizeof(unsigned long long)));
    store_tiles_lat<<<grid, 512>>>(C, M, N, lat);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    store_tiles_lat<<<grid, 512>>>(C, M, N, lat);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> h(grid);
    CK(hipMemcpy(h.data(), lat, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    const int tiles = (M / 256) * (N / 256);
    double s = 0;
    for (auto x : h) s += (double)x;
    printf("M=%d N=%d grid=%d store+vmcnt(0) per tile: %8.1f us total, mean wait %.0f cycles per tile-epilogue\n", M, N,
           grid, ms * 1e3, s / tiles);
    CK(hipFree(lat));
  }
  CK(hipFree(C));
  return 0;
}
