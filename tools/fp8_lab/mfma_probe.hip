// Probe the lane map of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 A and B, unit e8m0 scales) with exact
// small-integer data: lane l is assumed to hold A[row = l & 15][k = 32·(l >> 4) + j] (j = 0..31 in byte
// order) and B[k = 32·(l >> 4) + j][col = l & 15]; C/D as every 16x16 shape (col = l & 15,
// row = 4·(l >> 4) + i).  Prints max |err| vs a host reference for candidate maps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __host__ inline uint8_t enc(int v) {  // e4m3 for v in {-2,-1,0,1,2}
  switch (v) { case 1: return 0x38; case 2: return 0x40; case -1: return 0xB8; case -2: return 0xC0; default: return 0; }
}

// map 0: lane holds k = 32*(l>>4) + j ; map 1: k = 16*(l>>4) + j for j<16, 64 + 16*(l>>4) + (j-16) for j>=16
__global__ void probe(const int8_t* A, const int8_t* B, float* D, int map) {
  const int l = threadIdx.x;
  uint8_t a[32], b[32];
  for (int j = 0; j < 32; ++j) {
    int k = map == 0 ? 32 * (l >> 4) + j : (j < 16 ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + (j - 16));
    a[j] = enc(A[(l & 15) * 128 + k]);
    b[j] = enc(B[k * 16 + (l & 15)]);
  }
  i32x8 av, bv;
  for (int w = 0; w < 8; ++w) {
    av[w] = a[4 * w] | (a[4 * w + 1] << 8) | (a[4 * w + 2] << 16) | (a[4 * w + 3] << 24);
    bv[w] = b[4 * w] | (b[4 * w + 1] << 8) | (b[4 * w + 2] << 16) | (b[4 * w + 3] << 24);
  }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 127, 0, 127);
  for (int i = 0; i < 4; ++i) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main() {
  std::vector<int8_t> A(16 * 128), B(128 * 16);
  for (int r = 0; r < 16; ++r)
    for (int k = 0; k < 128; ++k) A[r * 128 + k] = (int8_t)(((r * 7 + k * 3) % 5) - 2);
  for (int k = 0; k < 128; ++k)
    for (int c = 0; c < 16; ++c) B[k * 16 + c] = (int8_t)(((k * 5 + c * 11 + 1) % 5) - 2);
  std::vector<float> ref(256, 0.f);
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      float s = 0;
      for (int k = 0; k < 128; ++k) s += A[r * 128 + k] * B[k * 16 + c];
      ref[r * 16 + c] = s;
    }
  int8_t *dA, *dB;
  float* dD;
  hipMalloc(&dA, A.size()); hipMalloc(&dB, B.size()); hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  for (int map = 0; map < 2; ++map) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, map);
    std::vector<float> D(256);
    hipMemcpy(D.data(), dD, 256 * 4, hipMemcpyDeviceToHost);
    float err = 0;
    for (int i = 0; i < 256; ++i) err = fmaxf(err, fabsf(D[i] - ref[i]));
    printf("map %d: max |err| = %g  (D[0]=%g ref[0]=%g D[17]=%g ref[17]=%g)\n", map, err, D[0], ref[0], D[17], ref[17]);
  }
  return 0;
}
