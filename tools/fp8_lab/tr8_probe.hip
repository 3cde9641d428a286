// Probe ds_read_b64_tr_b8 (gfx950 transposed LDS read of 8-bit elements) before building the fp8 TN
// (weight-gradient) GEMM on it.  LDS holds a [64 rows][128 B] image with byte (r, c) = r·128 + c encoded
// as (r & 63) | ((c & 3) << 6) in its own byte and the full (r, c) recoverable from a parallel 16-bit image.
// Hypothesis (the 8-bit analogue of ds_read_b64_tr_b16, cdna_hip_programming.md T10): per group of 16
// lanes the instruction reads 8 rows × 16 bytes; lane 2q + p supplies the address of row q, bytes 8p..8p+7;
// lane i of the group receives column i of those 8 rows (byte j of its 8-byte result = row j).
// The probe lets every lane address row (lane>>1)&7 of its group's row block, bytes 8·(lane&1) of a
// 16-byte column block, and prints what each lane received as (row, col) pairs.
// Build + run: hipcc -O2 --offload-arch=gfx950 tools/fp8_lab/tr8_probe.hip -o /tmp/tr8 && /tmp/tr8
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void probe(uint32_t* out, int row_stride) {
  __shared__ uint8_t img[64 * 128];
  const int l = threadIdx.x;
  for (int i = l; i < 64 * 128; i += 64) {
    const int r = i / 128, c = i % 128;
    img[r * 128 + c] = (uint8_t)((r * 13 + c * 7) & 0xFF);   // checked on the host against a table
  }
  __syncthreads();
  const int g = l >> 4, i = l & 15;
  const int q = i >> 1, p = i & 1;
  // group g reads rows 8g .. 8g+7, column block 16·g (so groups differ in rows AND columns)
  const int row = 8 * g + q, col = 16 * g + 8 * p;
  const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(img) + row * row_stride + col;
  typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
  u32x2 v;
  asm volatile("ds_read_b64_tr_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  out[2 * l] = v[0];
  out[2 * l + 1] = v[1];
}

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 64 * 2 * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 128);
  std::vector<uint32_t> h(128);
  if (hipMemcpy(h.data(), d, 128 * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  // inverse table: byte value -> list of (r, c) in the probed region
  int ok = 0, bad = 0;
  for (int l = 0; l < 64; ++l) {
    const int g = l >> 4, i = l & 15;
    uint8_t b[8];
    for (int j = 0; j < 8; ++j) b[j] = (uint8_t)((j < 4 ? h[2 * l] >> (8 * j) : h[2 * l + 1] >> (8 * (j - 4))) & 0xFF);
    // hypothesis: lane i of group g holds column 16g + i, rows 8g + j
    bool match = true;
    for (int j = 0; j < 8; ++j) {
      const int r = 8 * g + j, c = 16 * g + i;
      if (b[j] != (uint8_t)((r * 13 + c * 7) & 0xFF)) match = false;
    }
    match ? ++ok : ++bad;
    if (l < 20 || !match) {
      printf("lane %2d:", l);
      for (int j = 0; j < 8; ++j) {   // decode candidates (r, c) in the group's 8×16 block
        int found = 0;
        for (int r = 8 * g; r < 8 * g + 8 && !found; ++r)
          for (int c = 16 * g; c < 16 * g + 16 && !found; ++c)
            if (b[j] == (uint8_t)((r * 13 + c * 7) & 0xFF)) { printf(" (%d,%d)", r, c); found = 1; }
        if (!found) printf(" (?%02x)", b[j]);
      }
      printf("%s\n", match ? "" : "  <- differs from hypothesis");
    }
  }
  printf("hypothesis (lane i of group g = column 16g+i, rows 8g..8g+7): %d lanes match, %d differ\n", ok, bad);
  return bad ? 2 : 0;
}
