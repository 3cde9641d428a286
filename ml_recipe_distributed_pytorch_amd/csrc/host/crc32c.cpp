// CRC32C (Castagnoli) for the TensorBoard event writer's TFRecord framing (utils/tb.py).
#include "hq_host.h"

namespace {
struct Table {
  uint32_t t[8][256];
  Table() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
const Table& table() {
  static Table tb;
  return tb;
}
}  // namespace

uint32_t hq_crc32c(const uint8_t* p, size_t n) {
  const auto& T = table().t;
  uint32_t crc = 0xFFFFFFFFu;
  while (n >= 8) {  // slicing-by-8
    const uint32_t a = crc ^ (uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24);
    crc = T[7][a & 0xFF] ^ T[6][(a >> 8) & 0xFF] ^ T[5][(a >> 16) & 0xFF] ^ T[4][a >> 24] ^ T[3][p[4]] ^ T[2][p[5]] ^
          T[1][p[6]] ^ T[0][p[7]];
    p += 8;
    n -= 8;
  }
  while (n--) crc = T[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return crc ^ 0xFFFFFFFFu;
}
