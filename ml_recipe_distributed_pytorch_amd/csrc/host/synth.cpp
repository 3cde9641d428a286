// Native dummy-QA batch synthesiser (reference DummyDataset + collate_fun).
// The reference builds ~2-3k samples/s per CPU core in Python; this fills a whole [B, L] batch of
// int64 ids / token types / bool mask straight into (pinned) tensor memory with one xoshiro256**
// stream per row, rows split over std::threads.
#include "hq_host.h"

#include <algorithm>
#include <thread>
#include <vector>

namespace {

inline uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Xoshiro256 {
  uint64_t s[4];
  explicit Xoshiro256(uint64_t seed) {
    for (auto& v : s) v = splitmix64(seed);
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  inline uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
};

}  // namespace

void hq_synth_dummy(int64_t* ids, int64_t* type_ids, bool* mask, int B, int L, int q, int64_t vocab, int64_t pad,
                    int64_t unk, int64_t cls, int64_t sep, bool bert_types, uint64_t seed, int threads) {
  const uint64_t span = (uint64_t)(vocab - 1);
  auto work = [&](int r0, int r1) {
    for (int r = r0; r < r1; ++r) {
      Xoshiro256 rng(seed * 0x100000001B3ull + (uint64_t)r);
      int64_t* row = ids + (size_t)r * L;
      for (int i = 0; i < L; ++i) {
        const uint64_t x = rng.next() >> 32;
        int64_t v = 1 + (int64_t)((x * span) >> 32);
        if (v == pad || v == sep || v == cls) v = unk;
        row[i] = v;
      }
      row[0] = cls;
      row[q + 1] = sep;
      row[L - 1] = sep;
      int64_t* tt = type_ids + (size_t)r * L;
      bool* mk = mask + (size_t)r * L;
      for (int i = 0; i < L; ++i) {
        tt[i] = (bert_types && i > q + 1) ? 1 : 0;
        mk[i] = row[i] > 0;
      }
    }
  };
  threads = std::max(1, std::min(threads, B));
  if (threads == 1) {
    work(0, B);
    return;
  }
  std::vector<std::thread> pool;
  const int per = (B + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int a = t * per, b = std::min(B, a + per);
    if (a < b) pool.emplace_back(work, a, b);
  }
  for (auto& th : pool) th.join();
}
