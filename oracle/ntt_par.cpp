// ORACLE / CPU BASELINE — TEST INFRASTRUCTURE ONLY (see field.hpp header).
// An optimised iterative NTT for the Goldilocks field, all host cores: the "(b)" CPU
// baseline of BASELINE.md config 2 (the "(a)" baseline is the recursion-faithful
// restatement of src/fft.rs:90-106 in fft.hpp). Same output as fft.rs's CooleyTurkey
// (natural order in and out, X_k = sum_j a_j w^(jk)): bit-reversal permutation, then
// log2(n) radix-2 DIT levels over a precomputed twiddle table, products reduced with
// 2^64 = 2^32 - 1 and 2^96 = -1 (mod p). A batch is split over std::threads, one
// polynomial per task (the reference computes one transform, single-threaded).
#include <stdint.h>
#include <stddef.h>
#include <atomic>
#include <thread>
#include <vector>

namespace {
typedef unsigned __int128 u128;
constexpr uint64_t P = 0xFFFFFFFF00000001ull, EPS = 0xFFFFFFFFull;

inline uint64_t add(uint64_t a, uint64_t b) {
  uint64_t s;
  const bool c = __builtin_add_overflow(a, b, &s);
  return s + ((c || s >= P) ? EPS : 0);
}
inline uint64_t sub(uint64_t a, uint64_t b) {
  uint64_t d;
  const bool c = __builtin_sub_overflow(a, b, &d);
  return d - (c ? EPS : 0);
}
inline uint64_t mul(uint64_t a, uint64_t b) {
  const u128 x = (u128)a * b;
  const uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
  const uint64_t hh = hi >> 32, hl = hi & EPS;
  uint64_t t0;
  if (__builtin_sub_overflow(lo, hh, &t0)) t0 -= EPS;
  uint64_t r;
  if (__builtin_add_overflow(t0, hl * EPS, &r)) r += EPS;
  return r >= P ? r - P : r;
}
inline uint64_t pw(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mul(r, a);
    a = mul(a, a);
    e >>= 1;
  }
  return r;
}

void transform(uint64_t* a, size_t n, int logn, const std::vector<uint64_t>& tw, uint64_t scale) {
  for (size_t i = 1, j = 0; i < n; ++i) {  // bit reversal
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (int s = 1; s <= logn; ++s) {
    const size_t h = (size_t)1 << (s - 1), step = n >> s;  // tw[k * step] = w_(2h)^k
    for (size_t blk = 0; blk < n; blk += 2 * h)
      for (size_t k = 0; k < h; ++k) {
        const uint64_t u = a[blk + k], v = mul(a[blk + k + h], tw[k * step]);
        a[blk + k] = add(u, v);
        a[blk + k + h] = sub(u, v);
      }
  }
  if (scale != 1)
    for (size_t i = 0; i < n; ++i) a[i] = mul(a[i], scale);
}
}  // namespace

extern "C" int oracle_ntt_gl_par(uint64_t omega, const uint64_t* in, uint64_t* out, size_t n, size_t batch,
                                 int inverse, int threads) {
  if (n == 0 || (n & (n - 1))) return 1;
  int logn = 0;
  while (((size_t)1 << logn) < n) ++logn;
  const uint64_t w = inverse ? pw(omega, P - 2) : omega;
  std::vector<uint64_t> tw(n / 2 ? n / 2 : 1);
  tw[0] = 1;
  for (size_t i = 1; i < tw.size(); ++i) tw[i] = mul(tw[i - 1], w);
  const uint64_t scale = inverse ? pw(n % P, P - 2) : 1;
  if (threads < 1) threads = 1;
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t b; (b = next.fetch_add(1)) < batch;) {
      uint64_t* a = out + b * n;
      if (a != in + b * n)
        for (size_t i = 0; i < n; ++i) a[i] = in[b * n + i];
      transform(a, n, logn, tw, scale);
    }
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < threads && (size_t)t < batch; ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  return 0;
}
