// Host-side check of the device Goldilocks arithmetic (csrc/field.hpp, compiled for the
// host by hipcc) against unsigned __int128 arithmetic: edge values and random operands
// for add/sub/mul/reduce128, every compile-time shift mul_pow2<S>, S < 96, and every
// division gl_div_pow2<K>, 1 <= K <= 32.
#include "../../plonk-by-fingers_amd/csrc/field.hpp"
#include <cstdio>
#include <random>
#include <utility>
using namespace pbf;
typedef unsigned __int128 u128;
static const uint64_t P = Goldilocks::P;
static long bad = 0;
static void expect(const char* what, uint64_t got, uint64_t exp, uint64_t a, uint64_t b) {
  if (got != exp && bad++ < 8)
    printf("%s(%llx, %llx) = %llx, expected %llx\n", what, (unsigned long long)a, (unsigned long long)b,
           (unsigned long long)got, (unsigned long long)exp);
}
static uint64_t pow2mod(int s) {
  u128 x = 1;
  for (int i = 0; i < s; ++i) x = (x * 2) % P;
  return (uint64_t)x;
}
template <int S>
static void shift_check(const uint64_t* xs, int m) {
  const uint64_t t = pow2mod(S);
  for (int i = 0; i < m; ++i)
    expect("mul_pow2", Goldilocks::mul_pow2<S>(xs[i]), (uint64_t)(((u128)xs[i] * t) % P), xs[i], S);
}
template <int... S>
static void all_shifts(const uint64_t* xs, int m, std::integer_sequence<int, S...>) {
  (shift_check<S>(xs, m), ...);
}
static uint64_t inv2k(int k) {  // 2^-k mod p
  u128 x = 1, h = (P + 1) / 2;  // 1/2
  for (int i = 0; i < k; ++i) x = (x * h) % P;
  return (uint64_t)x;
}
template <int K>
static void div_check(const uint64_t* xs, int m) {
  const uint64_t t = inv2k(K);
  for (int i = 0; i < m; ++i)
    expect("gl_div_pow2", gl_div_pow2<K>(xs[i]), (uint64_t)(((u128)xs[i] * t) % P), xs[i], K);
}
template <int... K>
static void all_divs(const uint64_t* xs, int m, std::integer_sequence<int, K...>) {
  (div_check<K + 1>(xs, m), ...);
}
int main() {
  std::mt19937_64 g(1);
  const FieldArgs f{P, 0};
  uint64_t xs[64] = {0, 1, 2, P - 1, P - 2, 0xFFFFFFFFull, 0x100000000ull, 0xFFFFFFFF00000000ull, P >> 1,
                     0x7FFFFFFFFFFFFFFFull, 0x80000000ull, 0xFFFFFFFEFFFFFFFFull};
  for (int i = 12; i < 64; ++i) xs[i] = g() % P;
  for (uint64_t a : xs)
    for (uint64_t b : xs) {
      expect("add", Goldilocks::add(a, b, f), (uint64_t)(((u128)a + b) % P), a, b);
      expect("sub", Goldilocks::sub(a, b, f), (uint64_t)(((u128)a + P - b) % P), a, b);
      expect("mul", Goldilocks::mul(a, b, f), (uint64_t)(((u128)a * b) % P), a, b);
    }
  const uint64_t ex[] = {0, 1, 0xFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFF00000000ull, P, P - 1, 0x100000000ull};
  for (uint64_t lo : ex)
    for (uint64_t hi : ex) expect("reduce128", Goldilocks::reduce128(lo, hi), (uint64_t)((((u128)hi << 64) | lo) % P), lo, hi);
  for (int i = 0; i < 2000000; ++i) {
    const uint64_t a = g() % P, b = g() % P, lo = g(), hi = g();
    expect("mul", Goldilocks::mul(a, b, f), (uint64_t)(((u128)a * b) % P), a, b);
    expect("add", Goldilocks::add(a, b, f), (uint64_t)(((u128)a + b) % P), a, b);
    expect("reduce128", Goldilocks::reduce128(lo, hi), (uint64_t)((((u128)hi << 64) | lo) % P), lo, hi);
  }
  all_shifts(xs, 64, std::make_integer_sequence<int, 96>{});
  all_divs(xs, 64, std::make_integer_sequence<int, 32>{});
  {
    uint64_t ys[4096];
    for (int i = 0; i < 4096; ++i) ys[i] = i < 64 ? xs[i] : g() % P;
    all_divs(ys, 4096, std::make_integer_sequence<int, 32>{});
  }
  printf("field_host_check bad=%ld\n", bad);
  return bad != 0;
}
