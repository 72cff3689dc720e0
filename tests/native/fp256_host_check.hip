// Host-side check of the 256-bit Montgomery product (csrc/fp256.hpp): the 4 x 64-bit
// limb CIOS that the MSM's host Horner uses against the 8 x 32-bit limb CIOS, for Fr and
// Fq, on edge values (0, 1, p-1, R mod p, ...) and random canonical operands; also
// to_mont/from_mont round trips. Prints the product time of each form.
#include "../../plonk-by-fingers_amd/csrc/fp256.hpp"
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
using namespace pbf;
#if !defined(__HIP_DEVICE_COMPILE__)  // host-only check (mul_cios32 is a host function)
static long bad = 0;

template <class F, class Prm>
static U256 random_canonical(std::mt19937_64& g) {
  for (;;) {
    U256 r;
    for (int i = 0; i < 8; ++i) r.w[i] = (uint32_t)g();
    r.w[7] &= 0x3fffffffu;  // < 2^254
    if (!F::geq_p(r)) return r;
  }
}

template <class Prm>
static void check_field(const char* name) {
  typedef Fp256<Prm> F;
  std::mt19937_64 g(0x5EED0256);
  std::vector<U256> xs;
  U256 z{}, one{}, pm1{}, pm2{};
  one.w[0] = 1;
  for (int i = 0; i < 8; ++i) pm1.w[i] = Prm::P[i];
  pm1.w[0] -= 1;
  pm2 = pm1;
  pm2.w[0] -= 1;
  xs.push_back(z);
  xs.push_back(one);
  xs.push_back(pm1);
  xs.push_back(pm2);
  xs.push_back(F::r2());
  xs.push_back(F::to_mont(one));
  for (int i = 0; i < 200; ++i) xs.push_back(random_canonical<F, Prm>(g));
  for (const U256& a : xs)
    for (const U256& b : xs) {
      const U256 u = F::mul(a, b), v = F::mul_cios32(a, b);
      if (!F::eq(u, v) || F::geq_p(u)) {
        if (bad++ < 4) printf("%s mul mismatch\n", name);
      }
    }
  for (const U256& a : xs)
    if (!F::eq(F::from_mont(F::to_mont(a)), a) && bad++ < 8) printf("%s mont round trip\n", name);
  // timing: a dependent chain of products in each form
  const int N = 200000;
  U256 acc = xs[7];
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < N; ++i) acc = F::mul(acc, xs[8 + (i & 63)]);
  auto t1 = std::chrono::steady_clock::now();
  U256 acc2 = xs[7];
  for (int i = 0; i < N; ++i) acc2 = F::mul_cios32(acc2, xs[8 + (i & 63)]);
  auto t2 = std::chrono::steady_clock::now();
  if (!F::eq(acc, acc2) && bad++ < 8) printf("%s chain mismatch\n", name);
  printf("%s mul64 %.1f ns  mul32 %.1f ns\n", name, std::chrono::duration<double, std::nano>(t1 - t0).count() / N,
         std::chrono::duration<double, std::nano>(t2 - t1).count() / N);
}

int main() {
  check_field<Bn254FrParams>("Fr");
  check_field<Bn254FqParams>("Fq");
  printf("fp256_host_check bad=%ld\n", bad);
  return bad ? 1 : 0;
}
#endif
