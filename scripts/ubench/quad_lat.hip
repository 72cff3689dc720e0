// Latency of the quad-lane point addition and its parts on one wave (gfx950), cycles per call:
// G1Quad::add, mulN<4>, a lone Fq product, the select + product of mulN with the library's select
// and with a branch-free mask select, four DPP broadcasts, an add + sub, the single-lane add2.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o quad_lat quad_lat.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../plonk-by-fingers_amd/csrc/ec_bn254.hpp"
using namespace pbf;
__device__ __forceinline__ U256 sel_b(uint32_t l, const U256& a, const U256& b, const U256& c, const U256& d) {
  const uint32_t m0 = 0u - (uint32_t)(l == 0), m1 = 0u - (uint32_t)(l == 1), m2 = 0u - (uint32_t)(l == 2),
                 m3 = 0u - (uint32_t)(l == 3);
  U256 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = (a.w[i] & m0) | (b.w[i] & m1) | (c.w[i] & m2) | (d.w[i] & m3);
  return r;
}
template <int V>
__global__ void __launch_bounds__(64) k(int iters, const uint64_t* seed, uint64_t* out) {
  U256 x = u256_from_u64(seed), y = u256_from_u64(seed + 4);
  const U256 one = Fq::to_mont(Fq::one_plain());
  Xyzz P{x, y, one, one}, Q{y, x, one, one};
  U256 a = x, b = y, c = one, d = x;
  const uint64_t t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    if (V == 0) P = G1Quad::add(P, Q);
    if (V == 1) { const U256* xs[4] = {&a, &b, &c, &d}; const U256* ys[4] = {&b, &c, &d, &a}; U256* o[4] = {&a, &b, &c, &d}; G1Quad::mulN<4>(xs, ys, o); }
    if (V == 2) a = Fq::mul(a, b);
    if (V == 3) { const uint32_t l = threadIdx.x & 3; a = Fq::mul(G1Quad::sel(l, a, b, c, d), G1Quad::sel(l, b, c, d, a)); }
    if (V == 4) { a = G1Quad::bcast<1>(a); b = G1Quad::bcast<2>(a); c = G1Quad::bcast<3>(b); d = G1Quad::bcast<0>(c); }
    if (V == 5) a = Fq::sub(Fq::add(a, b), c);
    if (V == 6) P = G1::add2(P, Q);
    if (V == 8) {  // the pairing engine's Karatsuba operand select (r = role 0..2 per lane)
      const uint32_t r = threadIdx.x % 3;
      const U256 z = u256_zero();
      U256 xo, yo;
      unsigned cc = 0;
      for (int i = 0; i < 8; ++i) xo.w[i] = __builtin_addc((r == 1 ? b : a).w[i], (r == 2 ? b : z).w[i], cc, &cc);
      cc = 0;
      for (int i = 0; i < 8; ++i) yo.w[i] = __builtin_addc((r == 1 ? d : c).w[i], (r == 2 ? d : z).w[i], cc, &cc);
      a = Fq::mul(xo, yo);
    }
    if (V == 7) { const uint32_t l = threadIdx.x & 3; a = Fq::mul(sel_b(l, a, b, c, d), sel_b(l, b, c, d, a)); }
  }
  const uint64_t t1 = clock64();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = P.X.w[0] ^ a.w[0] ^ b.w[1] ^ c.w[2] ^ d.w[3]; }
}
int main() {
  uint64_t *ds, *dout, h[2];
  uint64_t seed[8] = {0x1234567, 0x89abcdef, 0x5555, 0x1000, 0x7777, 0x3333, 0x2222, 0x100};
  (void)hipMalloc(&ds, 64); (void)hipMalloc(&dout, 64);
  (void)hipMemcpy(ds, seed, 64, hipMemcpyHostToDevice);
  void (*ks[9])(int, const uint64_t*, uint64_t*) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>};
  const char* nm[9] = {"G1Quad::add", "mulN<4>", "Fq::mul", "sel+mul", "4 bcast", "add+sub", "G1::add2", "selb+mul", "kara sel+mul"};
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < 9; ++v) {
      hipLaunchKernelGGL(ks[v], 1, 64, 0, 0, 256, ds, dout);
      (void)hipMemcpy(h, dout, 16, hipMemcpyDeviceToHost);
      if (rep == 2) printf("%-14s %9.1f cycles\n", nm[v], h[0] / 256.0);
    }
  return 0;
}
