// Microbenchmark (not part of libpbf.so): Fr product throughput of the 32-bit single-chain
// Montgomery product (Fr::mul_tp, what the Fr NTT butterflies use) against the 29-bit-limb
// product (msm_l29.hpp's scheme with r's limbs, R = 2^261) wrapped for canonical 8 x 32-bit data:
// re-limb the data operand, multiply by a twiddle already in 29-bit limbs (or re-limbed per
// product too), canonicalise, pack back. Every lane of a full grid runs two independent chains.
// Build: make -C scripts/ubench fr_mul29; run: scripts/ubench/fr_mul29
#include "../../plonk-by-fingers_amd/csrc/ec_bn254.hpp"
#include "../../plonk-by-fingers_amd/csrc/msm_l29.hpp"
#include <cstdio>
#include <vector>

using namespace pbf;

namespace fr29 {
using l29::L29;
constexpr uint32_t R29[9] = {0x10000001u, 0x1f0fac9fu, 0x0e5c2450u, 0x07d090f3u, 0x1585d283u,
                             0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
constexpr uint32_t NR29 = 0x0fffffffu;
constexpr uint32_t MASK = l29::MASK;
__device__ __forceinline__ L29 mul(const L29& a, const L29& b) {
  uint32_t m[9];
  L29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    const int lo = k < 9 ? 0 : k - 8, hi = k < 9 ? k : 8;
#pragma unroll
    for (int i = lo; i <= hi; ++i) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = lo; i < (k < 9 ? k : 9); ++i) acc += (uint64_t)m[i] * R29[k - i];
    if (k < 9) {
      m[k] = ((uint32_t)acc * NR29) & MASK;
      acc += (uint64_t)m[k] * R29[0];
    } else {
      r.l[k - 9] = (uint32_t)acc & MASK;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}
__device__ __forceinline__ L29 canon(const L29& a) {  // a < 2r
  bool ge = true;
#pragma unroll
  for (int i = 8; i >= 0; --i) {
    if (a.l[i] != R29[i]) {
      ge = a.l[i] > R29[i];
      break;
    }
  }
  if (!ge) return a;
  L29 r;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int32_t d = (int32_t)a.l[i] - (int32_t)R29[i] - borrow;
    borrow = d < 0 ? 1 : 0;
    r.l[i] = (uint32_t)(d + (borrow << 29));
  }
  return r;
}
// canonical x (8 x 32) times w (29-bit limbs, w 2^261 mod r): canonical x w mod r
__device__ __forceinline__ U256 mulw(const U256& x, const L29& w) {
  return l29::to_u256(fr29::canon(fr29::mul(l29::from_u256(x), w)));
}
}  // namespace fr29

__global__ void __launch_bounds__(256) k_tp(int iters, const uint64_t* seed, uint64_t* out) {
  U256 x = u256_from_u64(seed), y = u256_from_u64(seed + 4), z = x;
  x.w[0] ^= threadIdx.x;
  z.w[1] ^= blockIdx.x;
  for (int i = 0; i < iters; ++i) {
    x = Fr::mul_tp(x, y);
    z = Fr::mul_tp(z, y);
  }
  if ((x.w[0] ^ z.w[0]) == 0x12345u) out[3] = 1;
}
template <bool RELIMB_W>
__global__ void __launch_bounds__(256) k_29(int iters, const uint64_t* seed, uint64_t* out) {
  U256 x = u256_from_u64(seed), y = u256_from_u64(seed + 4), z = x;
  x.w[0] ^= threadIdx.x;
  z.w[1] ^= blockIdx.x;
  l29::L29 w = l29::from_u256(y);
  for (int i = 0; i < iters; ++i) {
    if (RELIMB_W) {
      y.w[0] ^= i;  // a different twiddle every product, re-limbed like a table load
      w = l29::from_u256(y);
    }
    x = fr29::mulw(x, w);
    z = fr29::mulw(z, w);
  }
  if ((x.w[0] ^ z.w[0]) == 0x12345u) out[3] = 1;
}
// the 29-bit product alone: operands stay in 29-bit limbs (no re-limbing, no canonicalisation)
__global__ void __launch_bounds__(256) k_29raw(int iters, const uint64_t* seed, uint64_t* out) {
  U256 xu = u256_from_u64(seed), y = u256_from_u64(seed + 4);
  xu.w[0] ^= threadIdx.x;
  l29::L29 x = l29::from_u256(xu), z = x, w = l29::from_u256(y);
  z.l[1] ^= blockIdx.x & 0xFF;
  for (int i = 0; i < iters; ++i) {
    x = fr29::mul(x, w);
    z = fr29::mul(z, w);
  }
  if ((x.l[0] ^ z.l[0]) == 0x12345u) out[3] = 1;
}
// correctness: fr29::mulw(x, w 2^261) == Fr::mul(x, w 2^256) for random canonical x, w
__global__ void k_check(const uint64_t* xs, const uint64_t* ws32, const uint64_t* ws29, int n, int* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const U256 x = u256_from_u64(xs + 4 * i);
  const U256 a = Fr::mul(x, u256_from_u64(ws32 + 4 * i));
  const U256 b = fr29::mulw(x, l29::from_u256(u256_from_u64(ws29 + 4 * i)));
  for (int k = 0; k < 8; ++k)
    if (a.w[k] != b.w[k]) *bad = 1;
}

int main() {
  uint64_t *d_seed, *d_out;
  uint64_t seed[8] = {0x1234567, 0x89abcdef, 0x5555, 0x1000, 0x7777, 0x3333, 0x2222, 0x100};
  hipMalloc(&d_seed, 64);
  hipMalloc(&d_out, 64);
  hipMemcpy(d_seed, seed, 64, hipMemcpyHostToDevice);
  // correctness on the host-made operands: w 2^256 and w 2^261 mod r of the same w
  {
    const int n = 4096;
    std::vector<uint64_t> xs(4 * n), w32(4 * n), w29(4 * n);
    uint64_t s = 99;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return s; };
    U256 c32;  // 32 in Montgomery form: w 2^256 -> w 2^261 by one host product
    c32 = Fr::to_mont(Fr::one_plain());
    for (int k = 0; k < 5; ++k) c32 = Fr::add(c32, c32);
    for (int i = 0; i < n; ++i) {
      U256 x, w;
      for (int k = 0; k < 8; ++k) { x.w[k] = (uint32_t)rnd(); w.w[k] = (uint32_t)rnd(); }
      x.w[7] &= 0x0FFFFFFF;
      w.w[7] &= 0x0FFFFFFF;
      const U256 wm = Fr::to_mont(w), w5 = Fr::mul(wm, c32);
      for (int k = 0; k < 4; ++k) {
        xs[4 * i + k] = (uint64_t)x.w[2 * k] | ((uint64_t)x.w[2 * k + 1] << 32);
        w32[4 * i + k] = (uint64_t)wm.w[2 * k] | ((uint64_t)wm.w[2 * k + 1] << 32);
        w29[4 * i + k] = (uint64_t)w5.w[2 * k] | ((uint64_t)w5.w[2 * k + 1] << 32);
      }
    }
    uint64_t *dx, *d32, *d29;
    int* dbad;
    hipMalloc(&dx, xs.size() * 8);
    hipMalloc(&d32, xs.size() * 8);
    hipMalloc(&d29, xs.size() * 8);
    hipMalloc(&dbad, 4);
    hipMemset(dbad, 0, 4);
    hipMemcpy(dx, xs.data(), xs.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(d32, w32.data(), xs.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(d29, w29.data(), xs.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, dx, d32, d29, n, dbad);
    int bad = 0;
    hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
    printf("check fr29::mulw == Fr::mul on %d random pairs: %s\n", n, bad ? "MISMATCH" : "ok");
    if (bad) return 1;
  }
  const int blocks = 256 * 8, iters = 256;
  const double muls = 2.0 * iters * blocks * 256;
  const char* names[] = {"Fr::mul_tp (32-bit)", "29-bit, twiddle in limbs", "29-bit, twiddle re-limbed",
                         "29-bit product alone"};
  for (int v = 0; v < 4; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL(k_tp, dim3(blocks), dim3(256), 0, 0, iters, d_seed, d_out);
      if (v == 1) hipLaunchKernelGGL((k_29<false>), dim3(blocks), dim3(256), 0, 0, iters, d_seed, d_out);
      if (v == 2) hipLaunchKernelGGL((k_29<true>), dim3(blocks), dim3(256), 0, 0, iters, d_seed, d_out);
      if (v == 3) hipLaunchKernelGGL(k_29raw, dim3(blocks), dim3(256), 0, 0, iters, d_seed, d_out);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 2) printf("%-28s %.3f ms  %.3e Fr products/s\n", names[v], ms, muls / (ms * 1e-3));
    }
  }
  return 0;
}
