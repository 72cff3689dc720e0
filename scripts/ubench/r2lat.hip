// Round-2/3 recombination of the workgroup Fq12 product (csrc/pairing.hip w_mul) in isolation,
// five variants on one workgroup of four waves, cycles per call (min / mean of 10 launches):
// V0 one round of lazy 288-bit sums per output lane, V1 the same with 16-B LDS loads and
// three interleaved chains, V2 V0 without the final reduction, V3 two rounds (18 lanes sum,
// then one lane per output combines and reduces: the form pairing.hip keeps), V4 V3 without
// the reduction. Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o r2lat r2lat.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../plonk-by-fingers_amd/csrc/fp256.hpp"
namespace pbf {
using Fq = Fp256<Bn254FqParams>;
struct Fq2 { U256 c0, c1; };
__device__ __forceinline__ U256 u256_zero() { U256 z; for (int i = 0; i < 8; ++i) z.w[i] = 0; return z; }
// Lazy sums: 9 x 32-bit limbs (< 2^288) through __builtin_addc / __builtin_subc carry chains
// (v_add_co / v_addc with SGPR-pair carries; the compiler interleaves independent chains and
// places the carry wait states).
struct L9 {
  uint32_t w[9];
};
__device__ __forceinline__ L9 l9_of(const U256& x) {
  L9 r;
#pragma unroll
  for (int l = 0; l < 8; ++l) r.w[l] = x.w[l];
  r.w[8] = 0;
  return r;
}
__device__ __forceinline__ void l9_add(L9& a, const U256& x) {
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) a.w[l] = __builtin_addc(a.w[l], x.w[l], c, &c);
  a.w[8] += c;
}
__device__ __forceinline__ void l9_add(L9& a, const L9& b) {
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 9; ++l) a.w[l] = __builtin_addc(a.w[l], b.w[l], c, &c);
}
__device__ __forceinline__ void l9_sub(L9& a, const L9& b) {  // requires a >= b
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 9; ++l) a.w[l] = __builtin_subc(a.w[l], b.w[l], c, &c);
}
template <int S>
__device__ __forceinline__ L9 l9_shl(const L9& a) {  // a << S (no overflow for our bounds)
  L9 r;
  r.w[0] = a.w[0] << S;
#pragma unroll
  for (int l = 1; l < 9; ++l) r.w[l] = (a.w[l] << S) | (a.w[l - 1] >> (32 - S));
  return r;
}
// K q in 9 limbs, compile time
struct L9c {
  uint32_t w[9];
};
constexpr L9c l9_kq(uint32_t K) {
  L9c r{};
  uint64_t c = 0;
  for (int l = 0; l < 8; ++l) {
    const uint64_t p = (uint64_t)K * Bn254FqParams::P[l] + c;
    r.w[l] = (uint32_t)p;
    c = p >> 32;
  }
  r.w[8] = (uint32_t)c;
  return r;
}
template <uint32_t K>
__device__ __forceinline__ void l9_add_kq(L9& a) {
  constexpr L9c k = l9_kq(K);
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 9; ++l) a.w[l] = __builtin_addc(a.w[l], k.w[l], c, &c);
}
// x mod q for x < 2^262 (x < 340 q): d = floor(x / q) estimated from x's top 96 bits in double
// (relative error < 2^-50, so x / q - est < 1e-12 for x < 340 q) minus a 1e-9 margin, so that
// d is floor(x / q) or one less: x - d q < 2q, one conditional subtraction.
__device__ __forceinline__ U256 l9_reduce(L9 x) {
  const double top = ((double)x.w[8] * 18446744073709551616.0 + (double)x.w[7] * 4294967296.0) + (double)x.w[6];
  const double est = top * (1.0 / 3486998266802970666.0) - 1e-9;  // q / 2^192 = 0x30644e72e131a029.b8...
  const uint32_t d = est > 0.0 ? (uint32_t)est : 0u;
  L9 m;
  uint64_t c = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) {
    const uint64_t p = (uint64_t)d * Bn254FqParams::P[l] + c;
    m.w[l] = (uint32_t)p;
    c = p >> 32;
  }
  m.w[8] = (uint32_t)c;
  l9_sub(x, m);
  U256 r;
#pragma unroll
  for (int l = 0; l < 8; ++l) r.w[l] = x.w[l];  // < 2q < 2^255: limb 8 is 0
  return Fq::reduce_once(r);
}
// a + b without the reduction (< 2q for canonical a, b): a Montgomery product accepts operands
// below 2q (their product is below q R, so the result stays below 2q before its subtraction)
__device__ __forceinline__ U256 u256_add_raw(const U256& a, const U256& b) {
  U256 r;
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) r.w[l] = __builtin_addc(a.w[l], b.w[l], c, &c);
  return r;
}
__device__ __forceinline__ U256 kara_raw(const Fq2& a, int r) {
  return u256_add_raw(r == 1 ? a.c1 : a.c0, r == 2 ? a.c1 : u256_zero());
}


struct alignas(16) PL { U256 t[256]; Fq2 reg[12]; L9 acc[6][3]; };
__device__ __forceinline__ U256 ld16(const U256* p) {
  const uint4 a = ((const uint4*)p)[0], b = ((const uint4*)p)[1];
  U256 r;
  r.w[0] = a.x; r.w[1] = a.y; r.w[2] = a.z; r.w[3] = a.w; r.w[4] = b.x; r.w[5] = b.y; r.w[6] = b.z; r.w[7] = b.w;
  return r;
}
__device__ __forceinline__ void l9_add3(L9* s, const U256& a, const U256& b, const U256& c) {
  unsigned ca = 0, cb = 0, cc = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) {
    s[0].w[l] = __builtin_addc(s[0].w[l], a.w[l], ca, &ca);
    s[1].w[l] = __builtin_addc(s[1].w[l], b.w[l], cb, &cb);
    s[2].w[l] = __builtin_addc(s[2].w[l], c.w[l], cc, &cc);
  }
  s[0].w[8] += ca; s[1].w[8] += cb; s[2].w[8] += cc;
}
template <int V>
__device__ __forceinline__ void r2(Fq2* dst, PL& L, int tid) {
  const int wv = tid >> 6, k = tid & 63;
  if (k < 6) {
    L9 s[3];
    if (V == 0) {
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) {
      const int i = k - jj < 0 ? k - jj + 6 : k - jj;
      const U256* t = L.t + 3 * (i * 6 + jj);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        if (jj == 0) s[c] = l9_of(t[c]);
        else l9_add(s[c], t[c]);
      }
    }
    } else {
      U256 tv[18];
#pragma unroll
      for (int jj = 0; jj < 6; ++jj) {
        const int i = k - jj < 0 ? k - jj + 6 : k - jj;
        const U256* t = L.t + 3 * (i * 6 + jj);
#pragma unroll
        for (int c = 0; c < 3; ++c) tv[3 * jj + c] = ld16(t + c);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) s[c] = l9_of(tv[c]);
#pragma unroll
      for (int jj = 1; jj < 6; ++jj) l9_add3(s, tv[3 * jj], tv[3 * jj + 1], tv[3 * jj + 2]);
    }
    L9 v;
    if (wv == 0) {
      v = s[0]; l9_add_kq<6>(v); l9_sub(v, s[1]);
    } else if (wv == 1) {
      v = s[2]; l9_add_kq<12>(v); l9_sub(v, s[0]); l9_sub(v, s[1]);
    } else if (wv == 2) {
      L9 f = l9_shl<2>(s[0]); l9_add(f, s[0]); v = l9_shl<1>(f); l9_add_kq<54>(v);
      l9_sub(v, l9_shl<3>(s[1])); l9_sub(v, s[2]);
    } else {
      v = l9_shl<3>(s[2]); l9_add(v, s[2]); l9_add_kq<108>(v);
      L9 u = s[0]; l9_add(u, s[1]); l9_sub(v, l9_shl<3>(u)); l9_sub(v, l9_shl<1>(s[1]));
    }
    const U256 r = V == 2 ? U256{{v.w[0], v.w[1], v.w[2], v.w[3], v.w[4], v.w[5], v.w[6], v.w[7]}} : l9_reduce(v);
    Fq2& d = dst[k + (wv >> 1) * 6];
    if (wv & 1) d.c1 = r; else d.c0 = r;
  }
  __syncthreads();
}

// two rounds: 18 lanes sum t_c over the six pairs of output k; then wave (h, c) combines
template <int V>
__device__ __forceinline__ void r23(Fq2* dst, PL& L, int tid) {
  if (tid < 18) {
    const int k = tid / 3, c = tid - 3 * k;
    L9 s;
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) {
      const int i = k - jj < 0 ? k - jj + 6 : k - jj;
      const U256 t = L.t[3 * (i * 6 + jj) + c];
      if (jj == 0) s = l9_of(t); else l9_add(s, t);
    }
    L.acc[k][c] = s;
  }
  __syncthreads();
  const int wv = tid >> 6, k = tid & 63;
  if (k < 6) {
    L9 s[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) s[c] = L.acc[k][c];
    L9 v;
    if (wv == 0) {
      v = s[0]; l9_add_kq<6>(v); l9_sub(v, s[1]);
    } else if (wv == 1) {
      v = s[2]; l9_add_kq<12>(v); l9_sub(v, s[0]); l9_sub(v, s[1]);
    } else if (wv == 2) {
      L9 f = l9_shl<2>(s[0]); l9_add(f, s[0]); v = l9_shl<1>(f); l9_add_kq<54>(v);
      l9_sub(v, l9_shl<3>(s[1])); l9_sub(v, s[2]);
    } else {
      v = l9_shl<3>(s[2]); l9_add(v, s[2]); l9_add_kq<108>(v);
      L9 u = s[0]; l9_add(u, s[1]); l9_sub(v, l9_shl<3>(u)); l9_sub(v, l9_shl<1>(s[1]));
    }
    const U256 r = V == 4 ? U256{{v.w[0], v.w[1], v.w[2], v.w[3], v.w[4], v.w[5], v.w[6], v.w[7]}} : l9_reduce(v);
    Fq2& d = dst[k + (wv >> 1) * 6];
    if (wv & 1) d.c1 = r; else d.c0 = r;
  }
  __syncthreads();
}
template <int V>
__global__ void __launch_bounds__(256) r2k(int iters, uint64_t* out) {
  __shared__ PL L;
  const int tid = threadIdx.x;
  for (int l = 0; l < 8; ++l) L.t[tid].w[l] = (tid * 7 + l) & 0x0fffffff;
  __syncthreads();
  const uint64_t t0 = clock64();
  for (int it = 0; it < iters; ++it) { if (V >= 3) r23<V>(L.reg, L, tid); else r2<V>(L.reg, L, tid); }
  const uint64_t t1 = clock64();
  if (tid == 0) { out[0] = t1 - t0; out[1] = L.reg[0].c0.w[0]; }
}
}
using namespace pbf;
int main() {
  uint64_t* d; hipMalloc(&d, 64); uint64_t h[2];
  void (*ks[5])(int, uint64_t*) = {r2k<0>, r2k<1>, r2k<2>, r2k<3>, r2k<4>};
  const char* nm[5] = {"V0 current", "V1 b128+add3", "V2 no reduce", "V3 two rounds", "V4 two, no red"};
  double best[5] = {1e30, 1e30, 1e30, 1e30, 1e30}, sum[5] = {0};
  for (int rep = 0; rep < 12; ++rep)
    for (int v = 0; v < 5; ++v) {
      hipLaunchKernelGGL(ks[v], 1, 256, 0, 0, 256, d); hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
      const double c = h[0] / 256.0;
      if (rep >= 2) { best[v] = c < best[v] ? c : best[v]; sum[v] += c; }
    }
  for (int v = 0; v < 5; ++v) printf("%-16s min %8.1f  mean %8.1f cycles\n", nm[v], best[v], sum[v] / 10);
  return 0;
}
