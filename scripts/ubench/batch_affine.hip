// Microbenchmark (not part of libpbf.so): is batch-affine bucket accumulation cheaper than
// the XYZZ mixed additions of the MSM (verdict r03 item 7)?
//
// An affine addition P + Q needs lambda = (yQ - yP) / (xQ - xP): 3 products (lambda, lambda^2,
// lambda (xP - x3)) plus one inversion, which Montgomery's trick shares across a batch of K
// independent additions for 3 more products each (prefix product, and two in the backward
// sweep) plus one Fermat inversion (~380 products) per batch: 6 + 380 / K products per
// addition, against 10 for madd-2008-s. Independent additions are what Pippenger's buckets
// offer (one addition per bucket per round), so a thread's batch is K different buckets,
// whose accumulators and prefix products live in global memory ([k][thread], coalesced).
//
//   k_xyzz            M mixed XYZZ additions per thread into one accumulator (G1::madd_tp, the
//                     32-bit single-chain product; the production accumulation uses the
//                     29-bit-limb form, ~30 % fewer VALU per product)
//   k_affine<K, G>    rounds of K batched affine additions per thread, accumulators and prefix
//                     products in global memory (G = true) or registers (K <= 8, G = false)
// Operands are random field elements (the cost of the arithmetic does not depend on the
// points being on the curve; no addition degenerates). Prints additions/s of each.
//
// Build: make -C scripts/ubench batch_affine; run: scripts/ubench/batch_affine
#include "../../plonk-by-fingers_amd/csrc/ec_bn254.hpp"
#include <cstdio>
#include <vector>

using namespace pbf;

__device__ __forceinline__ U256 fq_inv(const U256& a) {  // a^(q-2), Montgomery
  U256 r = Fq::to_mont(Fq::one_plain());
  for (int i = 255; i >= 0; --i) {
    r = Fq::mul_tp(r, r);
    const uint32_t e = Bn254FqParams::P[i / 32] - (i < 32 ? 2u : 0u);
    if ((e >> (i % 32)) & 1) r = Fq::mul_tp(r, a);
  }
  return r;
}

__device__ __forceinline__ U256 ld(const uint64_t* base, uint64_t idx) { return u256_from_u64(base + 4 * idx); }
__device__ __forceinline__ void st(uint64_t* base, uint64_t idx, const U256& v) { u256_to_u64(v, base + 4 * idx); }

// pts: npts x (x, y) pairs, Montgomery, planar [2][npts]
__global__ void __launch_bounds__(256) k_xyzz(const uint64_t* pts, uint64_t npts, int M, uint64_t* out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, T = (uint64_t)gridDim.x * blockDim.x;
  Affine a;
  a.x = ld(pts, t % npts);
  a.y = ld(pts + 4 * npts, t % npts);
  Xyzz acc = G1::from_affine(a);
  for (int m = 1; m <= M; ++m) {
    const uint64_t i = (t + m * T) % npts;
    Affine q;
    q.x = ld(pts, i);
    q.y = ld(pts + 4 * npts, i);
    acc = G1::madd_tp(acc, q);
  }
  st(out, t, acc.X);
}

// K accumulators per thread; `rounds` rounds of one addition to each; acc / prefix in global
// memory ([k][T] planes) when G, in registers otherwise
template <int K, bool G>
__global__ void __launch_bounds__(256) k_affine(const uint64_t* pts, uint64_t npts, int rounds, uint64_t* accx,
                                                uint64_t* accy, uint64_t* pre, uint64_t* out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, T = (uint64_t)gridDim.x * blockDim.x;
  U256 rx[G ? 1 : K], ry[G ? 1 : K], rp[G ? 1 : K];
  for (int k = 0; k < K; ++k) {
    const uint64_t i = (t * K + k) % npts;
    if (G) {
      st(accx, k * T + t, ld(pts, i));
      st(accy, k * T + t, ld(pts + 4 * npts, i));
    } else {
      rx[k] = ld(pts, i);
      ry[k] = ld(pts + 4 * npts, i);
    }
  }
  for (int rd = 1; rd <= rounds; ++rd) {
    // forward: d_k = xQ - xP, prefix products
    U256 acc = Fq::to_mont(Fq::one_plain());
    for (int k = 0; k < K; ++k) {
      const uint64_t i = (t * K + k + (uint64_t)rd * T * K) % npts;
      const U256 xq = ld(pts, i);
      const U256 xp = G ? ld(accx, k * T + t) : rx[k];
      if (G) st(pre, k * T + t, acc); else rp[k] = acc;
      acc = Fq::mul_tp(acc, Fq::sub(xq, xp));
    }
    U256 inv = fq_inv(acc);
    // backward: 1 / d_k, lambda, the sum
    for (int k = K - 1; k >= 0; --k) {
      const uint64_t i = (t * K + k + (uint64_t)rd * T * K) % npts;
      const U256 xq = ld(pts, i), yq = ld(pts + 4 * npts, i);
      const U256 xp = G ? ld(accx, k * T + t) : rx[k];
      const U256 yp = G ? ld(accy, k * T + t) : ry[k];
      const U256 d = Fq::sub(xq, xp);
      const U256 dinv = Fq::mul_tp(inv, G ? ld(pre, k * T + t) : rp[k]);
      inv = Fq::mul_tp(inv, d);
      const U256 lam = Fq::mul_tp(Fq::sub(yq, yp), dinv);
      const U256 x3 = Fq::sub(Fq::sub(Fq::mul_tp(lam, lam), xp), xq);
      const U256 y3 = Fq::sub(Fq::mul_tp(lam, Fq::sub(xp, x3)), yp);
      if (G) {
        st(accx, k * T + t, x3);
        st(accy, k * T + t, y3);
      } else {
        rx[k] = x3;
        ry[k] = y3;
      }
    }
  }
  st(out, t, G ? ld(accx, t) : rx[0]);
}

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } \
  } while (0)

template <int K, bool G>
static int run_affine(const uint64_t* pts, uint64_t npts, uint64_t T, int rounds, uint64_t* ax, uint64_t* ay,
                      uint64_t* pre, uint64_t* out) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_affine<K, G>), dim3(T / 256), dim3(256), 0, 0, pts, npts, 1, ax, ay, pre, out);  // warm-up
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((k_affine<K, G>), dim3(T / 256), dim3(256), 0, 0, pts, npts, rounds, ax, ay, pre, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double adds = (double)T * K * rounds;
  printf("affine batch K=%3d %s  threads %7llu  %8.3f ms  %.3e additions/s  (%.2f products/addition modelled)\n", K,
         G ? "global" : "regs  ", (unsigned long long)T, ms, adds / (ms / 1e3), 6.0 + 380.0 / K);
  return 0;
}

int main() {
  const uint64_t npts = 1 << 20;
  std::vector<uint64_t> h(8 * npts);
  uint64_t s = 0x12345678ull;
  for (auto& v : h) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    v = s;
  }
  for (uint64_t i = 0; i < 2 * npts; ++i) h[4 * i + 3] &= 0x0FFFFFFFFFFFFFFFull;  // below q
  uint64_t *pts, *out, *ax, *ay, *pre;
  const uint64_t Tmax = 1 << 20;
  CK(hipMalloc(&pts, h.size() * 8));
  CK(hipMemcpy(pts, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, Tmax * 32));
  CK(hipMalloc(&ax, (size_t)64 * 65536 * 32 * 2));  // K x T planes, K*T <= 2^22
  CK(hipMalloc(&ay, (size_t)64 * 65536 * 32 * 2));
  CK(hipMalloc(&pre, (size_t)64 * 65536 * 32 * 2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  {
    const uint64_t T = 1 << 18;
    const int M = 64;
    hipLaunchKernelGGL(k_xyzz, dim3(T / 256), dim3(256), 0, 0, pts, npts, 4, out);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_xyzz, dim3(T / 256), dim3(256), 0, 0, pts, npts, M, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("xyzz madd_tp            threads %7llu  %8.3f ms  %.3e additions/s  (10 products/addition)\n",
           (unsigned long long)T, ms, (double)T * M / (ms / 1e3));
  }
  if (run_affine<4, false>(pts, npts, 1 << 18, 16, ax, ay, pre, out)) return 1;
  if (run_affine<8, false>(pts, npts, 1 << 17, 16, ax, ay, pre, out)) return 1;
  if (run_affine<16, true>(pts, npts, 1 << 18, 8, ax, ay, pre, out)) return 1;
  if (run_affine<64, true>(pts, npts, 1 << 16, 8, ax, ay, pre, out)) return 1;
  if (run_affine<128, true>(pts, npts, 1 << 15, 8, ax, ay, pre, out)) return 1;
  if (run_affine<256, true>(pts, npts, 1 << 14, 8, ax, ay, pre, out)) return 1;
  CK(hipDeviceSynchronize());
  return 0;
}
