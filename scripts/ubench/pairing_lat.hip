// Latency microbenchmark of the pairing kernels' building blocks on one wave (gfx950):
// cycles per dependent Fq product, Fq2 product, wave-cooperative Fq12 product and Miller
// doubling step. Build: make -C scripts/ubench; run on the GPU box: scripts/ubench/pairing_lat
#include "../../plonk-by-fingers_amd/csrc/pairing.hip"
#include <cstdio>

using namespace pbf;

// the two rounds of w_mul<W_DENSE> separately (copies of its halves)
__device__ __forceinline__ void r1_dense(const Fq2* x, const Fq2* y, PL& L, int tid) {
  if (tid < 108) {
    const int q = tid / 3, r = tid - 3 * q, i = q / 6, jj = q - 6 * i;
    const Fq2& xa = x[i + (i + jj >= 6 ? 6 : 0)];
    L.t[tid] = Fq::mul(kara_raw(xa, r), kara_raw(y[jj], r));
  }
  bsync();
}
__device__ __forceinline__ void r2_dense(Fq2* dst, PL& L, int tid) {
  const int wv = tid >> 6, k = tid & 63;
  if (k < 6) {
    L9 s[3];
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
    L9 v = s[wv & 1];
    l9_add_kq<108>(v);
    l9_sub(v, s[2]);
    const U256 r = l9_reduce(v);
    Fq2& d = dst[k + (wv >> 1) * 6];
    if (wv & 1) d.c1 = r; else d.c0 = r;
  }
  bsync();
}

__global__ void __launch_bounds__(PT) k_lat(int what, int iters, const uint64_t* seed, uint64_t* out, PairingConsts k) {
  __shared__ PL L;
  const int lane = threadIdx.x;
  load_consts(k, L, lane);
  U256 x = Fq::to_mont(u256_from_u64(seed)), y = Fq::to_mont(u256_from_u64(seed + 4));
  Fq2 a{x, y}, b{y, x};
  if (lane < 12) {
    L.reg[0][lane] = Fq2{x, y};
    L.reg[1][lane] = Fq2{y, x};
    L.reg[2][lane] = Fq2{y, y};
  }
  for (int e = lane; e < NSTEP * 12; e += PT) (&L.le[0][0])[e] = Fq2{x, y};
  if (lane < 26) L.sl[lane] = Fq2{x, y};
  __syncthreads();
  uint64_t t0 = clock64(), w0 = wall_clock64();
  switch (what) {
    case 0: for (int i = 0; i < iters; ++i) x = Fq::mul(x, y); break;
    case 1: for (int i = 0; i < iters; ++i) a = f2_mul(a, b); break;
    case 2: for (int i = 0; i < iters; ++i) w_mul<W_DENSE>(L.reg[0], L.reg[0], L.reg[1], L, lane); break;
    case 3: for (int i = 0; i < iters; ++i) w_mul<W_FIVE>(L.reg[0], L.reg[0], L.reg[1], L, lane); break;
    case 4: for (int i = 0; i < iters; ++i) w_mul<W_LINE>(L.reg[0], L.reg[0], L.reg[1], L, lane); break;
    case 5: for (int i = 0; i < iters; ++i) x = Fq::add(x, y); break;
    case 9: for (int i = 0; i < iters; ++i) { if (lane == 0) fq6_inv_flat(L.reg[2], k); bsync(); } break;
    case 10: for (int i = 0; i < iters; ++i) final_exp_w(k, L, lane); break;
    case 11: for (int i = 0; i < iters; ++i) pair_line_products(L, lane); break;
    case 12: for (int i = 0; i < iters; ++i) bsync(); break;
    case 13: for (int i = 0; i < iters; ++i) { if (lane < 64) x = Fq::mul(x, y); bsync(); } break;
    case 14: for (int i = 0; i < iters; ++i) w_frob1(L.reg[0], L.reg[0], L, lane); break;
    case 16: for (int i = 0; i < iters; ++i) { x = Fq::mul(x, y); bsync(); } break;
    case 17: for (int i = 0; i < iters; ++i) { if (lane < 128) x = Fq::mul(x, y); bsync(); } break;
    case 18: for (int i = 0; i < iters; ++i) r1_dense(L.reg[0], L.reg[1], L, lane); break;
    case 19: for (int i = 0; i < iters; ++i) r2_dense(L.reg[0], L, lane); break;
    case 20: {  // the waves' hardware ids: SIMD of each wave (HW_ID bits 5:4 on gfx9)
      uint32_t hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      if ((lane & 63) == 0) L.t[lane >> 6].w[0] = hw;
      bsync();
      if (lane == 0) x.w[0] = (L.t[0].w[0] >> 4 & 3) | (L.t[1].w[0] >> 4 & 3) << 4 | (L.t[2].w[0] >> 4 & 3) << 8 | (L.t[3].w[0] >> 4 & 3) << 12;
      break;
    }
    case 21: case 22: case 23: case 24: {  // G1 XYZZ chains on one wave: quad add / quad dbl / lane add / lane dbl
      const U256 one = Fq::to_mont(Fq::one_plain());
      Xyzz P{x, y, one, one}, Q{y, x, one, one};
      for (int i = 0; i < iters; ++i) {
        if (what == 21) P = G1Quad::add(P, Q);
        else if (what == 22) P = G1Quad::dbl(P);
        else if (what == 23) P = G1::add2(P, Q);
        else P = G1::dbl2(P);
      }
      x = P.X;
      break;
    }
    case 15: {
      L9 v = l9_of(x);
      for (int i = 0; i < iters; ++i) { l9_add_kq<100>(v); x = l9_reduce(v); v = l9_of(x); }
      break;
    }
    case 6: {  // one dependent v_mad_u64_u32 chain
      uint64_t acc = x.w[0];
      for (int i = 0; i < iters; ++i) acc = (uint64_t)(uint32_t)acc * y.w[1] + (acc >> 7);
      x.w[0] = (uint32_t)acc;
      break;
    }
    case 7: {  // four independent chains
      uint64_t a0 = x.w[0], a1 = x.w[1], a2 = x.w[2], a3 = x.w[3];
      for (int i = 0; i < iters; i += 4) {
        a0 = (uint64_t)(uint32_t)a0 * y.w[1] + (a0 >> 7);
        a1 = (uint64_t)(uint32_t)a1 * y.w[2] + (a1 >> 7);
        a2 = (uint64_t)(uint32_t)a2 * y.w[3] + (a2 >> 7);
        a3 = (uint64_t)(uint32_t)a3 * y.w[4] + (a3 >> 7);
      }
      x.w[0] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3);
      break;
    }
    default: {  // one dependent 32-bit add-with-carry chain
      uint32_t c = x.w[0];
      for (int i = 0; i < iters; ++i) c = c * 3u + y.w[1];
      x.w[0] = c;
      break;
    }
  }
  uint64_t t1 = clock64(), w1 = wall_clock64();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = w1 - w0;
    out[2] = what == 20 ? x.w[0] : (x.w[0] ^ a.c0.w[0] ^ L.reg[0][0].c0.w[0]);
  }
}

// throughput: every lane of a full grid runs two independent chains of Fq products
__global__ void __launch_bounds__(256) k_tput(int iters, const uint64_t* seed, uint64_t* out) {
  U256 x = u256_from_u64(seed), y = u256_from_u64(seed + 4), z = x;
  x.w[0] ^= threadIdx.x;
  z.w[1] ^= blockIdx.x;
  for (int i = 0; i < iters; ++i) {
    x = Fq::mul(x, y);
    z = Fq::mul(z, y);
  }
  if ((x.w[0] ^ z.w[0]) == 0x12345u) out[3] = 1;  // keeps the chains live
}

int main() {
  uint64_t *d_seed, *d_out, h[3];
  uint64_t seed[8] = {0x1234567, 0x89abcdef, 0x5555, 0x1000, 0x7777, 0x3333, 0x2222, 0x100};
  hipMalloc(&d_seed, 64);
  hipMalloc(&d_out, 64);
  hipMemcpy(d_seed, seed, 64, hipMemcpyHostToDevice);
  int wclk = 0;
  hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);  // kHz
  const char* names[] = {"fq_mul", "fq2_mul", "w_mul dense", "w_mul five", "w_mul line", "fq_add", "mad_u64_dep",
                         "mad_u64_x4", "mul_add_u32_dep", "fq6_inv_flat", "final_exp_w", "pair_line_products",
                         "barrier", "fq_mul+barrier", "w_frob1", "l9_reduce", "fq_mul x4 waves", "fq_mul x2 waves",
                         "w_mul round1", "w_mul round2", "(hw id)", "G1Quad::add", "G1Quad::dbl", "G1::add2 (lane)",
                         "G1::dbl2 (lane)"};
  const int iters[] = {4096, 2048, 256, 256, 256, 4096, 65536, 65536, 65536, 16, 2, 8, 4096, 1024, 256, 1024, 1024, 1024, 256, 256, 1, 128, 128, 128, 128};
  for (int w = 0; w < 25; ++w) {
    if (w == 20) continue;
    for (int rep = 0; rep < 2; ++rep) {  // first launch warms the code
      hipLaunchKernelGGL(k_lat, dim3(1), dim3(PT), 0, 0, w, iters[w], d_seed, d_out, make_consts());
      hipMemcpy(h, d_out, 24, hipMemcpyDeviceToHost);
    }
    printf("%-18s %10.1f cycles  %8.3f us   per op\n", names[w], (double)h[0] / iters[w],
           (double)h[1] / iters[w] * 1e3 / wclk);
  }
  hipLaunchKernelGGL(k_lat, dim3(1), dim3(PT), 0, 0, 20, 1, d_seed, d_out, make_consts());
  hipMemcpy(h, d_out, 24, hipMemcpyDeviceToHost);
  printf("SIMD of waves 0..3 (4 bits each): %04llx\n", (unsigned long long)(h[2] & 0xffff));
  {
    const int blocks = 256 * 8, iters = 256;  // 8 workgroups (32 waves) per CU
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k_tput, dim3(blocks), dim3(256), 0, 0, iters, d_seed, d_out);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double muls = 2.0 * iters * blocks * 256;
      printf("fq_mul throughput   %.3f ms  %.3e Fq products/s\n", ms, muls / (ms * 1e-3));
    }
  }
  return 0;
}
