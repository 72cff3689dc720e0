// Radix-sort microbenchmark (gfx950): the MSM's stable LSD sort (csrc/msm_sort.hpp) of m
// (key, value) u32 pairs by 16 key bits, as the fixed-base MSM calls it (keys uniform over
// the 2^15 + 1 bucket ids, values = entry index), at several tile sizes. Reports the
// per-sort time and the rate over the bytes one sort moves at least (per pass: keys read
// twice (histogram + scatter), values read once, both written once: 20 B per entry).
// Every variant's output is compared with the first one's (same stable order).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 sort_bench.hip -o sort_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include "../../plonk-by-fingers_amd/csrc/msm_sort.hpp"

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void k_fill(uint32_t* keys, uint32_t* vals, uint32_t m) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + 0x5EED0004ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    keys[i] = (uint32_t)(z % 32769u);
    vals[i] = i;
  }
}

template <int ITEMS>
static double run(uint32_t m, const uint32_t* k, const uint32_t* v, uint32_t* k2, uint32_t* v2, uint32_t* tk,
                  uint32_t* tv, uint32_t* hist, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  pbf::rs_sort<ITEMS>(k, v, k2, v2, tk, tv, m, 16, hist, 0);
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) pbf::rs_sort<ITEMS>(k, v, k2, v2, tk, tv, m, 16, hist, 0);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms / reps;
}

int main(int argc, char** argv) {
  const int logm = argc > 1 ? atoi(argv[1]) : 24;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const uint32_t m = 1u << logm;
  uint32_t *k, *v, *k2, *v2, *tk, *tv, *hist;
  CK(hipMalloc(&k, 4ull * m));
  CK(hipMalloc(&v, 4ull * m));
  CK(hipMalloc(&k2, 4ull * m));
  CK(hipMalloc(&v2, 4ull * m));
  CK(hipMalloc(&tk, 4ull * m));
  CK(hipMalloc(&tv, 4ull * m));
  CK(hipMalloc(&hist, 4ull * (256ull * (m / pbf::RS_TILE + 1) + 256)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, k, v, m);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> ref_k(m), ref_v(m), got_k(m), got_v(m);
  const double bytes = 2.0 * 20.0 * m;
  auto check = [&](const char* name, double ms, bool first) {
    CK(hipMemcpy(got_k.data(), k2, 4ull * m, hipMemcpyDeviceToHost));
    CK(hipMemcpy(got_v.data(), v2, 4ull * m, hipMemcpyDeviceToHost));
    bool ok = true;
    if (first) {
      for (uint32_t i = 1; i < m && ok; ++i)
        ok = got_k[i - 1] < got_k[i] || (got_k[i - 1] == got_k[i] && got_v[i - 1] < got_v[i]);
      ref_k = got_k;
      ref_v = got_v;
    } else {
      ok = got_k == ref_k && got_v == ref_v;
    }
    printf("m=2^%d %-10s %8.3f ms  %7.1f GB/s  %s\n", logm, name, ms, bytes / ms / 1e6, ok ? "ok" : "MISMATCH");
    fflush(stdout);
    return ok;
  };
  bool ok = check("items16", run<16>(m, k, v, k2, v2, tk, tv, hist, reps), true);
  ok &= check("items24", run<24>(m, k, v, k2, v2, tk, tv, hist, reps), false);
  ok &= check("items32", run<32>(m, k, v, k2, v2, tk, tv, hist, reps), false);
  ok &= check("items16", run<16>(m, k, v, k2, v2, tk, tv, hist, reps), false);
  return ok ? 0 : 1;
}
