// One-sweep radix sort against the three-kernel passes (gfx950, round 6): the MSM's digit sorts
// (csrc/msm_sort.hpp) as the library calls them, from planar digit codes (pass 1 derives key and
// value from the code and the entry index):
//   fx22: fixed-base MSM of 2^24 points, 22-bit windows (12 windows, 32-bit codes, 22 key bits:
//         passes of 8, 7, 7 bits)
//   fx16: fixed-base MSM of 2^20 points, 16-bit windows (16 windows, 16-bit codes, 16 key bits)
//   win:  windowed MSM of 2^20 points (16 windows, key = 2^15 w + |d| - 1, 20 key bits)
// Codes are uniform signed digits with ~1/64 no-entry codes. Each form's output (keys and
// values) must equal the three-kernel sort's, word for word; prints the time of each.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 sort_os_bench.hip -o sort_os_bench
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include "sort_os.hpp"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

namespace pbf {
uint32_t rs_os_next_epoch() {
  static std::atomic<uint32_t> e{0};
  uint32_t v = (e.fetch_add(1) % 0x7FFFFFFEu) + 1;
  return v;
}
}  // namespace pbf

template <typename C>
__global__ void k_codes(C* dig, uint64_t m, uint32_t mag_bits) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x5EED0006ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const bool none = (z >> 58) == 0;  // 1 / 64
    const uint32_t mag = (uint32_t)z & ((1u << mag_bits) - 1), neg = (uint32_t)(z >> 40) & 1;
    dig[i] = none ? (C)pbf::rs_none<C>() : (C)(mag | (neg ? pbf::rs_sign<C>() : 0u));
  }
}

template <typename C>
struct Case {
  const char* name;
  uint32_t n, nw, kbits, mag_bits, kw, zkey;
};

template <typename C>
static bool run_case(const Case<C>& cs, int reps) {
  const uint64_t m = (uint64_t)cs.n * cs.nw;
  C* dig;
  uint32_t *k1, *v1, *k2, *v2, *ko, *vo, *rk, *rv, *hist, *small;
  uint64_t* status;
  const uint64_t ntiles = (m + pbf::RS_TILE - 1) / pbf::RS_TILE;
  CK(hipMalloc(&dig, sizeof(C) * m));
  CK(hipMalloc(&k1, 4 * m));
  CK(hipMalloc(&v1, 4 * m));
  CK(hipMalloc(&k2, 4 * m));
  CK(hipMalloc(&v2, 4 * m));
  CK(hipMalloc(&ko, 4 * m));
  CK(hipMalloc(&vo, 4 * m));
  CK(hipMalloc(&rk, 4 * m));
  CK(hipMalloc(&rv, 4 * m));
  CK(hipMalloc(&hist, 4 * (256 * ntiles + 256)));
  CK(hipMalloc(&small, pbf::RS_OS_SMALL_BYTES));
  CK(hipMalloc(&status, pbf::rs_os_status_bytes(m)));
  CK(hipMemset(status, 0, pbf::rs_os_status_bytes(m)));
  hipLaunchKernelGGL(k_codes<C>, dim3(4096), dim3(256), 0, 0, dig, m, cs.mag_bits);
  CK(hipDeviceSynchronize());
  const pbf::RsDigitsT<C> dg{dig, cs.n, cs.n, 0, cs.kw, cs.zkey, 0x80000000u};
  const int np = pbf::rs_passes(cs.kbits);
  int widths[3];
  for (int p = 0; p < np; ++p) widths[p] = pbf::rs_width(cs.kbits, p);
  auto old_sort = [&]() {
    pbf::rs_pass<pbf::RS_ITEMS, true, C>(nullptr, nullptr, k1, v1, (uint32_t)m, 0, hist, 0, dg, widths[0]);
    if (np == 2) {
      pbf::rs_pass<pbf::RS_ITEMS>(k1, v1, rk, rv, (uint32_t)m, widths[0], hist, 0, pbf::RsDigits{}, widths[1]);
    } else {
      pbf::rs_pass<pbf::RS_ITEMS>(k1, v1, k2, v2, (uint32_t)m, widths[0], hist, 0, pbf::RsDigits{}, widths[1]);
      pbf::rs_pass<pbf::RS_ITEMS>(k2, v2, rk, rv, (uint32_t)m, widths[0] + widths[1], hist, 0, pbf::RsDigits{},
                                  widths[2]);
    }
  };
  auto new_sort = [&]() {
    CK((pbf::rs_os_sort<pbf::RS_ITEMS, true, C>(nullptr, nullptr, k1, v1, k2, v2, ko, vo, (uint32_t)m, np, widths,
                                                 small, status, 0, dg)));
  };
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](auto fn) {
    fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    return ms / reps;
  };
  const float t_old = timeit(old_sort);
  const float t_new = timeit(new_sort);
  const float t_old2 = timeit(old_sort);
  const float t_new2 = timeit(new_sort);
  uint32_t err = 0;
  CK(hipMemcpy(&err, small + pbf::RS_OS_REP * pbf::RS_OS_MAXP * 256 + pbf::RS_OS_ERR, 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> a1(m), a2(m), b1(m), b2(m);
  CK(hipMemcpy(a1.data(), rk, 4 * m, hipMemcpyDeviceToHost));
  CK(hipMemcpy(a2.data(), rv, 4 * m, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b1.data(), ko, 4 * m, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b2.data(), vo, 4 * m, hipMemcpyDeviceToHost));
  bool sorted = true;
  for (uint64_t i = 1; i < m && sorted; ++i) sorted = a1[i - 1] <= a1[i];
  const bool same = a1 == b1 && a2 == b2;
  printf("%-5s m=%llu passes=%d  three-kernel %.3f / %.3f ms  one-sweep %.3f / %.3f ms  sorted=%d same=%d err=%u\n",
         cs.name, (unsigned long long)m, np, t_old, t_old2, t_new, t_new2, sorted, same, err);
  fflush(stdout);
  CK(hipFree(dig));
  for (uint32_t* p : {k1, v1, k2, v2, ko, vo, rk, rv, hist, small}) CK(hipFree(p));
  CK(hipFree(status));
  return sorted && same && err == 0;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  bool ok = true;
  ok &= run_case(Case<uint16_t>{"fx16", 1u << 20, 16, 16, 15, 0, 1u << 15}, reps);
  ok &= run_case(Case<uint16_t>{"win", 1u << 20, 16, 20, 15, 1u << 15, 16u << 15}, reps);
  ok &= run_case(Case<uint32_t>{"fx22", 1u << 24, 12, 22, 21, 0, 1u << 21}, reps);
  return ok ? 0 : 1;
}
