// Data-movement microbenchmark for the NTT pass structure (gfx950): what a workgroup that
// loads a tile, (optionally) exchanges it through LDS and stores it achieves in HBM GB/s.
// Tile = 8192 u64 (64 KiB), 512 threads, 16 elements per thread, 2 workgroups per CU.
//   mode 0: contiguous tile load -> contiguous store (streaming copy shape)
//   mode 1: mode 0 + an LDS round trip with a barrier
//   mode 2: NTT pass shape: R rows x W columns, rows n/R apart (W*8-B runs), LDS round
//           trip, contiguous stores (the first pass)
//   mode 3: mode 2 with W-element runs on the store side too (the later passes)
// VEC = 2: each lane moves 16 B (two adjacent u64) per access instead of 8 B.
// Build: hipcc -O3 --offload-arch=gfx950 tile_copy.hip -o tile_copy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int NT = 512, PER = 16, TILE = NT * PER;

struct u64x2 {
  uint64_t a, b;
};

template <int MODE, int W, int VEC>
__global__ void __launch_bounds__(NT) k_tile(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t pad, uint64_t pstride) {
  __shared__ uint64_t lds[TILE + 64];
  constexpr int R = TILE / W;
  constexpr int PV = PER / VEC;  // accesses per thread
  const uint64_t tiles_per_poly = n / TILE;
  const uint64_t poly = blockIdx.x / tiles_per_poly, kb = blockIdx.x % tiles_per_poly;
  const uint64_t* src = in + poly * pstride;
  uint64_t* dst = out + poly * pstride;
  const uint64_t rs = n / R + pad;  // row stride (pad: breaks power-of-two strides)
  const int t = threadIdx.x;
  uint64_t v[PER];
  // element e = VEC * (t + NT * u) + c: column w = e % W, row r = e / W
#pragma unroll
  for (int u = 0; u < PV; ++u) {
    const int e = VEC * (t + NT * u);
    const uint64_t off = MODE <= 1 ? kb * TILE + e : kb * W + e % W + (uint64_t)(e / W) * rs;
    if constexpr (VEC == 2) {
      const u64x2 x = *(const u64x2*)(src + off);
      v[2 * u] = x.a;
      v[2 * u + 1] = x.b;
    } else {
      v[u] = src[off];
    }
  }
  if constexpr (MODE >= 1) {
#pragma unroll
    for (int u = 0; u < PER; ++u) lds[(t * VEC + (u % VEC)) + NT * VEC * (u / VEC)] = v[u] ^ 0x55;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int m = (t * VEC + (u % VEC)) + NT * VEC * (u / VEC);
      v[u] = lds[(m % R) * W + m / R];
    }
  }
#pragma unroll
  for (int u = 0; u < PV; ++u) {
    const int e = VEC * (t + NT * u);
    const uint64_t off = MODE <= 2 ? kb * TILE + e : kb * W + e % W + (uint64_t)(e / W) * rs;
    if constexpr (VEC == 2) {
      *(u64x2*)(dst + off) = u64x2{v[2 * u], v[2 * u + 1]};
    } else {
      dst[off] = v[u];
    }
  }
}

template <int MODE, int W, int VEC>
static void run(const char* name, const uint64_t* in, uint64_t* out, uint64_t n, int batch, uint64_t pad = 0) {
  const uint64_t pstride = pad ? 2 * n : n;
  const uint64_t blocks = (n / TILE) * batch;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_tile<MODE, W, VEC>), dim3(blocks), dim3(NT), 0, 0, in, out, n, pad, pstride);
  hipDeviceSynchronize();
  const int reps = 20;
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_tile<MODE, W, VEC>), dim3(blocks), dim3(NT), 0, 0, in, out, n, pad, pstride);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = 16.0 * n * batch;
  printf("n=2^%d b%d pad %4llu %-50s %8.1f us  %7.1f GB/s\n", __builtin_ctzll(n), batch, (unsigned long long)pad, name, ms * 1e3 / reps, bytes / (ms / reps * 1e-3) / 1e9);
}

int main() {
  const uint64_t n = 1 << 20;
  const int batch = 32;
  uint64_t *in, *out;
  hipMalloc(&in, n * batch * 8);
  hipMalloc(&out, n * batch * 8);
  hipMemset(in, 1, n * batch * 8);
  run<0, 8, 1>("contiguous copy 8B/lane", in, out, n, batch);
  run<0, 8, 2>("contiguous copy 16B/lane", in, out, n, batch);
  run<1, 8, 1>("contiguous + LDS round trip 8B/lane", in, out, n, batch);
  run<1, 8, 2>("contiguous + LDS round trip 16B/lane", in, out, n, batch);
  run<2, 8, 1>("strided W=8 load + LDS + contiguous store, 8B", in, out, n, batch);
  run<2, 8, 2>("strided W=8 load + LDS + contiguous store, 16B", in, out, n, batch);
  run<3, 8, 1>("strided W=8 load + LDS + strided store, 8B", in, out, n, batch);
  run<3, 8, 2>("strided W=8 load + LDS + strided store, 16B", in, out, n, batch);
  run<3, 16, 1>("strided W=16 both sides, 8B", in, out, n, batch);
  run<3, 16, 2>("strided W=16 both sides, 16B", in, out, n, batch);
  run<3, 32, 2>("strided W=32 both sides, 16B", in, out, n, batch);
  run<2, 4, 1>("strided W=4 load + LDS + contiguous store, 8B", in, out, n, batch);
  run<3, 4, 1>("strided W=4 both sides, 8B", in, out, n, batch);
  run<3, 4, 2>("strided W=4 both sides, 16B", in, out, n, batch);
  run<2, 4, 2>("strided W=4 load + LDS + contiguous store, 16B", in, out, n, batch);
  // 2^24 x 2: the north-star size (rows 2^24/R apart: 256-512 KiB power-of-two strides)
  const uint64_t n24 = 1ull << 24;
  uint64_t *in2, *out2;
  hipMalloc(&in2, n24 * 2 * 2 * 8);
  hipMalloc(&out2, n24 * 2 * 2 * 8);
  hipMemset(in2, 1, n24 * 2 * 2 * 8);
  for (uint64_t pad : {0ull, 8ull, 16ull, 64ull, 520ull}) {
    run<0, 8, 1>("contiguous copy 8B/lane", in2, out2, n24, 2, pad);
    run<2, 16, 1>("strided W=16 load + LDS + contiguous store, 8B", in2, out2, n24, 2, pad);
    run<3, 16, 1>("strided W=16 both sides, 8B", in2, out2, n24, 2, pad);
    run<3, 32, 1>("strided W=32 both sides, 8B", in2, out2, n24, 2, pad);
    run<3, 8, 1>("strided W=8 both sides, 8B", in2, out2, n24, 2, pad);
  }
  for (uint64_t pad : {8ull, 64ull}) {
    run<3, 8, 1>("2^20: strided W=8 both sides, 8B", in, out, n / 2, batch, pad);
    run<3, 16, 1>("2^20: strided W=16 both sides, 8B", in, out, n / 2, batch, pad);
  }
  return 0;
}
