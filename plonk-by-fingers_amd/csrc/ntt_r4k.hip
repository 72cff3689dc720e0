// Two-pass 2^24 Goldilocks NTT kernels (ntt_r4k.hpp), in their own translation unit: the
// fully unrolled 64-point register DFTs make them the slowest kernels of the library to compile.
#include "internal.hpp"
#include "ntt_r4k.hpp"

namespace pbf {

uint32_t persistent_grid(const void* fn, int nt, uint64_t tiles);  // ntt_launch.hip

typedef void (*R4kFn)(R4kArgs);
template <int E64>
static R4kFn r4k_fn(bool first, bool persist) {
  if (persist) return first ? ntt_r4k_pkernel<E64, true> : ntt_r4k_pkernel<E64, false>;
  return first ? ntt_r4k_kernel<E64, true> : ntt_r4k_kernel<E64, false>;
}

// one pass; `persist`: the pipelined persistent kernel (grid = resident workgroups)
int launch_r4k_pass(const R4kArgs& a, bool first, int e64, uint32_t tiles, bool persist, hipStream_t stream) {
  if (e64 != 39 && e64 != 153) return fail(1, "two-pass 2^24 plan needs a standard Goldilocks root");
  const R4kFn fn = e64 == 39 ? r4k_fn<39>(first, persist) : r4k_fn<153>(first, persist);
  const uint32_t grid = persist ? persistent_grid((const void*)fn, R4K_NT, tiles) : tiles;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(R4K_NT), 0, stream, a);
  PBF_HIP(hipGetLastError());
  return 0;
}

}  // namespace pbf
