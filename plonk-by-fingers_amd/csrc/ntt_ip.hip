// Round-3 Goldilocks NTT schedule (ntt_ip.hpp): kernel instantiation and launcher, in a
// translation unit of its own (the build compiles it in parallel with ntt_launch.hip).
#include <cstdlib>
#include <cstring>
#include "internal.hpp"
#include "ntt_ip.hpp"

namespace pbf {

uint32_t persistent_grid(const void* fn, int nt, uint64_t tiles);  // ntt_launch.hip
int ip_tile_of(int r);
int ip_w(int r);

// ---- round-3 schedule launcher (ntt_ip.hpp) --------------------------------------------
typedef void (*IpFn)(IpArgs);
template <int R, int E>
static IpFn ip_fn_r(int kind, bool split) {
  constexpr int T = R >= 10 ? 8192 : 4096;
  if (kind == 0) return ntt_ip_kernel<R, E, 0, T, false>;
  if (kind == 1) return ntt_ip_kernel<R, E, 1, T, false>;
  return split ? ntt_ip_kernel<R, E, 2, T, true> : ntt_ip_kernel<R, E, 2, T, false>;
}
template <int E>
static IpFn ip_fn_e(int r, int kind, bool split) {
  switch (r) {
    case 6: return ip_fn_r<6, E>(kind, split);
    case 7: return ip_fn_r<7, E>(kind, split);
    case 8: return ip_fn_r<8, E>(kind, split);
    case 9: return ip_fn_r<9, E>(kind, split);
    case 10: return ip_fn_r<10, E>(kind, split);
    default: return nullptr;
  }
}

int run_ip(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                  hipStream_t stream) {
  const size_t P = p.ip_r.size();
  int rc = s0.ensure(batch * p.n * 8);
  if (rc) return rc;
  uint64_t* S = (uint64_t*)s0.p;
  std::vector<int> lo(P);
  {
    int l = (int)p.log_n;
    for (size_t i = 0; i < P; ++i) { l -= p.ip_r[i]; lo[i] = l; }
  }
  for (size_t i = 0; i < P; ++i) {
    const int r = p.ip_r[i];
    const int kind = i == 0 ? 0 : (i + 1 == P ? 2 : 1);
    const bool split = kind == 2 && p.ip_twa;
    IpFn fn = p.e64 == 39 ? ip_fn_e<39>(r, kind, split) : ip_fn_e<153>(r, kind, split);
    if (!fn) return fail(1, "no round-3 NTT kernel for this radix");
    const int tile = ip_tile_of(r), W = ip_w(r);
    IpArgs a;
    memset(&a, 0, sizeof(a));
    a.in = i == 0 ? d_in : S;
    a.out = i + 1 == P ? d_out : S;
    a.tw = (const uint64_t*)p.ip_tw[i]->p;
    a.twa = split ? (const uint64_t*)p.ip_twa->p : nullptr;
    a.tc = (const uint64_t*)p.ip_tc[i]->p;
    a.pitch_in = a.pitch_out = p.n;
    a.blocks = (uint32_t)((p.n >> r) / (uint64_t)W);
    a.batch = (uint32_t)batch;
    const uint64_t tiles = (uint64_t)a.blocks * batch;
    if (tiles > 0x7fffffffull) return fail(1, "batch too large");
    a.tiles = (uint32_t)tiles;
    a.xcd = (tiles % 8 == 0 && !getenv("PBF_NTT_NO_XCD")) ? 1 : 0;
    if (kind < 2) {
      a.lo = (uint32_t)lo[i];
      uint32_t wl = 0;
      while ((1 << wl) < W) ++wl;
      a.ncb_log = (uint32_t)lo[i] - wl;
    } else {
      a.nd = (uint32_t)(P - 1);
      for (size_t j = 0; j + 1 < P; ++j) { a.dr[j] = (uint32_t)p.ip_r[j]; a.dlo[j] = (uint32_t)lo[j]; }
      a.out_log = p.log_n - (uint32_t)r;
    }
    // persistent grid (every resident slot once) by default; PBF_NTT_IP_GRID=0: one tile per
    // workgroup (A/B)
    const char* ge = getenv("PBF_NTT_IP_GRID");
    const uint32_t grid = (ge && atoi(ge) == 0) ? (uint32_t)tiles : persistent_grid((const void*)fn, tile / 16, tiles);
    a.prime = getenv("PBF_NTT_IP_NOPRIME") ? 0 : 1;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(tile / 16), 0, stream, a);
    PBF_HIP(hipGetLastError());
  }
  return 0;
}

}  // namespace pbf
