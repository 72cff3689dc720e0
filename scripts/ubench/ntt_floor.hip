// Data-movement floor of candidate 2^24-point NTT pass schedules (gfx950), round 3.
// Every "pass" moves one polynomial's (or a batch's) 2^24 u64 through tiles of 4096
// elements exactly as an NTT pass of that schedule would -- same global addresses on both
// sides, one LDS round trip per tile -- but computes nothing, so the chain time is the
// floor the memory system sets for that schedule. Schedules:
//   stockham3  the round-2 plan: 3 out-of-place radix-2^8 Stockham passes in->s0->s1->out
//   inplace3   radix-2^8 passes that write back where they read (digit slots replaced by
//              output digits), one scratch S: in->S, S->S, S->out (the last pass writes the
//              natural-order output)
//   inplace4   the same with 4 radix-2^6 passes (512-B runs everywhere)
// each per polynomial (chain of one polynomial, then the next: its scratch can stay in the
// 256 MiB Infinity Cache) or batched (every pass over both polynomials).
// Build: hipcc -O3 --offload-arch=gfx950 ntt_floor.hip -o ntt_floor
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

struct Side {
  uint64_t ia, ib;   // tile base = a*ia + b*ib
  uint32_t run_log;  // element e of the tile: row e >> run_log, offset e & (run-1)
  uint64_t rs;       // row stride (elements)
};
struct Pass {
  const uint64_t* in;
  uint64_t* out;
  uint32_t A;  // tile t -> (a, b) = (t % A, t / A)
  uint32_t tiles;  // per polynomial
  uint32_t polys;  // polynomials per launch, `pstride` elements apart
  uint64_t pstride;
  Side si, so;
  int nt_in, nt_out, xcd;
};

constexpr int NT = 256, PER = 16, TILE = NT * PER;

__global__ void __launch_bounds__(NT) k_move(Pass p) {
  __shared__ uint64_t lds[64 * 65];
  uint32_t t = blockIdx.x;
  const uint32_t total = p.tiles * p.polys;
  if (p.xcd) t = (t & 7) * (total >> 3) + (t >> 3);  // XCD x takes a contiguous range
  const uint64_t poly = t / p.tiles;
  t %= p.tiles;
  const uint64_t a = t % p.A, b = t / p.A;
  const uint64_t bi = a * p.si.ia + b * p.si.ib + poly * p.pstride, bo = a * p.so.ia + b * p.so.ib + poly * p.pstride;
  const uint32_t mi = (1u << p.si.run_log) - 1, mo = (1u << p.so.run_log) - 1;
  uint64_t v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const uint32_t e = threadIdx.x + NT * u;
    const uint64_t* src = p.in + bi + (uint64_t)(e >> p.si.run_log) * p.si.rs + (e & mi);
    v[u] = p.nt_in ? __builtin_nontemporal_load(src) : *src;
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const uint32_t e = threadIdx.x + NT * u;
    lds[(e >> 6) * 65 + (e & 63)] = v[u];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const uint32_t f = threadIdx.x + NT * u;  // transposed read: a real pass's exchange
    v[u] = lds[(f & 63) * 65 + (f >> 6)];
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const uint32_t f = threadIdx.x + NT * u;
    uint64_t* dst = p.out + bo + (uint64_t)(f >> p.so.run_log) * p.so.rs + (f & mo);
    if (p.nt_out)
      __builtin_nontemporal_store(v[u], dst);
    else
      *dst = v[u];
  }
}

static const uint64_t N = 1ull << 24;

static Pass mk(const uint64_t* in, uint64_t* out, uint32_t A, uint32_t tiles, Side si, Side so) {
  Pass p;
  p.in = in; p.out = out; p.A = A; p.tiles = tiles; p.si = si; p.so = so;
  p.nt_in = p.nt_out = 0; p.xcd = 0; p.polys = 1; p.pstride = 0;
  return p;
}

// one polynomial (offset already applied to the pointers)
static std::vector<Pass> stockham3(const uint64_t* in, uint64_t* s0, uint64_t* s1, uint64_t* out) {
  return {mk(in, s0, 4096, 4096, {16, 0, 4, 1ull << 16}, {4096, 0, 8, 256}),
          mk(s0, s1, 16, 4096, {16, 256, 4, 1ull << 16}, {16, 1ull << 16, 4, 256}),
          mk(s1, out, 4096, 4096, {16, 0, 4, 1ull << 16}, {16, 0, 4, 1ull << 16})};
}
static std::vector<Pass> inplace3(const uint64_t* in, uint64_t* S, uint64_t* out) {
  return {mk(in, S, 4096, 4096, {16, 0, 4, 1ull << 16}, {16, 0, 4, 1ull << 16}),
          mk(S, S, 16, 4096, {16, 1ull << 16, 4, 256}, {16, 1ull << 16, 4, 256}),
          mk(S, out, 16, 4096, {1ull << 20, 256, 8, 1ull << 16}, {16, 256, 4, 1ull << 16})};
}
static std::vector<Pass> inplace4(const uint64_t* in, uint64_t* S, uint64_t* out) {
  return {mk(in, S, 4096, 4096, {64, 0, 6, 1ull << 18}, {64, 0, 6, 1ull << 18}),
          mk(S, S, 64, 4096, {64, 1ull << 18, 6, 1ull << 12}, {64, 1ull << 18, 6, 1ull << 12}),
          mk(S, S, 64, 4096, {1ull << 12, 1ull << 18, 6, 64}, {1ull << 12, 1ull << 18, 6, 64}),
          mk(S, out, 64, 4096, {64, 4096, 6, 1ull << 18}, {4096, 64, 6, 1ull << 18})};
}

// two radix-2^12 passes (x = x0 + 2^12 x1): P1 over x1 (W-element runs 2^12 apart) in place,
// P2 over x0 (contiguous rows of 2^12) into natural order (W-element runs 2^12 apart). The
// real kernel's tile would be W x 4096 (W = 4: 128 KiB of LDS); here 4096-element tiles of
// W columns x 4096/W rows move the same addresses in the same order.
static std::vector<Pass> inplace2(const uint64_t* in, uint64_t* S, uint64_t* out, uint32_t wlog) {
  const uint32_t W = 1u << wlog, rows = 4096 >> wlog, groups = 4096 >> wlog;  // column groups
  const uint64_t q = (uint64_t)rows * 4096;  // one row-quarter (or 1/(W) part) of a column
  return {mk(in, S, groups, 4096, {W, q, wlog, 4096}, {W, q, wlog, 4096}),
          mk(S, out, groups, 4096, {(uint64_t)W * 4096, rows, 12 - wlog, 4096}, {W, (uint64_t)rows * 4096, wlog, 4096})};
}

static uint64_t g_limit = 0;  // elements in every buffer
// every term of an address grows with a, b, the row and the offset, so the last tile's last
// element bounds them all: refuse a pass that could leave the buffers
static uint64_t max_addr(const Pass& p, const Side& sd) {
  const uint64_t a = p.A - 1, b = p.tiles / p.A - 1, e = TILE - 1;
  return (p.polys - 1) * p.pstride + a * sd.ia + b * sd.ib + (e >> sd.run_log) * sd.rs + (e & ((1u << sd.run_log) - 1));
}
static const uint64_t* g_bufs[4];
static bool inside(const uint64_t* ptr, uint64_t last) {
  for (const uint64_t* b : g_bufs)
    if (ptr >= b && ptr < b + g_limit) return (uint64_t)(ptr - b) + last < g_limit;
  return false;
}
static void launch(const Pass& p) {
  if (p.tiles % p.A || !inside(p.in, max_addr(p, p.si)) || !inside(p.out, max_addr(p, p.so))) {
    fprintf(stderr, "pass out of bounds (tiles %u A %u): refusing to launch\n", p.tiles, p.A);
    exit(2);
  }
  hipLaunchKernelGGL(k_move, dim3(p.tiles * p.polys), dim3(NT), 0, 0, p);
}

// 2^20-point transforms (x = x0 + 2^10 x1), W-column tiles, over `polys` polynomials per launch
static std::vector<Pass> batched(std::vector<Pass> v, uint32_t polys, uint64_t n) {
  for (auto& p : v) { p.polys = polys; p.pstride = n; }
  return v;
}
static std::vector<Pass> stockham2_20(const uint64_t* in, uint64_t* s0, uint64_t* out, uint32_t wlog) {
  const uint32_t W = 1u << wlog, rows = 4096 >> wlog, groups = 1024 >> wlog;
  const uint64_t q = (uint64_t)rows * 1024;
  // P1: x[j + r 2^10] -> y[j 2^10 + k] (each column's 1024 outputs contiguous)
  // P2: x[j + r 2^10] -> y[j + k 2^10]
  return {mk(in, s0, groups, 256, {W, q, wlog, 1024}, {(uint64_t)W * 1024, rows, 12 - wlog, 1024}),
          mk(s0, out, groups, 256, {W, q, wlog, 1024}, {W, q, wlog, 1024})};
}
static std::vector<Pass> inplace2_20(const uint64_t* in, uint64_t* S, uint64_t* out, uint32_t wlog) {
  const uint32_t W = 1u << wlog, rows = 4096 >> wlog, groups = 1024 >> wlog;
  const uint64_t q = (uint64_t)rows * 1024;
  // P1 over x1 in place; P2 over x0: contiguous rows (k0 block) -> natural order X[k0 + 2^10 k1]
  return {mk(in, S, groups, 256, {W, q, wlog, 1024}, {W, q, wlog, 1024}),
          mk(S, out, groups, 256, {(uint64_t)W * 1024, rows, 12 - wlog, 1024}, {W, q, wlog, 1024})};
}

struct Sched {
  const char* name;
  std::vector<std::vector<Pass>> seq;  // launched in order (each inner vector: one chain)
};

static void timeit(const Sched& s, int reps = 20, double alg = 16.0 * (1ull << 25)) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& ch : s.seq)
    for (auto& p : ch) launch(p);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    for (auto& ch : s.seq)
      for (auto& p : ch) launch(p);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / reps;
  printf("%-44s %8.1f us per step   alg %6.0f GB/s (%.3f of 8 TB/s)\n", s.name, us, alg / (us * 1e-6) / 1e9,
         alg / (us * 1e-6) / 8e12);
  // per-pass split of the first chain
  for (size_t i = 0; i < s.seq[0].size(); ++i) {
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) {
      for (auto& ch : s.seq)
        for (size_t j = 0; j < ch.size(); ++j)
          if (j != i) launch(ch[j]);
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms2;
    hipEventElapsedTime(&ms2, e0, e1);
    printf("    without pass %zu: %8.1f us  (pass %zu ~ %6.1f us per chain set)\n", i, ms2 * 1e3 / reps, i,
           (ms - ms2) * 1e3 / reps);
  }
}

static Sched with(Sched s, int nt_in, int nt_out, int xcd, const char* name) {
  s.name = name;
  for (auto& ch : s.seq) {
    ch.front().nt_in = nt_in;
    ch.back().nt_out = nt_out;
    for (auto& p : ch) p.xcd = xcd;
  }
  return s;
}

int main() {
  uint64_t *in, *out, *s0, *s1;
  hipMalloc(&in, 2 * N * 8);
  hipMalloc(&out, 2 * N * 8);
  hipMalloc(&s0, 2 * N * 8);
  hipMalloc(&s1, 2 * N * 8);
  g_limit = 2 * N;
  g_bufs[0] = in; g_bufs[1] = out; g_bufs[2] = s0; g_bufs[3] = s1;
  hipMemset(in, 1, 2 * N * 8);
  hipMemset(s0, 0, 2 * N * 8);
  hipMemset(s1, 0, 2 * N * 8);
  hipMemset(out, 0, 2 * N * 8);
  // contiguous copy reference (2 x 2^24 in -> out); round 5: ~60 ms of it first, so every
  // figure below is taken at steady clocks (before, the first schedules ran while the clocks
  // were still rising)
  {
    Pass c = mk(in, out, 8192, 8192, {4096, 0, 12, 0}, {4096, 0, 12, 0});
    for (int w = 0; w < 600; ++w) launch(c);
    hipDeviceSynchronize();
    timeit(Sched{"copy (contiguous, both polynomials)", {{c}}});
  }
  Sched st{"stockham3 per polynomial", {stockham3(in, s0, s1, out), stockham3(in + N, s0 + N, s1 + N, out + N)}};
  timeit(st);
  Sched i3p{"inplace3 per polynomial (one 128 MiB S)", {inplace3(in, s0, out), inplace3(in + N, s0, out + N)}};
  timeit(i3p);
  timeit(with(i3p, 1, 1, 0, "inplace3 per polynomial, nt in/out"));
  timeit(with(i3p, 0, 0, 1, "inplace3 per polynomial, XCD tile ranges"));
  Sched i3b{"inplace3 two S (no reuse)", {inplace3(in, s0, out), inplace3(in + N, s0 + N, out + N)}};
  timeit(i3b);
  Sched i4p{"inplace4 per polynomial (one 128 MiB S)", {inplace4(in, s0, out), inplace4(in + N, s0, out + N)}};
  timeit(i4p);
  timeit(with(i4p, 1, 1, 0, "inplace4 per polynomial, nt in/out"));
  timeit(with(i4p, 0, 0, 1, "inplace4 per polynomial, XCD tile ranges"));
  timeit(with(i4p, 1, 1, 1, "inplace4 per polynomial, nt + XCD"));
  for (uint32_t wl : {2u, 3u}) {
    char nm[96];
    snprintf(nm, sizeof nm, "inplace2 W=%u per polynomial", 1u << wl);
    Sched i2{nm, {inplace2(in, s0, out, wl), inplace2(in + N, s0, out + N, wl)}};
    timeit(i2);
    snprintf(nm, sizeof nm, "inplace2 W=%u per polynomial, XCD tile ranges", 1u << wl);
    timeit(with(i2, 0, 0, 1, nm));
  }
  // 2^20 x 32 (the headline workload): whole batch per pass, or groups of 4 polynomials
  // chained (a group's scratch, 32 MiB, can stay in the Infinity Cache / L2)
  const uint64_t n20 = 1ull << 20;
  for (uint32_t wl : {3u, 4u}) {
    for (int grp : {32, 4}) {
      for (int kind = 0; kind < 2; ++kind) {
        Sched sc;
        char* nm = new char[96];
        snprintf(nm, 96, "2^20x32 %s W=%u groups of %d", kind ? "inplace2" : "stockham2", 1u << wl, grp);
        sc.name = nm;
        for (int g0 = 0; g0 < 32; g0 += grp) {
          const uint64_t off = (uint64_t)g0 * n20;
          sc.seq.push_back(batched(kind ? inplace2_20(in + off, s0 + off, out + off, wl)
                                        : stockham2_20(in + off, s0 + off, out + off, wl), grp, n20));
        }
        timeit(sc);
        char* nm2 = new char[96];
        snprintf(nm2, 96, "%s, XCD", nm);
        timeit(with(sc, 0, 0, 1, nm2));
      }
    }
  }
  Sched i4b{"inplace4 two S (no reuse)", {inplace4(in, s0, out), inplace4(in + N, s0 + N, out + N)}};
  timeit(i4b);
  return 0;
}
