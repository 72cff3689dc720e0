// Device-side MSM entry points shared by msm.hip and the prover (prover.hip).
#pragma once
#include "ec_bn254.hpp"
#include "internal.hpp"

namespace pbf {

// Window table (16 x n affine points, Montgomery) of the n canonical affine points at d_pts,
// cached in the context and revalidated by a fingerprint of the points (one stream sync).
int msm_fixed_table(pbf_ctx* ctx, const uint64_t* d_pts, uint64_t n, hipStream_t s, const Affine** out);
// The cached table of exactly these points (fingerprint checked), or null (nothing built).
int msm_fixed_lookup(pbf_ctx* ctx, const uint64_t* d_pts, uint64_t n, hipStream_t s, const Affine** out);
// sum_{i<n} scalars[i] * P_(first+i) against a table of n_table points; the XYZZ result
// (Montgomery) is written to *d_result by the context's side stream (see msm_fixed_wait);
// nothing on the host waits for it.
int msm_fixed_device(pbf_ctx* ctx, const Affine* table, uint64_t n_table, uint64_t first, const uint64_t* d_sc,
                     uint64_t n, hipStream_t s, Xyzz* d_result);
// Orders stream s after every fixed-base MSM tail enqueued on this context so far (call
// before reading a d_result of msm_fixed_device on s).
int msm_fixed_wait(pbf_ctx* ctx, hipStream_t s);
// 64-bit fingerprint of `words` u64 at d_words (position-mixed XOR hash; one stream sync):
// validates context caches against their inputs
int fingerprint_words(pbf_ctx* ctx, const uint64_t* d_words, uint64_t words, hipStream_t s, uint64_t* out);
// canonical affine (x, y as 4 + 4 little-endian u64; identity (0, 0)) of an XYZZ point
void xyzz_to_affine_u64(const Xyzz& p, uint64_t* out);

}  // namespace pbf
