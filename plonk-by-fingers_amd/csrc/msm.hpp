// Device-side MSM entry points shared by msm.hip and the prover (prover.hip).
#pragma once
#include "ec_bn254.hpp"
#include "internal.hpp"

namespace pbf {

// Window table (16 x n affine points, Montgomery) of the n canonical affine points at d_pts,
// cached in the context and revalidated against a device copy of the points (one compare
// kernel and one stream sync per call; rebuilt when they differ).
int msm_fixed_table(pbf_ctx* ctx, const uint64_t* d_pts, uint64_t n, hipStream_t s, const Affine** out);
// The cached table of exactly these points (content checked), or null (nothing built).
int msm_fixed_lookup(pbf_ctx* ctx, const uint64_t* d_pts, uint64_t n, hipStream_t s, const Affine** out);
// sum_{i<n} scalars[i] * P_(first+i) against a table of n_table points; the XYZZ result
// (Montgomery) is written to *d_result by the context's side stream (see msm_fixed_wait);
// nothing on the host waits for it.
// sc_ready (msm_scalars_ready): the scalars were complete when it was recorded on s, so the
// digits, the sort and the bucket bounds may run on the context's prep stream, overlapping the
// accumulation of an MSM enqueued before this one (null: everything on s).
int msm_fixed_device(pbf_ctx* ctx, const Affine* table, uint64_t n_table, uint64_t first, const uint64_t* d_sc,
                     uint64_t n, hipStream_t s, Xyzz* d_result, hipEvent_t sc_ready = nullptr);
// Records on s the point at which the scalars of the next MSMs are complete; returns the event
// for msm_fixed_device, or null when the prep stream is off (the default; PBF_MSM_PREP=1 turns
// it on: measured no faster, msm.hip).
hipEvent_t msm_scalars_ready(pbf_ctx* ctx, hipStream_t s);
// Orders stream s after every fixed-base MSM tail enqueued on this context so far (call
// before reading a d_result of msm_fixed_device on s).
int msm_fixed_wait(pbf_ctx* ctx, hipStream_t s);
// Exact-content validation of context caches: *same = every item's `words` u64 equal the
// context's snapshot named `name` (same length, word for word) AND that snapshot is the one
// `consumer`'s cache was last built from. Snapshots are named after the data and shared by
// every consumer (the prover's key, the verifier's key and the MSM window table all validate
// against one copy of q / copies / the SRS points). Items that differ (or have no snapshot
// yet) get their snapshot replaced by a device copy of the input, so the caller rebuilds its
// cache from these inputs. One compare kernel per item, one stream sync in all.
struct SnapItem {
  const char* name;
  const uint64_t* p;
  uint64_t words;
};
int snapshot_check(pbf_ctx* ctx, const char* consumer, const SnapItem* items, int k, hipStream_t s, bool* same);
// canonical affine (x, y as 4 + 4 little-endian u64; identity (0, 0)) of an XYZZ point
void xyzz_to_affine_u64(const Xyzz& p, uint64_t* out);

}  // namespace pbf
