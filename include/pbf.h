/*
 * pbf.h — C-ABI of the MI355X-native PLONK hot path (libpbf.so, gfx950).
 *
 * Drop-in boundary for adria0/plonk-by-fingers (Rust). The reference has no FFI;
 * every entry point below replaces one of its trait methods / free functions and
 * cites it as file:line relative to the reference root. A Rust caller binds these
 * with an `extern "C"` block; here they are exercised from C++
 * and from Python (ctypes) tests.
 *
 * Conventions:
 *   - Field elements cross the ABI canonical, in [0, modulus), one uint64_t each
 *     (the reference's U64Field<M> is one u64, u64field.rs:27-28). 256-bit
 *     elements are 4 x uint64_t little-endian limbs, canonical (never Montgomery).
 *   - Vectors are natural order (fft.rs:98-104 writes o[i] / o[i+len/2]).
 *   - Host-pointer entry points are synchronous: copy in, compute, copy out, on
 *     the context's host stream. `_dev` entry points take device pointers and a
 *     hipStream_t (void*) and are stream-ordered on that stream (NULL = the HIP null
 *     stream, as everywhere in HIP): their work starts after everything enqueued on
 *     it before the call and finishes before anything enqueued after. Two entry points
 *     also use streams private to the context, always joined back by events (waits in
 *     the command processor, never a spinning kernel) on the caller's stream before
 *     they return: a batched Goldilocks NTT of >= 8 polynomials
 *     (pbf_ntt_u64_batch_dev) forks half its groups onto a second stream, and the
 *     fixed-base MSM (pbf_msm_g1_bn254_fixed_dev, and the commitments inside
 *     pbf_plonk_prove_bn254*) runs its bucket join and reduction on a side stream while
 *     the caller's stream goes on; the fixed-base MSM, prove and verify order the
 *     caller's stream after that side stream (an event wait) before returning. Nothing
 *     else is ever enqueued on streams the caller did not pass.
 *   - Input and output may alias (in-place is allowed).
 *   - Supported moduli for the u64 entry points: Goldilocks p = 2^64-2^32+1, and any
 *     odd M < 2^32 (the range where the reference's `(a*b)%M` in u64 is exact,
 *     u64field.rs:177).
 *   - Errors are returned, never aborted on. pbf_last_error() gives the text.
 *   - One pbf_ctx per host thread; distinct contexts are independent (no shared
 *     streams, buffers or caches; every entry point selects the context's device).
 */
#ifndef PBF_H
#define PBF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum pbf_status {
  PBF_OK = 0,
  PBF_EINVAL = 1,      /* bad size / not a power of two / omega order != n / non-canonical input */
  PBF_ENOINV = 2,      /* n has no inverse mod M: the reference panics at fft.rs:73 `.unwrap()` */
  PBF_EDEVICE = 3,     /* HIP error (allocation, launch, copy) */
  PBF_ECOMM = 4,       /* RCCL / multi-GPU exchange error */
  PBF_EUNSUPPORTED = 5 /* modulus outside the supported set */
};

typedef struct pbf_ctx pbf_ctx;

/* ---- context ------------------------------------------------------------ */
/* Owns the device, a stream, twiddle tables (cached per (modulus, omega, n)) and
 * scratch buffers. Replaces nothing in the reference (its types are plain values). */
int pbf_ctx_create(int device, pbf_ctx** out);
void pbf_ctx_destroy(pbf_ctx* ctx);
const char* pbf_last_error(void);
/* Stream used by the synchronous host-pointer entry points (default: a private
 * non-blocking stream created with the context). `_dev` calls ignore it.     */
int pbf_ctx_set_stream(pbf_ctx* ctx, void* stream);
/* Context options: select among product code paths of this context (never read from the
 * environment). `value` NULL removes the option; unknown names return PBF_EINVAL. Every
 * option gives the same results, bit for bit; they exist for cross-checks and tuning:
 *   ntt.passes     "a,b,..."  radix bits per pass of u64 NTT plans (each 6..12, sum log2 n)
 *   ntt.group      G          polynomials per group of a batched Goldilocks NTT (0: one group)
 *   ntt.streams    k          streams the groups rotate over (1: the caller's stream only)
 *   ntt.twmax_log  L          per-pass twiddle tables up to 2^L entries (default 24)
 *   ntt.twsplit    1 / 0      last pass: force the split table / keep the two-level table
 *   ntt.no_rg      1          2^24: the round-2 passes instead of the regrouped plan
 *   ntt256.maxr    4..9       largest radix (bits) of the 256-bit NTT passes (default 9)
 *   ntt256.twlog   L          256-bit per-pass twiddle tables up to 2^L entries (default 26)
 *   ntt256.l29     0          256-bit NTT passes and the prover's quotient kernel on 8 x 32-bit
 *                             limbs instead of nine 29-bit ones
 *   msm.fx_c       16/20/22   fixed-base MSM window bits (default by size)
 *   g1.mul_base    "daa"      G1 fixed-base products by double-and-add instead of the comb
 *   pair.engine    "lane"/"wg" pairing engine (default: lanes from 4096 pairings)
 *   pair.lane_wpe  1 / 2      lane engine built for 1 or 2 waves per SIMD (default by size)
 *   prover.pk      0          no proving-key cache: every proof recomputes the preprocessed
 *                             polynomials, as the reference does (plonk.rs:233-243, 339-370)
 *   prover.timing  1          synchronise at every prover round mark (per-round times)
 *   verifier.vk    0          no verification-key cache
 * Options are read when used; an ntt* option also drops the context's cached NTT plans (after a
 * device synchronisation), which are rebuilt under the new value. */
int pbf_ctx_set_option(pbf_ctx* ctx, const char* name, const char* value);
int pbf_device_sync(pbf_ctx* ctx);
/* Frees the context's derived caches -- the prover's proving key, the verifier's
 * verification key, the fixed-base MSM window table, the pairing check's prepared lines
 * and the device copies that validate them -- after waiting for the context's streams.
 * The next call that needs one rebuilds it. Plans and scratch buffers stay.   */
int pbf_ctx_release_caches(pbf_ctx* ctx);

/* ---- FFT trait ------------------------------------------------------------ */
/* CooleyTurkey::new(EvaluationDomainGenerator{omega, size: n}) + fft / fft_inv
 * (fft.rs:6-21, 55-78). out[k] = sum_j in[j] * omega^(j*k)           (inverse = 0)
 *                       out[j] = n^-1 * sum_k in[k] * omega^(-j*k)    (inverse = 1)
 * omega must have multiplicative order exactly n (the reference assumes it).   */
int pbf_ntt_u64(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, const uint64_t* in, uint64_t* out,
                size_t n, int inverse);
/* Device-pointer, batched: `batch` independent transforms, polynomial b at
 * d_in + b*n. Inputs must already be canonical (not checked on this path).   */
int pbf_ntt_u64_batch_dev(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, const uint64_t* d_in,
                          uint64_t* d_out, size_t n, size_t batch, int inverse, void* stream);

/* ---- mul_ntt ---------------------------------------------------------------- */
/* fft.rs:109-132: zero-pad a (la) and b (lb) to la+lb (= the domain size, a power
 * of two), forward NTT both, multiply pointwise, inverse NTT. out has la+lb entries
 * and is NOT normalised (the reference's caller wraps it in Poly::new, fft.rs:180). */
int pbf_mul_ntt_u64(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, const uint64_t* a, size_t la,
                    const uint64_t* b, size_t lb, uint64_t* out);

/* ---- Poly ------------------------------------------------------------------- */
/* Poly::eval (poly.rs:71-79) at nx points: ys[i] = sum_j coeffs[j] * xs[i]^j. */
int pbf_poly_eval_u64(pbf_ctx* ctx, uint64_t modulus, const uint64_t* coeffs, size_t n,
                      const uint64_t* xs, size_t nx, uint64_t* ys);

/* ---- Poly arithmetic (poly.rs:165-247) -----------------------------------------------
 * Results normalised as Poly::normalize (poly.rs:96-105): trailing zeros stripped, at least
 * one coefficient; *lout / *lq / *lr receive the lengths. Inputs: >= 1 coefficient each.
 * pbf_poly_add_u64 / pbf_poly_sub_u64: AddAssign / SubAssign<&Poly> (poly.rs:165-176,
 *   192-203); `out` holds max(la, lb). Subtraction keeps the reference's quirk: where only
 *   b has a coefficient it is appended as +b[i] (poly.rs:196).
 * pbf_poly_div_u64: Div for Poly (poly.rs:230-247), num = q * den + r, deg r < deg den,
 *   computed in O(n log n) (reversed-series inverse by Newton's iteration, NTT products);
 *   `root` has multiplicative order 2^root_log and bounds the NTT sizes (Goldilocks:
 *   7^((p-1)/2^32), 32). q holds >= nn, r >= nn coefficients. PBF_ENOINV when the divisor's
 *   leading coefficient has no inverse (the reference's unwrap at poly.rs:238).         */
int pbf_poly_add_u64(pbf_ctx* ctx, uint64_t modulus, const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                     uint64_t* out, size_t* lout);
int pbf_poly_sub_u64(pbf_ctx* ctx, uint64_t modulus, const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                     uint64_t* out, size_t* lout);
int pbf_poly_div_u64(pbf_ctx* ctx, uint64_t modulus, uint64_t root, uint32_t root_log, const uint64_t* num,
                     size_t nn, const uint64_t* den, size_t nd, uint64_t* q, size_t* lq, uint64_t* r, size_t* lr);

/* ---- multi-GPU stride-sharded NTT ---------------------------
 * A transform of N = G * nl points (G = world size 2, 4 or 8; omega of order N) is
 * sharded by coefficient stride: rank g holds a[g + G*m], m < nl, for `batch`
 * polynomials ([b][m] layout). This is the top log2(G) levels of the reference's
 * even/odd recursion (fft.rs:94-96) assigned to ranks. Forward on every rank:
 *   pbf_ntt_shard_local_dev(fwd):  [b][m] stride shard -> send [dst][b][kk]   (S = nl/G)
 *   all-to-all (RCCL, nl*batch/G elements per peer): send -> recv [src][b][kk]
 *   pbf_ntt_shard_combine_dev(fwd): recv -> out[b][q*S + kk] = X[q*nl + rank*S + kk]
 * Inverse runs the same steps backwards with the same omega:
 *   combine(inv): out-layout X -> send [dst][b][kk]; all-to-all; local(inv): recv -> [b][m]
 * and returns the stride shard a[g + G*m] (scaled by N^-1 overall).                  */
int pbf_ntt_shard_local_dev(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, uint32_t world,
                            const uint64_t* d_in, uint64_t* d_out, size_t nl, size_t batch, int inverse,
                            void* stream);
int pbf_ntt_shard_combine_dev(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, uint32_t world,
                              uint32_t rank, const uint64_t* d_in, uint64_t* d_out, size_t nl,
                              size_t batch, int inverse, void* stream);

/* c[i] = a[i] * b[i] for `count` elements (the pointwise step of mul_ntt, fft.rs:125-129;
 * the sharded mul_ntt multiplies its blocks with it)                                  */
int pbf_pointwise_mul_u64_dev(pbf_ctx* ctx, uint64_t modulus, const uint64_t* d_a, const uint64_t* d_b,
                              uint64_t* d_c, size_t count, void* stream);

/* ---- BN254 scalar field (BASELINE config 3) ----------------------------------
 * r = 21888242871839275222246405745257275088548364400416034343698204186575808495617,
 * elements 4 x uint64_t little-endian, canonical; n a power of two <= 2^28.
 * The reference has no 256-bit field: these are fft.rs:66-78 and fft.rs:109-132
 * instantiated for the field SURVEY.md §0.5 picks for configs 3-5.              */
int pbf_ntt_fr256(pbf_ctx* ctx, const uint64_t* omega, const uint64_t* in, uint64_t* out, size_t n,
                  int inverse);
int pbf_ntt_fr256_batch_dev(pbf_ctx* ctx, const uint64_t* omega, const uint64_t* d_in, uint64_t* d_out,
                            size_t n, size_t batch, int inverse, void* stream);
int pbf_mul_ntt_fr256(pbf_ctx* ctx, const uint64_t* omega, const uint64_t* a, size_t la,
                      const uint64_t* b, size_t lb, uint64_t* out);
/* batched device mul_ntt: a, b already zero-padded to n = la + lb; out = batch x n  */
int pbf_mul_ntt_fr256_dev(pbf_ctx* ctx, const uint64_t* omega, const uint64_t* d_a, const uint64_t* d_b,
                          uint64_t* d_out, size_t n, size_t batch, void* stream);

/* Stride-sharded Fr NTT across G GPUs: pbf_ntt_shard_local_dev / _combine_dev (above) for
 * 256-bit elements (omega: 4 x u64, order G*nl). Same layouts, 4 x u64 per element.     */
int pbf_ntt_fr256_shard_local_dev(pbf_ctx* ctx, const uint64_t* omega, uint32_t world, const uint64_t* d_in,
                                  uint64_t* d_out, size_t nl, size_t batch, int inverse, void* stream);
int pbf_ntt_fr256_shard_combine_dev(pbf_ctx* ctx, const uint64_t* omega, uint32_t world, uint32_t rank,
                                    const uint64_t* d_in, uint64_t* d_out, size_t nl, size_t batch, int inverse,
                                    void* stream);
/* c[i] = a[i] * b[i] over Fr (canonical in and out)                                      */
int pbf_pointwise_mul_fr256_dev(pbf_ctx* ctx, const uint64_t* d_a, const uint64_t* d_b, uint64_t* d_c,
                                size_t count, void* stream);

/* ---- BN254 G1 MSM / SRS (BASELINE config 4) -----------------------------------
 * Points: affine, 8 x uint64_t (x then y, each 4 little-endian limbs, canonical in Fq);
 * (0, 0) encodes the identity. Scalars: Fr canonical, 4 x uint64_t.              */
/* SRS::eval_at_s (plonk.rs:51-58): out = sum_i scalars[i] * points[i]               */
int pbf_msm_g1_bn254(pbf_ctx* ctx, const uint64_t* points, const uint64_t* scalars, size_t n,
                     uint64_t* out);
int pbf_msm_g1_bn254_dev(pbf_ctx* ctx, const uint64_t* d_points, const uint64_t* d_scalars, size_t n,
                         uint64_t* out, void* stream);
/* The same sum against a FIXED base set (KZG commitments: the SRS): out = sum_{i<n}
 * scalars[i] * points[i], n <= n_points. The first call for a base set precomputes its
 * window table 2^(16w) P_i (16 x n_points affine points, cached in the context with a
 * device copy of the points it was built from, and revalidated against that copy word for
 * word on every call, so rewriting the points in place is safe); then every (point,
 * window) digit shares one set of 2^15 buckets.                                           */
int pbf_msm_g1_bn254_fixed_dev(pbf_ctx* ctx, const uint64_t* d_points, size_t n_points, const uint64_t* d_scalars,
                               size_t n, uint64_t* out, void* stream);
/* The same against points [first, first + n) of the fixed base set: out = sum_{i<n}
 * scalars[i] * points[first + i] (one rank's point range of a sharded commitment; the
 * window table still covers all n_points and is shared with the call above).               */
int pbf_msm_g1_bn254_fixed_range_dev(pbf_ctx* ctx, const uint64_t* d_points, size_t n_points, size_t first,
                                     const uint64_t* d_scalars, size_t n, uint64_t* out, void* stream);
/* out_i = scalars_i * G (G = (1, 2)), device pointers                               */
int pbf_g1_bn254_mul_base_dev(pbf_ctx* ctx, const uint64_t* d_scalars, uint64_t* d_out, size_t n,
                              void* stream);
/* SRS::create (plonk.rs:35-48): out = [G, G*s, ..., G*s^n] (n+1 points)             */
int pbf_srs_create_bn254(pbf_ctx* ctx, const uint64_t* s, size_t n, uint64_t* out);

/* ---- BN254 pairing (BASELINE config 4 "pairing check") ------------------------
 * The BN254 instance of Pairing::pairing (src/ec.rs:87-93; the reference's own is the
 * toy reduced Tate pairing, src/pbh/pairing.rs:12-47) as Plonk::verify uses it
 * (src/plonk.rs:646-647): optimal ate, e(P, Q) = f_{6u+2,Q}(P)...^((q^12-1)/r).
 * G1: 8 x uint64_t affine (as above). G2: 16 x uint64_t affine on the twist
 * y^2 = x^3 + 3/(9+u) over Fq2 = Fq[u]/(u^2+1): x.c0, x.c1, y.c0, y.c1 (4 limbs each),
 * all zero = identity. GT: 48 x uint64_t = 12 Fq in the tower order of
 * Fq12 = Fq6[w]/(w^2-v), Fq6 = Fq2[v]/(v^3-(9+u)): c0.a0, c0.a1, c0.a2, c1.a0, c1.a1,
 * c1.a2 (each Fq2 as c0, c1). Inputs must be subgroup points (not checked; coordinates
 * are checked canonical, else PBF_EINVAL).                                             */
int pbf_pairing_bn254(pbf_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, uint64_t* out);
int pbf_pairing_bn254_dev(pbf_ctx* ctx, const uint64_t* d_g1, const uint64_t* d_g2, size_t n, uint64_t* d_out,
                          void* stream);
/* *ok = (prod_i e(g1_i, g2_i) == 1): n Miller loops, one shared final exponentiation.
 * The KZG opening check of Plonk::verify (plonk.rs:646-650) is n = 2:
 * e(W, [s]G2) * e(-(C - y G + z W), G2) == 1.                                          */
int pbf_pairing_check_bn254(pbf_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, int* ok);
/* out_i = scalars_i * pts_i on the twist (G2P::mul, src/pbh/g2.rs:82-101): SRS [s]G2  */
int pbf_g2_bn254_mul(pbf_ctx* ctx, const uint64_t* pts, const uint64_t* scalars, size_t n, uint64_t* out);

/* ---- Generalised PLONK prover / verifier over BN254 (BASELINE config 5) ---------
 * Plonk::prove / Plonk::verify (src/plonk.rs:191-650) for n = 2^k >= 8 gates with
 * HF = GF = Fr, G1/G2 of BN254 and the pairing above; t(x) split into three parts of
 * n+2 coefficients (plonk.rs:376-378 generalised). Field elements canonical 4 x u64.
 *   q:      5 x n x 4   (columns q_l, q_r, q_o, q_m, q_c)
 *   copies: 3 x n x 2   (columns c_a, c_b, c_c; per wire (kind 0=A 1=B 2=C, 1-based index))
 *   abc:    3 x n x 4   (witness columns a, b, c)
 *   chal:   5 x 4       (alpha, beta, gamma, z, v)      rnd: 9 x 4 (b1..b9)
 *   k1k2:   2 x 4       (PlonkTypes::K1, K2: cosets k1 H, k2 H, plonk.rs:133-139)
 *   srs:    srs_m x 8   affine G1 [G, sG, s^2 G, ...] (SRS::create); prove needs
 *           srs_m >= 2n+2 in mode 0, >= n+3 in mode 1; verify >= n. g2: [G2, [s]G2].
 *   out_pts 9 x 8: a_s b_s c_s z_s t_lo_s t_mid_s t_hi_s w_z_s w_zw_s
 *   out_f   7 x 4: a_z b_z c_z s_sigma_1_z s_sigma_2_z r_z z_omega_z   (Proof, plonk.rs:61-95)
 * mode 0 = the reference's formulas (r_3(x) of plonk.rs:414-416; verifier step 7 of
 * plonk.rs:575-581), mode 1 = the paper linearisation the verifier checks (SURVEY §0.7:
 * with mode 0 an honest proof verifies only when (a_z+b*s1_z+g)(b_z+b*s2_z+g)*alpha = 0,
 * as in the reference's n = 4 KAT).
 * Errors: PBF_EINVAL for an unsatisfied circuit (constraints.rs:198), a zero permutation
 * denominator (plonk.rs:297), a non-divisible quotient (plonk.rs:370), short SRS.
 * Keys: the context keeps the circuit's preprocessed polynomials (q_*, s_sigma_*, l1:
 * 8 coefficient slots of n+8 and 9 coset slots of 4n (of 4n/world when sharded) Fr
 * elements, ~1.4 KiB per gate, ~23.6 GB at 2^24 gates on one GPU) and the verifier's 8
 * preprocessed commitments, plus device copies of the q / copies (and, for verify, SRS)
 * arrays they were built from (~0.2 KiB per gate each); every call compares its inputs
 * with those copies word for word and rebuilds on any difference. Outputs are identical
 * either way; PBF_PROVER_NO_PK=1 / PBF_VERIFIER_NO_VK=1 disable the keys, and
 * pbf_ctx_release_caches frees them (and the MSM window table) between circuits.        */
int pbf_plonk_prove_bn254(pbf_ctx* ctx, size_t n, const uint64_t* q, const uint64_t* copies, const uint64_t* abc,
                          const uint64_t* chal, const uint64_t* rnd, const uint64_t* k1k2, const uint64_t* srs,
                          size_t srs_m, int mode, uint64_t* out_pts, uint64_t* out_f);
int pbf_plonk_prove_bn254_dev(pbf_ctx* ctx, size_t n, const uint64_t* d_q, const uint64_t* d_copies,
                              const uint64_t* d_abc, const uint64_t* chal, const uint64_t* rnd, const uint64_t* k1k2,
                              const uint64_t* d_srs, size_t srs_m, int mode, uint64_t* out_pts, uint64_t* out_f,
                              void* stream);
int pbf_plonk_verify_bn254(pbf_ctx* ctx, size_t n, const uint64_t* q, const uint64_t* copies, const uint64_t* srs,
                           size_t srs_m, const uint64_t* g2, const uint64_t* proof_pts, const uint64_t* proof_f,
                           const uint64_t* chal, const uint64_t* u, const uint64_t* k1k2, int mode, int* ok);
int pbf_plonk_verify_bn254_dev(pbf_ctx* ctx, size_t n, const uint64_t* d_q, const uint64_t* d_copies,
                               const uint64_t* d_srs, size_t srs_m, const uint64_t* g2, const uint64_t* proof_pts,
                               const uint64_t* proof_f, const uint64_t* chal, const uint64_t* u, const uint64_t* k1k2,
                               int mode, int* ok, void* stream);

/* Config 5 across G GPUs ("NTT sharded across 8xMI355X"): one process (or thread) per GPU
 * calls pbf_plonk_prove_bn254_sharded_dev with the same inputs (circuit, SRS, challenges,
 * blinders) and its rank. The library computes nothing collective itself: it calls back
 * into the caller's communicator (RCCL via torch.distributed in multigpu.py, or the library's
 * own in pbf_plonk_prove_bn254_multi), always for buffers it names in `comm` and
 * stream-ordered on `stream`:
 *   all_to_all(user, b, stream):  send[g*b .. (g+1)*b) goes to rank g, recv[g*b ..) comes from g
 *   all_gather(user, b, stream):  send[0 .. b) of rank g lands in recv[g*b .. (g+1)*b)
 * Work split, every witness-dependent step on this rank's share: satisfies and
 * the accumulator's terms / prefix products on rows [r n/G, (r+1) n/G) (the ranks' products
 * all-gathered); interpolation of a b c and of the accumulator as sharded INTTs; every coset NTT
 * of size 4n and the coset INTT of t as stride-sharded transforms; the quotient on this rank's
 * evaluation blocks; commitments, evaluations, r(x) and the opening divisions on this rank's
 * contiguous coefficient range (one all-to-all transposes the NTTs' stride shards into it; the
 * divisions' and evaluations' per-range totals are all-gathered); every commitment is this
 * rank's point range, the partial sums all-gathered once at the end. The circuit's proving key
 * is built once per circuit on every rank. Outputs are identical on every rank and
 * bit-identical to the single-GPU proof. n >= world^2. send / recv: device buffers of
 * `capacity` >= 5 * (4n / world) * 32 bytes each.                                          */
typedef struct pbf_comm {
  uint32_t world, rank;
  void* user;
  void* send;
  void* recv;
  size_t capacity;
  int (*all_to_all)(void* user, size_t bytes_per_peer, void* stream);
  int (*all_gather)(void* user, size_t bytes_per_rank, void* stream);
} pbf_comm;
int pbf_plonk_prove_bn254_sharded_dev(pbf_ctx* ctx, const pbf_comm* comm, size_t n, const uint64_t* d_q,
                                      const uint64_t* d_copies, const uint64_t* d_abc, const uint64_t* chal,
                                      const uint64_t* rnd, const uint64_t* k1k2, const uint64_t* d_srs,
                                      size_t srs_m, int mode, uint64_t* out_pts, uint64_t* out_f, void* stream);

/* ---- multi-GPU from ONE host process (SURVEY.md §8b pbf_ntt_u64_multi) -------------------
 * `ctxs` = G contexts (G = 2, 4, 8), rank g = ctxs[g]. The library owns the exchange: on G
 * distinct devices it uses RCCL (librccl loaded at run time; ncclCommInitAll, grouped
 * ncclSend / ncclRecv for the all-to-all, ncclAllGather), on one shared device (virtual ranks)
 * stream-ordered device copies ordered by events. The communicator and its buffers are kept
 * per context list (pointers and creation order) until a member context is destroyed. Each
 * rank runs in a library-owned host thread; errors name the failing rank. Outputs are
 * bit-identical to the single-GPU entry points.
 *
 * pbf_ntt_u64_multi: CooleyTurkey::fft / fft_inv (fft.rs:66-78) of one host vector of n points
 *   (n = G * nl, nl a power of two >= G), natural order in and out, with the top log2(G) levels of
 *   the recursion (fft.rs:94-96) across the ranks: the stride shards go to the G devices, one
 *   all-to-all, the blocks come back (pbf_ntt_shard_local_dev / _combine_dev, one rank each).
 * _dev: per-rank device buffers and streams: d_in[g] = rank g's stride shards [batch][nl]
 *   (forward) or blocks (inverse), d_out[g] likewise the other way round (streams may be NULL).
 * pbf_mul_ntt_*_multi: mul_ntt (fft.rs:109-132), la + lb = G * nl; out has la + lb entries.
 * pbf_plonk_prove_bn254_multi: Plonk::prove (plonk.rs:191-466) with the work split of
 *   pbf_plonk_prove_bn254_sharded_dev, the host inputs uploaded to every rank's device; _dev
 *   takes per-rank device copies (d_q[g] ... on rank g's device) and streams. The ranks'
 *   proofs are compared (PBF_ECOMM if they differ) and returned once.
 * pbf_multi_backend: *backend = 0 (device copies, one device) or 1 (RCCL).                   */
int pbf_ntt_u64_multi(pbf_ctx* const* ctxs, uint32_t world, uint64_t modulus, uint64_t omega, const uint64_t* in,
                      uint64_t* out, size_t n, int inverse);
int pbf_ntt_u64_multi_dev(pbf_ctx* const* ctxs, uint32_t world, uint64_t modulus, uint64_t omega,
                          const uint64_t* const* d_in, uint64_t* const* d_out, size_t nl, size_t batch, int inverse,
                          void* const* streams);
int pbf_ntt_fr256_multi(pbf_ctx* const* ctxs, uint32_t world, const uint64_t* omega, const uint64_t* in, uint64_t* out,
                        size_t n, int inverse);
int pbf_ntt_fr256_multi_dev(pbf_ctx* const* ctxs, uint32_t world, const uint64_t* omega, const uint64_t* const* d_in,
                            uint64_t* const* d_out, size_t nl, size_t batch, int inverse, void* const* streams);
int pbf_mul_ntt_u64_multi(pbf_ctx* const* ctxs, uint32_t world, uint64_t modulus, uint64_t omega, const uint64_t* a,
                          size_t la, const uint64_t* b, size_t lb, uint64_t* out);
int pbf_mul_ntt_fr256_multi(pbf_ctx* const* ctxs, uint32_t world, const uint64_t* omega, const uint64_t* a, size_t la,
                            const uint64_t* b, size_t lb, uint64_t* out);
int pbf_plonk_prove_bn254_multi(pbf_ctx* const* ctxs, uint32_t world, size_t n, const uint64_t* q, const uint64_t* copies,
                                const uint64_t* abc, const uint64_t* chal, const uint64_t* rnd, const uint64_t* k1k2,
                                const uint64_t* srs, size_t srs_m, int mode, uint64_t* out_pts, uint64_t* out_f);
int pbf_plonk_prove_bn254_multi_dev(pbf_ctx* const* ctxs, uint32_t world, size_t n, const uint64_t* const* d_q,
                                    const uint64_t* const* d_copies, const uint64_t* const* d_abc, const uint64_t* chal,
                                    const uint64_t* rnd, const uint64_t* k1k2, const uint64_t* const* d_srs,
                                    size_t srs_m, int mode, uint64_t* out_pts, uint64_t* out_f, void* const* streams);
int pbf_multi_backend(pbf_ctx* const* ctxs, uint32_t world, int* backend);

/* synthetic config-5 circuit on the device (bench / tests): every gate a*b = c, a, b
 * uniform (splitmix64 of seed), every 4th gate's c copied into the next gate's a       */
int pbf_plonk_synth_circuit_bn254_dev(pbf_ctx* ctx, size_t n, uint64_t seed, uint64_t* d_q, uint64_t* d_copies,
                                      uint64_t* d_abc, void* stream);
/* SRS::create with the output left on the device (n+1 points)                          */
int pbf_srs_create_bn254_dev(pbf_ctx* ctx, const uint64_t* s, size_t n, uint64_t* d_out, void* stream);

/* ---- Plonk-by-hand types (BASELINE config 1; src/pbh/{g1,g2,gt,pairing}.rs) -------------------
 * 32-bit words: G1 [x, y, inf] over F101 (y^2 = x^3 + 3), G2 [a, b] (a + b*u over
 * F101[u]/(u^2+2)), GT [a, b]. Inputs must be on the curve (else PBF_EINVAL, where the
 * reference would panic or compute garbage).                                        */
int pbf_pbh_g1_mul(pbf_ctx* ctx, const uint32_t* pts, const uint32_t* scalars, size_t n, uint32_t* out);
int pbf_pbh_g2_mul(pbf_ctx* ctx, const uint32_t* pts, const uint32_t* scalars, size_t n, uint32_t* out);
int pbf_pbh_gt_pow(pbf_ctx* ctx, const uint32_t* x, const uint32_t* e, size_t n, uint32_t* out);
/* PBHPairing::pairing (pairing.rs:12-47), batched                                    */
int pbf_pbh_pairing(pbf_ctx* ctx, const uint32_t* g1, const uint32_t* g2, size_t n, uint32_t* out);
/* Plonk::prove (+ Plonk::verify when verify_u < 17) over PlonkByHandTypes
 * (plonk.rs:120-650, pbh/mod.rs:18-33). gates: n x [q_l q_r q_o q_m q_c]; copies:
 * 3 columns x n x [kind (0=A,1=B,2=C), 1-based index]; abc: 3 x n witness; chal:
 * [alpha beta gamma z v]; rnd: 9 blinders; s: toxic waste; srs_n: SRS degree;
 * omega_pows: |H|. out_pts: 9 x [x y inf] (a_s b_s c_s z_s t_lo t_mid t_hi w_z w_zw),
 * out_f: [a_z b_z c_z s_sigma_1_z s_sigma_2_z r_z z_omega_z]; *verified = 1/0 (or -1).  */
int pbf_pbh_prove(pbf_ctx* ctx, size_t n, const uint64_t* gates, const uint64_t* copies,
                  const uint64_t* abc, const uint64_t* chal, const uint64_t* rnd, uint64_t s,
                  uint64_t srs_n, uint64_t omega_pows, uint64_t verify_u, uint64_t* out_pts,
                  uint64_t* out_f, int* verified);

/* ---- synthetic inputs (bench / tests) ------------------------------------- */
/* d_out[i] = splitmix64 stream of (seed, i) with rejection of values >= modulus;
 * identical to tests/golden/gen_golden.py:splitmix_field.                     */
int pbf_fill_random_u64_dev(pbf_ctx* ctx, uint64_t modulus, uint64_t seed, uint64_t* d_out,
                            size_t count, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PBF_H */
