/* grandine_bls_gpu.h -- C ABI of the MI355X BLS12-381 signature engine.
 *
 * Drop-in boundary for Grandine's signature hot path.  The reference has no FFI of
 * its own: its `bls` crate calls the blst 0.3.11 Rust bindings.  Each entry point
 * below replaces one of those call sites (reference = /root/reference):
 *
 *   gbls_g1_decompress          PublicKey: TryFrom<PublicKeyBytes>   bls/src/public_key.rs:16-31
 *                               (blst_p1_uncompress + PublicKey::validate)
 *   gbls_g2_decompress          Signature: TryFrom<SignatureBytes>   bls/src/signature.rs:36-45
 *   gbls_g1_compress            From<PublicKey> for PublicKeyBytes    bls/src/public_key.rs:9-14
 *   gbls_g2_compress            From<Signature> for SignatureBytes    bls/src/signature.rs:29-34
 *   gbls_g1_aggregate           PublicKey::aggregate_nonempty        bls/src/public_key.rs:34-55
 *   gbls_g1_aggregate_segments  Triple::verify_aggregate (batched)   helper_functions/src/verifier.rs:387-405
 *   gbls_g2_aggregate           Signature::aggregate                  bls/src/signature.rs:62-75
 *   gbls_verify                 Signature::verify                     bls/src/signature.rs:47-60
 *   gbls_fast_aggregate_verify  Signature::fast_aggregate_verify      bls/src/signature.rs:77-93
 *   gbls_aggregate_verify_batch many independent verify calls         (SingleVerifier::extend, verifier.rs:215-236)
 *   gbls_verify_batch_compressed  SingleVerifier::extend in ONE submission per call: signature
 *                               decompression (signature.rs:36-45) fused into the checks, keys
 *                               single (Triple) or aggregated per check (deferred
 *                               Triple::verify_aggregate, verifier.rs:387-405)
 *   gbls_multi_verify           Signature::multi_verify               bls/src/signature.rs:95-129
 *                               (reached from MultiVerifier::finish, verifier.rs:301-323)
 *   gbls_multi_verify_segments  several independent multi_verify batches in one submission
 *   gbls_multi_verify_bisect    per-set verdicts of a failed batch (replaces the per-item CPU
 *                               fallbacks p2p/src/attestation_verifier.rs:228-240,373-386 and
 *                               transition_functions/src/unphased/block_processing.rs:376-441)
 *   gbls_registry_set           CachedPublicKey::decompress for a whole validator registry
 *                               bls/src/cached_public_key.rs:104-108 (Validator.pubkey,
 *                               types/src/phase0/containers.rs:229), device-resident
 *   gbls_multi_verify_indexed   multi_verify / Triple::verify_aggregate over registry indices
 *   gbls_multi_verify_compressed  MultiVerifier::finish in one submission: signature
 *                               decompression (verifier.rs:309-313) fused into the batch verify
 *   gbls_multi_verify_compressed_ex  the same with a priority class (block import,
 *                               transition_functions/src/deneb/state_transition.rs:69-71)
 *   gbls_g1_aggregate_indexed   AggregatePublicKey::aggregate over registry indices (e.g. the
 *                               512-key get_next_sync_committee aggregate,
 *                               helper_functions/src/accessors.rs:605-628)
 *   gbls_g2_aggregate_segments  Signature::aggregate_in_place batched (op pools:
 *                               operation_pools/src/attestation_agg_pool/tasks.rs:253,
 *                               sync_committee_agg_pool/pool.rs:114,190)
 *   gbls_fast_aggregate_verify_indexed  sync-committee fast_aggregate_verify over indices
 *                               (operation_pools/src/sync_committee_agg_pool/tasks.rs:412-430)
 *   gbls_sk_to_pk / gbls_sign   SecretKey::to_public_key / sign       bls/src/secret_key.rs:74-86
 *                               FIXTURE GENERATION ONLY: not constant time (the scalar
 *                               multiplication branches on key bits); never sign with it.
 *
 * Conventions
 *   - gbls_p1_affine / gbls_p2_affine are byte-compatible with blst_p1_affine /
 *     blst_p2_affine: little-endian limbs in Montgomery form (R = 2^384); all-zero
 *     encodes the point at infinity.
 *   - Status codes mirror BLST_ERROR.  Verification entry points return
 *     GBLS_SUCCESS (valid) or GBLS_VERIFY_FAIL.  ANY engine/device/driver failure of
 *     ANY entry point returns GBLS_VERIFY_FAIL (fail closed), fills verdict arrays
 *     with GBLS_VERIFY_FAIL and status arrays with a failure code first, and sets the
 *     thread-local gbls_last_error().
 *   - Every entry point is reentrant and thread-safe: each call leases its own
 *     streams and workspaces from a per-device pool.  Host-pointer entry points are
 *     synchronous; buffers are borrowed for the call only.  *_device variants take
 *     device pointers (inputs already resident in HBM), run on the calling thread's
 *     current HIP device and are asynchronous on the given stream.
 *   - gbls_init(device_mask, flags): one engine per set bit of device_mask (0: the
 *     current device); flags & 0xff = engines per device (default 1; >1 lets tests
 *     exercise the multi-device paths on one GPU).  Host-pointer calls shard large
 *     batches over the engines: whole segments per engine, or per-engine Miller
 *     partials of one batch combined by a single final exponentiation.
 *   - Segment offsets must satisfy seg_off[0] == 0, seg_off[i] <= seg_off[i+1] and
 *     seg_off[nseg] == n (else GBLS_ERR_ARG).
 *   - A zero random scalar fails its batch (the reference only draws NonZeroU64).
 *   - Concurrent host-pointer multi_verify calls (gbls_multi_verify, _segments,
 *     _indexed) are coalesced: callers that arrive while the engine is busy are merged
 *     into one segmented submission, each keeping its own verdicts.
 *   - There is NO CPU fallback inside this library: without a usable gfx950 device
 *     every call fails with GBLS_ERR_NO_DEVICE.
 */
#ifndef GRANDINE_BLS_GPU_H
#define GRANDINE_BLS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint64_t x[6], y[6];
} gbls_p1_affine;
typedef struct {
  uint64_t x[2][6], y[2][6];
} gbls_p2_affine;
typedef struct {
  uint64_t c[12][6]; /* Fp12 as 12 Fp limbs-vectors (tower order c0.c0.c0 ... c1.c2.c1) */
} gbls_fp12;

enum {
  GBLS_SUCCESS = 0,
  GBLS_BAD_ENCODING = 1,
  GBLS_POINT_NOT_ON_CURVE = 2,
  GBLS_POINT_NOT_IN_GROUP = 3,
  GBLS_AGGR_TYPE_MISMATCH = 4,
  GBLS_VERIFY_FAIL = 5,
  GBLS_PK_IS_INFINITY = 6,
  GBLS_BAD_SCALAR = 7,
};
/* side-channel error codes (gbls_last_error) */
enum {
  GBLS_ERR_NONE = 0,
  GBLS_ERR_NO_DEVICE = 100,
  GBLS_ERR_HIP = 101,
  GBLS_ERR_ARG = 102,
};

/* gbls_init flags: low byte = engines per device; GBLS_INIT_NO_COALESCE turns off the
 * cross-caller coalescing of concurrent host-pointer multi_verify calls (f3).
 * GBLS_INIT_TUNING (tests and benchmark sweeps only) lets gbls_init read the engine's
 * tuning environment variables (GBLS_MSM_MIN, GBLS_LINE_BUDGET_MB, GBLS_ML_G,
 * GBLS_ML_ROUNDS, GBLS_PRIO_MODE, GBLS_SIDE2_HIGH, GBLS_ROW_CLEAR_MAX); without it the
 * measured defaults are fixed and no environment variable changes the engine.
 * GBLS_INIT_PER_CHECK: batches of independent checks get one Miller product and final
 * exponentiation per check (deterministic, as the reference's fast_aggregate_verify) instead
 * of the grouped form described at gbls_fast_aggregate_verify_batch.
 * The policy flags (GBLS_INIT_NO_COALESCE, GBLS_INIT_PER_CHECK) are sticky: a gbls_init call
 * that names one turns it on, also on an engine that is already open, and no gbls_init call
 * turns it off (a library's lazy gbls_init(mask, 0) cannot undo a harness's PER_CHECK).  The
 * other bits apply on the first call only.  gbls_set_policy sets both policies outright
 * (flags & (GBLS_INIT_NO_COALESCE | GBLS_INIT_PER_CHECK), the rest ignored) and returns the
 * previous policy bits; it needs no device. */
#define GBLS_INIT_NO_COALESCE 0x100u
#define GBLS_INIT_TUNING 0x200u
#define GBLS_INIT_PER_CHECK 0x400u
int gbls_init(uint32_t device_mask, uint32_t flags);
uint32_t gbls_set_policy(uint32_t flags);
int gbls_last_error(void);
const char *gbls_version(void);
int gbls_device_count(void); /* engines (devices x replicas) after gbls_init; 0 before */

/* a9 / a8 / a10 */
int gbls_g1_decompress(const uint8_t (*in)[48], size_t n, int validate, gbls_p1_affine *out,
                       int32_t *status);
int gbls_g2_decompress(const uint8_t (*in)[96], size_t n, gbls_p2_affine *out, int32_t *status);
int gbls_g2_validate(const gbls_p2_affine *in, size_t n, int32_t *status); /* sig subgroup check */
int gbls_g1_compress(const gbls_p1_affine *in, size_t n, uint8_t (*out)[48]);
int gbls_g2_compress(const gbls_p2_affine *in, size_t n, uint8_t (*out)[96]);

/* a4 / a5 / a11: n == 0 -> GBLS_AGGR_TYPE_MISMATCH */
int gbls_g1_aggregate(const gbls_p1_affine *pks, size_t n, gbls_p1_affine *out);
int gbls_g1_aggregate_segments(const gbls_p1_affine *pks, const uint32_t *seg_offsets, size_t nseg,
                               gbls_p1_affine *out, int32_t *status);
int gbls_g2_aggregate(const gbls_p2_affine *sigs, size_t n, gbls_p2_affine *out);
int gbls_g2_aggregate_segments(const gbls_p2_affine *sigs, const uint32_t *seg_offsets,
                               size_t nseg, gbls_p2_affine *out, int32_t *status);

/* f1: device-resident validator registry.  gbls_registry_set decompresses and validates
 * (PublicKey::try_from semantics) keys [first, first + n) on every engine device;
 * invalid keys are stored as infinity (rejected by every verification) and reported in
 * status.  The registry grows as needed; indices past its size are BAD_ENCODING. */
int gbls_registry_set(size_t first, const uint8_t (*pks)[48], size_t n, int32_t *status);
size_t gbls_registry_size(void);
/* sum of registry keys idx[seg_offsets[s] .. seg_offsets[s+1]) per segment */
int gbls_g1_aggregate_indexed(const uint32_t *idx, const uint32_t *seg_offsets, size_t nseg,
                              gbls_p1_affine *out, int32_t *status);

/* a6 / a7: returns GBLS_SUCCESS iff the signature verifies (blst semantics:
 * sig_groupcheck = true, pk_validate = false, infinite pk rejected). */
int gbls_verify(const gbls_p2_affine *sig, const uint8_t *msg, size_t msg_len,
                const gbls_p1_affine *pk);
int gbls_fast_aggregate_verify(const gbls_p2_affine *sig, const uint8_t *msg, size_t msg_len,
                               const gbls_p1_affine *pks, size_t n);
/* m independent (sig, msg, pk) checks; messages packed in msg_data with msg_off[m+1];
 * verdicts[i] = GBLS_SUCCESS or GBLS_VERIFY_FAIL.
 * Single checks whose messages are all 32 bytes (signing roots: gbls_verify,
 * gbls_fast_aggregate_verify and the _batch forms with msg_off[i] == 32 i) are coalesced
 * across concurrent callers like multi_verify (f3): callers that arrive while the engine is
 * busy become segments of one submission, each keeping its own verdicts. */
int gbls_aggregate_verify_batch(const gbls_p2_affine *sigs, const uint8_t *msg_data,
                                const uint32_t *msg_off, const gbls_p1_affine *pks, size_t m,
                                int32_t *verdicts);
/* SingleVerifier::extend (helper_functions/src/verifier.rs:215-236) as ONE coalesced
 * submission: m checks of 32-byte messages against 96-byte compressed signatures, decompressed
 * on the device (a8 semantics: sig_status[i] = its BLST_ERROR, the reference's
 * Signature::try_from) and then verified with Signature::verify semantics (subgroup check,
 * infinite key rejected).  Keys: pks[i] (pk_off == NULL), or the sum of
 * pks[pk_off[i] .. pk_off[i+1]) (fast_aggregate_verify; an empty range fails).  verdicts[i] is
 * GBLS_SUCCESS only when check i decodes and verifies.  Returns GBLS_SUCCESS when every output
 * was written, else GBLS_VERIFY_FAIL (engine error: gbls_last_error). */
int gbls_verify_batch_compressed(const uint8_t (*msgs)[32], const uint8_t (*sigs)[96],
                                 const gbls_p1_affine *pks, const uint32_t *pk_off, size_t m,
                                 int32_t *sig_status, int32_t *verdicts);
/* C3 shape: m fast_aggregate_verify calls, pks of message i = pks[seg_off[i] .. seg_off[i+1]).
 *
 * Grouped verdicts (batches of 2048..65536 independent checks: gbls_aggregate_verify_batch,
 * gbls_fast_aggregate_verify_batch / _indexed / _indexed_device).  Each check i is weighted by
 * a secret random 64-bit r_i drawn from getrandom(2) on every call, and 8 consecutive checks
 * share ONE Miller product and final exponentiation: prod_i (e(pk_i, H_i) e(-g1, sig_i))^r_i.
 * A group whose check passes gives SUCCESS to all its members; every member of a failed group
 * is re-checked on its own (deterministically: its own pairing product of the same pairs).
 * So a verdict can differ from the reference's deterministic check (signature.rs:77-93) only
 * when an invalid check sits in a group that passes, which happens with probability <= 2^-64
 * per group over the r_i (the random-linear-combination soundness of Signature::multi_verify,
 * signature.rs:95-129); a valid check is never rejected.  GBLS_INIT_PER_CHECK turns grouping
 * off (e.g. for spec tests). */
int gbls_fast_aggregate_verify_batch(const gbls_p2_affine *sigs, const uint8_t *msg_data,
                                     const uint32_t *msg_off, const gbls_p1_affine *pks,
                                     const uint32_t *seg_off, size_t m, int32_t *verdicts);

/* sync-committee shape over the registry: message i is checked against the aggregate of
 * registry keys pk_idx[seg_off[i] .. seg_off[i+1]) */
int gbls_fast_aggregate_verify_indexed(const gbls_p2_affine *sigs, const uint8_t *msg_data,
                                       const uint32_t *msg_off, const uint32_t *pk_idx,
                                       const uint32_t *seg_off, size_t m, int32_t *verdicts);

/* a1: random-linear-combination batch verification with caller-supplied nonzero
 * 64-bit scalars (bls/src/signature.rs:106-115 draws them); n == 0 -> VERIFY_FAIL
 * (MultiVerifier::finish short-circuits n == 0 before calling, verifier.rs:303-305). */
int gbls_multi_verify(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n);
/* nseg independent multi_verify batches: sets [seg_off[s], seg_off[s+1]) form batch s */
int gbls_multi_verify_segments(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                               const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                               const uint32_t *seg_off, size_t nseg, int32_t *verdicts);

/* a1 + a4 over the registry: set i's key = registry[pk_idx[i]] (pk_off == NULL) or the
 * aggregate of registry[pk_idx[pk_off[i] .. pk_off[i+1])] (Triple::verify_aggregate). */
int gbls_multi_verify_indexed(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                              const uint32_t *pk_idx, const uint32_t *pk_off,
                              const uint64_t *rands, size_t n);
/* a2, MultiVerifier::finish (helper_functions/src/verifier.rs:301-323) as ONE submission:
 * the 96-byte compressed signatures are decompressed on the device (a8 semantics, status
 * per signature in sig_status) on the signature-side stream while hash_to_G2 runs, then
 * multi_verify.  Keys: pks (points) or registry indices pk_idx (exactly one of them), each
 * either one key per set (pk_off == NULL) or summed per set over [pk_off[i], pk_off[i+1]) --
 * Triple::verify_aggregate's key sums (verifier.rs:387-405) done inside this one submission
 * instead of on rayon before it (an empty range fails the batch).  Returns the first nonzero
 * decompression status if any (finish's Err(DecompressionFailed), checked before the
 * verdict), else GBLS_SUCCESS / GBLS_VERIFY_FAIL. */
int gbls_multi_verify_compressed(const uint8_t (*msgs)[32], const uint8_t (*sigs)[96],
                                 const gbls_p1_affine *pks, const uint32_t *pk_idx,
                                 const uint32_t *pk_off, const uint64_t *rands, size_t n,
                                 int32_t *sig_status);
/* f3 priority class.  call_flags & GBLS_CALL_BLOCK marks block import (the block's
 * MultiVerifier::finish, which transition_functions/src/deneb/state_transition.rs:69-71 runs
 * on the critical path of importing it): the call has its own queue and leader slot per
 * device, so it never waits behind merged gossip submissions (themselves capped at 65536
 * sets), is merged only with other block calls (up to 8192 sets), and runs on streams of
 * the highest priority.  Otherwise identical to gbls_multi_verify_compressed. */
#define GBLS_CALL_BLOCK 0x1u
int gbls_multi_verify_compressed_ex(const uint8_t (*msgs)[32], const uint8_t (*sigs)[96],
                                    const gbls_p1_affine *pks, const uint32_t *pk_idx,
                                    const uint32_t *pk_off, const uint64_t *rands, size_t n,
                                    int32_t *sig_status, uint32_t call_flags);
/* f2: per-set verdicts (GBLS_SUCCESS / GBLS_VERIFY_FAIL, as each set would fare in
 * multi_verify alone) by GPU bisection: the batch, then rounds that split every failing
 * range 16 ways and verify all pieces as segments of one submission.  Keys come from
 * pks (points) or, when pks == NULL, from the registry as in gbls_multi_verify_indexed. */
int gbls_multi_verify_bisect(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                             const gbls_p1_affine *pks, const uint32_t *pk_idx,
                             const uint32_t *pk_off, const uint64_t *rands, size_t n,
                             int32_t *set_verdicts);

/* Device-pointer variants: inputs, outputs, verdicts and partials are device memory
 * (already resident in HBM); seg_off is a HOST array of nseg + 1 offsets (it sets the
 * launch geometry).  Asynchronous on `stream` (NULL = the legacy default stream, which
 * orders with PyTorch's default stream): the caller synchronises the stream. */
int gbls_multi_verify_segments_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                                      const uint32_t *seg_off, size_t nseg, int32_t *verdicts,
                                      void *stream);
/* registry-indexed: pk_idx / pk_off (may be NULL) are device arrays */
int gbls_multi_verify_indexed_segments_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                              const uint32_t *pk_idx, const uint32_t *pk_off,
                                              const uint64_t *rands, size_t n,
                                              const uint32_t *seg_off, size_t nseg,
                                              int32_t *verdicts, void *stream);
/* Multi-GPU split: per-segment Miller partial  F_s = prod_i ML(r_i pk_i, H(m_i)) * ML(-g1, S_s)
 * (no final exponentiation) + per-segment error flags; then the product of k partials
 * per segment and one final exponentiation.  An empty segment's partial is the identity
 * with no error (a shard may receive no sets); partials are laid out [part][segment]. */
int gbls_fast_aggregate_verify_indexed_device(const gbls_p2_affine *sigs, const uint8_t *msgs,
                                              const uint32_t *pk_idx, const uint32_t *pk_off,
                                              size_t m, int32_t *verdicts, void *stream);
int gbls_multi_verify_partials_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                                      const uint32_t *seg_off, size_t nseg, gbls_fp12 *partials,
                                      int32_t *seg_err, void *stream);
int gbls_multi_verify_indexed_partials_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                              const uint32_t *pk_idx, const uint32_t *pk_off,
                                              const uint64_t *rands, size_t n,
                                              const uint32_t *seg_off, size_t nseg,
                                              gbls_fp12 *partials, int32_t *seg_err,
                                              void *stream);
int gbls_final_verify_partials_device(const gbls_fp12 *partials, const int32_t *seg_err,
                                      size_t nparts, size_t nseg, int32_t *verdicts, void *stream);

/* a15 (fixture generation): sk = 32-byte big-endian scalars < r */
int gbls_sk_to_pk(const uint8_t (*sks)[32], size_t n, gbls_p1_affine *out);
int gbls_sign(const uint8_t (*sks)[32], const uint8_t *msg_data, const uint32_t *msg_off, size_t n,
              gbls_p2_affine *out);
/* hash_to_G2 with an explicit DST (RFC 9380 test vectors) -> affine points; dst == NULL with
 * dst_len == 0 selects the proof-of-possession scheme's DST that every verify entry uses */
int gbls_hash_to_g2(const uint8_t *msg_data, const uint32_t *msg_off, size_t n, const uint8_t *dst,
                    size_t dst_len, gbls_p2_affine *out);

/* roofline helper: measured v_mad_u64_u32 throughput of this device (mad64/s) */
double gbls_measure_mad64_peak(void);

/* Per-stage timing for bench.py: when enabled, HIP events bracket every pipeline stage
 * on the stream it is launched on.  gbls_profile_read() waits for recorded events,
 * accumulates milliseconds / launch counts per stage (names: gbls_stage_name) and
 * returns the number of stages. */
int gbls_profile(int enable);
int gbls_profile_read(double *ms, uint32_t *calls, int max_stages);
void gbls_profile_reset(void);
const char *gbls_stage_name(int stage);

#ifdef __cplusplus
}
#endif
#endif
