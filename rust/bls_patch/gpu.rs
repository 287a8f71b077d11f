//! bls/src/gpu.rs -- routing between the MI355X engine and blst.
//!
//! This module contains no unsafe code: the `bls` crate keeps Grandine's workspace lints
//! (`unsafe_code = 'forbid'`, reference `Cargo.toml:65-66`, `bls/Cargo.toml:6-7`), and every
//! FFI call and point conversion is a safe function of `bls_gpu_sys`.
//!
//! Routing rule: a patched body runs on the engine when it is open and returns a verdict;
//! when the engine is absent (no gfx950 device, `gbls_init` failed) or a call reports an
//! engine error (`bls_gpu_sys::EngineError`: HIP/driver failure, argument outside the
//! engine's limits), the body runs its original blst code instead ("the Rust
//! shim falls back to the CPU path").  A verdict of the engine is never second-guessed: an
//! invalid signature is `false` on both paths, and only a missing verdict goes to the CPU.
//! A failed engine call therefore costs time, never a wrong answer or a silently kept value.

use core::sync::atomic::{AtomicU64, Ordering};
use std::sync::OnceLock;

pub use bls_gpu_sys::{CallClass, EngineError, P1, P2};

use crate::{PublicKey, Signature};

static CPU_FALLBACKS: AtomicU64 = AtomicU64::new(0);

/// Calls that ran on blst because the engine was absent or failed (for metrics / logs).
#[must_use]
pub fn cpu_fallbacks() -> u64 {
    CPU_FALLBACKS.load(Ordering::Relaxed)
}

/// `true` when the engine is open (opened on first use; cached for the process).
#[must_use]
pub fn available() -> bool {
    bls_gpu_sys::available()
}

/// Runs `gpu` when the engine is open and takes its result; otherwise, or when it reports an
/// engine error, runs `cpu` (the original blst body).
pub(crate) fn route<T>(gpu: impl FnOnce() -> Result<T, EngineError>, cpu: impl FnOnce() -> T) -> T {
    if available() {
        if let Ok(value) = gpu() {
            return value;
        }
    }
    CPU_FALLBACKS.fetch_add(1, Ordering::Relaxed);
    cpu()
}

/// Lone single checks -- one `verify`, one `fast_aggregate_verify`, one signature decompression,
/// a `SingleVerifier::extend` of fewer than `SINGLE_MIN_BATCH` triples -- run on the engine only
/// when `GBLS_SINGLE_CHECKS=engine`.  A lone check is latency-bound on the GPU (r05, idle MI355X,
/// `profiles/r05/z_bench_c1.json`: verify 3.0 ms p50, fast_aggregate_verify over 512 keys 3.1 ms,
/// decompression 0.58 ms; 16 threads of single verifies 3.5k/s even with cross-caller
/// coalescing), so by default blst answers it on the calling thread; batches always go to the
/// engine.
pub const SINGLE_MIN_BATCH: usize = 16;

#[must_use]
pub fn single_checks_on_engine() -> bool {
    static ON: OnceLock<bool> = OnceLock::new();
    *ON.get_or_init(|| std::env::var("GBLS_SINGLE_CHECKS").is_ok_and(|v| v == "engine"))
}

/// `route` for a lone single check: the engine only under `GBLS_SINGLE_CHECKS=engine`, else the
/// blst body directly (a policy choice, not a fallback: the fallback counter is not touched).
pub(crate) fn route_single<T>(gpu: impl FnOnce() -> Result<T, EngineError>, cpu: impl FnOnce() -> T) -> T {
    if single_checks_on_engine() {
        route(gpu, cpu)
    } else {
        cpu()
    }
}

/// Engine layout of a public key (for callers outside the crate, e.g. `MultiVerifier`).
#[must_use]
pub fn public_key_point(public_key: &PublicKey) -> P1 {
    bls_gpu_sys::p1_of_public_key(public_key.as_raw())
}

/// Engine layout of a signature.
#[must_use]
pub fn signature_point(signature: &Signature) -> P2 {
    bls_gpu_sys::p2_of_signature(signature.as_raw())
}

/// `MultiVerifier::finish` as one engine submission: 96-byte signatures decompressed on the
/// device, set i's key = the sum of `key_points[key_offsets[i] .. key_offsets[i + 1]]` formed on
/// the device (deferred `Triple::verify_aggregate`), then the random-linear-combination check
/// with the caller's nonzero scalars.
/// `None`: no engine verdict (absent engine or engine error) -- the caller runs its blst body.
/// `Some(Err(e))`: a signature does not decode (`DecompressionFailed(e)`);
/// `Some(Ok(v))`: the verdict.
#[must_use]
pub fn multi_verify_compressed(
    messages: &[[u8; 32]],
    signature_bytes: &[[u8; 96]],
    key_points: &[P1],
    key_offsets: &[u32],
    scalars: &[u64],
    class: CallClass,
) -> Option<Result<bool, blst::BLST_ERROR>> {
    counted(|| {
        bls_gpu_sys::multi_verify_compressed(messages, signature_bytes, key_points, key_offsets, scalars, class)
    })
}

/// `SingleVerifier::extend` as one engine submission (coalesced with concurrent callers):
/// per set, `Err(e)` when its signature does not decode, else whether it verifies against the
/// sum of its keys.  `None`: no engine verdict -- the caller runs its blst body.
#[must_use]
pub fn verify_batch_compressed(
    messages: &[[u8; 32]],
    signature_bytes: &[[u8; 96]],
    key_points: &[P1],
    key_offsets: &[u32],
) -> Option<Vec<Result<bool, blst::BLST_ERROR>>> {
    counted(|| bls_gpu_sys::verify_batch_compressed(messages, signature_bytes, key_points, key_offsets))
}

/// The engine call's value, or `None` (counted as a CPU fallback) when the engine is absent or
/// reports an error.
fn counted<T>(call: impl FnOnce() -> Result<T, EngineError>) -> Option<T> {
    if !available() {
        CPU_FALLBACKS.fetch_add(1, Ordering::Relaxed);
        return None;
    }
    let result = call();
    if result.is_err() {
        CPU_FALLBACKS.fetch_add(1, Ordering::Relaxed);
    }
    result.ok()
}

/// `MultiVerifier::finish` with registry indices (f1): as [`multi_verify_compressed`], set i's key
/// the sum of the registry keys `indices[index_offsets[i] .. index_offsets[i + 1]]`.
#[must_use]
pub fn multi_verify_compressed_indexed(
    messages: &[[u8; 32]],
    signature_bytes: &[[u8; 96]],
    indices: &[u32],
    index_offsets: &[u32],
    scalars: &[u64],
    class: CallClass,
) -> Option<Result<bool, blst::BLST_ERROR>> {
    counted(|| {
        bls_gpu_sys::multi_verify_compressed_indexed(messages, signature_bytes, indices, index_offsets, scalars, class)
    })
}

/// f4: `aggregate_in_place` of many message signatures into many aggregates in two engine calls
/// (the op-pool loops, `operation_pools/src/sync_committee_agg_pool/pool.rs:90-115,159-192`):
/// `additions[i] = (k, bytes)` adds the signature `bytes` to `bases[k]`, in order.  The encodings
/// are decoded in one call (`Signature::try_from` semantics) and every aggregate's sum is formed
/// in one `gbls_g2_aggregate_segments` submission.  When an encoding does not decode, only the
/// additions before the FIRST such one are summed and `Err((i, error))` names it, which is the
/// state the reference's `try_into()?` loop stops in.
/// `None`: no engine verdict (absent engine, engine error) -- `bases` is untouched and the
/// caller runs its blst loop.
#[must_use]
pub fn aggregate_into(
    bases: &mut [Signature],
    additions: &[(usize, crate::SignatureBytes)],
) -> Option<Result<(), (usize, crate::Error)>> {
    if additions.iter().any(|(k, _)| *k >= bases.len()) {
        return None;
    }
    let encodings = additions.iter().map(|(_, bytes)| bytes.to_fixed_bytes()).collect::<Vec<[u8; 96]>>();
    let decoded = counted(|| bls_gpu_sys::g2_decompress_many(&encodings))?;
    let first_bad = decoded.iter().position(Result::is_err);
    let upto = first_bad.unwrap_or(additions.len());
    let mut segments = bases.iter().map(|base| vec![signature_point(base)]).collect::<Vec<Vec<P2>>>();
    for ((k, _), point) in additions[..upto].iter().zip(&decoded) {
        segments[*k].push(*point.as_ref().ok()?);
    }
    let mut offsets = vec![0_u32];
    for segment in &segments {
        offsets.push(offsets[offsets.len() - 1] + u32::try_from(segment.len()).ok()?);
    }
    let points = segments.concat();
    let sums = counted(|| bls_gpu_sys::g2_aggregate_segments(&points, &offsets))?;
    // every sum converted before any base is replaced: a failure leaves `bases` as it was
    let raws = sums.iter().map(|sum| bls_gpu_sys::signature_of_p2(sum).ok()).collect::<Option<Vec<_>>>()?;
    for (base, raw) in bases.iter_mut().zip(raws) {
        *base = Signature::from(raw);
    }
    Some(match first_bad {
        None => Ok(()),
        Some(i) => Err((i, crate::Error::DecompressionFailed(decoded[i].err()?))),
    })
}

/// f1: the engine's copy of the validator registry (device-resident keys, decompressed once).
///
/// Validator indices name the same key on every fork only up to the finalized state: a deposit
/// processed on two branches can give one index two keys.  So the node mirrors the FINALIZED
/// state's validators (`mirror_finalized`, called where finalization advances and for the anchor
/// state at start-up), and a batch goes to the engine by indices only when every
/// index it names is below the mirrored length (`covers`); otherwise it keeps the key points.
pub mod registry {
    use std::sync::Mutex;

    use crate::PublicKeyBytes;

    /// validators loaded into the engine (a prefix of the finalized validator list)
    static MIRRORED: Mutex<usize> = Mutex::new(0);

    /// Loads validators `[mirrored, keys.len())` of a finalized state's validator list into the
    /// engine's registry (one `gbls_registry_set` for the new tail) and returns the mirrored
    /// length.  Keys never change once a validator is finalized, so the prefix already loaded is
    /// not sent again.  A key that does not decode leaves its slot empty (sets naming it fail,
    /// as `CachedPublicKey::decompress` would fail them).  Without an engine: 0.
    pub fn mirror_finalized(keys: &[PublicKeyBytes]) -> usize {
        let mut mirrored = MIRRORED.lock().unwrap_or_else(std::sync::PoisonError::into_inner);
        if !super::available() || keys.len() <= *mirrored {
            return *mirrored;
        }
        let tail = keys[*mirrored..].iter().map(|bytes| bytes.to_fixed_bytes()).collect::<Vec<[u8; 48]>>();
        if bls_gpu_sys::registry_set(*mirrored, &tail).is_ok() {
            *mirrored = keys.len();
        }
        *mirrored
    }

    /// The mirrored length (validators whose keys the engine resolves by index).
    #[must_use]
    pub fn mirrored() -> usize {
        *MIRRORED.lock().unwrap_or_else(std::sync::PoisonError::into_inner)
    }

    /// `true` when every index is below the mirrored length.
    #[must_use]
    pub fn covers(indices: &[u32]) -> bool {
        let mirrored = mirrored();
        indices.iter().all(|&index| usize::try_from(index).is_ok_and(|index| index < mirrored))
    }
}
