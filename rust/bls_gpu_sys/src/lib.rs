//! Safe API of the MI355X BLS12-381 engine (`include/grandine_bls_gpu.h`).
//!
//! Grandine's workspace forbids unsafe code (`unsafe_code = 'forbid'`, reference
//! `Cargo.toml:65-66`, inherited by `bls/Cargo.toml:6-7`), so EVERY `unsafe` block of the
//! drop-in lives in this crate, which does not inherit the workspace lints.  The `bls` crate
//! calls only the safe functions below (`rust/bls_patch/`).
//!
//! * `ffi`: the raw prototypes, one per header entry point.
//! * Slice-taking wrappers that check lengths before the call, so no wrapper can hand the
//!   engine a pointer/length pair that does not describe a live Rust slice.
//! * Engine errors are values: every wrapper returns `Err(EngineError)` when the library
//!   reports a device, driver or argument failure (`gbls_last_error() != GBLS_ERR_NONE`), and
//!   `Ok(verdict)` only for a real verdict.  The `bls` crate answers `Err` by running the
//!   original blst body, so a node whose GPU is missing or broken still verifies on the CPU.
//! * Conversions between blst's raw points (`blst::min_pk::{PublicKey, Signature}`) and the
//!   engine's point layout copy the public limb arrays of `blst_fp` / `blst_fp2` field by field:
//!   blst -> engine through blst's safe `From<&PublicKey> for blst_p1_affine` (and the G2 twin),
//!   a plain copy of the Montgomery limbs (no serialisation, no curve check: the finish of a
//!   block converts ~66k keys); engine -> blst through blst's uncompressed decoder, which checks
//!   the point.  No `transmute`, no reliance on the private layout of blst's wrapper types.
#![deny(unsafe_op_in_unsafe_fn)]

pub mod ffi;

use core::{ffi::c_int, ptr};
use std::sync::OnceLock;

use blst::{
    blst_fp, blst_fp2, blst_p1_affine, blst_p2_affine,
    min_pk::{PublicKey as RawPublicKey, Signature as RawSignature},
    BLST_ERROR,
};

pub use ffi::{gbls_p1_affine as P1, gbls_p2_affine as P2};

// the engine's 64-bit limbs are blst's limb_t on every target Grandine builds for
const _: () = assert!(core::mem::size_of::<blst::limb_t>() == 8);
const _: () = assert!(core::mem::size_of::<P1>() == 96 && core::mem::size_of::<P2>() == 192);

/// Why an engine call produced no verdict (the library's `gbls_last_error` codes).
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum EngineError {
    /// no usable gfx950 device (or `gbls_init` failed)
    NoDevice,
    /// a HIP runtime / driver failure during the call
    Hip,
    /// arguments the engine rejects (lengths, offsets, sizes past its limits)
    Argument,
    /// any other code (a newer library)
    Other(i32),
}

impl EngineError {
    fn from_code(code: c_int) -> Self {
        match code {
            ffi::GBLS_ERR_NO_DEVICE => Self::NoDevice,
            ffi::GBLS_ERR_HIP => Self::Hip,
            ffi::GBLS_ERR_ARG => Self::Argument,
            other => Self::Other(other),
        }
    }
}

pub type EngineResult<T> = Result<T, EngineError>;

/// Call class of a batch verification (the engine's block-import priority class, f3).
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum CallClass {
    /// gossip, sync committee, API: merged with other normal calls
    Normal,
    /// the signatures of a block being imported (its own queue and high-priority streams)
    BlockImport,
}

/// The engine's error code for the call just made on this thread, if any.
fn last_error() -> Option<EngineError> {
    // SAFETY: reads a thread-local integer of the library; no arguments.
    let code = unsafe { ffi::gbls_last_error() };
    (code != ffi::GBLS_ERR_NONE).then(|| EngineError::from_code(code))
}

/// A verification return code -> verdict, or the engine error behind a fail-closed
/// `GBLS_VERIFY_FAIL`.
fn verdict(rc: c_int) -> EngineResult<bool> {
    if let Some(e) = last_error() {
        return Err(e);
    }
    match rc {
        ffi::GBLS_SUCCESS => Ok(true),
        ffi::GBLS_VERIFY_FAIL => Ok(false),
        other => Err(EngineError::Other(other)),
    }
}

/// A non-verification return code -> `()` or the engine error.
fn status(rc: c_int) -> EngineResult<()> {
    if let Some(e) = last_error() {
        return Err(e);
    }
    if rc == ffi::GBLS_SUCCESS {
        Ok(())
    } else {
        Err(EngineError::Other(rc))
    }
}

/// BLST_ERROR of an engine status code (the engine mirrors BLST_ERROR's numbering).
#[must_use]
pub fn blst_error(code: i32) -> BLST_ERROR {
    match code {
        0 => BLST_ERROR::BLST_SUCCESS,
        1 => BLST_ERROR::BLST_BAD_ENCODING,
        2 => BLST_ERROR::BLST_POINT_NOT_ON_CURVE,
        3 => BLST_ERROR::BLST_POINT_NOT_IN_GROUP,
        4 => BLST_ERROR::BLST_AGGR_TYPE_MISMATCH,
        6 => BLST_ERROR::BLST_PK_IS_INFINITY,
        7 => BLST_ERROR::BLST_BAD_SCALAR,
        _ => BLST_ERROR::BLST_VERIFY_FAIL,
    }
}

// ------------------------------------------------------------------ engine lifetime

static ENGINE: OnceLock<EngineResult<usize>> = OnceLock::new();

/// Opens the engine once per process on every GPU in `GBLS_DEVICE_MASK` (hex or decimal;
/// default: every device) and returns the number of engines, or why there is none.  The
/// result is cached: a node without a usable GPU pays for the probe once and then takes the
/// CPU path on every call without touching the library again.  `GBLS_PER_CHECK=1` asks for
/// deterministic per-check verdicts (`GBLS_INIT_PER_CHECK`, e.g. spec-test runs) and
/// `GBLS_NO_COALESCE=1` turns cross-caller coalescing off; both are sticky in the library, so
/// no later initialisation clears them (see also [`set_policy`]).
pub fn engine() -> EngineResult<usize> {
    *ENGINE.get_or_init(|| {
        let mask = std::env::var("GBLS_DEVICE_MASK")
            .ok()
            .and_then(|v| {
                let v = v.trim();
                v.strip_prefix("0x")
                    .map_or_else(|| v.parse().ok(), |h| u32::from_str_radix(h, 16).ok())
            })
            .unwrap_or(u32::MAX);
        let on = |name: &str| std::env::var(name).is_ok_and(|v| v.trim() == "1");
        let mut flags = 0;
        if on("GBLS_PER_CHECK") {
            flags |= ffi::GBLS_INIT_PER_CHECK;
        }
        if on("GBLS_NO_COALESCE") {
            flags |= ffi::GBLS_INIT_NO_COALESCE;
        }
        // SAFETY: plain integers in; the library serialises its own initialisation.
        let rc = unsafe { ffi::gbls_init(mask, flags) };
        status(rc)?;
        // SAFETY: no arguments.
        let n = unsafe { ffi::gbls_device_count() };
        usize::try_from(n).ok().filter(|&n| n > 0).ok_or(EngineError::NoDevice)
    })
}

/// Sets the engine's policies outright (`GBLS_INIT_PER_CHECK`, `GBLS_INIT_NO_COALESCE`; other
/// bits ignored) and returns the previous ones.  Needs no device.
pub fn set_policy(flags: u32) -> u32 {
    // SAFETY: a plain integer in and out.
    unsafe { ffi::gbls_set_policy(flags) }
}

/// `true` when the engine is open (see [`engine`]).
#[must_use]
pub fn available() -> bool {
    engine().is_ok()
}

// ------------------------------------------------------------------ point conversions

/// Engine layout of a blst public key: blst's affine point (its safe `From`), limbs copied.
/// Both sides hold Montgomery limbs (R = 2^384) with all-zero infinity, so nothing is recomputed.
#[cfg(not(feature = "serialized-points"))]
#[must_use]
pub fn p1_of_public_key(key: &RawPublicKey) -> P1 {
    let point = blst_p1_affine::from(key);
    P1 { x: point.x.l, y: point.y.l }
}

/// Engine layout of a blst public key (feature `serialized-points`): its uncompressed
/// serialisation decoded by blst's own decoder into the affine limbs (infinity -> all zero).
#[cfg(feature = "serialized-points")]
#[must_use]
pub fn p1_of_public_key(key: &RawPublicKey) -> P1 {
    let bytes = key.serialize();
    let mut point = blst_p1_affine::default();
    // SAFETY: `bytes` is a live 96-byte uncompressed encoding and `point` a valid output; a key
    // of blst's own type always decodes (its status carries no information here).
    let _status = unsafe { blst::blst_p1_deserialize(&mut point, bytes.as_ptr()) };
    P1 { x: point.x.l, y: point.y.l }
}

/// blst public key of an engine point (limb copy -> uncompressed serialisation -> blst's own
/// decoder, which checks that the point is on the curve).
pub fn public_key_of_p1(point: &P1) -> Result<RawPublicKey, BLST_ERROR> {
    let affine = blst_p1_affine { x: blst_fp { l: point.x }, y: blst_fp { l: point.y } };
    let mut bytes = [0_u8; 96];
    // SAFETY: `bytes` has room for the 96-byte encoding; `affine` is a valid input.
    unsafe { blst::blst_p1_affine_serialize(bytes.as_mut_ptr(), &affine) };
    RawPublicKey::deserialize(&bytes)
}

/// Engine layout of a blst signature (see [`p1_of_public_key`]).
#[cfg(not(feature = "serialized-points"))]
#[must_use]
pub fn p2_of_signature(signature: &RawSignature) -> P2 {
    let point = blst_p2_affine::from(signature);
    P2 { x: [point.x.fp[0].l, point.x.fp[1].l], y: [point.y.fp[0].l, point.y.fp[1].l] }
}

/// Engine layout of a blst signature (feature `serialized-points`, see [`p1_of_public_key`]).
#[cfg(feature = "serialized-points")]
#[must_use]
pub fn p2_of_signature(signature: &RawSignature) -> P2 {
    let bytes = signature.serialize();
    let mut point = blst_p2_affine::default();
    // SAFETY: `bytes` is a live 192-byte uncompressed encoding and `point` a valid output.
    let _status = unsafe { blst::blst_p2_deserialize(&mut point, bytes.as_ptr()) };
    P2 { x: [point.x.fp[0].l, point.x.fp[1].l], y: [point.y.fp[0].l, point.y.fp[1].l] }
}

/// blst signature of an engine point (on-curve checked by blst's decoder).
pub fn signature_of_p2(point: &P2) -> Result<RawSignature, BLST_ERROR> {
    let fp2 = |c: &[[u64; 6]; 2]| blst_fp2 { fp: [blst_fp { l: c[0] }, blst_fp { l: c[1] }] };
    let affine = blst_p2_affine { x: fp2(&point.x), y: fp2(&point.y) };
    let mut bytes = [0_u8; 192];
    // SAFETY: `bytes` has room for the 192-byte encoding; `affine` is a valid input.
    unsafe { blst::blst_p2_affine_serialize(bytes.as_mut_ptr(), &affine) };
    RawSignature::deserialize(&bytes)
}

// ------------------------------------------------------------------ safe entry points

/// a9: `PublicKey::try_from` (decompression + `validate()` when `validate`).  `Ok(Err(e))` is
/// the decoder's BLST_ERROR for these bytes; `Err` is an engine failure.
pub fn g1_decompress(bytes: &[u8; 48], validate: bool) -> EngineResult<Result<P1, BLST_ERROR>> {
    let mut out = P1::default();
    let mut st = ffi::GBLS_BAD_ENCODING;
    // SAFETY: one 48-byte input, one output point and one status, as n = 1 says.
    let rc = unsafe { ffi::gbls_g1_decompress(bytes, 1, c_int::from(validate), &mut out, &mut st) };
    status(rc)?;
    Ok(if st == ffi::GBLS_SUCCESS { Ok(out) } else { Err(blst_error(st)) })
}

/// a8: `Signature::try_from` (decompression, on-curve, no subgroup check).
pub fn g2_decompress(bytes: &[u8; 96]) -> EngineResult<Result<P2, BLST_ERROR>> {
    let mut out = P2::default();
    let mut st = ffi::GBLS_BAD_ENCODING;
    // SAFETY: one 96-byte input, one output point and one status, as n = 1 says.
    let rc = unsafe { ffi::gbls_g2_decompress(bytes, 1, &mut out, &mut st) };
    status(rc)?;
    Ok(if st == ffi::GBLS_SUCCESS { Ok(out) } else { Err(blst_error(st)) })
}

/// a5: the sum of `points` (infinity-aware).  An empty slice is an argument error.
pub fn g1_aggregate(points: &[P1]) -> EngineResult<P1> {
    if points.is_empty() {
        return Err(EngineError::Argument);
    }
    let mut out = P1::default();
    // SAFETY: `points` is a live slice of `points.len()` elements; one output point.
    let rc = unsafe { ffi::gbls_g1_aggregate(points.as_ptr(), points.len(), &mut out) };
    status(rc).map(|()| out)
}

/// a11: the sum of `points` (infinity-aware).  An empty slice is an argument error.
pub fn g2_aggregate(points: &[P2]) -> EngineResult<P2> {
    if points.is_empty() {
        return Err(EngineError::Argument);
    }
    let mut out = P2::default();
    // SAFETY: as in g1_aggregate.
    let rc = unsafe { ffi::gbls_g2_aggregate(points.as_ptr(), points.len(), &mut out) };
    status(rc).map(|()| out)
}

/// f4: `Signature::try_from` of many 96-byte encodings in one call: per input the point or the
/// decoder's BLST_ERROR (on-curve check only, as `RawSignature::uncompress`).
pub fn g2_decompress_many(bytes: &[[u8; 96]]) -> EngineResult<Vec<Result<P2, BLST_ERROR>>> {
    let n = bytes.len();
    if n == 0 {
        return Ok(Vec::new());
    }
    let mut out = vec![P2::default(); n];
    let mut statuses = vec![ffi::GBLS_BAD_ENCODING; n];
    // SAFETY: `bytes` is a live slice of n 96-byte encodings; n output points and n statuses.
    let rc = unsafe { ffi::gbls_g2_decompress(bytes.as_ptr(), n, out.as_mut_ptr(), statuses.as_mut_ptr()) };
    status(rc)?;
    Ok(out
        .into_iter()
        .zip(statuses)
        .map(|(point, s)| if s == ffi::GBLS_SUCCESS { Ok(point) } else { Err(blst_error(s)) })
        .collect())
}

/// f4: per segment s the sum of `points[offsets[s] .. offsets[s + 1]]`, every segment in one
/// submission (`Signature::aggregate_in_place` over an op-pool batch).  `offsets` starts at 0,
/// strictly increases (no empty segment) and ends at `points.len()`; otherwise an argument error.
pub fn g2_aggregate_segments(points: &[P2], offsets: &[u32]) -> EngineResult<Vec<P2>> {
    let nseg = offsets.len().checked_sub(1).ok_or(EngineError::Argument)?;
    let spans_points = usize::try_from(offsets[nseg]).is_ok_and(|end| end == points.len());
    if offsets[0] != 0 || !spans_points || offsets.windows(2).any(|w| w[1] <= w[0]) {
        return Err(EngineError::Argument);
    }
    if nseg == 0 {
        return Ok(Vec::new());
    }
    let mut out = vec![P2::default(); nseg];
    let mut statuses = vec![ffi::GBLS_AGGR_TYPE_MISMATCH; nseg];
    // SAFETY: `points` holds offsets[nseg] points and `offsets` nseg + 1 entries (checked above);
    // nseg output points and nseg statuses.
    let rc = unsafe {
        ffi::gbls_g2_aggregate_segments(points.as_ptr(), offsets.as_ptr(), nseg, out.as_mut_ptr(), statuses.as_mut_ptr())
    };
    status(rc)?;
    if statuses.iter().any(|&s| s != ffi::GBLS_SUCCESS) {
        return Err(EngineError::Argument);
    }
    Ok(out)
}

/// a6: `Signature::verify` semantics (signature subgroup check, infinite key rejected).
pub fn verify(signature: &P2, message: &[u8], key: &P1) -> EngineResult<bool> {
    // SAFETY: `message` is a live slice of `message.len()` bytes; single points by reference.
    let rc = unsafe { ffi::gbls_verify(signature, message.as_ptr(), message.len(), key) };
    verdict(rc)
}

/// a7: `Signature::fast_aggregate_verify` (no keys -> `Ok(false)`, as blst).
pub fn fast_aggregate_verify(signature: &P2, message: &[u8], keys: &[P1]) -> EngineResult<bool> {
    if keys.is_empty() {
        return Ok(false);
    }
    // SAFETY: live slices with their own lengths.
    let rc = unsafe {
        ffi::gbls_fast_aggregate_verify(signature, message.as_ptr(), message.len(), keys.as_ptr(), keys.len())
    };
    verdict(rc)
}

/// a1: `Signature::multi_verify` with caller-drawn nonzero scalars.  Slices of different
/// lengths, an empty batch or a zero scalar are argument errors (the caller falls back).
pub fn multi_verify(messages: &[[u8; 32]], signatures: &[P2], keys: &[P1], scalars: &[u64]) -> EngineResult<bool> {
    let n = messages.len();
    if n == 0 || signatures.len() != n || keys.len() != n || scalars.len() != n || scalars.contains(&0) {
        return Err(EngineError::Argument);
    }
    // SAFETY: four live slices of n elements each.
    let rc = unsafe {
        ffi::gbls_multi_verify(messages.as_ptr(), signatures.as_ptr(), keys.as_ptr(), scalars.as_ptr(), n)
    };
    verdict(rc)
}

/// `key_offsets` describe `n` key ranges over `keys`: n + 1 non-decreasing entries from 0 to
/// `keys.len()`.
fn key_ranges_ok(keys: &[P1], key_offsets: &[u32], n: usize) -> bool {
    key_offsets.len() == n + 1
        && key_offsets.first() == Some(&0)
        && key_offsets.windows(2).all(|w| w[0] <= w[1])
        && usize::try_from(key_offsets[n]).is_ok_and(|last| last == keys.len())
}

/// Per-set outcome of a compressed check: `Err` = the signature's BLST_ERROR (not decoded).
fn outcome(status: i32, verdict: i32) -> Result<bool, BLST_ERROR> {
    if status == ffi::GBLS_SUCCESS {
        Ok(verdict == ffi::GBLS_SUCCESS)
    } else {
        Err(blst_error(status))
    }
}

/// a2: `MultiVerifier::finish` as one submission (96-byte signatures decompressed on the
/// device; set i's key = the sum of `keys[key_offsets[i] .. key_offsets[i + 1]]`, formed on the
/// device).  `Ok(Err(e))`: the first signature that does not decode, with its BLST_ERROR
/// (finish's `DecompressionFailed`); `Ok(Ok(v))`: the verdict.
pub fn multi_verify_compressed(
    messages: &[[u8; 32]],
    signatures: &[[u8; 96]],
    keys: &[P1],
    key_offsets: &[u32],
    scalars: &[u64],
    class: CallClass,
) -> EngineResult<Result<bool, BLST_ERROR>> {
    let n = messages.len();
    if n == 0 || signatures.len() != n || scalars.len() != n || scalars.contains(&0) || !key_ranges_ok(keys, key_offsets, n)
    {
        return Err(EngineError::Argument);
    }
    let mut statuses = vec![ffi::GBLS_BAD_ENCODING; n];
    let flags = match class {
        CallClass::Normal => 0,
        CallClass::BlockImport => ffi::GBLS_CALL_BLOCK,
    };
    // SAFETY: live slices of n elements each, `keys` of key_offsets[n] points and
    // `key_offsets` of n + 1 entries (checked above; no index arrays).
    let rc = unsafe {
        ffi::gbls_multi_verify_compressed_ex(
            messages.as_ptr(),
            signatures.as_ptr(),
            keys.as_ptr(),
            ptr::null(),
            key_offsets.as_ptr(),
            scalars.as_ptr(),
            n,
            statuses.as_mut_ptr(),
            flags,
        )
    };
    if let Some(e) = last_error() {
        return Err(e);
    }
    Ok(match rc {
        ffi::GBLS_SUCCESS => Ok(true),
        ffi::GBLS_VERIFY_FAIL => Ok(false),
        decode => Err(blst_error(decode)),
    })
}

/// a6/a7 for `SingleVerifier::extend`: independent checks of 32-byte messages against 96-byte
/// signatures (decompressed on the device) and key sums `keys[key_offsets[i] ..
/// key_offsets[i + 1]]`, in one coalesced submission.  Per set: `Err(e)` = the signature does not
/// decode (its BLST_ERROR), else whether it verifies.
pub fn verify_batch_compressed(
    messages: &[[u8; 32]],
    signatures: &[[u8; 96]],
    keys: &[P1],
    key_offsets: &[u32],
) -> EngineResult<Vec<Result<bool, BLST_ERROR>>> {
    let n = messages.len();
    if signatures.len() != n || !key_ranges_ok(keys, key_offsets, n) {
        return Err(EngineError::Argument);
    }
    if n == 0 {
        return Ok(Vec::new());
    }
    let mut statuses = vec![ffi::GBLS_BAD_ENCODING; n];
    let mut verdicts = vec![ffi::GBLS_VERIFY_FAIL; n];
    // SAFETY: live slices of n elements each, `keys` of key_offsets[n] points and `key_offsets`
    // of n + 1 entries (checked above); n status and n verdict slots.
    let rc = unsafe {
        ffi::gbls_verify_batch_compressed(
            messages.as_ptr(),
            signatures.as_ptr(),
            keys.as_ptr(),
            key_offsets.as_ptr(),
            n,
            statuses.as_mut_ptr(),
            verdicts.as_mut_ptr(),
        )
    };
    status(rc)?;
    Ok(statuses.into_iter().zip(verdicts).map(|(s, v)| outcome(s, v)).collect())
}

/// f1: loads compressed public keys at registry slots `first ..` (decompressed and validated once
/// on the device, replicated to every engine device).  Per key: `Ok(())`, or the decoder's
/// BLST_ERROR (that slot stays empty and a set naming it fails).
pub fn registry_set(first: usize, keys: &[[u8; 48]]) -> EngineResult<Vec<Result<(), BLST_ERROR>>> {
    let mut statuses = vec![ffi::GBLS_BAD_ENCODING; keys.len()];
    // SAFETY: `keys` is a live slice of keys.len() 48-byte entries and `statuses` as many slots.
    let rc = unsafe { ffi::gbls_registry_set(first, keys.as_ptr(), keys.len(), statuses.as_mut_ptr()) };
    status(rc)?;
    Ok(statuses.into_iter().map(|s| if s == ffi::GBLS_SUCCESS { Ok(()) } else { Err(blst_error(s)) }).collect())
}

/// f1: the number of registry slots loaded (0 before any `registry_set`).
#[must_use]
pub fn registry_size() -> usize {
    // SAFETY: no arguments; the library guards its registry with its own lock.
    unsafe { ffi::gbls_registry_size() }
}

/// a2 + f1: `MultiVerifier::finish` as one submission with REGISTRY INDICES: set i's key is the
/// sum of the registry keys `indices[index_offsets[i] .. index_offsets[i + 1]]` (gathered and
/// summed on the device), signatures as 96-byte encodings decompressed in the same submission.
/// `Ok(Err(e))`: the first signature that does not decode; `Ok(Ok(v))`: the verdict.  An index
/// past the registry fails its set (a verdict, not an error).
pub fn multi_verify_compressed_indexed(
    messages: &[[u8; 32]],
    signatures: &[[u8; 96]],
    indices: &[u32],
    index_offsets: &[u32],
    scalars: &[u64],
    class: CallClass,
) -> EngineResult<Result<bool, BLST_ERROR>> {
    let n = messages.len();
    let ranges_ok = index_offsets.len() == n + 1
        && index_offsets.first() == Some(&0)
        && index_offsets.windows(2).all(|w| w[0] <= w[1])
        && usize::try_from(index_offsets[n]).is_ok_and(|last| last == indices.len());
    if n == 0 || signatures.len() != n || scalars.len() != n || scalars.contains(&0) || !ranges_ok {
        return Err(EngineError::Argument);
    }
    let mut statuses = vec![ffi::GBLS_BAD_ENCODING; n];
    let flags = match class {
        CallClass::Normal => 0,
        CallClass::BlockImport => ffi::GBLS_CALL_BLOCK,
    };
    // SAFETY: live slices of n elements each, `indices` of index_offsets[n] entries and
    // `index_offsets` of n + 1 (checked above); no key points.
    let rc = unsafe {
        ffi::gbls_multi_verify_compressed_ex(
            messages.as_ptr(),
            signatures.as_ptr(),
            ptr::null(),
            indices.as_ptr(),
            index_offsets.as_ptr(),
            scalars.as_ptr(),
            n,
            statuses.as_mut_ptr(),
            flags,
        )
    };
    if let Some(e) = last_error() {
        return Err(e);
    }
    Ok(match rc {
        ffi::GBLS_SUCCESS => Ok(true),
        ffi::GBLS_VERIFY_FAIL => Ok(false),
        decode => Err(blst_error(decode)),
    })
}

/// f2: per-set verdicts of a batch (`true` = the set verifies on its own).
pub fn multi_verify_bisect(
    messages: &[[u8; 32]],
    signatures: &[P2],
    keys: &[P1],
    scalars: &[u64],
) -> EngineResult<Vec<bool>> {
    let n = messages.len();
    if signatures.len() != n || keys.len() != n || scalars.len() != n || scalars.contains(&0) {
        return Err(EngineError::Argument);
    }
    if n == 0 {
        return Ok(Vec::new());
    }
    let mut verdicts = vec![ffi::GBLS_VERIFY_FAIL; n];
    // SAFETY: live slices of n elements each; n verdict slots.
    let rc = unsafe {
        ffi::gbls_multi_verify_bisect(
            messages.as_ptr(),
            signatures.as_ptr(),
            keys.as_ptr(),
            ptr::null(),
            ptr::null(),
            scalars.as_ptr(),
            n,
            verdicts.as_mut_ptr(),
        )
    };
    status(rc)?;
    Ok(verdicts.into_iter().map(|v| v == ffi::GBLS_SUCCESS).collect())
}
