//! bls/src/gpu.rs -- the one module of the `bls` crate that talks to the MI355X engine.
//!
//! blst's affine point types have exactly the engine's layout (48-byte little-endian
//! Montgomery coordinates, all-zero = infinity); the assertions below keep that true at compile
//! time.  Every wrapper is fail-closed: an engine or device error is a verification failure.
#![allow(unsafe_code)]

use core::{mem::size_of, ptr};

use bls_gpu_sys as sys;
use blst::{blst_p1_affine, blst_p2_affine, BLST_ERROR};
use static_assertions::assert_eq_size;

assert_eq_size!(blst_p1_affine, sys::gbls_p1_affine);
assert_eq_size!(blst_p2_affine, sys::gbls_p2_affine);

/// `gbls_init` once per process (idempotent on the C side): every GPU of the node.
pub fn init(device_mask: u32) -> bool {
    unsafe { sys::gbls_init(device_mask, 0) == sys::GBLS_SUCCESS }
}

#[inline]
pub(crate) fn p1(p: &blst_p1_affine) -> sys::gbls_p1_affine {
    unsafe { core::mem::transmute_copy(p) }
}

#[inline]
pub(crate) fn p2(p: &blst_p2_affine) -> sys::gbls_p2_affine {
    unsafe { core::mem::transmute_copy(p) }
}

#[inline]
pub(crate) fn from_p1(p: &sys::gbls_p1_affine) -> blst_p1_affine {
    unsafe { core::mem::transmute_copy(p) }
}

#[inline]
pub(crate) fn from_p2(p: &sys::gbls_p2_affine) -> blst_p2_affine {
    unsafe { core::mem::transmute_copy(p) }
}

/// BLST_ERROR from an engine status code (the engine mirrors BLST_ERROR's numbering).
/// The engine's view of a public key (for callers outside the crate, e.g. MultiVerifier).
pub fn public_key_point(pk: &crate::PublicKey) -> sys::gbls_p1_affine {
    p1(&pk.as_raw().into())
}

pub(crate) fn blst_error(status: i32) -> BLST_ERROR {
    match status {
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

pub(crate) fn g1_decompress_validate(bytes: &[u8; 48]) -> Result<blst_p1_affine, BLST_ERROR> {
    let mut out = sys::gbls_p1_affine::default();
    let mut status = sys::GBLS_BAD_ENCODING;
    let rc = unsafe { sys::gbls_g1_decompress(bytes, 1, 1, &mut out, &mut status) };
    match (rc, status) {
        (sys::GBLS_SUCCESS, 0) => Ok(from_p1(&out)),
        (sys::GBLS_SUCCESS, s) => Err(blst_error(s)),
        _ => Err(BLST_ERROR::BLST_BAD_ENCODING),
    }
}

pub(crate) fn g2_decompress(bytes: &[u8; 96]) -> Result<blst_p2_affine, BLST_ERROR> {
    let mut out = sys::gbls_p2_affine::default();
    let mut status = sys::GBLS_BAD_ENCODING;
    let rc = unsafe { sys::gbls_g2_decompress(bytes, 1, &mut out, &mut status) };
    match (rc, status) {
        (sys::GBLS_SUCCESS, 0) => Ok(from_p2(&out)),
        (sys::GBLS_SUCCESS, s) => Err(blst_error(s)),
        _ => Err(BLST_ERROR::BLST_BAD_ENCODING),
    }
}

pub(crate) fn g1_sum(points: &[sys::gbls_p1_affine]) -> Option<sys::gbls_p1_affine> {
    let mut out = sys::gbls_p1_affine::default();
    let rc = unsafe { sys::gbls_g1_aggregate(points.as_ptr(), points.len(), &mut out) };
    (rc == sys::GBLS_SUCCESS).then_some(out)
}

pub(crate) fn g2_sum(points: &[sys::gbls_p2_affine]) -> Option<sys::gbls_p2_affine> {
    let mut out = sys::gbls_p2_affine::default();
    let rc = unsafe { sys::gbls_g2_aggregate(points.as_ptr(), points.len(), &mut out) };
    (rc == sys::GBLS_SUCCESS).then_some(out)
}

pub(crate) fn verify(sig: &blst_p2_affine, msg: &[u8], pk: &blst_p1_affine) -> bool {
    let (s, p) = (p2(sig), p1(pk));
    unsafe { sys::gbls_verify(&s, msg.as_ptr(), msg.len(), &p) == sys::GBLS_SUCCESS }
}

pub(crate) fn fast_aggregate_verify(sig: &blst_p2_affine, msg: &[u8], pks: &[sys::gbls_p1_affine]) -> bool {
    let s = p2(sig);
    unsafe {
        sys::gbls_fast_aggregate_verify(&s, msg.as_ptr(), msg.len(), pks.as_ptr(), pks.len())
            == sys::GBLS_SUCCESS
    }
}

pub(crate) fn multi_verify(
    msgs: &[[u8; 32]],
    sigs: &[sys::gbls_p2_affine],
    pks: &[sys::gbls_p1_affine],
    rands: &[u64],
) -> bool {
    let n = msgs.len();
    if n == 0 || sigs.len() != n || pks.len() != n || rands.len() != n {
        return false;
    }
    unsafe {
        sys::gbls_multi_verify(msgs.as_ptr(), sigs.as_ptr(), pks.as_ptr(), rands.as_ptr(), n)
            == sys::GBLS_SUCCESS
    }
}

/// MultiVerifier::finish as one submission: the 96-byte signatures are decompressed on the
/// device.  Err(first failing status) when a signature does not decode, Ok(verdict) otherwise.
pub fn multi_verify_compressed(
    msgs: &[[u8; 32]],
    sig_bytes: &[[u8; 96]],
    pks: &[sys::gbls_p1_affine],
    rands: &[u64],
    block_import: bool,
) -> Result<bool, BLST_ERROR> {
    let n = msgs.len();
    if n == 0 || sig_bytes.len() != n || pks.len() != n || rands.len() != n {
        return Ok(false);
    }
    let mut status = vec![0_i32; n];
    let flags = if block_import { sys::GBLS_CALL_BLOCK } else { 0 };
    let rc = unsafe {
        sys::gbls_multi_verify_compressed_ex(
            msgs.as_ptr(),
            sig_bytes.as_ptr(),
            pks.as_ptr(),
            ptr::null(),
            ptr::null(),
            rands.as_ptr(),
            n,
            status.as_mut_ptr(),
            flags,
        )
    };
    match rc {
        sys::GBLS_SUCCESS => Ok(true),
        sys::GBLS_VERIFY_FAIL => Ok(false),
        s => Err(blst_error(s)),
    }
}

const _: () = assert!(size_of::<sys::gbls_p2_affine>() == 192 && size_of::<sys::gbls_p1_affine>() == 96);
