//! Raw bindings of `include/grandine_bls_gpu.h`, the C ABI of the MI355X BLS12-381 engine.
//!
//! Every prototype of the header is declared here with the same name, argument order and
//! meaning (`tests/test_rust_binding.py` parses both files and checks them against each other).
//! Point types have the layout of `blst_p1_affine` / `blst_p2_affine` (little-endian 64-bit
//! limbs, Montgomery form with R = 2^384, all-zero = infinity); the safe API of this crate
//! (`lib.rs`) converts blst values field by field.  Status codes mirror `BLST_ERROR`.  Any
//! device or driver failure is fail-closed (`GBLS_VERIFY_FAIL`, `gbls_last_error()` set).
#![allow(non_camel_case_types)]

use core::ffi::{c_char, c_int, c_void};

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct gbls_p1_affine {
    pub x: [u64; 6],
    pub y: [u64; 6],
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct gbls_p2_affine {
    pub x: [[u64; 6]; 2],
    pub y: [[u64; 6]; 2],
}

#[repr(C)]
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct gbls_fp12 {
    pub c: [[u64; 6]; 12],
}

// status codes (BLST_ERROR mirror)
pub const GBLS_SUCCESS: c_int = 0;
pub const GBLS_BAD_ENCODING: c_int = 1;
pub const GBLS_POINT_NOT_ON_CURVE: c_int = 2;
pub const GBLS_POINT_NOT_IN_GROUP: c_int = 3;
pub const GBLS_AGGR_TYPE_MISMATCH: c_int = 4;
pub const GBLS_VERIFY_FAIL: c_int = 5;
pub const GBLS_PK_IS_INFINITY: c_int = 6;
pub const GBLS_BAD_SCALAR: c_int = 7;
// gbls_last_error codes
pub const GBLS_ERR_NONE: c_int = 0;
pub const GBLS_ERR_NO_DEVICE: c_int = 100;
pub const GBLS_ERR_HIP: c_int = 101;
pub const GBLS_ERR_ARG: c_int = 102;
// gbls_init flags
pub const GBLS_INIT_NO_COALESCE: u32 = 0x100;
pub const GBLS_INIT_TUNING: u32 = 0x200;
pub const GBLS_INIT_PER_CHECK: u32 = 0x400;
// gbls_multi_verify_compressed_ex call flags
pub const GBLS_CALL_BLOCK: u32 = 0x1;

extern "C" {
    pub fn gbls_init(device_mask: u32, flags: u32) -> c_int;
    pub fn gbls_set_policy(flags: u32) -> u32;
    pub fn gbls_last_error() -> c_int;
    pub fn gbls_version() -> *const c_char;
    pub fn gbls_device_count() -> c_int;

    // a9 / a8 / a10
    pub fn gbls_g1_decompress(
        inp: *const [u8; 48],
        n: usize,
        validate: c_int,
        out: *mut gbls_p1_affine,
        status: *mut i32,
    ) -> c_int;
    pub fn gbls_g2_decompress(
        inp: *const [u8; 96],
        n: usize,
        out: *mut gbls_p2_affine,
        status: *mut i32,
    ) -> c_int;
    pub fn gbls_g2_validate(inp: *const gbls_p2_affine, n: usize, status: *mut i32) -> c_int;
    pub fn gbls_g1_compress(inp: *const gbls_p1_affine, n: usize, out: *mut [u8; 48]) -> c_int;
    pub fn gbls_g2_compress(inp: *const gbls_p2_affine, n: usize, out: *mut [u8; 96]) -> c_int;

    // a4 / a5 / a11
    pub fn gbls_g1_aggregate(pks: *const gbls_p1_affine, n: usize, out: *mut gbls_p1_affine) -> c_int;
    pub fn gbls_g1_aggregate_segments(
        pks: *const gbls_p1_affine,
        seg_offsets: *const u32,
        nseg: usize,
        out: *mut gbls_p1_affine,
        status: *mut i32,
    ) -> c_int;
    pub fn gbls_g2_aggregate(sigs: *const gbls_p2_affine, n: usize, out: *mut gbls_p2_affine) -> c_int;
    pub fn gbls_g2_aggregate_segments(
        sigs: *const gbls_p2_affine,
        seg_offsets: *const u32,
        nseg: usize,
        out: *mut gbls_p2_affine,
        status: *mut i32,
    ) -> c_int;

    // f1: device-resident validator registry
    pub fn gbls_registry_set(first: usize, pks: *const [u8; 48], n: usize, status: *mut i32) -> c_int;
    pub fn gbls_registry_size() -> usize;
    pub fn gbls_g1_aggregate_indexed(
        idx: *const u32,
        seg_offsets: *const u32,
        nseg: usize,
        out: *mut gbls_p1_affine,
        status: *mut i32,
    ) -> c_int;

    // a6 / a7
    pub fn gbls_verify(
        sig: *const gbls_p2_affine,
        msg: *const u8,
        msg_len: usize,
        pk: *const gbls_p1_affine,
    ) -> c_int;
    pub fn gbls_fast_aggregate_verify(
        sig: *const gbls_p2_affine,
        msg: *const u8,
        msg_len: usize,
        pks: *const gbls_p1_affine,
        n: usize,
    ) -> c_int;
    pub fn gbls_aggregate_verify_batch(
        sigs: *const gbls_p2_affine,
        msg_data: *const u8,
        msg_off: *const u32,
        pks: *const gbls_p1_affine,
        m: usize,
        verdicts: *mut i32,
    ) -> c_int;
    pub fn gbls_verify_batch_compressed(
        msgs: *const [u8; 32],
        sigs: *const [u8; 96],
        pks: *const gbls_p1_affine,
        pk_off: *const u32,
        m: usize,
        sig_status: *mut i32,
        verdicts: *mut i32,
    ) -> c_int;
    pub fn gbls_fast_aggregate_verify_batch(
        sigs: *const gbls_p2_affine,
        msg_data: *const u8,
        msg_off: *const u32,
        pks: *const gbls_p1_affine,
        seg_off: *const u32,
        m: usize,
        verdicts: *mut i32,
    ) -> c_int;
    pub fn gbls_fast_aggregate_verify_indexed(
        sigs: *const gbls_p2_affine,
        msg_data: *const u8,
        msg_off: *const u32,
        pk_idx: *const u32,
        seg_off: *const u32,
        m: usize,
        verdicts: *mut i32,
    ) -> c_int;

    // a1 / a2 / f2 / f3
    pub fn gbls_multi_verify(
        msgs: *const [u8; 32],
        sigs: *const gbls_p2_affine,
        pks: *const gbls_p1_affine,
        rands: *const u64,
        n: usize,
    ) -> c_int;
    pub fn gbls_multi_verify_segments(
        msgs: *const [u8; 32],
        sigs: *const gbls_p2_affine,
        pks: *const gbls_p1_affine,
        rands: *const u64,
        n: usize,
        seg_off: *const u32,
        nseg: usize,
        verdicts: *mut i32,
    ) -> c_int;
    pub fn gbls_multi_verify_indexed(
        msgs: *const [u8; 32],
        sigs: *const gbls_p2_affine,
        pk_idx: *const u32,
        pk_off: *const u32,
        rands: *const u64,
        n: usize,
    ) -> c_int;
    pub fn gbls_multi_verify_compressed(
        msgs: *const [u8; 32],
        sigs: *const [u8; 96],
        pks: *const gbls_p1_affine,
        pk_idx: *const u32,
        pk_off: *const u32,
        rands: *const u64,
        n: usize,
        sig_status: *mut i32,
    ) -> c_int;
    pub fn gbls_multi_verify_compressed_ex(
        msgs: *const [u8; 32],
        sigs: *const [u8; 96],
        pks: *const gbls_p1_affine,
        pk_idx: *const u32,
        pk_off: *const u32,
        rands: *const u64,
        n: usize,
        sig_status: *mut i32,
        call_flags: u32,
    ) -> c_int;
    pub fn gbls_multi_verify_bisect(
        msgs: *const [u8; 32],
        sigs: *const gbls_p2_affine,
        pks: *const gbls_p1_affine,
        pk_idx: *const u32,
        pk_off: *const u32,
        rands: *const u64,
        n: usize,
        set_verdicts: *mut i32,
    ) -> c_int;

    // device-pointer variants (inputs resident in HBM; asynchronous on `stream`)
    pub fn gbls_multi_verify_segments_device(
        msgs: *const u8,
        sigs: *const gbls_p2_affine,
        pks: *const gbls_p1_affine,
        rands: *const u64,
        n: usize,
        seg_off: *const u32,
        nseg: usize,
        verdicts: *mut i32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn gbls_multi_verify_indexed_segments_device(
        msgs: *const u8,
        sigs: *const gbls_p2_affine,
        pk_idx: *const u32,
        pk_off: *const u32,
        rands: *const u64,
        n: usize,
        seg_off: *const u32,
        nseg: usize,
        verdicts: *mut i32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn gbls_fast_aggregate_verify_indexed_device(
        sigs: *const gbls_p2_affine,
        msgs: *const u8,
        pk_idx: *const u32,
        pk_off: *const u32,
        m: usize,
        verdicts: *mut i32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn gbls_multi_verify_partials_device(
        msgs: *const u8,
        sigs: *const gbls_p2_affine,
        pks: *const gbls_p1_affine,
        rands: *const u64,
        n: usize,
        seg_off: *const u32,
        nseg: usize,
        partials: *mut gbls_fp12,
        seg_err: *mut i32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn gbls_multi_verify_indexed_partials_device(
        msgs: *const u8,
        sigs: *const gbls_p2_affine,
        pk_idx: *const u32,
        pk_off: *const u32,
        rands: *const u64,
        n: usize,
        seg_off: *const u32,
        nseg: usize,
        partials: *mut gbls_fp12,
        seg_err: *mut i32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn gbls_final_verify_partials_device(
        partials: *const gbls_fp12,
        seg_err: *const i32,
        nparts: usize,
        nseg: usize,
        verdicts: *mut i32,
        stream: *mut c_void,
    ) -> c_int;

    // a15: fixture generation only (not constant time)
    pub fn gbls_sk_to_pk(sks: *const [u8; 32], n: usize, out: *mut gbls_p1_affine) -> c_int;
    pub fn gbls_sign(
        sks: *const [u8; 32],
        msg_data: *const u8,
        msg_off: *const u32,
        n: usize,
        out: *mut gbls_p2_affine,
    ) -> c_int;
    pub fn gbls_hash_to_g2(
        msg_data: *const u8,
        msg_off: *const u32,
        n: usize,
        dst: *const u8,
        dst_len: usize,
        out: *mut gbls_p2_affine,
    ) -> c_int;

    // measurement helpers
    pub fn gbls_measure_mad64_peak() -> f64;
    pub fn gbls_profile(enable: c_int) -> c_int;
    pub fn gbls_profile_read(ms: *mut f64, calls: *mut u32, max_stages: c_int) -> c_int;
    pub fn gbls_profile_reset();
    pub fn gbls_stage_name(stage: c_int) -> *const c_char;
}
