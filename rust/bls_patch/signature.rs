// Replacement bodies for bls/src/signature.rs:36-129 (the struct, its derives, the
// SignatureBytes conversions and the tests stay as they are).  Every body first asks the
// MI355X engine (crate::gpu::route) and runs the original blst code, kept verbatim in
// `mod cpu` below, when the engine is absent or reports an error.  No unsafe code.

impl TryFrom<SignatureBytes> for Signature {
    type Error = Error;

    #[inline]
    fn try_from(bytes: SignatureBytes) -> Result<Self, Self::Error> {
        // signature.rs:40-44: decompression with blst semantics (on-curve, no group check); a lone
        // decompression stays on blst unless GBLS_SINGLE_CHECKS=engine (crate::gpu::route_single)
        crate::gpu::route_single(
            || {
                bls_gpu_sys::g2_decompress(bytes.as_fixed_bytes()).map(|decoded| {
                    decoded.and_then(|point| bls_gpu_sys::signature_of_p2(&point)).map(Self)
                })
            },
            || cpu::decompress(bytes).map(Self),
        )
        .map_err(Into::into)
    }
}

impl Signature {
    /// signature.rs:47-60: sig_groupcheck = true, pk_validate = false (the engine checks the
    /// signature's subgroup membership and rejects an infinite public key).
    #[must_use]
    pub fn verify(self, message: impl AsRef<[u8]>, public_key: PublicKey) -> bool {
        let message = message.as_ref();
        crate::gpu::route_single(
            || {
                bls_gpu_sys::verify(
                    &crate::gpu::signature_point(&self),
                    message,
                    &crate::gpu::public_key_point(&public_key),
                )
            },
            || cpu::verify(&self, message, &public_key),
        )
    }

    #[inline]
    #[must_use]
    pub fn aggregate(mut self, other: Self) -> Self {
        self.aggregate_in_place(other);
        self
    }

    /// signature.rs:69-75, unchanged: the sum of TWO points is one G2 addition (~1 us in
    /// blst), far below one PCIe round trip to the engine, so it stays on the CPU and can
    /// never fail.  Many-signature sums go to the engine as one call
    /// (`bls_gpu_sys::g2_aggregate`, or `gbls_g2_aggregate_segments` for op-pool batches).
    #[inline]
    pub fn aggregate_in_place(&mut self, other: Self) {
        cpu::aggregate_in_place(self, other);
    }

    /// signature.rs:77-93: the keys are aggregated on the device (no key validation, as
    /// blst's `aggregate(pks, false)`); no keys -> false.
    #[must_use]
    pub fn fast_aggregate_verify<'keys>(
        &self,
        message: impl AsRef<[u8]>,
        public_keys: impl IntoIterator<Item = &'keys PublicKey>,
    ) -> bool {
        let message = message.as_ref();
        let public_keys = public_keys.into_iter().collect_vec();
        crate::gpu::route_single(
            || {
                let points = public_keys.iter().map(|key| crate::gpu::public_key_point(key)).collect_vec();
                bls_gpu_sys::fast_aggregate_verify(&crate::gpu::signature_point(self), message, &points)
            },
            || cpu::fast_aggregate_verify(self, message, &public_keys),
        )
    }

    /// signature.rs:95-129: the random 64-bit scalars are drawn here, from ThreadRng, one
    /// NonZeroU64 per set, as in the reference.  Messages of any length are accepted: the
    /// engine path takes 32-byte signing roots (every consensus caller), anything else runs
    /// the blst body.
    #[must_use]
    pub fn multi_verify<'all>(
        messages: impl IntoIterator<Item = &'all [u8]>,
        signatures: impl IntoIterator<Item = &'all Self>,
        public_keys: impl IntoIterator<Item = &'all PublicKey>,
    ) -> bool {
        let messages = messages.into_iter().collect_vec();
        let signatures = signatures.into_iter().collect_vec();
        let public_keys = public_keys.into_iter().collect_vec();

        let mut rng = rand::thread_rng();
        let randoms = core::iter::repeat_with(|| rng.gen::<NonZeroU64>().get())
            .take(signatures.len())
            .collect_vec();

        crate::gpu::route(
            || {
                let roots = messages
                    .iter()
                    .map(|message| <[u8; 32]>::try_from(*message).map_err(|_| crate::gpu::EngineError::Argument))
                    .collect::<Result<Vec<_>, _>>()?;
                let sigs = signatures.iter().map(|s| crate::gpu::signature_point(s)).collect_vec();
                let keys = public_keys.iter().map(|k| crate::gpu::public_key_point(k)).collect_vec();
                bls_gpu_sys::multi_verify(&roots, &sigs, &keys, &randoms)
            },
            || cpu::multi_verify(&messages, &signatures, &public_keys, &randoms),
        )
    }

    pub(crate) const fn as_raw(&self) -> &RawSignature {
        &self.0
    }
}

/// The reference's blst bodies (signature.rs:36-129), the path taken without an engine verdict.
mod cpu {
    use itertools::Itertools as _;

    use super::*;

    pub(super) fn decompress(bytes: SignatureBytes) -> Result<RawSignature, BLST_ERROR> {
        RawSignature::uncompress(bytes.as_bytes())
    }

    pub(super) fn verify(signature: &Signature, message: &[u8], public_key: &PublicKey) -> bool {
        let result = signature.as_raw().verify(true, message, DOMAIN_SEPARATION_TAG, &[], public_key.as_raw(), false);
        result == BLST_ERROR::BLST_SUCCESS
    }

    pub(super) fn aggregate_in_place(signature: &mut Signature, other: Signature) {
        let mut sum = RawAggregateSignature::from_signature(signature.as_raw());
        sum.add_aggregate(&RawAggregateSignature::from_signature(other.as_raw()));
        signature.0 = sum.to_signature();
    }

    pub(super) fn fast_aggregate_verify(signature: &Signature, message: &[u8], public_keys: &[&PublicKey]) -> bool {
        let raw_keys = public_keys.iter().map(|key| key.as_raw()).collect_vec();
        let result = signature.as_raw().fast_aggregate_verify(true, message, DOMAIN_SEPARATION_TAG, &raw_keys);
        result == BLST_ERROR::BLST_SUCCESS
    }

    pub(super) fn multi_verify(
        messages: &[&[u8]],
        signatures: &[&Signature],
        public_keys: &[&PublicKey],
        randoms: &[u64],
    ) -> bool {
        let raw_signatures = signatures.iter().map(|s| s.as_raw()).collect_vec();
        let raw_keys = public_keys.iter().map(|k| k.as_raw()).collect_vec();
        let scalars = randoms
            .iter()
            .map(|random| {
                let mut scalar = blst_scalar::default();
                scalar.b[..MULTI_VERIFY_RANDOM_BYTES].copy_from_slice(&random.to_le_bytes());
                scalar
            })
            .collect_vec();
        let result = RawSignature::verify_multiple_aggregate_signatures(
            messages,
            DOMAIN_SEPARATION_TAG,
            &raw_keys,
            false,
            &raw_signatures,
            false,
            &scalars,
            MULTI_VERIFY_RANDOM_BITS,
        );
        result == BLST_ERROR::BLST_SUCCESS
    }
}
