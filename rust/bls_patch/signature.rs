// Replacement bodies for bls/src/signature.rs:36-129 (the struct, its derives, the
// SignatureBytes conversions and the tests stay as they are).  blst stays a dependency for
// its types; the arithmetic runs on the MI355X engine through crate::gpu.

impl TryFrom<SignatureBytes> for Signature {
    type Error = Error;

    #[inline]
    fn try_from(bytes: SignatureBytes) -> Result<Self, Self::Error> {
        // signature.rs:40-44: decompression with blst semantics (on-curve, no group check)
        crate::gpu::g2_decompress(bytes.as_bytes().try_into().expect("96 bytes"))
            .map(|raw| Self(RawSignature::from(raw)))
            .map_err(Error::DecompressionFailed)
    }
}

impl Signature {
    /// signature.rs:47-60: sig_groupcheck = true, pk_validate = false (the engine checks the
    /// signature's subgroup membership and rejects an infinite public key).
    #[must_use]
    pub fn verify(self, message: impl AsRef<[u8]>, public_key: PublicKey) -> bool {
        crate::gpu::verify(&self.as_raw().into(), message.as_ref(), &public_key.as_raw().into())
    }

    #[inline]
    #[must_use]
    pub fn aggregate(mut self, other: Self) -> Self {
        self.aggregate_in_place(other);
        self
    }

    /// signature.rs:69-75: the sum of two G2 points (infinity-aware).
    pub fn aggregate_in_place(&mut self, other: Self) {
        let pts = [crate::gpu::p2(&self.as_raw().into()), crate::gpu::p2(&other.as_raw().into())];
        if let Some(sum) = crate::gpu::g2_sum(&pts) {
            self.0 = RawSignature::from(crate::gpu::from_p2(&sum));
        }
    }

    /// signature.rs:77-93: the keys are aggregated on the device (no key validation, as
    /// blst's `aggregate(pks, false)`); no keys -> false.
    #[must_use]
    pub fn fast_aggregate_verify<'keys>(
        &self,
        message: impl AsRef<[u8]>,
        public_keys: impl IntoIterator<Item = &'keys PublicKey>,
    ) -> bool {
        let keys = public_keys
            .into_iter()
            .map(|key| crate::gpu::p1(&key.as_raw().into()))
            .collect_vec();
        crate::gpu::fast_aggregate_verify(&self.as_raw().into(), message.as_ref(), &keys)
    }

    /// signature.rs:95-129: the random 64-bit scalars are still drawn here, from ThreadRng,
    /// one NonZeroU64 per set, and handed to the engine.
    #[must_use]
    pub fn multi_verify<'all>(
        messages: impl IntoIterator<Item = &'all [u8]>,
        signatures: impl IntoIterator<Item = &'all Self>,
        public_keys: impl IntoIterator<Item = &'all PublicKey>,
    ) -> bool {
        let messages = messages
            .into_iter()
            .map(|message| <[u8; 32]>::try_from(message).expect("signing roots are 32 bytes"))
            .collect_vec();
        let signatures = signatures
            .into_iter()
            .map(|signature| crate::gpu::p2(&signature.as_raw().into()))
            .collect_vec();
        let public_keys = public_keys
            .into_iter()
            .map(|key| crate::gpu::p1(&key.as_raw().into()))
            .collect_vec();

        let mut rng = rand::thread_rng();
        let randoms = core::iter::repeat_with(|| rng.gen::<NonZeroU64>().get())
            .take(signatures.len())
            .collect_vec();

        crate::gpu::multi_verify(&messages, &signatures, &public_keys, &randoms)
    }
}
