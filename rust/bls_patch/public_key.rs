// Replacement bodies for bls/src/public_key.rs:16-55.  Engine first (crate::gpu::route), the
// original blst code (`mod cpu`) when the engine is absent or reports an error.  No unsafe code.

/// Below this many keys an aggregate is a few microseconds of blst additions, less than one
/// engine round trip; from here on the engine's segmented G1 sum wins.
const ENGINE_MIN_KEYS: usize = 64;

impl TryFrom<PublicKeyBytes> for PublicKey {
    type Error = Error;

    /// public_key.rs:20-30: decompression + key validation (not infinity, in G1), which the
    /// reference needs for the fast_aggregate_verify spec tests.
    #[inline]
    fn try_from(bytes: PublicKeyBytes) -> Result<Self, Self::Error> {
        crate::gpu::route(
            || {
                bls_gpu_sys::g1_decompress(bytes.as_fixed_bytes(), true)
                    .map(|decoded| decoded.and_then(|point| bls_gpu_sys::public_key_of_p1(&point)).map(Self))
            },
            || cpu::decompress_validate(bytes).map(Self),
        )
        .map_err(Into::into)
    }
}

impl PublicKey {
    /// eth_aggregate_pubkeys: the sum of every key, Err for none.  Large sets (sync committees,
    /// attesting indices) are one engine call; an engine error re-runs the sum on blst.
    pub fn aggregate_nonempty(public_keys: impl IntoIterator<Item = Self>) -> Result<Self, Error> {
        let keys = public_keys.into_iter().collect::<Vec<_>>();
        if keys.is_empty() {
            return Err(Error::NoPublicKeysToAggregate);
        }
        if keys.len() < ENGINE_MIN_KEYS {
            return Ok(cpu::sum(&keys));
        }
        Ok(crate::gpu::route(
            || {
                let points = keys.iter().map(crate::gpu::public_key_point).collect::<Vec<_>>();
                let sum = bls_gpu_sys::g1_aggregate(&points)?;
                // the sum of valid keys is on the curve; anything else is an engine fault
                bls_gpu_sys::public_key_of_p1(&sum).map(Self).map_err(|_| crate::gpu::EngineError::Hip)
            },
            || cpu::sum(&keys),
        ))
    }

    #[inline]
    #[must_use]
    pub fn aggregate(mut self, other: Self) -> Self {
        self.aggregate_in_place(other);
        self
    }

    /// public_key.rs:47-53, unchanged: one G1 addition stays on blst (it cannot fail, and
    /// is far cheaper than an engine round trip).
    #[inline]
    pub fn aggregate_in_place(&mut self, other: Self) {
        cpu::aggregate_in_place(self, other);
    }

    pub(crate) const fn as_raw(&self) -> &RawPublicKey {
        &self.0
    }
}

/// The reference's blst bodies (public_key.rs:16-55).
mod cpu {
    use blst::BLST_ERROR;

    use super::*;

    pub(super) fn decompress_validate(bytes: PublicKeyBytes) -> Result<RawPublicKey, BLST_ERROR> {
        let raw = RawPublicKey::uncompress(bytes.as_bytes())?;
        raw.validate()?;
        Ok(raw)
    }

    pub(super) fn aggregate_in_place(public_key: &mut PublicKey, other: PublicKey) {
        let mut sum = RawAggregatePublicKey::from_public_key(public_key.as_raw());
        sum.add_aggregate(&RawAggregatePublicKey::from_public_key(other.as_raw()));
        public_key.0 = sum.to_public_key();
    }

    pub(super) fn sum(keys: &[PublicKey]) -> PublicKey {
        let mut total = keys[0];
        for key in &keys[1..] {
            aggregate_in_place(&mut total, *key);
        }
        total
    }
}
