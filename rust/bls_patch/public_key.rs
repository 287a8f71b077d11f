// Replacement bodies for bls/src/public_key.rs:16-55.

impl TryFrom<PublicKeyBytes> for PublicKey {
    type Error = Error;

    /// public_key.rs:20-30: decompression + key validation (not infinity, in G1), which the
    /// reference needs for the fast_aggregate_verify spec tests.
    #[inline]
    fn try_from(bytes: PublicKeyBytes) -> Result<Self, Self::Error> {
        crate::gpu::g1_decompress_validate(bytes.as_bytes().try_into().expect("48 bytes"))
            .map(|raw| Self(RawPublicKey::from(raw)))
            .map_err(Error::DecompressionFailed)
    }
}

impl PublicKey {
    /// eth_aggregate_pubkeys: the sum of every key, Err for none.
    pub fn aggregate_nonempty(public_keys: impl IntoIterator<Item = Self>) -> Result<Self, Error> {
        let keys = public_keys
            .into_iter()
            .map(|key| crate::gpu::p1(&key.as_raw().into()))
            .collect::<Vec<_>>();
        if keys.is_empty() {
            return Err(Error::NoPublicKeysToAggregate);
        }
        let sum = crate::gpu::g1_sum(&keys).ok_or(Error::NoPublicKeysToAggregate)?;
        Ok(Self(RawPublicKey::from(crate::gpu::from_p1(&sum))))
    }

    #[inline]
    #[must_use]
    pub fn aggregate(mut self, other: Self) -> Self {
        self.aggregate_in_place(other);
        self
    }

    #[inline]
    pub fn aggregate_in_place(&mut self, other: Self) {
        let keys = [crate::gpu::p1(&self.as_raw().into()), crate::gpu::p1(&other.as_raw().into())];
        if let Some(sum) = crate::gpu::g1_sum(&keys) {
            self.0 = RawPublicKey::from(crate::gpu::from_p1(&sum));
        }
    }

    pub(crate) const fn as_raw(&self) -> &RawPublicKey {
        &self.0
    }
}
