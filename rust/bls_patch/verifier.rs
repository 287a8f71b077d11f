// Replacement bodies for helper_functions/src/verifier.rs (the Verifier trait, NullVerifier and the
// options enum stay as they are).  No unsafe code (helper_functions keeps the workspace's
// `unsafe_code = 'forbid'`).
//
// What changes, and why:
//
// * `Triple` DEFERS key aggregation.  The reference reduces an attestation's keys on rayon as
//   soon as the triple is built (`Triple::verify_aggregate`, verifier.rs:387-405:
//   `par_bridge().reduce(AggregatePublicKey::default, AggregatePublicKey::aggregate)`, one blst
//   addition plus a field inversion per key).  Here the triple keeps its key list and
//   `MultiVerifier::finish` hands every list to the engine with per-set offsets
//   (`gbls_multi_verify_compressed_ex`, points + pk_off): the sums are formed on the device
//   inside the same submission as decompression, hash_to_G2 and the batch check.  Nothing on
//   this path calls `AggregatePublicKey::aggregate`; the block path builds its attestation
//   triples with `Triple::verify_aggregate` directly (transition_functions/src/deneb/
//   state_transition.rs:161, p2p/src/attestation_verifier.rs:442), so deferring in `Triple`
//   covers it as well as `MultiVerifier::verify_aggregate`.
// * `SingleVerifier::extend` verifies all its triples in ONE engine submission
//   (`gbls_verify_batch_compressed`): decompression and verification together, coalesced with
//   concurrent callers, instead of a decompression call and a verify call per triple.  Errors
//   come out in the reference's order: the first triple that fails to decode gives
//   `DecompressionFailed`, the first that fails to verify `SignatureInvalid(kind)`.
// * `MultiVerifier::finish` is one submission (verifier.rs:301-323); block import asks for the
//   engine's block-import priority class through one new option, added to the enum at
//   verifier.rs:432-436:
//
//       pub enum VerifierOption { SkipBlockBaseSignatures, SkipBlockSyncAggregateSignature,
//                                 SkipRandaoVerification, BlockImport }
//
//   which the block paths pass when they build their verifier
//   (p2p/src/block_verification_pool.rs:109, fork_choice_control/src/tasks.rs:101).
//
// * f1 (r06): the `Verifier` trait gains one provided method, added at verifier.rs:16-69 and
//   forwarded by `impl<V: Verifier> Verifier for &mut V` (verifier.rs:73-119):
//
//       fn verify_aggregate_indexed<'keys>(&mut self, message: H256, signature_bytes: SignatureBytes,
//           validator_indices: &[ValidatorIndex],
//           public_keys: impl IntoIterator<IntoIter = impl Iterator<Item = &'keys PublicKey> + Send>,
//           signature_kind: SignatureKind) -> Result<()> {
//           self.verify_aggregate(message, signature_bytes, public_keys, signature_kind)
//       }
//
//   `Triple` and `MultiVerifier` override it to keep the indices; the attestation predicate calls
//   it (rust/bls_patch/predicates.rs).  `finish` then names registry slots (4 bytes per key)
//   instead of 96-byte points when the engine mirrors those validators (bls::gpu::registry).
//
// Without an engine verdict (no device, engine error) each body runs the reference's blst code,
// with the deferred sums formed by blst first (`Triple::public_key`).

/// verifier.rs:349-354, plus the deferred key list of `verify_aggregate` and, when the caller
/// knows them, the keys' validator indices (f1, `verify_aggregate_indexed`).
#[derive(Default)]
pub struct Triple {
    message: H256,
    signature_bytes: SignatureBytes,
    public_key: PublicKey,
    // Some(keys): the public key is the sum of `keys` (Triple::verify_aggregate), not yet formed
    deferred: Option<Vec<PublicKey>>,
    // Some(indices): the deferred keys are these validators' (the engine's registry can resolve
    // them on the device, bls::gpu::registry)
    indices: Option<Vec<u32>>,
}

assert_not_impl_any!(Triple: Copy);

impl Triple {
    /// The reference's `derive(Constructor)` (verifier.rs:349): one resolved key.
    #[must_use]
    pub const fn new(message: H256, signature_bytes: SignatureBytes, public_key: PublicKey) -> Self {
        Self { message, signature_bytes, public_key, deferred: None, indices: None }
    }

    /// The set's key for the blst bodies: the deferred sum formed now (reference reduce, identity
    /// `AggregatePublicKey::default`), or the resolved key.
    fn public_key(&self) -> PublicKey {
        match &self.deferred {
            Some(keys) => keys.iter().copied().fold(AggregatePublicKey::default(), AggregatePublicKey::aggregate),
            None => self.public_key,
        }
    }

    /// The set's keys in the engine's layout, appended to `points` (one point, or the deferred list).
    fn push_key_points(&self, points: &mut Vec<bls::gpu::P1>) {
        match &self.deferred {
            Some(keys) => points.extend(keys.iter().map(bls::gpu::public_key_point)),
            None => points.push(bls::gpu::public_key_point(&self.public_key)),
        }
    }
}

/// Registry arguments of a run of triples (f1): every set's validator indices and per-set offsets,
/// or `None` when some set has no indices or names a validator the engine's registry does not
/// mirror (the caller then ships key points, engine_sets).
fn engine_indices(triples: &[Triple]) -> Option<(Vec<u32>, Vec<u32>)> {
    let mut indices = Vec::new();
    let mut offsets = Vec::with_capacity(triples.len() + 1);
    offsets.push(0);
    for triple in triples {
        indices.extend_from_slice(triple.indices.as_deref()?);
        offsets.push(u32::try_from(indices.len()).ok()?);
    }
    bls::gpu::registry::covers(&indices).then_some((indices, offsets))
}

/// Engine arguments of a run of triples: 32-byte messages, 96-byte signatures, key points and
/// per-set key offsets (pk_off[i] .. pk_off[i + 1] are set i's keys).
fn engine_sets(triples: &[Triple]) -> (Vec<[u8; 32]>, Vec<[u8; 96]>, Vec<bls::gpu::P1>, Vec<u32>) {
    let messages = triples.iter().map(|triple| triple.message.to_fixed_bytes()).collect_vec();
    let signature_bytes = triples.iter().map(|triple| triple.signature_bytes.to_fixed_bytes()).collect_vec();
    let mut points = Vec::with_capacity(triples.len());
    let mut offsets = Vec::with_capacity(triples.len() + 1);
    offsets.push(0);
    for triple in triples {
        triple.push_key_points(&mut points);
        // a key count past u32 is an argument the engine rejects: the caller falls back to blst
        offsets.push(u32::try_from(points.len()).unwrap_or(u32::MAX));
    }
    (messages, signature_bytes, points, offsets)
}

impl Verifier for Triple {
    const IS_NULL: bool = false;

    #[inline]
    fn reserve(&mut self, _additional: usize) {
        unimplemented!("<Triple as Verifier>::reserve is not used anywhere")
    }

    #[inline]
    fn verify_singular(
        &mut self,
        _message: H256,
        _signature_bytes: SignatureBytes,
        _cached_public_key: &CachedPublicKey,
        _signature_kind: SignatureKind,
    ) -> Result<()> {
        unimplemented!("<Triple as Verifier>::verify_singular is not used anywhere")
    }

    /// verifier.rs:387-405 without the rayon reduce: the keys are kept and summed on the device
    /// by the submission that verifies the triple.
    #[inline]
    fn verify_aggregate<'keys>(
        &mut self,
        message: H256,
        signature_bytes: SignatureBytes,
        public_keys: impl IntoIterator<IntoIter = impl Iterator<Item = &'keys PublicKey> + Send>,
        _signature_kind: SignatureKind,
    ) -> Result<()> {
        let keys = public_keys.into_iter().copied().collect_vec();
        *self = Self { message, signature_bytes, public_key: PublicKey::default(), deferred: Some(keys), indices: None };
        Ok(())
    }

    /// f1 (r06): `verify_aggregate` that also keeps the keys' validator indices, so that
    /// `MultiVerifier::finish` can name registry slots instead of shipping 96-byte points when the
    /// engine's registry mirrors those validators (bls::gpu::registry::covers).  The keys are kept
    /// as well: the points path and the blst fallback use them.
    #[inline]
    fn verify_aggregate_indexed<'keys>(
        &mut self,
        message: H256,
        signature_bytes: SignatureBytes,
        validator_indices: &[ValidatorIndex],
        public_keys: impl IntoIterator<IntoIter = impl Iterator<Item = &'keys PublicKey> + Send>,
        signature_kind: SignatureKind,
    ) -> Result<()> {
        self.verify_aggregate(message, signature_bytes, public_keys, signature_kind)?;
        // an index past u32 (no such validator set exists) keeps the points path
        self.indices = validator_indices.iter().map(|&index| u32::try_from(index).ok()).collect();
        Ok(())
    }

    #[inline]
    fn extend(&mut self, _triples: impl IntoIterator<Item = Self>, _signature_kind: SignatureKind) -> Result<()> {
        unimplemented!("<Triple as Verifier>::extend is not used anywhere")
    }

    #[inline]
    fn finish(&self) -> Result<()> {
        unimplemented!("<Triple as Verifier>::finish is not used anywhere")
    }

    #[inline]
    fn has_option(&self, _option: VerifierOption) -> bool {
        false
    }
}

// ---------------------------------------------------------------- SingleVerifier::extend
// (verifier.rs:215-236; verify_singular and verify_aggregate keep the reference bodies: the
// first calls extend, the second Signature::fast_aggregate_verify, which is one engine call)

#[inline]
fn extend(&mut self, triples: impl IntoIterator<Item = Triple>, signature_kind: SignatureKind) -> Result<()> {
    let triples = triples.into_iter().collect_vec();
    if triples.is_empty() {
        return Ok(());
    }
    // a few triples are lone checks: blst on this thread unless GBLS_SINGLE_CHECKS=engine
    if triples.len() < bls::gpu::SINGLE_MIN_BATCH && !bls::gpu::single_checks_on_engine() {
        return extend_on_cpu(&triples, signature_kind);
    }
    let (messages, signature_bytes, points, offsets) = engine_sets(&triples);
    match bls::gpu::verify_batch_compressed(&messages, &signature_bytes, &points, &offsets) {
        Some(outcomes) => {
            for outcome in outcomes {
                // the reference's order per triple: try_from (`?`), then verify
                let verified = outcome.map_err(bls::Error::DecompressionFailed)?;
                ensure!(verified, Error::SignatureInvalid(signature_kind));
            }
            Ok(())
        }
        None => extend_on_cpu(&triples, signature_kind),
    }
}

// The reference body (verifier.rs:221-233), a private function next to `impl SingleVerifier`.
fn extend_on_cpu(triples: &[Triple], signature_kind: SignatureKind) -> Result<()> {
    for triple in triples {
        let signature = Signature::try_from(triple.signature_bytes)?;
        ensure!(signature.verify(triple.message, triple.public_key()), Error::SignatureInvalid(signature_kind));
    }
    Ok(())
}

// ---------------------------------------------------------------- MultiVerifier::verify_aggregate_indexed
// (f1, r06; in `impl Verifier for MultiVerifier` next to verify_aggregate, verifier.rs:275-287)

#[inline]
fn verify_aggregate_indexed<'keys>(
    &mut self,
    message: H256,
    signature_bytes: SignatureBytes,
    validator_indices: &[ValidatorIndex],
    public_keys: impl IntoIterator<IntoIter = impl Iterator<Item = &'keys PublicKey> + Send>,
    signature_kind: SignatureKind,
) -> Result<()> {
    let mut triple = Triple::default();
    triple.verify_aggregate_indexed(message, signature_bytes, validator_indices, public_keys, signature_kind)?;
    self.triples.push(triple);
    Ok(())
}

// ---------------------------------------------------------------- MultiVerifier::finish

#[inline]
fn finish(&self) -> Result<()> {
    if self.triples.is_empty() {
        return Ok(());
    }

    let (messages, signature_bytes, points, offsets) = engine_sets(&self.triples);

    let mut rng = rand::thread_rng();
    let randoms = core::iter::repeat_with(|| rng.gen::<NonZeroU64>().get())
        .take(messages.len())
        .collect_vec();

    // block verification (transition_functions/src/deneb/state_transition.rs:69-71) is the
    // latency-critical caller; gossip batches go through the normal class
    let class = if self.has_option(VerifierOption::BlockImport) {
        bls::gpu::CallClass::BlockImport
    } else {
        bls::gpu::CallClass::Normal
    };

    // f1: registry indices (4 bytes per key, resolved on the device) when every set has them and
    // the registry mirrors those validators; else the key points
    let verdict = match engine_indices(&self.triples) {
        Some((indices, index_offsets)) => bls::gpu::multi_verify_compressed_indexed(
            &messages,
            &signature_bytes,
            &indices,
            &index_offsets,
            &randoms,
            class,
        ),
        None => bls::gpu::multi_verify_compressed(&messages, &signature_bytes, &points, &offsets, &randoms, class),
    };

    match verdict {
        Some(verdict) => {
            let verdict = verdict.map_err(bls::Error::DecompressionFailed)?;
            ensure!(verdict, Error::SignatureInvalid(SignatureKind::Multi));
            Ok(())
        }
        None => self.finish_on_cpu(),
    }
}

// The reference body (verifier.rs:301-323), added to `impl MultiVerifier` as a private method;
// deferred sums are formed by blst here (Triple::public_key).
fn finish_on_cpu(&self) -> Result<()> {
    let messages = self.triples.iter().map(|triple| triple.message.as_bytes());

    let signatures = self
        .triples
        .par_iter()
        .map(|triple| triple.signature_bytes.try_into())
        .collect::<Result<Vec<_>, _>>()?;

    let public_keys = self.triples.par_iter().map(Triple::public_key).collect::<Vec<_>>();

    ensure!(
        Signature::multi_verify(messages, signatures.iter(), public_keys.iter()),
        Error::SignatureInvalid(SignatureKind::Multi),
    );

    Ok(())
}

// ---------------------------------------------------------------- MultiVerifier::verify_each (f2)
// A new public method of `impl MultiVerifier` (r06): which collected sets verify ON THEIR OWN, in
// ONE engine submission (`gbls_verify_batch_compressed`: every set its own check with
// `Signature::verify` / `fast_aggregate_verify` semantics -- the verdict the singular path would
// reach -- coalesced with concurrent callers; from 2048 sets the engine groups 8 checks per
// final exponentiation and re-checks failed groups' members on the device).  A set whose
// signature does not decode is `false`.  For a caller whose batch failed, so that only the
// failing items take its singular path (rust/bls_patch/attestation_verifier.rs, replacing the
// per-item loops of p2p/src/attestation_verifier.rs:231-238,379-384).
// `None`: no engine verdict (absent engine or engine error) -- the caller keeps the reference's
// per-item fallback.

#[must_use]
pub fn verify_each(&self) -> Option<Vec<bool>> {
    if self.triples.is_empty() {
        return Some(Vec::new());
    }
    let (messages, signature_bytes, points, offsets) = engine_sets(&self.triples);
    bls::gpu::verify_batch_compressed(&messages, &signature_bytes, &points, &offsets)
        .map(|outcomes| outcomes.into_iter().map(|outcome| matches!(outcome, Ok(true))).collect())
}
