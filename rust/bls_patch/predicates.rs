// Replacement body for helper_functions/src/predicates.rs `validate_indexed_attestation`
// (reference predicates.rs:107-141), f1 (r06).  No unsafe code.
//
// The only change: the aggregate check hands the verifier the attestation's validator indices
// with the keys (`Verifier::verify_aggregate_indexed`, a provided method whose default is the
// reference's `verify_aggregate`; rust/bls_patch/verifier.rs).  `MultiVerifier` keeps them, so
// `finish` can name the engine's registry slots instead of shipping 96-byte key points when the
// registry mirrors those validators (bls::gpu::registry).  Every other verifier behaves as before:
// the keys are decompressed and checked exactly as in the reference (a key that does not
// decompress still fails the attestation here, before any verifier sees it).

fn validate_indexed_attestation<P: Preset>(
    config: &Config,
    state: &impl BeaconState<P>,
    indexed_attestation: &IndexedAttestation<P>,
    mut verifier: impl Verifier,
    validate_indices_sorted_and_unique: bool,
) -> Result<()> {
    let indices = &indexed_attestation.attesting_indices;

    ensure!(!indices.is_empty(), Error::AttestationHasNoAttestingIndices);

    if validate_indices_sorted_and_unique {
        // > Verify indices are sorted and unique
        ensure!(
            indices.iter().tuple_windows().all(|(a, b)| a < b),
            Error::AttestingIndicesNotSortedAndUnique,
        );
    }

    // > Verify aggregate signature
    let validator_indices = indices.iter().copied().collect_vec();

    itertools::process_results(
        validator_indices.iter().copied().map(|validator_index| {
            accessors::public_key(state, validator_index)?
                .decompress()
                .map_err(AnyhowError::new)
        }),
        |public_keys| {
            verifier.verify_aggregate_indexed(
                indexed_attestation.data.signing_root(config, state),
                indexed_attestation.signature,
                &validator_indices,
                public_keys,
                SignatureKind::Attestation,
            )
        },
    )?
}
