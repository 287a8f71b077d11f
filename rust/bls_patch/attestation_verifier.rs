// Replacement bodies for the two gossip batch tasks of p2p/src/attestation_verifier.rs (f2,
// r06).  No unsafe code (p2p keeps the workspace's `unsafe_code = 'forbid'`).
//
// The reference verifies a gossip batch (<= MAX_BATCH_SIZE = 64 items, attestation_verifier.rs:37)
// with one MultiVerifier; when that batch fails it re-verifies EVERY item on its singular path
// (`process_singular_attestation` / `process_singular_aggregate`, attestation_verifier.rs:231-238,
// 379-384), i.e. up to 64 full validations with their own blst checks for one bad signature.
// Here the failed batch's sets go to the engine once more, as independent checks in ONE
// submission (`MultiVerifier::verify_each`, rust/bls_patch/verifier.rs); only the items with a
// failing set take the singular path (which reports their error exactly as before), and the
// others keep the results their batch already computed.  Without an engine verdict (no device,
// engine error) the bodies run the reference's loops.
//
// The triples are built IN ITEM ORDER here (the batch path's `attestation_batch_triples` uses
// `par_bridge`, whose `collect` does not keep order): a slice's `par_iter().map().collect()`
// keeps it.  An item whose sets cannot be built counts as failing (the singular path says why).
//
// Needs in the file's imports: `rayon::iter::IntoParallelRefIterator as _` and
// `helper_functions::verifier::Verifier as _` (already imported for the batch path).

// ---- VerifyAttestationBatchTask::process_attestation_batch, the `Err` arm (reference :379-384)

            Err(error) => {
                warn!("signature verification for gossip attestation batch failed: {error}");

                match self.failing_attestations(&accepted_attestations_wo, &snapshot.head_state()) {
                    Some(failing) => {
                        let mut passed = Vec::with_capacity(accepted.len());
                        for ((attestation_wo, result), failed) in
                            accepted_attestations_wo.into_iter().zip(accepted).zip(failing)
                        {
                            if failed {
                                self.process_singular_attestation(attestation_wo);
                            } else {
                                passed.push(result);
                            }
                        }
                        self.send_results_to_fork_choice(passed);
                    }
                    None => {
                        for attestation_wo in accepted_attestations_wo {
                            self.process_singular_attestation(attestation_wo);
                        }
                    }
                }
            }

// ---- a new method of `impl<P: Preset> VerifyAttestationBatchTask<P>`

    /// Per attestation: `true` when its signature set does not verify on its own (or cannot be
    /// built).  One engine submission; `None` without an engine verdict.
    fn failing_attestations(
        &self,
        attestations_wo: &[AttestationWithOrigin<P>],
        state: &BeaconState<P>,
    ) -> Option<Vec<bool>> {
        let config = self.controller.chain_config().as_ref();

        let built = attestations_wo
            .par_iter()
            .map(|attestation_wo| {
                let indexed_attestation =
                    accessors::get_indexed_attestation(state, attestation_wo.attestation.as_ref()).ok()?;
                let mut triple = Triple::default();
                predicates::validate_constructed_indexed_attestation(
                    config,
                    state,
                    &indexed_attestation,
                    &mut triple,
                )
                .ok()?;
                Some(vec![triple])
            })
            .collect::<Vec<_>>();

        failing_items(built)
    }

// ---- VerifyAggregateBatchTask::process_aggregate_batch, the `Err` arm (reference :231-238)

            Err(error) => {
                warn!(
                    "signature verification for gossip aggregate and proof batch failed: {error}",
                );

                match self.failing_aggregates(&accepted_aggregates_wo, &snapshot.head_state()) {
                    Some(failing) => {
                        let mut passed = Vec::with_capacity(accepted.len());
                        for ((aggregate_wo, result), failed) in
                            accepted_aggregates_wo.into_iter().zip(accepted).zip(failing)
                        {
                            if failed {
                                self.process_singular_aggregate(aggregate_wo);
                            } else {
                                passed.push(result);
                            }
                        }
                        self.send_results_to_fork_choice(passed);
                    }
                    None => {
                        for aggregate_wo in accepted_aggregates_wo {
                            self.process_singular_aggregate(aggregate_wo);
                        }
                    }
                }
            }

// ---- a new method of `impl<P: Preset> VerifyAggregateBatchTask<P>`

    /// Per aggregate: `true` when one of its three sets (selection proof, aggregate-and-proof
    /// signature, the attestation: the sets of `verify_aggregate_batch_signatures`, reference
    /// :262-305) does not verify on its own, or they cannot be built.  One engine submission;
    /// `None` without an engine verdict.
    fn failing_aggregates(
        &self,
        aggregates_wo: &[AggregateWithOrigin<P>],
        state: &BeaconState<P>,
    ) -> Option<Vec<bool>> {
        let config = self.controller.chain_config().as_ref();

        let built = aggregates_wo
            .par_iter()
            .map(|aggregate_wo| {
                let SignedAggregateAndProof {
                    ref message,
                    signature,
                } = *aggregate_wo.aggregate;

                let AggregateAndProof {
                    aggregator_index,
                    ref aggregate,
                    selection_proof,
                } = *message;

                let public_key = *accessors::public_key(state, aggregator_index)
                    .ok()?
                    .decompress()
                    .ok()?;

                let indexed_attestation = accessors::get_indexed_attestation(state, aggregate).ok()?;
                let mut attestation_triple = Triple::default();
                predicates::validate_constructed_indexed_attestation(
                    config,
                    state,
                    &indexed_attestation,
                    &mut attestation_triple,
                )
                .ok()?;

                Some(vec![
                    Triple::new(
                        aggregate.data.slot.signing_root(config, state),
                        selection_proof,
                        public_key,
                    ),
                    Triple::new(message.signing_root(config, state), signature, public_key),
                    attestation_triple,
                ])
            })
            .collect::<Vec<_>>();

        failing_items(built)
    }

// ---- a private function of the module

/// Items' sets (in item order; `None` = not buildable) -> per item, whether any of its sets fails
/// on its own (one `MultiVerifier::verify_each` submission), or `None` without an engine verdict.
fn failing_items(built: Vec<Option<Vec<Triple>>>) -> Option<Vec<bool>> {
    let mut owners = Vec::new();
    let mut triples = Vec::new();
    let mut failing = Vec::with_capacity(built.len());

    for (item, sets) in built.into_iter().enumerate() {
        failing.push(sets.is_none());
        for triple in sets.into_iter().flatten() {
            owners.push(item);
            triples.push(triple);
        }
    }

    let mut verifier = MultiVerifier::default();
    verifier.extend(triples, SignatureKind::Multi).ok()?;

    for (item, verified) in owners.into_iter().zip(verifier.verify_each()?) {
        if !verified {
            failing[item] = true;
        }
    }

    Some(failing)
}
