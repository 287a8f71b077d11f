// Replacement body of MultiVerifier::finish, helper_functions/src/verifier.rs:301-323.  No
// unsafe code (helper_functions keeps the workspace's `unsafe_code = 'forbid'`).
//
// The reference decompresses every signature on rayon workers (verifier.rs:309-313), then calls
// Signature::multi_verify.  Here the 96-byte signatures go to the device with the messages, keys
// and scalars in ONE submission: decompression runs on a side stream while hash_to_G2 runs, a
// signature that fails to decode fails the call with its BLST_ERROR (the reference's `?` on
// try_into), and block import asks for the engine's block-import priority class through one
// new option, added to the enum at verifier.rs:432-436:
//
//     pub enum VerifierOption { SkipBlockBaseSignatures, SkipBlockSyncAggregateSignature,
//                               SkipRandaoVerification, BlockImport }
//
// which the block paths pass when they build their verifier
// (p2p/src/block_verification_pool.rs:109, fork_choice_control/src/tasks.rs:101).
// Without an engine verdict (no device, engine error) the reference body runs unchanged.

#[inline]
fn finish(&self) -> Result<()> {
    if self.triples.is_empty() {
        return Ok(());
    }

    let messages = self
        .triples
        .iter()
        .map(|triple| triple.message.to_fixed_bytes())
        .collect_vec();
    let signature_bytes = self
        .triples
        .iter()
        .map(|triple| triple.signature_bytes.to_fixed_bytes())
        .collect_vec();
    let public_keys = self
        .triples
        .iter()
        .map(|triple| bls::gpu::public_key_point(&triple.public_key))
        .collect_vec();

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

    match bls::gpu::multi_verify_compressed(&messages, &signature_bytes, &public_keys, &randoms, class) {
        Some(verdict) => {
            let verdict = verdict.map_err(bls::Error::DecompressionFailed)?;
            ensure!(verdict, Error::SignatureInvalid(SignatureKind::Multi));
            Ok(())
        }
        None => self.finish_on_cpu(),
    }
}

// The reference body (verifier.rs:301-323), added to `impl MultiVerifier` as a private method.
fn finish_on_cpu(&self) -> Result<()> {
    let messages = self.triples.iter().map(|triple| triple.message.as_bytes());

    let signatures = self
        .triples
        .par_iter()
        .map(|triple| triple.signature_bytes.try_into())
        .collect::<Result<Vec<_>, _>>()?;

    let public_keys = self.triples.iter().map(|triple| &triple.public_key);

    ensure!(
        Signature::multi_verify(messages, signatures.iter(), public_keys),
        Error::SignatureInvalid(SignatureKind::Multi),
    );

    Ok(())
}
