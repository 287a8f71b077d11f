"""Python mirror of ``helper_functions::verifier`` (/root/reference/helper_functions/src/verifier.rs).

The pluggable batching layer in front of the signature hot path:

* ``Verifier``        -- trait, verifier.rs:16-69 (``IS_NULL``, reserve, verify_singular,
                         verify_aggregate, verify_aggregate_allowing_empty, extend, finish,
                         has_option)
* ``NullVerifier``    -- verifier.rs:121-169 (skips cryptography)
* ``SingleVerifier``  -- verifier.rs:171-244 (verifies each triple immediately)
* ``MultiVerifier``   -- verifier.rs:246-347 (collects triples; ``finish`` runs one
                         random-linear-combination batch on the MI355X engine)
* ``Triple``          -- verifier.rs:349-429 (``verify_aggregate`` DEFERS the key sum: the key
                         list is summed on the device by the submission that verifies it)
* ``VerifierOption``  -- verifier.rs:431-436

Errors follow helper_functions/src/error.rs: ``SignatureInvalid(kind)``; decompression
failures surface as ``bls.DecompressionFailed``.
"""

from __future__ import annotations

import enum
from typing import Iterable, List, Optional

from . import bls


class SignatureKind(enum.Enum):  # helper_functions/src/error.rs:40-74 (subset used here)
    AggregateAndProof = "aggregate and proof"
    Attestation = "attestation"
    Block = "block"
    BlsToExecutionChange = "BLS to execution change"
    ContributionAndProof = "contribution and proof"
    Deposit = "deposit"
    Multi = "multiple signatures"
    Randao = "RANDAO reveal"
    SelectionProof = "selection proof"
    SyncCommitteeMessage = "sync committee message"
    SyncCommitteeContribution = "sync committee contribution"
    VoluntaryExit = "voluntary exit"


class SignatureInvalid(Exception):
    def __init__(self, kind: SignatureKind):
        super().__init__(f"{kind.value} signature is invalid")
        self.kind = kind


class VerifierOption(enum.Enum):
    SkipBlockBaseSignatures = 0
    SkipBlockSyncAggregateSignature = 1
    SkipRandaoVerification = 2
    BlockImport = 3  # the drop-in's one new option: the engine's block-import class (f3)


class Triple:
    """(message: H256, signature_bytes: SignatureBytes, public_key: PublicKey), or, after
    ``verify_aggregate``, the message, signature and the KEY LIST whose sum is the key."""

    IS_NULL = False
    __slots__ = ("message", "signature_bytes", "_key", "deferred", "indices")

    def __init__(self, message: bytes = bytes(32), signature_bytes: bytes = None,
                 public_key: "bls.PublicKey" = None):
        self.message = bytes(message)
        self.signature_bytes = bls.SignatureBytes(signature_bytes if signature_bytes is not None else bytes(96))
        self._key = public_key if public_key is not None else bls.PublicKey.default()
        self.deferred = None  # list of keys once verify_aggregate has run
        self.indices = None   # their validator indices (verify_aggregate_indexed, f1)

    def verify_aggregate(self, message, signature_bytes, public_keys, signature_kind=None):
        """verifier.rs:387-405 without the reduce: the keys are kept and summed on the device by
        the submission that verifies this triple (MultiVerifier.finish /
        SingleVerifier.extend)."""
        self.message = bytes(message)
        self.signature_bytes = bls.SignatureBytes(bytes(signature_bytes))
        self._key = bls.PublicKey.default()
        self.deferred = list(public_keys)

    def verify_aggregate_indexed(self, message, signature_bytes, validator_indices, public_keys,
                                 signature_kind=None):
        """f1 (r06): verify_aggregate that also keeps the keys' validator indices
        (rust/bls_patch/verifier.rs), so MultiVerifier.finish can name registry slots."""
        self.verify_aggregate(message, signature_bytes, public_keys, signature_kind)
        self.indices = [int(i) for i in validator_indices]

    @property
    def public_key(self) -> "bls.PublicKey":
        """The set's key: the reference's reduce(AggregatePublicKey::default, aggregate) over a
        deferred list (one engine sum), or the resolved key."""
        if self.deferred is None:
            return self._key
        if not self.deferred:
            return bls.PublicKey.default()  # identity of the reduce
        return bls.PublicKey.aggregate_nonempty(self.deferred)

    def keys(self):
        """The engine's key operand: the deferred list, or [the key]."""
        return list(self.deferred) if self.deferred is not None else [self._key]


class Verifier:
    IS_NULL = False

    def reserve(self, additional: int) -> None:
        pass

    def verify_singular(self, message, signature_bytes, cached_public_key, signature_kind):
        raise NotImplementedError

    def verify_aggregate(self, message, signature_bytes, public_keys, signature_kind):
        raise NotImplementedError

    def verify_aggregate_allowing_empty(self, message, signature_bytes, public_keys, signature_kind):
        """verifier.rs:41-58 (eth_fast_aggregate_verify's emptiness rule)."""
        keys = list(public_keys)
        if bls.SignatureBytes(bytes(signature_bytes)).is_empty():
            if keys:
                raise SignatureInvalid(signature_kind)
            return None
        return self.verify_aggregate(message, signature_bytes, keys, signature_kind)

    def extend(self, triples: Iterable[Triple], signature_kind):
        raise NotImplementedError

    def finish(self) -> None:
        raise NotImplementedError

    def has_option(self, option: VerifierOption) -> bool:
        return False


class NullVerifier(Verifier):
    IS_NULL = True

    def verify_singular(self, message, signature_bytes, cached_public_key, signature_kind):
        return None

    def verify_aggregate(self, message, signature_bytes, public_keys, signature_kind):
        return None

    def extend(self, triples, signature_kind):
        return None

    def finish(self):
        return None


class SingleVerifier(Verifier):
    def verify_singular(self, message, signature_bytes, cached_public_key, signature_kind):
        public_key = cached_public_key.decompress()
        self.extend([Triple(message, signature_bytes, public_key)], signature_kind)

    def verify_aggregate(self, message, signature_bytes, public_keys, signature_kind):
        """verifier.rs:193-212: Signature::fast_aggregate_verify."""
        signature = bls.Signature.try_from(signature_bytes)
        if not signature.fast_aggregate_verify(message, list(public_keys)):
            raise SignatureInvalid(signature_kind)

    def extend(self, triples, signature_kind):
        """verifier.rs:215-236 as ONE coalesced device submission: every triple's decompression
        and check together, errors in the reference's order (the first triple whose signature
        does not decode -> DecompressionFailed, the first that does not verify ->
        SignatureInvalid)."""
        triples = list(triples)
        if not triples:
            return None
        outcomes = bls.Signature.verify_batch_compressed(
            [t.message for t in triples], [t.signature_bytes for t in triples], [t.keys() for t in triples])
        for status, ok in outcomes:
            if status != 0:
                raise bls.DecompressionFailed(status)
            if not ok:
                raise SignatureInvalid(signature_kind)
        return None

    def finish(self):
        return None


class MultiVerifier(Verifier):
    def __init__(self, options: Iterable[VerifierOption] = (), triples: Optional[List[Triple]] = None):
        self.triples: List[Triple] = list(triples or [])
        self.options = set(options)
        self.last_path = None  # "indices" or "points": the key form of the last finish (tests)

    @classmethod
    def from_triples(cls, triples: List[Triple]) -> "MultiVerifier":  # From<Vec<Triple>>
        return cls(triples=triples)

    def verify_singular(self, message, signature_bytes, cached_public_key, signature_kind):
        public_key = cached_public_key.decompress()
        self.triples.append(Triple(message, signature_bytes, public_key))

    def verify_aggregate(self, message, signature_bytes, public_keys, signature_kind):
        t = Triple()
        t.verify_aggregate(message, signature_bytes, public_keys, signature_kind)
        self.triples.append(t)

    def extend(self, triples, signature_kind):
        self.triples.extend(triples)

    def verify_aggregate_indexed(self, message, signature_bytes, validator_indices, public_keys, signature_kind):
        t = Triple()
        t.verify_aggregate_indexed(message, signature_bytes, validator_indices, public_keys, signature_kind)
        self.triples.append(t)

    def finish(self, randoms=None):
        """verifier.rs:301-323."""
        if not self.triples:
            return None
        # decompression (verifier.rs:309-313) and multi_verify in one device submission
        # key sums of deferred triples (Triple.verify_aggregate) on the device, same submission;
        # f1: registry indices instead of key points when every set has them and the engine's
        # registry mirrors those validators (bls.Registry)
        flags = 0x1 if VerifierOption.BlockImport in self.options else 0
        msgs = [t.message for t in self.triples]
        sigs = [t.signature_bytes for t in self.triples]
        if all(t.indices is not None and bls.Registry.covers(t.indices) for t in self.triples):
            self.last_path = "indices"
            rc = bls.Signature.multi_verify_compressed_indexed(msgs, sigs, [t.indices for t in self.triples],
                                                               randoms, flags)
        else:
            self.last_path = "points"
            rc = bls.Signature.multi_verify_compressed(msgs, sigs, [t.keys() for t in self.triples], randoms, flags)
        if rc not in (0, 5):
            raise bls.DecompressionFailed(rc)
        if rc != 0:
            raise SignatureInvalid(SignatureKind.Multi)
        return None

    def verify_each(self) -> List[bool]:
        """f2 (r06, a new method of the drop-in's MultiVerifier): which collected sets verify ON
        THEIR OWN, in ONE device submission (gbls_verify_batch_compressed: every set its own
        check with Signature::verify / fast_aggregate_verify semantics -- the verdict the
        singular path would reach).  A set whose signature does not decode is False.  For a
        caller whose batch failed, so that only the failing items take the singular path
        (split_failed_batch)."""
        if not self.triples:
            return []
        outcomes = bls.Signature.verify_batch_compressed(
            [t.message for t in self.triples], [t.signature_bytes for t in self.triples],
            [t.keys() for t in self.triples])
        return [status == 0 and ok for status, ok in outcomes]

    def has_option(self, option: VerifierOption) -> bool:
        return option in self.options


def split_failed_batch(items: List, item_triples: List[Optional[List[Triple]]]):
    """The drop-in's fallback after a failed gossip batch (rust/bls_patch/attestation_verifier.rs,
    replacing /root/reference/p2p/src/attestation_verifier.rs:231-238 and 379-384, where every
    item of the failed batch is re-verified one by one on the CPU).

    item_triples[k]: the signature sets of item k IN ORDER (an attestation has one; an aggregate
    three: selection proof, aggregate-and-proof signature, attestation), or None when they cannot
    be built (the singular path then reports why).  One submission (MultiVerifier.verify_each)
    decides every set; returns (passed, failing): the items whose sets all verify keep their batch
    results, only the failing ones go to the singular path."""
    if len(items) != len(item_triples):
        raise ValueError("one triple list per item")
    owner, triples = [], []
    for k, ts in enumerate(item_triples):
        for t in ts or []:
            owner.append(k)
            triples.append(t)
    verified = MultiVerifier(triples=triples).verify_each()
    bad = [ts is None for ts in item_triples]
    for k, ok in zip(owner, verified):
        if not ok:
            bad[k] = True
    passed = [it for it, b in zip(items, bad) if not b]
    failing = [it for it, b in zip(items, bad) if b]
    return passed, failing
