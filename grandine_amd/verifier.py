"""Python mirror of ``helper_functions::verifier`` (/root/reference/helper_functions/src/verifier.rs).

The pluggable batching layer in front of the signature hot path:

* ``Verifier``        -- trait, verifier.rs:16-69 (``IS_NULL``, reserve, verify_singular,
                         verify_aggregate, verify_aggregate_allowing_empty, extend, finish,
                         has_option)
* ``NullVerifier``    -- verifier.rs:121-169 (skips cryptography)
* ``SingleVerifier``  -- verifier.rs:171-244 (verifies each triple immediately)
* ``MultiVerifier``   -- verifier.rs:246-347 (collects triples; ``finish`` runs one
                         random-linear-combination batch on the MI355X engine)
* ``Triple``          -- verifier.rs:349-429 (``verify_aggregate`` aggregates the keys)
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


class Triple:
    """(message: H256, signature_bytes: SignatureBytes, public_key: PublicKey)."""

    IS_NULL = False
    __slots__ = ("message", "signature_bytes", "public_key")

    def __init__(self, message: bytes = bytes(32), signature_bytes: bytes = None,
                 public_key: "bls.PublicKey" = None):
        self.message = bytes(message)
        self.signature_bytes = bls.SignatureBytes(signature_bytes if signature_bytes is not None else bytes(96))
        self.public_key = public_key if public_key is not None else bls.PublicKey.default()

    def verify_aggregate(self, message, signature_bytes, public_keys, signature_kind=None):
        """verifier.rs:387-405: reduce(AggregatePublicKey::default, aggregate)."""
        keys = list(public_keys)
        if keys:
            pk = bls.PublicKey.aggregate_nonempty(keys)
        else:
            pk = bls.PublicKey.default()  # identity of the reduce
        self.message = bytes(message)
        self.signature_bytes = bls.SignatureBytes(bytes(signature_bytes))
        self.public_key = pk


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
        for t in triples:
            signature = bls.Signature.try_from(t.signature_bytes)
            if not signature.verify(t.message, t.public_key):
                raise SignatureInvalid(signature_kind)

    def finish(self):
        return None


class MultiVerifier(Verifier):
    def __init__(self, options: Iterable[VerifierOption] = (), triples: Optional[List[Triple]] = None):
        self.triples: List[Triple] = list(triples or [])
        self.options = set(options)

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

    def finish(self, randoms=None):
        """verifier.rs:301-323."""
        if not self.triples:
            return None
        # decompression (verifier.rs:309-313) and multi_verify in one device submission
        rc = bls.Signature.multi_verify_compressed([t.message for t in self.triples],
                                                   [t.signature_bytes for t in self.triples],
                                                   [t.public_key for t in self.triples], randoms)
        if rc not in (0, 5):
            raise bls.DecompressionFailed(rc)
        if rc != 0:
            raise SignatureInvalid(SignatureKind.Multi)
        return None

    def has_option(self, option: VerifierOption) -> bool:
        return option in self.options
