"""Python mirror of the reference ``bls`` crate (/root/reference/bls/src), backed by the
MI355X engine through the C ABI (include/grandine_bls_gpu.h).

Names, argument meaning and error behaviour follow the crate:

* ``PublicKey``  -- bls/src/public_key.rs (try_from validates; aggregate / aggregate_nonempty)
* ``Signature``  -- bls/src/signature.rs (verify, fast_aggregate_verify, multi_verify, aggregate)
* ``SecretKey``  -- bls/src/secret_key.rs (try_from, to_public_key, sign)
* ``CachedPublicKey`` -- bls/src/cached_public_key.rs (decompress once, cache)
* ``Error.DecompressionFailed(BLST_ERROR)`` / ``Error.NoPublicKeysToAggregate`` -- bls/src/error.rs

Points are held as the engine's 96/192-byte affine encodings (blst_p1_affine /
blst_p2_affine layout, Montgomery limbs, all-zero = infinity).
"""

from __future__ import annotations

import ctypes
import secrets
from typing import Iterable, List, Sequence

from . import _lib as G

DOMAIN_SEPARATION_TAG = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"  # bls/src/consts.rs:1
CURVE_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class Error(Exception):
    """bls::Error (bls/src/error.rs:7-14)."""


class DecompressionFailed(Error):
    def __init__(self, code: int):
        super().__init__(f"decompression failed: {code}")
        self.code = code


class NoPublicKeysToAggregate(Error):
    def __init__(self):
        super().__init__("no public keys to aggregate")


Error.DecompressionFailed = DecompressionFailed
Error.NoPublicKeysToAggregate = NoPublicKeysToAggregate


# ----------------------------------------------------------------------------- bytes types
class PublicKeyBytes(bytes):
    SIZE = 48

    def __new__(cls, data: bytes = bytes(48)):
        if len(data) != 48:
            raise ValueError("PublicKeyBytes must be 48 bytes")
        return super().__new__(cls, data)


class SignatureBytes(bytes):
    SIZE = 96

    def __new__(cls, data: bytes = bytes(96)):
        if len(data) != 96:
            raise ValueError("SignatureBytes must be 96 bytes")
        return super().__new__(cls, data)

    @classmethod
    def empty(cls) -> "SignatureBytes":
        """bls/src/signature_bytes.rs:46-56: 0xc0 followed by zeros."""
        return cls(b"\xc0" + bytes(95))

    def is_empty(self) -> bool:
        return self == SignatureBytes.empty()


class SecretKeyBytes(bytes):
    def __new__(cls, data: bytes):
        if len(data) != 32:
            raise ValueError("SecretKeyBytes must be 32 bytes")
        return super().__new__(cls, data)


# ----------------------------------------------------------------------------- batched helpers
def decompress_public_keys(items: Sequence[bytes], validate: bool = True):
    """Batched PublicKey::try_from: returns [(status, affine96 or None)]."""
    n = len(items)
    if n == 0:
        return []
    L = G.lib()
    inb = G.buf(b"".join(bytes(x) for x in items))
    out = ctypes.create_string_buffer(96 * n)
    st = G.i32_array(n)
    G.check(L.gbls_g1_decompress(inb, n, int(validate), out, st), "gbls_g1_decompress")
    raw = out.raw
    return [(st[i], raw[96 * i:96 * (i + 1)] if st[i] == G.SUCCESS else None) for i in range(n)]


def decompress_signatures(items: Sequence[bytes]):
    """Batched Signature::try_from (on-curve check only): [(status, affine192 or None)]."""
    n = len(items)
    if n == 0:
        return []
    L = G.lib()
    inb = G.buf(b"".join(bytes(x) for x in items))
    out = ctypes.create_string_buffer(192 * n)
    st = G.i32_array(n)
    G.check(L.gbls_g2_decompress(inb, n, out, st), "gbls_g2_decompress")
    raw = out.raw
    return [(st[i], raw[192 * i:192 * (i + 1)] if st[i] == G.SUCCESS else None) for i in range(n)]


# ----------------------------------------------------------------------------- PublicKey
class PublicKey:
    """bls::PublicKey (bls/src/public_key.rs)."""

    __slots__ = ("raw",)

    def __init__(self, raw: bytes = bytes(96)):
        self.raw = bytes(raw)

    @classmethod
    def default(cls) -> "PublicKey":  # blst default = all-zero = infinity
        return cls()

    @classmethod
    def try_from(cls, data: bytes) -> "PublicKey":
        """public_key.rs:16-31: uncompress, then validate (rejects infinity / non-G1)."""
        st, raw = decompress_public_keys([PublicKeyBytes(bytes(data))], validate=True)[0]
        if st != G.SUCCESS:
            raise DecompressionFailed(st)
        return cls(raw)

    def to_bytes(self) -> PublicKeyBytes:
        L = G.lib()
        out = ctypes.create_string_buffer(48)
        G.check(L.gbls_g1_compress(G.buf(self.raw), 1, out), "gbls_g1_compress")
        return PublicKeyBytes(out.raw)

    def is_infinity(self) -> bool:
        return not any(self.raw)

    def aggregate(self, other: "PublicKey") -> "PublicKey":
        return PublicKey.aggregate_nonempty([self, other])

    def aggregate_in_place(self, other: "PublicKey") -> None:
        self.raw = self.aggregate(other).raw

    @staticmethod
    def aggregate_nonempty(public_keys: Iterable["PublicKey"]) -> "PublicKey":
        """public_key.rs:34-40 (eth_aggregate_pubkeys)."""
        keys = list(public_keys)
        if not keys:
            raise NoPublicKeysToAggregate()
        L = G.lib()
        out = ctypes.create_string_buffer(96)
        rc = L.gbls_g1_aggregate(G.buf(b"".join(k.raw for k in keys)), len(keys), out)
        if rc != G.SUCCESS:
            raise G.EngineUnavailable(f"gbls_g1_aggregate rc={rc}")
        return PublicKey(out.raw)

    def __eq__(self, other):
        return isinstance(other, PublicKey) and self.raw == other.raw

    def __hash__(self):
        return hash(self.raw)


AggregatePublicKey = PublicKey


class CachedPublicKey:
    """bls::CachedPublicKey: bytes + a lazily decompressed key (cached_public_key.rs:11-108)."""

    def __init__(self, data: bytes, decompressed: PublicKey = None):
        self.bytes = PublicKeyBytes(bytes(data))
        self._pk = decompressed

    def decompress(self) -> PublicKey:
        if self._pk is None:
            self._pk = PublicKey.try_from(self.bytes)
        return self._pk


# ----------------------------------------------------------------------------- Signature
class Signature:
    """bls::Signature (bls/src/signature.rs)."""

    __slots__ = ("raw",)

    def __init__(self, raw: bytes = bytes(192)):
        self.raw = bytes(raw)

    @classmethod
    def default(cls) -> "Signature":  # signature.rs:20-27
        return cls.try_from(SignatureBytes.empty())

    @classmethod
    def try_from(cls, data: bytes) -> "Signature":
        st, raw = decompress_signatures([SignatureBytes(bytes(data))])[0]
        if st != G.SUCCESS:
            raise DecompressionFailed(st)
        return cls(raw)

    def to_bytes(self) -> SignatureBytes:
        L = G.lib()
        out = ctypes.create_string_buffer(96)
        G.check(L.gbls_g2_compress(G.buf(self.raw), 1, out), "gbls_g2_compress")
        return SignatureBytes(out.raw)

    def verify(self, message: bytes, public_key: PublicKey) -> bool:
        """signature.rs:47-60."""
        L = G.lib()
        m = bytes(message)
        return L.gbls_verify(G.buf(self.raw), G.buf(m), len(m), G.buf(public_key.raw)) == G.SUCCESS

    def aggregate(self, other: "Signature") -> "Signature":
        L = G.lib()
        out = ctypes.create_string_buffer(192)
        G.check(L.gbls_g2_aggregate(G.buf(self.raw + other.raw), 2, out), "gbls_g2_aggregate")
        return Signature(out.raw)

    def aggregate_in_place(self, other: "Signature") -> None:
        self.raw = self.aggregate(other).raw

    def fast_aggregate_verify(self, message: bytes, public_keys: Iterable[PublicKey]) -> bool:
        """signature.rs:77-93."""
        keys = list(public_keys)
        L = G.lib()
        m = bytes(message)
        return L.gbls_fast_aggregate_verify(G.buf(self.raw), G.buf(m), len(m),
                                            G.buf(b"".join(k.raw for k in keys)), len(keys)) == G.SUCCESS

    @staticmethod
    def multi_verify(messages: Iterable[bytes], signatures: Iterable["Signature"],
                     public_keys: Iterable[PublicKey], randoms: Sequence[int] = None) -> bool:
        """signature.rs:95-129: random nonzero 64-bit scalars (ThreadRng -> secrets)."""
        msgs = [bytes(m) for m in messages]
        sigs = list(signatures)
        pks = list(public_keys)
        n = len(sigs)
        if n == 0 or len(msgs) != n or len(pks) != n:
            return False
        if any(len(m) != 32 for m in msgs):
            # the engine's batch path takes 32-byte signing roots (H256), as MultiVerifier does
            raise ValueError("multi_verify messages must be 32-byte signing roots")
        if randoms is None:
            randoms = [secrets.randbits(64) or 1 for _ in range(n)]
        L = G.lib()
        return L.gbls_multi_verify(G.buf(b"".join(msgs)), G.buf(b"".join(s.raw for s in sigs)),
                                   G.buf(b"".join(p.raw for p in pks)), G.u64_array(randoms), n) == G.SUCCESS

    @staticmethod
    def multi_verify_compressed(messages: Iterable[bytes], signature_bytes: Iterable[bytes],
                                public_keys: Iterable, randoms: Sequence[int] = None,
                                call_flags: int = 0) -> int:
        """MultiVerifier::finish's decompress + multi_verify (verifier.rs:301-323) as one device
        submission (gbls_multi_verify_compressed_ex): 0 = valid, 5 = VERIFY_FAIL, otherwise the
        first signature's decompression status (finish's Err(DecompressionFailed)).  Each set's
        key is a PublicKey or a list of them, summed on the device inside the same submission
        (a deferred Triple::verify_aggregate, verifier.rs:387-405)."""
        msgs = [bytes(m) for m in messages]
        sigs = [bytes(s) for s in signature_bytes]
        keys = [list(k) if isinstance(k, (list, tuple)) else [k] for k in public_keys]
        n = len(sigs)
        if n == 0 or len(msgs) != n or len(keys) != n:
            return G.VERIFY_FAIL
        if any(len(m) != 32 for m in msgs) or any(len(s) != 96 for s in sigs):
            raise ValueError("messages must be 32-byte signing roots and signatures 96 bytes")
        if randoms is None:
            randoms = [secrets.randbits(64) or 1 for _ in range(n)]
        off = [0]
        for k in keys:
            off.append(off[-1] + len(k))
        L = G.lib()
        st = G.i32_array(n)
        return L.gbls_multi_verify_compressed_ex(
            G.buf(b"".join(msgs)), G.buf(b"".join(sigs)), G.buf(b"".join(p.raw for k in keys for p in k)),
            None, G.u32_array(off), G.u64_array(randoms), n, st, call_flags)

    @staticmethod
    def multi_verify_compressed_indexed(messages: Iterable[bytes], signature_bytes: Iterable[bytes],
                                        validator_indices: Iterable[Sequence[int]], randoms: Sequence[int] = None,
                                        call_flags: int = 0) -> int:
        """multi_verify_compressed with each set's keys named by REGISTRY INDICES (f1: the engine
        gathers and sums the registry's keys on the device; 4 bytes per key instead of 96).
        Returns as multi_verify_compressed; an index past the registry fails its set."""
        msgs = [bytes(m) for m in messages]
        sigs = [bytes(s) for s in signature_bytes]
        idx = [list(v) for v in validator_indices]
        n = len(sigs)
        if n == 0 or len(msgs) != n or len(idx) != n:
            return G.VERIFY_FAIL
        if any(len(m) != 32 for m in msgs) or any(len(s) != 96 for s in sigs):
            raise ValueError("messages must be 32-byte signing roots and signatures 96 bytes")
        if randoms is None:
            randoms = [secrets.randbits(64) or 1 for _ in range(n)]
        off = [0]
        for v in idx:
            off.append(off[-1] + len(v))
        flat = [i for v in idx for i in v]
        L = G.lib()
        st = G.i32_array(n)
        return L.gbls_multi_verify_compressed_ex(
            G.buf(b"".join(msgs)), G.buf(b"".join(sigs)), None, G.u32_array(flat or [0]), G.u32_array(off),
            G.u64_array(randoms), n, st, call_flags)

    @staticmethod
    def verify_batch_compressed(messages: Iterable[bytes], signature_bytes: Iterable[bytes],
                                public_keys: Iterable) -> List:
        """SingleVerifier::extend's try_from + verify per triple (verifier.rs:215-236) as ONE
        coalesced device submission (gbls_verify_batch_compressed).  Per check: a decompression
        status (0 = decoded, else its BLST_ERROR) and whether it verifies; keys as in
        multi_verify_compressed (a list = fast_aggregate_verify over it)."""
        msgs = [bytes(m) for m in messages]
        sigs = [bytes(s) for s in signature_bytes]
        keys = [list(k) if isinstance(k, (list, tuple)) else [k] for k in public_keys]
        n = len(sigs)
        if len(msgs) != n or len(keys) != n:
            raise ValueError("one message and one key set per signature")
        if n == 0:
            return []
        if any(len(m) != 32 for m in msgs) or any(len(s) != 96 for s in sigs):
            raise ValueError("messages must be 32-byte signing roots and signatures 96 bytes")
        off = [0]
        for k in keys:
            off.append(off[-1] + len(k))
        L = G.lib()
        st, v = G.i32_array(n), G.i32_array(n)
        G.check(L.gbls_verify_batch_compressed(
            G.buf(b"".join(msgs)), G.buf(b"".join(sigs)), G.buf(b"".join(p.raw for k in keys for p in k) or bytes(96)),
            G.u32_array(off), n, st, v), "gbls_verify_batch_compressed")
        return [(st[i], v[i] == G.SUCCESS) for i in range(n)]

    def __eq__(self, other):
        return isinstance(other, Signature) and self.raw == other.raw

    def __hash__(self):
        return hash(self.raw)


AggregateSignature = Signature


# ----------------------------------------------------------------------------- SecretKey
class SecretKey:
    """bls::SecretKey (bls/src/secret_key.rs): 32-byte big-endian scalar, 0 < sk < r."""

    __slots__ = ("_b",)

    def __init__(self, b: bytes):
        self._b = bytes(b)

    @classmethod
    def try_from(cls, data: bytes) -> "SecretKey":
        data = bytes(data)
        k = int.from_bytes(data, "big") if len(data) == 32 else 0
        if len(data) != 32 or k == 0 or k >= CURVE_ORDER:
            raise DecompressionFailed(G.BAD_ENCODING)
        return cls(data)

    def to_bytes(self) -> SecretKeyBytes:
        return SecretKeyBytes(self._b)

    def to_public_key(self) -> PublicKey:
        L = G.lib()
        out = ctypes.create_string_buffer(96)
        G.check(L.gbls_sk_to_pk(G.buf(self._b), 1, out), "gbls_sk_to_pk")
        return PublicKey(out.raw)

    def sign(self, message: bytes) -> Signature:
        L = G.lib()
        m = bytes(message)
        out = ctypes.create_string_buffer(192)
        G.check(L.gbls_sign(G.buf(self._b), G.buf(m), G.u32_array([0, len(m)]), 1, out), "gbls_sign")
        return Signature(out.raw)

    def __eq__(self, other):
        return isinstance(other, SecretKey) and self._b == other._b

    def __repr__(self):
        return "SecretKey([REDACTED])"


def sign_batch(secret_keys: Sequence[bytes], messages: Sequence[bytes]) -> List[Signature]:
    """Batched SecretKey::sign on the device (fixture / workload generation)."""
    n = len(secret_keys)
    L = G.lib()
    msgs = [bytes(m) for m in messages]
    off = [0]
    for m in msgs:
        off.append(off[-1] + len(m))
    out = ctypes.create_string_buffer(192 * max(n, 1))
    G.check(L.gbls_sign(G.buf(b"".join(secret_keys)), G.buf(b"".join(msgs)), G.u32_array(off), n, out),
            "gbls_sign")
    return [Signature(out.raw[192 * i:192 * (i + 1)]) for i in range(n)]


def public_keys_batch(secret_keys: Sequence[bytes]) -> List[PublicKey]:
    n = len(secret_keys)
    L = G.lib()
    out = ctypes.create_string_buffer(96 * max(n, 1))
    G.check(L.gbls_sk_to_pk(G.buf(b"".join(secret_keys)), n, out), "gbls_sk_to_pk")
    return [PublicKey(out.raw[96 * i:96 * (i + 1)]) for i in range(n)]


class Registry:
    """Mirror of ``bls::gpu::registry`` (rust/bls_patch/gpu.rs, f1): the engine's device-resident
    copy of a FINALIZED validator list (indices name the same key on every fork only up to the
    finalized state).  ``mirror_finalized`` loads the new tail of the list with one
    gbls_registry_set; ``covers`` says whether a batch may name registry slots instead of key
    points."""

    _mirrored = 0

    @classmethod
    def mirror_finalized(cls, keys: Sequence[bytes]) -> int:
        n = len(keys) - cls._mirrored
        if n <= 0:
            return cls._mirrored
        tail = b"".join(bytes(k) for k in keys[cls._mirrored:])
        L = G.lib()
        st = G.i32_array(n)
        G.check(L.gbls_registry_set(cls._mirrored, G.buf(tail), n, st), "gbls_registry_set")
        cls._mirrored = len(keys)
        return cls._mirrored

    @classmethod
    def mirrored(cls) -> int:
        return cls._mirrored

    @classmethod
    def covers(cls, indices: Iterable[int]) -> bool:
        return all(0 <= int(i) < cls._mirrored for i in indices)

    @classmethod
    def forget(cls) -> None:
        """Tests: the process's engine registry was overwritten by someone else."""
        cls._mirrored = 0
