"""Synthetic signed inputs for the benchmark configs and the at-size parity tests.

Plays the role of the reference's ``factory`` crate (/root/reference/factory/src/lib.rs:
219,487-582: fully signed blocks built from interop keys): every key, message and
signature is derived deterministically from a seed, and the expensive steps (sk -> pk,
hash-and-sign, compression) run on the engine itself, whose kernels the parity suite pins
to the oracle and to the reference's KATs.  Shapes follow SURVEY.md 8(d):

* C2 -- n single-pubkey sets, distinct 32-byte signing roots, nonzero u64 scalars;
* C3 -- m messages, one 512-key committee, sig = (sum sk) * H(m), a seeded 1 % invalid;
* C4 -- a registry, committees partitioning it (Triple::verify_aggregate), one message per
  committee, sig = (sum of the committee's sk) * H(m);
* C5 -- a large registry, 2^k sets with uniformly drawn key indices.
"""

from __future__ import annotations

import ctypes
import hashlib
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib as G

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def interop_sk(i: int) -> int:
    """interop/src/lib.rs:65-76: LE-int(SHA-256(LE64(i) || 0^24)) mod r."""
    h = hashlib.sha256(i.to_bytes(8, "little") + bytes(24)).digest()
    return int.from_bytes(h, "little") % R_ORDER


def seeded_sks(n: int, seed: bytes, start: int = 0) -> List[int]:
    """n nonzero secret keys sha256(seed || i) mod r."""
    out = []
    for i in range(start, start + n):
        k = int.from_bytes(hashlib.sha256(seed + b"/sk/%d" % i).digest(), "big") % R_ORDER
        out.append(k or 1)
    return out


def sk_bytes(sks: Sequence[int]) -> bytes:
    return b"".join(k.to_bytes(32, "big") for k in sks)


def messages(n: int, seed: bytes) -> bytes:
    """n distinct 32-byte signing roots, packed."""
    return b"".join(hashlib.sha256(seed + b"/m/%d" % i).digest() for i in range(n))


def rands(n: int, seed: int) -> List[int]:
    """xorshift64*: deterministic nonzero 64-bit scalars (signature.rs:106-115 draws them
    from ThreadRng)."""
    x = (seed * 0x9E3779B97F4A7C15 + 12345) & ((1 << 64) - 1) or 1
    out = []
    for _ in range(n):
        x ^= x >> 12
        x ^= (x << 25) & ((1 << 64) - 1)
        x ^= x >> 27
        out.append(((x * 0x2545F4914F6CDD1D) & ((1 << 64) - 1)) or 1)
    return out


# ----------------------------------------------------------------------------- engine helpers
CHUNK = 1 << 18


def public_keys(sks: Sequence[int]) -> bytes:
    """Affine (96-byte) public keys of sks, computed on the device."""
    L = G.lib()
    out = []
    for b in range(0, len(sks), CHUNK):
        part = sks[b:b + CHUNK]
        buf = ctypes.create_string_buffer(96 * len(part))
        G.check(L.gbls_sk_to_pk(sk_bytes(part), len(part), buf), "gbls_sk_to_pk")
        out.append(buf.raw)
    return b"".join(out)


def compress_g1(points96: bytes) -> bytes:
    L = G.lib()
    n = len(points96) // 96
    out = []
    for b in range(0, n, CHUNK):
        e = min(n, b + CHUNK)
        buf = ctypes.create_string_buffer(48 * (e - b))
        G.check(L.gbls_g1_compress(G.buf(points96[96 * b:96 * e]), e - b, buf), "gbls_g1_compress")
        out.append(buf.raw)
    return b"".join(out)


def sign(sks: Sequence[int], msgs: bytes, msg_len: int = 32) -> bytes:
    """Affine (192-byte) signatures sk_i * H(m_i) for packed fixed-length messages."""
    L = G.lib()
    n = len(sks)
    out = []
    for b in range(0, n, CHUNK):
        e = min(n, b + CHUNK)
        buf = ctypes.create_string_buffer(192 * (e - b))
        off = G.u32_array(range(0, msg_len * (e - b) + 1, msg_len))
        G.check(L.gbls_sign(sk_bytes(sks[b:e]), G.buf(msgs[msg_len * b:msg_len * e]), off, e - b, buf),
                "gbls_sign")
        out.append(buf.raw)
    return b"".join(out)


def registry(n_keys: int, seed: bytes = b"registry") -> Tuple[List[int], bytes]:
    """(secret keys, compressed 48-byte public keys) of a synthetic validator registry."""
    sks = seeded_sks(n_keys, seed)
    return sks, compress_g1(public_keys(sks))


def load_registry(compressed: bytes, first: int = 0) -> np.ndarray:
    """gbls_registry_set in chunks; returns the per-key statuses."""
    L = G.lib()
    n = len(compressed) // 48
    st = np.zeros(n, dtype=np.int32)
    for b in range(0, n, CHUNK):
        e = min(n, b + CHUNK)
        part = np.zeros(e - b, dtype=np.int32)
        G.check(L.gbls_registry_set(first + b, G.buf(compressed[48 * b:48 * e]), e - b,
                                    part.ctypes.data_as(ctypes.c_void_p)), "gbls_registry_set")
        st[b:e] = part
    return st


# ----------------------------------------------------------------------------- configs
def c2_batch(n: int, seed: int = 1):
    """C2: (msgs, sigs, pks, rands) for n single-pubkey sets."""
    sks = seeded_sks(n, b"c2/%d" % seed)
    msgs = messages(n, b"c2/%d" % seed)
    return msgs, sign(sks, msgs), public_keys(sks), rands(n, seed)


def committees(n_active: int, n_committees: int, seed: int) -> Tuple[np.ndarray, np.ndarray]:
    """A seeded shuffle of validator indices [0, n_active) split into n_committees
    contiguous committees (sizes differ by at most one, as compute_committee does)."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n_active).astype(np.uint32)
    off = np.array([n_active * c // n_committees for c in range(n_committees + 1)], dtype=np.uint32)
    return perm, off


def committee_signatures(reg_sks: Sequence[int], idx: np.ndarray, off: np.ndarray, msgs: bytes):
    """sig_c = (sum of the committee's secret keys) * H(m_c), plus those sums."""
    sums = []
    for c in range(len(off) - 1):
        s = 0
        for v in idx[off[c]:off[c + 1]]:
            s += reg_sks[int(v)]
        sums.append(s % R_ORDER)
    return sign(sums, msgs), sums
