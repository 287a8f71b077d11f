"""Host mirror of the sync-committee contribution pool's signature aggregation (f4):
operation_pools/src/sync_committee_agg_pool/pool.rs `aggregate_messages` (:142-195) and the
message loop of `add_sync_committee_contribution` (:90-115).  The reference decompresses each
message signature and adds it into every aggregate that lacks the message's subcommittee
position, one `aggregate_in_place` per (position, aggregate); the mirror plans the same additions
in the same loop order, decompresses the messages' signatures in ONE engine call and forms every
aggregate's sum in ONE `gbls_g2_aggregate_segments` submission (segment k = aggregate k's signature
followed by its additions).  A signature that does not decode ends the reference at its first
use with that addition's bit already set (`?` after `set`), so the mirror keeps exactly the
bits and sums the reference holds at that point and raises the same DecompressionFailed.
Rust: rust/bls_patch/sync_committee_pool.rs."""
import ctypes
from typing import List, Optional, Sequence, Tuple

from . import _lib as G
from .bls import DecompressionFailed, Signature, decompress_signatures


class Aggregate:
    """sync_committee_agg_pool/types.rs Aggregate: aggregation bits + aggregate signature."""

    __slots__ = ("bits", "signature")

    def __init__(self, size: int, signature: Optional[Signature] = None, bits: Sequence[bool] = ()):
        self.bits = list(bits) if bits else [False] * size
        self.signature = signature if signature is not None else Signature.default()


def plan_additions(aggregates: List[Aggregate], messages: Sequence[Tuple[Sequence[int], bytes]]):
    """The reference's loop order (pool.rs:159-192 / :90-115) without the point arithmetic: for
    message m, each of its subcommittee positions, each aggregate without that bit -> the bit is
    set and (aggregate k, position, m) is one addition.  Returns the additions in order."""
    plan = []
    for m, (positions, _) in enumerate(messages):
        for pos in positions:
            for k, agg in enumerate(aggregates):
                if agg.bits[pos]:
                    continue  # the reference logs a duplicate and skips
                agg.bits[pos] = True
                plan.append((k, pos, m))
    return plan


def cut_at_first_bad(plan, aggregates: List[Aggregate], bad_messages) -> Optional[int]:
    """The reference returns at the first addition whose message signature does not decode, with
    that addition's bit set and no later one: clear the later additions' bits, return the index
    of the failing addition (None: every addition decodes)."""
    first = next((i for i, (_, _, m) in enumerate(plan) if m in bad_messages), None)
    if first is not None:
        for k, pos, _ in plan[first + 1:]:
            aggregates[k].bits[pos] = False
    return first


def aggregate_signature_segments(segments: Sequence[Sequence[bytes]]) -> List[bytes]:
    """gbls_g2_aggregate_segments: the sum of each segment's affine points (192-byte engine
    layout), one submission for all segments (none empty)."""
    nseg = len(segments)
    L = G.lib()
    flat = b"".join(p for seg in segments for p in seg)
    off = [0]
    for seg in segments:
        off.append(off[-1] + len(seg))
    out = ctypes.create_string_buffer(192 * nseg)
    st = G.i32_array(nseg)
    G.check(L.gbls_g2_aggregate_segments(G.buf(flat), G.u32_array(off), nseg, out, st),
            "gbls_g2_aggregate_segments")
    assert all(st[s] == G.SUCCESS for s in range(nseg)), [st[s] for s in range(nseg)]
    return [out.raw[192 * s:192 * (s + 1)] for s in range(nseg)]


def aggregate_messages(aggregates: List[Aggregate], messages: Sequence[Tuple[Sequence[int], bytes]],
                       size: int) -> None:
    """pool.rs:142-195 (`aggregate_messages`) on the engine: `messages` are (the message's
    positions in the subcommittee, its 96-byte signature).  An empty pool starts with one default
    aggregate, as the reference does."""
    if not aggregates:
        aggregates.append(Aggregate(size))
    plan = plan_additions(aggregates, messages)
    dec = decompress_signatures([sig for _, sig in messages]) if messages else []
    bad = {m for m, (st, _) in enumerate(dec) if st != G.SUCCESS}
    first = cut_at_first_bad(plan, aggregates, bad)
    done = plan if first is None else plan[:first]
    segments = [[agg.signature.raw] for agg in aggregates]
    for k, _, m in done:
        segments[k].append(dec[m][1])
    sums = aggregate_signature_segments(segments)
    for agg, raw in zip(aggregates, sums):
        agg.signature = Signature(raw)
    if first is not None:
        raise DecompressionFailed(dec[plan[first][2]][0])
