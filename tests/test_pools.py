"""CPU: the sync-committee pool mirror's planning (grandine_amd/pools.py, f4) against the
reference loop of operation_pools/src/sync_committee_agg_pool/pool.rs:159-192 -- the same bits
and the same additions per aggregate, in the same order, including the early return at the first
message signature that does not decode (its bit set, no later one)."""
import random

from grandine_amd import pools


def reference_loop(bits, messages, bad):
    """pool.rs:159-192 with `message.signature.try_into()?` failing for the messages in `bad`."""
    added = [[] for _ in bits]
    for m, (positions, _) in enumerate(messages):
        for pos in positions:
            for k, b in enumerate(bits):
                if b[pos]:
                    continue
                b[pos] = True
                if m in bad:
                    return added, m
                added[k].append(m)
    return added, None


def test_plan_matches_the_reference_loop():
    rng = random.Random(7)
    for case in range(300):
        size = rng.choice((4, 8, 16))
        naggr = rng.randint(1, 4)
        init = [[rng.random() < 0.3 for _ in range(size)] for _ in range(naggr)]
        nmsg = rng.randint(0, 12)
        messages = [(rng.sample(range(size), rng.randint(0, 2)), b"") for _ in range(nmsg)]
        bad = {m for m in range(nmsg) if rng.random() < 0.15}
        want_bits = [list(b) for b in init]
        want_added, want_err = reference_loop(want_bits, messages, bad)
        aggs = [pools.Aggregate(size, signature="sig%d" % k, bits=b) for k, b in enumerate(init)]
        plan = pools.plan_additions(aggs, messages)
        first = pools.cut_at_first_bad(plan, aggs, bad)
        done = plan if first is None else plan[:first]
        got_added = [[m for k2, _, m in done if k2 == k] for k in range(naggr)]
        assert [a.bits for a in aggs] == want_bits, case
        assert got_added == want_added, case
        assert (None if first is None else plan[first][2]) == want_err, case
