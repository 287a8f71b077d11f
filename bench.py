#!/usr/bin/env python3
"""Headline benchmark: verified BLS signature sets/s on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1], SURVEY.md 8(d) "C2"): synthetic batches of
4096 single-pubkey signature sets -- seeded secret keys, distinct 32-byte signing roots,
sig_i = sk_i * H(m_i), nonzero 64-bit random scalars r_i -- each verified by ONE
random-linear-combination batch check, exactly Signature::multi_verify (reference
bls/src/signature.rs:95-129, reached from MultiVerifier::finish,
helper_functions/src/verifier.rs:301-323).  A "step" = --batches (default 16) such
batches, submitted together as segments of one device call the way the engine's
cross-caller coalescer merges concurrent MultiVerifier::finish calls: every batch keeps
its own scalars, its own S = sum r_i sig_i, its own final exponentiation and its own
verdict.  --inflight (default 2) submissions run at once on separate streams (step k on
stream k mod 2), as the coalescer keeps two leaders per device: one step's serial tail
(Horner, final exponentiation) overlaps the next step's hash_to_G2.  Inputs are resident in HBM (decompressed points, as blst takes them);
hash_to_G2 of every message, both scalar sides, the Miller products and the final
exponentiations all run inside the timed region.  The same run also times ONE batch per
step ("single_batch": the 4096-set latency view).

Other legs (--config): C3 sync-committee fast_aggregate_verify (10,000 messages x 512
registry keys; unit = messages), C4 an epoch of attestations (2,048 committees over a
2^20-key registry: key aggregation + multi_verify; unit = sets), C5 Holesky-scale
(2^20 sets over the GPUs, keys drawn from a 1.7M-key registry), C1 a mainnet-shaped
block (~131 sets) through the host-pointer ABI: latency, plus 64-set gossip batches.

N > 1 (torch.distributed.run, one rank per GPU, backend nccl = RCCL): every rank verifies
its own sets; the per-rank Miller partial (one Fp12, 576 B) and error flag are
all-gathered over xGMI, and every rank runs ONE final exponentiation over the product
(SURVEY.md 8(e)).  C2 is weak scaling (a fixed batch per GPU); C4 (one mainnet epoch, its
2048 committees split into whole committees per rank) and C5 (2^20 sets in total) are strong
scaling; C3 needs no exchange (per-message verdicts).

Extra JSON fields: "roofline" (dominant kernel's integer-multiply throughput vs the
measured v_mad_u64_u32 peak, HIP events on the launch stream, W frozen in BASELINE.md 4)
and "cpu_baseline" (the C restatement of blst's multi-verify built with BLS_REF_FAST, timed on
this host's cores).
"""

import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic work per unit, in Fp products (12-limb Montgomery, 288 v_mad_u64_u32
# each), FROZEN in BASELINE.md section 4 from tools/count_work.cpp (the engine's own
# serial formulas compiled for the host with -DGBLS_COUNT_FPMUL; a binary-GCD inversion
# counts as one product).  Per set unless noted.  The G2 side is priced at the reference
# algorithm (one 64-bit r_i sig_i per set, as blst does it), so the bucket MSM doing a
# tenth of that work raises the achieved fraction; a faster algorithm never lowers W.
MAD_PER_FPMUL = 288
W_FPMUL = {
    "k_h2c_field": 0,           # SHA-256 only
    "k_h2c_map": 2110,          # 2 SSWU maps (2 Fp exponentiations each) + 3-isogeny
    "k_h2c_clear": 2754,        # Q0+Q1, 2 x [|x|] (63 dbl + 5 add), psi, adds, affine
    "k_mv_g1mul": 783,          # r_i pk_i: 64-bit G1 double-and-add + affine
    "k_mv_g2mul": 1940,         # r_i sig_i: 64-bit G2 double-and-add (1897) + the sum (43)
    "k_msm": 1940,              # the same r_i sig_i work, done as a bucket MSM
    "k_g2sum": 43,              # one Jacobian G2 addition
    "k_lines": 1508,            # per pair: 63 doubling + 5 addition line steps
    "k_lines_S": 1508,          # per segment: the (-g1, S) pair's lines
    "k_ml_group": 2924,         # per pair: 68 events x (line evaluation 4 + sparse-dense product 39)
    "k_ml_reduce": 0,           # per pair: counted in k_ml_group (the wave levels fold <= 1/G of it)
    "k_ml_horner": 6030,        # per segment: 67 Fp12 squarings + 67 products
    "k_final_verdict": 13357,   # per segment: final exponentiation
    "k_pk_resolve": 11,   # per aggregated key: one mixed G1 addition
}
W_PAIR = W_FPMUL["k_lines"] + 884 + 1836  # lines + round-1 leaf + tree (frozen)      # 4228
W_SEGMENT = W_FPMUL["k_ml_horner"] + W_FPMUL["k_final_verdict"] + W_PAIR          # 23615
W_SET = (W_FPMUL["k_h2c_map"] + W_FPMUL["k_h2c_clear"] + W_FPMUL["k_mv_g1mul"]
         + W_FPMUL["k_mv_g2mul"] + W_PAIR)                                            # 11815
DTYPE = ("u32 (exact 381-bit Montgomery: 12 x 32-bit limbs; 14 x 28-bit limbs in the Miller "
         "products and the square-root exponentiations)")
W_G2_CHECK = 1251  # sigma subgroup check (fast_aggregate_verify)
W_C3_MESSAGE = (511 * W_FPMUL["k_pk_resolve"] + W_G2_CHECK + W_FPMUL["k_h2c_map"] + W_FPMUL["k_h2c_clear"]
                + 2 * W_PAIR + W_FPMUL["k_ml_horner"] + W_FPMUL["k_final_verdict"])            # 39579
assert W_C3_MESSAGE == 39579, W_C3_MESSAGE  # BASELINE.md 4, frozen


def cpu_threads():
    """Host cores this process may use: the affinity mask, capped by OMP_NUM_THREADS
    (the GPU box sets it to this job's CPU share)."""
    n = len(os.sched_getaffinity(0))
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, n)


def pmc_traffic(kernel, default_cmd):
    """HBM bytes per launch of `kernel` (a stage name: k_ml_group is the radix-2^28
    k_ml_group28 of the default build) from the committed rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE
    summary of the default command's 16-batch launches (profiles/r06/g_c2_pmc_bytes.csv,
    tools/prof/pmc_bytes.py --largest; FETCH_SIZE doubled per the gfx950 correction).  None for
    other commands or if absent."""
    # the round's final pass, else its latest checkpoint pass
    for tag in ("g", "f", "z", "x", "o"):
        path = os.path.join(ROOT, "profiles", "r06", tag + "_c2_pmc_bytes.csv")
        if os.path.exists(path):
            break
    if not default_cmd or not os.path.exists(path):
        return None
    with open(path) as f:
        for row in f.read().splitlines()[1:]:
            cols = row.split(",")
            name = cols[0].split("::")[-1].split("<")[0]
            if name in (kernel, kernel + "28"):
                return float(cols[4])
    return None


def cpu_baseline(n_sample, threads):
    """Time the C port (oracle/_build/bls_ref_bench_fast: oracle/bls_ref.c with BLS_REF_FAST) on
    a bounded sample of the C2 workload shape; None if it is not built."""
    exe = os.path.join(ROOT, "oracle", "_build", "bls_ref_bench_fast")
    if not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe, str(n_sample), str(threads)], capture_output=True, text=True,
                             timeout=300, check=True).stdout
        rec = json.loads(out.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 -- report, never fake a number
        return {"value": None, "unit": "sets/s", "cores": threads, "kind": "port", "error": str(e)[:200]}
    return {"value": rec["sets_per_s"], "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": "%d-set multi_verify batch, %d threads: oracle/bls_ref.c built with BLS_REF_FAST, a C "
                      "restatement of blst's multi-verify algorithm (Karatsuba Fp2/Fp6/Fp12, complex "
                      "squarings, 4-bit windowed exponentiations; portable C with 64-bit limbs, Fermat "
                      "inversion, plain 1269-bit hard part, no assembly / cyclotomic squaring), so it still "
                      "understates rayon+blst" % (n_sample, threads),
            "verdict_ok": rec.get("ok")}


def to_i64(vals):
    return [v - (1 << 64) if v >= 1 << 63 else v for v in vals]


class Leg:
    """One benchmark config: device-resident inputs + a step() that enqueues one pass."""
    metric = "verified BLS signature sets/sec (whole node)"
    unit = "sets/s"
    scaling = "weak"
    units = 0

    def stage_units(self, stage):
        return self.units


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2", choices=["C1", "C2", "C3", "C4", "C5"])
    ap.add_argument("--sets", type=int, default=0, help="override the per-config batch size")
    ap.add_argument("--inflight", type=int, default=2,
                    help="submissions in flight per GPU: step k runs on stream k %% inflight, so one step's "
                         "serial tail (Horner, final exponentiation) overlaps the next step's hash_to_G2, as "
                         "the engine's coalescer keeps two leaders per device")
    ap.add_argument("--batches", type=int, default=16,
                    help="C2: independent batches per step, verified as segments of ONE device submission "
                         "(each its own random linear combination, final exponentiation and verdict), as "
                         "the engine's coalescer merges concurrent callers")
    ap.add_argument("--cpu-sample", type=int, default=2048)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = this process's host CPU share")
    ap.add_argument("--emulate-shard", type=int, default=0,
                    help="C4 on one GPU: verify only rank 0's committees of an N-way split (its per-GPU "
                         "shard shape) and report the node rate that shape predicts (DESIGN.md 5)")
    ap.add_argument("--load-threads", type=int, default=16,
                    help="C1: gossip threads of the concurrent window and of the block-under-load legs")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stages", action="store_true",
                    help="no per-stage HIP-event timing in the timed region (roofline stage times absent)")
    ap.add_argument("--no-single", action="store_true",
                    help="C2: skip the one-batch-per-step leg (PMC passes then see only the 16-batch launches)")
    ap.add_argument("--tuning", action="store_true",
                    help="let the engine read its GBLS_* tuning environment variables (sweeps)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GBLS_BENCH_ONE_DEVICE=1 (rehearsal of the N-rank flow on a one-GPU box): every rank on
    # cuda:0, gloo instead of RCCL (RCCL refuses two ranks on one device)
    one_dev = os.environ.get("GBLS_BENCH_ONE_DEVICE") == "1"
    if world > 1:
        local = 0 if one_dev else local
        torch.cuda.set_device(local)
        if one_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from grandine_amd import _lib as G
    from grandine_amd import factory as F

    if args.tuning:
        G.enable_tuning()
    L = G.lib(1 << dev.index, 0)

    def dbytes(b):
        return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)

    def dnp(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)

    def ptr(t):
        return ctypes.c_void_p(t.data_ptr())

    def cur_stream():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def gather(out, inp):
        # the rank partials' exchange: one all-gather over RCCL (gloo rehearsal: list form)
        if not one_dev:
            dist.all_gather_into_tensor(out, inp)
            return
        torch.cuda.current_stream().synchronize()
        parts = [torch.empty_like(inp) for _ in range(world)]
        dist.all_gather(parts, inp)
        out.copy_(torch.cat(parts))

    leg = Leg()
    cfg = args.config
    # ------------------------------------------------------------------ batch-verify legs
    if cfg in ("C2", "C4", "C5"):
        nb = 1
        if cfg == "C2":
            per = args.sets or 4096
            nb = max(1, args.batches)
            parts = [F.c2_batch(per, seed=rank * 1000 + b + 1) for b in range(nb)]
            msgs = b"".join(p[0] for p in parts)
            sigs = b"".join(p[1] for p in parts)
            pks = b"".join(p[2] for p in parts)
            rands = [r for p in parts for r in p[3]]
            n = per * nb
            d_pks = dbytes(pks)
            idx = off = None
            leg.workload = ("C2: %d single-pubkey sets per GPU, random-scalar multi_verify" % per if nb == 1 else
                            "C2: %d independent batches of %d single-pubkey sets per GPU per step, each its own "
                            "random-scalar multi_verify (segments of one submission)" % (nb, per))
        elif cfg == "C4":
            # ONE mainnet epoch (32 slots x 64 committees, reference types/src/preset.rs:158,219),
            # the same on every rank; rank r verifies whole committees [r C / N, (r+1) C / N) and
            # the ranks' Miller partials meet in one final exponentiation: strong
            # scaling, as BASELINE.json configs[3] ("sharded over 8 GPUs")
            ncom_all = args.sets or 2048
            nreg = 1 << 20
            nact = nreg - 576  # committee sizes 511/512 (a shuffle remainder)
            sks, comp = F.registry(nreg, seed=b"c4-registry")
            assert not F.load_registry(comp).any()
            idx_all, off_all = F.committees(nact, ncom_all, seed=4)
            shard = world
            if args.emulate_shard:
                if world != 1:
                    raise SystemExit("--emulate-shard runs on one GPU")
                shard = args.emulate_shard
            c0, c1 = ncom_all * rank // shard, ncom_all * (rank + 1) // shard
            idx = idx_all[off_all[c0]:off_all[c1]]
            off = (off_all[c0:c1 + 1] - off_all[c0]).astype(np.uint32)
            msgs = F.messages(ncom_all, b"c4")[32 * c0:32 * c1]
            sigs, _ = F.committee_signatures(sks, idx, off, msgs)
            rands = F.rands(ncom_all, 4)[c0:c1]
            n = c1 - c0
            leg.pks_per_step = int(off[-1])
            leg.scaling = "strong"
            leg.epoch = {"committees": ncom_all, "keys": int(off_all[-1])}
            leg.workload = ("C4: one mainnet epoch of attestations -- %d committees (%d keys, sizes %d-%d) aggregated "
                            "from a %d-key device registry + one multi_verify, whole committees split over the GPUs "
                            "(%d on this rank)" % (ncom_all, int(off_all[-1]), int(np.diff(off_all).min()),
                                                   int(np.diff(off_all).max()), nreg, n))
        else:
            nreg = 1_700_000
            total = args.sets or (1 << 20)
            n = total // world
            sks, comp = F.registry(nreg, seed=b"holesky")
            assert not F.load_registry(comp).any()
            rng = np.random.default_rng(rank + 5)
            idx = rng.integers(0, nreg, size=n, dtype=np.uint32)
            off = None
            msgs = F.messages(n, b"c5/%d" % rank)
            sigs = F.sign([sks[int(i)] for i in idx], msgs)
            rands = F.rands(n, rank + 5)
            leg.scaling = "strong"
            leg.workload = ("C5: %d sets in total (%d per GPU), keys drawn uniformly from a %d-key device "
                            "registry, distinct messages, one multi_verify per GPU" % (total, n, nreg))
        d_msgs, d_sigs = dbytes(msgs), dbytes(sigs)
        d_rands = torch.tensor(to_i64(rands), dtype=torch.int64, device=dev)
        d_idx = dnp(idx) if idx is not None else None
        d_off = dnp(off) if off is not None else None
        # per in-flight slot: verdicts, and for N > 1 the partial / error buffers of the exchange
        slots = max(1, args.inflight)
        d_verdicts = [torch.full((nb,), -1, dtype=torch.int32, device=dev) for _ in range(slots)]
        d_part = [torch.zeros(nb * 576, dtype=torch.uint8, device=dev) for _ in range(slots)]
        d_err = [torch.zeros(nb, dtype=torch.int32, device=dev) for _ in range(slots)]
        d_parts = [torch.zeros(world * nb * 576, dtype=torch.uint8, device=dev) for _ in range(slots)]
        d_errs = [torch.zeros(world * nb, dtype=torch.int32, device=dev) for _ in range(slots)]
        seg = G.u32_array([n * b // nb for b in range(nb + 1)])
        # the fills above ran on the default stream; the steps run on their own streams, which
        # do not wait for it: without this a late fill can overwrite a warm-up step's partial
        # or verdict (seen as "verdicts of the warm-up step are WRONG" in 2-rank runs on one GPU)
        torch.cuda.synchronize()
        leg.units = n
        leg.segments = nb

        def step(slot=0):
            st = cur_stream()
            pidx = ptr(d_idx) if d_idx is not None else None
            poff = ptr(d_off) if d_off is not None else None
            v = d_verdicts[slot]
            if world == 1:
                if cfg == "C2":
                    rc = L.gbls_multi_verify_segments_device(ptr(d_msgs), ptr(d_sigs), ptr(d_pks), ptr(d_rands), n,
                                                             seg, nb, ptr(v), st)
                else:
                    rc = L.gbls_multi_verify_indexed_segments_device(ptr(d_msgs), ptr(d_sigs), pidx, poff,
                                                                     ptr(d_rands), n, seg, 1, ptr(v), st)
                G.check(rc, "multi_verify device")
                return
            if cfg == "C2":
                rc = L.gbls_multi_verify_partials_device(ptr(d_msgs), ptr(d_sigs), ptr(d_pks), ptr(d_rands), n, seg,
                                                         nb, ptr(d_part[slot]), ptr(d_err[slot]), st)
            else:
                rc = L.gbls_multi_verify_indexed_partials_device(ptr(d_msgs), ptr(d_sigs), pidx, poff, ptr(d_rands),
                                                                 n, seg, 1, ptr(d_part[slot]), ptr(d_err[slot]), st)
            G.check(rc, "multi_verify partials")
            gather(d_parts[slot], d_part[slot])
            gather(d_errs[slot], d_err[slot])
            rc = L.gbls_final_verify_partials_device(ptr(d_parts[slot]), ptr(d_errs[slot]), world, nb, ptr(v),
                                                     cur_stream())
            G.check(rc, "final_verify_partials")

        def verdict_ok():
            return all(bool((v == G.SUCCESS).all()) for v in d_verdicts)

        leg.stage_units = lambda s: {"k_ml_group": n + nb, "k_ml_reduce": n + nb, "k_lines_S": nb,
                                     "k_ml_horner": nb, "k_final_verdict": nb,
                                     "k_pk_resolve": getattr(leg, "pks_per_step", n)}.get(s, n)
        # whole step, frozen W: sets + per-batch pair/Horner/final exp + key aggregation
        leg.path_fpmul = lambda: (n * W_SET + nb * W_SEGMENT
                                  + (getattr(leg, "pks_per_step", n) - n) * W_FPMUL["k_pk_resolve"])
    # ------------------------------------------------------------------ C3
    elif cfg == "C3":
        m = args.sets or 10_000
        k = 512
        sks, comp = F.registry(1 << 16, seed=b"c3-registry")
        assert not F.load_registry(comp).any()
        rng = np.random.default_rng(rank + 3)
        committee = rng.choice(1 << 16, size=k, replace=False).astype(np.uint32)
        ssum = sum(sks[int(i)] for i in committee) % F.R_ORDER
        msgs = F.messages(m, b"c3/%d" % rank)
        sigs = bytearray(F.sign([ssum] * m, msgs))
        invalid = sorted(rng.choice(m, size=m // 100, replace=False).tolist())
        wrong = F.sign([(ssum + 1) % F.R_ORDER], msgs[:32])
        for i in invalid:
            sigs[192 * i:192 * i + 192] = wrong
        d_msgs, d_sigs = dbytes(msgs), dbytes(bytes(sigs))
        d_idx = dnp(np.tile(committee, m))
        d_off = dnp(np.arange(0, k * m + 1, k, dtype=np.uint32))
        # one verdict buffer per in-flight slot (two submissions at once, as C2)
        d_vs = [torch.full((m,), -1, dtype=torch.int32, device=dev) for _ in range(max(1, args.inflight))]
        torch.cuda.synchronize()
        want = torch.zeros(m, dtype=torch.int32)
        want[invalid] = G.VERIFY_FAIL
        leg.units = m
        leg.metric = "sync-committee fast_aggregate_verify messages/sec (whole node)"
        leg.unit = "messages/s"
        leg.workload = ("C3: %d messages per GPU, each fast_aggregate_verify against the same %d-key sync "
                        "committee (registry indices, aggregated on device every step), 1%% invalid" % (m, k))

        def step(slot=0):
            G.check(L.gbls_fast_aggregate_verify_indexed_device(ptr(d_sigs), ptr(d_msgs), ptr(d_idx), ptr(d_off), m,
                                                                ptr(d_vs[slot]), cur_stream()), "fav indexed device")

        def verdict_ok():
            return all(bool(torch.equal(v.cpu(), want)) for v in d_vs)

        # Batches of 2048..65536 checks take the grouped form (gbls_capi.hip grouped_verdicts):
        # r_i-weighted pairs, one Horner step + final exponentiation per group of GROUP checks,
        # then every member of a failing group re-checked on its own (its 2 pairs' Miller
        # products, Horner step and final exponentiation again).  The work counted is that.
        GROUP = 8
        if 2048 <= m <= 65536:
            bad_groups = {i // GROUP for i in invalid}
            redo = sum(min(GROUP, m - GROUP * g) for g in bad_groups)
            segs, g1muls = (m + GROUP - 1) // GROUP + redo, 2 * m
        else:
            redo, segs, g1muls = 0, m, 0
        leg.stage_units = lambda s: {"k_pk_resolve": m * k, "k_lines_S": m,
                                     "k_ml_group": 2 * m + 2 * redo, "k_ml_reduce": 2 * m + 2 * redo,
                                     "k_ml_horner": segs, "k_final_verdict": segs,
                                     "k_mv_g1mul": max(g1muls // 2, 1)}.get(s, m)
        # the whole path at BASELINE.md 4's FROZEN 39,579 Fp products per message (511 key
        # additions, sigma subgroup check, hash_to_G2, 2 pairs, Horner, final exponentiation):
        # the grouped form does less work per message, which raises the fraction, never W
        leg.path_fpmul = lambda: m * W_C3_MESSAGE
        leg.grouped = {"checks_per_group": GROUP, "miller_segments": segs, "rechecked": redo} if g1muls else None
    # ------------------------------------------------------------------ C1 (latency, host ABI)
    else:
        return bench_c1(args, L, G, F, np)

    D = max(1, args.inflight)
    streams = [torch.cuda.Stream() for _ in range(D)] if D > 1 else None

    def run(k):
        if streams is None:
            step()
            return
        s = streams[k % D]
        s.wait_stream(torch.cuda.default_stream()) if k < D else None
        with torch.cuda.stream(s):
            step(k % D)

    for k in range(max(args.warmup, D)):
        run(k)
    torch.cuda.synchronize()
    if not verdict_ok():
        if world > 1 and cfg in ("C2", "C4", "C5"):  # which side is wrong: each slot's own partial
            for sl in range(len(d_part)):
                vo = torch.full((nb,), -1, dtype=torch.int32, device=dev)
                L.gbls_final_verify_partials_device(ptr(d_part[sl]), ptr(d_err[sl]), 1, nb, ptr(vo), cur_stream())
                vg = torch.full((nb,), -1, dtype=torch.int32, device=dev)
                L.gbls_final_verify_partials_device(ptr(d_parts[sl]), ptr(d_errs[sl]), world, nb, ptr(vg), cur_stream())
                torch.cuda.synchronize()
                print("rank %d slot %d: verdict %s own-partial %s err %s gathered-again %s parts-equal-own %s" % (
                    rank, sl, d_verdicts[sl].tolist(), vo.tolist(), d_err[sl].tolist(), vg.tolist(),
                    bool(torch.equal(d_parts[sl][rank * nb * 576:(rank + 1) * nb * 576], d_part[sl]))),
                    file=sys.stderr, flush=True)
        raise SystemExit("verdicts of the warm-up step are WRONG")

    L.gbls_profile_reset()
    L.gbls_profile(0 if args.no_stages else 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enq = []  # host time of each step's enqueue (the device entry points return before the GPU work)
    for k in range(args.steps):
        te = time.perf_counter()
        run(k)
        enq.append(time.perf_counter() - te)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    L.gbls_profile(0)
    ok = verdict_ok()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
    if not ok:
        raise SystemExit("verdicts changed during the timed region")

    # ---- C4: every committee's own verdict (each committee one segment), on every rank
    committee_check = None
    if cfg == "C4":
        segc = G.u32_array(range(n + 1))
        vc = torch.full((n,), -1, dtype=torch.int32, device=dev)
        G.check(L.gbls_multi_verify_indexed_segments_device(ptr(d_msgs), ptr(d_sigs), ptr(d_idx), ptr(d_off),
                                                            ptr(d_rands), n, segc, n, ptr(vc), cur_stream()),
                "per-committee check")
        torch.cuda.synchronize()
        good = torch.tensor([int((vc == G.SUCCESS).sum().item())], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(good, op=dist.ReduceOp.SUM)
        expect = n if args.emulate_shard else leg.epoch["committees"]
        committee_check = {"committees_verified": int(good.item()), "committees": expect}
        if committee_check["committees_verified"] != expect:
            raise SystemExit("per-committee verdicts WRONG: %s" % committee_check)

    # ---- one batch per step (the 4096-set latency view), same inputs, after the main timing
    single = None
    if cfg == "C2" and world == 1 and leg.segments > 1 and not args.no_single:
        per = leg.units // leg.segments
        seg1 = G.u32_array([0, per])
        v1 = torch.full((1,), -1, dtype=torch.int32, device=dev)

        def step1():
            G.check(L.gbls_multi_verify_segments_device(ptr(d_msgs), ptr(d_sigs), ptr(d_pks), ptr(d_rands), per,
                                                        seg1, 1, ptr(v1), cur_stream()), "single batch")
        step1()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step1()
        torch.cuda.synchronize()
        d1 = time.perf_counter() - t1
        if int(v1.item()) != G.SUCCESS:
            raise SystemExit("single-batch verdict WRONG")
        single = {"batches_per_step": 1, "sets_per_step": per, "value": round(per * args.steps / d1, 1),
                  "ms_per_step": round(d1 / args.steps * 1e3, 4)}

    # ---- roofline of the dominant kernel (HIP events on the launch stream)
    nst = 32
    ms = (ctypes.c_double * nst)()
    calls = (ctypes.c_uint32 * nst)()
    ns = L.gbls_profile_read(ms, calls, nst)
    stages = {L.gbls_stage_name(i).decode(): (ms[i], calls[i]) for i in range(ns) if calls[i]}
    peak = L.gbls_measure_mad64_peak()
    # dominant kernel: the single-kernel stage with the most algorithmic work per step
    # (W x units; rocprofv3 reports the same kernel's duration).  Not by wall time: with two
    # submissions in flight a low-priority side-stream stage (k_mv_g1mul) spans most of a
    # step waiting for SIMDs.  Not roofline rows: the multi-kernel stages k_msm /
    # k_ml_reduce / k_g2sum, and k_lines_S.
    multi = {"k_msm", "k_ml_reduce", "k_g2sum", "k_lines_S"}
    cand = [k for k in stages if W_FPMUL.get(k, 0) > 0 and k not in multi]
    dom = max(cand, key=lambda k: leg.stage_units(k) * W_FPMUL[k]) if cand else None
    roof = None
    if dom:
        tot_ms, ncalls = stages[dom]
        avg_s = tot_ms / args.steps * 1e-3  # the stage's time per step (one or more launches)
        mads = leg.stage_units(dom) * W_FPMUL.get(dom, 0) * MAD_PER_FPMUL
        ach = mads / avg_s / 1e12
        roof = {"bound": "valu-int", "kernel": dom, "achieved": round(ach, 4),
                "peak": round(peak / 1e12, 3), "unit": "Tmad64/s",
                "frac": round(ach / (peak / 1e12), 5) if peak else None,
                "traffic": pmc_traffic(dom, cfg == "C2" and args.sets in (0, 4096) and args.batches == 16
                                       and args.inflight == 2),
                "avg_launch_ms": round(tot_ms / ncalls, 4),
                "path": {"work": "W-normalised: BASELINE.md 4's frozen blst-algorithm Fp products per unit "
                                 "(the engine may execute fewer, e.g. C3's grouped form)",
                         "fpmul_per_step": leg.path_fpmul(),
                         "stage_formula_fpmul_per_step": sum(leg.stage_units(k) * W_FPMUL.get(k, 0) for k in stages),
                         "achieved": round(leg.path_fpmul() * MAD_PER_FPMUL * args.steps / dt / 1e12, 4),
                         "frac": round(leg.path_fpmul() * MAD_PER_FPMUL * args.steps / dt / peak, 5)
                         if peak else None},
                "stage_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in stages.items()}}

    if rank == 0:
        # whole-job throughput: every rank's units (C5/C4 strong: the ranks' shares add up to the
        # one workload; C2 weak: world x the per-GPU batch)
        total_units = leg.epoch["committees"] if cfg == "C4" else world * leg.units
        value = total_units * args.steps / dt
        cpu = None
        if not args.no_cpu and world == 1 and cfg == "C2":
            cpu = cpu_baseline(args.cpu_sample, args.cpu_threads or cpu_threads())
        line = {"metric": leg.metric, "value": round(value, 1),
                "unit": leg.unit, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
                "scaling": leg.scaling, "vs_baseline": None, "dtype": DTYPE,
                "data": "synthetic (seeded keys, messages and scalars; signed on device)",
                "config": {"workload": leg.workload, "config": cfg, "units_per_gpu_per_step": leg.units,
                           "batches_per_step": getattr(leg, "segments", 1), "streams_in_flight": D,
                           "parallelism": "shard sets, RCCL all-gather of Fp12 partials" if world > 1 else "1 GPU"},
                "roofline": roof, "cpu_baseline": cpu}
        line["host_enqueue_ms"] = {"p50": round(sorted(enq)[len(enq) // 2] * 1e3, 3),
                                   "max": round(max(enq) * 1e3, 3), "argmax": enq.index(max(enq))}
        if cfg in ("C2", "C4", "C5"):
            line["pairings_per_s"] = round((total_units + world * leg.segments) * args.steps / dt, 1)
        if single:
            line["single_batch"] = single
        if getattr(leg, "grouped", None):
            line["config"]["grouped_checks"] = leg.grouped
        if cfg == "C4" and args.emulate_shard:
            # one rank's shard of an N-way split on this GPU: its own rate, and the node rate the
            # shape predicts when every rank runs its shard in the same time (the all-gather of
            # 576-B partials and the one final exponentiation are not included)
            per_rank = leg.units
            line["value"] = round(per_rank * args.steps / dt, 1)
            line["config"]["workload"] = ("C4 shard emulation: rank 0's %d of %d committees (a %d-way split) on one "
                                          "GPU" % (per_rank, leg.epoch["committees"], args.emulate_shard))
            line["shard_emulation"] = {"n_gpus_emulated": args.emulate_shard, "committees_per_rank": per_rank,
                                       "ms_per_step": round(dt / args.steps * 1e3, 4),
                                       "predicted_node_sets_per_s": round(leg.epoch["committees"] * args.steps / dt, 1)}
            line["epoch"] = dict(leg.epoch, per_committee_check=committee_check)
        elif cfg == "C4":
            line["pks_aggregated_per_s"] = round(leg.epoch["keys"] * args.steps / dt, 1)
            line["epoch"] = dict(leg.epoch, per_committee_check=committee_check)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_c1(args, L, G, F, np):
    """C1: a mainnet-shaped block's signature sets (1 proposer + 1 RANDAO + 128 aggregate
    attestations of ~512 registry keys + a 512-key sync aggregate = 131 sets) through the
    host-pointer ABI as MultiVerifier::finish calls it (G2 decompression of the 131
    signatures fused into one indexed multi_verify submission; the two-call form, decompress
    then verify, is timed beside it): per-call latency, PCIe included.
    Also: 64-set gossip batches (p2p/src/attestation_verifier.rs:37), serial and from 16
    concurrent threads (the node's verifier tasks)."""
    import threading
    nreg = 1 << 20
    sks, comp = F.registry(nreg, seed=b"c1-registry")
    assert not F.load_registry(comp).any()
    rng = np.random.default_rng(1)
    sizes = [1, 1] + [512] * 128 + [512]
    idx = np.concatenate([rng.choice(nreg, size=s, replace=False) for s in sizes]).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    n = len(sizes)
    msgs = F.messages(n, b"c1")
    sigs, _ = F.committee_signatures(sks, idx, off, msgs)
    comp_sigs = ctypes.create_string_buffer(96 * n)
    G.check(L.gbls_g2_compress(sigs, n, comp_sigs), "compress")
    rands = F.rands(n, 1)

    pidx, poff = idx.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p)

    def finish():  # one submission: device decompression fused into the batch verify
        st = G.i32_array(n)
        return L.gbls_multi_verify_compressed(msgs, comp_sigs, None, pidx, poff,
                                              (ctypes.c_uint64 * n)(*rands), n, st)

    def finish_two_calls():  # decompress, then verify (two submissions)
        dec = ctypes.create_string_buffer(192 * n)
        st = G.i32_array(n)
        G.check(L.gbls_g2_decompress(comp_sigs, n, dec, st), "decompress")
        assert all(st[i] == 0 for i in range(n))
        return L.gbls_multi_verify_indexed(msgs, dec, pidx, poff, (ctypes.c_uint64 * n)(*rands), n)

    def timed(fn):
        for _ in range(args.warmup):
            assert fn() == G.SUCCESS
        out = []
        for _ in range(args.steps):
            t = time.perf_counter()
            assert fn() == G.SUCCESS
            out.append(time.perf_counter() - t)
        return sorted(out)

    # the Rust drop-in's form (rust/bls_patch/verifier.rs): deferred Triple key LISTS handed over
    # as points + per-set offsets, summed on the device inside the same submission
    pts = F.public_keys([sks[int(i)] for i in idx])

    def finish_points():
        st = G.i32_array(n)
        return L.gbls_multi_verify_compressed_ex(msgs, comp_sigs, pts, None, poff,
                                                 (ctypes.c_uint64 * n)(*rands), n, st, 0)

    lat = timed(finish)
    lat2 = timed(finish_two_calls)
    latp = timed(finish_points)
    # single checks at n = 1 (SingleVerifier, sync-committee messages and contributions):
    # Signature::verify, fast_aggregate_verify over 512 keys, a decompression, and
    # SingleVerifier::extend of one triple (decompression + verify in one submission)
    sm, ss, sp, _ = F.c2_batch(1, seed=65)
    scomp = ctypes.create_string_buffer(96)
    G.check(L.gbls_g2_compress(ss, 1, scomp), "compress")
    fav_keys = pts[96 * int(off[2]):96 * int(off[3])]
    fav_sig = sigs[192 * 2:192 * 3]
    one = G.u32_array([0, 1])

    def v1():
        return L.gbls_verify(ss, sm, 32, sp)

    def fav1():
        return L.gbls_fast_aggregate_verify(fav_sig, msgs[64:96], 32, fav_keys, 512)

    def dec1():
        out, st = ctypes.create_string_buffer(192), G.i32_array(1)
        rc = L.gbls_g2_decompress(scomp, 1, out, st)
        return rc if st[0] == 0 else 1

    def ext1():
        st, v = G.i32_array(1), G.i32_array(1)
        G.check(L.gbls_verify_batch_compressed(sm, scomp, sp, one, 1, st, v), "extend")
        return v[0] if st[0] == 0 else 1

    single = {name: timed(fn) for name, fn in (("verify", v1), ("fast_aggregate_verify_512", fav1),
                                               ("g2_decompress", dec1), ("single_verifier_extend_1", ext1))}
    # 16 threads of single verifies for 2 s (coalesced into shared submissions)
    sv_calls = [0] * 16
    sv_errs = []
    sv_go = threading.Event()
    sv_end = [0.0]

    def sv_worker(k):
        sv_go.wait()
        while True:
            if v1() != G.SUCCESS:
                sv_errs.append(1)
            if time.perf_counter() > sv_end[0]:
                break
            sv_calls[k] += 1

    ths = [threading.Thread(target=sv_worker, args=(k,)) for k in range(16)]
    for x in ths:
        x.start()
    sv_end[0] = time.perf_counter() + 2.0
    sv_go.set()
    for x in ths:
        x.join()
    assert not sv_errs
    # gossip: 64 single-key sets per call
    gm, gs, gp, gr = F.c2_batch(64, seed=64)
    r64 = (ctypes.c_uint64 * 64)(*gr)
    glat = []
    for _ in range(args.steps):
        t = time.perf_counter()
        assert L.gbls_multi_verify(gm, gs, gp, r64, 64) == G.SUCCESS
        glat.append(time.perf_counter() - t)
    # 16 threads for a fixed 2 s window (steady state: the calls completed inside it count)
    nthr, window = args.load_threads, 2.0
    errs = []
    done_calls = [0] * nthr
    go = threading.Event()
    t_end = [0.0]

    def worker(k):
        go.wait()
        while True:
            if L.gbls_multi_verify(gm, gs, gp, r64, 64) != G.SUCCESS:
                errs.append(1)
            if time.perf_counter() > t_end[0]:
                break
            done_calls[k] += 1

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(nthr)]
    for x in ths:
        x.start()
    t = time.perf_counter()
    t_end[0] = t + window
    go.set()
    for x in ths:
        x.join()
    conc = window
    assert not errs
    glat.sort()
    # f3: the block under gossip load -- 16 threads keep submitting 64-set batches while the
    # block's finish runs with the block-import priority class (GBLS_CALL_BLOCK) and without
    stop = threading.Event()

    def loader():
        while not stop.is_set():
            if L.gbls_multi_verify(gm, gs, gp, r64, 64) != G.SUCCESS:
                errs.append(1)

    def finish_flags(flags):
        st = G.i32_array(n)
        return L.gbls_multi_verify_compressed_ex(msgs, comp_sigs, None, pidx, poff,
                                                 (ctypes.c_uint64 * n)(*rands), n, st, flags)

    ths = [threading.Thread(target=loader) for _ in range(nthr)]
    for x in ths:
        x.start()
    time.sleep(0.05)
    lat_prio = timed(lambda: finish_flags(G.CALL_BLOCK))
    lat_noprio = timed(lambda: finish_flags(0))
    stop.set()
    for x in ths:
        x.join()
    assert not errs
    # gossip latency while blocks are imported back to back (sync / backfill): every normal call
    # that arrives during a block call is held up to 4 ms (measure the hold's cost)
    stop2 = threading.Event()

    def blocks():
        while not stop2.is_set():
            if finish_flags(G.CALL_BLOCK) != G.SUCCESS:
                errs.append(1)

    bt = threading.Thread(target=blocks)
    bt.start()
    time.sleep(0.02)
    glat_b = []
    for _ in range(args.steps):
        t = time.perf_counter()
        assert L.gbls_multi_verify(gm, gs, gp, r64, 64) == G.SUCCESS
        glat_b.append(time.perf_counter() - t)
    stop2.set()
    bt.join()
    assert not errs
    glat_b.sort()
    line = {"metric": "MultiVerifier::finish latency, mainnet-shaped block (C1)", "value": round(lat[len(lat) // 2] * 1e3, 3),
            "unit": "ms (p50)", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(sum(lat) / len(lat) * 1e3, 3), "higher_is_better": False, "scaling": "n/a",
            "vs_baseline": None, "dtype": DTYPE,
            "data": "synthetic (seeded registry, committees and messages)",
            "config": {"workload": "C1: %d sets (%d keys aggregated from the registry), 96-byte signatures "
                                   "decompressed on the device inside the verify submission, host pointers, PCIe "
                                   "included" % (n, int(off[-1])), "config": "C1"},
            "p99_ms": round(lat[min(len(lat) - 1, int(len(lat) * 0.99))] * 1e3, 3),
            "decompress_then_verify_p50_ms": round(lat2[len(lat2) // 2] * 1e3, 3),
            "points_pk_off": {"p50_ms": round(latp[len(latp) // 2] * 1e3, 3),
                              "p99_ms": round(latp[min(len(latp) - 1, int(len(latp) * 0.99))] * 1e3, 3),
                              "form": "the Rust drop-in's deferred Triple key lists: %d affine keys (96 B each) + "
                                      "per-set offsets, summed on the device in the same submission" % int(off[-1])},
            "single_checks_n1_p50_ms": {k: round(v[len(v) // 2] * 1e3, 3) for k, v in single.items()},
            "single_verify_16_threads_per_s": round(sum(sv_calls) / 2.0, 1),
            "gossip64": {"p50_ms": round(glat[len(glat) // 2] * 1e3, 3),
                         "p99_ms": round(glat[min(len(glat) - 1, int(len(glat) * 0.99))] * 1e3, 3),
                         "concurrent_16_threads_sets_per_s": round(sum(done_calls) * 64 / conc, 1),
                         "concurrent_window_s": window},
            "block_under_gossip_load": {
                "block_priority_p50_ms": round(lat_prio[len(lat_prio) // 2] * 1e3, 3),
                "block_priority_p99_ms": round(lat_prio[min(len(lat_prio) - 1, int(len(lat_prio) * 0.99))] * 1e3, 3),
                "no_priority_p50_ms": round(lat_noprio[len(lat_noprio) // 2] * 1e3, 3),
                "no_priority_p99_ms": round(lat_noprio[min(len(lat_noprio) - 1, int(len(lat_noprio) * 0.99))] * 1e3, 3),
                "load": "%d threads x 64-set gbls_multi_verify in a loop" % nthr},
            "gossip64_under_back_to_back_blocks": {
                "p50_ms": round(glat_b[len(glat_b) // 2] * 1e3, 3),
                "p99_ms": round(glat_b[min(len(glat_b) - 1, int(len(glat_b) * 0.99))] * 1e3, 3),
                "load": "one thread importing the C1 block (GBLS_CALL_BLOCK) back to back"},
            "roofline": None, "cpu_baseline": None}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
