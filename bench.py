#!/usr/bin/env python3
"""Headline benchmark: verified BLS signature sets/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY.md 8(d) "C2"): per rank, a synthetic batch of
4096 single-pubkey signature sets -- interop-style secret keys, distinct 32-byte
signing roots, sig_i = sk_i * H(m_i), nonzero 64-bit random scalars r_i -- verified by
ONE random-linear-combination batch check, exactly Signature::multi_verify
(reference bls/src/signature.rs:95-129, reached from MultiVerifier::finish,
helper_functions/src/verifier.rs:301-323).  A "step" = one multi_verify of the batch,
inputs already resident in HBM (decompressed points, as blst takes them).

N > 1 (torch.distributed.run, one rank per GPU, backend nccl = RCCL): every rank
verifies its own 4096 sets; the per-rank Miller partial (one Fp12, 576 B) and error
flag are all-gathered over xGMI, and every rank runs ONE final exponentiation over the
product.  Weak scaling: value = N * 4096 * steps / max-rank time.

Extra JSON fields: "roofline" (dominant kernel's integer-multiply throughput vs the
measured v_mad_u64_u32 peak, HIP events on the launch stream) and "cpu_baseline" (the
C oracle restating blst's multi-verify algorithm, timed on this host's cores).
"""

import argparse
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

# Algorithmic work per unit, in Fp products (12-limb Montgomery, 288 v_mad_u64_u32
# each), counted from the formulas each kernel executes (DESIGN.md "Roofline").
# Frozen here; a faster algorithm raises the achieved fraction, never lowers W.
MAD_PER_FPMUL = 288
W_FPMUL = {
    "k_h2c_field": 0,        # SHA-256 only
    "k_h2c_map": 2 * 1009,   # per set: 2 SSWU maps (2 sliding-window exps each) + isogeny
    "k_h2c_clear": 2360,     # per set: Q0+Q1, 2 x [|x|] (63 dbl + 5 add), 5 adds, psi
    "k_mv_g1mul": 1240,      # per set: 64-bit G1 double-and-add + affine
    "k_mv_g2mul": 3150,      # per set: 64-bit G2 double-and-add
    "k_g2sum": 48,           # per set: one Jacobian G2 add
    "k_lines": 1530,         # per pair: 63 doubling + 5 addition line steps
    "k_lines_S": 1530,       # per segment: the (-g1, S) pair's lines
    "k_ml_leaf": 34 * 68 // 2,  # per pair: 68 events x (eval + half a sparse*sparse)
    "k_ml_reduce": 54 * 68 // 2,  # per pair: 68 events x ~1/2 dense product
    "k_ml_horner": 0,
    "k_final_verdict": 0,
}


def interop_sk(i: int) -> bytes:
    """interop/src/lib.rs:65-76 secret key derivation (big-endian 32 bytes)."""
    h = hashlib.sha256(i.to_bytes(8, "little") + bytes(24)).digest()
    return (int.from_bytes(h, "little") % R_ORDER).to_bytes(32, "big")


def make_workload(G, L, n, seed):
    sks = b"".join(interop_sk(seed * 1_000_000 + i) for i in range(n))
    msgs = b"".join(hashlib.sha256(b"c2/%d/%d" % (seed, i)).digest() for i in range(n))
    pks = ctypes.create_string_buffer(96 * n)
    sigs = ctypes.create_string_buffer(192 * n)
    G.check(L.gbls_sk_to_pk(sks, n, pks), "gbls_sk_to_pk")
    G.check(L.gbls_sign(sks, msgs, G.u32_array(range(0, 32 * n + 1, 32)), n, sigs), "gbls_sign")
    x = (seed * 0x9E3779B97F4A7C15 + 12345) & ((1 << 64) - 1)
    rands = []
    for _ in range(n):  # xorshift64*: deterministic nonzero scalars
        x ^= (x >> 12)
        x ^= (x << 25) & ((1 << 64) - 1)
        x ^= (x >> 27)
        rands.append(((x * 0x2545F4914F6CDD1D) & ((1 << 64) - 1)) or 1)
    return msgs, sigs.raw, pks.raw, rands


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE
    summary of this same command at the same n (profiles/r01/pmc_bytes.csv, written by
    tools/prof/pmc_bytes.py; FETCH_SIZE doubled per the gfx950 correction).  None if absent."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01", "pmc_bytes.csv")
    if n != 4096 or not os.path.exists(path):
        return None
    with open(path) as f:
        for row in f.read().splitlines()[1:]:
            cols = row.split(",")
            if cols[0].split("::")[-1] == kernel:
                return float(cols[4])
    return None


def cpu_baseline(n_sample, threads):
    """Time the C oracle (oracle/_build/bls_ref, restatement of blst's multi-verify) on a
    bounded sample of the same workload shape; None if the oracle is not built."""
    exe = os.path.join(ROOT, "oracle", "_build", "bls_ref_bench")
    if not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe, str(n_sample), str(threads)], capture_output=True, text=True,
                             timeout=300, check=True).stdout
        rec = json.loads(out.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 -- report, never fake a number
        return {"value": None, "unit": "sets/s", "cores": threads, "kind": "port", "error": str(e)[:200]}
    return {"value": rec["sets_per_s"], "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": "%d-set multi_verify batch (C restatement of blst's algorithm, %d threads)"
                      % (n_sample, threads), "verdict_ok": rec.get("ok")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets", type=int, default=4096)
    ap.add_argument("--cpu-sample", type=int, default=2048)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from grandine_amd import _lib as G

    L = G.load_library()
    if L.gbls_init(1 << dev.index, 0) != G.SUCCESS:
        raise G.EngineUnavailable("gbls_init failed: no gfx950 device")
    n = args.sets
    msgs, sigs, pks, rands = make_workload(G, L, n, seed=rank + 1)

    def dev_bytes(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
        return t

    d_msgs, d_sigs, d_pks = dev_bytes(msgs), dev_bytes(sigs), dev_bytes(pks)
    d_rands = torch.tensor([r - (1 << 64) if r >= (1 << 63) else r for r in rands], dtype=torch.int64,
                           device=dev)
    d_verdict = torch.full((1,), -1, dtype=torch.int32, device=dev)
    d_part = torch.zeros(576, dtype=torch.uint8, device=dev)
    d_err = torch.zeros(1, dtype=torch.int32, device=dev)
    d_parts = torch.zeros(world * 576, dtype=torch.uint8, device=dev)
    d_errs = torch.zeros(world, dtype=torch.int32, device=dev)
    seg = G.u32_array([0, n])

    def ptr(t):
        return ctypes.c_void_p(t.data_ptr())

    def step():
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        if world == 1:
            rc = L.gbls_multi_verify_segments_device(ptr(d_msgs), ptr(d_sigs), ptr(d_pks), ptr(d_rands), n, seg,
                                                     1, ptr(d_verdict), st)
            G.check(rc, "multi_verify_segments_device")
        else:
            rc = L.gbls_multi_verify_partials_device(ptr(d_msgs), ptr(d_sigs), ptr(d_pks), ptr(d_rands), n, seg,
                                                     1, ptr(d_part), ptr(d_err), st)
            G.check(rc, "multi_verify_partials_device")
            dist.all_gather_into_tensor(d_parts, d_part)
            dist.all_gather_into_tensor(d_errs, d_err)
            st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            rc = L.gbls_final_verify_partials_device(ptr(d_parts), ptr(d_errs), world, 1, ptr(d_verdict), st)
            G.check(rc, "final_verify_partials_device")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if int(d_verdict.item()) != G.SUCCESS:
        raise SystemExit("verification of the valid batch FAILED (verdict %d)" % int(d_verdict.item()))

    L.gbls_profile_reset()
    L.gbls_profile(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    L.gbls_profile(0)
    ok = int(d_verdict.item()) == G.SUCCESS
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
    if not ok:
        raise SystemExit("verdict changed during the timed region")

    # ---- roofline of the dominant kernel (HIP events on the launch stream)
    nst = 16
    ms = (ctypes.c_double * nst)()
    calls = (ctypes.c_uint32 * nst)()
    ns = L.gbls_profile_read(ms, calls, nst)
    stages = {L.gbls_stage_name(i).decode(): (ms[i], calls[i]) for i in range(ns) if calls[i]}
    peak = L.gbls_measure_mad64_peak()
    dom = max(stages, key=lambda k: stages[k][0]) if stages else None
    roof = None
    if dom:
        tot_ms, ncalls = stages[dom]
        avg_s = tot_ms / ncalls * 1e-3
        units = {"k_ml_leaf": n + 1, "k_ml_reduce": n + 1, "k_lines_S": 1}.get(dom, n)
        mads = units * W_FPMUL.get(dom, 0) * MAD_PER_FPMUL
        ach = mads / avg_s / 1e12
        roof = {"bound": "valu-int", "kernel": dom, "achieved": round(ach, 4),
                "peak": round(peak / 1e12, 3), "unit": "Tmad64/s", "frac": round(ach / (peak / 1e12), 5) if peak else None,
                "traffic": pmc_traffic(dom, n), "avg_launch_ms": round(tot_ms / ncalls, 4),
                "stage_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in stages.items()}}

    if rank == 0:
        value = world * n * args.steps / dt
        cpu = None if args.no_cpu or world > 1 else cpu_baseline(args.cpu_sample, args.cpu_threads)
        line = {"metric": "verified BLS signature sets/sec (whole node)", "value": round(value, 1),
                "unit": "sets/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u32 (381-bit Montgomery, 12x32 limbs)",
                "data": "synthetic (interop keys, seeded messages / scalars)",
                "config": {"workload": "C2: %d single-pubkey sets per GPU, random-scalar multi_verify" % n,
                           "sets_per_gpu": n, "parallelism": "shard sets, RCCL all-gather of Fp12 partials"
                           if world > 1 else "1 GPU"},
                "pairings_per_s": round(world * (n + 1) * args.steps / dt, 1),
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
