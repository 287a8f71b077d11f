"""The latency regime's wave-per-point G2 engine (grandine_amd/csrc/bls_w4.h, row-distributed
Fp products of bls_dfp.h) bit by bit on the GPU, not only through
verdicts:

* tools/ubench/w4_prim: every primitive (products, squarings, lazy sums, biased subtractions,
  halving, the doubling and addition with every intermediate) on random operands, written as
  engine words and recomputed here with Python integers (tools/ubench/w4_prim.py); it caught
  the DPP-combined v_subrev_u32_dpp miscompile;
* tools/ubench/w4_check: every W4 formula (dbl, add with its degenerate cases, madd, psi,
  psi^2, [|x|]P, h_eff, the affine conversion, the Miller doubling / addition steps, a 32-bit
  scalar chain) against the engine's one-lane formulas on 64 points.

Both binaries are built in-tree by `make -C tools/ubench` (__graft_entry__.build)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "ubench", "_bin")


def _exe(name):
    path = os.path.join(BIN, name)
    if not os.path.exists(path):
        raise AssertionError("%s not built (make -C tools/ubench)" % path)
    return path


def test_w4_primitives_bit_exact(tmp_path):
    out = str(tmp_path / "prim.bin")
    r = subprocess.run([_exe("w4_prim"), out], capture_output=True, text=True, timeout=90)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    chk = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ubench", "w4_prim.py"), out],
                         capture_output=True, text=True, timeout=90)
    assert chk.returncode == 0, chk.stdout[-2000:] + chk.stderr[-2000:]
    assert "mismatches by op: none" in chk.stdout, chk.stdout[-3000:]


def test_w4_formulas_match_lane_engine():
    r = subprocess.run([_exe("w4_check")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "check: 0 / 64 points with a mismatch" in r.stdout, r.stdout[-2000:]


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bls12_381 as O  # test infrastructure (oracle/ header)
    return O


def test_w4_formulas_against_python_integers(tmp_path):
    """the W4 formula outputs against an INDEPENDENT recomputation
    with Python integers (oracle/bls12_381.py affine arithmetic), not against the engine's own
    lane formulas.  w4_check writes every W4 result (engine words, x 2^384) for its 64 seeded
    points; for the first 16 the points P = [s | 1] G2 and Q = [(s >> 7) 3 + 5] G2 are
    recomputed here from the seeds, and every result is compared as an affine point (Jacobian
    or homogeneous, as the formula outputs it) or, for Miller lines, as a line proportional to
    the oracle's (lambda x_T - y_T, -lambda, 1) (the engine's lines carry an Fp2 factor, which
    the final exponentiation removes)."""
    O = _oracle()
    path = str(tmp_path / "w4_dump.bin")
    r = subprocess.run([_exe("w4_check"), path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    raw = open(path, "rb").read()
    n, slots, words = 64, 16, 72
    assert len(raw) == 8 * n + 4 * n * slots * words
    seeds = [int.from_bytes(raw[8 * i:8 * i + 8], "little") for i in range(n)]
    body = raw[8 * n:]
    RI = pow(1 << 384, -1, O.P)
    M64 = (1 << 64) - 1

    def fp_at(blk, slot, k):  # the k-th 12-word Fp of a slot, canonical
        o = 4 * ((blk * slots + slot) * words + 12 * k)
        return int.from_bytes(body[o:o + 48], "little") * RI % O.P

    def f2_at(blk, slot, k):
        return (fp_at(blk, slot, 2 * k), fp_at(blk, slot, 2 * k + 1))

    def jac(blk, slot):
        X, Y, Z = (f2_at(blk, slot, k) for k in range(3))
        if Z == (0, 0):
            return None
        zi = O.f2_inv(Z)
        zi2 = O.f2_sqr(zi)
        return (O.f2_mul(X, zi2), O.f2_mul(Y, O.f2_mul(zi2, zi)))

    def hom(blk, slot):
        X, Y, Z = (f2_at(blk, slot, k) for k in range(3))
        zi = O.f2_inv(Z)
        return (O.f2_mul(X, zi), O.f2_mul(Y, zi))

    def line_ok(blk, slot, T, lam):
        L0, L2, L3 = (f2_at(blk, slot, k) for k in range(3))
        if L3 == (0, 0):
            return False
        i3 = O.f2_inv(L3)
        want0 = O.f2_sub(O.f2_mul(lam, T[0]), T[1])
        return O.f2_mul(L2, i3) == O.f2_neg(lam) and O.f2_mul(L0, i3) == want0

    def tangent(T):
        return O.f2_mul(O.f2_muls(O.f2_sqr(T[0]), 3), O.f2_inv(O.f2_add(T[1], T[1])))

    def chord(T, Q):
        return O.f2_mul(O.f2_sub(T[1], Q[1]), O.f2_inv(O.f2_sub(T[0], Q[0])))

    bad = {}
    for b in range(16):
        s = seeds[b]
        Pp = O.g2_mul(O.G2_GEN, s | 1)
        Qp = O.g2_mul(O.G2_GEN, (((s >> 7) * 3) & M64) + 5 & M64)
        P2, Q2 = O.g2_add(Pp, Pp), O.g2_add(Qp, Qp)
        k = ((s * 0x2545F4914F6CDD1D) & M64) >> 32 | 1
        hP = O.clear_cofactor_g2(Pp)
        checks = {
            "dbl": jac(b, 0) == P2,
            "add": jac(b, 1) == O.g2_add(Pp, Qp),
            "add(P,P)": jac(b, 2) == P2,
            "psi": jac(b, 3) == O.g2_psi(Pp),
            "psi2": jac(b, 4) == O.g2_psi(O.g2_psi(Pp)),
            "[|x|]P": jac(b, 5) == O.g2_mul(Pp, O.X_ABS),
            "h_eff P": jac(b, 6) == hP,
            "h_eff P affine": (f2_at(b, 7, 0), f2_at(b, 7, 1)) == hP,
            "line_dbl T": hom(b, 8) == Q2,
            "line_dbl lines": line_ok(b, 9, Qp, tangent(Qp)),
            "line_add_aff T": hom(b, 10) == O.g2_add(Q2, P2),
            "line_add_aff lines": line_ok(b, 11, Q2, chord(Q2, P2)),
            "madd": jac(b, 12) == O.g2_add(Pp, Qp),
            "[k]Q chain": jac(b, 13) == O.g2_mul(Qp, k),
            "line_add_proj T": hom(b, 14) == O.g2_add(Q2, Qp),
            "line_add_proj lines": line_ok(b, 15, Q2, chord(Q2, Qp)),
        }
        for name, ok in checks.items():
            if not ok:
                bad.setdefault(name, []).append(b)
    assert not bad, bad
