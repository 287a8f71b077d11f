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
