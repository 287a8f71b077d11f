"""CPU: the C-ABI library builds for gfx950, loads, and exports every symbol the public
header declares (no compute calls without a GPU)."""
import os
import re

from grandine_amd import _lib as G

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "grandine_bls_gpu.h")


def declared():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(gbls_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert declared() == sorted(G.EXPORTS)


def test_library_exports_every_symbol():
    L = G.load_library()
    for name in declared():
        assert hasattr(L, name), name


def test_version_string_without_device():
    L = G.load_library()
    assert b"gfx950" in L.gbls_version()
