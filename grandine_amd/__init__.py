"""MI355X-native BLS12-381 signature verification engine for Grandine's hot path.

Python mirror of the reference's ``bls`` crate (``grandine_amd.bls``) and of
``helper_functions::verifier`` (``grandine_amd.verifier``) on top of the C ABI in
``include/grandine_bls_gpu.h`` (``grandine_amd._lib``).
"""

__version__ = "0.1.0"
