"""MI355X (gfx950) BLS12-381 engine: drop-in for eth2spec.utils.bls.

`bls381_amd.bls` mirrors the reference module; `bls381_amd._native` is the
ctypes binding of include/bls381.h; `bls381_amd.sharding` splits a
bls_verify_multiple across ranks (one Fp12 partial per GPU, one final
exponentiation on rank 0).
"""
from . import _native  # noqa: F401
