"""Seeded structured encodings for codec parity tests (test infrastructure).

Compressed G1 (48 B) and G2 (96 B) encodings chosen to reach every branch of both codecs
(py_ecc 1.7.0's lax one, SURVEY A.4, and the spec's strict one, bls_signature.md:47-64):
all eight flag combinations, x with and without a square root on the curve, x + q and
other values at or above q, x = 0, junk below a set b_flag, and G2 imaginary parts whose
own top bits are set.  The expected results come from the oracle at test time; nothing
here is a reference file.
"""
import random

Q = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
M381 = (1 << 381) - 1


def _x_value(rng):
    r = rng.random()
    if r < 0.06:
        return 0
    if r < 0.12:
        return Q + rng.randrange(0, (1 << 381) - Q)        # >= q, still below 2^381
    if r < 0.16:
        return Q
    if r < 0.20:
        return M381
    return rng.randrange(1, Q)


def g1_encodings(seed: int, n: int):
    rng = random.Random(seed)
    out = [(0xC0 << 376).to_bytes(48, "big")]                # the canonical infinity
    for i in range(n - 1):
        flags = i % 8 if i < 64 else rng.randrange(8)      # bit 2: c_flag, bit 1: b_flag, bit 0: a_flag
        x = _x_value(rng)
        if flags & 2 and rng.random() < 0.5:
            x = rng.randrange(0, 1 << 381)                   # junk under a set b_flag
        z = (flags << 381) | (x & M381)
        out.append(z.to_bytes(48, "big"))
    return out


def g2_encodings(seed: int, n: int):
    rng = random.Random(seed)
    out = [(0xC0 << 376).to_bytes(48, "big") + bytes(48)]   # the canonical infinity
    for i in range(n - 1):
        flags = i % 8 if i < 64 else rng.randrange(8)
        x_im = _x_value(rng)
        x_re = _x_value(rng)
        top2 = rng.randrange(8) if rng.random() < 0.25 else 0   # flag bits of the real part's word
        if flags & 2 and rng.random() < 0.5:
            x_im, x_re = rng.randrange(0, 1 << 381), rng.randrange(0, 1 << 381)
        z1 = (flags << 381) | (x_im & M381)
        z2 = (top2 << 381) | (x_re & M381)
        out.append(z1.to_bytes(48, "big") + z2.to_bytes(48, "big"))
    return out
