"""
ORACLE -- TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement of the reference's BLS12-381 path, used only by `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg, as the checker.

What it restates
----------------
The reference (`sigp/consensus-specs`, mounted at /root/reference) routes every
BLS call through `test_libs/pyspec/eth2spec/utils/bls.py:1,24-46` into the
third-party package **py_ecc == 1.7.0** (`test_generators/bls/requirements.txt:1`),
which is neither vendored in the reference nor installed here.  This module
restates py_ecc 1.7.0's published algorithms in plain Python integers:

* `specs/bls_signature.md:36-52`   G1 compressed format        -> compress_G1 / decompress_G1
* `specs/bls_signature.md:54-64`   G2 compressed format        -> compress_G2 / decompress_G2
* `specs/bls_signature.md:68-87`   hash_to_G2 (try-and-increment, G2 cofactor)
* `specs/bls_signature.md:89-109`  modular_squareroot (Fq2, eighth roots of unity)
* `specs/bls_signature.md:113-119` aggregation
* `specs/bls_signature.md:131-146` bls_verify / bls_verify_multiple
* py_ecc `optimized_bls12_381` homogeneous-projective `double`/`add`/recursive
  `multiply` -- mirrored formula-for-formula because the
  `msg_hash_g2_uncompressed` vectors (`test_generators/bls/main.py:56-72`) print
  the raw, un-normalised projective triple.
* py_ecc `bls.api` verify / verify_multiple / aggregate_* / sign / privtopub
  semantics: the infinity short-circuit inside
  `pairing`, the exception-to-False mapping, distinct-message grouping, a single
  final exponentiation per call, the length-mismatch exception.
* Pairing: ate Miller loop over |x| in Fq12 coordinates (tower w^12 - 2w^6 + 2,
  as py_ecc) and the naive final exponentiation f^((q^12-1)/r) (Appendix A.9).

Decoding: two codecs.  The default is py_ecc 1.7.0's own `decompress_G1` /
`decompress_G2`: b_flag set means infinity whatever the other bits,
x = z mod 2^381 (G2: the imaginary part; the real part is all 384 bits of z2) reduced
mod q by FQ / FQ2, and neither c_flag nor x < q is checked.  `strict=True` applies the
spec's checks instead (`bls_signature.md:47-52,58-64`: c_flag, x < q, canonical
infinity, G2's z2 flags clear) -- the codec of the strict policy.  Both give the same
point for every canonical encoding.

Domain serialisation: py_ecc 1.7.0 feeds `domain.to_bytes(8, DOMAIN_BYTEORDER)`
into SHA-256 ("medium, recalled"); the single switch is
`DOMAIN_BYTEORDER` below.

Pinning: see tests/test_oracle_known_answers.py (SURVEY.md Appendix B values,
which match the published eth2 priv_to_pub / aggregate_pubkeys vectors).
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------
# Curve constants (bls_signature.md:71-72, :126-127)
# ---------------------------------------------------------------------------
q = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
BLS_X = -0xd201000000010000
G2_cofactor = 305502333931268344200999753193121504214466019254188142667664032982267604182971884026507427359259977847832272839041616661285803823378372096355777062779109
G1_cofactor = 0x396c8c005555e1568c00aaab0000aaab

g_x = 3685416753713387016781088315183077757961620795782546409894578378688607592378376318836054947676345821548104185464507
g_y = 1339506544944476473020471379941921221584933875938349620426543736416511423956333506472724655353366534992391756441569

# Standard G2 generator (zkcrypto/pairing bls12_381, referenced by
# bls_signature.md:34).  Only used to build synthetic test data.
G2_gen_x = (0x024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8,
            0x13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e)
G2_gen_y = (0x0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801,
            0x0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be)

POW_2_381 = 2 ** 381
POW_2_382 = 2 ** 382
POW_2_383 = 2 ** 383

# py_ecc 1.7.0 serialises the int domain big-endian to 8 bytes.
DOMAIN_BYTEORDER = "big"

# ---------------------------------------------------------------------------
# Fq2 = Fq[i]/(i^2 + 1) as (re, im) tuples of ints in [0, q)
# ---------------------------------------------------------------------------
FQ2_ZERO = (0, 0)
FQ2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % q, (a[1] + b[1]) % q)


def f2_sub(a, b):
    return ((a[0] - b[0]) % q, (a[1] - b[1]) % q)


def f2_neg(a):
    return ((-a[0]) % q, (-a[1]) % q)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    return ((a0 * b0 - a1 * b1) % q, (a0 * b1 + a1 * b0) % q)


def f2_muls(a, k):
    return ((a[0] * k) % q, (a[1] * k) % q)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_inv(a):
    a0, a1 = a
    n = (a0 * a0 + a1 * a1) % q
    # py_ecc's prime_field_inv(0) returns 0; keep that convention.
    ni = pow(n, q - 2, q) if n else 0
    return ((a0 * ni) % q, (-a1 * ni) % q)


def f2_div(a, b):
    return f2_mul(a, f2_inv(b))


def f2_pow(a, e):
    result = FQ2_ONE
    base = a
    while e > 0:
        if e & 1:
            result = f2_mul(result, base)
        base = f2_sqr(base)
        e >>= 1
    return result


# ---------------------------------------------------------------------------
# modular_squareroot -- bls_signature.md:89-109, verbatim algorithm
# ---------------------------------------------------------------------------
FQ2_ORDER = q ** 2 - 1
EIGHTH_ROOTS_OF_UNITY = [f2_pow((1, 1), (FQ2_ORDER * k) // 8) for k in range(8)]


def modular_squareroot(value) -> Optional[Tuple[int, int]]:
    """bls_signature.md:99-108 (py_ecc `modular_squareroot_in_FQ2`)."""
    candidate_squareroot = f2_pow(value, (FQ2_ORDER + 8) // 16)
    check = f2_div(f2_sqr(candidate_squareroot), value)
    even_roots = EIGHTH_ROOTS_OF_UNITY[::2]
    if check in even_roots:
        x1 = f2_div(candidate_squareroot,
                    EIGHTH_ROOTS_OF_UNITY[EIGHTH_ROOTS_OF_UNITY.index(check) // 2])
        x2 = f2_neg(x1)
        x1_re, x1_im = x1
        x2_re, x2_im = x2
        return x1 if (x1_im > x2_im or (x1_im == x2_im and x1_re > x2_re)) else x2
    return None


# ---------------------------------------------------------------------------
# Generic homogeneous-projective curve arithmetic, py_ecc optimized_* formulas
# (SURVEY.md Appendix A.3).  A field is given as an ops tuple so the same
# formulas serve G1 (Fq), G2 (Fq2) and the twisted points in Fq12.
# ---------------------------------------------------------------------------
class _FqOps:
    zero = 0
    one = 1

    @staticmethod
    def add(a, b): return (a + b) % q

    @staticmethod
    def sub(a, b): return (a - b) % q

    @staticmethod
    def mul(a, b): return (a * b) % q

    @staticmethod
    def muls(a, k): return (a * k) % q

    @staticmethod
    def neg(a): return (-a) % q

    @staticmethod
    def inv(a): return pow(a, q - 2, q) if a else 0


class _Fq2Ops:
    zero = FQ2_ZERO
    one = FQ2_ONE
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    mul = staticmethod(f2_mul)
    muls = staticmethod(f2_muls)
    neg = staticmethod(f2_neg)
    inv = staticmethod(f2_inv)


def pt_is_inf(F, pt):
    return pt[2] == F.zero


def pt_double(F, pt):
    """py_ecc optimized `double`: W=3x^2, S=yz, B=xyS, H=W^2-8B."""
    x, y, z = pt
    W = F.muls(F.mul(x, x), 3)
    S = F.mul(y, z)
    B = F.mul(F.mul(x, y), S)
    H = F.sub(F.mul(W, W), F.muls(B, 8))
    S_squared = F.mul(S, S)
    newx = F.muls(F.mul(H, S), 2)
    newy = F.sub(F.mul(W, F.sub(F.muls(B, 4), H)),
                 F.muls(F.mul(F.mul(y, y), S_squared), 8))
    newz = F.muls(F.mul(S, S_squared), 8)
    return (newx, newy, newz)


def pt_add(F, p1, p2):
    """py_ecc optimized `add` (homogeneous projective, infinity z == 0)."""
    one, zero = F.one, F.zero
    if p1[2] == zero or p2[2] == zero:
        return p1 if p2[2] == zero else p2
    x1, y1, z1 = p1
    x2, y2, z2 = p2
    U1 = F.mul(y2, z1)
    U2 = F.mul(y1, z2)
    V1 = F.mul(x2, z1)
    V2 = F.mul(x1, z2)
    if V1 == V2 and U1 == U2:
        return pt_double(F, p1)
    elif V1 == V2:
        return (one, one, zero)
    U = F.sub(U1, U2)
    V = F.sub(V1, V2)
    V_squared = F.mul(V, V)
    V_squared_times_V2 = F.mul(V_squared, V2)
    V_cubed = F.mul(V, V_squared)
    W = F.mul(z1, z2)
    A = F.sub(F.sub(F.mul(F.mul(U, U), W), V_cubed), F.muls(V_squared_times_V2, 2))
    newx = F.mul(V, A)
    newy = F.sub(F.mul(U, F.sub(V_squared_times_V2, A)), F.mul(V_cubed, U2))
    newz = F.mul(V_cubed, W)
    return (newx, newy, newz)


def pt_multiply(F, pt, n: int):
    """py_ecc optimized recursive `multiply` (right-to-left), iterative form.

    multiply(pt, n): n == 0 -> inf; n == 1 -> pt; even -> multiply(double(pt), n//2);
    odd -> add(multiply(double(pt), n//2), pt).  Unrolled: the doublings
    P_i = double^i(pt) are taken in increasing i, and the set bits are then
    added from the most significant downward with `add(acc, P_i)`.
    """
    if n == 0:
        return (F.one, F.one, F.zero)
    pts = []
    cur = pt
    m = n
    while m > 1:
        pts.append((m & 1, cur))
        cur = pt_double(F, cur)
        m >>= 1
    acc = cur
    for bit, p in reversed(pts):
        if bit:
            acc = pt_add(F, acc, p)
    return acc


def pt_neg(F, pt):
    x, y, z = pt
    return (x, F.neg(y), z)


def pt_normalize(F, pt):
    x, y, z = pt
    zi = F.inv(z)
    return (F.mul(x, zi), F.mul(y, zi))


def pt_eq(F, p1, p2):
    x1, y1, z1 = p1
    x2, y2, z2 = p2
    return F.mul(x1, z2) == F.mul(x2, z1) and F.mul(y1, z2) == F.mul(y2, z1)


B1 = 4
B2 = (4, 4)


def pt_is_on_curve(F, pt, b):
    if pt_is_inf(F, pt):
        return True
    x, y, z = pt
    lhs = F.sub(F.mul(F.mul(y, y), z), F.mul(F.mul(x, x), x))
    z3 = F.mul(F.mul(z, z), z)
    return lhs == F.mul(b, z3)


G1 = (g_x, g_y, 1)
Z1 = (1, 1, 0)
G2 = (G2_gen_x, G2_gen_y, FQ2_ONE)
Z2 = (FQ2_ONE, FQ2_ONE, FQ2_ZERO)


# ---------------------------------------------------------------------------
# Hash -- SHA-256 (specs/core/0_beacon-chain.md:591-595)
# ---------------------------------------------------------------------------
def sha256(data: bytes) -> bytes:
    return hashlib.sha256(data).digest()


def domain_to_bytes8(domain: int) -> bytes:
    return int(domain).to_bytes(8, DOMAIN_BYTEORDER)


def hash_to_G2_affine_candidate(message_hash: bytes, domain: int):
    """Try-and-increment part of bls_signature.md:74-86 (before the cofactor)."""
    dom8 = domain_to_bytes8(domain)
    x_re = int.from_bytes(sha256(message_hash + dom8 + b"\x01"), "big")
    x_im = int.from_bytes(sha256(message_hash + dom8 + b"\x02"), "big")
    x_coordinate = (x_re % q, x_im % q)
    trials = 0
    while True:
        trials += 1
        y_coordinate_squared = f2_add(f2_mul(f2_sqr(x_coordinate), x_coordinate), B2)
        y_coordinate = modular_squareroot(y_coordinate_squared)
        if y_coordinate is not None:
            return x_coordinate, y_coordinate, trials
        x_coordinate = f2_add(x_coordinate, FQ2_ONE)


def hash_to_G2(message_hash: bytes, domain: int):
    """bls_signature.md:74-87; returns py_ecc's un-normalised projective triple."""
    x, y, _ = hash_to_G2_affine_candidate(message_hash, domain)
    return pt_multiply(_Fq2Ops, (x, y, FQ2_ONE), G2_cofactor)


# ---------------------------------------------------------------------------
# Codecs -- bls_signature.md:36-64 (strict), py_ecc y-selection rules
# ---------------------------------------------------------------------------
def compress_G1(pt) -> int:
    if pt_is_inf(_FqOps, pt):
        return POW_2_383 + POW_2_382
    x, y = pt_normalize(_FqOps, pt)
    a_flag = (y * 2) // q
    return x + a_flag * POW_2_381 + POW_2_383


def decompress_G1(z: int, strict: bool = False):
    """py_ecc 1.7.0 `decompress_G1`; strict=True: the spec's checks
    (bls_signature.md:47-52).  Raises ValueError.  The lax decoder reads bits 381-382 and
    z mod 2^381 only, so any bits from 383 up (c_flag, and those of a pubkey longer than
    48 bytes, which pubkey_to_G1 reads as one big-endian integer) are ignored."""
    if strict and z >= 2 ** 384:
        raise ValueError("G1 encoding longer than 384 bits")
    c_flag = (z >> 383) & 1
    b_flag = (z >> 382) & 1
    a_flag = (z >> 381) & 1
    x = z % POW_2_381
    if strict:
        if c_flag != 1:
            raise ValueError("c_flag must be 1")
        if b_flag == 1 and (a_flag != 0 or x != 0):
            raise ValueError("bad infinity encoding")
        if b_flag == 0 and x >= q:
            raise ValueError("x >= q")
    # py_ecc: b_flag == 1 indicates the infinity point (no other bit is looked at)
    if b_flag == 1:
        return Z1
    # py_ecc: FQ(x) reduces mod q; x**3 + b is taken mod q before the root
    rhs = (x * x * x + B1) % q
    y = pow(rhs, (q + 1) // 4, q)
    if (y * y) % q != rhs:
        raise ValueError("The given point is not on G1: y**2 = x**3 + b")
    if (y * 2) // q != a_flag:
        y = q - y
    return (x % q, y, 1)


def compress_G2(pt) -> Tuple[int, int]:
    if not pt_is_on_curve(_Fq2Ops, pt, B2):
        raise ValueError("The given point is not on the twisted curve over FQ**2")
    if pt_is_inf(_Fq2Ops, pt):
        return (POW_2_383 + POW_2_382, 0)
    (x_re, x_im), (y_re, y_im) = pt_normalize(_Fq2Ops, pt)
    # py_ecc: a_flag1 from y_im, or from y_re when y_im == 0
    a_flag1 = (y_im * 2) // q if y_im > 0 else (y_re * 2) // q
    z1 = x_im + a_flag1 * POW_2_381 + POW_2_383
    z2 = x_re
    return (z1, z2)


def decompress_G2(p: Tuple[int, int], strict: bool = False):
    """py_ecc 1.7.0 `decompress_G2`: x = FQ2([z2, z1 mod 2^381]), both
    reduced mod q (z2 with its top bits, of any length); strict=True: the spec's checks
    (bls_signature.md:58-64).  Raises ValueError."""
    z1, z2 = p
    if strict and (z1 >= 2 ** 384 or z2 >= 2 ** 384):
        raise ValueError("G2 encoding longer than 384 bits")
    c1 = (z1 >> 383) & 1
    b1 = (z1 >> 382) & 1
    a1 = (z1 >> 381) & 1
    x1 = z1 % POW_2_381
    x2 = z2
    if strict:
        if z2 >> 381:
            raise ValueError("flags of z2 must be zero")
        if c1 != 1:
            raise ValueError("c_flag1 must be 1")
        if b1 == 1 and (a1 != 0 or x1 != 0 or x2 != 0):
            raise ValueError("bad infinity encoding")
        if b1 == 0 and (x1 >= q or x2 >= q):
            raise ValueError("x >= q")
    # py_ecc: b_flag1 == 1 indicates the infinity point
    if b1 == 1:
        return Z2
    x = (x2 % q, x1 % q)
    y = modular_squareroot(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise ValueError("Failed to find a modular squareroot")
    y_re, y_im = y
    if (y_im > 0 and (y_im * 2) // q != a1) or (y_im == 0 and (y_re * 2) // q != a1):
        y = f2_neg(y)
    pt = (x, y, FQ2_ONE)
    if not pt_is_on_curve(_Fq2Ops, pt, B2):
        raise ValueError("The given point is not on the twisted curve over FQ**2")
    return pt


def g1_canonical(pubkey) -> bool:
    """True iff the 48-byte encoding has the strict codec's form (c_flag set, x < q,
    infinity only as 0xc0 || 00..); decodability is not part of it."""
    z = int.from_bytes(bytes(pubkey), "big")
    c, b, a, x = z >> 383, (z >> 382) & 1, (z >> 381) & 1, z % POW_2_381
    return c == 1 and ((a == 0 and x == 0) if b else x < q)


def _to_bytes(b) -> bytes:
    return bytes(b)


def pubkey_to_G1(pubkey, strict: bool = False) -> tuple:
    """py_ecc 1.7.0: decompress_G1(big_endian_to_int(pubkey)) for a pubkey of any length
    (b"" is z = 0, the order-3 point (0, 2)); strict: the spec's Bytes48 only."""
    pubkey = _to_bytes(pubkey)
    if strict and len(pubkey) != 48:
        raise ValueError("pubkey must be 48 bytes")
    return decompress_G1(int.from_bytes(pubkey, "big"), strict)


def G1_to_pubkey(pt) -> bytes:
    return compress_G1(pt).to_bytes(48, "big")


def signature_to_G2(signature, strict: bool = False) -> tuple:
    """py_ecc 1.7.0: decompress_G2((big_endian_to_int(signature[:48]),
    big_endian_to_int(signature[48:]))) for a signature of any length; strict: Bytes96 only."""
    signature = _to_bytes(signature)
    if strict and len(signature) != 96:
        raise ValueError("signature must be 96 bytes")
    return decompress_G2((int.from_bytes(signature[:48], "big"),
                          int.from_bytes(signature[48:], "big")), strict)


def G2_to_signature(pt) -> bytes:
    z1, z2 = compress_G2(pt)
    return z1.to_bytes(48, "big") + z2.to_bytes(48, "big")


# ---------------------------------------------------------------------------
# Fq12 = Fq[w]/(w^12 - 2w^6 + 2), py_ecc's representation (Appendix A.9)
# ---------------------------------------------------------------------------
FQ12_ONE = (1,) + (0,) * 11


def f12_mul(a, b):
    t = [0] * 23
    for i in range(12):
        ai = a[i]
        if ai:
            for j in range(12):
                t[i + j] += ai * b[j]
    # reduce with w^12 = 2w^6 - 2
    for k in range(22, 11, -1):
        c = t[k]
        if c:
            t[k - 6] += 2 * c
            t[k - 12] -= 2 * c
    return tuple(v % q for v in t[:12])


def f12_pow(a, e):
    result = FQ12_ONE
    base = a
    while e > 0:
        if e & 1:
            result = f12_mul(result, base)
        base = f12_mul(base, base)
        e >>= 1
    return result


def _poly_deg(p):
    d = len(p) - 1
    while d and p[d] == 0:
        d -= 1
    return d


def f12_inv(a):
    """Extended Euclid over Fq[w] (py_ecc FQP.inv)."""
    lm, hm = [1] + [0] * 12, [0] * 13
    low, high = list(a) + [0], [2, 0, 0, 0, 0, 0, (-2) % q, 0, 0, 0, 0, 0, 1]
    while _poly_deg(low):
        # poly_rounded_div(high, low)
        dega, degb = _poly_deg(high), _poly_deg(low)
        temp = list(high)
        o = [0] * len(high)
        inv_lead = pow(low[degb], q - 2, q)
        for i in range(dega - degb, -1, -1):
            o[i] = (o[i] + temp[degb + i] * inv_lead) % q
            for c in range(degb + 1):
                temp[c + i] = (temp[c + i] - o[i] * low[c]) % q
        rr = o[: _poly_deg(o) + 1] + [0] * (13 - (_poly_deg(o) + 1))
        nm = list(hm)
        new = list(high)
        for i in range(13):
            for j in range(13 - i):
                nm[i + j] = (nm[i + j] - lm[i] * rr[j]) % q
                new[i + j] = (new[i + j] - low[i] * rr[j]) % q
        lm, low, hm, high = nm, new, lm, low
    inv0 = pow(low[0], q - 2, q)
    return tuple((c * inv0) % q for c in lm[:12])


class _Fq12Ops:
    zero = (0,) * 12
    one = FQ12_ONE

    @staticmethod
    def add(a, b): return tuple((x + y) % q for x, y in zip(a, b))

    @staticmethod
    def sub(a, b): return tuple((x - y) % q for x, y in zip(a, b))

    mul = staticmethod(f12_mul)

    @staticmethod
    def muls(a, k): return tuple((x * k) % q for x in a)

    @staticmethod
    def neg(a): return tuple((-x) % q for x in a)

    inv = staticmethod(f12_inv)


def _fq_to_f12(c):
    return (c % q,) + (0,) * 11


def _fq2_to_f12(c):
    # i -> w^6 - 1  (since (w^6 - 1)^2 = -1 under w^12 = 2w^6 - 2)
    re, im = c
    out = [0] * 12
    out[0] = (re - im) % q
    out[6] = im % q
    return tuple(out)


_W = (0, 1) + (0,) * 10
_W_INV = f12_inv(_W)
_W_INV2 = f12_mul(_W_INV, _W_INV)
_W_INV3 = f12_mul(_W_INV2, _W_INV)


def twist(pt):
    """E'(Fq2): y^2 = x^3 + 4(1+i)  ->  E(Fq12): y^2 = x^3 + 4 ; (x,y) -> (x w^-2, y w^-3).

    With i -> w^6 - 1 we have 1 + i -> w^6, so (y w^-3)^2 = x^3 w^-6 + 4.
    """
    x, y, z = pt
    return (f12_mul(_fq2_to_f12(x), _W_INV2), f12_mul(_fq2_to_f12(y), _W_INV3), _fq2_to_f12(z))


def cast_point_to_fq12(pt):
    x, y, z = pt
    return (_fq_to_f12(x), _fq_to_f12(y), _fq_to_f12(z))


ATE_LOOP_COUNT = -BLS_X  # |x|
FINAL_EXP = (q ** 12 - 1) // r


def _linefunc(P1, P2, T):
    """Line through P1, P2 (projective, Fq12) evaluated at T: (num, den)."""
    F = _Fq12Ops
    zero = F.zero
    x1, y1, z1 = P1
    x2, y2, z2 = P2
    xt, yt, zt = T
    m_num = F.sub(F.mul(y2, z1), F.mul(y1, z2))
    m_den = F.sub(F.mul(x2, z1), F.mul(x1, z2))
    if m_den != zero:
        return (F.sub(F.mul(m_num, F.sub(F.mul(xt, z1), F.mul(x1, zt))),
                      F.mul(m_den, F.sub(F.mul(yt, z1), F.mul(y1, zt)))),
                F.mul(F.mul(m_den, zt), z1))
    elif m_num == zero:
        m_num = F.muls(F.mul(x1, x1), 3)
        m_den = F.muls(F.mul(y1, z1), 2)
        return (F.sub(F.mul(m_num, F.sub(F.mul(xt, z1), F.mul(x1, zt))),
                      F.mul(m_den, F.sub(F.mul(yt, z1), F.mul(y1, zt)))),
                F.mul(F.mul(m_den, zt), z1))
    else:
        return (F.sub(F.mul(xt, z1), F.mul(x1, zt)), F.mul(z1, zt))


def miller_loop(Q12, P12):
    """Ate Miller loop f_{|x|,Q}(P) in Fq12 coordinates, num/den form."""
    F = _Fq12Ops
    R = Q12
    f_num, f_den = F.one, F.one
    for i in range(ATE_LOOP_COUNT.bit_length() - 2, -1, -1):
        n, d = _linefunc(R, R, P12)
        f_num = F.mul(F.mul(f_num, f_num), n)
        f_den = F.mul(F.mul(f_den, f_den), d)
        R = pt_double(F, R)
        if (ATE_LOOP_COUNT >> i) & 1:
            n, d = _linefunc(R, Q12, P12)
            f_num = F.mul(f_num, n)
            f_den = F.mul(f_den, d)
            R = pt_add(F, R, Q12)
    return F.mul(f_num, F.inv(f_den))


def final_exponentiate(f):
    return f12_pow(f, FINAL_EXP)


def pairing(Q, P, final_exponentiate_: bool = True):
    """py_ecc `pairing(Q: G2, P: G1)`: asserts on-curve; infinity -> one."""
    assert pt_is_on_curve(_Fq2Ops, Q, B2)
    assert pt_is_on_curve(_FqOps, P, B1)
    if P[2] == 0 or Q[2] == FQ2_ZERO:
        return FQ12_ONE
    f = miller_loop(twist(Q), cast_point_to_fq12(P))
    return final_exponentiate(f) if final_exponentiate_ else f


# ---------------------------------------------------------------------------
# bls API (py_ecc.bls.api; eth2spec/utils/bls.py:24-46)
# ---------------------------------------------------------------------------
class ValidationError(ValueError):
    """py_ecc raises eth_utils.ValidationError; we subclass ValueError."""


def privtopub(k: int) -> bytes:
    return G1_to_pubkey(pt_multiply(_FqOps, G1, k))


def sign(message_hash: bytes, privkey: int, domain: int) -> bytes:
    return G2_to_signature(pt_multiply(_Fq2Ops, hash_to_G2(message_hash, domain), privkey))


def verify(message_hash: bytes, pubkey: bytes, signature: bytes, domain: int) -> bool:
    try:
        final = final_exponentiate(
            f12_mul(
                pairing(signature_to_G2(signature), G1, final_exponentiate_=False),
                pairing(hash_to_G2(message_hash, domain),
                        pt_neg(_FqOps, pubkey_to_G1(pubkey)), final_exponentiate_=False),
            )
        )
        return final == FQ12_ONE
    except (ValidationError, ValueError, AssertionError):
        return False


def verify_multiple(pubkeys: Sequence[bytes], message_hashes: Sequence[bytes],
                    signature: bytes, domain: int) -> bool:
    len_msgs = len(message_hashes)
    if len(pubkeys) != len_msgs:
        raise ValidationError(
            "len(pubkeys) (%s) should be equal to len(message_hashes) (%s)" % (len(pubkeys), len_msgs))
    try:
        o = FQ12_ONE
        msgs = [bytes(m) for m in message_hashes]
        # py_ecc iterates set(message_hashes), whose order is Python's hash order; the
        # product is the same in any order, and only what comes first when a decode fails
        # or the domain is out of range (its groups' pubkeys are decoded before hash_to_G2
        # serialises the domain) depends on it: sorted order here and in the shim
        for m_pubs in sorted(set(msgs)):
            group_pub = Z1
            for i in range(len_msgs):
                if msgs[i] == m_pubs:
                    group_pub = pt_add(_FqOps, group_pub, pubkey_to_G1(pubkeys[i]))
            o = f12_mul(o, pairing(hash_to_G2(m_pubs, domain), group_pub, final_exponentiate_=False))
        o = f12_mul(o, pairing(signature_to_G2(signature), pt_neg(_FqOps, G1), final_exponentiate_=False))
        return final_exponentiate(o) == FQ12_ONE
    except (ValidationError, ValueError, AssertionError):
        return False


def aggregate_signatures(signatures: Sequence[bytes], strict: bool = False) -> bytes:
    o = Z2
    for s in signatures:
        o = pt_add(_Fq2Ops, o, signature_to_G2(s, strict))
    return G2_to_signature(o)


def aggregate_pubkeys(pubkeys: Sequence[bytes], strict: bool = False) -> bytes:
    o = Z1
    for p in pubkeys:
        o = pt_add(_FqOps, o, pubkey_to_G1(p, strict))
    return G1_to_pubkey(o)


# ---------------------------------------------------------------------------
# Spec-strict policy -- NOT py_ecc's behaviour.  bls_signature.md:135-136 and
# :143-144 ask that each pubkey be "a valid G1 point" and the signature "a valid
# G2 point", in the format of :47-52,58-64; py_ecc 1.7.0 decodes laxly and checks
# only that the points lie on the curve.  These give the BLS381_POLICY_STRICT
# columns of tests/golden/*.json.
# ---------------------------------------------------------------------------
def in_G1(pt) -> bool:
    return pt_is_inf(_FqOps, pt_multiply(_FqOps, pt, r))


def in_G2(pt) -> bool:
    return pt_is_inf(_Fq2Ops, pt_multiply(_Fq2Ops, pt, r))


# The spec types domain as uint64 (bls_signature.md:131,139), so under this policy an
# out-of-range domain raises OverflowError before anything is decoded; py_ecc (verify,
# verify_multiple above) serialises it inside hash_to_G2, after the decodes before it.
def verify_strict(message_hash: bytes, pubkey: bytes, signature: bytes, domain: int) -> bool:
    domain_to_bytes8(domain)
    try:
        if not in_G1(pubkey_to_G1(pubkey, True)) or not in_G2(signature_to_G2(signature, True)):
            return False
    except (ValidationError, ValueError, AssertionError):
        return False
    return verify(message_hash, pubkey, signature, domain)


def verify_multiple_strict(pubkeys: Sequence[bytes], message_hashes: Sequence[bytes],
                           signature: bytes, domain: int) -> bool:
    if len(pubkeys) != len(message_hashes):
        raise ValidationError(
            "len(pubkeys) (%s) should be equal to len(message_hashes) (%s)" % (len(pubkeys), len(message_hashes)))
    domain_to_bytes8(domain)
    try:
        if not all(in_G1(pubkey_to_G1(p, True)) for p in pubkeys) or not in_G2(signature_to_G2(signature, True)):
            return False
    except (ValidationError, ValueError, AssertionError):
        return False
    return verify_multiple(pubkeys, message_hashes, signature, domain)


# ---------------------------------------------------------------------------
# Helpers used by fixture generation and tests
# ---------------------------------------------------------------------------
def g2_projective_to_hex(pt) -> List[List[str]]:
    """test_generators/bls/main.py:66-72 output shape: 3 x [re, im] 48-byte hex."""
    return [["0x" + c[0].to_bytes(48, "big").hex(), "0x" + c[1].to_bytes(48, "big").hex()]
            for c in pt]


def g2_affine(pt):
    return pt_normalize(_Fq2Ops, pt)


FqOps = _FqOps
Fq2Ops = _Fq2Ops
Fq12Ops = _Fq12Ops
