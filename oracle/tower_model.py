"""
TEST INFRASTRUCTURE ONLY -- model of OUR device algorithms (not the reference's).

`bls_oracle.py` restates the reference path (py_ecc 1.7.0) and anchors every
parity claim.  This module restates, in plain Python integers, the *different*
algorithms the HIP kernels use -- Fp2/Fp6/Fp12 tower, projective Miller-loop
lines on the M-type twist, the final-exponentiation chain with cyclotomic
squaring, the complex-method Fp2 square root, endomorphism subgroup checks and
windowed scalar multiplication -- so each device layer can be unit-tested
against a transparent model, and the model itself is tested against the oracle
(tests/test_tower_model.py).  Nothing here is shipped or called by the product.

Tower (DESIGN.md "Data layout"):
    Fp2  = Fp[u]/(u^2 + 1)
    Fp6  = Fp2[v]/(v^3 - xi),  xi = 1 + u
    Fp12 = Fp6[w]/(w^2 - v)          (so w^6 = xi)
Fp12 elements are 6-tuples of Fp2 (a0, a1, a2, b0, b1, b2) = a + b w.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bls_oracle as O  # noqa: E402

q = O.q
r = O.r
X_ABS = 0xd201000000010000   # |x|, x < 0

# ------------------------------ Fp2 ---------------------------------------
add2, sub2, mul2, neg2, inv2 = O.f2_add, O.f2_sub, O.f2_mul, O.f2_neg, O.f2_inv
ZERO2, ONE2 = O.FQ2_ZERO, O.FQ2_ONE
XI = (1, 1)


def mul_xi(a):
    # (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
    return ((a[0] - a[1]) % q, (a[0] + a[1]) % q)


def conj2(a):
    return (a[0], (-a[1]) % q)


def frob2(a):
    return conj2(a)


# ------------------------------ Fp6 ---------------------------------------
def add6(a, b): return tuple(add2(x, y) for x, y in zip(a, b))


def sub6(a, b): return tuple(sub2(x, y) for x, y in zip(a, b))


def neg6(a): return tuple(neg2(x) for x in a)


def mul6(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0, t1, t2 = mul2(a0, b0), mul2(a1, b1), mul2(a2, b2)
    c0 = add2(t0, mul_xi(sub2(mul2(add2(a1, a2), add2(b1, b2)), add2(t1, t2))))
    c1 = add2(sub2(mul2(add2(a0, a1), add2(b0, b1)), add2(t0, t1)), mul_xi(t2))
    c2 = add2(sub2(mul2(add2(a0, a2), add2(b0, b2)), add2(t0, t2)), t1)
    return (c0, c1, c2)


def mul6_by_v(a):
    return (mul_xi(a[2]), a[0], a[1])


def inv6(a):
    a0, a1, a2 = a
    c0 = sub2(mul2(a0, a0), mul_xi(mul2(a1, a2)))
    c1 = sub2(mul_xi(mul2(a2, a2)), mul2(a0, a1))
    c2 = sub2(mul2(a1, a1), mul2(a0, a2))
    t = add2(mul2(a0, c0), mul_xi(add2(mul2(a2, c1), mul2(a1, c2))))
    ti = inv2(t)
    return (mul2(c0, ti), mul2(c1, ti), mul2(c2, ti))


ZERO6 = (ZERO2, ZERO2, ZERO2)
ONE6 = (ONE2, ZERO2, ZERO2)


# ------------------------------ Fp12 --------------------------------------
def f12(a, b): return tuple(a) + tuple(b)


def split12(f): return f[:3], f[3:]


ONE12 = f12(ONE6, ZERO6)


def mul12(f, g):
    a, b = split12(f)
    c, d = split12(g)
    ac, bd = mul6(a, c), mul6(b, d)
    e0 = add6(ac, mul6_by_v(bd))
    e1 = sub6(sub6(mul6(add6(a, b), add6(c, d)), ac), bd)
    return f12(e0, e1)


def sqr12(f):
    return mul12(f, f)


def conj12(f):
    a, b = split12(f)
    return f12(a, neg6(b))


def inv12(f):
    a, b = split12(f)
    t = sub6(mul6(a, a), mul6_by_v(mul6(b, b)))
    ti = inv6(t)
    return f12(mul6(a, ti), neg6(mul6(b, ti)))


def pow12(f, e):
    res = ONE12
    while e:
        if e & 1:
            res = mul12(res, f)
        f = sqr12(f)
        e >>= 1
    return res


# Frobenius: (sum c_k w^k)^q = sum conj(c_k) w^{kq} = sum conj(c_k) * gamma_k w^k,
# gamma_k = w^{k(q-1)} = xi^{k(q-1)/6}.  Power p: gamma_{p,k} = xi^{k(q^p-1)/6}
def _f2pow(a, e): return O.f2_pow(a, e)


FROB_GAMMA = {p: [_f2pow(XI, k * (q ** p - 1) // 6) for k in range(6)] for p in (1, 2, 3)}
# w-power order of (a0,a1,a2,b0,b1,b2): a_j -> w^{2j}, b_j -> w^{2j+1}
_WPOW = [0, 2, 4, 1, 3, 5]


def frob12(f, p=1):
    out = []
    for idx, c in enumerate(f):
        k = _WPOW[idx]
        cc = c if p % 2 == 0 else conj2(c)
        out.append(mul2(cc, FROB_GAMMA[p][k]))
    return tuple(out)


# -------------------------- map to py_ecc Fq12 -----------------------------
def to_pyecc12(f):
    """Our tower -> py_ecc's Fq[w]/(w^12-2w^6+2): the same w, u -> w^6 - 1."""
    out = [0] * 12
    for idx, c in enumerate(f):
        k = _WPOW[idx]
        re, im = c
        out[k] = (out[k] + re - im) % q
        out[k + 6] = (out[k + 6] + im) % q
    return tuple(out)


# --------------------------- cyclotomic ops --------------------------------
def cyclotomic_sqr(f):
    """Granger-Scott squaring for f with f^(q^6+1)... (cyclotomic subgroup).

    View Fp12 = Fp4[w]/(w^3 - z), Fp4 = Fp2[z]/(z^2 - xi), z = w^3.
    f = A + B w + C w^2 with A = a0 + b1 z, B = b0 + a2 z, C = a1 + b2 z.
    """
    a0, a1, a2, b0, b1, b2 = f

    def sq4(x0, x1):
        # (x0 + x1 z)^2 = x0^2 + xi x1^2 + 2 x0 x1 z
        t0 = mul2(x0, x0)
        t1 = mul2(x1, x1)
        return add2(t0, mul_xi(t1)), mul2(add2(x0, x0), x1)

    A0, A1 = sq4(a0, b1)
    B0, B1 = sq4(b0, a2)
    C0, C1 = sq4(a1, b2)
    # A' = 3A^2 - 2 conj(A); conj(A) = a0 - b1 z
    na0 = sub2(O.f2_muls(A0, 3), O.f2_muls(a0, 2))
    nb1 = add2(O.f2_muls(A1, 3), O.f2_muls(b1, 2))
    # B' = 3 z C^2 + 2 conj(B);  z*(C0 + C1 z) = xi C1 + C0 z
    zc0, zc1 = mul_xi(C1), C0
    nb0 = add2(O.f2_muls(zc0, 3), O.f2_muls(b0, 2))
    na2 = sub2(O.f2_muls(zc1, 3), O.f2_muls(a2, 2))
    # C' = 3 B^2 - 2 conj(C)
    na1 = sub2(O.f2_muls(B0, 3), O.f2_muls(a1, 2))
    nb2 = add2(O.f2_muls(B1, 3), O.f2_muls(b2, 2))
    return (na0, na1, na2, nb0, nb1, nb2)


def cyc_exp_abs_x(f):
    """f^|x| by square-and-multiply over |x| = 0xd201000000010000."""
    res = f
    for i in range(X_ABS.bit_length() - 2, -1, -1):
        res = cyclotomic_sqr(res)
        if (X_ABS >> i) & 1:
            res = mul12(res, f)
    return res


def cyc_exp_x(f):
    return conj12(cyc_exp_abs_x(f))   # x < 0


# Karabina compressed squaring (bls381_pairing.hpp cyc_csqr / cyc_decompress / cyc_exp_x):
# (g2, g3, g4, g5) = (b0, a2, a1, b2) squares on its own; (a0, b1) comes back from
# the norm condition.
def cyc_compress(f):
    a0, a1, a2, b0, b1, b2 = f
    return (b0, a2, a1, b2)


def cyc_csqr(g):
    g2, g3, g4, g5 = g
    t0, t1, t2 = mul2(g4, g4), mul2(g5, g5), mul2(add2(g4, g5), add2(g4, g5))
    t3, t4, t5 = mul2(g2, g2), mul2(g3, g3), mul2(add2(g2, g3), add2(g2, g3))
    m = O.f2_muls
    return (add2(m(mul_xi(sub2(sub2(t2, t0), t1)), 3), m(g2, 2)),
            sub2(m(add2(t0, mul_xi(t1)), 3), m(g3, 2)),
            sub2(m(add2(t3, mul_xi(t4)), 3), m(g4, 2)),
            add2(m(sub2(sub2(t5, t3), t4), 3), m(g5, 2)))


def cyc_decompress(g):
    g2, g3, g4, g5 = g
    m = O.f2_muls
    num = sub2(add2(mul_xi(mul2(g5, g5)), m(mul2(g4, g4), 3)), m(g3, 2))
    b1 = mul2(num, inv2(m(g2, 4)))
    a0 = add2(mul_xi(sub2(add2(m(mul2(b1, b1), 2), mul2(g2, g5)), m(mul2(g3, g4), 3))), ONE2)
    return (a0, g4, g3, g2, b1, g5)


def cyc_exp_abs_x_compressed(f):
    """f^|x| right to left: 63 compressed squarings, the six set bits' snapshots
    decompressed and multiplied.  Requires every snapshot's g2 != 0."""
    g = cyc_compress(f)
    res = None
    for run in (16, 32, 9, 3, 2, 1):
        for _ in range(run):
            g = cyc_csqr(g)
        x = cyc_decompress(g)
        res = x if res is None else mul12(res, x)
    return res


def final_exp(f):
    """Returns f^(3 (q^12-1)/r).  The factor 3 is coprime to r, so
    final_exp(f) == 1  <=>  f^((q^12-1)/r) == 1 (DESIGN.md "Final exponentiation").

    Hard part: 3 (q^4 - q^2 + 1)/r = (x-1)^2 (x+q) (x^2+q^2-1) + 3.
    """
    t = mul12(conj12(f), inv12(f))          # f^(q^6-1)
    t = mul12(frob12(t, 2), t)              # ^(q^2+1)
    a = mul12(cyc_exp_x(t), conj12(t))      # t^(x-1)
    a = mul12(cyc_exp_x(a), conj12(a))      # t^((x-1)^2)
    b = mul12(cyc_exp_x(a), frob12(a, 1))   # a^(x+q)
    c = mul12(mul12(cyc_exp_x(cyc_exp_x(b)), frob12(b, 2)), conj12(b))  # b^(x^2+q^2-1)
    t3 = mul12(cyclotomic_sqr(t), t)
    return mul12(c, t3)


# ----------------------------- curves --------------------------------------
B_G1 = 4
B_G2 = (4, 4)


class Fq:
    add = staticmethod(lambda a, b: (a + b) % q)
    sub = staticmethod(lambda a, b: (a - b) % q)
    mul = staticmethod(lambda a, b: (a * b) % q)
    neg = staticmethod(lambda a: (-a) % q)
    inv = staticmethod(lambda a: pow(a, q - 2, q))
    zero, one = 0, 1
    muls = staticmethod(lambda a, k: (a * k) % q)


class Fq2:
    add, sub, mul, neg, inv = add2, sub2, mul2, neg2, inv2
    zero, one = ZERO2, ONE2
    muls = staticmethod(O.f2_muls)


# Jacobian coordinates (X/Z^2, Y/Z^3), a = 0
def jac_dbl(F, p):
    X, Y, Z = p
    if Z == F.zero:
        return p
    A = F.mul(X, X)
    B = F.mul(Y, Y)
    C = F.mul(B, B)
    D = F.muls(F.sub(F.sub(F.mul(F.add(X, B), F.add(X, B)), A), C), 2)
    E = F.muls(A, 3)
    Fv = F.mul(E, E)
    X3 = F.sub(Fv, F.muls(D, 2))
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), F.muls(C, 8))
    Z3 = F.muls(F.mul(Y, Z), 2)
    return (X3, Y3, Z3)


def jac_add(F, p1, p2):
    X1, Y1, Z1 = p1
    X2, Y2, Z2 = p2
    if Z1 == F.zero:
        return p2
    if Z2 == F.zero:
        return p1
    Z1Z1 = F.mul(Z1, Z1)
    Z2Z2 = F.mul(Z2, Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
    S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
    H = F.sub(U2, U1)
    Rr = F.sub(S2, S1)
    if H == F.zero:
        if Rr == F.zero:
            return jac_dbl(F, p1)
        return (F.one, F.one, F.zero)
    HH = F.mul(H, H)
    HHH = F.mul(H, HH)
    V = F.mul(U1, HH)
    X3 = F.sub(F.sub(F.mul(Rr, Rr), HHH), F.muls(V, 2))
    Y3 = F.sub(F.mul(Rr, F.sub(V, X3)), F.mul(S1, HHH))
    Z3 = F.mul(F.mul(Z1, Z2), H)
    return (X3, Y3, Z3)


def jac_neg(F, p):
    return (p[0], F.neg(p[1]), p[2])


def jac_to_affine(F, p):
    X, Y, Z = p
    if Z == F.zero:
        return None
    zi = F.inv(Z)
    zi2 = F.mul(zi, zi)
    return (F.mul(X, zi2), F.mul(F.mul(Y, zi2), zi))


def jac_mul(F, p, n):
    res = (F.one, F.one, F.zero)
    for i in range(n.bit_length() - 1, -1, -1):
        res = jac_dbl(F, res)
        if (n >> i) & 1:
            res = jac_add(F, res, p)
    return res


def wnaf(n, w):
    digits = []
    while n > 0:
        if n & 1:
            d = n % (1 << w)
            if d >= 1 << (w - 1):
                d -= 1 << w
            n -= d
        else:
            d = 0
        digits.append(d)
        n >>= 1
    return digits  # little-endian


def jac_mul_wnaf(F, p, n, w=5):
    table = [p]
    p2 = jac_dbl(F, p)
    for _ in range((1 << (w - 2)) - 1):
        table.append(jac_add(F, table[-1], p2))
    res = (F.one, F.one, F.zero)
    for d in reversed(wnaf(n, w)):
        res = jac_dbl(F, res)
        if d > 0:
            res = jac_add(F, res, table[d >> 1])
        elif d < 0:
            res = jac_add(F, res, jac_neg(F, table[(-d) >> 1]))
    return res


# ----------------------- endomorphisms / subgroup --------------------------
# psi on E'(Fp2): untwist -> Frobenius -> twist.  psi(x, y) = (cx * conj(x), cy * conj(y))
PSI_CX = O.f2_inv(O.f2_pow(XI, (q - 1) // 3))
PSI_CY = O.f2_inv(O.f2_pow(XI, (q - 1) // 2))


def psi_affine(pt):
    x, y = pt
    return (mul2(PSI_CX, conj2(x)), mul2(PSI_CY, conj2(y)))


def psi_jac(p):
    X, Y, Z = p
    return (mul2(PSI_CX, conj2(X)), mul2(PSI_CY, conj2(Y)), conj2(Z))


def g2_in_subgroup(p):
    """psi(Q) == [x] Q  (x < 0): psi(Q) + [|x|] Q == O."""
    t = jac_mul(Fq2, p, X_ABS)
    s = jac_add(Fq2, t, psi_jac(p))
    return s[2] == ZERO2


# G1 endomorphism sigma(x, y) = (beta x, y), beta a cube root of unity chosen so
# that sigma acts on G1 as multiplication by -x^2 (mod r).
def _find_beta():
    g = (O.g_x, O.g_y, 1)
    lam = (-(X_ABS ** 2)) % r
    target = jac_to_affine(Fq, jac_mul(Fq, g, lam))
    c = pow(2, (q - 1) // 3, q)
    for beta in (c, (c * c) % q):
        if ((beta * O.g_x) % q, O.g_y) == target:
            return beta
    raise AssertionError("no beta")


BETA = _find_beta()


def g1_in_subgroup(p):
    """sigma(P) == [-x^2] P  <=>  sigma(P) + [x^2] P == O."""
    X, Y, Z = p
    t = jac_mul(Fq, jac_mul(Fq, p, X_ABS), X_ABS)
    s = jac_add(Fq, t, ((BETA * X) % q, Y, Z))
    return s[2] == 0


# ------------------------------- sqrt --------------------------------------
def sqrt_fp(a):
    s = pow(a, (q + 1) // 4, q)
    return s if (s * s) % q == a % q else None


def sqrt_fp2(a):
    """Complex-method square root (q = 3 mod 4).  Returns some root or None."""
    a0, a1 = a
    if a1 == 0:
        s = sqrt_fp(a0)
        if s is not None:
            return (s, 0)
        s = sqrt_fp((-a0) % q)
        return (0, s)  # -a0 is a QR when a0 is not (and a0 != 0)
    alpha = (a0 * a0 + a1 * a1) % q
    gamma = pow(alpha, (q + 1) // 4, q)
    if (gamma * gamma) % q != alpha:
        return None
    delta = ((a0 + gamma) * pow(2, q - 2, q)) % q
    t = pow(delta, (q + 1) // 4, q)
    inv2t = pow((2 * t) % q, q - 2, q)
    if (t * t) % q == delta:
        return (t, (a1 * inv2t) % q)
    # t^2 == -delta
    return ((a1 * inv2t) % q, t)


def choose_root(y):
    """bls_signature.md:91: prefer larger imaginary part, then larger real part."""
    ny = neg2(y)
    if y[1] > ny[1] or (y[1] == ny[1] and y[0] > ny[0]):
        return y
    return ny


def map_candidate(message_hash, dom8: bytes):
    x_re = int.from_bytes(O.sha256(message_hash + dom8 + b"\x01"), "big") % q
    x_im = int.from_bytes(O.sha256(message_hash + dom8 + b"\x02"), "big") % q
    x = (x_re, x_im)
    while True:
        rhs = add2(mul2(mul2(x, x), x), B_G2)
        y = sqrt_fp2(rhs)
        if y is not None:
            return x, choose_root(y)
        x = add2(x, ONE2)


def g2_bp(P):
    """Budroni-Pintore BP(P) = [x^2-x-1]P + [x-1]psi(P) + psi^2(2P) = [3(x^2-1) h2]P
    (device g2_mul_bp: the verification hash of the verify kernels)."""
    X = X_ABS
    F = Fq2
    neg = lambda p: jac_neg(F, p)
    add = lambda a, b: jac_add(F, a, b)
    t1 = jac_mul(F, P, X)
    Q0 = add(add(add(jac_mul(F, t1, X), t1), neg(P)), psi_jac(add(neg(t1), neg(P))))
    return add(Q0, psi_jac(psi_jac(jac_dbl(F, P))))


def clear_cofactor_h2(P):
    """[h2]P exactly, via [c^-1 mod r] BP(P) with c = 3(x^2-1) (device g2_mul_cofactor)."""
    e0 = (X_ABS + 1) // 3
    F = Fq2
    neg = lambda p: jac_neg(F, p)
    add = lambda a, b: jac_add(F, a, b)
    Q0 = g2_bp(P)
    Q1 = neg(psi_jac(Q0))
    Q2 = neg(psi_jac(Q1))
    T = add(add(jac_dbl(F, Q2), Q1), neg(psi_jac(Q2)))
    S = add(add(T, Q1), Q0)
    return add(jac_mul(F, S, e0), neg(T))


def hash_to_g2_affine(message_hash, dom8):
    x, y = map_candidate(message_hash, dom8)
    return jac_to_affine(Fq2, clear_cofactor_h2((x, y, ONE2)))


# ----------------------------- Miller loop ---------------------------------
def line_dbl(T, P):
    """Tangent at T (homogeneous projective on E'), evaluated at P=(xp,yp) in E(Fp).

    Returns (new T, sparse line (c0, c1, c2)) meaning c0 + c1 v + c2 v w.
    Line scaled by Fp2 factors (killed by the final exponentiation):
        c0 = Y^2 - 3 b' Z^2,  c1 = -3 X^2 xp,  c2 = 2 Y Z yp
    Doubling (a = 0): X3 = XY/2 (Y^2 - 9b'Z^2), Y3 = ((Y^2 + 9b'Z^2)/2)^2 - 27 b'^2 Z^4,
    Z3 = 2 Y^3 Z.
    """
    X, Y, Z = T
    xp, yp = P
    b = B_G2
    XX, YY, ZZ = mul2(X, X), mul2(Y, Y), mul2(Z, Z)
    bZZ = mul2(b, ZZ)
    c0 = sub2(YY, O.f2_muls(bZZ, 3))
    c1 = O.f2_muls(XX, (-3 * xp) % q)
    c2 = O.f2_muls(mul2(Y, Z), (2 * yp) % q)
    inv2_ = pow(2, q - 2, q)
    b9 = O.f2_muls(bZZ, 9)
    X3 = O.f2_muls(mul2(mul2(X, Y), sub2(YY, b9)), inv2_)
    h = O.f2_muls(add2(YY, b9), inv2_)
    Y3 = sub2(mul2(h, h), O.f2_muls(mul2(bZZ, bZZ), 27))
    Z3 = O.f2_muls(mul2(mul2(YY, Y), Z), 2)
    return (X3, Y3, Z3), (c0, c1, c2)


def line_add(T, Qa, P):
    """T + Q (Q affine) and the line through them evaluated at P."""
    X, Y, Z = T
    xq, yq = Qa
    xp, yp = P
    u = sub2(mul2(yq, Z), Y)
    v = sub2(mul2(xq, Z), X)
    c0 = sub2(mul2(u, xq), mul2(v, yq))
    c1 = O.f2_muls(u, (-xp) % q)
    c2 = O.f2_muls(v, yp)
    vv = mul2(v, v)
    vvv = mul2(vv, v)
    vvX = mul2(vv, X)
    A = sub2(sub2(mul2(mul2(u, u), Z), vvv), O.f2_muls(vvX, 2))
    X3 = mul2(v, A)
    Y3 = sub2(mul2(u, sub2(vvX, A)), mul2(vvv, Y))
    Z3 = mul2(vvv, Z)
    return (X3, Y3, Z3), (c0, c1, c2)


def mul_by_line(f, line):
    c0, c1, c2 = line
    return mul12(f, (c0, c1, ZERO2, ZERO2, c2, ZERO2))


def miller_loop_multi(pairs):
    """pairs: list of (Q affine on E'(Fp2), P affine on E(Fp)); returns f (conjugated for x<0)."""
    f = ONE12
    Ts = [(Qa[0], Qa[1], ONE2) for Qa, _ in pairs]
    for i in range(X_ABS.bit_length() - 2, -1, -1):
        f = sqr12(f)
        for k, (Qa, P) in enumerate(pairs):
            Ts[k], l = line_dbl(Ts[k], P)
            f = mul_by_line(f, l)
        if (X_ABS >> i) & 1:
            for k, (Qa, P) in enumerate(pairs):
                Ts[k], l = line_add(Ts[k], Qa, P)
                f = mul_by_line(f, l)
    return conj12(f)


def pairing(Qa, Pa):
    return final_exp(miller_loop_multi([(Qa, Pa)]))
