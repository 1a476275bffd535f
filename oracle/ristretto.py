"""ristretto255 / curve25519 spec oracle (pure Python big ints) — TEST ONLY.

Restates, from the published specifications, what curve25519-dalek-ng 4.1.1
provides to the reference (not vendored; pinned in bp-perm/Cargo.lock):

  * GF(p), p = 2^255 - 19                       (dalek `field.rs`)
  * Scalar mod l, `from_bytes_mod_order_wide`    (dalek `scalar.rs`)
  * twisted Edwards a = -1 group law, extended coordinates (HWCD'08)
  * ristretto255 encode / decode / Elligator / from_uniform_bytes (RFC 9496)

Reference call sites this backs: `circuit_lib.rs:187,202,216` (MSM),
`circuit_lib.rs:231-233` (compress), `circuit_lib.rs:532` (decompress),
`circuit_lib.rs:180-182,213-214,361-404` (Scalar::random), `weights.rs:58-61`
(PedersenGens::commit).

Pinned by tests/test_oracle_kat.py against RFC 9496 §A.1/§A.3 and an OpenSSL
Ed25519 public-key cross-check.
"""
from __future__ import annotations

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493


def inv(x: int) -> int:
    return pow(x % P, P - 2, P)


D = (-121665 * inv(121666)) % P
SQRT_M1 = 19681161376707505956807079304988542015446066515923890162744021073123829784752
SQRT_AD_MINUS_ONE = 25063068953384623474111414158702152701244531502492656460079210482610430750235
INVSQRT_A_MINUS_D = 54469307008909316920995813868745141605393597292927456921205312896311721017578
ONE_MINUS_D_SQ = 1159843021668779879193775521855586647937357759715417654439879720876111806838
D_MINUS_ONE_SQ = 40440834346308536858101042469323190826248399146238708352240133220865137265952

assert SQRT_M1 * SQRT_M1 % P == P - 1
assert (1 - D * D) % P == ONE_MINUS_D_SQ
assert (D - 1) ** 2 % P == D_MINUS_ONE_SQ


def is_negative(x: int) -> bool:
    return (x % P) & 1 == 1


def ct_abs(x: int) -> int:
    x %= P
    return (-x) % P if is_negative(x) else x


def sqrt_ratio_m1(u: int, v: int):
    """RFC 9496 §4.2 SQRT_RATIO_M1 -> (was_square, r)."""
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = (u * v3) % P * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct_sign = check == u
    flipped_sign = check == (-u) % P
    flipped_sign_i = check == (-u * SQRT_M1) % P
    if flipped_sign or flipped_sign_i:
        r = r * SQRT_M1 % P
    r = ct_abs(r)
    return (correct_sign or flipped_sign), r


# --------------------------------------------------------------------------
# Edwards group, extended coordinates (X:Y:Z:T), x = X/Z, y = Y/Z, T = XY/Z
# --------------------------------------------------------------------------
IDENTITY = (0, 1, 1, 0)
BX = 15112221349535400772501151409588531511454012693041857206046113283949847762202
BY = 46316835694926478169428394003475163141307993866256225615783033603165251855960
BASEPOINT = (BX, BY, 1, BX * BY % P)


def ed_add(p1, p2):
    """Unified HWCD'08 addition (a = -1), complete on this curve."""
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    A = (Y1 - X1) * (Y2 - X2) % P
    B = (Y1 + X1) * (Y2 + X2) % P
    C = T1 * 2 * D % P * T2 % P
    Dd = Z1 * 2 * Z2 % P
    E, F, G, H = B - A, Dd - C, Dd + C, B + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def ed_neg(p1):
    X, Y, Z, T = p1
    return ((-X) % P, Y, Z, (-T) % P)


def ed_double(p1):
    return ed_add(p1, p1)


def ed_mul(k: int, p1):
    """Variable-time double-and-add; k may be any non-negative integer."""
    r = IDENTITY
    q = p1
    while k:
        if k & 1:
            r = ed_add(r, q)
        q = ed_double(q)
        k >>= 1
    return r


def ed_affine(p1):
    X, Y, Z, _ = p1
    zi = inv(Z)
    return X * zi % P, Y * zi % P


def ed_on_curve(p1) -> bool:
    x, y = ed_affine(p1)
    return (-x * x + y * y - 1 - D * x * x % P * y * y) % P == 0


# --------------------------------------------------------------------------
# ristretto255 (RFC 9496 §4.3)
# --------------------------------------------------------------------------
class DecodeError(ValueError):
    pass


def decode(b: bytes):
    if len(b) != 32:
        raise DecodeError("length")
    s = int.from_bytes(b, "little")
    if s >= P or is_negative(s):
        raise DecodeError("non-canonical or negative s")
    ss = s * s % P
    u1 = (1 - ss) % P
    u2 = (1 + ss) % P
    u2_sqr = u2 * u2 % P
    v = (-(D * u1 % P * u1) - u2_sqr) % P
    was_square, invsqrt = sqrt_ratio_m1(1, v * u2_sqr % P)
    den_x = invsqrt * u2 % P
    den_y = invsqrt * den_x % P * v % P
    x = ct_abs(2 * s * den_x)
    y = u1 * den_y % P
    t = x * y % P
    if (not was_square) or is_negative(t) or y == 0:
        raise DecodeError("not a valid encoding")
    return (x, y, 1, t)


def encode(p1) -> bytes:
    x0, y0, z0, t0 = (c % P for c in p1)
    u1 = (z0 + y0) * (z0 - y0) % P
    u2 = x0 * y0 % P
    _, invsqrt = sqrt_ratio_m1(1, u1 * u2 % P * u2 % P)
    den1 = invsqrt * u1 % P
    den2 = invsqrt * u2 % P
    z_inv = den1 * den2 % P * t0 % P
    ix0 = x0 * SQRT_M1 % P
    iy0 = y0 * SQRT_M1 % P
    enchanted = den1 * INVSQRT_A_MINUS_D % P
    rotate = is_negative(t0 * z_inv)
    if rotate:
        x, y, den_inv = iy0, ix0, enchanted
    else:
        x, y, den_inv = x0, y0, den2
    if is_negative(x * z_inv):
        y = (-y) % P
    s = ct_abs(den_inv * (z0 - y))
    return s.to_bytes(32, "little")


def equal(p1, p2) -> bool:
    X1, Y1, _, _ = p1
    X2, Y2, _, _ = p2
    return (X1 * Y2 - Y1 * X2) % P == 0 or (Y1 * Y2 - X1 * X2) % P == 0


def elligator_map(t: int):
    """RFC 9496 §4.3.4 MAP."""
    r = SQRT_M1 * t % P * t % P
    u = (r + 1) * ONE_MINUS_D_SQ % P
    v = (-1 - r * D) * (r + D) % P
    was_square, s = sqrt_ratio_m1(u, v)
    s_prime = (-ct_abs(s * t)) % P
    if not was_square:
        s = s_prime
        c = r
    else:
        c = P - 1
    N = (c * (r - 1) % P * D_MINUS_ONE_SQ - v) % P
    w0 = 2 * s * v % P
    w1 = N * SQRT_AD_MINUS_ONE % P
    w2 = (1 - s * s) % P
    w3 = (1 + s * s) % P
    return (w0 * w3 % P, w2 * w1 % P, w1 * w3 % P, w0 * w2 % P)


def from_uniform_bytes(b: bytes):
    """dalek `RistrettoPoint::from_uniform_bytes` (64 bytes)."""
    assert len(b) == 64
    mask = (1 << 255) - 1
    t1 = int.from_bytes(b[:32], "little") & mask
    t2 = int.from_bytes(b[32:], "little") & mask
    return ed_add(elligator_map(t1 % P), elligator_map(t2 % P))


# --------------------------------------------------------------------------
# Scalars mod l
# --------------------------------------------------------------------------
def scalar_from_wide(b: bytes) -> int:
    assert len(b) == 64
    return int.from_bytes(b, "little") % L


def scalar_bytes(s: int) -> bytes:
    return (s % L).to_bytes(32, "little")


def scalar_from_canonical(b: bytes) -> int:
    s = int.from_bytes(b, "little")
    if s >= L:
        raise ValueError("non-canonical scalar")
    return s


def scalar_inv(s: int) -> int:
    return pow(s % L, L - 2, L)


# --------------------------------------------------------------------------
# Multiscalar multiplication (naive reference semantics of
# `VartimeMultiscalarMul::vartime_multiscalar_mul`)
# --------------------------------------------------------------------------
def msm(scalars, points):
    if len(scalars) != len(points):
        raise ValueError("scalar/point count mismatch")  # dalek panics here
    acc = IDENTITY
    for s, pt in zip(scalars, points):
        acc = ed_add(acc, ed_mul(s % L, pt))
    return acc


def msm_pippenger(scalars, points, w: int = 6):
    """Bucket method with signed radix-2^w digits (dalek Pippenger shape);
    faster than `msm` for a few hundred terms in pure Python."""
    n = len(scalars)
    if n != len(points):
        raise ValueError("scalar/point count mismatch")
    digits = [signed_digits(s % L, w) for s in scalars]
    ndig = len(digits[0]) if n else 0
    total = IDENTITY
    for col in reversed(range(ndig)):
        for _ in range(w):
            total = ed_double(total)
        buckets = [IDENTITY] * (1 << (w - 1))
        for i in range(n):
            dg = digits[i][col]
            if dg > 0:
                buckets[dg - 1] = ed_add(buckets[dg - 1], points[i])
            elif dg < 0:
                buckets[-dg - 1] = ed_add(buckets[-dg - 1], ed_neg(points[i]))
        run = IDENTITY
        s = IDENTITY
        for b in reversed(buckets):
            run = ed_add(run, b)
            s = ed_add(s, run)
        total = ed_add(total, s)
    return total


def signed_digits(s: int, w: int):
    """Signed radix-2^w digits in [-2^(w-1), 2^(w-1)) (last digit may reach
    2^(w-1)); sum d_i 2^(w i) == s."""
    out = []
    carry = 0
    nd = (256 + w - 1) // w
    for i in range(nd):
        v = ((s >> (w * i)) & ((1 << w) - 1)) + carry
        if v >= (1 << (w - 1)) and i != nd - 1:
            out.append(v - (1 << w))
            carry = 1
        else:
            out.append(v)
            carry = 0
    assert sum(dg << (w * i) for i, dg in enumerate(out)) == s
    return out


def msm_window_partial(scalars, points, c: int, W: int, wb: int, we: int):
    """sum_{w in [wb, we)} 2^(c w) sum_i d_{i,w} P_i for the signed radix-2^c
    recoding the GPU engine uses (msm_kernels.cuh for_each_digit: digit
    v >= 2^(c-1) becomes v - 2^c with a carry, except in the last of W
    windows).  Summing the partials of a partition of [0, W) gives the MSM."""
    half = 1 << (c - 1)
    mask = (1 << c) - 1
    acc = IDENTITY
    for s, P in zip(scalars, points):
        carry = 0
        k = 0
        for w in range(we):
            v = ((s >> (c * w)) & mask) + carry
            if v >= half and w + 1 < W:
                d, carry = v - (1 << c), 1
            else:
                d, carry = v, 0
            if w >= wb:
                k += d << (c * w)
        if k:
            acc = ed_add(acc, ed_mul(k, P) if k > 0 else ed_neg(ed_mul(-k, P)))
    return acc


def raw_point_bytes(p) -> bytes:
    """128-byte raw extended form (X, Y, Z, T little-endian) exchanged between
    ranks; the same layout bpp_msm_table_dev_partial emits."""
    return b"".join((c % P).to_bytes(32, "little") for c in p)
