// Edwards25519 group law + ristretto255 encoding for gfx950.
//
// Replaces dalek's EdwardsPoint / RistrettoPoint / CompressedRistretto
// (curve25519-dalek-ng 4.1.1, not vendored) used by the reference at
// circuit_lib.rs:187-233 (MSM + compress), :491 (H*y^-i), :532 (decompress).
//
// Coordinates: extended (X:Y:Z:T), x = X/Z, y = Y/Z, XY = ZT, a = -1.
// Addition is the unified HWCD'08 law, complete on this curve (a square,
// d non-square), so bucket accumulation needs no identity/doubling branches.
#pragma once
#include "fe25519.cuh"

struct ge_p3 {
  fe X, Y, Z, T;
};

// Affine Niels form of a point with Z = 1: (y+x, y-x, 2d*x*y).  96 bytes.
struct ge_niels {
  fe ypx, ymx, xy2d;
};

// Projective Niels form: (Y+X, Y-X, Z, 2d*T).
struct ge_cached {
  fe YpX, YmX, Z, T2d;
};

FE_INLINE ge_p3 ge_identity() {
  ge_p3 r;
  r.X = fe_zero();
  r.Y = fe_one();
  r.Z = fe_one();
  r.T = fe_zero();
  return r;
}

FE_INLINE ge_niels ge_niels_identity() {
  ge_niels n;
  n.ypx = fe_one();
  n.ymx = fe_one();
  n.xy2d = fe_zero();
  return n;
}

// p + q, q affine Niels: 7M.  Sums feeding only multipliers stay
// uncarried (fe_add_nc / fe_sub_nc bounds in fe25519.cuh); F = D - C has a
// non-tight minuend and is carried.  Inputs and outputs are tight.
FE_INLINE ge_p3 ge_madd(const ge_p3& p, const ge_niels& q) {
  fe A = fe_mul(fe_sub_nc(p.Y, p.X), q.ymx);
  fe B = fe_mul(fe_add_nc(p.Y, p.X), q.ypx);
  fe C = fe_mul(p.T, q.xy2d);
  fe D = fe_add_nc(p.Z, p.Z);
  fe E = fe_sub_nc(B, A);
  fe F = fe_sub(D, C);
  fe G = fe_add_nc(D, C);
  fe H = fe_add_nc(B, A);
  ge_p3 r;
  r.X = fe_mul(E, F);
  r.Y = fe_mul(G, H);
  r.Z = fe_mul(G, F);  // F as the second operand in X and Z: its 19x limbs are shared
  r.T = fe_mul(E, H);
  return r;
}

// p - q, q affine Niels (-q = (y-x, y+x, -2dxy)): 7M.
FE_INLINE ge_p3 ge_msub(const ge_p3& p, const ge_niels& q) {
  fe A = fe_mul(fe_sub_nc(p.Y, p.X), q.ypx);
  fe B = fe_mul(fe_add_nc(p.Y, p.X), q.ymx);
  fe C = fe_mul(p.T, q.xy2d);
  fe D = fe_add_nc(p.Z, p.Z);
  fe E = fe_sub_nc(B, A);
  fe F = fe_add_nc(D, C);
  fe G = fe_sub(D, C);
  fe H = fe_add_nc(B, A);
  ge_p3 r;
  r.X = fe_mul(E, F);
  r.Y = fe_mul(G, H);
  r.Z = fe_mul(G, F);  // F as the second operand in X and Z: its 19x limbs are shared
  r.T = fe_mul(E, H);
  return r;
}

// p + q (neg = false) or p - q (neg = true) without divergence: the sign
// only swaps the (y+x, y-x) operands and the two D +- C sums, so a wave
// whose lanes disagree on signs runs one 7M formula instead of both
// ge_madd and ge_msub (or a carried fe_neg of 2dxy).  F, G are each either
// the carried difference or the uncarried sum: both only feed multipliers.
FE_INLINE ge_p3 ge_madd_signed(const ge_p3& p, const ge_niels& q, bool neg) {
  fe qa, qb;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    qa.v[i] = neg ? q.ypx.v[i] : q.ymx.v[i];
    qb.v[i] = neg ? q.ymx.v[i] : q.ypx.v[i];
  }
  fe A = fe_mul(fe_sub_nc(p.Y, p.X), qa);
  fe B = fe_mul(fe_add_nc(p.Y, p.X), qb);
  fe C = fe_mul(p.T, q.xy2d);
  fe D = fe_add_nc(p.Z, p.Z);
  fe E = fe_sub_nc(B, A);
  fe H = fe_add_nc(B, A);
  const fe Dm = fe_sub(D, C), Dp = fe_add_nc(D, C);
  fe F, G;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    F.v[i] = neg ? Dp.v[i] : Dm.v[i];
    G.v[i] = neg ? Dm.v[i] : Dp.v[i];
  }
  ge_p3 r;
  r.X = fe_mul(E, F);
  r.Y = fe_mul(G, H);
  r.Z = fe_mul(G, F);  // F as the second operand in X and Z: its 19x limbs are shared
  r.T = fe_mul(E, H);
  return r;
}

// ge_madd_signed in two halves, so that a caller can issue the loads of its
// next operand between them (the operand is dead after the first half):
// half 1 = the three multiplies that read q, half 2 = the four that do not.
struct ge_madd_mid {
  fe E, F, G, H;
};
FE_INLINE ge_madd_mid ge_madd_signed_h1(const ge_p3& p, const ge_niels& q, bool neg) {
  fe qa, qb;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    qa.v[i] = neg ? q.ypx.v[i] : q.ymx.v[i];
    qb.v[i] = neg ? q.ymx.v[i] : q.ypx.v[i];
  }
  fe A = fe_mul(fe_sub_nc(p.Y, p.X), qa);
  fe B = fe_mul(fe_add_nc(p.Y, p.X), qb);
  fe C = fe_mul(p.T, q.xy2d);
  fe D = fe_add_nc(p.Z, p.Z);
  ge_madd_mid m;
  m.E = fe_sub_nc(B, A);
  m.H = fe_add_nc(B, A);
  const fe Dm = fe_sub(D, C), Dp = fe_add_nc(D, C);
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    m.F.v[i] = neg ? Dp.v[i] : Dm.v[i];
    m.G.v[i] = neg ? Dm.v[i] : Dp.v[i];
  }
  return m;
}
FE_INLINE ge_p3 ge_madd_h2(const ge_madd_mid& m) {
  ge_p3 r;
  r.X = fe_mul(m.E, m.F);
  r.Y = fe_mul(m.G, m.H);
  r.Z = fe_mul(m.G, m.F);  // F second in X and Z: its 19x limbs are shared
  r.T = fe_mul(m.E, m.H);
  return r;
}

FE_INLINE ge_niels ge_niels_neg(const ge_niels& q) {
  ge_niels r;
  r.ypx = q.ymx;
  r.ymx = q.ypx;
  r.xy2d = fe_neg(q.xy2d);
  return r;
}

// YpX / YmX only ever feed multipliers: left uncarried.
FE_INLINE ge_cached ge_to_cached(const ge_p3& p) {
  ge_cached c;
  c.YpX = fe_add_nc(p.Y, p.X);
  c.YmX = fe_sub_nc(p.Y, p.X);
  c.Z = p.Z;
  c.T2d = fe_mul(p.T, fe_const(FE_D2));
  return c;
}

// p + q (q projective Niels): 8M.
FE_INLINE ge_p3 ge_add_cached(const ge_p3& p, const ge_cached& q) {
  fe A = fe_mul(fe_sub_nc(p.Y, p.X), q.YmX);
  fe B = fe_mul(fe_add_nc(p.Y, p.X), q.YpX);
  fe C = fe_mul(p.T, q.T2d);
  fe ZZ = fe_mul(p.Z, q.Z);
  fe D = fe_add_nc(ZZ, ZZ);
  fe E = fe_sub_nc(B, A);
  fe F = fe_sub(D, C);
  fe G = fe_add_nc(D, C);
  fe H = fe_add_nc(B, A);
  ge_p3 r;
  r.X = fe_mul(E, F);
  r.Y = fe_mul(G, H);
  r.Z = fe_mul(G, F);  // F as the second operand in X and Z: its 19x limbs are shared
  r.T = fe_mul(E, H);
  return r;
}

FE_INLINE ge_p3 ge_add(const ge_p3& p, const ge_p3& q) { return ge_add_cached(p, ge_to_cached(q)); }

FE_INLINE ge_p3 ge_neg(const ge_p3& p) {
  ge_p3 r = p;
  r.X = fe_neg(p.X);
  r.T = fe_neg(p.T);
  return r;
}

// 2p: 4M + 4S (dalek ProjectivePoint::double -> CompletedPoint -> extended).
// YY+XX and YY-XX are subtrahends later, so carried; so is cT (its minuend
// ZZ2 is not tight).
FE_INLINE ge_p3 ge_dbl(const ge_p3& p) {
  fe XX = fe_sq(p.X);
  fe YY = fe_sq(p.Y);
  fe ZZ = fe_sq(p.Z);
  fe ZZ2 = fe_add_nc(ZZ, ZZ);
  fe XpY2 = fe_sq(fe_add_nc(p.X, p.Y));
  fe YYpXX = fe_add(YY, XX);
  fe YYmXX = fe_sub(YY, XX);
  fe cX = fe_sub_nc(XpY2, YYpXX);
  fe cT = fe_sub(ZZ2, YYmXX);
  ge_p3 r;
  r.X = fe_mul(cX, cT);
  r.Y = fe_mul(YYpXX, YYmXX);
  r.Z = fe_mul(YYmXX, cT);
  r.T = fe_mul(cX, YYpXX);
  return r;
}

FE_INLINE ge_p3 ge_dbl_n(ge_p3 p, int n) {
  for (int i = 0; i < n; ++i) p = ge_dbl(p);
  return p;
}

// Affine (x, y) -> Niels
FE_INLINE ge_niels ge_niels_from_affine(const fe& x, const fe& y) {
  ge_niels n;
  n.ypx = fe_add(y, x);
  n.ymx = fe_sub(y, x);
  n.xy2d = fe_mul(fe_mul(x, y), fe_const(FE_D2));
  return n;
}

// Extended -> Niels (one field inversion; used once per table entry).
FE_INLINE ge_niels ge_to_niels(const ge_p3& p) {
  fe zi = fe_invert(p.Z);
  return ge_niels_from_affine(fe_mul(p.X, zi), fe_mul(p.Y, zi));
}

FE_INLINE ge_p3 ge_from_niels(const ge_niels& n) {
  // X0 = ypx - ymx = 2x, Y0 = ypx + ymx = 2y.  (2X0 : 2Y0 : 4 : X0*Y0)
  // has x = X0/2, y = Y0/2 and XY = ZT without a halving.
  fe X0 = fe_sub(n.ypx, n.ymx);
  fe Y0 = fe_add(n.ypx, n.ymx);
  ge_p3 r;
  r.T = fe_mul(X0, Y0);
  r.X = fe_add(X0, X0);
  r.Y = fe_add(Y0, Y0);
  r.Z = fe_small(4);
  return r;
}

// Ristretto equality: X1*Y2 == Y1*X2 || Y1*Y2 == X1*X2
FE_INLINE bool ge_ristretto_eq(const ge_p3& a, const ge_p3& b) {
  return fe_eq(fe_mul(a.X, b.Y), fe_mul(a.Y, b.X)) || fe_eq(fe_mul(a.Y, b.Y), fe_mul(a.X, b.X));
}

// ---------------------------------------------------------------- RFC 9496
// SQRT_RATIO_M1(u, v) -> (was_square, r)
FE_INLINE bool fe_sqrt_ratio_m1(const fe& u, const fe& v, fe& r_out) {
  fe v3 = fe_mul(fe_sq(v), v);
  fe v7 = fe_mul(fe_sq(v3), v);
  fe r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  fe check = fe_mul(v, fe_sq(r));
  fe nu = fe_neg(u);
  bool correct = fe_eq(check, u);
  bool flipped = fe_eq(check, nu);
  bool flipped_i = fe_eq(check, fe_mul(nu, fe_const(FE_SQRT_M1)));
  fe r_prime = fe_mul(r, fe_const(FE_SQRT_M1));
  r = fe_select(r, r_prime, flipped || flipped_i);
  r_out = fe_abs(r);
  return correct || flipped;
}

// Decode 32 bytes (as 8 LE words).  Returns false on invalid encoding.
FE_INLINE bool ge_ristretto_decode(const uint32_t w[8], ge_p3& out) {
  // canonical: s < p and s non-negative (even)
  if (!fe_words_canonical(w) || (w[0] & 1)) return false;
  fe s = fe_load_words(w);
  fe ss = fe_sq(s);
  fe u1 = fe_sub(fe_one(), ss);
  fe u2 = fe_add(fe_one(), ss);
  fe u2_sqr = fe_sq(u2);
  fe v = fe_sub(fe_neg(fe_mul(fe_const(FE_D), fe_sq(u1))), u2_sqr);
  fe invsqrt;
  bool was_square = fe_sqrt_ratio_m1(fe_one(), fe_mul(v, u2_sqr), invsqrt);
  fe den_x = fe_mul(invsqrt, u2);
  fe den_y = fe_mul(fe_mul(invsqrt, den_x), v);
  fe x = fe_abs(fe_mul(fe_add(s, s), den_x));
  fe y = fe_mul(u1, den_y);
  fe t = fe_mul(x, y);
  if (!was_square || fe_isneg(t) || fe_iszero(y)) return false;
  out.X = x;
  out.Y = y;
  out.Z = fe_one();
  out.T = t;
  return true;
}

FE_INLINE void ge_ristretto_encode(const ge_p3& p, uint32_t w[8]) {
  fe u1 = fe_mul(fe_add(p.Z, p.Y), fe_sub(p.Z, p.Y));
  fe u2 = fe_mul(p.X, p.Y);
  fe invsqrt;
  (void)fe_sqrt_ratio_m1(fe_one(), fe_mul(u1, fe_sq(u2)), invsqrt);
  fe den1 = fe_mul(invsqrt, u1);
  fe den2 = fe_mul(invsqrt, u2);
  fe z_inv = fe_mul(fe_mul(den1, den2), p.T);
  fe ix0 = fe_mul(p.X, fe_const(FE_SQRT_M1));
  fe iy0 = fe_mul(p.Y, fe_const(FE_SQRT_M1));
  fe enchanted = fe_mul(den1, fe_const(FE_INVSQRT_A_MINUS_D));
  bool rotate = fe_isneg(fe_mul(p.T, z_inv));
  fe x = fe_select(p.X, iy0, rotate);
  fe y = fe_select(p.Y, ix0, rotate);
  fe den_inv = fe_select(den2, enchanted, rotate);
  y = fe_select(y, fe_neg(y), fe_isneg(fe_mul(x, z_inv)));
  fe s = fe_canon(fe_abs(fe_mul(den_inv, fe_sub(p.Z, y))));
  fe_store_words(w, s);
}

// RFC 9496 MAP (Elligator 2 for ristretto)
FE_INLINE ge_p3 ge_elligator(const fe& t) {
  fe one = fe_one();
  fe r = fe_mul(fe_const(FE_SQRT_M1), fe_sq(t));
  fe u = fe_mul(fe_add(r, one), fe_const(FE_ONE_MINUS_D_SQ));
  fe dd = fe_const(FE_D);
  fe v = fe_mul(fe_sub(fe_neg(one), fe_mul(r, dd)), fe_add(r, dd));
  fe s;
  bool was_square = fe_sqrt_ratio_m1(u, v, s);
  fe s_prime = fe_neg(fe_abs(fe_mul(s, t)));
  s = fe_select(s_prime, s, was_square);
  fe c = fe_select(r, fe_neg(one), was_square);
  fe N = fe_sub(fe_mul(fe_mul(c, fe_sub(r, one)), fe_const(FE_D_MINUS_ONE_SQ)), v);
  fe w0 = fe_mul(fe_add(s, s), v);
  fe w1 = fe_mul(N, fe_const(FE_SQRT_AD_MINUS_ONE));
  fe ss = fe_sq(s);
  fe w2 = fe_sub(one, ss);
  fe w3 = fe_add(one, ss);
  ge_p3 P;
  P.X = fe_mul(w0, w3);
  P.Y = fe_mul(w2, w1);
  P.Z = fe_mul(w1, w3);
  P.T = fe_mul(w0, w2);
  return P;
}

// dalek RistrettoPoint::from_uniform_bytes (64 bytes as 16 LE words)
FE_INLINE ge_p3 ge_from_uniform(const uint32_t w[16]) {
  uint32_t a[8], b[8];  // bit 255 of each half is dropped
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    a[i] = w[i];
    b[i] = w[8 + i];
  }
  a[7] &= 0x7fffffffu;
  b[7] &= 0x7fffffffu;
  fe t1 = fe_load_words(a);
  fe t2 = fe_load_words(b);
  return ge_add(ge_elligator(t1), ge_elligator(t2));
}
