// Host-side GF(2^255-19) / Edwards / ristretto255 (radix 2^51, 5 limbs).
//
// Product code, not the oracle: finishes what the GPU hands back (the
// Horner combine of a large MSM's W window sums, compression of a single
// result point, proof-level point equality) where a lone GPU lane would be
// latency-bound.  Independent of the device's 10 x 32-bit representation
// and of the oracle's C port.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

namespace h25519 {

typedef unsigned __int128 u128;

// radix 2^51, five limbs; every function returns "carried" limbs
// (< 2^51 + 2^18), which is what fe_mul / fe_sub accept.
struct fe {
  uint64_t v[5];
};

static const uint64_t FE_M51 = (1ULL << 51) - 1;

static inline fe fe_zero() { return fe{{0, 0, 0, 0, 0}}; }
static inline fe fe_one() { return fe{{1, 0, 0, 0, 0}}; }

static inline fe fe_carry(fe a) {
  uint64_t c;
  c = a.v[0] >> 51; a.v[0] &= FE_M51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= FE_M51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= FE_M51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= FE_M51; a.v[4] += c;
  c = a.v[4] >> 51; a.v[4] &= FE_M51; a.v[0] += 19 * c;
  return a;
}

static inline fe fe_add(const fe& a, const fe& b) {
  fe r;
  for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + b.v[i];
  return fe_carry(r);
}

// a + 4p - b (4p limbs exceed any carried limb)
static inline fe fe_sub(const fe& a, const fe& b) {
  fe r;
  r.v[0] = a.v[0] + 0x1fffffffffffb4ULL - b.v[0];
  for (int i = 1; i < 5; ++i) r.v[i] = a.v[i] + 0x1ffffffffffffcULL - b.v[i];
  return fe_carry(r);
}

static inline fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

static inline fe fe_reduce128(u128 t0, u128 t1, u128 t2, u128 t3, u128 t4) {
  fe r;
  t1 += (uint64_t)(t0 >> 51); r.v[0] = (uint64_t)t0 & FE_M51;
  t2 += (uint64_t)(t1 >> 51); r.v[1] = (uint64_t)t1 & FE_M51;
  t3 += (uint64_t)(t2 >> 51); r.v[2] = (uint64_t)t2 & FE_M51;
  t4 += (uint64_t)(t3 >> 51); r.v[3] = (uint64_t)t3 & FE_M51;
  const uint64_t c = (uint64_t)(t4 >> 51);
  r.v[4] = (uint64_t)t4 & FE_M51;
  r.v[0] += 19 * c;
  r.v[1] += r.v[0] >> 51;
  r.v[0] &= FE_M51;
  return r;
}

static inline fe fe_mul(const fe& a, const fe& b) {
  const uint64_t b1 = 19 * b.v[1], b2 = 19 * b.v[2], b3 = 19 * b.v[3], b4 = 19 * b.v[4];
  const u128 t0 = (u128)a.v[0] * b.v[0] + (u128)a.v[1] * b4 + (u128)a.v[2] * b3 + (u128)a.v[3] * b2 +
                  (u128)a.v[4] * b1;
  const u128 t1 = (u128)a.v[0] * b.v[1] + (u128)a.v[1] * b.v[0] + (u128)a.v[2] * b4 + (u128)a.v[3] * b3 +
                  (u128)a.v[4] * b2;
  const u128 t2 = (u128)a.v[0] * b.v[2] + (u128)a.v[1] * b.v[1] + (u128)a.v[2] * b.v[0] + (u128)a.v[3] * b4 +
                  (u128)a.v[4] * b3;
  const u128 t3 = (u128)a.v[0] * b.v[3] + (u128)a.v[1] * b.v[2] + (u128)a.v[2] * b.v[1] + (u128)a.v[3] * b.v[0] +
                  (u128)a.v[4] * b4;
  const u128 t4 = (u128)a.v[0] * b.v[4] + (u128)a.v[1] * b.v[3] + (u128)a.v[2] * b.v[2] + (u128)a.v[3] * b.v[1] +
                  (u128)a.v[4] * b.v[0];
  return fe_reduce128(t0, t1, t2, t3, t4);
}

static inline fe fe_sq(const fe& a) {
  const uint64_t d0 = 2 * a.v[0], d1 = 2 * a.v[1], d3_19 = 38 * a.v[3], a3_19 = 19 * a.v[3], a4_19 = 19 * a.v[4];
  const u128 t0 = (u128)a.v[0] * a.v[0] + (u128)d1 * a4_19 + (u128)(2 * a.v[2]) * a3_19;
  const u128 t1 = (u128)d0 * a.v[1] + (u128)(2 * a.v[2]) * a4_19 + (u128)a.v[3] * a3_19;
  const u128 t2 = (u128)d0 * a.v[2] + (u128)a.v[1] * a.v[1] + (u128)d3_19 * a.v[4];
  const u128 t3 = (u128)d0 * a.v[3] + (u128)d1 * a.v[2] + (u128)a.v[4] * a4_19;
  const u128 t4 = (u128)d0 * a.v[4] + (u128)d1 * a.v[3] + (u128)a.v[2] * a.v[2];
  return fe_reduce128(t0, t1, t2, t3, t4);
}

static inline fe fe_sqn(fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

// canonical little-endian 256-bit value (< p) of a (limbs < 2^53)
static inline void fe_to_u256(uint64_t w[4], const fe& a) {
  u128 acc = (u128)a.v[0] + ((u128)a.v[1] << 51);
  w[0] = (uint64_t)acc;
  acc >>= 64;
  acc += (u128)a.v[2] << 38;
  w[1] = (uint64_t)acc;
  acc >>= 64;
  acc += (u128)a.v[3] << 25;
  w[2] = (uint64_t)acc;
  acc >>= 64;
  acc += (u128)a.v[4] << 12;
  w[3] = (uint64_t)acc;
  uint64_t top = (uint64_t)(acc >> 64);
  for (int pass = 0; pass < 2; ++pass) {  // fold bits >= 255 (2^255 = 19)
    const uint64_t hi = (top << 1) | (w[3] >> 63);
    w[3] &= 0x7fffffffffffffffULL;
    u128 c = (u128)w[0] + (u128)hi * 19u;
    w[0] = (uint64_t)c;
    for (int i = 1; i < 4; ++i) {
      c = (u128)w[i] + (uint64_t)(c >> 64);
      w[i] = (uint64_t)c;
    }
    top = 0;
  }
  // now < 2^255; subtract p when value + 19 >= 2^255
  uint64_t t[4];
  u128 c = (u128)w[0] + 19u;
  t[0] = (uint64_t)c;
  for (int i = 1; i < 4; ++i) {
    c = (u128)w[i] + (uint64_t)(c >> 64);
    t[i] = (uint64_t)c;
  }
  if (t[3] >> 63) {
    t[3] &= 0x7fffffffffffffffULL;
    for (int i = 0; i < 4; ++i) w[i] = t[i];
  }
}

static inline fe fe_from_u256(const uint64_t w[4], uint64_t top);
// fully reduced: limbs < 2^51 and value < p
static inline fe fe_canon(const fe& a) {
  uint64_t w[4];
  fe_to_u256(w, a);
  return fe_from_u256(w, 0);
}

static inline bool fe_iszero(const fe& a) {
  fe c = fe_canon(a);
  return (c.v[0] | c.v[1] | c.v[2] | c.v[3] | c.v[4]) == 0;
}
static inline bool fe_eq(const fe& a, const fe& b) { return fe_iszero(fe_sub(a, b)); }
static inline bool fe_isneg(const fe& a) { return fe_canon(a).v[0] & 1; }
static inline fe fe_abs(const fe& a) { return fe_isneg(a) ? fe_neg(a) : a; }

static inline void fe_pow_core(const fe& z, fe& z_250_0, fe& z11) {
  fe z2 = fe_sq(z);
  fe z9 = fe_mul(z, fe_sqn(z2, 2));
  z11 = fe_mul(z2, z9);
  fe z_5_0 = fe_mul(z9, fe_sq(z11));
  fe z_10_0 = fe_mul(fe_sqn(z_5_0, 5), z_5_0);
  fe z_20_0 = fe_mul(fe_sqn(z_10_0, 10), z_10_0);
  fe z_40_0 = fe_mul(fe_sqn(z_20_0, 20), z_20_0);
  fe z_50_0 = fe_mul(fe_sqn(z_40_0, 10), z_10_0);
  fe z_100_0 = fe_mul(fe_sqn(z_50_0, 50), z_50_0);
  fe z_200_0 = fe_mul(fe_sqn(z_100_0, 100), z_100_0);
  z_250_0 = fe_mul(fe_sqn(z_200_0, 50), z_50_0);
}
static inline fe fe_invert(const fe& z) {
  fe a, z11;
  fe_pow_core(z, a, z11);
  return fe_mul(fe_sqn(a, 5), z11);
}
static inline fe fe_pow22523(const fe& z) {
  fe a, z11;
  fe_pow_core(z, a, z11);
  return fe_mul(fe_sqn(a, 2), z);
}

// 256-bit little-endian value (+ top * 2^256), reduced mod p on the way in
static inline fe fe_from_u256(const uint64_t w[4], uint64_t top) {
  fe r;
  r.v[0] = w[0] & FE_M51;
  r.v[1] = ((w[0] >> 51) | (w[1] << 13)) & FE_M51;
  r.v[2] = ((w[1] >> 38) | (w[2] << 26)) & FE_M51;
  r.v[3] = ((w[2] >> 25) | (w[3] << 39)) & FE_M51;
  r.v[4] = (w[3] >> 12) & FE_M51;
  // bit 255 and top * 2^256 (2^255 = 19, 2^256 = 38 mod p)
  r.v[0] += 19 * (w[3] >> 63) + 38 * top;
  return fe_carry(r);
}
static inline fe fe_from_bytes(const uint8_t b[32]) {
  uint64_t w[4];
  memcpy(w, b, 32);  // little-endian host
  return fe_from_u256(w, 0);
}
static inline void fe_to_bytes(uint8_t b[32], const fe& a) {
  uint64_t w[4];
  fe_to_u256(w, a);
  memcpy(b, w, 32);
}
static inline fe fe_from_words(const uint32_t w[8]) {
  uint64_t q[4];
  for (int i = 0; i < 4; ++i) q[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  return fe_from_u256(q, 0);
}
static inline void fe_to_words(uint32_t w[8], const fe& a) {
  uint64_t q[4];
  fe_to_u256(q, a);
  for (int i = 0; i < 4; ++i) {
    w[2 * i] = (uint32_t)q[i];
    w[2 * i + 1] = (uint32_t)(q[i] >> 32);
  }
}

static inline fe fe_c(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  const uint64_t w[4] = {a, b, c, d};
  return fe_from_u256(w, 0);
}
static const fe FE_D = fe_c(0x75eb4dca135978a3ULL, 0x00700a4d4141d8abULL, 0x8cc740797779e898ULL, 0x52036cee2b6ffe73ULL);
static const fe FE_D2 = fe_c(0xebd69b9426b2f159ULL, 0x00e0149a8283b156ULL, 0x198e80f2eef3d130ULL, 0x2406d9dc56dffce7ULL);
static const fe FE_SQRT_M1 =
    fe_c(0xc4ee1b274a0ea0b0ULL, 0x2f431806ad2fe478ULL, 0x2b4d00993dfbd7a7ULL, 0x2b8324804fc1df0bULL);
static const fe FE_INVSQRT_A_MINUS_D =
    fe_c(0x99c8fdaa805d40eaULL, 0x9d2f16175a4172beULL, 0x16c27b91fe01d840ULL, 0x786c8905cfaffca2ULL);

struct ge {
  fe X, Y, Z, T;
};

static inline ge ge_identity() { return ge{fe_zero(), fe_one(), fe_one(), fe_zero()}; }

static inline ge ge_add(const ge& p, const ge& q) {
  fe A = fe_mul(fe_sub(p.Y, p.X), fe_sub(q.Y, q.X));
  fe B = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));
  fe C = fe_mul(fe_mul(p.T, FE_D2), q.T);
  fe ZZ = fe_mul(p.Z, q.Z);
  fe D = fe_add(ZZ, ZZ);
  fe E = fe_sub(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
  return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}

static inline ge ge_neg(const ge& p) { return ge{fe_neg(p.X), p.Y, p.Z, fe_neg(p.T)}; }

static inline ge ge_dbl(const ge& p) {
  fe XX = fe_sq(p.X), YY = fe_sq(p.Y), ZZ = fe_sq(p.Z);
  fe ZZ2 = fe_add(ZZ, ZZ);
  fe XpY2 = fe_sq(fe_add(p.X, p.Y));
  fe YYpXX = fe_add(YY, XX), YYmXX = fe_sub(YY, XX);
  fe cX = fe_sub(XpY2, YYpXX), cT = fe_sub(ZZ2, YYmXX);
  return ge{fe_mul(cX, cT), fe_mul(YYpXX, YYmXX), fe_mul(YYmXX, cT), fe_mul(cX, YYpXX)};
}

static inline bool ge_eq(const ge& a, const ge& b) {
  return fe_eq(fe_mul(a.X, b.Y), fe_mul(a.Y, b.X)) || fe_eq(fe_mul(a.Y, b.Y), fe_mul(a.X, b.X));
}

static inline bool sqrt_ratio_m1(const fe& u, const fe& v, fe& out) {
  fe v3 = fe_mul(fe_sq(v), v);
  fe v7 = fe_mul(fe_sq(v3), v);
  fe r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  fe check = fe_mul(v, fe_sq(r));
  fe nu = fe_neg(u);
  bool correct = fe_eq(check, u);
  bool flipped = fe_eq(check, nu);
  bool flipped_i = fe_eq(check, fe_mul(nu, FE_SQRT_M1));
  if (flipped || flipped_i) r = fe_mul(r, FE_SQRT_M1);
  out = fe_abs(r);
  return correct || flipped;
}

static inline void encode(uint8_t out[32], const ge& p) {
  fe u1 = fe_mul(fe_add(p.Z, p.Y), fe_sub(p.Z, p.Y));
  fe u2 = fe_mul(p.X, p.Y);
  fe inv;
  sqrt_ratio_m1(fe_one(), fe_mul(u1, fe_sq(u2)), inv);
  fe den1 = fe_mul(inv, u1), den2 = fe_mul(inv, u2);
  fe z_inv = fe_mul(fe_mul(den1, den2), p.T);
  bool rotate = fe_isneg(fe_mul(p.T, z_inv));
  fe x = p.X, y = p.Y, den_inv = den2;
  if (rotate) {
    x = fe_mul(p.Y, FE_SQRT_M1);
    y = fe_mul(p.X, FE_SQRT_M1);
    den_inv = fe_mul(den1, FE_INVSQRT_A_MINUS_D);
  }
  if (fe_isneg(fe_mul(x, z_inv))) y = fe_neg(y);
  fe_to_bytes(out, fe_abs(fe_mul(den_inv, fe_sub(p.Z, y))));
}

// Encodings of 2*P_i for a batch with ONE field inversion per call
// (RFC 9496's encode needs an inverse square root per point; for a doubled
// point it is rational).  With e = 2XY, f = Z^2 + dT^2, g = Y^2 + X^2,
// h = Z^2 - dT^2, 2P = (eh : gf : fh : eg), and for that representative
// u1 * u2^2 = W^2 (a - d) with W = 2 e f^2 g h T Z (curve equation:
// h^2 - g^2 = -4 (1 + d) T^2 Z^2), so SQRT_RATIO_M1(1, u1 u2^2) =
// |INVSQRT_A_MINUS_D / W|.  W = 0 exactly for the torsion representatives
// of the identity, whose double encodes to zero.  The rest is encode().
// (The prover computes P = C/2 with halved scalars and encodes C = 2P.)
static inline void encode_double_batch(const ge* pts, size_t n, uint8_t* out) {
  struct St {
    fe X, Y, Z, T, W;
  };
  std::vector<St> st(n);
  std::vector<fe> acc(n);
  fe run = fe_one();
  for (size_t i = 0; i < n; ++i) {
    const ge& p = pts[i];
    const fe XX = fe_sq(p.X), YY = fe_sq(p.Y), ZZ = fe_sq(p.Z), dTT = fe_mul(fe_sq(p.T), FE_D);
    const fe e = fe_mul(fe_add(p.X, p.X), p.Y);
    const fe f = fe_add(ZZ, dTT), g = fe_add(YY, XX), h = fe_sub(ZZ, dTT);
    St& q = st[i];
    q.X = fe_mul(e, h);
    q.Y = fe_mul(g, f);
    q.Z = fe_mul(f, h);
    q.T = fe_mul(e, g);
    // W = 2 e f^2 g h T Z = 2 * X' * Z'... : (eh)(fg)(f)(T Z) * 2
    fe W = fe_mul(fe_mul(q.X, q.Y), fe_mul(f, fe_mul(p.T, p.Z)));
    W = fe_add(W, W);
    q.W = fe_iszero(W) ? fe_zero() : W;
    acc[i] = run;
    if (!fe_iszero(q.W)) run = fe_mul(run, q.W);
  }
  fe inv = fe_invert(run);
  for (size_t i = n; i-- > 0;) {
    St& q = st[i];
    uint8_t* o = out + 32 * i;
    if (fe_iszero(q.W)) {
      memset(o, 0, 32);
      continue;
    }
    const fe Winv = fe_mul(inv, acc[i]);
    inv = fe_mul(inv, q.W);
    const fe isq = fe_abs(fe_mul(FE_INVSQRT_A_MINUS_D, Winv));
    const fe u1 = fe_mul(fe_add(q.Z, q.Y), fe_sub(q.Z, q.Y));
    const fe u2 = fe_mul(q.X, q.Y);
    const fe den1 = fe_mul(isq, u1), den2 = fe_mul(isq, u2);
    const fe z_inv = fe_mul(fe_mul(den1, den2), q.T);
    const bool rotate = fe_isneg(fe_mul(q.T, z_inv));
    fe x = q.X, y = q.Y, den_inv = den2;
    if (rotate) {
      x = fe_mul(q.Y, FE_SQRT_M1);
      y = fe_mul(q.X, FE_SQRT_M1);
      den_inv = fe_mul(den1, FE_INVSQRT_A_MINUS_D);
    }
    if (fe_isneg(fe_mul(x, z_inv))) y = fe_neg(y);
    fe_to_bytes(o, fe_abs(fe_mul(den_inv, fe_sub(q.Z, y))));
  }
}

// The same on eight points per AVX-512 IFMA vector (host/encode_x8.cpp;
// byte-identical).  encode_double_batch_auto takes it when the CPU has IFMA
// and BPP_HOST_IFMA is not 0.
bool encode_x8_available();
void encode_double_batch_x8(const ge* pts, size_t n, uint8_t* out);
static inline void encode_double_batch_auto(const ge* pts, size_t n, uint8_t* out) {
  const char* e = getenv("BPP_HOST_IFMA");
  if (n >= 8 && encode_x8_available() && !(e && e[0] == '0'))
    encode_double_batch_x8(pts, n, out);
  else
    encode_double_batch(pts, n, out);
}

// out[i] = in[i J] + ... + in[i J + J - 1] (i < n): eight additions per
// AVX-512 IFMA vector (host/encode_x8.cpp) when the CPU has IFMA and
// BPP_HOST_IFMA is not 0, else one chain per point
void ge_sum_x8(const ge* in, size_t n, uint32_t J, ge* out);
static inline void ge_sum_auto(const ge* in, size_t n, uint32_t J, ge* out) {
  const char* e = getenv("BPP_HOST_IFMA");
  if (J >= 4 && encode_x8_available() && !(e && e[0] == '0')) {
    ge_sum_x8(in, n, J, out);
    return;
  }
  for (size_t i = 0; i < n; ++i) {
    ge t = in[i * J];
    for (uint32_t j = 1; j < J; ++j) t = ge_add(t, in[i * J + j]);
    out[i] = t;
  }
}

static inline bool decode(ge& out, const uint8_t in[32]) {
  fe s = fe_from_bytes(in);
  uint8_t chk[32];
  fe_to_bytes(chk, s);
  if (memcmp(chk, in, 32) != 0 || (in[0] & 1)) return false;
  fe ss = fe_sq(s);
  fe u1 = fe_sub(fe_one(), ss), u2 = fe_add(fe_one(), ss);
  fe u2_sqr = fe_sq(u2);
  fe v = fe_sub(fe_neg(fe_mul(FE_D, fe_sq(u1))), u2_sqr);
  fe inv;
  bool was_square = sqrt_ratio_m1(fe_one(), fe_mul(v, u2_sqr), inv);
  fe den_x = fe_mul(inv, u2);
  fe den_y = fe_mul(fe_mul(inv, den_x), v);
  fe x = fe_abs(fe_mul(fe_add(s, s), den_x));
  fe y = fe_mul(u1, den_y);
  fe t = fe_mul(x, y);
  if (!was_square || fe_isneg(t) || fe_iszero(y)) return false;
  out = ge{x, y, fe_one(), t};
  return true;
}

// Device element: 10 u32 limbs at bit offsets ceil(25.5 i) (limbs may
// exceed their nominal width; see csrc/fe25519.cuh) -> loose fe.  Limb pair
// (2k, 2k + 1) sits at offsets 51k and 51k + 26, so radix-2^51 limb k is
// w[2k] + w[2k+1] 2^26 (< 2^59), and one carry pass (2^255 = 19) leaves the
// same value mod p in carried limbs.
static inline fe fe_from_dev(const uint32_t w[10]) {
  fe r;
  for (int k = 0; k < 5; ++k) r.v[k] = (uint64_t)w[2 * k] + ((uint64_t)w[2 * k + 1] << 26);
  return fe_carry(r);
}
// device extended point (40 words, csrc/layout.h P3_WORDS) -> host point
static inline ge ge_from_dev(const uint32_t* w) {
  return ge{fe_from_dev(w), fe_from_dev(w + 10), fe_from_dev(w + 20), fe_from_dev(w + 30)};
}

static inline ge ge_from_words(const uint32_t w[32]) {
  return ge{fe_from_words(w), fe_from_words(w + 8), fe_from_words(w + 16), fe_from_words(w + 24)};
}
static inline void ge_to_words(uint32_t w[32], const ge& p) {
  fe_to_words(w, p.X);
  fe_to_words(w + 8, p.Y);
  fe_to_words(w + 16, p.Z);
  fe_to_words(w + 24, p.T);
}

}  // namespace h25519
