// Host-side GF(2^255-19) / Edwards / ristretto255 (radix 2^64, 4 limbs).
//
// Product code, not the oracle: finishes what the GPU hands back (the
// Horner combine of a large MSM's W window sums, compression of a single
// result point, proof-level point equality) where a lone GPU lane would be
// latency-bound.  Independent of the device's 8 x 32-bit representation and
// of the oracle's radix-2^51 port.
#pragma once
#include <stdint.h>
#include <string.h>

namespace h25519 {

typedef unsigned __int128 u128;

struct fe {
  uint64_t v[4];
};

static inline fe fe_zero() { return fe{{0, 0, 0, 0}}; }
static inline fe fe_one() { return fe{{1, 0, 0, 0}}; }

// value = a (256 bits) + top * 2^256 -> loose (< 2^256)
static inline fe fe_fold(fe a, uint64_t top) {
  uint64_t hi = (top << 1) | (a.v[3] >> 63);
  a.v[3] &= 0x7fffffffffffffffULL;
  u128 c = (u128)a.v[0] + (u128)hi * 19u;
  a.v[0] = (uint64_t)c;
  for (int i = 1; i < 4; ++i) {
    c = (u128)a.v[i] + (uint64_t)(c >> 64);
    a.v[i] = (uint64_t)c;
  }
  return a;
}

static inline fe fe_add(const fe& a, const fe& b) {
  fe r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c = (u128)a.v[i] + b.v[i] + (uint64_t)(c >> 64);
    r.v[i] = (uint64_t)c;
  }
  return fe_fold(r, (uint64_t)(c >> 64));
}

static inline fe fe_sub(const fe& a, const fe& b) {
  // a + (4p - b), 4p = 2^257 - 76
  const uint64_t fp[4] = {0xffffffffffffffb4ULL, ~0ULL, ~0ULL, ~0ULL};
  uint64_t t[4];
  uint64_t borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)fp[i] - b.v[i] - borrow;
    t[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 64) & 1;
  }
  uint64_t top = 1 - borrow;
  fe r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c = (u128)a.v[i] + t[i] + (uint64_t)(c >> 64);
    r.v[i] = (uint64_t)c;
  }
  return fe_fold(r, (uint64_t)(c >> 64) + top);
}

static inline fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

static inline fe fe_mul(const fe& a, const fe& b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c = (u128)a.v[i] * b.v[j] + t[i + j] + (uint64_t)(c >> 64);
      t[i + j] = (uint64_t)c;
    }
    t[i + 4] = (uint64_t)(c >> 64);
  }
  fe r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c = (u128)t[4 + i] * 38u + t[i] + (uint64_t)(c >> 64);
    r.v[i] = (uint64_t)c;
  }
  return fe_fold(r, (uint64_t)(c >> 64));
}

static inline fe fe_sq(const fe& a) { return fe_mul(a, a); }

static inline fe fe_sqn(fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

static inline fe fe_canon(fe a) {
  a = fe_fold(a, 0);
  uint64_t t[4];
  u128 c = (u128)a.v[0] + 19u;
  t[0] = (uint64_t)c;
  for (int i = 1; i < 4; ++i) {
    c = (u128)a.v[i] + (uint64_t)(c >> 64);
    t[i] = (uint64_t)c;
  }
  if (t[3] >> 63) {
    t[3] &= 0x7fffffffffffffffULL;
    for (int i = 0; i < 4; ++i) a.v[i] = t[i];
  }
  return a;
}

static inline bool fe_iszero(const fe& a) {
  fe c = fe_canon(a);
  return (c.v[0] | c.v[1] | c.v[2] | c.v[3]) == 0;
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

static inline fe fe_from_bytes(const uint8_t b[32]) {
  fe r;
  memcpy(r.v, b, 32);  // little-endian host
  return r;
}
static inline void fe_to_bytes(uint8_t b[32], const fe& a) {
  fe c = fe_canon(a);
  memcpy(b, c.v, 32);
}
static inline fe fe_from_words(const uint32_t w[8]) {
  fe r;
  for (int i = 0; i < 4; ++i) r.v[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  return r;
}
static inline void fe_to_words(uint32_t w[8], const fe& a) {
  for (int i = 0; i < 4; ++i) {
    w[2 * i] = (uint32_t)a.v[i];
    w[2 * i + 1] = (uint32_t)(a.v[i] >> 32);
  }
}

static const fe FE_D = {{0x75eb4dca135978a3ULL, 0x00700a4d4141d8abULL, 0x8cc740797779e898ULL, 0x52036cee2b6ffe73ULL}};
static const fe FE_D2 = {{0xebd69b9426b2f159ULL, 0x00e0149a8283b156ULL, 0x198e80f2eef3d130ULL, 0x2406d9dc56dffce7ULL}};
static const fe FE_SQRT_M1 = {{0xc4ee1b274a0ea0b0ULL, 0x2f431806ad2fe478ULL, 0x2b4d00993dfbd7a7ULL, 0x2b8324804fc1df0bULL}};
static const fe FE_INVSQRT_A_MINUS_D = {{0x99c8fdaa805d40eaULL, 0x9d2f16175a4172beULL, 0x16c27b91fe01d840ULL, 0x786c8905cfaffca2ULL}};

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
// exceed their nominal width; see csrc/fe25519.cuh) -> loose fe.
static inline fe fe_from_dev(const uint32_t w[10]) {
  static const int OFF[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  uint64_t t[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 10; ++i) {
    const int q = OFF[i] >> 6, s = OFF[i] & 63;
    const u128 x = (u128)w[i] << s;
    u128 c = (u128)t[q] + (uint64_t)x;
    t[q] = (uint64_t)c;
    c = (u128)t[q + 1] + (uint64_t)(x >> 64) + (uint64_t)(c >> 64);
    t[q + 1] = (uint64_t)c;
    for (int k = q + 2; k < 5 && (c >> 64); ++k) {
      c = (u128)t[k] + (uint64_t)(c >> 64);
      t[k] = (uint64_t)c;
    }
  }
  return fe_fold(fe{{t[0], t[1], t[2], t[3]}}, t[4]);
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
