// Host scalar field Z/lZ, l = 2^252 + 27742317777372353535851937790883648493.
//
// Product code for the host-side protocol logic (challenges, circuit
// linear algebra, batch inversion) that the reference performs with dalek's
// `Scalar` (circuit_lib.rs:256-302 compute_per_challenges, util.rs:6-94,
// poly.rs:5-77).  Values are kept canonical (< l) in 4 x u64 limbs;
// multiplication is two Montgomery (CIOS, R = 2^256) steps.
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

namespace hsc {

typedef unsigned __int128 u128;

struct Sc {
  uint64_t v[4];
  bool operator==(const Sc& o) const { return !memcmp(v, o.v, 32); }
  bool operator!=(const Sc& o) const { return !(*this == o); }
};

static const Sc L = {{0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0x0ULL, 0x1000000000000000ULL}};
static const Sc R2 = {{0xa40611e3449c0f01ULL, 0xd00e1ba768859347ULL, 0xceec73d217f5be65ULL, 0x0399411b7c309a3dULL}};
static const Sc R3 = {{0x2a9e49687b83a2dbULL, 0x278324e6aef7f3ecULL, 0x8065dc6c04ec5b65ULL, 0x0e530b773599cec7ULL}};
static const uint64_t LINV = 0xd2b51da312547e1bULL;  // -l^-1 mod 2^64

static inline Sc zero() { return Sc{{0, 0, 0, 0}}; }
static inline Sc one() { return Sc{{1, 0, 0, 0}}; }
static inline Sc from_u64(uint64_t x) { return Sc{{x, 0, 0, 0}}; }

static inline bool geq(const Sc& a, const Sc& b) {
  for (int i = 3; i >= 0; --i) {
    if (a.v[i] != b.v[i]) return a.v[i] > b.v[i];
  }
  return true;
}

static inline Sc sub_raw(const Sc& a, const Sc& b, uint64_t* borrow_out) {
  Sc r;
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (borrow_out) *borrow_out = br;
  return r;
}

static inline Sc add(const Sc& a, const Sc& b) {
  Sc r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c = (u128)a.v[i] + b.v[i] + (uint64_t)(c >> 64);
    r.v[i] = (uint64_t)c;
  }
  // a, b < l < 2^253: no 256-bit overflow
  if (geq(r, L)) r = sub_raw(r, L, nullptr);
  return r;
}

// a / 2 mod l for canonical a: a even -> a >> 1, odd -> (a + l) >> 1
static inline Sc half(const Sc& a) {
  Sc t = a;
  if (a.v[0] & 1) {
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; ++i) {
      c += (unsigned __int128)a.v[i] + L.v[i];
      t.v[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  for (int i = 0; i < 3; ++i) t.v[i] = (t.v[i] >> 1) | (t.v[i + 1] << 63);
  t.v[3] >>= 1;
  return t;
}

static inline Sc sub(const Sc& a, const Sc& b) {
  uint64_t br;
  Sc r = sub_raw(a, b, &br);
  if (br) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
      c = (u128)r.v[i] + L.v[i] + (uint64_t)(c >> 64);
      r.v[i] = (uint64_t)c;
    }
  }
  return r;
}

static inline Sc neg(const Sc& a) { return sub(zero(), a); }

// Montgomery product a*b*R^-1 mod l (a*b < l*R required)
static inline Sc mont(const Sc& a, const Sc& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c = (u128)a.v[i] * b.v[j] + t[j] + (uint64_t)(c >> 64);
      t[j] = (uint64_t)c;
    }
    c = (u128)t[4] + (uint64_t)(c >> 64);
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    const uint64_t m = t[0] * LINV;
    c = (u128)m * L.v[0] + t[0];
    for (int j = 1; j < 4; ++j) {
      c = (u128)m * L.v[j] + t[j] + (uint64_t)(c >> 64);
      t[j - 1] = (uint64_t)c;
    }
    c = (u128)t[4] + (uint64_t)(c >> 64);
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  Sc r = {{t[0], t[1], t[2], t[3]}};
  if (t[4] || geq(r, L)) r = sub_raw(r, L, nullptr);
  return r;
}

static inline Sc mul(const Sc& a, const Sc& b) { return mont(mont(a, b), R2); }
static inline Sc sq(const Sc& a) { return mul(a, a); }
// Montgomery form b*R mod l of a canonical b; then mulm(a, to_mont(b)) = a*b
// with one Montgomery step (for operands reused across many products).
static inline Sc to_mont(const Sc& b) { return mont(b, R2); }
static inline Sc mulm(const Sc& a, const Sc& bR) { return mont(a, bR); }

// from 32 canonical little-endian bytes; false if >= l
static inline bool from_canonical(Sc& out, const uint8_t b[32]) {
  memcpy(out.v, b, 32);
  return !geq(out, L);
}

// dalek Scalar::from_bytes_mod_order_wide (64 bytes)
// x = lo + hi * 2^256: hi * 2^256 mod l = mont(hi, R2) (one Montgomery
// product), lo mod l by folding its top 4 bits (2^252 = -delta mod l with
// delta = l - 2^252 < 2^125).
static inline Sc reduce256(Sc a) {
  const uint64_t q = a.v[3] >> 60;  // a = q * 2^252 + (a mod 2^252)
  a.v[3] &= 0x0fffffffffffffffULL;
  // a - q * delta, delta = L.v[0..1] (L = 2^252 + delta)
  const u128 p0 = (u128)q * L.v[0], p1 = (u128)q * L.v[1] + (uint64_t)(p0 >> 64);
  const Sc qd = {{(uint64_t)p0, (uint64_t)p1, (uint64_t)(p1 >> 64), 0}};
  uint64_t br;
  Sc r = sub_raw(a, qd, &br);
  if (br) {  // negative (> -2^129): add l once
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
      c = (u128)r.v[i] + L.v[i] + (uint64_t)(c >> 64);
      r.v[i] = (uint64_t)c;
    }
  }
  return r;
}

// x = H 2^252 + Lo and 2^252 = -delta (mod l), delta = l - 2^252 < 2^125:
// x = Lo - H delta, H delta = T1 2^252 + T0 (T1 < 2^133), so
// x = Lo - T0 + T1 delta, and T1 delta = U1 2^252 + U0 (U1 < 2^6):
// x = Lo + U0 - T0 - U1 delta, in (-2^253, 2^253): at most one l added and
// two subtracted.  18 64x64 products (the Montgomery form took 32 + 16) --
// the prover reduces ~370 wide draws per proof (host profile: 2/3 of the
// SHAKE draw phase was this reduction).
static inline Sc from_wide(const uint8_t b[64]) {
  uint64_t x[8];
  memcpy(x, b, 64);
  const uint64_t d0 = L.v[0], d1 = L.v[1];  // delta
  const uint64_t M60 = 0x0fffffffffffffffULL;
  // H = x >> 252 (5 limbs, top < 2^4); Lo = x mod 2^252
  uint64_t H[5];
  for (int i = 0; i < 4; ++i) H[i] = (x[3 + i] >> 60) | (x[4 + i] << 4);
  H[4] = x[7] >> 60;
  // T = H * delta (7 limbs)
  uint64_t T[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 5; ++i) {
    u128 c = (u128)H[i] * d0 + T[i];
    T[i] = (uint64_t)c;
    c = (u128)H[i] * d1 + T[i + 1] + (uint64_t)(c >> 64);
    T[i + 1] = (uint64_t)c;
    T[i + 2] += (uint64_t)(c >> 64);
  }
  // T1 = T >> 252 (3 limbs), T0 = T mod 2^252
  const uint64_t T1[3] = {(T[3] >> 60) | (T[4] << 4), (T[4] >> 60) | (T[5] << 4), (T[5] >> 60) | (T[6] << 4)};
  // U = T1 * delta (5 limbs, < 2^258)
  uint64_t U[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 3; ++i) {
    u128 c = (u128)T1[i] * d0 + U[i];
    U[i] = (uint64_t)c;
    c = (u128)T1[i] * d1 + U[i + 1] + (uint64_t)(c >> 64);
    U[i + 1] = (uint64_t)c;
    U[i + 2] += (uint64_t)(c >> 64);
  }
  const uint64_t U1 = (U[3] >> 60) | (U[4] << 4);
  // V = U1 * delta (< 2^131)
  const u128 v0 = (u128)U1 * d0;
  const u128 v1 = (u128)U1 * d1 + (uint64_t)(v0 >> 64);
  const uint64_t V[3] = {(uint64_t)v0, (uint64_t)v1, (uint64_t)(v1 >> 64)};
  // r = Lo + U0 - T0 - V as a signed 5-limb value (two's complement)
  const uint64_t lo[4] = {x[0], x[1], x[2], x[3] & M60};
  const uint64_t u0[4] = {U[0], U[1], U[2], U[3] & M60};
  const uint64_t t0[4] = {T[0], T[1], T[2], T[3] & M60};
  uint64_t r[5];
  __int128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (__int128)lo[i] + u0[i] - t0[i] - (i < 3 ? V[i] : 0);
    r[i] = (uint64_t)c;
    c >>= 64;  // arithmetic shift: carry / borrow
  }
  r[4] = (uint64_t)c;
  // bring into [0, l): add l while negative, subtract while >= l
  auto add_l = [&]() {
    u128 k = 0;
    for (int i = 0; i < 4; ++i) {
      k += (u128)r[i] + L.v[i];
      r[i] = (uint64_t)k;
      k >>= 64;
    }
    r[4] += (uint64_t)k;
  };
  while ((int64_t)r[4] < 0) add_l();
  Sc out = {{r[0], r[1], r[2], r[3]}};
  while (r[4] || geq(out, L)) {
    uint64_t br;
    out = sub_raw(out, L, &br);
    r[4] -= br;
    r[0] = out.v[0];
  }
  return out;
}

// (the previous form, kept as the reference the fast path is tested against)
static inline Sc from_wide_mont(const uint8_t b[64]) {
  Sc lo, hi;
  memcpy(lo.v, b, 32);
  memcpy(hi.v, b + 32, 32);
  return add(reduce256(lo), mont(hi, R2));
}

// dalek Scalar::from_bytes_mod_order (32 bytes, any value)
static inline Sc from_bytes_mod(const uint8_t b[32]) {
  uint8_t w[64] = {0};
  memcpy(w, b, 32);
  return from_wide(w);
}

static inline void to_bytes(uint8_t out[32], const Sc& a) { memcpy(out, a.v, 32); }

// square-and-multiply in the Montgomery domain (one step per operation)
static inline Sc pow(const Sc& a, const Sc& e) {
  const Sc aR = to_mont(a);
  Sc rR = to_mont(one());
  for (int i = 255; i >= 0; --i) {
    rR = mont(rR, rR);
    if ((e.v[i >> 6] >> (i & 63)) & 1) rR = mont(rR, aR);
  }
  return mont(rR, one());
}

static inline bool is_zero(const Sc& a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }

static inline Sc invert(const Sc& a) {
  Sc e = sub_raw(L, from_u64(2), nullptr);
  return pow(a, e);
}

// a^-1 mod l by the binary extended Euclidean algorithm, in time that depends
// on a: only for public values (the inner-product argument's challenges u,
// which the transcript publishes).  Invariants x1 a = u, x2 a = v (mod l);
// each step halves an even one of u, v (and its x mod l) or subtracts the
// smaller odd one from the larger.  ~3x fewer 64-bit operations than
// invert's 250 squarings (config 2 spends one per IPA round on the host).
// a != 0 mod l.
static inline Sc invert_vartime(const Sc& a) {
  auto shr1 = [](Sc s) {
    for (int i = 0; i < 3; ++i) s.v[i] = (s.v[i] >> 1) | (s.v[i + 1] << 63);
    s.v[3] >>= 1;
    return s;
  };
  auto is_one = [](const Sc& s) { return s.v[0] == 1 && (s.v[1] | s.v[2] | s.v[3]) == 0; };
  Sc u = a, v = L, x1 = one(), x2 = zero();
  while (!is_one(u) && !is_one(v)) {
    while (!(u.v[0] & 1)) {
      u = shr1(u);
      x1 = half(x1);
    }
    while (!(v.v[0] & 1)) {
      v = shr1(v);
      x2 = half(x2);
    }
    if (is_one(u) || is_one(v)) break;
    if (geq(u, v)) {
      u = sub_raw(u, v, nullptr);
      x1 = sub(x1, x2);
    } else {
      v = sub_raw(v, u, nullptr);
      x2 = sub(x2, x1);
    }
  }
  return is_one(u) ? x1 : x2;
}

// Montgomery's trick; returns the inverse of the product.  Zero inputs
// are not allowed (dalek batch_invert has the same precondition).
// One Montgomery product per step on canonical values: acc_i = prod_{j<i}
// x_j R^-i, inv_{i+1} = acc_{i+1}^-1 = prod_{j<=i} x_j^-1 R^(i+1), so
// mont(inv_{i+1}, acc_i) = x_i^-1 and mont(inv_{i+1}, x_i) = inv_i: 3n
// products + one inversion (the canonical-product form took 6n).
// vartime: the one inversion by invert_vartime (public inputs only).
static inline Sc batch_invert(std::vector<Sc>& xs, bool want_allinv = true, bool vartime = false) {
  const size_t n = xs.size();
  std::vector<Sc> pref(n);
  Sc acc = one();
  for (size_t i = 0; i < n; ++i) {
    pref[i] = acc;
    acc = mont(acc, xs[i]);
  }
  Sc inv = vartime ? invert_vartime(acc) : invert(acc);  // prod x^-1 R^n
  Sc allinv = zero();
  if (want_allinv) {  // prod x^-1 = inv R^-n
    allinv = inv;
    for (size_t i = 0; i < n; ++i) allinv = mont(allinv, one());
  }
  for (size_t i = n; i-- > 0;) {
    const Sc t = mont(inv, pref[i]);
    inv = mont(inv, xs[i]);
    xs[i] = t;
  }
  return allinv;
}

// sum a_i b_i: Montgomery products accumulated, one correction at the end
static inline Sc inner_product(const std::vector<Sc>& a, const std::vector<Sc>& b) {
  Sc r = zero();
  for (size_t i = 0; i < a.size(); ++i) r = add(r, mont(a[i], b[i]));
  return mont(r, R2);
}

// r[i] = r[0] x^i from r[0] (canonical or Montgomery form alike: mont by xR
// multiplies by x): four interleaved chains r[i] = r[i-4] x^4 after the
// first four, so four independent products overlap in the core's pipeline
// instead of one chain of n dependent ones (2^10 powers ~3x faster)
static inline void powers_fill(std::vector<Sc>& r, Sc c, const Sc& x) {
  const size_t n = r.size();
  const Sc xR = to_mont(x);
  size_t i = 0;
  for (; i < n && i < 4; ++i) {
    r[i] = c;
    c = mont(c, xR);
  }
  if (i == n) return;
  Sc x4 = mont(x, xR);   // x^2
  x4 = mont(x4, x4);     // x^4 R^-1 ... (mont(a, a) = a^2 R^-1)
  x4 = mont(x4, R3);     // x^4 R
  for (; i < n; ++i) r[i] = mont(r[i - 4], x4);
}

// (1, x, x^2, ..., x^{n-1})
static inline std::vector<Sc> powers(const Sc& x, size_t n) {
  std::vector<Sc> r(n);
  powers_fill(r, one(), x);
  return r;
}

// (R, xR, x^2 R, ...): Montgomery forms of the powers, for mulm
static inline std::vector<Sc> powers_mont(const Sc& x, size_t n) {
  std::vector<Sc> r(n);
  powers_fill(r, to_mont(one()), x);
  return r;
}

}  // namespace hsc
