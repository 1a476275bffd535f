/*
 * dalek_port.c — serial C restatement of curve25519-dalek-ng 4.1.1's u64
 * backend MSM path.  TEST INFRASTRUCTURE / CPU BASELINE ONLY ("port").
 *
 * The reference (bp-perm, Rust) calls `RistrettoPoint::vartime_multiscalar_mul`
 * at circuit_lib.rs:187,202,216,363,...,568; dalek is
 * not vendored under /root/reference and no Rust toolchain exists here, so
 * this restates its published algorithms:
 *
 *   - FieldElement51: radix 2^51, 5 x u64 limbs, u128 products
 *   - EdwardsPoint extended coords; ProjectiveNiels / AffineNiels /
 *     Completed intermediate forms (an add = 4M to Completed + 4M back)
 *   - vartime MSM dispatch: Straus (width-5 NAF, odd-multiple tables) when
 *     n < 190, else Pippenger with w = 6 (n < 500), 7 (n < 800), 8, signed
 *     radix-2^w digits, 2^(w-1) buckets, running-sum bucket reduction,
 *     columns combined by mul_by_pow_2(w)
 *   - ristretto255 encode / decode / from_uniform_bytes (RFC 9496)
 *
 * Parity: checked against the Python spec oracle (tests/test_oracle_cport.py),
 * which is itself pinned by the RFC 9496 / Merlin / OpenSSL KATs.
 * Single-threaded like dalek's serial backend; bench entry points time it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t l[5]; } fe51;
#define MASK51 ((1ULL << 51) - 1)


static const fe51 FE_ZERO = {{0, 0, 0, 0, 0}};
static const fe51 FE_ONE = {{1, 0, 0, 0, 0}};

static fe51 fe_reduce(uint64_t l0, uint64_t l1, uint64_t l2, uint64_t l3, uint64_t l4) {
  uint64_t c0 = l0 >> 51, c1 = l1 >> 51, c2 = l2 >> 51, c3 = l3 >> 51, c4 = l4 >> 51;
  fe51 r;
  r.l[0] = (l0 & MASK51) + c4 * 19;
  r.l[1] = (l1 & MASK51) + c0;
  r.l[2] = (l2 & MASK51) + c1;
  r.l[3] = (l3 & MASK51) + c2;
  r.l[4] = (l4 & MASK51) + c3;
  return r;
}

static fe51 fe_add(fe51 a, fe51 b) {
  fe51 r;
  for (int i = 0; i < 5; ++i) r.l[i] = a.l[i] + b.l[i];
  return r;
}

/* a - b: add 16p first so limbs stay non-negative (dalek's approach) */
static fe51 fe_sub(fe51 a, fe51 b) {
  return fe_reduce(a.l[0] + 36028797018963664ULL - b.l[0], a.l[1] + 36028797018963952ULL - b.l[1],
                   a.l[2] + 36028797018963952ULL - b.l[2], a.l[3] + 36028797018963952ULL - b.l[3],
                   a.l[4] + 36028797018963952ULL - b.l[4]);
}

static fe51 fe_neg(fe51 a) { return fe_sub(FE_ZERO, a); }

static fe51 fe_mul(fe51 a, fe51 b) {
  const uint64_t b1_19 = b.l[1] * 19, b2_19 = b.l[2] * 19, b3_19 = b.l[3] * 19, b4_19 = b.l[4] * 19;
  u128 c0 = (u128)a.l[0] * b.l[0] + (u128)a.l[4] * b1_19 + (u128)a.l[3] * b2_19 + (u128)a.l[2] * b3_19 + (u128)a.l[1] * b4_19;
  u128 c1 = (u128)a.l[1] * b.l[0] + (u128)a.l[0] * b.l[1] + (u128)a.l[4] * b2_19 + (u128)a.l[3] * b3_19 + (u128)a.l[2] * b4_19;
  u128 c2 = (u128)a.l[2] * b.l[0] + (u128)a.l[1] * b.l[1] + (u128)a.l[0] * b.l[2] + (u128)a.l[4] * b3_19 + (u128)a.l[3] * b4_19;
  u128 c3 = (u128)a.l[3] * b.l[0] + (u128)a.l[2] * b.l[1] + (u128)a.l[1] * b.l[2] + (u128)a.l[0] * b.l[3] + (u128)a.l[4] * b4_19;
  u128 c4 = (u128)a.l[4] * b.l[0] + (u128)a.l[3] * b.l[1] + (u128)a.l[2] * b.l[2] + (u128)a.l[1] * b.l[3] + (u128)a.l[0] * b.l[4];
  c1 += (uint64_t)(c0 >> 51);
  uint64_t o0 = (uint64_t)c0 & MASK51;
  c2 += (uint64_t)(c1 >> 51);
  uint64_t o1 = (uint64_t)c1 & MASK51;
  c3 += (uint64_t)(c2 >> 51);
  uint64_t o2 = (uint64_t)c2 & MASK51;
  c4 += (uint64_t)(c3 >> 51);
  uint64_t o3 = (uint64_t)c3 & MASK51;
  uint64_t carry = (uint64_t)(c4 >> 51);
  uint64_t o4 = (uint64_t)c4 & MASK51;
  o0 += carry * 19;
  o1 += o0 >> 51;
  o0 &= MASK51;
  fe51 r = {{o0, o1, o2, o3, o4}};
  return r;
}

static fe51 fe_sq(fe51 a) { return fe_mul(a, a); }
static fe51 fe_sqn(fe51 a, int n) { while (n--) a = fe_sq(a); return a; }

static void fe_tobytes(uint8_t out[32], fe51 a) {
  /* full carry, then subtract p if needed */
  fe51 t = fe_reduce(a.l[0], a.l[1], a.l[2], a.l[3], a.l[4]);
  uint64_t q = (t.l[0] + 19) >> 51;
  q = (t.l[1] + q) >> 51;
  q = (t.l[2] + q) >> 51;
  q = (t.l[3] + q) >> 51;
  q = (t.l[4] + q) >> 51;
  t.l[0] += 19 * q;
  t.l[1] += t.l[0] >> 51; t.l[0] &= MASK51;
  t.l[2] += t.l[1] >> 51; t.l[1] &= MASK51;
  t.l[3] += t.l[2] >> 51; t.l[2] &= MASK51;
  t.l[4] += t.l[3] >> 51; t.l[3] &= MASK51;
  t.l[4] &= MASK51;
  uint64_t w[4];
  w[0] = t.l[0] | (t.l[1] << 51);
  w[1] = (t.l[1] >> 13) | (t.l[2] << 38);
  w[2] = (t.l[2] >> 26) | (t.l[3] << 25);
  w[3] = (t.l[3] >> 39) | (t.l[4] << 12);
  memcpy(out, w, 32);
}

static fe51 fe_frombytes(const uint8_t in[32]) {
  uint64_t w[4];
  memcpy(w, in, 32);
  fe51 r;
  r.l[0] = w[0] & MASK51;
  r.l[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
  r.l[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
  r.l[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
  r.l[4] = (w[3] >> 12) & MASK51;
  return r;
}

static int fe_iszero(fe51 a) {
  uint8_t b[32];
  fe_tobytes(b, a);
  uint8_t o = 0;
  for (int i = 0; i < 32; ++i) o |= b[i];
  return o == 0;
}
static int fe_isneg(fe51 a) { uint8_t b[32]; fe_tobytes(b, a); return b[0] & 1; }
static int fe_eq(fe51 a, fe51 b) { return fe_iszero(fe_sub(a, b)); }
static fe51 fe_abs(fe51 a) { return fe_isneg(a) ? fe_neg(a) : a; }

static void fe_pow_core(fe51 z, fe51* z_250_0, fe51* z11) {
  fe51 z2 = fe_sq(z);
  fe51 z9 = fe_mul(z, fe_sqn(z2, 2));
  *z11 = fe_mul(z2, z9);
  fe51 z_5_0 = fe_mul(z9, fe_sq(*z11));
  fe51 z_10_0 = fe_mul(fe_sqn(z_5_0, 5), z_5_0);
  fe51 z_20_0 = fe_mul(fe_sqn(z_10_0, 10), z_10_0);
  fe51 z_40_0 = fe_mul(fe_sqn(z_20_0, 20), z_20_0);
  fe51 z_50_0 = fe_mul(fe_sqn(z_40_0, 10), z_10_0);
  fe51 z_100_0 = fe_mul(fe_sqn(z_50_0, 50), z_50_0);
  fe51 z_200_0 = fe_mul(fe_sqn(z_100_0, 100), z_100_0);
  *z_250_0 = fe_mul(fe_sqn(z_200_0, 50), z_50_0);
}

static fe51 fe_pow22523(fe51 z) { fe51 a, b; fe_pow_core(z, &a, &b); return fe_mul(fe_sqn(a, 2), z); }

static fe51 fe_const_bytes(const char* hex) {
  uint8_t b[32];
  for (int i = 0; i < 32; ++i) {
    char t[3] = {hex[2 * i], hex[2 * i + 1], 0};
    b[i] = (uint8_t)strtoul(t, NULL, 16);
  }
  return fe_frombytes(b);
}

/* constants (little-endian hex) */
static fe51 C_D, C_D2, C_SQRT_M1, C_INVSQRT_A_MINUS_D, C_SQRT_AD_MINUS_ONE, C_ONE_MINUS_D_SQ, C_D_MINUS_ONE_SQ;
static int consts_ready = 0;
static void init_consts(void) {
  if (consts_ready) return;
  C_D = fe_const_bytes("a3785913ca4deb75abd841414d0a700098e879777940c78c73fe6f2bee6c0352");
  C_D2 = fe_add(C_D, C_D);
  C_SQRT_M1 = fe_const_bytes("b0a00e4a271beec478e42fad0618432fa7d7fb3d99004d2b0bdfc14f8024832b");
  C_INVSQRT_A_MINUS_D = fe_const_bytes("ea405d80aafdc899be72415a17162f9d40d801fe917bc216a2fcafcf05896c78");
  C_SQRT_AD_MINUS_ONE = fe_const_bytes("1b2e7b49a0f6977ebd54781b0c8e9daffdd1f531c9fc3c0fac48832bbf316937");
  C_ONE_MINUS_D_SQ = fe_const_bytes("76c15f94c1097ce20f355ecd38a1812ce4df70beddab9499d7e0b3b2a8729002");
  C_D_MINUS_ONE_SQ = fe_const_bytes("204ded44aa5aad3199191eb02c4a9ed2eb4e9b522fd3dc4c41226cf67ab36859");
  consts_ready = 1;
}

/* ------------------------------------------------------------ group */
typedef struct { fe51 X, Y, Z, T; } ge_ext;
typedef struct { fe51 X, Y, Z, T; } ge_completed; /* x = X/Z, y = Y/T */
typedef struct { fe51 X, Y, Z; } ge_proj;
typedef struct { fe51 YpX, YmX, Z, T2d; } ge_pniels;

static ge_ext ge_identity(void) { ge_ext r = {FE_ZERO, FE_ONE, FE_ONE, FE_ZERO}; return r; }
static ge_proj ge_proj_identity(void) { ge_proj r = {FE_ZERO, FE_ONE, FE_ONE}; return r; }

static ge_pniels to_pniels(const ge_ext* p) {
  ge_pniels n = {fe_add(p->Y, p->X), fe_sub(p->Y, p->X), p->Z, fe_mul(p->T, C_D2)};
  return n;
}
static ge_ext completed_to_ext(const ge_completed* c) {
  ge_ext r = {fe_mul(c->X, c->T), fe_mul(c->Y, c->Z), fe_mul(c->Z, c->T), fe_mul(c->X, c->Y)};
  return r;
}
static ge_proj completed_to_proj(const ge_completed* c) {
  ge_proj r = {fe_mul(c->X, c->T), fe_mul(c->Y, c->Z), fe_mul(c->Z, c->T)};
  return r;
}
static ge_ext proj_to_ext(const ge_proj* p) {
  ge_ext r = {fe_mul(p->X, p->Z), fe_mul(p->Y, p->Z), fe_sq(p->Z), fe_mul(p->X, p->Y)};
  return r;
}
static ge_completed ge_add_pn(const ge_ext* p, const ge_pniels* q) {
  fe51 PP = fe_mul(fe_add(p->Y, p->X), q->YpX);
  fe51 MM = fe_mul(fe_sub(p->Y, p->X), q->YmX);
  fe51 TT2d = fe_mul(p->T, q->T2d);
  fe51 ZZ = fe_mul(p->Z, q->Z);
  fe51 ZZ2 = fe_add(ZZ, ZZ);
  ge_completed c = {fe_sub(PP, MM), fe_add(PP, MM), fe_add(ZZ2, TT2d), fe_sub(ZZ2, TT2d)};
  return c;
}
static ge_completed ge_sub_pn(const ge_ext* p, const ge_pniels* q) {
  fe51 PM = fe_mul(fe_add(p->Y, p->X), q->YmX);
  fe51 MP = fe_mul(fe_sub(p->Y, p->X), q->YpX);
  fe51 TT2d = fe_mul(p->T, q->T2d);
  fe51 ZZ = fe_mul(p->Z, q->Z);
  fe51 ZZ2 = fe_add(ZZ, ZZ);
  ge_completed c = {fe_sub(PM, MP), fe_add(PM, MP), fe_sub(ZZ2, TT2d), fe_add(ZZ2, TT2d)};
  return c;
}
static ge_completed proj_double(const ge_proj* p) {
  fe51 XX = fe_sq(p->X), YY = fe_sq(p->Y), ZZ2 = fe_sq(p->Z);
  ZZ2 = fe_add(ZZ2, ZZ2);
  fe51 XpY2 = fe_sq(fe_add(p->X, p->Y));
  fe51 YYpXX = fe_add(YY, XX), YYmXX = fe_sub(YY, XX);
  ge_completed c = {fe_sub(XpY2, YYpXX), YYpXX, YYmXX, fe_sub(ZZ2, YYmXX)};
  return c;
}
static ge_ext ge_add(const ge_ext* p, const ge_ext* q) {
  ge_pniels n = to_pniels(q);
  ge_completed c = ge_add_pn(p, &n);
  return completed_to_ext(&c);
}
static ge_ext ge_mul_pow2(const ge_ext* p, unsigned k) {
  ge_proj s = {p->X, p->Y, p->Z};
  ge_completed c;
  for (unsigned i = 0; i < k - 1; ++i) {
    c = proj_double(&s);
    s = completed_to_proj(&c);
  }
  c = proj_double(&s);
  return completed_to_ext(&c);
}

/* ------------------------------------------------------------ ristretto */
static int sqrt_ratio_m1(fe51 u, fe51 v, fe51* out) {
  fe51 v3 = fe_mul(fe_sq(v), v);
  fe51 v7 = fe_mul(fe_sq(v3), v);
  fe51 r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  fe51 check = fe_mul(v, fe_sq(r));
  fe51 nu = fe_neg(u);
  int correct = fe_eq(check, u), flipped = fe_eq(check, nu), flipped_i = fe_eq(check, fe_mul(nu, C_SQRT_M1));
  if (flipped || flipped_i) r = fe_mul(r, C_SQRT_M1);
  *out = fe_abs(r);
  return correct || flipped;
}

static int ristretto_decode(ge_ext* out, const uint8_t in[32]) {
  fe51 s = fe_frombytes(in);
  uint8_t chk[32];
  fe_tobytes(chk, s);
  if (memcmp(chk, in, 32) != 0 || (in[0] & 1)) return 0;
  fe51 ss = fe_sq(s), u1 = fe_sub(FE_ONE, ss), u2 = fe_add(FE_ONE, ss), u2s = fe_sq(u2);
  fe51 v = fe_sub(fe_neg(fe_mul(C_D, fe_sq(u1))), u2s);
  fe51 inv;
  int ok = sqrt_ratio_m1(FE_ONE, fe_mul(v, u2s), &inv);
  fe51 dx = fe_mul(inv, u2), dy = fe_mul(fe_mul(inv, dx), v);
  fe51 x = fe_abs(fe_mul(fe_add(s, s), dx)), y = fe_mul(u1, dy), t = fe_mul(x, y);
  if (!ok || fe_isneg(t) || fe_iszero(y)) return 0;
  ge_ext r = {x, y, FE_ONE, t};
  *out = r;
  return 1;
}

static void ristretto_encode(uint8_t out[32], const ge_ext* p) {
  fe51 u1 = fe_mul(fe_add(p->Z, p->Y), fe_sub(p->Z, p->Y)), u2 = fe_mul(p->X, p->Y), inv;
  sqrt_ratio_m1(FE_ONE, fe_mul(u1, fe_sq(u2)), &inv);
  fe51 den1 = fe_mul(inv, u1), den2 = fe_mul(inv, u2), z_inv = fe_mul(fe_mul(den1, den2), p->T);
  int rotate = fe_isneg(fe_mul(p->T, z_inv));
  fe51 x = p->X, y = p->Y, den_inv = den2;
  if (rotate) {
    x = fe_mul(p->Y, C_SQRT_M1);
    y = fe_mul(p->X, C_SQRT_M1);
    den_inv = fe_mul(den1, C_INVSQRT_A_MINUS_D);
  }
  if (fe_isneg(fe_mul(x, z_inv))) y = fe_neg(y);
  fe_tobytes(out, fe_abs(fe_mul(den_inv, fe_sub(p->Z, y))));
}

static ge_ext elligator(fe51 t) {
  fe51 r = fe_mul(C_SQRT_M1, fe_sq(t));
  fe51 u = fe_mul(fe_add(r, FE_ONE), C_ONE_MINUS_D_SQ);
  fe51 v = fe_mul(fe_sub(fe_neg(FE_ONE), fe_mul(r, C_D)), fe_add(r, C_D));
  fe51 s;
  int sq = sqrt_ratio_m1(u, v, &s);
  fe51 s_prime = fe_neg(fe_abs(fe_mul(s, t)));
  fe51 c = sq ? fe_neg(FE_ONE) : r;
  if (!sq) s = s_prime;
  fe51 N = fe_sub(fe_mul(fe_mul(c, fe_sub(r, FE_ONE)), C_D_MINUS_ONE_SQ), v);
  fe51 w0 = fe_mul(fe_add(s, s), v), w1 = fe_mul(N, C_SQRT_AD_MINUS_ONE);
  fe51 ss = fe_sq(s), w2 = fe_sub(FE_ONE, ss), w3 = fe_add(FE_ONE, ss);
  ge_ext P = {fe_mul(w0, w3), fe_mul(w2, w1), fe_mul(w1, w3), fe_mul(w0, w2)};
  return P;
}

static ge_ext from_uniform(const uint8_t b[64]) {
  uint8_t t[32];
  memcpy(t, b, 32); t[31] &= 0x7f;
  ge_ext p1 = elligator(fe_frombytes(t));
  memcpy(t, b + 32, 32); t[31] &= 0x7f;
  ge_ext p2 = elligator(fe_frombytes(t));
  return ge_add(&p1, &p2);
}

/* ------------------------------------------------------------ scalars */
static void to_radix_2w(const uint8_t s[32], unsigned w, int8_t digits[64], unsigned* count) {
  uint64_t x[4];
  memcpy(x, s, 32);
  const uint64_t radix = 1ULL << w, mask = radix - 1;
  unsigned n = (256 + w - 1) / w;
  uint64_t carry = 0;
  memset(digits, 0, 64);
  for (unsigned i = 0; i < n; ++i) {
    unsigned off = i * w, idx = off / 64, bit = off % 64;
    uint64_t buf;
    if (bit < 64 - w || idx == 3) buf = x[idx] >> bit;
    else buf = (x[idx] >> bit) | (x[idx + 1] << (64 - bit));
    uint64_t coef = carry + (buf & mask);
    carry = (coef + radix / 2) >> w;
    digits[i] = (int8_t)((int64_t)coef - (int64_t)(carry << w));
  }
  if (w == 8) { digits[n] += (int8_t)carry; n += 1; }
  else digits[n - 1] += (int8_t)(carry << w);
  *count = n;
}

static void naf5(const uint8_t s[32], int8_t naf[256]) {
  uint64_t x[5] = {0};
  memcpy(x, s, 32);
  const unsigned w = 5;
  const uint64_t width = 1ULL << w, mask = width - 1;
  memset(naf, 0, 256);
  unsigned pos = 0;
  uint64_t carry = 0;
  while (pos < 256) {
    unsigned idx = pos / 64, bit = pos % 64;
    uint64_t buf = (bit < 64 - w) ? (x[idx] >> bit) : ((x[idx] >> bit) | (x[idx + 1] << (64 - bit)));
    uint64_t window = carry + (buf & mask);
    if ((window & 1) == 0) { pos += 1; continue; }
    if (window < width / 2) { carry = 0; naf[pos] = (int8_t)window; }
    else { carry = 1; naf[pos] = (int8_t)((int64_t)window - (int64_t)width); }
    pos += w;
  }
}

/* ------------------------------------------------------------ MSM */
static ge_ext straus_vartime(const uint8_t* scalars, const ge_ext* pts, size_t n) {
  int8_t* nafs = (int8_t*)malloc(256 * (n ? n : 1));
  ge_pniels* tbl = (ge_pniels*)malloc(sizeof(ge_pniels) * 8 * (n ? n : 1));
  for (size_t i = 0; i < n; ++i) {
    naf5(scalars + 32 * i, nafs + 256 * i);
    ge_pniels* t = tbl + 8 * i;
    t[0] = to_pniels(&pts[i]);
    ge_ext P2 = ge_add(&pts[i], &pts[i]);
    for (int k = 0; k < 7; ++k) {
      ge_completed c = ge_add_pn(&P2, &t[k]);
      ge_ext e = completed_to_ext(&c);
      t[k + 1] = to_pniels(&e);
    }
  }
  ge_proj r = ge_proj_identity();
  for (int i = 255; i >= 0; --i) {
    ge_completed t = proj_double(&r);
    for (size_t j = 0; j < n; ++j) {
      int d = nafs[256 * j + i];
      if (d > 0) { ge_ext e = completed_to_ext(&t); t = ge_add_pn(&e, &tbl[8 * j + d / 2]); }
      else if (d < 0) { ge_ext e = completed_to_ext(&t); t = ge_sub_pn(&e, &tbl[8 * j + (-d) / 2]); }
    }
    r = completed_to_proj(&t);
  }
  free(nafs);
  free(tbl);
  return proj_to_ext(&r);
}

static ge_ext pippenger_vartime(const uint8_t* scalars, const ge_ext* pts, size_t n) {
  unsigned w = n < 500 ? 6 : (n < 800 ? 7 : 8);
  unsigned buckets_count = 1u << (w - 1), digits_count = 0;
  int8_t* digits = (int8_t*)malloc(64 * n);
  ge_pniels* pn = (ge_pniels*)malloc(sizeof(ge_pniels) * n);
  for (size_t i = 0; i < n; ++i) {
    to_radix_2w(scalars + 32 * i, w, digits + 64 * i, &digits_count);
    pn[i] = to_pniels(&pts[i]);
  }
  ge_ext* buckets = (ge_ext*)malloc(sizeof(ge_ext) * buckets_count);
  ge_ext total = ge_identity();
  for (int col = (int)digits_count - 1; col >= 0; --col) {
    for (unsigned b = 0; b < buckets_count; ++b) buckets[b] = ge_identity();
    for (size_t i = 0; i < n; ++i) {
      int d = digits[64 * i + col];
      if (d > 0) { ge_completed c = ge_add_pn(&buckets[d - 1], &pn[i]); buckets[d - 1] = completed_to_ext(&c); }
      else if (d < 0) { ge_completed c = ge_sub_pn(&buckets[-d - 1], &pn[i]); buckets[-d - 1] = completed_to_ext(&c); }
    }
    ge_ext inter = buckets[buckets_count - 1], sum = buckets[buckets_count - 1];
    for (int b = (int)buckets_count - 2; b >= 0; --b) {
      inter = ge_add(&inter, &buckets[b]);
      sum = ge_add(&sum, &inter);
    }
    if (col == (int)digits_count - 1) total = sum;
    else { total = ge_mul_pow2(&total, w); total = ge_add(&total, &sum); }
  }
  free(digits);
  free(pn);
  free(buckets);
  return total;
}

/* ------------------------------------------------------------ exported */
int port_from_uniform(const uint8_t* bytes64, size_t n, uint8_t* out32) {
  init_consts();
  for (size_t i = 0; i < n; ++i) {
    ge_ext p = from_uniform(bytes64 + 64 * i);
    ristretto_encode(out32 + 32 * i, &p);
  }
  return 0;
}

static int decode_all(const uint8_t* pts32, size_t n, ge_ext* out) {
  for (size_t i = 0; i < n; ++i)
    if (!ristretto_decode(&out[i], pts32 + 32 * i)) return -(int)(i + 1);
  return 0;
}

/* dalek's dispatch: Straus below 190 terms, Pippenger from 190 up. */
int port_msm(const uint8_t* scalars, const uint8_t* pts32, size_t n, uint8_t out[32]) {
  init_consts();
  ge_ext* P = (ge_ext*)malloc(sizeof(ge_ext) * (n ? n : 1));
  int rc = decode_all(pts32, n, P);
  if (rc == 0) {
    ge_ext r = n < 190 ? straus_vartime(scalars, P, n) : pippenger_vartime(scalars, P, n);
    ristretto_encode(out, &r);
  }
  free(P);
  return rc;
}

/* Times `reps` MSMs over pre-decoded points (decode excluded, as the GPU
 * bench excludes table upload).  Returns elapsed seconds. */
double port_time_msm(const uint8_t* scalars, const uint8_t* pts32, size_t n, int reps, uint8_t out[32]) {
  init_consts();
  ge_ext* P = (ge_ext*)malloc(sizeof(ge_ext) * (n ? n : 1));
  if (decode_all(pts32, n, P) != 0) { free(P); return -1.0; }
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  ge_ext r = ge_identity();
  for (int k = 0; k < reps; ++k) r = n < 190 ? straus_vartime(scalars, P, n) : pippenger_vartime(scalars, P, n);
  clock_gettime(CLOCK_MONOTONIC, &b);
  ristretto_encode(out, &r);
  free(P);
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

int port_encode_basepoint_multiple(uint64_t k, uint8_t out[32]) {
  init_consts();
  static const uint8_t B_ENC[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9,
                                    0x61, 0xc5, 0x00, 0x51, 0x5f, 0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82,
                                    0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
  uint8_t s[32] = {0};
  memcpy(s, &k, 8);
  return port_msm(s, B_ENC, 1, out);
}
