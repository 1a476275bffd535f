// encode_double_batch (host/fe64.h) on eight points at once with AVX-512
// IFMA: the prover's host step of every IPA round encodes its batch's L and
// R (2 x 256 points per round, seven rounds) plus the T and V-x
// commitments, and that encoding was ~25 % of the prover's host CPU samples
// (tools/hostprof, 256-proof batches x 12 in flight).  Same field (radix
// 2^51, five 64-bit limbs, so a lane holds exactly h25519::fe's limbs) and
// the same formulas as the scalar code; the field multiply takes its 25
// limb products from vpmadd52luq / vpmadd52huq (52 x 52 -> low / high 52
// bits): in radix 2^51 the high half of a_i b_j weighs 2^(51 (i + j + 1)) x 2,
// so the high accumulators are doubled once per column.  Callers check
// encode_x8_available() (runtime CPUID; the GPU boxes' EPYC hosts have
// IFMA) and fall back to the scalar loop; both give identical bytes
// (tests/test_host_encode.py runs both).
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "fe64.h"

namespace h25519 {

bool encode_x8_available() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512ifma");
  return ok;
}

#define X8 __attribute__((target("avx512f,avx512ifma"), always_inline)) static inline

namespace {

// eight field elements, lane j of limb i = limb i of element j; every
// function returns limbs < 2^52 (what vpmadd52* reads) holding any value
// mod p (not canonical)
struct F8 {
  __m512i l[5];
};

X8 __m512i m51() { return _mm512_set1_epi64((long long)FE_M51); }
X8 __m512i times19(__m512i x) {  // 19 x = x + 2 x + 16 x
  return _mm512_add_epi64(_mm512_add_epi64(x, _mm512_slli_epi64(x, 1)), _mm512_slli_epi64(x, 4));
}

// limbs < 2^64 -> l0 < 2^51 + 19 * 2^13, the rest < 2^51
X8 F8 carry(F8 a) {
  const __m512i M = m51();
  __m512i c;
  for (int i = 0; i < 4; ++i) {
    c = _mm512_srli_epi64(a.l[i], 51);
    a.l[i] = _mm512_and_si512(a.l[i], M);
    a.l[i + 1] = _mm512_add_epi64(a.l[i + 1], c);
  }
  c = _mm512_srli_epi64(a.l[4], 51);
  a.l[4] = _mm512_and_si512(a.l[4], M);
  a.l[0] = _mm512_add_epi64(a.l[0], times19(c));
  return a;
}

X8 F8 add(const F8& a, const F8& b) {
  F8 r;
  for (int i = 0; i < 5; ++i) r.l[i] = _mm512_add_epi64(a.l[i], b.l[i]);
  return carry(r);
}

// a + 4p - b (4p's limbs exceed any limb < 2^52)
X8 F8 sub(const F8& a, const F8& b) {
  F8 r;
  r.l[0] = _mm512_sub_epi64(_mm512_add_epi64(a.l[0], _mm512_set1_epi64(0x1fffffffffffb4LL)), b.l[0]);
  for (int i = 1; i < 5; ++i)
    r.l[i] = _mm512_sub_epi64(_mm512_add_epi64(a.l[i], _mm512_set1_epi64(0x1ffffffffffffcLL)), b.l[i]);
  return carry(r);
}

X8 F8 neg(const F8& a) {
  F8 z;
  for (int i = 0; i < 5; ++i) z.l[i] = _mm512_setzero_si512();
  return sub(z, a);
}

// Column k of the product collects lo(a_i b_j), i + j = k, and 2 hi(a_i b_j),
// i + j = k - 1 (each < 2^52 for limbs < 2^52): z_k < 2^56; columns 5..9
// fold in with 2^255 = 19 (19 z < 2^61), then one carry pass.
X8 F8 mul(const F8& a, const F8& b) {
  __m512i lo[10], hi[10];
  for (int k = 0; k < 10; ++k) lo[k] = hi[k] = _mm512_setzero_si512();
#pragma GCC unroll 5
  for (int i = 0; i < 5; ++i)
#pragma GCC unroll 5
    for (int j = 0; j < 5; ++j) {
      lo[i + j] = _mm512_madd52lo_epu64(lo[i + j], a.l[i], b.l[j]);
      hi[i + j] = _mm512_madd52hi_epu64(hi[i + j], a.l[i], b.l[j]);
    }
  __m512i z[10];
  z[0] = lo[0];
  for (int k = 1; k < 9; ++k) z[k] = _mm512_add_epi64(lo[k], _mm512_slli_epi64(hi[k - 1], 1));
  z[9] = _mm512_slli_epi64(hi[8], 1);
  F8 r;
  for (int k = 0; k < 5; ++k) r.l[k] = _mm512_add_epi64(z[k], times19(z[k + 5]));
  r = carry(r);
  // l0 < 2^51 + 2^18: one more step keeps every limb < 2^52 for the next multiply
  const __m512i c = _mm512_srli_epi64(r.l[0], 51);
  r.l[0] = _mm512_and_si512(r.l[0], m51());
  r.l[1] = _mm512_add_epi64(r.l[1], c);
  return r;
}

X8 F8 sqn(F8 a, int n) {
  for (int i = 0; i < n; ++i) a = mul(a, a);
  return a;
}

X8 F8 invert(const F8& z) {  // z^(p-2), fe_pow_core's chain
  F8 z2 = mul(z, z);
  F8 z9 = mul(z, sqn(z2, 2));
  F8 z11 = mul(z2, z9);
  F8 z_5_0 = mul(z9, mul(z11, z11));
  F8 z_10_0 = mul(sqn(z_5_0, 5), z_5_0);
  F8 z_20_0 = mul(sqn(z_10_0, 10), z_10_0);
  F8 z_40_0 = mul(sqn(z_20_0, 20), z_20_0);
  F8 z_50_0 = mul(sqn(z_40_0, 10), z_10_0);
  F8 z_100_0 = mul(sqn(z_50_0, 50), z_50_0);
  F8 z_200_0 = mul(sqn(z_100_0, 100), z_100_0);
  F8 z_250_0 = mul(sqn(z_200_0, 50), z_50_0);
  return mul(sqn(z_250_0, 5), z11);
}

// the canonical representative (< p, limbs < 2^51): curve25519-donna's
// fcontract -- two carry passes, + 19, a third, then + 2^255 - 19 with the
// 2^255 dropped
X8 F8 canon(const F8& a) {
  const __m512i M = m51();
  F8 t = carry(carry(a));
  t.l[0] = _mm512_add_epi64(t.l[0], _mm512_set1_epi64(19));
  t = carry(t);
  t.l[0] = _mm512_add_epi64(t.l[0], _mm512_set1_epi64((long long)((1ULL << 51) - 19)));
  for (int i = 1; i < 5; ++i) t.l[i] = _mm512_add_epi64(t.l[i], M);
  for (int i = 0; i < 4; ++i) {
    t.l[i + 1] = _mm512_add_epi64(t.l[i + 1], _mm512_srli_epi64(t.l[i], 51));
    t.l[i] = _mm512_and_si512(t.l[i], M);
  }
  t.l[4] = _mm512_and_si512(t.l[4], M);
  return t;
}

X8 __mmask8 is_zero(const F8& a) {
  const F8 c = canon(a);
  __m512i o = c.l[0];
  for (int i = 1; i < 5; ++i) o = _mm512_or_si512(o, c.l[i]);
  return _mm512_testn_epi64_mask(o, o);
}

X8 __mmask8 is_neg(const F8& a) {
  const F8 c = canon(a);
  return _mm512_test_epi64_mask(c.l[0], _mm512_set1_epi64(1));
}

X8 F8 select(__mmask8 m, const F8& a, const F8& b) {  // m ? b : a, lane by lane
  F8 r;
  for (int i = 0; i < 5; ++i) r.l[i] = _mm512_mask_blend_epi64(m, a.l[i], b.l[i]);
  return r;
}

X8 F8 bcast(const fe& c) {
  F8 r;
  for (int i = 0; i < 5; ++i) r.l[i] = _mm512_set1_epi64((long long)c.v[i]);
  return r;
}

// coordinate `off` (0 X, 1 Y, 2 Z, 3 T) of points p[0..8) into lanes
X8 F8 gather(const ge* p, int off) {
  alignas(64) uint64_t w[5][8];
  for (int j = 0; j < 8; ++j) {
    const fe& f = (&p[j].X)[off];
    for (int i = 0; i < 5; ++i) w[i][j] = f.v[i];
  }
  F8 r;
  for (int i = 0; i < 5; ++i) r.l[i] = _mm512_load_si512(w[i]);
  return r;
}

// p + q in extended coordinates, ge_add's formulas (fe64.h) lane by lane
struct G8 {
  F8 X, Y, Z, T;
};
X8 G8 ge_add8(const G8& p, const G8& q, const F8& D2) {
  const F8 A = mul(sub(p.Y, p.X), sub(q.Y, q.X));
  const F8 B = mul(add(p.Y, p.X), add(q.Y, q.X));
  const F8 C = mul(mul(p.T, D2), q.T);
  const F8 ZZ = mul(p.Z, q.Z);
  const F8 D = add(ZZ, ZZ);
  const F8 E = sub(B, A), F = sub(D, C), G = add(D, C), H = add(B, A);
  return G8{mul(E, F), mul(G, H), mul(F, G), mul(E, H)};
}

X8 G8 gather_ge(const ge* const* p) {
  G8 r;
  F8* f = &r.X;
  for (int off = 0; off < 4; ++off) {
    alignas(64) uint64_t w[5][8];
    for (int j = 0; j < 8; ++j) {
      const fe& c = (&p[j]->X)[off];
      for (int i = 0; i < 5; ++i) w[i][j] = c.v[i];
    }
    for (int i = 0; i < 5; ++i) f[off].l[i] = _mm512_load_si512(w[i]);
  }
  return r;
}

}  // namespace

// out[i] = in[i J] + ... + in[i J + J - 1] for i < n, eight additions per
// vector: each point's J terms are cut into S runs (S the power of two <= J
// that fills the 8 lanes best, J % S == 0), every lane sums one run, and the
// S run sums of a point are added on the scalar path.  The IPA's split
// rounds: config 2 sums 2 x 32 partials per round (62 scalar additions, ~6.5
// us of the host step; here 7 vector additions and 6 scalar ones), a batch
// of 16 proofs 32 x 8.  Same points as the scalar sums (any representative:
// callers encode).
__attribute__((target("avx512f,avx512ifma"))) void ge_sum_x8(const ge* in, size_t n, uint32_t J, ge* out) {
  if (!n) return;
  uint32_t S = 1;
  while (S < J && n * S < 8 && J % (2 * S) == 0) S *= 2;
  const uint32_t Lr = J / S;        // terms per run
  const size_t items = n * S;       // runs
  const F8 D2 = bcast(FE_D2);
  const ge idt = ge_identity();
  std::vector<ge> runs(items);
  for (size_t g0 = 0; g0 < items; g0 += 8) {
    const ge* src[8];
    for (int j = 0; j < 8; ++j) {
      const size_t it = g0 + j;
      src[j] = it < items ? &in[(it / S) * J + (it % S) * Lr] : &idt;
    }
    G8 acc = gather_ge(src);
    for (uint32_t k = 1; k < Lr; ++k) {
      const ge* q[8];
      for (int j = 0; j < 8; ++j) q[j] = g0 + j < items ? src[j] + k : &idt;
      acc = ge_add8(acc, gather_ge(q), D2);
    }
    alignas(64) uint64_t w[4][5][8];
    const F8* f = &acc.X;
    for (int off = 0; off < 4; ++off)
      for (int i = 0; i < 5; ++i) _mm512_store_si512(w[off][i], carry(f[off]).l[i]);
    for (int j = 0; j < 8 && g0 + j < items; ++j) {
      ge& r = runs[g0 + j];
      fe* c = &r.X;
      for (int off = 0; off < 4; ++off)
        for (int i = 0; i < 5; ++i) c[off].v[i] = w[off][i][j];
    }
  }
  for (size_t i = 0; i < n; ++i) {
    ge t = runs[i * S];
    for (uint32_t s = 1; s < S; ++s) t = ge_add(t, runs[i * S + s]);
    out[i] = t;
  }
}

// As encode_double_batch (fe64.h), eight points per vector: one running
// product per lane, one 8-lane inversion for the whole call.
__attribute__((target("avx512f,avx512ifma"))) void encode_double_batch_x8(const ge* pts, size_t n,
                                                                           uint8_t* out) {
  if (!n) return;
  const size_t G = (n + 7) / 8;
  struct St {
    F8 X, Y, Z, T, W, acc;
    __mmask8 zero;
  };
  // (64-byte aligned storage for the vectors: a std::vector of them measured
  // a crash at -O3, aligned loads from a 16-byte-aligned block)
  St* st = static_cast<St*>(aligned_alloc(64, G * sizeof(St)));
  if (!st) {  // (runs on pool threads too: no exception from here)
    encode_double_batch(pts, n, out);
    return;
  }
  const F8 D = bcast(FE_D);
  F8 run = bcast(fe_one());
  ge pad[8];
  for (size_t g = 0; g < G; ++g) {
    const ge* p = pts + 8 * g;
    if (8 * g + 8 > n) {  // the last group: repeat point 0 in the missing lanes
      for (size_t j = 0; j < 8; ++j) pad[j] = 8 * g + j < n ? pts[8 * g + j] : pts[0];
      p = pad;
    }
    const F8 X = gather(p, 0), Y = gather(p, 1), Z = gather(p, 2), T = gather(p, 3);
    const F8 XX = mul(X, X), YY = mul(Y, Y), ZZ = mul(Z, Z), dTT = mul(mul(T, T), D);
    const F8 e = mul(add(X, X), Y);
    const F8 f = add(ZZ, dTT), gg = add(YY, XX), h = sub(ZZ, dTT);
    St& q = st[g];
    q.X = mul(e, h);
    q.Y = mul(gg, f);
    q.Z = mul(f, h);
    q.T = mul(e, gg);
    const F8 W = mul(mul(q.X, q.Y), mul(f, mul(T, Z)));
    q.W = add(W, W);
    q.zero = is_zero(q.W);
    q.acc = run;
    run = select((__mmask8)~q.zero, run, mul(run, q.W));
  }
  F8 inv = invert(run);
  const F8 C_ISQ = bcast(FE_INVSQRT_A_MINUS_D), C_SQRT_M1 = bcast(FE_SQRT_M1);
  for (size_t g = G; g-- > 0;) {
    const St& q = st[g];
    const F8 Winv = mul(inv, q.acc);
    inv = select((__mmask8)~q.zero, inv, mul(inv, q.W));
    F8 isq = mul(C_ISQ, Winv);
    isq = select(is_neg(isq), isq, neg(isq));
    const F8 u1 = mul(add(q.Z, q.Y), sub(q.Z, q.Y));
    const F8 u2 = mul(q.X, q.Y);
    const F8 den1 = mul(isq, u1), den2 = mul(isq, u2);
    const F8 z_inv = mul(mul(den1, den2), q.T);
    const __mmask8 rot = is_neg(mul(q.T, z_inv));
    const F8 x = select(rot, q.X, mul(q.Y, C_SQRT_M1));
    F8 y = select(rot, q.Y, mul(q.X, C_SQRT_M1));
    const F8 den_inv = select(rot, den2, mul(den1, C_ISQ));
    y = select(is_neg(mul(x, z_inv)), y, neg(y));
    F8 s = canon(mul(den_inv, sub(q.Z, y)));
    s = canon(select(_mm512_test_epi64_mask(s.l[0], _mm512_set1_epi64(1)), s, neg(s)));
    alignas(64) uint64_t w[5][8];
    for (int i = 0; i < 5; ++i) _mm512_store_si512(w[i], s.l[i]);
    for (size_t j = 0; j < 8 && 8 * g + j < n; ++j) {
      uint8_t* o = out + 32 * (8 * g + j);
      if ((q.zero >> j) & 1) {
        memset(o, 0, 32);
        continue;
      }
      // canonical limbs -> 32 little-endian bytes
      const uint64_t b0 = w[0][j] | (w[1][j] << 51), b1 = (w[1][j] >> 13) | (w[2][j] << 38),
                     b2 = (w[2][j] >> 26) | (w[3][j] << 25), b3 = (w[3][j] >> 39) | (w[4][j] << 12);
      memcpy(o, &b0, 8);
      memcpy(o + 8, &b1, 8);
      memcpy(o + 16, &b2, 8);
      memcpy(o + 24, &b3, 8);
    }
  }
  free(st);
}

}  // namespace h25519
