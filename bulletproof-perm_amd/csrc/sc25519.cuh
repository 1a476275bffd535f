// Scalar field Z/lZ on gfx950: Montgomery (R = 2^256), 8 x 32-bit storage.
//
// Device counterpart of dalek's `Scalar` for the data-parallel scalar work
// of the inner-product argument (bulletproofs 4.0.0 InnerProductProof: the
// a/b folds a' = a_lo*u + u^-1*a_hi, b' = b_lo*u^-1 + u*b_hi and the cross
// inner products c_L, c_R) and of the proof's vector polynomials.
// Values in Montgomery form (x*R mod l) unless a name says otherwise.
#pragma once
#include "fe25519.cuh"

struct sc {
  uint32_t v[8];
};

__device__ __constant__ static const uint32_t SC_L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                                                          0x00000000u, 0x00000000u, 0x00000000u, 0x10000000u};
__device__ __constant__ static const uint32_t SC_R2[8] = {0x449c0f01u, 0xa40611e3u, 0x68859347u, 0xd00e1ba7u,
                                                           0x17f5be65u, 0xceec73d2u, 0x7c309a3du, 0x0399411bu};
#define SC_LINV 0x12547e1bu

FE_INLINE sc sc_zero() { sc r; _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = 0; return r; }

FE_INLINE bool sc_geq_l(const uint32_t a[8]) {
  _Pragma("unroll") for (int i = 7; i >= 0; --i) {
    if (a[i] != SC_L[i]) return a[i] > SC_L[i];
  }
  return true;
}

FE_INLINE void sc_sub_l(uint32_t a[8]) {
  int64_t br = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    int64_t d = (int64_t)a[i] - (int64_t)SC_L[i] + br;
    a[i] = (uint32_t)d;
    br = d >> 32;
  }
}

FE_INLINE sc sc_add(const sc& a, const sc& b) {
  sc r;
  uint64_t c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    c = (uint64_t)a.v[i] + b.v[i] + (c >> 32);
    r.v[i] = (uint32_t)c;
  }
  if (sc_geq_l(r.v)) sc_sub_l(r.v);
  return r;
}

FE_INLINE sc sc_sub(const sc& a, const sc& b) {
  sc r;
  int64_t br = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    int64_t d = (int64_t)a.v[i] - (int64_t)b.v[i] + br;
    r.v[i] = (uint32_t)d;
    br = d >> 32;
  }
  if (br) {
    uint64_t c = 0;
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      c = (uint64_t)r.v[i] + SC_L[i] + (c >> 32);
      r.v[i] = (uint32_t)c;
    }
  }
  return r;
}

FE_INLINE sc sc_neg(const sc& a) { return sc_sub(sc_zero(), a); }

// a*b*R^-1 mod l (R = 2^256); requires a*b < l*R (true for a, b < 2^256
// when one is < l); canonical result.
//
// Radix 2^29 inside: 32 a and b as 9 limbs of 29 bits, the 17 product
// columns as plain v_mad_u64_u32 sums (each < 18 * 2^58 with the reduction
// terms: no carries while accumulating), then Montgomery reduction by 2^29
// per step with R' = 2^261 -- mont'(32 a, b) = a b 2^-256.  The columns are
// independent chains, and a reduction step waits only on the previous
// step's carry, where sc_mont_cios's carries serialize all ~130
// multiply-adds: a lone wave (the prover's per-proof scalar kernels) runs
// the product several times faster (tools/ubench/scbench.hip).
// l's 29-bit limbs 5..7 are zero, so a reduction step is 6 multiply-adds.
__device__ __constant__ static const uint32_t SC_L29[9] = {0x1cf5d3edu, 0x009318d2u, 0x1de73596u, 0x1df3bd45u, 0x0000014du,
                                                            0u, 0u, 0u, 0x00100000u};
#define SC_M29 0x1fffffffu
FE_INLINE void sc_to29(const uint32_t w[8], uint32_t sh, uint32_t r[9]) {  // (w << sh) in 29-bit limbs, sh < 29
  _Pragma("unroll") for (int k = 0; k < 9; ++k) {
    // bits [29 k - sh, 29 k - sh + 29) of w
    const int lo = 29 * k - (int)sh;
    uint64_t x;
    if (lo < 0) {
      x = (uint64_t)w[0] << (-lo);
    } else {
      const int q = lo >> 5, b = lo & 31;
      x = (uint64_t)w[q] >> b;
      if (q + 1 < 8) x |= (uint64_t)w[q + 1] << (32 - b);
    }
    r[k] = (uint32_t)x & SC_M29;
  }
}
FE_INLINE sc sc_mont(const sc& a, const sc& b) {
  uint32_t A[9], B[9];
  sc_to29(a.v, 5, A);
  sc_to29(b.v, 0, B);
  uint64_t col[17];
  _Pragma("unroll") for (int k = 0; k < 17; ++k) {
    uint64_t c = 0;
    _Pragma("unroll") for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 9) c = (uint64_t)A[i] * B[j] + c;
    }
    col[k] = c;
  }
  _Pragma("unroll") for (int i = 0; i < 9; ++i) {
    const uint32_t m = ((uint32_t)col[i] * SC_LINV) & SC_M29;
    _Pragma("unroll") for (int j = 0; j < 9; ++j)
      if (SC_L29[j] != 0 && i + j < 17) col[i + j] = (uint64_t)m * SC_L29[j] + col[i + j];
    if (i + 1 < 17) col[i + 1] += col[i] >> 29;
  }
  // r = col[9..16] normalized (< 2 l < 2^254), as 8 x 32-bit words
  uint32_t r29[9];
  uint64_t c = 0;
  _Pragma("unroll") for (int k = 0; k < 8; ++k) {
    c += col[9 + k];
    r29[k] = (uint32_t)c & SC_M29;
    c >>= 29;
  }
  r29[8] = (uint32_t)c;
  sc r;
  _Pragma("unroll") for (int w = 0; w < 8; ++w) {
    const int lo = 32 * w, k = lo / 29, b = lo % 29;
    uint64_t x = (uint64_t)r29[k] >> b;
    if (k + 1 < 9) x |= (uint64_t)r29[k + 1] << (29 - b);
    if (k + 2 < 9 && 58 - b < 32) x |= (uint64_t)r29[k + 2] << (58 - b);
    r.v[w] = (uint32_t)x;
  }
  if (sc_geq_l(r.v)) sc_sub_l(r.v);
  return r;
}

// The same product by CIOS over 8 x 32-bit words (the round-1 form, kept as
// the reference of tests / tools/ubench/scbench.hip): every multiply-add of
// a row waits for the previous one's carry, a ~130-deep chain.
FE_INLINE sc sc_mont_cios(const sc& a, const sc& b) {
  uint32_t t[10];
  _Pragma("unroll") for (int i = 0; i < 10; ++i) t[i] = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {
      c = (uint64_t)a.v[i] * b.v[j] + t[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
    c = (uint64_t)t[8] + (c >> 32);
    t[8] = (uint32_t)c;
    t[9] = (uint32_t)(c >> 32);
    const uint32_t m = t[0] * SC_LINV;
    c = (uint64_t)m * SC_L[0] + t[0];
    _Pragma("unroll") for (int j = 1; j < 8; ++j) {
      c = (uint64_t)m * SC_L[j] + t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    c = (uint64_t)t[8] + (c >> 32);
    t[7] = (uint32_t)c;
    t[8] = t[9] + (uint32_t)(c >> 32);
  }
  sc r;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = t[i];
  if (t[8] || sc_geq_l(r.v)) sc_sub_l(r.v);
  return r;
}

// a / 2 mod l for canonical a: (a + (a odd ? l : 0)) >> 1 (a + l < 2^254)
FE_INLINE sc sc_half(const sc& a) {
  const uint32_t odd = a.v[0] & 1u;
  sc r;
  uint64_t c = 0;
  _Pragma("unroll") for (int k = 0; k < 8; ++k) {
    c += (uint64_t)a.v[k] + (odd ? SC_L[k] : 0u);
    r.v[k] = (uint32_t)c;
    c >>= 32;
  }
  _Pragma("unroll") for (int k = 0; k < 7; ++k) r.v[k] = (r.v[k] >> 1) | (r.v[k + 1] << 31);
  r.v[7] >>= 1;
  return r;
}

FE_INLINE sc sc_load(const uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  sc r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}

FE_INLINE void sc_store(uint32_t* p, const sc& a) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  q[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}

// canonical -> Montgomery and back
FE_INLINE sc sc_to_mont(const sc& a) {
  sc r2;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r2.v[i] = SC_R2[i];
  return sc_mont(a, r2);
}
FE_INLINE sc sc_from_mont(const sc& a) {
  sc one = sc_zero();
  one.v[0] = 1;
  return sc_mont(a, one);
}

FE_INLINE sc sc_one_mont() {
  sc one = sc_zero();
  one.v[0] = 1;
  return sc_to_mont(one);
}

// canonical w mod l for w < 2^256: w = q 2^252 + rest (q < 16), w - q l =
// rest - q delta is in (-l, 2^252), one conditional addition of l
FE_INLINE sc sc_reduce256(const uint32_t w[8]) {
  const uint32_t q = w[7] >> 28;
  sc r;
  uint64_t pc = 0;   // q * l carry
  uint32_t br = 0;   // borrow
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    const uint64_t pr = (uint64_t)q * SC_L[i] + pc;
    pc = pr >> 32;
    const uint64_t d = (uint64_t)w[i] - (uint32_t)pr - br;
    r.v[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  if (br) {
    uint64_t c = 0;
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      c += (uint64_t)r.v[i] + SC_L[i];
      r.v[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  return r;
}

// Scalar::from_bytes_mod_order_wide of 16 little-endian words, canonical:
// x = lo + hi 2^256 = lo + hi R, and mont(hi, R^2) = hi R (mod l)
FE_INLINE sc sc_from_wide_w(const uint32_t* __restrict__ w) {
  sc hi, r2;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    hi.v[i] = w[8 + i];
    r2.v[i] = SC_R2[i];
  }
  uint32_t lo[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) lo[i] = w[i];
  return sc_add(sc_reduce256(lo), sc_mont(hi, r2));
}

// 64-lane wave reduction of a Montgomery scalar sum (result valid in lane 0)
FE_INLINE sc sc_wave_sum(sc a) {
  _Pragma("unroll") for (int d = 32; d >= 1; d >>= 1) {
    sc o;
    _Pragma("unroll") for (int i = 0; i < 8; ++i) o.v[i] = __shfl_down(a.v[i], d, 64);
    a = sc_add(a, o);
  }
  return a;
}

// value of lane src of the wave
FE_INLINE sc sc_shfl(const sc& a, int src) {
  sc r;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = __shfl(a.v[i], src, 64);
  return r;
}
