// GF(2^255 - 19) arithmetic for gfx950 (CDNA4), 8 x 32-bit limbs.
//
// Replaces curve25519-dalek-ng 4.1.1's FieldElement51 (u64 serial backend,
// radix 2^51) that the reference reaches through every RistrettoPoint
// operation.  gfx950 has no 64x64 multiply; the
// measured rates (tools/ubench/intrate.hip, profiles/r01_intrate.txt) are
// v_mad_u64_u32 ~4.5 cycles / wave-instruction vs ~2.4 for v_add_u32, so
// the multiply is a Comba product scan built from v_mad_u64_u32 whose
// carry-out feeds a v_addc_co_u32 (2 instructions per 32x32 limb product).
//
// Representation invariant ("loose"): limbs hold any value < 2^256; every
// operation returns a value < 2^256 that is congruent mod p.  Canonical
// form (< p) is produced only by fe_canon / fe_tobytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FE_INLINE __device__ __forceinline__

struct fe {
  uint32_t v[8];
};

// ---------------------------------------------------------------- helpers
FE_INLINE fe fe_zero() { fe r; _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = 0; return r; }
FE_INLINE fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }
FE_INLINE fe fe_small(uint32_t x) { fe r = fe_zero(); r.v[0] = x; return r; }

// r = (value < 2^256 + 2^256*top) folded: returns low 255 bits + 19*(bits >= 255)
// `top` is the word of weight 2^256 (small).
FE_INLINE fe fe_fold(fe a, uint32_t top) {
  uint32_t hi = (top << 1) | (a.v[7] >> 31);
  a.v[7] &= 0x7fffffffu;
  uint64_t c = (uint64_t)a.v[0] + (uint64_t)hi * 19u;
  a.v[0] = (uint32_t)c;
  _Pragma("unroll") for (int i = 1; i < 8; ++i) {
    c = (uint64_t)a.v[i] + (c >> 32);
    a.v[i] = (uint32_t)c;
  }
  return a;  // < 2^255 + 2^37 (cannot carry past bit 255 twice)
}

FE_INLINE fe fe_add(const fe& a, const fe& b) {
  fe r;
  uint64_t c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    c = (uint64_t)a.v[i] + b.v[i] + (c >> 32);
    r.v[i] = (uint32_t)c;
  }
  return fe_fold(r, (uint32_t)(c >> 32));
}

// a - b computed as a + (4p - b); 4p = 2^257 - 76 > any loose b.
FE_INLINE fe fe_sub(const fe& a, const fe& b) {
  // 4p limbs: [0xffffffb4, 0xffffffff x7] with an extra top word 1.
  fe r;
  int64_t c = 0;
  // t = 4p - b (9 limbs, non-negative), then r = a + t
  uint64_t s = 0;
  uint32_t t[8];
  {
    int64_t bw = (int64_t)0xffffffb4u - (int64_t)b.v[0];
    t[0] = (uint32_t)bw;
    bw >>= 32;
    _Pragma("unroll") for (int i = 1; i < 8; ++i) {
      bw = (int64_t)0xffffffffu - (int64_t)b.v[i] + bw;
      t[i] = (uint32_t)bw;
      bw >>= 32;
    }
    c = 1 + bw;  // top word of t (0 or 1)
  }
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    s = (uint64_t)a.v[i] + t[i] + (s >> 32);
    r.v[i] = (uint32_t)s;
  }
  return fe_fold(r, (uint32_t)(s >> 32) + (uint32_t)c);
}

FE_INLINE fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

// 96-bit column accumulator step: {hi:acc} += a*b, via v_mad_u64_u32's
// carry-out feeding v_addc_co_u32.
#define FE_MAC(acc, hi, a, b)                                              \
  do {                                                                     \
    uint64_t _cc;                                                          \
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"                             \
        "v_addc_co_u32 %2, %1, %2, 0, %1"                                  \
        : "+v"(acc), "=&s"(_cc), "+v"(hi)                                  \
        : "v"(a), "v"(b));                                                 \
  } while (0)

// Reduce a 512-bit product t[0..15] to a loose element: lo + 38*hi.
FE_INLINE fe fe_reduce512(const uint32_t t[16]) {
  fe r;
  uint64_t c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    c = (uint64_t)t[8 + i] * 38u + (uint64_t)t[i] + (c >> 32);
    r.v[i] = (uint32_t)c;
  }
  return fe_fold(r, (uint32_t)(c >> 32));
}

FE_INLINE fe fe_mul(const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t hi = 0;
  _Pragma("unroll") for (int k = 0; k < 15; ++k) {
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 8) FE_MAC(acc, hi, a.v[i], b.v[j]);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[15] = (uint32_t)acc;
  return fe_reduce512(t);
}

// Squaring: cross products once, doubled, plus the diagonal.
FE_INLINE fe fe_sq(const fe& a) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t hi = 0;
  t[0] = 0;
  _Pragma("unroll") for (int k = 1; k < 14; ++k) {
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (j > i && j < 8) FE_MAC(acc, hi, a.v[i], a.v[j]);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[14] = (uint32_t)acc;
  t[15] = (uint32_t)(acc >> 32);
  // double (cross terms < 2^511, so the doubled value fits in 512 bits)
  _Pragma("unroll") for (int k = 15; k > 0; --k) t[k] = (t[k] << 1) | (t[k - 1] >> 31);
  t[0] = 0;
  // add diagonal a_i^2 at position 2i
  uint64_t c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    uint64_t sq = (uint64_t)a.v[i] * a.v[i];
    c = (uint64_t)t[2 * i] + (uint32_t)sq + (c >> 32);
    t[2 * i] = (uint32_t)c;
    c = (uint64_t)t[2 * i + 1] + (uint32_t)(sq >> 32) + (c >> 32);
    t[2 * i + 1] = (uint32_t)c;
  }
  return fe_reduce512(t);
}

FE_INLINE fe fe_sqn(fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

// multiply by a small constant (< 2^31)
FE_INLINE fe fe_mul_small(const fe& a, uint32_t k) {
  fe r;
  uint64_t c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    c = (uint64_t)a.v[i] * k + (c >> 32);
    r.v[i] = (uint32_t)c;
  }
  // top word < 2^31: fold twice
  uint32_t top = (uint32_t)(c >> 32);
  uint64_t d = (uint64_t)r.v[0] + (uint64_t)top * 38u;
  r.v[0] = (uint32_t)d;
  _Pragma("unroll") for (int i = 1; i < 8; ++i) {
    d = (uint64_t)r.v[i] + (d >> 32);
    r.v[i] = (uint32_t)d;
  }
  return fe_fold(r, (uint32_t)(d >> 32));
}

// Fully reduce to [0, p).
FE_INLINE fe fe_canon(fe a) {
  a = fe_fold(a, 0);  // < 2^255 + 2^37 < 2p
  // subtract p if a >= p: compute a + 19 and look at bit 255
  uint64_t c = (uint64_t)a.v[0] + 19u;
  uint32_t t[8];
  t[0] = (uint32_t)c;
  _Pragma("unroll") for (int i = 1; i < 8; ++i) {
    c = (uint64_t)a.v[i] + (c >> 32);
    t[i] = (uint32_t)c;
  }
  const uint32_t ge = t[7] >> 31;  // a + 19 >= 2^255  <=> a >= p
  const uint32_t m = 0u - ge;
  t[7] &= 0x7fffffffu;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) a.v[i] = (t[i] & m) | (a.v[i] & ~m);
  return a;
}

FE_INLINE bool fe_iszero(const fe& a) {
  fe c = fe_canon(a);
  uint32_t o = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) o |= c.v[i];
  return o == 0;
}

FE_INLINE bool fe_eq(const fe& a, const fe& b) { return fe_iszero(fe_sub(a, b)); }

FE_INLINE bool fe_isneg(const fe& a) { return fe_canon(a).v[0] & 1; }

FE_INLINE fe fe_select(const fe& a, const fe& b, bool pick_b) {
  fe r;
  const uint32_t m = 0u - (uint32_t)pick_b;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = (a.v[i] & ~m) | (b.v[i] & m);
  return r;
}

FE_INLINE fe fe_abs(const fe& a) { return fe_select(a, fe_neg(a), fe_isneg(a)); }

// z^(2^250 - 1) and z^11 helpers (standard curve25519 addition chain)
FE_INLINE void fe_pow_core(const fe& z, fe& z_250_0, fe& z11) {
  fe z2 = fe_sq(z);
  fe z8 = fe_sqn(z2, 2);
  fe z9 = fe_mul(z, z8);
  z11 = fe_mul(z2, z9);
  fe z22 = fe_sq(z11);
  fe z_5_0 = fe_mul(z9, z22);
  fe z_10_0 = fe_mul(fe_sqn(z_5_0, 5), z_5_0);
  fe z_20_0 = fe_mul(fe_sqn(z_10_0, 10), z_10_0);
  fe z_40_0 = fe_mul(fe_sqn(z_20_0, 20), z_20_0);
  fe z_50_0 = fe_mul(fe_sqn(z_40_0, 10), z_10_0);
  fe z_100_0 = fe_mul(fe_sqn(z_50_0, 50), z_50_0);
  fe z_200_0 = fe_mul(fe_sqn(z_100_0, 100), z_100_0);
  z_250_0 = fe_mul(fe_sqn(z_200_0, 50), z_50_0);
}

// z^(p-2)
FE_INLINE fe fe_invert(const fe& z) {
  fe z_250_0, z11;
  fe_pow_core(z, z_250_0, z11);
  return fe_mul(fe_sqn(z_250_0, 5), z11);
}

// z^((p-5)/8) = z^(2^252 - 3)
FE_INLINE fe fe_pow22523(const fe& z) {
  fe z_250_0, z11;
  fe_pow_core(z, z_250_0, z11);
  return fe_mul(fe_sqn(z_250_0, 2), z);
}

// ---------------------------------------------------------------- bytes
FE_INLINE fe fe_load_words(const uint32_t* w) {
  fe r;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = w[i];
  return r;
}
FE_INLINE void fe_store_words(uint32_t* w, const fe& a) {
  _Pragma("unroll") for (int i = 0; i < 8; ++i) w[i] = a.v[i];
}

// ---------------------------------------------------------------- constants
// (little-endian 32-bit limbs, canonical)
__device__ __constant__ static const uint32_t FE_D[8] = {0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du, 0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu};
__device__ __constant__ static const uint32_t FE_D2[8] = {0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au, 0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu};
__device__ __constant__ static const uint32_t FE_SQRT_M1[8] = {0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u, 0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};
__device__ __constant__ static const uint32_t FE_INVSQRT_A_MINUS_D[8] = {0x805d40eau, 0x99c8fdaau, 0x5a4172beu, 0x9d2f1617u, 0xfe01d840u, 0x16c27b91u, 0xcfaffca2u, 0x786c8905u};
__device__ __constant__ static const uint32_t FE_SQRT_AD_MINUS_ONE[8] = {0x497b2e1bu, 0x7e97f6a0u, 0x1b7854bdu, 0xaf9d8e0cu, 0x31f5d1fdu, 0x0f3cfcc9u, 0x2b8348acu, 0x376931bfu};
__device__ __constant__ static const uint32_t FE_ONE_MINUS_D_SQ[8] = {0x945fc176u, 0xe27c09c1u, 0xcd5e350fu, 0x2c81a138u, 0xbe70dfe4u, 0x9994abddu, 0xb2b3e0d7u, 0x029072a8u};
__device__ __constant__ static const uint32_t FE_D_MINUS_ONE_SQ[8] = {0x44ed4d20u, 0x31ad5aaau, 0xb01e1999u, 0xd29e4a2cu, 0x529b4eebu, 0x4cdcd32fu, 0xf66c2241u, 0x5968b37au};

FE_INLINE fe fe_const(const uint32_t* c) { return fe_load_words(c); }
