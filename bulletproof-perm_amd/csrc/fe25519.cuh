// GF(2^255 - 19) arithmetic for gfx950 (CDNA4), 10 limbs of radix 2^25.5.
//
// Replaces curve25519-dalek-ng 4.1.1's FieldElement51 (u64 serial backend,
// radix 2^51) that the reference reaches through every RistrettoPoint
// operation.  gfx950 has no 64x64 multiply; its
// v_mad_u64_u32 (32x32+64 -> 64, ~4.5 cycles per wave instruction) is the
// workhorse.  Limb i sits at bit ceil(25.5 i) (26 bits even, 25 bits odd),
// so a product column is a chain of v_mad_u64_u32 into one 64-bit
// accumulator that starts from the previous column's carry: no
// add-with-carry instructions (tools/gen_fe10.py generates fe_mul/fe_sq;
// tools/ubench/fe10bench.hip: +17 % multiply and +20 % squaring throughput
// over the round-1 8 x 32-bit Comba, bit-identical results).
//
// Representation invariant ("tight"): limb i < 2^{w_i} + 2^18 (w_i = 26 for
// even i, 25 for odd).  fe_mul / fe_sq accept limbs < 2^27.6 and return tight
// limbs; fe_add / fe_sub / fe_neg carry once and return tight limbs, so every
// value in flight is a valid multiplier operand.  The value is < 2^256 but
// may exceed p; fe_canon gives the unique representative < p with exact
// limb widths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FE_INLINE __device__ __forceinline__
#define FE_LIMBS 10

struct fe {
  uint32_t v[FE_LIMBS];
};

#define MAD64(a, b, c) ((uint64_t)(uint32_t)(a) * (uint64_t)(uint32_t)(b) + (uint64_t)(c))
// (an opaque inline-asm v_mad_u64_u32 for the column chains measured +5-7 %
// multiply throughput at 16 waves/SIMD but 25 % slower on a lone wave, and
// no gain in the MSM: not kept; the compiler re-associates
// each column instead)
#define MADC(a, b, c) MAD64(a, b, c)
#define FE_M26 0x3ffffffu
#define FE_M25 0x1ffffffu

// ---------------------------------------------------------------- helpers
FE_INLINE fe fe_zero() { fe r; _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = 0; return r; }
FE_INLINE fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }
FE_INLINE fe fe_small(uint32_t x) {  // x < 2^26
  fe r = fe_zero();
  r.v[0] = x;
  return r;
}

// One carry pass: limbs < 2^32 in, tight out (limb 0 < 2^26 + 19 * 2^7).
FE_INLINE fe fe_carry(fe a) {
  uint32_t c;
  _Pragma("unroll") for (int i = 0; i < 9; ++i) {
    const int w = (i & 1) ? 25 : 26;
    c = a.v[i] >> w;
    a.v[i] &= (1u << w) - 1u;
    a.v[i + 1] += c;
  }
  c = a.v[9] >> 25;
  a.v[9] &= FE_M25;
  a.v[0] += 19u * c;
  return a;
}

FE_INLINE fe fe_add(const fe& a, const fe& b) {
  fe r;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = a.v[i] + b.v[i];
  return fe_carry(r);
}

// a - b + 2p (each 2p limb exceeds a tight limb), carried
FE_INLINE fe fe_sub(const fe& a, const fe& b) {
  fe r;
  r.v[0] = a.v[0] + 0x7ffffdau - b.v[0];
  _Pragma("unroll") for (int i = 1; i < FE_LIMBS; ++i) r.v[i] = a.v[i] + ((i & 1) ? 0x3fffffeu : 0x7fffffeu) - b.v[i];
  return fe_carry(r);
}

FE_INLINE fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

// Non-carrying forms for the point formulas, where a result only feeds
// multiplier operands (limit 2^27.6): a, b tight ->
//   fe_add_nc < 2^27 + 2^19,  fe_sub_nc < 2^27 + 2^26 + 2^18 (= 2^27.59).
// Neither result may be the subtrahend of a later fe_sub / fe_sub_nc.
FE_INLINE fe fe_add_nc(const fe& a, const fe& b) {
  fe r;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}
FE_INLINE fe fe_sub_nc(const fe& a, const fe& b) {
  fe r;
  r.v[0] = a.v[0] + 0x7ffffdau - b.v[0];
  _Pragma("unroll") for (int i = 1; i < FE_LIMBS; ++i) r.v[i] = a.v[i] + ((i & 1) ? 0x3fffffeu : 0x7fffffeu) - b.v[i];
  return r;
}

#include "fe10_ops.inc"

FE_INLINE fe fe_sqn(fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

// multiply by a small constant k < 2^31
FE_INLINE fe fe_mul_small(const fe& a, uint32_t k) {
  fe r;
  uint64_t acc = 0;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    const int w = (i & 1) ? 25 : 26;
    acc = MAD64(a.v[i], k, acc);
    r.v[i] = (uint32_t)acc & ((1u << w) - 1u);
    acc >>= w;
  }
  // acc < 2^34: bits >= 255, worth 19
  const uint64_t t = MAD64((uint32_t)acc, 19u, (uint64_t)r.v[0]) + ((uint64_t)((uint32_t)(acc >> 32) * 19u) << 32);
  r.v[0] = (uint32_t)t & FE_M26;
  r.v[1] += (uint32_t)(t >> 26);
  return r;
}

// Fully reduce: exact limb widths, value < p.
FE_INLINE fe fe_canon(fe a) {
  a = fe_carry(a);
  a = fe_carry(a);  // limb 0 < 2^26 + 19, others exact
  // exact widths everywhere (limb 0 may still carry 1 into limb 1)
  {
    const uint32_t c = a.v[0] >> 26;
    a.v[0] &= FE_M26;
    a.v[1] += c;
    _Pragma("unroll") for (int i = 1; i < 9; ++i) {
      const int w = (i & 1) ? 25 : 26;
      const uint32_t cc = a.v[i] >> w;
      a.v[i] &= (1u << w) - 1u;
      a.v[i + 1] += cc;
    }
    const uint32_t c9 = a.v[9] >> 25;  // value < 2^255 + 2^26: c9 in {0, 1}
    a.v[9] &= FE_M25;
    a.v[0] += 19u * c9;  // then limb 0 < 2^26 + 19 and value < 2^255
    const uint32_t c0 = a.v[0] >> 26;
    a.v[0] &= FE_M26;
    a.v[1] += c0;  // cannot ripple further: limb 1 was < 2^25 - 1 whenever c0 = 1
  }
  // a >= p  <=>  a + 19 >= 2^255
  uint32_t q = (a.v[0] + 19u) >> 26;
  _Pragma("unroll") for (int i = 1; i < FE_LIMBS; ++i) q = (a.v[i] + q) >> ((i & 1) ? 25 : 26);
  a.v[0] += 19u * q;
  _Pragma("unroll") for (int i = 0; i < 9; ++i) {
    const int w = (i & 1) ? 25 : 26;
    const uint32_t c = a.v[i] >> w;
    a.v[i] &= (1u << w) - 1u;
    a.v[i + 1] += c;
  }
  a.v[9] &= FE_M25;  // drop 2^255 (q * 2^255 subtracted)
  return a;
}

FE_INLINE bool fe_iszero(const fe& a) {
  const fe c = fe_canon(a);
  uint32_t o = 0;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) o |= c.v[i];
  return o == 0;
}

FE_INLINE bool fe_eq(const fe& a, const fe& b) { return fe_iszero(fe_sub(a, b)); }

FE_INLINE bool fe_isneg(const fe& a) { return fe_canon(a).v[0] & 1; }

FE_INLINE fe fe_select(const fe& a, const fe& b, bool pick_b) {
  fe r;
  const uint32_t m = 0u - (uint32_t)pick_b;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = (a.v[i] & ~m) | (b.v[i] & m);
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
// 8 little-endian 32-bit words (any value < 2^256; bit 255 is worth 19)
FE_INLINE fe fe_load_words(const uint32_t* w) {
  fe r;
  const int OFF[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    const int o = OFF[i], q = o >> 5, s = o & 31, wd = (i & 1) ? 25 : 26;
    uint64_t x = w[q];
    if (q + 1 < 8) x |= (uint64_t)w[q + 1] << 32;
    r.v[i] = (uint32_t)(x >> s) & ((1u << wd) - 1u);
  }
  r.v[0] += 19u * (w[7] >> 31);
  return r;
}

// canonical 8 x 32-bit words
FE_INLINE void fe_store_words(uint32_t* w, const fe& x) {
  const fe a = fe_canon(x);
  const int OFF[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  uint32_t o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    const int q = OFF[i] >> 5, s = OFF[i] & 31;
    const uint64_t t = (uint64_t)a.v[i] << s;
    o[q] |= (uint32_t)t;
    if (q + 1 < 8) o[q + 1] |= (uint32_t)(t >> 32);
  }
  _Pragma("unroll") for (int i = 0; i < 8; ++i) w[i] = o[i];
}

// 32-byte encoding (8 LE words) is canonical: value < p
FE_INLINE bool fe_words_canonical(const uint32_t* w) {
  if (w[7] < 0x7fffffffu) return true;
  if (w[7] > 0x7fffffffu) return false;
  _Pragma("unroll") for (int i = 6; i >= 1; --i) if (w[i] != 0xffffffffu) return true;
  return w[0] < 0xffffffedu;
}

// ---------------------------------------------------------------- constants
// (10-limb radix-2^25.5, canonical; generated from oracle/ristretto.py)
__device__ __constant__ static const uint32_t FE_D[10] = {0x35978a3u, 0x0d37284u, 0x3156ebdu, 0x06a0a0eu, 0x001c029u, 0x179e898u, 0x3a03cbbu, 0x1ce7198u, 0x2e2b6ffu, 0x1480db3u};
__device__ __constant__ static const uint32_t FE_D2[10] = {0x2b2f159u, 0x1a6e509u, 0x22add7au, 0x0d4141du, 0x0038052u, 0x0f3d130u, 0x3407977u, 0x19ce331u, 0x1c56dffu, 0x0901b67u};
__device__ __constant__ static const uint32_t FE_SQRT_M1[10] = {0x20ea0b0u, 0x186c9d2u, 0x08f189du, 0x035697fu, 0x0bd0c60u, 0x1fbd7a7u, 0x2804c9eu, 0x1e16569u, 0x004fc1du, 0x0ae0c92u};
__device__ __constant__ static const uint32_t FE_INVSQRT_A_MINUS_D[10] = {0x05d40eau, 0x03f6aa0u, 0x257d339u, 0x0bad20bu, 0x274bc58u, 0x001d840u, 0x13dc8ffu, 0x19442d8u, 0x05cfaffu, 0x1e1b224u};
__device__ __constant__ static const uint32_t FE_SQRT_AD_MINUS_ONE[10] = {0x17b2e1bu, 0x1fda812u, 0x297afd2u, 0x060dbc2u, 0x2be7638u, 0x1f5d1fdu, 0x27e6498u, 0x11581e7u, 0x3f2b834u, 0x0dda4c6u};
__device__ __constant__ static const uint32_t FE_ONE_MINUS_D_SQ[10] = {0x05fc176u, 0x1027065u, 0x2a1fc4fu, 0x1c66af1u, 0x0b20684u, 0x070dfe4u, 0x255eedfu, 0x01af332u, 0x28b2b3eu, 0x00a41cau};
__device__ __constant__ static const uint32_t FE_D_MINUS_ONE_SQ[10] = {0x0ed4d20u, 0x156aa91u, 0x3332635u, 0x16580f0u, 0x34a7928u, 0x09b4eebu, 0x26997a9u, 0x048299bu, 0x3af66c2u, 0x165a2cdu};

FE_INLINE fe fe_const(const uint32_t* c) {
  fe r;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = c[i];
  return r;
}
