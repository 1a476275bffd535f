// Frozen copy of the 8 x 32-bit Comba field (round-1 design, replaced by the
// 10-limb radix-2^25.5 field in csrc/fe25519.cuh); kept as the baseline for
// tools/ubench/fe10bench.hip.
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

// 32-bit carry chains (v_add_co_u32 / v_addc_co_u32, v_sub_co / v_subb):
// no 64-bit zero-extended temporaries, so no register-pair copies.
#define ADDC(x, y, ci, co) __builtin_addc((x), (y), (ci), (co))
#define SUBC(x, y, bi, bo) __builtin_subc((x), (y), (bi), (bo))

// r += k (k small), carry out returned
FE_INLINE uint32_t fe_add_small(fe& r, uint32_t k) {
  uint32_t c;
  r.v[0] = ADDC(r.v[0], k, 0u, &c);
  _Pragma("unroll") for (int i = 1; i < 8; ++i) r.v[i] = ADDC(r.v[i], 0u, c, &c);
  return c;
}

// value = a + top * 2^256 (top small): fold bits >= 255 back with 2^255 = 19
FE_INLINE fe fe_fold(fe a, uint32_t top) {
  const uint32_t hi = (top << 1) | (a.v[7] >> 31);
  a.v[7] &= 0x7fffffffu;
  (void)fe_add_small(a, hi * 19u);
  return a;  // < 2^255 + 2^12
}

// a + b mod p, loose: a carry out of 2^256 is worth 38 (folded twice; the
// second fold can only touch limb 0).  Inline asm so that the carry chain
// stays in one SGPR pair with no compiler padding: hipcc pads every
// VCC-carried v_addc with s_nop 1 on gfx950, which measured unnecessary
// (tools/ubench/carrychain.hip: 0 errors in 3.4e9 words, both carry forms).
FE_INLINE fe fe_add(const fe& a, const fe& b) {
  fe r;
  uint32_t t;
  uint64_t c;
  asm("v_add_co_u32 %[r0], %[c], %[a0], %[b0]\n\t"
      "v_addc_co_u32 %[r1], %[c], %[a1], %[b1], %[c]\n\t"
      "v_addc_co_u32 %[r2], %[c], %[a2], %[b2], %[c]\n\t"
      "v_addc_co_u32 %[r3], %[c], %[a3], %[b3], %[c]\n\t"
      "v_addc_co_u32 %[r4], %[c], %[a4], %[b4], %[c]\n\t"
      "v_addc_co_u32 %[r5], %[c], %[a5], %[b5], %[c]\n\t"
      "v_addc_co_u32 %[r6], %[c], %[a6], %[b6], %[c]\n\t"
      "v_addc_co_u32 %[r7], %[c], %[a7], %[b7], %[c]\n\t"
      "v_cndmask_b32 %[t], 0, 38, %[c]\n\t"
      "v_add_co_u32 %[r0], %[c], %[r0], %[t]\n\t"
      "v_addc_co_u32 %[r1], %[c], %[r1], 0, %[c]\n\t"
      "v_addc_co_u32 %[r2], %[c], %[r2], 0, %[c]\n\t"
      "v_addc_co_u32 %[r3], %[c], %[r3], 0, %[c]\n\t"
      "v_addc_co_u32 %[r4], %[c], %[r4], 0, %[c]\n\t"
      "v_addc_co_u32 %[r5], %[c], %[r5], 0, %[c]\n\t"
      "v_addc_co_u32 %[r6], %[c], %[r6], 0, %[c]\n\t"
      "v_addc_co_u32 %[r7], %[c], %[r7], 0, %[c]\n\t"
      "v_cndmask_b32 %[t], 0, 38, %[c]\n\t"
      "v_add_u32 %[r0], %[r0], %[t]"
      : [r0] "=&v"(r.v[0]), [r1] "=&v"(r.v[1]), [r2] "=&v"(r.v[2]), [r3] "=&v"(r.v[3]), [r4] "=&v"(r.v[4]),
        [r5] "=&v"(r.v[5]), [r6] "=&v"(r.v[6]), [r7] "=&v"(r.v[7]), [t] "=&v"(t), [c] "=&s"(c)
      : [a0] "v"(a.v[0]), [a1] "v"(a.v[1]), [a2] "v"(a.v[2]), [a3] "v"(a.v[3]), [a4] "v"(a.v[4]),
        [a5] "v"(a.v[5]), [a6] "v"(a.v[6]), [a7] "v"(a.v[7]), [b0] "v"(b.v[0]), [b1] "v"(b.v[1]),
        [b2] "v"(b.v[2]), [b3] "v"(b.v[3]), [b4] "v"(b.v[4]), [b5] "v"(b.v[5]), [b6] "v"(b.v[6]),
        [b7] "v"(b.v[7]));
  return r;
}

// a - b mod p, loose: a borrow out of 2^256 is worth -38 (twice at most;
// after the first, r >= 2^256 - 38 unless r < 38, so the second fold can
// borrow only when r wrapped and then cannot borrow again).
FE_INLINE fe fe_sub(const fe& a, const fe& b) {
  fe r;
  uint32_t t;
  uint64_t c;
  asm("v_sub_co_u32 %[r0], %[c], %[a0], %[b0]\n\t"
      "v_subb_co_u32 %[r1], %[c], %[a1], %[b1], %[c]\n\t"
      "v_subb_co_u32 %[r2], %[c], %[a2], %[b2], %[c]\n\t"
      "v_subb_co_u32 %[r3], %[c], %[a3], %[b3], %[c]\n\t"
      "v_subb_co_u32 %[r4], %[c], %[a4], %[b4], %[c]\n\t"
      "v_subb_co_u32 %[r5], %[c], %[a5], %[b5], %[c]\n\t"
      "v_subb_co_u32 %[r6], %[c], %[a6], %[b6], %[c]\n\t"
      "v_subb_co_u32 %[r7], %[c], %[a7], %[b7], %[c]\n\t"
      "v_cndmask_b32 %[t], 0, 38, %[c]\n\t"
      "v_sub_co_u32 %[r0], %[c], %[r0], %[t]\n\t"
      "v_subb_co_u32 %[r1], %[c], %[r1], 0, %[c]\n\t"
      "v_subb_co_u32 %[r2], %[c], %[r2], 0, %[c]\n\t"
      "v_subb_co_u32 %[r3], %[c], %[r3], 0, %[c]\n\t"
      "v_subb_co_u32 %[r4], %[c], %[r4], 0, %[c]\n\t"
      "v_subb_co_u32 %[r5], %[c], %[r5], 0, %[c]\n\t"
      "v_subb_co_u32 %[r6], %[c], %[r6], 0, %[c]\n\t"
      "v_subb_co_u32 %[r7], %[c], %[r7], 0, %[c]\n\t"
      "v_cndmask_b32 %[t], 0, 38, %[c]\n\t"
      "v_sub_u32 %[r0], %[r0], %[t]"
      : [r0] "=&v"(r.v[0]), [r1] "=&v"(r.v[1]), [r2] "=&v"(r.v[2]), [r3] "=&v"(r.v[3]), [r4] "=&v"(r.v[4]),
        [r5] "=&v"(r.v[5]), [r6] "=&v"(r.v[6]), [r7] "=&v"(r.v[7]), [t] "=&v"(t), [c] "=&s"(c)
      : [a0] "v"(a.v[0]), [a1] "v"(a.v[1]), [a2] "v"(a.v[2]), [a3] "v"(a.v[3]), [a4] "v"(a.v[4]),
        [a5] "v"(a.v[5]), [a6] "v"(a.v[6]), [a7] "v"(a.v[7]), [b0] "v"(b.v[0]), [b1] "v"(b.v[1]),
        [b2] "v"(b.v[2]), [b3] "v"(b.v[3]), [b4] "v"(b.v[4]), [b5] "v"(b.v[5]), [b6] "v"(b.v[6]),
        [b7] "v"(b.v[7]));
  return r;
}

FE_INLINE fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

// Reduce a 512-bit product t[0..15] to a loose element: lo + 38*hi, then
// fold bits >= 255 (2^255 = 19).  Products 38*t_{8+i} as 64-bit pairs (the
// halves feed the asm chain without copies); one SGPR carry throughout.
FE_INLINE fe fe_reduce512(const uint32_t t[16]) {
  uint64_t p[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) p[i] = (uint64_t)t[8 + i] * 38u;
  fe r;
  uint32_t top, x;
  uint64_t c;
  asm("v_add_co_u32 %[r0], %[c], %[t0], %[l0]\n\t"
      "v_addc_co_u32 %[r1], %[c], %[t1], %[l1], %[c]\n\t"
      "v_addc_co_u32 %[r2], %[c], %[t2], %[l2], %[c]\n\t"
      "v_addc_co_u32 %[r3], %[c], %[t3], %[l3], %[c]\n\t"
      "v_addc_co_u32 %[r4], %[c], %[t4], %[l4], %[c]\n\t"
      "v_addc_co_u32 %[r5], %[c], %[t5], %[l5], %[c]\n\t"
      "v_addc_co_u32 %[r6], %[c], %[t6], %[l6], %[c]\n\t"
      "v_addc_co_u32 %[r7], %[c], %[t7], %[l7], %[c]\n\t"
      "v_addc_co_u32 %[top], %[c], %[h7], 0, %[c]\n\t"
      "v_add_co_u32 %[r1], %[c], %[r1], %[h0]\n\t"
      "v_addc_co_u32 %[r2], %[c], %[r2], %[h1], %[c]\n\t"
      "v_addc_co_u32 %[r3], %[c], %[r3], %[h2], %[c]\n\t"
      "v_addc_co_u32 %[r4], %[c], %[r4], %[h3], %[c]\n\t"
      "v_addc_co_u32 %[r5], %[c], %[r5], %[h4], %[c]\n\t"
      "v_addc_co_u32 %[r6], %[c], %[r6], %[h5], %[c]\n\t"
      "v_addc_co_u32 %[r7], %[c], %[r7], %[h6], %[c]\n\t"
      "v_addc_co_u32 %[top], %[c], %[top], 0, %[c]\n\t"
      "v_lshrrev_b32 %[x], 31, %[r7]\n\t"
      "v_lshl_or_b32 %[x], %[top], 1, %[x]\n\t"
      "v_and_b32 %[r7], 0x7fffffff, %[r7]\n\t"
      "v_mul_u32_u24 %[x], 19, %[x]\n\t"
      "v_add_co_u32 %[r0], %[c], %[r0], %[x]\n\t"
      "v_addc_co_u32 %[r1], %[c], %[r1], 0, %[c]\n\t"
      "v_addc_co_u32 %[r2], %[c], %[r2], 0, %[c]\n\t"
      "v_addc_co_u32 %[r3], %[c], %[r3], 0, %[c]\n\t"
      "v_addc_co_u32 %[r4], %[c], %[r4], 0, %[c]\n\t"
      "v_addc_co_u32 %[r5], %[c], %[r5], 0, %[c]\n\t"
      "v_addc_co_u32 %[r6], %[c], %[r6], 0, %[c]\n\t"
      "v_addc_co_u32 %[r7], %[c], %[r7], 0, %[c]"
      : [r0] "=&v"(r.v[0]), [r1] "=&v"(r.v[1]), [r2] "=&v"(r.v[2]), [r3] "=&v"(r.v[3]), [r4] "=&v"(r.v[4]),
        [r5] "=&v"(r.v[5]), [r6] "=&v"(r.v[6]), [r7] "=&v"(r.v[7]), [top] "=&v"(top), [x] "=&v"(x),
        [c] "=&s"(c)
      : [t0] "v"(t[0]), [t1] "v"(t[1]), [t2] "v"(t[2]), [t3] "v"(t[3]), [t4] "v"(t[4]), [t5] "v"(t[5]),
        [t6] "v"(t[6]), [t7] "v"(t[7]), [l0] "v"((uint32_t)p[0]), [l1] "v"((uint32_t)p[1]),
        [l2] "v"((uint32_t)p[2]), [l3] "v"((uint32_t)p[3]), [l4] "v"((uint32_t)p[4]), [l5] "v"((uint32_t)p[5]),
        [l6] "v"((uint32_t)p[6]), [l7] "v"((uint32_t)p[7]), [h0] "v"((uint32_t)(p[0] >> 32)),
        [h1] "v"((uint32_t)(p[1] >> 32)), [h2] "v"((uint32_t)(p[2] >> 32)), [h3] "v"((uint32_t)(p[3] >> 32)),
        [h4] "v"((uint32_t)(p[4] >> 32)), [h5] "v"((uint32_t)(p[5] >> 32)), [h6] "v"((uint32_t)(p[6] >> 32)),
        [h7] "v"((uint32_t)(p[7] >> 32)));
  return r;  // < 2^255 + 2^12
}

#include "fe8_cols.inc"

FE_INLINE fe fe_mul(const fe& a, const fe& b) {
  uint32_t t[16];
  FE_MUL_COLUMNS(a, b, t);
  return fe_reduce512(t);
}

// Squaring: cross products once, doubled, plus the diagonal.
FE_INLINE fe fe_sq(const fe& a) {
  uint32_t t[16];
  FE_SQ_CROSS_COLUMNS(a, t);
  // double (cross terms < 2^511, so the doubled value fits in 512 bits)
  _Pragma("unroll") for (int k = 15; k > 0; --k) t[k] = __builtin_amdgcn_alignbit(t[k], t[k - 1], 31);
  t[0] = 0;
  // add diagonal a_i^2 at position 2i (one carry chain through all 16 words)
  uint64_t q[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) q[i] = (uint64_t)a.v[i] * a.v[i];
  uint64_t c;
  asm("v_add_co_u32 %[t0], %[c], %[t0], %[q0l]\n\t"
      "v_addc_co_u32 %[t1], %[c], %[t1], %[q0h], %[c]\n\t"
      "v_addc_co_u32 %[t2], %[c], %[t2], %[q1l], %[c]\n\t"
      "v_addc_co_u32 %[t3], %[c], %[t3], %[q1h], %[c]\n\t"
      "v_addc_co_u32 %[t4], %[c], %[t4], %[q2l], %[c]\n\t"
      "v_addc_co_u32 %[t5], %[c], %[t5], %[q2h], %[c]\n\t"
      "v_addc_co_u32 %[t6], %[c], %[t6], %[q3l], %[c]\n\t"
      "v_addc_co_u32 %[t7], %[c], %[t7], %[q3h], %[c]\n\t"
      "v_addc_co_u32 %[t8], %[c], %[t8], %[q4l], %[c]\n\t"
      "v_addc_co_u32 %[t9], %[c], %[t9], %[q4h], %[c]\n\t"
      "v_addc_co_u32 %[t10], %[c], %[t10], %[q5l], %[c]\n\t"
      "v_addc_co_u32 %[t11], %[c], %[t11], %[q5h], %[c]\n\t"
      "v_addc_co_u32 %[t12], %[c], %[t12], %[q6l], %[c]\n\t"
      "v_addc_co_u32 %[t13], %[c], %[t13], %[q6h], %[c]\n\t"
      "v_addc_co_u32 %[t14], %[c], %[t14], %[q7l], %[c]\n\t"
      "v_addc_co_u32 %[t15], %[c], %[t15], %[q7h], %[c]"
      : [t0] "+v"(t[0]), [t1] "+v"(t[1]), [t2] "+v"(t[2]), [t3] "+v"(t[3]), [t4] "+v"(t[4]), [t5] "+v"(t[5]),
        [t6] "+v"(t[6]), [t7] "+v"(t[7]), [t8] "+v"(t[8]), [t9] "+v"(t[9]), [t10] "+v"(t[10]),
        [t11] "+v"(t[11]), [t12] "+v"(t[12]), [t13] "+v"(t[13]), [t14] "+v"(t[14]), [t15] "+v"(t[15]),
        [c] "=&s"(c)
      : [q0l] "v"((uint32_t)q[0]), [q0h] "v"((uint32_t)(q[0] >> 32)), [q1l] "v"((uint32_t)q[1]),
        [q1h] "v"((uint32_t)(q[1] >> 32)), [q2l] "v"((uint32_t)q[2]), [q2h] "v"((uint32_t)(q[2] >> 32)),
        [q3l] "v"((uint32_t)q[3]), [q3h] "v"((uint32_t)(q[3] >> 32)), [q4l] "v"((uint32_t)q[4]),
        [q4h] "v"((uint32_t)(q[4] >> 32)), [q5l] "v"((uint32_t)q[5]), [q5h] "v"((uint32_t)(q[5] >> 32)),
        [q6l] "v"((uint32_t)q[6]), [q6h] "v"((uint32_t)(q[6] >> 32)), [q7l] "v"((uint32_t)q[7]),
        [q7h] "v"((uint32_t)(q[7] >> 32)));
  return fe_reduce512(t);
}

FE_INLINE fe fe_sqn(fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

// multiply by a small constant (< 2^31)
FE_INLINE fe fe_mul_small(const fe& a, uint32_t k) {
  uint32_t plo[8], phi[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    const uint64_t p = (uint64_t)a.v[i] * k;
    plo[i] = (uint32_t)p;
    phi[i] = (uint32_t)(p >> 32);
  }
  fe r;
  uint32_t c;
  r.v[0] = plo[0];
  r.v[1] = ADDC(plo[1], phi[0], 0u, &c);
  _Pragma("unroll") for (int i = 2; i < 8; ++i) r.v[i] = ADDC(plo[i], phi[i - 1], c, &c);
  const uint32_t top = phi[7] + c;  // < 2^31
  // r + top*2^256 = r + 38*top
  const uint64_t t38 = (uint64_t)top * 38u;
  uint32_t cc;
  r.v[0] = ADDC(r.v[0], (uint32_t)t38, 0u, &cc);
  r.v[1] = ADDC(r.v[1], (uint32_t)(t38 >> 32), cc, &cc);
  _Pragma("unroll") for (int i = 2; i < 8; ++i) r.v[i] = ADDC(r.v[i], 0u, cc, &cc);
  return fe_fold(r, cc);
}

// Fully reduce to [0, p).
FE_INLINE fe fe_canon(fe a) {
  a = fe_fold(a, 0);  // < 2^255 + 2^12 < 2p
  // a >= p  <=>  a + 19 >= 2^255
  fe t = a;
  (void)fe_add_small(t, 19u);
  const uint32_t m = 0u - (t.v[7] >> 31);
  t.v[7] &= 0x7fffffffu;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) a.v[i] = (t.v[i] & m) | (a.v[i] & ~m);
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
