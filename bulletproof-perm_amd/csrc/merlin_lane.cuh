// Merlin transcripts on the device, one transcript per lane (merlin 3.0.0 /
// STROBE-128 over Keccak-f[1600]; the reference's TranscriptProtocol,
// transcript_protocol.rs:26-67).  Byte-exact with host/merlin.h.
//
// The transcripts of one launch perform the same operations with the same
// lengths (a batch of proofs of one circuit), so the STROBE position
// registers pos / pos_begin are wave-uniform and only the 200-byte sponge
// states differ.  Each lane's sponge lives in LDS (a uniform byte offset is
// then one LDS address per lane); 32-byte messages and 64-byte challenges
// move as dwords (a uniform byte shift, v_alignbit), everything else byte by
// byte.  The permutation is one out-of-line function, so the long straight
// transcript schedules of the verifier do not inline Keccak at every
// absorb that may cross the rate.
#pragma once
#include "keccak_dev.cuh"
#include "sc25519.cuh"

#define LANE_STROBE_R 166
#define LANE_ST_BYTES 200  // one lane's sponge in LDS (8-byte aligned rows)

// (an LDS-typed pointer: through a generic one the out-of-line function's
// loads and stores would be flat instructions)
typedef __attribute__((address_space(3))) uint64_t lds_u64;
__device__ __noinline__ static void lane_keccak(lds_u64* st) {
  uint64_t a[25];
  _Pragma("unroll") for (int i = 0; i < 25; ++i) a[i] = st[i];
  keccak_f1600_dev(a);
  _Pragma("unroll") for (int i = 0; i < 25; ++i) st[i] = a[i];
}

struct LaneStrobe {
  uint8_t* st;  // this lane's 200 bytes in LDS
  uint32_t pos, pos_begin;

  FE_INLINE void run_f() {
    st[pos] ^= (uint8_t)pos_begin;
    st[pos + 1] ^= 0x04;
    st[LANE_STROBE_R + 1] ^= 0x80;
    lane_keccak((lds_u64*)st);
    pos = 0;
    pos_begin = 0;
  }
  FE_INLINE void absorb_byte(uint32_t b) {
    st[pos] ^= (uint8_t)b;
    if (++pos == LANE_STROBE_R) run_f();
  }
  FE_INLINE void absorb_bytes(const uint8_t* d, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) absorb_byte(d[i]);
  }
  // the 4 little-endian bytes of x
  FE_INLINE void absorb_le32(uint32_t x) {
    absorb_byte(x & 0xffu);
    absorb_byte((x >> 8) & 0xffu);
    absorb_byte((x >> 16) & 0xffu);
    absorb_byte(x >> 24);
  }
  // 32 bytes given as 8 little-endian words: when the message does not reach
  // the end of the rate, 9 dword read-modify-writes at the uniform byte shift
  FE_INLINE void absorb32(const uint32_t w[8]) {
    if (pos + 32 < LANE_STROBE_R) {
      uint32_t* d = reinterpret_cast<uint32_t*>(st) + (pos >> 2);
      const uint32_t sh = 8 * (pos & 3);
      if (sh == 0) {
        _Pragma("unroll") for (int i = 0; i < 8; ++i) d[i] ^= w[i];
      } else {
        d[0] ^= w[0] << sh;
        _Pragma("unroll") for (int i = 1; i < 8; ++i) d[i] ^= __builtin_amdgcn_alignbit(w[i], w[i - 1], 32 - sh);
        d[8] ^= w[7] >> (32 - sh);
      }
      pos += 32;
      return;
    }
    _Pragma("unroll") for (int i = 0; i < 8; ++i) absorb_le32(w[i]);
  }
  FE_INLINE void begin_op(uint32_t flags) {
    const uint32_t old_begin = pos_begin;
    pos_begin = pos + 1;
    absorb_byte(old_begin);
    absorb_byte(flags);
    if ((flags & (4u | 32u)) && pos != 0) run_f();  // FLAG_C | FLAG_K
  }
  // merlin append_message's meta part: meta_ad(label), meta_ad(le32(n), more)
  FE_INLINE void meta(const char* label, uint32_t ln, uint32_t n) {
    begin_op(16u | 2u);  // FLAG_M | FLAG_A
    absorb_bytes(reinterpret_cast<const uint8_t*>(label), ln);
    absorb_le32(n);
  }
  // append_message(label, 32-byte msg): points and scalars
  FE_INLINE void append32(const char* label, uint32_t ln, const uint32_t w[8]) {
    meta(label, ln, 32);
    begin_op(2u);  // FLAG_A
    absorb32(w);
  }
  FE_INLINE void append_bytes(const char* label, uint32_t ln, const uint8_t* msg, uint32_t n) {
    meta(label, ln, n);
    begin_op(2u);
    absorb_bytes(msg, n);
  }
  FE_INLINE void append_u64(const char* label, uint32_t ln, uint64_t x) {
    meta(label, ln, 8);
    begin_op(2u);
    absorb_le32((uint32_t)x);
    absorb_le32((uint32_t)(x >> 32));
  }
  // challenge_bytes(label, 64) as 16 little-endian words.  begin_op(FLAG_C)
  // leaves pos = 0 (it permutes unless pos already is 0), so the squeeze
  // reads and clears 16 whole dwords.
  FE_INLINE void challenge64(const char* label, uint32_t ln, uint32_t out[16]) {
    meta(label, ln, 64);
    begin_op(1u | 2u | 4u);  // FLAG_I | FLAG_A | FLAG_C
    uint32_t* d = reinterpret_cast<uint32_t*>(st);
    _Pragma("unroll") for (int i = 0; i < 16; ++i) {
      out[i] = d[i];
      d[i] = 0;
    }
    pos = 64;
  }
  // challenge_scalar (transcript_protocol.rs:62-67): 64 bytes ->
  // Scalar::from_bytes_mod_order_wide, canonical
  FE_INLINE sc challenge_scalar(const char* label, uint32_t ln) {
    uint32_t w[16];
    challenge64(label, ln, w);
    return sc_from_wide_w(w);
  }
};

FE_INLINE bool w8_is_one(const uint32_t a[8]) {
  uint32_t o = a[0] ^ 1u;
  _Pragma("unroll") for (int i = 1; i < 8; ++i) o |= a[i];
  return o == 0;
}
FE_INLINE bool w8_geq(const uint32_t a[8], const uint32_t b[8]) {
  for (int i = 7; i >= 0; --i)
    if (a[i] != b[i]) return a[i] > b[i];
  return true;
}
FE_INLINE void w8_sub(uint32_t a[8], const uint32_t b[8]) {
  uint64_t br = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)a[i] - b[i] - br;
    a[i] = (uint32_t)d;
    br = (d >> 32) & 1u;
  }
}
FE_INLINE void w8_shr1(uint32_t a[8]) {
  _Pragma("unroll") for (int i = 0; i < 7; ++i) a[i] = (a[i] >> 1) | (a[i + 1] << 31);
  a[7] >>= 1;
}

// a^-1 mod l for canonical a != 0 by the binary extended Euclidean algorithm
// (variable time: the inverted challenges are public).  Bounded loop: every
// outer step removes at least one bit from u + v.
FE_INLINE sc sc_inv_vartime(const sc& a) {
  uint32_t u[8], v[8];
  sc x1 = sc_zero(), x2 = sc_zero();
  x1.v[0] = 1;
  bool zero = true;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    u[i] = a.v[i];
    v[i] = SC_L[i];
    zero &= a.v[i] == 0;
  }
  if (zero) return sc_zero();
  for (int it = 0; it < 2048 && !w8_is_one(u) && !w8_is_one(v); ++it) {
    while (!(u[0] & 1u)) {
      w8_shr1(u);
      x1 = sc_half(x1);
    }
    while (!(v[0] & 1u)) {
      w8_shr1(v);
      x2 = sc_half(x2);
    }
    if (w8_geq(u, v)) {
      w8_sub(u, v);
      x1 = sc_sub(x1, x2);
    } else {
      w8_sub(v, u);
      x2 = sc_sub(x2, x1);
    }
  }
  return w8_is_one(u) ? x1 : x2;
}

// Per lane a^-1 (Montgomery in, Montgomery out) with one inversion per
// wave: inclusive and exclusive products over the lanes (Hillis-Steele
// scans, 6 shuffle steps each way), the wave's total inverted once
// (uniform control flow), a^-1 = total^-1 * prefix * suffix.  A zero lane
// value makes every lane's result wrong (its proof is rejected anyway).
FE_INLINE sc sc_wave_inverse_mont(const sc& aR) {
  const int lane = threadIdx.x & 63;
  const sc oneR = sc_one_mont();
  sc pre = aR, suf = aR;  // inclusive prefix / suffix products
  _Pragma("unroll") for (int d = 1; d < 64; d <<= 1) {
    const sc a = sc_shfl(pre, lane - d < 0 ? lane : lane - d);
    const sc b = sc_shfl(suf, lane + d > 63 ? lane : lane + d);
    if (lane >= d) pre = sc_mont(a, pre);
    if (lane + d <= 63) suf = sc_mont(suf, b);
  }
  const sc total = sc_shfl(pre, 63);
  const sc tinv = sc_to_mont(sc_inv_vartime(sc_from_mont(total)));  // (every lane: the same value)
  const sc xp = sc_shfl(pre, lane ? lane - 1 : 0), xs = sc_shfl(suf, lane < 63 ? lane + 1 : 63);  // (all lanes shuffle)
  const sc ex_pre = lane ? xp : oneR;
  const sc ex_suf = lane < 63 ? xs : oneR;
  return sc_mont(tinv, sc_mont(ex_pre, ex_suf));
}
