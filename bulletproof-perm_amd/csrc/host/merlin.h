// Merlin transcript (STROBE-128 over Keccak-f[1600]) for the host side.
//
// Byte-exact with merlin 3.0.0 (not vendored; bp-perm/Cargo.lock), which
// the reference drives through its TranscriptProtocol trait
// (bp-perm/src/transcript_protocol.rs:26-67):
//   arithmetic_domain_sep  :27-30   append_scalar :32-34
//   append_point           :45-47   validate_and_append_point :48-60
//   challenge_scalar       :62-67 (64 bytes -> from_bytes_mod_order_wide)
// plus bulletproofs 4.0.0's innerproduct_domain_sep ("ipp v1").
// Fiat-Shamir is sequential, so this stays on the host.
#pragma once
#include <stdint.h>
#include <string.h>

#include "scalar.h"

namespace merlin {

static inline uint64_t rol(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

// Keccak-f[1600], 24 rounds, state in locals (generated unrolled theta /
// rho-pi / chi; the loop form with % 5 indexing measured ~2x slower).
static inline void keccak_f1600(uint64_t st[25]) {
  static const uint64_t RC[24] = {
      0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
      0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
      0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
      0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
      0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
      0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL,
  };
  uint64_t a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16, a17, a18, a19, a20, a21, a22, a23, a24;
  a0 = st[0];
  a1 = st[1];
  a2 = st[2];
  a3 = st[3];
  a4 = st[4];
  a5 = st[5];
  a6 = st[6];
  a7 = st[7];
  a8 = st[8];
  a9 = st[9];
  a10 = st[10];
  a11 = st[11];
  a12 = st[12];
  a13 = st[13];
  a14 = st[14];
  a15 = st[15];
  a16 = st[16];
  a17 = st[17];
  a18 = st[18];
  a19 = st[19];
  a20 = st[20];
  a21 = st[21];
  a22 = st[22];
  a23 = st[23];
  a24 = st[24];
  for (int round = 0; round < 24; ++round) {
    const uint64_t c0 = a0 ^ a5 ^ a10 ^ a15 ^ a20;
    const uint64_t c1 = a1 ^ a6 ^ a11 ^ a16 ^ a21;
    const uint64_t c2 = a2 ^ a7 ^ a12 ^ a17 ^ a22;
    const uint64_t c3 = a3 ^ a8 ^ a13 ^ a18 ^ a23;
    const uint64_t c4 = a4 ^ a9 ^ a14 ^ a19 ^ a24;
    const uint64_t d0 = c4 ^ rol(c1, 1);
    const uint64_t d1 = c0 ^ rol(c2, 1);
    const uint64_t d2 = c1 ^ rol(c3, 1);
    const uint64_t d3 = c2 ^ rol(c4, 1);
    const uint64_t d4 = c3 ^ rol(c0, 1);
    const uint64_t b0 = (a0 ^ d0);
    const uint64_t b1 = rol(a6 ^ d1, 44);
    const uint64_t b2 = rol(a12 ^ d2, 43);
    const uint64_t b3 = rol(a18 ^ d3, 21);
    const uint64_t b4 = rol(a24 ^ d4, 14);
    const uint64_t b5 = rol(a3 ^ d3, 28);
    const uint64_t b6 = rol(a9 ^ d4, 20);
    const uint64_t b7 = rol(a10 ^ d0, 3);
    const uint64_t b8 = rol(a16 ^ d1, 45);
    const uint64_t b9 = rol(a22 ^ d2, 61);
    const uint64_t b10 = rol(a1 ^ d1, 1);
    const uint64_t b11 = rol(a7 ^ d2, 6);
    const uint64_t b12 = rol(a13 ^ d3, 25);
    const uint64_t b13 = rol(a19 ^ d4, 8);
    const uint64_t b14 = rol(a20 ^ d0, 18);
    const uint64_t b15 = rol(a4 ^ d4, 27);
    const uint64_t b16 = rol(a5 ^ d0, 36);
    const uint64_t b17 = rol(a11 ^ d1, 10);
    const uint64_t b18 = rol(a17 ^ d2, 15);
    const uint64_t b19 = rol(a23 ^ d3, 56);
    const uint64_t b20 = rol(a2 ^ d2, 62);
    const uint64_t b21 = rol(a8 ^ d3, 55);
    const uint64_t b22 = rol(a14 ^ d4, 39);
    const uint64_t b23 = rol(a15 ^ d0, 41);
    const uint64_t b24 = rol(a21 ^ d1, 2);
    a0 = b0 ^ ((~b1) & b2);
    a1 = b1 ^ ((~b2) & b3);
    a2 = b2 ^ ((~b3) & b4);
    a3 = b3 ^ ((~b4) & b0);
    a4 = b4 ^ ((~b0) & b1);
    a5 = b5 ^ ((~b6) & b7);
    a6 = b6 ^ ((~b7) & b8);
    a7 = b7 ^ ((~b8) & b9);
    a8 = b8 ^ ((~b9) & b5);
    a9 = b9 ^ ((~b5) & b6);
    a10 = b10 ^ ((~b11) & b12);
    a11 = b11 ^ ((~b12) & b13);
    a12 = b12 ^ ((~b13) & b14);
    a13 = b13 ^ ((~b14) & b10);
    a14 = b14 ^ ((~b10) & b11);
    a15 = b15 ^ ((~b16) & b17);
    a16 = b16 ^ ((~b17) & b18);
    a17 = b17 ^ ((~b18) & b19);
    a18 = b18 ^ ((~b19) & b15);
    a19 = b19 ^ ((~b15) & b16);
    a20 = b20 ^ ((~b21) & b22);
    a21 = b21 ^ ((~b22) & b23);
    a22 = b22 ^ ((~b23) & b24);
    a23 = b23 ^ ((~b24) & b20);
    a24 = b24 ^ ((~b20) & b21);
    a0 ^= RC[round];
  }
  st[0] = a0;
  st[1] = a1;
  st[2] = a2;
  st[3] = a3;
  st[4] = a4;
  st[5] = a5;
  st[6] = a6;
  st[7] = a7;
  st[8] = a8;
  st[9] = a9;
  st[10] = a10;
  st[11] = a11;
  st[12] = a12;
  st[13] = a13;
  st[14] = a14;
  st[15] = a15;
  st[16] = a16;
  st[17] = a17;
  st[18] = a18;
  st[19] = a19;
  st[20] = a20;
  st[21] = a21;
  st[22] = a22;
  st[23] = a23;
  st[24] = a24;
}

// SHAKE256 XOF (rate 136, domain 0x1F): bulletproofs' GeneratorsChain and
// PedersenGens::default's SHA3-512 hash-to-point need it.
struct Shake256 {
  uint64_t s[25];
  uint8_t buf[136];
  size_t n = 0;
  bool squeezing = false;
  size_t rpos = 0;
  Shake256() { memset(s, 0, sizeof s); }
  void absorb_block(const uint8_t* b) {
    for (int i = 0; i < 17; ++i) {
      uint64_t w;
      memcpy(&w, b + 8 * i, 8);
      s[i] ^= w;
    }
    keccak_f1600(s);
  }
  void update(const uint8_t* d, size_t len) {
    for (size_t i = 0; i < len; ++i) {
      buf[n++] = d[i];
      if (n == 136) {
        absorb_block(buf);
        n = 0;
      }
    }
  }
  void finish() {
    memset(buf + n, 0, 136 - n);
    buf[n] ^= 0x1F;
    buf[135] ^= 0x80;
    absorb_block(buf);
    squeezing = true;
    rpos = 0;
  }
  void read(uint8_t* out, size_t len) {
    if (!squeezing) finish();
    while (len) {
      if (rpos == 136) {
        keccak_f1600(s);
        rpos = 0;
      }
      const size_t k = len < 136 - rpos ? len : 136 - rpos;
      memcpy(out, reinterpret_cast<const uint8_t*>(s) + rpos, k);  // little-endian lanes
      out += k;
      len -= k;
      rpos += k;
    }
  }

};

// SHA3-512 (rate 72, domain 0x06)
static inline void sha3_512(const uint8_t* d, size_t len, uint8_t out[64]) {
  uint64_t s[25];
  memset(s, 0, sizeof s);
  uint8_t block[72];
  size_t off = 0;
  while (len - off >= 72) {
    for (int i = 0; i < 9; ++i) {
      uint64_t w;
      memcpy(&w, d + off + 8 * i, 8);
      s[i] ^= w;
    }
    keccak_f1600(s);
    off += 72;
  }
  memset(block, 0, 72);
  memcpy(block, d + off, len - off);
  block[len - off] ^= 0x06;
  block[71] ^= 0x80;
  for (int i = 0; i < 9; ++i) {
    uint64_t w;
    memcpy(&w, block + 8 * i, 8);
    s[i] ^= w;
  }
  keccak_f1600(s);
  memcpy(out, s, 64);
}

enum : uint8_t { FLAG_I = 1, FLAG_A = 2, FLAG_C = 4, FLAG_T = 8, FLAG_M = 16, FLAG_K = 32 };
static const int STROBE_R = 166;

struct Strobe128 {
  uint8_t st[200];
  uint8_t pos = 0, pos_begin = 0, cur_flags = 0;

  void run_f() {
    st[pos] ^= pos_begin;
    st[pos + 1] ^= 0x04;
    st[STROBE_R + 1] ^= 0x80;
    uint64_t lanes[25];
    memcpy(lanes, st, 200);  // little-endian host
    keccak_f1600(lanes);
    memcpy(st, lanes, 200);
    pos = 0;
    pos_begin = 0;
  }
  void absorb(const uint8_t* d, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      st[pos] ^= d[i];
      if (++pos == STROBE_R) run_f();
    }
  }
  void squeeze(uint8_t* d, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      d[i] = st[pos];
      st[pos] = 0;
      if (++pos == STROBE_R) run_f();
    }
  }
  void begin_op(uint8_t flags, bool more) {
    if (more) return;  // continuation of the same op (flags equal by construction)
    const uint8_t old_begin = pos_begin;
    pos_begin = pos + 1;
    cur_flags = flags;
    const uint8_t hdr[2] = {old_begin, flags};
    absorb(hdr, 2);
    if ((flags & (FLAG_C | FLAG_K)) && pos != 0) run_f();
  }
  void meta_ad(const uint8_t* d, size_t n, bool more) {
    begin_op(FLAG_M | FLAG_A, more);
    absorb(d, n);
  }
  void ad(const uint8_t* d, size_t n, bool more) {
    begin_op(FLAG_A, more);
    absorb(d, n);
  }
  void prf(uint8_t* d, size_t n, bool more) {
    begin_op(FLAG_I | FLAG_A | FLAG_C, more);
    squeeze(d, n);
  }
  void init(const uint8_t* label, size_t n) {
    memset(st, 0, sizeof st);
    const uint8_t hdr[6] = {1, STROBE_R + 2, 1, 0, 1, 96};
    memcpy(st, hdr, 6);
    memcpy(st + 6, "STROBEv1.0.2", 12);
    uint64_t lanes[25];
    memcpy(lanes, st, 200);
    keccak_f1600(lanes);
    memcpy(st, lanes, 200);
    pos = pos_begin = cur_flags = 0;
    meta_ad(label, n, false);
  }
};

struct Transcript {
  Strobe128 s;

  explicit Transcript(const uint8_t* label = nullptr, size_t n = 0) {
    static const char kMerlin[] = "Merlin v1.0";
    s.init((const uint8_t*)kMerlin, sizeof(kMerlin) - 1);
    append_message((const uint8_t*)"dom-sep", 7, label, n);
  }
  void append_message(const uint8_t* label, size_t ln, const uint8_t* msg, size_t n) {
    const uint32_t len = (uint32_t)n;
    uint8_t le[4];
    memcpy(le, &len, 4);
    s.meta_ad(label, ln, false);
    s.meta_ad(le, 4, true);
    s.ad(msg, n, false);
  }
  void append(const char* label, const uint8_t* msg, size_t n) {
    append_message((const uint8_t*)label, strlen(label), msg, n);
  }
  void append_u64(const char* label, uint64_t x) {
    uint8_t b[8];
    memcpy(b, &x, 8);
    append(label, b, 8);
  }
  void challenge_bytes(const char* label, uint8_t* out, size_t n) {
    const uint32_t len = (uint32_t)n;
    uint8_t le[4];
    memcpy(le, &len, 4);
    s.meta_ad((const uint8_t*)label, strlen(label), false);
    s.meta_ad(le, 4, true);
    s.prf(out, n, false);
  }
  // --- TranscriptProtocol (transcript_protocol.rs)
  void arithmetic_domain_sep(uint64_t n) {
    append("dom-sep", (const uint8_t*)"acp v1", 6);
    append_u64("n", n);
  }
  void innerproduct_domain_sep(uint64_t n) {
    append("dom-sep", (const uint8_t*)"ipp v1", 6);
    append_u64("n", n);
  }
  void append_scalar(const char* label, const hsc::Sc& x) {
    uint8_t b[32];
    hsc::to_bytes(b, x);
    append(label, b, 32);
  }
  void append_point(const char* label, const uint8_t p[32]) { append(label, p, 32); }
  bool validate_and_append_point(const char* label, const uint8_t p[32]) {
    static const uint8_t zero[32] = {0};
    if (!memcmp(p, zero, 32)) return false;  // identity -> VerificationError
    append(label, p, 32);
    return true;
  }
  hsc::Sc challenge_scalar(const char* label) {
    uint8_t buf[64];
    challenge_bytes(label, buf, 64);
    return hsc::from_wide(buf);
  }
};

}  // namespace merlin
