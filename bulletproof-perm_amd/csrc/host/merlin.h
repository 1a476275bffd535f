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

#include <algorithm>
#include <vector>

#include "scalar.h"

namespace merlin {

static inline uint64_t rol(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

// Keccak-f[1600] (host/keccak.cpp, compiled by the host C++ compiler)
void keccak_f1600(uint64_t st[25]);
// host/keccak_x8.cpp: eight states per AVX-512 permutation
bool keccak_x8_available();
void keccak_f1600_x8(uint64_t lanes[25][8]);  // lanes[i][j] = word i of state j
void shake256_x8(const uint8_t* const in[8], size_t inlen, uint8_t* const out[8], size_t len);

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

// Eight transcripts in lockstep.  Proofs of one batch run the same
// transcript operations with the same lengths, so their STROBE positions
// agree and their permutations can run together on the 8-way Keccak:
// load() takes 8 transcripts (equal positions), the ops below take one
// message per instance, store() writes the states back.  Byte-identical to
// running each Transcript alone.
struct TranscriptX8 {
  alignas(64) uint64_t L[25][8];
  uint8_t pos = 0, pos_begin = 0, cur_flags = 0;

  uint8_t& byte(int j, int k) { return reinterpret_cast<uint8_t*>(&L[k >> 3][j])[k & 7]; }
  bool load(Transcript* const t[8]) {
    for (int j = 0; j < 8; ++j) {
      const Strobe128& s = t[j]->s;
      if (s.pos != t[0]->s.pos || s.pos_begin != t[0]->s.pos_begin || s.cur_flags != t[0]->s.cur_flags) return false;
      for (int i = 0; i < 25; ++i) memcpy(&L[i][j], s.st + 8 * i, 8);
    }
    pos = t[0]->s.pos;
    pos_begin = t[0]->s.pos_begin;
    cur_flags = t[0]->s.cur_flags;
    return true;
  }
  void store(Transcript* const t[8]) {
    for (int j = 0; j < 8; ++j) {
      Strobe128& s = t[j]->s;
      for (int i = 0; i < 25; ++i) memcpy(s.st + 8 * i, &L[i][j], 8);
      s.pos = pos;
      s.pos_begin = pos_begin;
      s.cur_flags = cur_flags;
    }
  }
  void run_f() {
    for (int j = 0; j < 8; ++j) {
      byte(j, pos) ^= pos_begin;
      byte(j, pos + 1) ^= 0x04;
      byte(j, STROBE_R + 1) ^= 0x80;
    }
    keccak_f1600_x8(L);
    pos = 0;
    pos_begin = 0;
  }
  // d[j] = instance j's bytes (stride 0 when `same`: one buffer for all)
  // (whole 64-bit words of the state where pos is word-aligned: a 32-byte
  // point is mostly four word XORs per lane instead of 32 byte XORs)
  void absorb(const uint8_t* const d[8], size_t n) {
    for (size_t i = 0; i < n;) {
      if ((pos & 7) == 0 && n - i >= 8 && pos + 8 <= STROBE_R) {
        uint64_t* row = L[pos >> 3];
        for (int j = 0; j < 8; ++j) {
          uint64_t x;
          memcpy(&x, d[j] + i, 8);
          row[j] ^= x;
        }
        i += 8;
        pos += 8;  // (STROBE_R = 166 is not a multiple of 8: the last 6 bytes go below)
        continue;
      }
      for (int j = 0; j < 8; ++j) byte(j, pos) ^= d[j][i];
      ++i;
      if (++pos == STROBE_R) run_f();
    }
  }
  void absorb_same(const uint8_t* d, size_t n) {
    const uint8_t* const dd[8] = {d, d, d, d, d, d, d, d};
    absorb(dd, n);
  }
  void squeeze(uint8_t* const d[8], size_t n) {
    for (size_t i = 0; i < n;) {
      if ((pos & 7) == 0 && n - i >= 8 && pos + 8 <= STROBE_R) {
        uint64_t* row = L[pos >> 3];
        for (int j = 0; j < 8; ++j) {
          memcpy(d[j] + i, &row[j], 8);
          row[j] = 0;
        }
        i += 8;
        pos += 8;
        continue;
      }
      for (int j = 0; j < 8; ++j) {
        d[j][i] = byte(j, pos);
        byte(j, pos) = 0;
      }
      ++i;
      if (++pos == STROBE_R) run_f();
    }
  }
  void begin_op(uint8_t flags, bool more) {
    if (more) return;
    const uint8_t old_begin = pos_begin;
    pos_begin = pos + 1;
    cur_flags = flags;
    const uint8_t hdr[2] = {old_begin, flags};
    absorb_same(hdr, 2);
    if ((flags & (FLAG_C | FLAG_K)) && pos != 0) run_f();
  }
  void meta_label_len(const char* label, uint32_t len) {
    begin_op(FLAG_M | FLAG_A, false);
    absorb_same((const uint8_t*)label, strlen(label));
    uint8_t le[4];
    memcpy(le, &len, 4);
    absorb_same(le, 4);  // meta_ad(more = true)
  }
  void append(const char* label, const uint8_t* const msg[8], size_t n) {
    meta_label_len(label, (uint32_t)n);
    begin_op(FLAG_A, false);
    absorb(msg, n);
  }
  void challenge_bytes(const char* label, uint8_t* const out[8], size_t n) {
    meta_label_len(label, (uint32_t)n);
    begin_op(FLAG_I | FLAG_A | FLAG_C, false);
    squeeze(out, n);
  }
  void challenge_scalar(const char* label, hsc::Sc out[8]) {
    uint8_t buf[8][64];
    uint8_t* const o[8] = {buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], buf[7]};
    challenge_bytes(label, o, 64);
    for (int j = 0; j < 8; ++j) out[j] = hsc::from_wide(buf[j]);
  }
};

// Runs transcript operations on P transcripts that are in lockstep, eight at
// a time on the 8-way Keccak: fx8(X, idx, real) performs the group's ops on X
// (instance j is transcript idx[j]; lanes j >= real pad a short last group
// with copies of its last transcript, whose results the caller drops);
// f1(p) performs the same ops on transcript p alone when a group is not in
// lockstep.  `for_groups` runs the groups (the host pool's for_each).
template <class ForGroups, class FX8, class F1>
void lockstep_x8(const std::vector<Transcript*>& trs, ForGroups&& for_groups, FX8&& fx8, F1&& f1) {
  const size_t P = trs.size();
  for_groups((P + 7) / 8, [&](size_t gi) {
    Transcript pad;  // (a short last group's padding lanes share one copy)
    Transcript* t[8];
    size_t idx[8];
    const size_t real = std::min<size_t>(8, P - 8 * gi);
    for (size_t j = 0; j < 8; ++j) idx[j] = 8 * gi + std::min(j, real - 1);
    if (real < 8) pad = *trs[idx[real - 1]];
    for (size_t j = 0; j < 8; ++j) t[j] = j < real ? trs[idx[j]] : &pad;
    TranscriptX8 X;
    if (!X.load(t)) {
      for (size_t j = 0; j < real; ++j) f1(idx[j]);
      return;
    }
    fx8(X, idx, real);
    // padding lanes share `pad`: store only the real ones (pad's state is dropped)
    Transcript* tr[8];
    for (size_t j = 0; j < 8; ++j) tr[j] = j < real ? t[j] : &pad;
    X.store(tr);
  });
}

}  // namespace merlin
