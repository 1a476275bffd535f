/* A caller-owned Merlin transcript for tests/c/abi_gpu.c: merlin 3.0.0
 * (STROBE-128 over Keccak-f[1600]) written from the published spec in plain
 * C, sharing no code with the library -- the stand-in for the Rust crate's
 * own merlin::Transcript behind bpp_transcript_hooks.  Test infrastructure. */
#ifndef MERLIN_MIN_H
#define MERLIN_MIN_H
#include <stdint.h>
#include <string.h>

static const uint64_t mm_rc[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

static uint64_t mm_rol(uint64_t x, unsigned r) { return r ? (x << r) | (x >> (64 - r)) : x; }

/* lanes a[x + 5 y], little-endian bytes of the 200-byte state */
static void mm_keccak(uint8_t st[200]) {
  uint64_t a[25], b[25], c[5], d[5];
  for (int i = 0; i < 25; ++i) {
    a[i] = 0;
    for (int k = 0; k < 8; ++k) a[i] |= (uint64_t)st[8 * i + k] << (8 * k);
  }
  /* rotation offsets r[x][y] */
  static const unsigned rot[5][5] = {
      {0, 36, 3, 41, 18}, {1, 44, 10, 45, 2}, {62, 6, 43, 15, 61}, {28, 55, 25, 21, 56}, {27, 20, 39, 8, 14}};
  for (int r = 0; r < 24; ++r) {
    for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ mm_rol(c[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) a[i] ^= d[i % 5];
    /* rho + pi: B[y, 2x + 3y] = rot(A[x, y], r[x, y]) */
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = mm_rol(a[x + 5 * y], rot[x][y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= mm_rc[r];
  }
  for (int i = 0; i < 25; ++i)
    for (int k = 0; k < 8; ++k) st[8 * i + k] = (uint8_t)(a[i] >> (8 * k));
}

enum { MM_R = 166, MM_I = 1, MM_A = 2, MM_C = 4, MM_M = 16, MM_K = 32 };

typedef struct {
  uint8_t st[200];
  uint8_t pos, pos_begin, cur_flags;
} mm_transcript;

static void mm_run_f(mm_transcript* t) {
  t->st[t->pos] ^= t->pos_begin;
  t->st[t->pos + 1] ^= 0x04;
  t->st[MM_R + 1] ^= 0x80;
  mm_keccak(t->st);
  t->pos = 0;
  t->pos_begin = 0;
}
static void mm_absorb(mm_transcript* t, const uint8_t* d, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    t->st[t->pos++] ^= d[i];
    if (t->pos == MM_R) mm_run_f(t);
  }
}
static void mm_squeeze(mm_transcript* t, uint8_t* d, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    d[i] = t->st[t->pos];
    t->st[t->pos++] = 0;
    if (t->pos == MM_R) mm_run_f(t);
  }
}
static void mm_begin_op(mm_transcript* t, uint8_t flags, int more) {
  if (more) return;
  const uint8_t hdr[2] = {t->pos_begin, flags};
  t->pos_begin = (uint8_t)(t->pos + 1);
  t->cur_flags = flags;
  mm_absorb(t, hdr, 2);
  if ((flags & (MM_C | MM_K)) && t->pos != 0) mm_run_f(t);
}
static void mm_meta_ad(mm_transcript* t, const uint8_t* d, size_t n, int more) {
  mm_begin_op(t, MM_M | MM_A, more);
  mm_absorb(t, d, n);
}
static void mm_append_message(mm_transcript* t, const uint8_t* label, size_t llen, const uint8_t* msg, size_t n) {
  const uint8_t le[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  mm_meta_ad(t, label, llen, 0);
  mm_meta_ad(t, le, 4, 1);
  mm_begin_op(t, MM_A, 0);
  mm_absorb(t, msg, n);
}
static void mm_challenge_bytes(mm_transcript* t, const uint8_t* label, size_t llen, uint8_t* out, size_t n) {
  const uint8_t le[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  mm_meta_ad(t, label, llen, 0);
  mm_meta_ad(t, le, 4, 1);
  mm_begin_op(t, MM_I | MM_A | MM_C, 0);
  mm_squeeze(t, out, n);
}
static void mm_new(mm_transcript* t, const uint8_t* label, size_t llen) {
  memset(t, 0, sizeof *t);
  const uint8_t hdr[6] = {1, MM_R + 2, 1, 0, 1, 96};
  memcpy(t->st, hdr, 6);
  memcpy(t->st + 6, "STROBEv1.0.2", 12);
  mm_keccak(t->st);
  mm_meta_ad(t, (const uint8_t*)"Merlin v1.0", 11, 0);
  mm_append_message(t, (const uint8_t*)"dom-sep", 7, label, llen);
}
#endif
