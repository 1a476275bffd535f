// Eight Keccak-f[1600] states at once in AVX-512 registers (lane i of
// instance j = 64-bit element j of zmm i), and the prover's eight SHAKE256
// random streams built on it.  The EPYC hosts of the GPU boxes (Zen 5) run
// 512-bit vprolq / vpternlogq at full width: eight permutations cost about
// two scalar ones.  Callers check keccak_x8_available() (runtime CPUID) and
// fall back to the scalar keccak_f1600 otherwise; both give identical bytes.
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include "perm.h"

namespace merlin {

static const uint64_t RCX[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL,
};

bool keccak_x8_available() {
  static const bool ok = __builtin_cpu_supports("avx512f");
  return ok;
}

#define X8_TARGET __attribute__((target("avx512f")))

// rho offsets and pi destinations: B[pi(i)] = rol(A[i] ^ D[i % 5], RHO[i])
X8_TARGET static inline void keccak_x8_rounds(__m512i a[25]) {
  for (int round = 0; round < 24; ++round) {
    __m512i c[5], d[5];
#pragma GCC unroll 5
    for (int x = 0; x < 5; ++x)
      c[x] = _mm512_ternarylogic_epi64(_mm512_ternarylogic_epi64(a[x], a[x + 5], a[x + 10], 0x96), a[x + 15],
                                       a[x + 20], 0x96);
#pragma GCC unroll 5
    for (int x = 0; x < 5; ++x) d[x] = _mm512_xor_si512(c[(x + 4) % 5], _mm512_rol_epi64(c[(x + 1) % 5], 1));
    __m512i b[25];
    b[0] = _mm512_xor_si512(a[0], d[0]);
    b[1] = _mm512_rol_epi64(_mm512_xor_si512(a[6], d[1]), 44);
    b[2] = _mm512_rol_epi64(_mm512_xor_si512(a[12], d[2]), 43);
    b[3] = _mm512_rol_epi64(_mm512_xor_si512(a[18], d[3]), 21);
    b[4] = _mm512_rol_epi64(_mm512_xor_si512(a[24], d[4]), 14);
    b[5] = _mm512_rol_epi64(_mm512_xor_si512(a[3], d[3]), 28);
    b[6] = _mm512_rol_epi64(_mm512_xor_si512(a[9], d[4]), 20);
    b[7] = _mm512_rol_epi64(_mm512_xor_si512(a[10], d[0]), 3);
    b[8] = _mm512_rol_epi64(_mm512_xor_si512(a[16], d[1]), 45);
    b[9] = _mm512_rol_epi64(_mm512_xor_si512(a[22], d[2]), 61);
    b[10] = _mm512_rol_epi64(_mm512_xor_si512(a[1], d[1]), 1);
    b[11] = _mm512_rol_epi64(_mm512_xor_si512(a[7], d[2]), 6);
    b[12] = _mm512_rol_epi64(_mm512_xor_si512(a[13], d[3]), 25);
    b[13] = _mm512_rol_epi64(_mm512_xor_si512(a[19], d[4]), 8);
    b[14] = _mm512_rol_epi64(_mm512_xor_si512(a[20], d[0]), 18);
    b[15] = _mm512_rol_epi64(_mm512_xor_si512(a[4], d[4]), 27);
    b[16] = _mm512_rol_epi64(_mm512_xor_si512(a[5], d[0]), 36);
    b[17] = _mm512_rol_epi64(_mm512_xor_si512(a[11], d[1]), 10);
    b[18] = _mm512_rol_epi64(_mm512_xor_si512(a[17], d[2]), 15);
    b[19] = _mm512_rol_epi64(_mm512_xor_si512(a[23], d[3]), 56);
    b[20] = _mm512_rol_epi64(_mm512_xor_si512(a[2], d[2]), 62);
    b[21] = _mm512_rol_epi64(_mm512_xor_si512(a[8], d[3]), 55);
    b[22] = _mm512_rol_epi64(_mm512_xor_si512(a[14], d[4]), 39);
    b[23] = _mm512_rol_epi64(_mm512_xor_si512(a[15], d[0]), 41);
    b[24] = _mm512_rol_epi64(_mm512_xor_si512(a[21], d[1]), 2);
    // chi: a = b0 ^ (~b1 & b2)  (ternary-logic table 0xD2)
#pragma GCC unroll 5
    for (int y = 0; y < 25; y += 5) {
#pragma GCC unroll 5
      for (int x = 0; x < 5; ++x)
        a[y + x] = _mm512_ternarylogic_epi64(b[y + x], b[y + (x + 1) % 5], b[y + (x + 2) % 5], 0xD2);
    }
    a[0] = _mm512_xor_si512(a[0], _mm512_set1_epi64((long long)RCX[round]));
  }
}

X8_TARGET static void keccak_x8_lanes(uint64_t lanes[25][8]) {
  __m512i a[25];
  for (int i = 0; i < 25; ++i) a[i] = _mm512_loadu_si512((const void*)lanes[i]);
  keccak_x8_rounds(a);
  for (int i = 0; i < 25; ++i) _mm512_storeu_si512((void*)lanes[i], a[i]);
}

// 8 SHAKE256 streams of `len` bytes each (len a multiple of 136 not needed),
// inputs of one common length < 136 bytes.
X8_TARGET void shake256_x8(const uint8_t* const in[8], size_t inlen, uint8_t* const out[8], size_t len) {
  alignas(64) uint64_t lanes[25][8];
  memset(lanes, 0, sizeof lanes);
  for (int j = 0; j < 8; ++j) {
    uint8_t blk[136];
    memset(blk, 0, sizeof blk);
    memcpy(blk, in[j], inlen);
    blk[inlen] ^= 0x1F;
    blk[135] ^= 0x80;
    for (int i = 0; i < 17; ++i) memcpy(&lanes[i][j], blk + 8 * i, 8);
  }
  __m512i a[25];
  for (int i = 0; i < 25; ++i) a[i] = _mm512_load_si512((const void*)lanes[i]);
  for (size_t pos = 0; pos < len; pos += 136) {
    keccak_x8_rounds(a);
    for (int i = 0; i < 17; ++i) _mm512_store_si512((void*)lanes[i], a[i]);
    const size_t k = len - pos < 136 ? len - pos : 136;
    for (int j = 0; j < 8; ++j) {
      uint8_t blk[136];
      for (int i = 0; i < 17; ++i) memcpy(blk + 8 * i, &lanes[i][j], 8);
      memcpy(out[j] + pos, blk, k);
    }
  }
}

// Eight lane-interleaved states (lanes[i][j] = word i of state j) permuted
// together (StrobeX8, merlin.h).
void keccak_f1600_x8(uint64_t lanes[25][8]) {
  if (!keccak_x8_available()) {
    for (int j = 0; j < 8; ++j) {
      uint64_t st[25];
      for (int i = 0; i < 25; ++i) st[i] = lanes[i][j];
      keccak_f1600(st);
      for (int i = 0; i < 25; ++i) lanes[i][j] = st[i];
    }
    return;
  }
  keccak_x8_lanes(lanes);
}

}  // namespace merlin

namespace perm {

// pi of eight proofs: Fisher-Yates over the first 8 (k - 1) bytes of their
// SHAKE256("bpperm-prove" || seed) streams
static void draw_pi_x8(const Circuit& C, const Seed seeds[8], RandomDraws* const out[8]) {
  const size_t len = 8 * (size_t)(C.k - 1);
  uint8_t st[8][8 * 1024];
  static thread_local std::vector<uint8_t> big;  // (k > 1025)
  uint8_t* outp[8];
  if (len > sizeof st[0]) big.resize(8 * len);
  for (int j = 0; j < 8; ++j) outp[j] = len > sizeof st[0] ? big.data() + (size_t)j * len : st[j];
  if (!merlin::keccak_x8_available()) {
    for (int j = 0; j < 8; ++j) {
      Rng rng("bpperm-prove", seeds[j]);
      rng.bytes(outp[j], len);
    }
  } else if (len) {
    uint8_t in[8][12 + 32];
    const uint8_t* inp[8];
    for (int j = 0; j < 8; ++j) {
      memcpy(in[j], "bpperm-prove", 12);
      memcpy(in[j] + 12, seeds[j].b, seeds[j].len);
      inp[j] = in[j];
    }
    merlin::shake256_x8(inp, 12 + seeds[0].len, outp, len);
  }
  for (int j = 0; j < 8; ++j) {
    std::vector<uint32_t>& pi = out[j]->pi;
    pi.resize(C.k);
    for (uint32_t i = 0; i < C.k; ++i) pi[i] = i;
    const uint8_t* s = outp[j];
    for (uint32_t i = C.k - 1; i > 0; --i) {
      uint64_t x;
      memcpy(&x, s, 8);
      s += 8;
      std::swap(pi[i], pi[(uint32_t)(x % (uint64_t)(i + 1))]);
    }
  }
}

// scalar draw `idx` of eight proofs (draw_scalar, 8-way)
static void draw_scalar_x8(const Seed seeds[8], uint32_t idx, hsc::Sc* const out[8]) {
  if (!merlin::keccak_x8_available()) {
    for (int j = 0; j < 8; ++j) *out[j] = draw_scalar(seeds[j], idx);
    return;
  }
  uint8_t in[8][BPP_DRAW_DOMAIN_LEN + 32 + 4], wide[8][64];
  const uint8_t* inp[8];
  uint8_t* outp[8];
  const size_t sl = seeds[0].len;
  for (int j = 0; j < 8; ++j) {
    memcpy(in[j], BPP_DRAW_DOMAIN, BPP_DRAW_DOMAIN_LEN);
    memcpy(in[j] + BPP_DRAW_DOMAIN_LEN, seeds[j].b, sl);
    for (int b = 0; b < 4; ++b) in[j][BPP_DRAW_DOMAIN_LEN + sl + b] = (uint8_t)(idx >> (8 * b));
    inp[j] = in[j];
    outp[j] = wide[j];
  }
  merlin::shake256_x8(inp, BPP_DRAW_DOMAIN_LEN + sl + 4, outp, 64);
  for (int j = 0; j < 8; ++j) *out[j] = hsc::from_wide(wide[j]);
}

void draw_prover_randomness_x8(const Circuit& C, const Seed seeds[8], RandomDraws* const out[8]) {
  draw_pi_x8(C, seeds, out);
  hsc::Sc* o[8];
  uint32_t idx = 0;
  auto vec = [&](std::vector<hsc::Sc> RandomDraws::*v, uint32_t n) {
    for (int j = 0; j < 8; ++j) (out[j]->*v).resize(n);
    for (uint32_t i = 0; i < n; ++i, ++idx) {
      for (int j = 0; j < 8; ++j) o[j] = &(out[j]->*v)[i];
      draw_scalar_x8(seeds, idx, o);
    }
  };
  auto one = [&](hsc::Sc RandomDraws::*f) {
    for (int j = 0; j < 8; ++j) o[j] = &(out[j]->*f);
    draw_scalar_x8(seeds, idx++, o);
  };
  vec(&RandomDraws::gamma, C.m);
  one(&RandomDraws::alpha);
  one(&RandomDraws::beta);
  one(&RandomDraws::rho);
  vec(&RandomDraws::sL, C.n_p);
  vec(&RandomDraws::sR, C.n_p);
  vec(&RandomDraws::taus, 5);
}

void draw_prover_host_x8(const Circuit& C, const Seed seeds[8], RandomDraws* const out[8]) {
  draw_pi_x8(C, seeds, out);
  hsc::Sc* o[8];
  hsc::Sc RandomDraws::*abr[3] = {&RandomDraws::alpha, &RandomDraws::beta, &RandomDraws::rho};
  for (uint32_t i = 0; i < 3; ++i) {
    for (int j = 0; j < 8; ++j) o[j] = &(out[j]->*abr[i]);
    draw_scalar_x8(seeds, draw_alpha_index(C) + i, o);
  }
  for (int j = 0; j < 8; ++j) {
    out[j]->gamma.clear();
    out[j]->sL.clear();
    out[j]->sR.clear();
    out[j]->taus.resize(5);
  }
  for (uint32_t i = 0; i < 5; ++i) {
    for (int j = 0; j < 8; ++j) o[j] = &out[j]->taus[i];
    draw_scalar_x8(seeds, draw_tau_index(C) + i, o);
  }
}

}  // namespace perm
