// Keccak-f[1600] on gfx950, one state per lane in registers (25 x 64-bit
// lanes): the device Merlin transcript (merlin_dev.hip) and the prover's
// indexed blinding draws (poly.hip k_draws).  Byte-exact with the host's
// Keccak (host/keccak.cpp; tests/test_gpu_merlin.py, the prover parity
// tests).
#pragma once
#include "fe25519.cuh"

__device__ __constant__ static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

// 64-bit rotation by a constant as two v_alignbit_b32 on the halves (the
// generic (x << n) | (x >> (64 - n)) compiles to 64-bit shifts, which issue
// at half rate on gfx950, plus an OR)
FE_INLINE uint64_t rotl64(uint64_t x, int n) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n >= 32) {
    const uint32_t t = lo;
    lo = hi;
    hi = t;
    n -= 32;
  }
  if (n == 0) return ((uint64_t)hi << 32) | lo;
  const uint32_t nh = __builtin_amdgcn_alignbit(hi, lo, 32 - n), nl = __builtin_amdgcn_alignbit(lo, hi, 32 - n);
  return ((uint64_t)nh << 32) | nl;
}

FE_INLINE uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// Keccak-f[1600] on 32-bit halves (the state's 64-bit words as lo / hi
// register pairs): theta's column parities as two 3-input XORs per half
// (v_bitop3_b32, gfx950), rotations as v_alignbit_b32 pairs, chi's
// a ^ (~b & c) as one v_bitop3_b32 per half (formed by the compiler).
// 24 rounds of ~190 VALU instructions instead of ~260 with 64-bit ops.
FE_INLINE void keccak_f1600_dev(uint64_t st[25]) {
  uint32_t lo[25], hi[25];
  _Pragma("unroll") for (int i = 0; i < 25; ++i) {
    lo[i] = (uint32_t)st[i];
    hi[i] = (uint32_t)(st[i] >> 32);
  }
  for (int r = 0; r < 24; ++r) {
    uint32_t cl[5], ch[5], dl[5], dh[5];
    _Pragma("unroll") for (int x = 0; x < 5; ++x) {
      cl[x] = xor3(xor3(lo[x], lo[x + 5], lo[x + 10]), lo[x + 15], lo[x + 20]);
      ch[x] = xor3(xor3(hi[x], hi[x + 5], hi[x + 10]), hi[x + 15], hi[x + 20]);
    }
    _Pragma("unroll") for (int x = 0; x < 5; ++x) {  // d = c[x-1] ^ rotl(c[x+1], 1)
      const int a1 = (x + 1) % 5, a4 = (x + 4) % 5;
      dh[x] = ch[a4] ^ __builtin_amdgcn_alignbit(ch[a1], cl[a1], 31);
      dl[x] = cl[a4] ^ __builtin_amdgcn_alignbit(cl[a1], ch[a1], 31);
    }
    _Pragma("unroll") for (int i = 0; i < 25; ++i) {
      lo[i] ^= dl[i % 5];
      hi[i] ^= dh[i % 5];
    }
    // rho + pi: b[pi(i)] = rotl(a[i], rho(i))
    uint32_t bl[25], bh[25];
#define KROT(dst, src, n)                                                                  \
  do {                                                                                     \
    const uint64_t v_ = rotl64(((uint64_t)hi[src] << 32) | lo[src], n);                    \
    bl[dst] = (uint32_t)v_;                                                                \
    bh[dst] = (uint32_t)(v_ >> 32);                                                        \
  } while (0)
    bl[0] = lo[0];
    bh[0] = hi[0];
    KROT(10, 1, 1);
    KROT(7, 10, 3);
    KROT(11, 7, 6);
    KROT(17, 11, 10);
    KROT(18, 17, 15);
    KROT(3, 18, 21);
    KROT(5, 3, 28);
    KROT(16, 5, 36);
    KROT(8, 16, 45);
    KROT(21, 8, 55);
    KROT(24, 21, 2);
    KROT(4, 24, 14);
    KROT(15, 4, 27);
    KROT(23, 15, 41);
    KROT(19, 23, 56);
    KROT(13, 19, 8);
    KROT(12, 13, 25);
    KROT(2, 12, 43);
    KROT(20, 2, 62);
    KROT(14, 20, 18);
    KROT(22, 14, 39);
    KROT(9, 22, 61);
    KROT(6, 9, 20);
    KROT(1, 6, 44);
#undef KROT
    // chi
    _Pragma("unroll") for (int y = 0; y < 25; y += 5) {
      _Pragma("unroll") for (int x = 0; x < 5; ++x) {
        lo[y + x] = bl[y + x] ^ (~bl[y + (x + 1) % 5] & bl[y + (x + 2) % 5]);
        hi[y + x] = bh[y + x] ^ (~bh[y + (x + 1) % 5] & bh[y + (x + 2) % 5]);
      }
    }
    lo[0] ^= (uint32_t)KECCAK_RC[r];
    hi[0] ^= (uint32_t)(KECCAK_RC[r] >> 32);
  }
  _Pragma("unroll") for (int i = 0; i < 25; ++i) st[i] = ((uint64_t)hi[i] << 32) | lo[i];
}
