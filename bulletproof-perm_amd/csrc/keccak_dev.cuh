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

FE_INLINE uint64_t rotl64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

// Keccak-f[1600], fully unrolled over the 25 lanes (state in registers)
FE_INLINE void keccak_f1600_dev(uint64_t a[25]) {
  for (int r = 0; r < 24; ++r) {
    uint64_t c[5], d[5];
    _Pragma("unroll") for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    _Pragma("unroll") for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
    _Pragma("unroll") for (int i = 0; i < 25; ++i) a[i] ^= d[i % 5];
    // rho + pi
    uint64_t b[25];
    b[0] = a[0];
    b[10] = rotl64(a[1], 1);
    b[7] = rotl64(a[10], 3);
    b[11] = rotl64(a[7], 6);
    b[17] = rotl64(a[11], 10);
    b[18] = rotl64(a[17], 15);
    b[3] = rotl64(a[18], 21);
    b[5] = rotl64(a[3], 28);
    b[16] = rotl64(a[5], 36);
    b[8] = rotl64(a[16], 45);
    b[21] = rotl64(a[8], 55);
    b[24] = rotl64(a[21], 2);
    b[4] = rotl64(a[24], 14);
    b[15] = rotl64(a[4], 27);
    b[23] = rotl64(a[15], 41);
    b[19] = rotl64(a[23], 56);
    b[13] = rotl64(a[19], 8);
    b[12] = rotl64(a[13], 25);
    b[2] = rotl64(a[12], 43);
    b[20] = rotl64(a[2], 62);
    b[14] = rotl64(a[20], 18);
    b[22] = rotl64(a[14], 39);
    b[9] = rotl64(a[22], 61);
    b[6] = rotl64(a[9], 20);
    b[1] = rotl64(a[6], 44);
    // chi
    _Pragma("unroll") for (int y = 0; y < 25; y += 5) {
      _Pragma("unroll") for (int x = 0; x < 5; ++x) a[y + x] = b[y + x] ^ (~b[y + (x + 1) % 5] & b[y + (x + 2) % 5]);
    }
    a[0] ^= KECCAK_RC[r];
  }
}

