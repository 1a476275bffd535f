// Keccak-f[1600] permutation for the host transcript / SHAKE code
// (host/merlin.h).  Compiled by the host C++ compiler (build.py): g++ made
// it 1.3x faster than the HIP toolchain's host pass here.  (A 4-state AVX2
// version measured no faster per state than this scalar one: 25 ymm lanes
// spill and AVX2 has no 64-bit rotate.)
#include <stdint.h>

namespace merlin {

static inline uint64_t rol(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

// Keccak-f[1600], 24 rounds, state in locals (generated unrolled theta /
// rho-pi / chi; the loop form with % 5 indexing measured ~2x slower).
void keccak_f1600(uint64_t st[25]) {
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

}  // namespace merlin
