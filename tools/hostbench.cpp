// CPU microbenchmark of the prover's host-side pieces (per 52-card proof and
// per batch step), to see where the host time of a lockstep batch goes.
//   g++ -O3 -march=x86-64-v3 -std=c++17 -I bulletproof-perm_amd/csrc tools/hostbench.cpp \
//       bulletproof-perm_amd/csrc/host/keccak.cpp bulletproof-perm_amd/csrc/host/perm_circuit.cpp -o /tmp/hostbench
#include <chrono>
#include <cstdio>
#include <vector>

#include "host/fe64.h"
#include "host/merlin.h"
#include "host/perm.h"
#include "host/scalar.h"

using clk = std::chrono::steady_clock;
template <class F>
static double time_us(F&& f, int reps) {
  f();
  auto t0 = clk::now();
  for (int i = 0; i < reps; ++i) f();
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
}

int main() {
  const perm::Circuit C = perm::build(52);
  uint64_t st[25] = {1};
  printf("keccak_f1600            %8.3f us\n", time_us([&] { merlin::keccak_f1600(st); }, 100000));
  std::vector<uint32_t> pi;
  std::vector<hsc::Sc> gamma, sL, sR, taus;
  hsc::Sc al, be, rh;
  uint64_t seed = 1;
  printf("draw_prover_randomness  %8.3f us/proof\n",
         time_us([&] { perm::draw_prover_randomness(C, perm::Seed::u64(seed++), pi, gamma, al, be, rh, sL, sR, taus); }, 2000));
  {
    perm::Seed sd[8];
    perm::RandomDraws d[8];
    perm::RandomDraws* dp[8];
    for (int j = 0; j < 8; ++j) dp[j] = &d[j];
    printf("draw_prover_randomness_x8 %6.3f us/proof\n", time_us([&] {
             for (int j = 0; j < 8; ++j) sd[j] = perm::Seed::u64(seed++);
             perm::draw_prover_randomness_x8(C, sd, dp);
           }, 500) / 8);
    uint8_t wide[64];
    for (int i = 0; i < 64; ++i) wide[i] = (uint8_t)(i * 37 + 1);
    volatile uint64_t sink = 0;
    printf("from_wide               %8.3f ns\n", time_us([&] {
             for (int r = 0; r < 1000; ++r) { wide[0] = (uint8_t)r; sink += hsc::from_wide(wide).v[0]; }
           }, 200));
  }
  uint8_t pt[32] = {0};
  printf("transcript 105 V + ch   %8.3f us/proof\n", time_us(
                                                           [&] {
                                                             merlin::Transcript tr((const uint8_t*)"bp", 2);
                                                             tr.arithmetic_domain_sep(128);
                                                             for (int i = 0; i < 105; ++i) tr.append_point("V", pt);
                                                             volatile auto x = tr.challenge_scalar("x_perm");
                                                             (void)x;
                                                           },
                                                           2000));
  std::vector<hsc::Sc> v, aL, aR, aO;
  const hsc::Sc x = hsc::from_u64(12345);
  printf("witness                 %8.3f us/proof\n", time_us([&] { perm::witness(C, pi, x, v, aL, aR, aO); }, 5000));
  printf("powers(z, Q+1)          %8.3f us/proof\n", time_us([&] { volatile auto p = hsc::powers(x, C.Q + 1); }, 5000));
  std::vector<hsc::Sc> zq = hsc::powers(x, C.Q + 1);
  zq.erase(zq.begin());
  printf("zW(WV)                  %8.3f us/proof\n", time_us([&] { volatile auto p = perm::zW(C.WV, zq, C.m); }, 5000));
  printf("scalar mul              %8.3f ns\n",
         time_us([&] { for (int i = 0; i < 1000; ++i) gamma[i & 63] = hsc::mul(gamma[i & 63], x); }, 2000) * 1e3 / 1000);
  printf("scalar invert           %8.3f us\n", time_us([&] { volatile auto y = hsc::invert(x); }, 2000));
  // field / group ops
  // ristretto255 basepoint encoding (RFC 9496)
  static const uint8_t Benc[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9,
                                   0x61, 0xc5, 0x00, 0x51, 0x5f, 0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82,
                                   0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
  h25519::ge P;
  if (!h25519::decode(P, Benc)) return 1;
  printf("fe_mul                  %8.3f ns\n", time_us([&] { for (int i = 0; i < 1000; ++i) P.X = h25519::fe_mul(P.X, P.Y); }, 2000) * 1e3 / 1000);
  printf("ge_dbl                  %8.3f ns\n", time_us([&] { for (int i = 0; i < 1000; ++i) P = h25519::ge_dbl(P); }, 500) * 1e3 / 1000);
  h25519::ge Q = h25519::ge_dbl(P);
  printf("ge_add                  %8.3f ns\n", time_us([&] { for (int i = 0; i < 1000; ++i) P = h25519::ge_add(P, Q); }, 500) * 1e3 / 1000);
  std::vector<h25519::ge> pts(256, P);
  for (int i = 1; i < 256; ++i) pts[i] = h25519::ge_add(pts[i - 1], Q);
  std::vector<uint8_t> enc(256 * 32);
  printf("encode_double_batch 256 %8.3f us\n", time_us([&] { h25519::encode_double_batch(pts.data(), 256, enc.data()); }, 200));
  printf("encode (single)         %8.3f us\n", time_us([&] { h25519::encode(enc.data(), P); }, 2000));
  return 0;
}
