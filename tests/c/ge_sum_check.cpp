// h25519::ge_sum_x8 (the IPA split rounds' J-partial sums, eight additions
// per AVX-512 IFMA vector) against one scalar ge_add chain per point, on
// random projective representatives of multiples of the base point, for the
// (n, J) shapes the rounds use and ragged ones; compared by encoding
// (tests/test_host_sanitizers.py compiles it with host/encode_x8.cpp).
#include <cstdio>
#include <random>
#include <vector>
#include "host/fe64.h"
using namespace h25519;
int main() {
  if (!encode_x8_available()) {
    puts("no IFMA: skipped, mismatches: 0");
    return 0;
  }
  const uint8_t B[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9, 0x61, 0xc5, 0x00, 0x51, 0x5f,
                         0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82, 0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
  ge g;
  if (!decode(g, B)) return 2;
  std::mt19937_64 rng(5);
  std::vector<ge> pool(997);
  ge cur = g;
  for (auto& p : pool) {
    cur = ge_add(cur, ge_dbl(cur));
    const fe lam = fe_c(rng() | 1, rng(), rng(), rng() >> 2);
    p = ge{fe_mul(cur.X, lam), fe_mul(cur.Y, lam), fe_mul(cur.Z, lam), fe_mul(cur.T, lam)};
  }
  long bad = 0, checked = 0;
  const size_t ns[] = {1, 2, 3, 5, 8, 16, 17, 64};
  const uint32_t Js[] = {2, 4, 8, 12, 16, 32, 64};
  for (size_t n : ns)
    for (uint32_t J : Js) {
      std::vector<ge> in(n * J), got(n);
      for (size_t k = 0; k < in.size(); ++k) in[k] = pool[(k * 7 + n + J) % pool.size()];
      if (n == 3 && J == 4) in[5] = ge_identity();  // an identity term
      ge_sum_x8(in.data(), n, J, got.data());
      for (size_t i = 0; i < n; ++i) {
        ge t = in[i * J];
        for (uint32_t j = 1; j < J; ++j) t = ge_add(t, in[i * J + j]);
        uint8_t a[32], b[32];
        encode(a, t);
        encode(b, got[i]);
        ++checked;
        if (memcmp(a, b, 32) != 0 && bad++ < 5) printf("mismatch n=%zu J=%u i=%zu\n", n, J, i);
      }
    }
  printf("checked %ld, mismatches: %ld\n", checked, bad);
  return bad ? 1 : 0;
}
