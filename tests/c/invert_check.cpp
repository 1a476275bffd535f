// hsc::invert_vartime (binary extended Euclid) against hsc::invert (Fermat,
// a^(l-2)) on random scalars and edge values 1, 2, l-1, l-2, 2^k, small and
// sparse ones, and batch_invert's vartime form against its constant-time
// form (tests/test_host_sanitizers.py compiles and runs it).
#include <chrono>
#include <cstdio>
#include <random>
#include "host/scalar.h"
int main() {
  std::mt19937_64 g(7);
  long bad = 0, n = 0;
  auto check = [&](const hsc::Sc& a) {
    if (hsc::is_zero(a)) return;
    ++n;
    const hsc::Sc x = hsc::invert_vartime(a), y = hsc::invert(a);
    if (x != y || hsc::mul(x, a) != hsc::one()) {
      if (bad++ < 5) printf("mismatch %016llx..\n", (unsigned long long)a.v[0]);
    }
  };
  check(hsc::one());
  check(hsc::from_u64(2));
  check(hsc::sub(hsc::zero(), hsc::one()));
  check(hsc::sub(hsc::zero(), hsc::from_u64(2)));
  for (int k = 0; k < 253; ++k) {
    hsc::Sc p = hsc::zero();
    p.v[k >> 6] = 1ULL << (k & 63);
    check(p);
  }
  for (uint64_t s = 1; s < 2000; ++s) check(hsc::from_u64(s));
  for (long it = 0; it < 200000; ++it) {
    uint8_t b[64];
    for (int i = 0; i < 64; i += 8) {
      const uint64_t w = g();
      memcpy(b + i, &w, 8);
    }
    hsc::Sc a = hsc::from_wide(b);
    if (it % 5 == 0) a.v[1] = a.v[2] = 0;
    if (it % 7 == 0) a.v[0] = 0;
    check(a);
  }
  std::vector<hsc::Sc> xs, ys;
  for (int i = 0; i < 37; ++i) {
    uint8_t b[64];
    for (int j = 0; j < 64; j += 8) {
      const uint64_t w = g() | 1;
      memcpy(b + j, &w, 8);
    }
    xs.push_back(hsc::from_wide(b));
  }
  ys = xs;
  const hsc::Sc pa = hsc::batch_invert(xs, true, false), pb = hsc::batch_invert(ys, true, true);
  if (xs != ys || pa != pb) ++bad, puts("batch_invert vartime mismatch");
  // powers / powers_mont (four interleaved chains) against one chain of mul
  for (int t = 0; t < 40; ++t) {
    const hsc::Sc x = t == 0 ? hsc::one() : t == 1 ? hsc::zero() : xs[t % xs.size()];
    const size_t n = t < 20 ? (size_t)t : 1024 + t;
    const std::vector<hsc::Sc> p = hsc::powers(x, n), pm = hsc::powers_mont(x, n);
    hsc::Sc c = hsc::one();
    for (size_t i = 0; i < n; ++i) {
      if (p[i] != c || pm[i] != hsc::to_mont(c)) {
        if (bad++ < 5) printf("powers mismatch t=%d i=%zu\n", t, i);
        break;
      }
      c = hsc::mul(c, x);
    }
  }
  const auto tp0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 200; ++i) xs[0].v[0] ^= hsc::powers(xs[1], 1024)[1023].v[0] & 1;
  const auto tp1 = std::chrono::steady_clock::now();
  printf("powers(1024) %.2f us\n", std::chrono::duration<double, std::micro>(tp1 - tp0).count() / 200);
  const auto t0 = std::chrono::steady_clock::now();
  hsc::Sc acc = xs[0];
  for (int i = 0; i < 20000; ++i) acc = hsc::add(hsc::invert_vartime(acc), hsc::one());
  const auto t1 = std::chrono::steady_clock::now();
  for (int i = 0; i < 2000; ++i) acc = hsc::add(hsc::invert(acc), hsc::one());
  const auto t2 = std::chrono::steady_clock::now();
  printf("checked %ld, mismatches: %ld; invert_vartime %.2f us, invert %.2f us (%llx)\n", n, bad,
         std::chrono::duration<double, std::micro>(t1 - t0).count() / 20000,
         std::chrono::duration<double, std::micro>(t2 - t1).count() / 2000, (unsigned long long)acc.v[0]);
  return bad ? 1 : 0;
}
