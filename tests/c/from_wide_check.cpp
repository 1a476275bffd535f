// hsc::from_wide (2^252 = -delta folding) against its Montgomery-form
// restatement hsc::from_wide_mont on random, all-ones, sparse and zero 64-byte
// inputs (tests/test_host_sanitizers.py compiles and runs it).
#include <cstdio>
#include <random>
#include <chrono>
#include "host/scalar.h"
int main() {
  std::mt19937_64 g(1);
  uint8_t b[64];
  long bad = 0;
  for (long it = 0; it < 2000000; ++it) {
    uint64_t w[8];
    for (int i = 0; i < 8; ++i) w[i] = g();
    if (it % 7 == 0) for (int i = 0; i < 8; ++i) w[i] = ~0ULL;       // max
    if (it % 11 == 0) for (int i = 0; i < 8; ++i) w[i] = it % 3 ? 0 : w[i];
    if (it % 13 == 0) { for (int i = 0; i < 8; ++i) w[i] = 0; w[it % 8] = g() >> (it % 64); }
    memcpy(b, w, 64);
    hsc::Sc a = hsc::from_wide(b), c = hsc::from_wide_mont(b);
    if (a != c) { if (bad++ < 5) printf("mismatch at %ld\n", it); }
  }
  printf("mismatches: %ld\n", bad);
  return bad ? 1 : 0;
}
