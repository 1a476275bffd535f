// Host-side parallel-for over independent proofs (transcripts, challenge
// scalars, witness polynomials).  Threads = BPP_HOST_THREADS or
// min(hardware threads, 16); work items are claimed from an atomic counter.
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>
#include <vector>

namespace par {

inline unsigned threads() {
  static unsigned n = 0;
  if (!n) {
    const char* e = getenv("BPP_HOST_THREADS");
    unsigned v = e ? (unsigned)atoi(e) : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    n = std::max(1u, v);
  }
  return n;
}

template <class F>
void for_each(size_t n, F&& f) {
  const unsigned nt = (unsigned)std::min<size_t>(n, threads());
  if (nt <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
  };
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

}  // namespace par
