// Host-side parallel-for over independent proofs (transcripts, challenge
// scalars, witness polynomials).  A persistent pool (spawning threads per
// call costs ~20 us each, more than a batch of transcript operations):
// threads = BPP_HOST_THREADS or min(granted CPUs, 16); items are claimed
// from an atomic counter; the calling thread works too.  Calls are
// serialised; a call from inside a pool task runs inline.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace par {

// CPUs granted to this process: the cgroup v2 quota when one is set (the
// GPU box reports 256 CPUs but grants 16 per GPU), else the hardware count.
inline unsigned granted_cpus() {
  unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long period = 0;
    if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
      hw = std::min<unsigned>(hw, std::max(1L, atol(q) / period));
    fclose(f);
  }
  return hw;
}

inline unsigned threads() {
  static const unsigned n = [] {
    const char* e = getenv("BPP_HOST_THREADS");
    // measured on the box (16-CPU quota): 16 threads 6.8 ms vs 8 threads
    // 7.4 ms per 128-proof batch, 19 vs 25 ms per 512
    const unsigned v = e ? (unsigned)atoi(e) : std::min(16u, granted_cpus());
    return std::max(1u, v);
  }();
  return n;
}

// Workers spin (with pause) for ~BPP_POOL_SPIN_US after each job before
// sleeping on a condition variable, so the prover's stream of short host
// phases (one every 0.1-0.3 ms) is not paid in futex wake-ups; the caller
// waits only until every item is done and every worker that entered the
// job has left it.
class Pool {
 public:
  explicit Pool(unsigned workers) {
    const char* e = getenv("BPP_POOL_SPIN_US");
    spin_us_ = e ? atoi(e) : 300;
    for (unsigned i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_.store(true);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(size_t n, const std::function<void(size_t)>& f) {
    std::lock_guard<std::mutex> call(call_mu_);
    n_ = n;
    next_.store(0);
    done_.store(0);
    job_.store(&f);
    gen_.fetch_add(1);
    if (sleepers_.load() > 0) {
      { std::lock_guard<std::mutex> g(mu_); }
      cv_.notify_all();
    }
    work(f, n);
    while (done_.load() < n) cpu_relax();
    job_.store(nullptr);
    while (inside_.load() != 0) cpu_relax();
  }
  static bool in_worker() { return tl_worker(); }

 private:
  static void cpu_relax() { __builtin_ia32_pause(); }
  static bool& tl_worker() {
    static thread_local bool w = false;
    return w;
  }
  void work(const std::function<void(size_t)>& f, size_t n) {
    size_t k = 0;
    for (size_t i; (i = next_.fetch_add(1)) < n; ++k) f(i);
    if (k) done_.fetch_add(k);
  }
  void loop() {
    tl_worker() = true;
    uint64_t seen = gen_.load();
    for (;;) {
      // spin for a new generation, then sleep
      auto t0 = std::chrono::steady_clock::now();
      for (unsigned it = 0; gen_.load() == seen && !stop_.load(); ++it) {
        cpu_relax();
        if ((it & 255u) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) {
          std::unique_lock<std::mutex> g(mu_);
          sleepers_.fetch_add(1);
          cv_.wait(g, [&] { return stop_.load() || gen_.load() != seen; });
          sleepers_.fetch_sub(1);
          break;
        }
      }
      if (stop_.load()) return;
      seen = gen_.load();
      inside_.fetch_add(1);
      if (const std::function<void(size_t)>* f = job_.load()) work(*f, n_);
      inside_.fetch_sub(1);
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_;
  std::atomic<const std::function<void(size_t)>*> job_{nullptr};
  size_t n_ = 0;
  std::atomic<size_t> next_{0}, done_{0};
  std::atomic<unsigned> inside_{0}, sleepers_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
  int spin_us_ = 300;
};

inline Pool& pool() {
  static Pool p(threads() - 1);
  return p;
}

template <class F>
void for_each(size_t n, F&& f) {
  if (n <= 1 || threads() <= 1 || Pool::in_worker()) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  const std::function<void(size_t)> fn = [&](size_t i) { f(i); };
  pool().run(n, fn);
}

}  // namespace par
