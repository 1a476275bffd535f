// Host-side parallel-for over independent proofs (transcripts, challenge
// scalars, witness polynomials).  A persistent pool (spawning threads per
// call costs ~20 us each, more than a batch of transcript operations):
// threads = BPP_HOST_THREADS or min(granted CPUs, 16); items are claimed
// from an atomic counter; the calling thread works too.  Calls are
// serialised; a call from inside a pool task runs inline.
#pragma once
#include <algorithm>
#include <atomic>
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

class Pool {
 public:
  explicit Pool(unsigned workers) {
    for (unsigned i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(size_t n, const std::function<void(size_t)>& f) {
    std::lock_guard<std::mutex> call(call_mu_);
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &f;
      n_ = n;
      next_.store(0);
      active_ = (unsigned)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work(f, n);
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [this] { return active_ == 0; });
    job_ = nullptr;
  }
  static bool in_worker() { return tl_worker(); }

 private:
  static bool& tl_worker() {
    static thread_local bool w = false;
    return w;
  }
  void work(const std::function<void(size_t)>& f, size_t n) {
    for (size_t i; (i = next_.fetch_add(1)) < n;) f(i);
  }
  void loop() {
    tl_worker() = true;
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(size_t)>* f;
      size_t n;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
        n = n_;
      }
      work(*f, n);
      {
        std::lock_guard<std::mutex> g(mu_);
        if (--active_ == 0) done_.notify_one();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  unsigned active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
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
