// Host-side parallel-for over independent proofs (transcripts, challenge
// scalars, witness polynomials).  A persistent pool (spawning threads per
// call costs ~20 us each, more than a batch of transcript operations):
// threads = BPP_HOST_THREADS or min(granted CPUs / LOCAL_WORLD_SIZE, 16) / 4;
// items are claimed
// from an atomic counter; the calling thread works too.  Concurrent calls
// share the workers; a call from inside a pool task runs inline.
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
#include <pthread.h>
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
    // A quarter of the granted CPUs (4 of the box's 16): every batch in
    // flight has its own driver thread that works on its jobs too, and the
    // prover is GPU-bound, so more workers only spin.  Measured on the box
    // (tools/gpu_batch_sweep.sh, 52-card proofs/s, two runs each): 256-proof
    // batches x 8 in flight with 2 / 4 / 8 threads 196-206 K / 212-220 K /
    // 206-213 K (8 threads: 9.4 cores busy, 45 us CPU per proof, against 6.5
    // and 30 us with 4); 128 x 12 with 8 / 4 threads 138-144 K / 172-180 K.
    // (round 1: 16 threads x 4 in flight 52-64 K, 8 x 8 75-80 K;
    // tools/EXPERIMENTS.md exp2-4)
    // Several ranks on one node (torchrun's LOCAL_WORLD_SIZE) share the
    // cgroup's CPUs: each sizes its pool from its share.
    unsigned share = granted_cpus();
    if (const char* lw = getenv("LOCAL_WORLD_SIZE")) share = std::max(1u, share / std::max(1, atoi(lw)));
    const unsigned v = e ? (unsigned)atoi(e) : std::max(1u, std::min(16u, share) / 4);
    return std::max(1u, v);
  }();
  return n;
}

// Workers spin (with pause) for ~BPP_POOL_SPIN_US after their last item
// before sleeping on a condition variable, so the prover's stream of short
// host phases (one every 0.1-0.3 ms) is not paid in futex wake-ups.  Several
// callers (independent proof batches in flight, one driver thread each) may
// run jobs at once: active jobs sit in a list and workers claim items from
// any of them, so one batch's host phase does not queue behind another's.
// A caller works on its own job, waits until every item is done, unlists
// the job and waits for the workers still inside it to leave.
class Pool {
 public:
  explicit Pool(unsigned workers, int spin_us = -1) {
    const char* e = getenv("BPP_POOL_SPIN_US");
    spin_us_ = spin_us >= 0 ? spin_us : e ? atoi(e) : 300;
    for (unsigned i = 0; i < workers; ++i)
      th_.emplace_back([this] {
        pthread_setname_np(pthread_self(), "bpp-pool");  // (host profiles tell workers from drivers)
        loop();
      });
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
    Job j;
    j.f = &f;
    j.n = n;
    {
      std::lock_guard<std::mutex> g(mu_);
      jobs_.push_back(&j);
      njobs_.fetch_add(1);
      avail_.fetch_add(1);  // (the thread that exhausts j's items takes it back, work())
    }
    if (sleepers_.load() > 0) cv_.notify_all();
    // the caller works on its own job too; a for_each from one of its tasks
    // runs inline, as it does from a worker's (found by TSan: the nested
    // call went to the pool and ran the inner body on several threads)
    tl_task() = true;
    work(j);
    tl_task() = false;
    while (j.done.load() < n) cpu_relax();
    {
      std::lock_guard<std::mutex> g(mu_);
      jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &j));
      njobs_.fetch_sub(1);
    }
    while (j.inside.load() != 0) cpu_relax();
  }
  static bool in_worker() { return tl_worker() || tl_task(); }

 private:
  struct Job {
    const std::function<void(size_t)>* f = nullptr;
    size_t n = 0;
    std::atomic<size_t> next{0}, done{0};
    std::atomic<unsigned> inside{0};
  };
  static void cpu_relax() { __builtin_ia32_pause(); }
  static bool& tl_worker() {
    static thread_local bool w = false;
    return w;
  }
  static bool& tl_task() {
    static thread_local bool t = false;
    return t;
  }
  void work(Job& j) {
    size_t k = 0, i;
    while ((i = j.next.fetch_add(1)) < j.n) {
      (*j.f)(i);
      ++k;
    }
    if (i == j.n) avail_.fetch_sub(1);  // exactly one claimer sees i == n
    if (k) j.done.fetch_add(k);
  }
  // a listed job with unclaimed items, entered (inside + 1), or null
  Job* claim() {
    std::lock_guard<std::mutex> g(mu_);
    for (Job* j : jobs_)
      if (j->next.load() < j->n) {
        j->inside.fetch_add(1);
        return j;
      }
    return nullptr;
  }
  void loop() {
    tl_worker() = true;
    auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0; !stop_.load(); ++it) {
      // (claim() takes the mutex: only when some listed job still has
      // unclaimed items -- spinning workers polling claim() contended the
      // mutex with every caller, ~10 % of the host CPU samples in futex calls)
      if (avail_.load(std::memory_order_relaxed) > 0) {
        if (Job* j = claim()) {
          work(*j);
          j->inside.fetch_sub(1);
          t0 = std::chrono::steady_clock::now();
          continue;
        }
      }
      cpu_relax();
      if ((it & 255u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) {
        std::unique_lock<std::mutex> g(mu_);
        sleepers_.fetch_add(1);
        cv_.wait(g, [&] { return stop_.load() || avail_.load() > 0; });
        sleepers_.fetch_sub(1);
        t0 = std::chrono::steady_clock::now();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Job*> jobs_;
  std::atomic<unsigned> njobs_{0}, sleepers_{0};
  std::atomic<int> avail_{0};  // listed jobs whose items are not all claimed
  std::atomic<bool> stop_{false};
  int spin_us_ = 300;
};

inline Pool& pool() {
  static Pool p(threads() - 1);
  return p;
}

// Threads for bulk host copies into the pinned staging arena (ctx_stage_copy):
// BPP_COPY_THREADS or min(granted CPUs / LOCAL_WORLD_SIZE, 4).  Its own pool,
// so that a batch verification's 17 MB of staging does not queue behind the
// prover's host phases on the compute pool; 8 threads measured the same as 4
// on the config-5 upload (0.23-0.28 ms either way: the copy engine paces it,
// profiles/r04_copy_ab.txt).
inline unsigned copy_threads() {
  static const unsigned n = [] {
    const char* e = getenv("BPP_COPY_THREADS");
    unsigned share = granted_cpus();
    if (const char* lw = getenv("LOCAL_WORLD_SIZE")) share = std::max(1u, share / std::max(1, atoi(lw)));
    return std::max(1u, e ? (unsigned)atoi(e) : std::min(4u, share));
  }();
  return n;
}

inline Pool& copy_pool() {
  static Pool p(copy_threads() - 1, 50);  // (copies come in bursts: a short spin)
  return p;
}

template <class F>
void for_each_copy(size_t n, F&& f) {
  if (n <= 1 || copy_threads() <= 1 || Pool::in_worker()) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  const std::function<void(size_t)> fn = [&](size_t i) { f(i); };
  copy_pool().run(n, fn);
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
