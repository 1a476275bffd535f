// Context, workspace, profiling and device-memory entry points of the C ABI.
#include <execinfo.h>
#include <malloc.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "ctx.h"
#include "host/par.h"

// memcpy to / from the pinned arena, split over the copy pool above 512 KB
// (a 2.6 MB scalar upload is ~0.25 ms on one core of the box; par.h
// copy_threads)
// Pinned host buffers handed out by bpp_host_alloc (start -> bytes), so that
// an entry point can tell them from pageable memory without a runtime
// query; other pointers are then looked up with hipPointerGetAttributes
// (memory a caller pinned itself with hipHostRegister; BPP_PIN_QUERY=0
// skips it -- config 5 single batches measured the same either way, r05)
static std::mutex g_pin_mu;
static std::map<uintptr_t, size_t> g_pinned;
void host_pinned_add(const void* p, size_t n) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[(uintptr_t)p] = n;
}
void host_pinned_remove(const void* p) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned.erase((uintptr_t)p);
}
bool host_is_pinned(const void* p, size_t n) {
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pinned.upper_bound((uintptr_t)p);
    if (it != g_pinned.begin()) {
      --it;
      if ((uintptr_t)p >= it->first && (uintptr_t)p + n <= it->first + it->second) return true;
    }
  }
  static const bool query = [] {  // (BPP_PIN_QUERY=0: the registry alone; measured the same, r05)
    const char* e = getenv("BPP_PIN_QUERY");
    return !e || atoi(e) != 0;
  }();
  if (!query) return false;
  // both ends of [p, p + n) must be page-locked (a buffer the caller
  // registered only in part is staged as pageable)
  auto pinned_at = [](const void* q) {
    hipPointerAttribute_t at;
    const bool pin = hipPointerGetAttributes(&at, q) == hipSuccess && at.type == hipMemoryTypeHost;
    (void)hipGetLastError();  // (a pageable pointer leaves an error code behind)
    return pin;
  };
  return pinned_at(p) && (n <= 1 || pinned_at((const uint8_t*)p + n - 1));
}

// Non-temporal copy into the pinned arena: the arena is only read back by
// the copy engine, so streaming stores skip the read-for-ownership of every
// destination line (a plain memcpy moves each byte three times over the
// memory bus, this one twice).  BPP_STAGE_NT=0 falls back to memcpy (A/B).
static void copy_nt(uint8_t* d, const uint8_t* s, size_t n) {
  while (n && ((uintptr_t)d & 31)) {
    *d++ = *s++;
    --n;
  }
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256((const __m256i*)(s + i));
    const __m256i b = _mm256_loadu_si256((const __m256i*)(s + i + 32));
    const __m256i c = _mm256_loadu_si256((const __m256i*)(s + i + 64));
    const __m256i e = _mm256_loadu_si256((const __m256i*)(s + i + 96));
    _mm256_stream_si256((__m256i*)(d + i), a);
    _mm256_stream_si256((__m256i*)(d + i + 32), b);
    _mm256_stream_si256((__m256i*)(d + i + 64), c);
    _mm256_stream_si256((__m256i*)(d + i + 96), e);
  }
  if (i < n) memcpy(d + i, s + i, n - i);
  _mm_sfence();  // (the DMA is enqueued by this thread or after the pool's join)
}

void ctx_stage_copy(void* dst, const void* src, size_t bytes) {
  static const bool nt = [] {
    const char* e = getenv("BPP_STAGE_NT");
    return !e || atoi(e) != 0;
  }();
  auto cp = [&](uint8_t* d, const uint8_t* s, size_t n) {
    if (nt && n >= 4096)
      copy_nt(d, s, n);
    else
      memcpy(d, s, n);
  };
  const size_t chunk = 128u << 10;
  if (bytes < (512u << 10)) {
    cp((uint8_t*)dst, (const uint8_t*)src, bytes);
    return;
  }
  par::for_each_copy((bytes + chunk - 1) / chunk, [&](size_t i) {
    const size_t o = i * chunk;
    cp((uint8_t*)dst + o, (const uint8_t*)src + o, std::min(chunk, bytes - o));
  });
}

int ctx_ws(bpp_ctx* ctx, const char* name, size_t bytes, void** out) {
  auto& b = ctx->ws[name];
  if (b.bytes < bytes) {
    ctx->off_cache_ptr = nullptr;  // an address may be reused: forget cached contents
    ctx->h2d_cache.clear();
    if (b.p) BPP_HIP(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    size_t want = bytes + bytes / 8 + 256;
    BPP_HIP(hipMalloc(&b.p, want));
    b.bytes = want;
  }
  *out = b.p;
  return BPP_OK;
}

int ctx_pinned(bpp_ctx* ctx, size_t bytes, void** out) {
  if (ctx->pinned_bytes < bytes) {
    if (ctx->pinned) BPP_HIP(hipHostFree(ctx->pinned));
    ctx->pinned = nullptr;
    ctx->pinned_bytes = 0;
    BPP_HIP(hipHostMalloc(&ctx->pinned, bytes));
    ctx->pinned_bytes = bytes;
  }
  *out = ctx->pinned;
  return BPP_OK;
}

int ctx_host_buf(bpp_ctx* ctx, const char* name, size_t bytes, void** out) {
  auto& b = ctx->host_bufs[name];
  if (b.second < bytes) {
    if (b.first) BPP_HIP(hipHostFree(b.first));
    b = {nullptr, 0};
    void* h = nullptr;
    BPP_HIP(hipHostMalloc(&h, bytes));
    b = {h, bytes};
  }
  void* d = nullptr;
  BPP_HIP(hipHostGetDevicePointer(&d, b.first, 0));
  if (d != b.first) {  // (the kernels and the host share one pointer)
    ctx->err = "ctx_host_buf: pinned buffer has a distinct device address";
    return BPP_ERR_DEVICE;
  }
  *out = b.first;
  return BPP_OK;
}

int ctx_zc_out(bpp_ctx* ctx, const char* name, size_t bytes, uint32_t** d) {
  if (ctx->zc_live.count(name)) BPP_TRY(ctx_sync(ctx));
  void* b = nullptr;
  BPP_TRY(ctx_host_buf(ctx, name, std::max<size_t>(bytes, 32), &b));
  ctx->zc_live.insert(name);
  *d = (uint32_t*)b;
  return BPP_OK;
}

int ctx_zc_in(bpp_ctx* ctx, const char* name, const void* h, size_t bytes, uint32_t** d) {
  BPP_TRY(ctx_zc_out(ctx, name, bytes, d));
  if (bytes) memcpy(*d, h, bytes);
  return BPP_OK;
}

// The waiting thread polls an event with 5 us sleeps instead of
// hipStreamSynchronize's spin: with 8-12 proof batches in flight, their
// driver threads spinning in the HSA signal wait were ~25 % of the host CPU
// samples (tools/hostprof).  12 batches in flight: 104-108.5 K vs 99.5-100.6
// K proofs/s with 8 and the spin, 11.9 vs 14.3 host cores busy
// (tools/ab_sync.sh; 2 / 10 us sleeps measured the same; a
// hipEventBlockingSync event kept the spin's CPU and throughput).  A 5 us
// nanosleep sleeps ~55 us under the default 50 us timer slack (65 vs 16 us
// per launch + copy + wait round trip, tools/ubench/hipapi), but a 1 us slack,
// with or without a 15 us spin first, measured within noise (105-117 K vs
// 101-120 K proofs/s at 12 in flight).
int ctx_sync(bpp_ctx* ctx) {
  if (ctx->sync_spin_us) return ctx_sync_latency(ctx, ctx->sync_spin_us);
  if (!ctx->sync_ev) BPP_HIP(hipEventCreateWithFlags(&ctx->sync_ev, hipEventDisableTiming));
  BPP_HIP(hipEventRecord(ctx->sync_ev, ctx->stream));
  for (hipError_t r; (r = hipEventQuery(ctx->sync_ev)) != hipSuccess;) {
    if (r != hipErrorNotReady) BPP_HIP(r);
    struct timespec ts = {0, 5000L};
    nanosleep(&ts, nullptr);
  }
  ctx->zc_live.clear();
  ctx->stage_used = 0;
  return BPP_OK;
}

int ctx_sync_latency(bpp_ctx* ctx, unsigned spin_us) {
  static const int spin_env = [] {  // (BPP_SYNC_SPIN_US overrides, for A/B; 0 = ctx_sync)
    const char* e = getenv("BPP_SYNC_SPIN_US");
    return e ? atoi(e) : -1;
  }();
  if (spin_env >= 0) spin_us = (unsigned)spin_env;
  if (!ctx->sync_ev) BPP_HIP(hipEventCreateWithFlags(&ctx->sync_ev, hipEventDisableTiming));
  BPP_HIP(hipEventRecord(ctx->sync_ev, ctx->stream));
  const auto t0 = std::chrono::steady_clock::now();
  for (hipError_t r; (r = hipEventQuery(ctx->sync_ev)) != hipSuccess;) {
    if (r != hipErrorNotReady) BPP_HIP(r);
    if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(spin_us)) {
      __builtin_ia32_pause();
      continue;
    }
    struct timespec ts = {0, 5000L};
    nanosleep(&ts, nullptr);
  }
  ctx->zc_live.clear();
  ctx->stage_used = 0;
  return BPP_OK;
}

int ctx_done_flag(bpp_ctx* ctx, uint32_t** ticket, uint32_t** word, uint32_t* tag) {
  if (!ctx->done_ticket) {
    BPP_HIP(hipMalloc(&ctx->done_ticket, 4));
    BPP_HIP(hipMemsetAsync(ctx->done_ticket, 0, 4, ctx->stream));
  }
  if (!ctx->done_word) {
    BPP_HIP(hipHostMalloc((void**)&ctx->done_word, 64, hipHostMallocCoherent));
    __atomic_store_n(ctx->done_word, 0u, __ATOMIC_RELEASE);
  }
  if (++ctx->done_tag == 0) ++ctx->done_tag;  // (0: never a live tag)
  *ticket = ctx->done_ticket;
  *word = ctx->done_word;
  *tag = ctx->done_tag;
  return BPP_OK;
}

int ctx_wait_flag(bpp_ctx* ctx, const uint32_t* word, uint32_t tag) {
  const auto t0 = std::chrono::steady_clock::now();
  const auto cap = std::chrono::microseconds(ctx->sync_spin_us);
  while (__atomic_load_n(word, __ATOMIC_ACQUIRE) != tag) {
    if (std::chrono::steady_clock::now() - t0 >= cap) {
      BPP_TRY(ctx_sync(ctx));  // the launch has ended (or failed: reported here)
      if (__atomic_load_n(word, __ATOMIC_ACQUIRE) != tag) {
        // a launch that ended without its flag (none should): the results
        // are complete after the sync; re-zero the ticket for the next one
        BPP_HIP(hipMemsetAsync(ctx->done_ticket, 0, 4, ctx->stream));
      }
      return BPP_OK;
    }
    __builtin_ia32_pause();
  }
  return BPP_OK;
}

static int stage_take(bpp_ctx* ctx, size_t bytes, uint8_t** out) {
  const size_t need = (bytes + 255) & ~(size_t)255;
  if (ctx->stage_used + need > ctx->stage_cap) {
    BPP_TRY(ctx_sync(ctx));  // every staged copy has completed
    if (need > ctx->stage_cap) {
      // secret spans recorded in the old arena (prove_wipe's list) are zeroed
      // now and dropped: after the free they would point at unmapped memory
      for (auto& st : ctx->secret_stage) memset(st.first, 0, st.second);
      ctx->secret_stage.clear();
      ctx->wiped.clear();
      if (ctx->stage) BPP_HIP(hipHostFree(ctx->stage));
      ctx->stage = nullptr;
      ctx->stage_cap = 0;
      const size_t cap = std::max<size_t>(need, 16u << 20);
      BPP_HIP(hipHostMalloc((void**)&ctx->stage, cap));
      ctx->stage_cap = cap;
    }
  }
  *out = ctx->stage + ctx->stage_used;
  ctx->stage_used += need;
  // the arena is reused after every sync: bytes handed out again no longer
  // belong to the last wipe, so they leave its span list (what is left of a
  // span still holds the wipe's zeros for bpp_debug_secret_residue)
  if (!ctx->wiped.empty()) {
    uint8_t *lo = *out, *hi = *out + need;
    std::vector<std::pair<uint8_t*, size_t>> keep;
    keep.reserve(ctx->wiped.size() + 1);
    for (const auto& s : ctx->wiped) {
      uint8_t *a = s.first, *b = s.first + s.second;
      if (b <= lo || hi <= a) {
        keep.push_back(s);
        continue;
      }
      if (a < lo) keep.push_back({a, (size_t)(lo - a)});
      if (hi < b) keep.push_back({hi, (size_t)(b - hi)});
    }
    ctx->wiped.swap(keep);
  }
  return BPP_OK;
}

int ctx_h2d_stage(bpp_ctx* ctx, size_t bytes, uint8_t** p) { return stage_take(ctx, bytes, p); }

void ctx_secret_span(bpp_ctx* ctx, uint8_t* p, size_t bytes) {
  if (!bytes) return;
  uint8_t *lo = p, *hi = p + bytes;
  auto& v = ctx->secret_stage;
  for (size_t i = 0; i < v.size();) {  // absorb every span that overlaps or touches [lo, hi)
    uint8_t *a = v[i].first, *b = v[i].first + v[i].second;
    if (a <= hi && lo <= b) {
      lo = std::min(lo, a);
      hi = std::max(hi, b);
      v[i] = v.back();
      v.pop_back();
    } else {
      ++i;
    }
  }
  v.emplace_back(lo, (size_t)(hi - lo));
}

int ctx_h2d_staged(bpp_ctx* ctx, void* d, const uint8_t* p, size_t bytes) {
  if (bytes) BPP_HIP(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, ctx->stream));
  return BPP_OK;
}

int ctx_h2d(bpp_ctx* ctx, void* d, const void* h, size_t bytes) {
  if (!bytes) return BPP_OK;
  uint8_t* p = nullptr;
  BPP_TRY(stage_take(ctx, bytes, &p));
  ctx_stage_copy(p, h, bytes);
  BPP_HIP(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, ctx->stream));
  return BPP_OK;
}

// In pieces of 2 MB: the DMA of piece i runs while the host stages piece
// i + 1 (a batch verification's 17 MB of proofs and V: the copy engine's
// ~0.35 ms then hides under the staging instead of following it).
int ctx_h2d2(bpp_ctx* ctx, void* d, const void* h0, size_t n0, const void* h1, size_t n1) {
  if (!n0 && !n1) return BPP_OK;
  uint8_t* p = nullptr;
  const size_t total = n0 + n1, piece = (size_t)2 << 20;
  BPP_TRY(stage_take(ctx, total, &p));
  for (size_t off = 0; off < total;) {
    const size_t e = std::min(total, off + piece);
    if (off < n0) ctx_stage_copy(p + off, (const uint8_t*)h0 + off, std::min(e, n0) - off);
    if (e > n0) {
      const size_t s = std::max(off, n0);
      ctx_stage_copy(p + s, (const uint8_t*)h1 + (s - n0), e - s);
    }
    BPP_HIP(hipMemcpyAsync((uint8_t*)d + off, p + off, e - off, hipMemcpyHostToDevice, ctx->stream));
    off = e;
  }
  return BPP_OK;
}

int ctx_h2d_const(bpp_ctx* ctx, const char* name, void* d, const void* h, size_t bytes) {
  auto& e = ctx->h2d_cache[name];
  if (e.first == d && e.second.size() == bytes && !memcmp(e.second.data(), h, bytes)) return BPP_OK;
  BPP_TRY(ctx_h2d(ctx, d, h, bytes));
  e.first = d;
  e.second.assign((const uint8_t*)h, (const uint8_t*)h + bytes);
  return BPP_OK;
}

int ctx_d2h(bpp_ctx* ctx, void* h, const void* d, size_t bytes) {
  if (!bytes) return ctx_sync(ctx);
  uint8_t* p = nullptr;
  BPP_TRY(stage_take(ctx, bytes, &p));
  BPP_HIP(hipMemcpyAsync(p, d, bytes, hipMemcpyDeviceToHost, ctx->stream));
  BPP_TRY(ctx_sync(ctx));
  ctx_stage_copy(h, p, bytes);
  return BPP_OK;
}

int ctx_child(bpp_ctx* ctx, size_t i, bpp_ctx** out) {
  while (ctx->children.size() <= i) {
    bpp_ctx* c = nullptr;
    const int rc = bpp_ctx_create(ctx->device, &c);
    if (rc) {
      ctx->err = "creating a child context failed";
      return rc;
    }
    ctx->children.push_back(c);
  }
  *out = ctx->children[i];
  return BPP_OK;
}

int ctx_check_launch(bpp_ctx* ctx, const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    ctx->err = std::string(what) + ": " + hipGetErrorString(e);
    return BPP_ERR_DEVICE;
  }
  return BPP_OK;
}

static hipEvent_t ev_get(bpp_ctx* ctx) {
  if (!ctx->ev_pool.empty()) {
    hipEvent_t e = ctx->ev_pool.back();
    ctx->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  hipEventCreate(&e);
  return e;
}

ProfScope::ProfScope(bpp_ctx* c, const char* n) : ctx(c), name(n) {
  if (!ctx->prof) return;
  a = ev_get(ctx);
  b = ev_get(ctx);
  hipEventRecord(a, ctx->stream);
}

ProfScope::~ProfScope() {
  if (!ctx->prof || !a) return;
  hipEventRecord(b, ctx->stream);
  ctx->pending.push_back({name, a, b});
}

static void prof_resolve(bpp_ctx* ctx) {
  // stages that ran on child streams count under the parent
  for (bpp_ctx* c : ctx->children) {
    prof_resolve(c);
    for (auto& kv : c->prof_acc) {
      auto& acc = ctx->prof_acc[kv.first];
      acc.first += kv.second.first;
      acc.second += kv.second.second;
    }
    c->prof_acc.clear();
  }
  if (ctx->pending.empty()) return;
  hipStreamSynchronize(ctx->stream);
  for (auto& p : ctx->pending) {
    float ms = 0;
    hipEventElapsedTime(&ms, p.a, p.b);
    auto& acc = ctx->prof_acc[p.name];
    acc.first += ms;
    acc.second += 1;
    ctx->ev_pool.push_back(p.a);
    ctx->ev_pool.push_back(p.b);
  }
  ctx->pending.clear();
}

extern "C" {

// glibc's dynamic mmap threshold makes every batch's few-hundred-KB to
// few-MB host vectors (scalar arrays, encodings, staging) alternate between
// mmap and trimmed arena tops: mprotect, munmap and fresh-page faults showed
// up in a host profile of 8 batches in flight.  A fixed threshold and no
// trimming keep that memory in the arenas; a 64 MB top pad makes each
// per-thread arena grow in large steps (its mprotect calls were still 7.7 %
// of the host samples at 12 batches in flight: 315 -> 320 K proofs/s with
// the pad, tools/hostprof + prove_inflight_exp.py).  This changes the allocator policy
// of the whole host process, so it is opt-in (bench.py asks for it); loading
// the library changes nothing.
// BPP_TUNE_HW_QUEUES: HIP's hardware queues per process come from
// GPU_MAX_HW_QUEUES, read once when the HIP runtime starts; a prover with
// many batches in flight (one context and stream each) measured +2.5 % on 8
// queues over HIP's default 4 (368 vs 359 K proofs/s, profiles/
// r05_hw_queues_ab.txt).  The flag sets GPU_MAX_HW_QUEUES=8 unless the
// caller set it, so it only takes effect before anything in the process
// initialises HIP.
int bpp_host_tuning(uint32_t flags) {
  return bpp_guard(nullptr, [&]() -> int {
    if (flags & ~(uint32_t)(BPP_TUNE_MALLOC | BPP_TUNE_HW_QUEUES)) return BPP_ERR_ARG;
    if (flags & BPP_TUNE_MALLOC) {
      mallopt(M_MMAP_THRESHOLD, 64 << 20);
      mallopt(M_TRIM_THRESHOLD, 1 << 30);
      mallopt(M_TOP_PAD, 64 << 20);
    }
    if (flags & BPP_TUNE_HW_QUEUES) setenv("GPU_MAX_HW_QUEUES", "8", 0);
    return BPP_OK;
  });
}

uint32_t bpp_host_threads(void) { return par::threads(); }

// BPP_SEGV_TRACE=1: a SIGSEGV prints the host backtrace (addresses of this
// library's frames) and then runs the handler that was installed before
// (Python's faulthandler under pytest) -- a diagnostic for host-side faults on
// the GPU box, where no debugger may attach.
static struct sigaction g_prev_segv;
static void segv_trace(int sig, siginfo_t* si, void* uc) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  static const char msg[] = "libbpperm: fatal signal, host backtrace:\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(fr, n, 2);
  if (g_prev_segv.sa_flags & SA_SIGINFO) {
    if (g_prev_segv.sa_sigaction) return g_prev_segv.sa_sigaction(sig, si, uc);
  } else if (g_prev_segv.sa_handler != SIG_DFL && g_prev_segv.sa_handler != SIG_IGN) {
    return g_prev_segv.sa_handler(sig);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

int bpp_ctx_create(int device, bpp_ctx** out) {
  static const bool trace = [] {
    const char* e = getenv("BPP_SEGV_TRACE");
    if (e && e[0] == '1') {
      struct sigaction sa;
      memset(&sa, 0, sizeof sa);
      sa.sa_sigaction = segv_trace;
      sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
      sigemptyset(&sa.sa_mask);
      sigaction(SIGSEGV, &sa, &g_prev_segv);
    }
    return true;
  }();
  (void)trace;
  return bpp_guard(nullptr, [&]() -> int {
    if (!out) return BPP_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return BPP_ERR_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return BPP_ERR_DEVICE;
    bpp_ctx* ctx = new bpp_ctx();
    ctx->device = device;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
      delete ctx;
      return BPP_ERR_DEVICE;
    }
    *out = ctx;
    return BPP_OK;
  });
}

void bpp_ctx_destroy(bpp_ctx* ctx) {
  if (!ctx) return;
  for (bpp_ctx* c : ctx->children) bpp_ctx_destroy(c);
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  for (auto& kv : ctx->ws)
    if (kv.second.p) hipFree(kv.second.p);
  if (ctx->pinned) hipHostFree(ctx->pinned);
  for (auto& kv : ctx->host_bufs)
    if (kv.second.first) hipHostFree(kv.second.first);
  if (ctx->stage) hipHostFree(ctx->stage);
  for (auto& p : ctx->pending) {
    hipEventDestroy(p.a);
    hipEventDestroy(p.b);
  }
  for (auto e : ctx->ev_pool) hipEventDestroy(e);
  if (ctx->sync_ev) hipEventDestroy(ctx->sync_ev);
  if (ctx->done_ticket) hipFree(ctx->done_ticket);
  if (ctx->done_word) hipHostFree(ctx->done_word);
  if (ctx->up_sc) hipFree(ctx->up_sc);
  for (auto e : ctx->up_ev)
    if (e) hipEventDestroy(e);
  for (auto s : ctx->up_stream)
    if (s) {
      hipStreamSynchronize(s);
      hipStreamDestroy(s);
    }
  if (ctx->vj_ev_in) hipEventDestroy(ctx->vj_ev_in);
  if (ctx->vj_ev_dec) hipEventDestroy(ctx->vj_ev_dec);
  for (auto e : ctx->vj_ev_chunk) hipEventDestroy(e);
  for (auto e : ctx->vj_ev_chunk2) hipEventDestroy(e);
  if (ctx->vj_ev_vrep) hipEventDestroy(ctx->vj_ev_vrep);
  for (auto& sl : ctx->msm_slot)
    if (sl.done) hipEventDestroy(sl.done);
  hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* bpp_ctx_last_error(const bpp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void* bpp_ctx_stream(bpp_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int bpp_ctx_profile(bpp_ctx* ctx, int enable) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx) return BPP_ERR_ARG;
    ctx->prof = enable != 0;
    for (bpp_ctx* c : ctx->children) bpp_ctx_profile(c, enable);
    return BPP_OK;
  });
}

int bpp_ctx_profile_get(bpp_ctx* ctx, const char* stage, double* ms, uint64_t* launches) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !stage) return BPP_ERR_ARG;
    prof_resolve(ctx);
    auto it = ctx->prof_acc.find(stage);
    if (ms) *ms = it == ctx->prof_acc.end() ? 0.0 : it->second.first;
    if (launches) *launches = it == ctx->prof_acc.end() ? 0 : it->second.second;
    return BPP_OK;
  });
}

static void work_resolve(bpp_ctx* ctx) {
  for (bpp_ctx* c : ctx->children) {
    work_resolve(c);
    for (auto& kv : c->work) ctx->work[kv.first] += kv.second;
    c->work.clear();
  }
}

int bpp_ctx_work_get(bpp_ctx* ctx, const char* name, uint64_t* value) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !name || !value) return BPP_ERR_ARG;
    work_resolve(ctx);
    auto it = ctx->work.find(name);
    *value = it == ctx->work.end() ? 0 : it->second;
    return BPP_OK;
  });
}

void bpp_ctx_work_reset(bpp_ctx* ctx) {
  if (!ctx) return;
  work_resolve(ctx);
  ctx->work.clear();
}

void bpp_ctx_profile_reset(bpp_ctx* ctx) {
  if (!ctx) return;
  prof_resolve(ctx);
  ctx->prof_acc.clear();
}

int bpp_dev_alloc(bpp_ctx* ctx, size_t bytes, void** dptr) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !dptr) return BPP_ERR_ARG;
    BPP_HIP(hipSetDevice(ctx->device));
    BPP_HIP(hipMalloc(dptr, bytes ? bytes : 1));
    return BPP_OK;
  });
}

int bpp_dev_free(bpp_ctx* ctx, void* dptr) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx) return BPP_ERR_ARG;
    BPP_HIP(hipFree(dptr));
    return BPP_OK;
  });
}

int bpp_memcpy_htod(bpp_ctx* ctx, void* dst, const void* src, size_t bytes) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx) return BPP_ERR_ARG;
    BPP_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    BPP_HIP(hipStreamSynchronize(ctx->stream));
    return BPP_OK;
  });
}

int bpp_memcpy_dtoh(bpp_ctx* ctx, void* dst, const void* src, size_t bytes) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx) return BPP_ERR_ARG;
    BPP_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    BPP_HIP(hipStreamSynchronize(ctx->stream));
    return BPP_OK;
  });
}

int bpp_synchronize(bpp_ctx* ctx) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx) return BPP_ERR_ARG;
    BPP_HIP(hipStreamSynchronize(ctx->stream));
    return BPP_OK;
  });
}

}  // extern "C"
