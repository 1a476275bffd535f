// Internal context / workspace / error plumbing shared by the HIP sources.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <exception>
#include <map>
#include <new>
#include <set>
#include <string>
#include <vector>

#include "../../include/bpperm.h"

struct bpp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
  };
  std::map<std::string, Buf> ws;
  // pinned host staging
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  // named pinned host buffers that kernels read / write in place (ctx_host_buf)
  std::map<std::string, std::pair<void*, size_t>> host_bufs;
  std::set<std::string> zc_live;  // host buffers handed to kernels since the last ctx_sync
  // pinned upload arena: bump-allocated, recycled after a stream sync
  uint8_t* stage = nullptr;
  size_t stage_cap = 0, stage_used = 0;
  hipEvent_t sync_ev = nullptr;  // ctx_sync's completion event
  // > 0: ctx_sync spins this many us before it sleeps (SyncSpin, for the
  // latency-bound callers: one IPA, small prover batches); 0 = sleep at once
  unsigned sync_spin_us = 0;
  // kernel -> host completion flag (ctx_done_flag): a device ticket counter
  // the last block of a launch resets, a coherent pinned word it then writes
  // with the launch's tag, and the tag counter
  uint32_t* done_ticket = nullptr;
  uint32_t* done_word = nullptr;
  uint32_t done_tag = 0;
  // profiling
  bool prof = false;
  struct Pend {
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<Pend> pending;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, std::pair<double, uint64_t>> prof_acc;
  // child contexts (own stream + workspaces) for sub-batches in flight
  // concurrently with this one
  std::vector<bpp_ctx*> children;
  // bpp_msm_submit / bpp_msm_collect: up to BPP_MSM_INFLIGHT single MSMs in
  // flight, slot s running on child context s
  struct MsmSlot {
    bool busy = false;
    uint64_t ticket = 0;
    hipEvent_t done = nullptr;
    uint32_t c = 0, wb = 0, Wn = 0, nterms = 1;
    void* h = nullptr;  // window terms (child's pinned buffer)
  };
  MsmSlot msm_slot[BPP_MSM_INFLIGHT];
  uint64_t msm_next_ticket = 1;
  // extra dynamic LDS per accumulation workgroup (bpp_msm_submit sets it when
  // another MSM is in flight: 3 instead of 4 workgroups per CU, so the other
  // MSM's sort kernels run beside the accumulation)
  size_t acc_lds_pad = 0;
  // contents of the "multi_off" workspace as last uploaded (msm.hip
  // upload_offsets): the prover's IPA rounds pass the same MSM offsets every
  // round, so an unchanged array skips its copy.  Cleared by any workspace
  // reallocation (ctx_ws).
  void* off_cache_ptr = nullptr;
  std::vector<uint32_t> off_cache;
  // ctx_h2d_const: per workspace name, the address and bytes last uploaded
  // (cleared with off_cache on any workspace reallocation)
  std::map<std::string, std::pair<void*, std::vector<uint8_t>>> h2d_cache;
  // algorithmic work issued on this context (bpp_ctx_work_get): "msm_terms"
  // (scalar-point terms of every MSM and Pedersen commitment launched),
  // "madds" (mixed additions of a table point), "padds" (additions of two
  // extended points: trees, bucket reductions), "msm_launches"
  std::map<std::string, uint64_t> work;
  // device batch-verification jobs (bpp_perm_verify_begin_dev) keep their
  // records and decompressed points in this context's "vj_*" workspaces; a
  // job is valid while its generation is the context's latest
  uint64_t vjob_gen = 0;
  // the device job's proof-point decompression runs on child context
  // VJ_CHILD beside the replay: vj_ev_in (inputs uploaded, ctx stream) ->
  // decompress -> vj_ev_dec (child stream), waited for before the MSM and
  // before the next upload overwrites the inputs
  hipEvent_t vj_ev_in = nullptr, vj_ev_dec = nullptr;
  bool vj_dec_pending = false;
  // one event per upload chunk (verify_begin_dev: each chunk's points are
  // decompressed as soon as its copy lands)
  std::vector<hipEvent_t> vj_ev_chunk;
  // the split replay (BPP_VERIFY_SPLIT): the proof-byte chunks' events, and
  // the end of the V-part replays on their child stream
  std::vector<hipEvent_t> vj_ev_chunk2;
  hipEvent_t vj_ev_vrep = nullptr;
  // bpp_msm_submit_host: the uploaded scalars of this (child) context's MSM,
  // copied on the parent's upload streams (up_stream, created on first use;
  // one per chunk of the copy) and signalled to this context's stream by
  // up_ev
  void* up_sc = nullptr;
  size_t up_sc_bytes = 0;
  hipStream_t up_stream[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t up_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // spans of the pinned arena that the last prover batch on this context
  // filled with secrets (draw templates and pi, the host-path witness), for
  // prove_wipe; `wiped` keeps the spans of the last wipe for
  // bpp_debug_secret_residue
  std::vector<std::pair<uint8_t*, size_t>> secret_stage, wiped;
};
#define VJ_CHILD BPP_MSM_INFLIGHT

inline void bpp_guard_note(bpp_ctx* ctx, const char* what) noexcept {
  if (!ctx) return;
  try {
    ctx->err = what;
  } catch (...) {
  }
}

struct bpp_points {
  bpp_ctx* ctx = nullptr;
  uint32_t* d = nullptr;  // n x 24 words (affine Niels)
  size_t n = 0;
};

#define BPP_HIP(call)                                                          \
  do {                                                                         \
    hipError_t _e = (call);                                                    \
    if (_e != hipSuccess) {                                                    \
      ctx->err = std::string(#call) + ": " + hipGetErrorString(_e);            \
      return BPP_ERR_DEVICE;                                                   \
    }                                                                          \
  } while (0)

#define BPP_TRY(expr)            \
  do {                           \
    int _rc = (expr);            \
    if (_rc != BPP_OK) return _rc; \
  } while (0)

// The C-ABI boundary: every int-returning bpp_* entry point runs its body
// through bpp_guard, so no C++ exception (std::bad_alloc from a host vector
// sized by the caller's arguments, a std::length_error, ...) unwinds into a
// C, Rust or Python caller; it becomes BPP_ERR_NOMEM / BPP_ERR_DEVICE with
// the text in bpp_ctx_last_error when the entry point has a context.
template <class F>
inline int bpp_guard(bpp_ctx* ctx, F&& body) noexcept {
  try {
    return body();
  } catch (const std::bad_alloc&) {
    bpp_guard_note(ctx, "out of host memory");
    return BPP_ERR_NOMEM;
  } catch (const std::exception& e) {
    bpp_guard_note(ctx, e.what());
  } catch (...) {
    bpp_guard_note(ctx, "unexpected C++ exception");
  }
  return BPP_ERR_DEVICE;
}

// Scratch buffer that grows on demand (never shrinks until ctx destroy).
int ctx_ws(bpp_ctx* ctx, const char* name, size_t bytes, void** out);
int ctx_pinned(bpp_ctx* ctx, size_t bytes, void** out);
// A named pinned host buffer of at least `bytes` that kernels on this
// context access in place (zero copy: no copy launch, and its values are
// visible to the host once ctx_sync returns / to kernels launched after the
// host writes them).  Grows on demand; freed by bpp_ctx_destroy.
int ctx_host_buf(bpp_ctx* ctx, const char* name, size_t bytes, void** out);
// Zero-copy exchange through such buffers, no copy launch: ctx_zc_in copies
// `bytes` of host data into buffer `name` for kernels to read in place;
// ctx_zc_out hands out buffer `name` for kernels to write, its contents valid
// after the next ctx_sync.  A buffer handed out since the last ctx_sync is
// waited for (ctx_sync) before it is handed out again.
int ctx_zc_in(bpp_ctx* ctx, const char* name, const void* h, size_t bytes, uint32_t** d);
int ctx_zc_out(bpp_ctx* ctx, const char* name, size_t bytes, uint32_t** d);
// Host->device copy staged through the ctx's pinned arena (pageable
// hipMemcpyAsync measured up to ~25 ms on a 20 KB copy on the box); the host
// buffer may be freed as soon as this returns.
int ctx_h2d(bpp_ctx* ctx, void* d, const void* h, size_t bytes);
// memcpy into / out of the pinned arena, split over the host pool above 512 KB
void ctx_stage_copy(void* dst, const void* src, size_t bytes);
// bpp_host_alloc's pinned buffers (ctx.hip): is [p, p + n) inside one?
void host_pinned_add(const void* p, size_t n);
void host_pinned_remove(const void* p);
bool host_is_pinned(const void* p, size_t n);
// Two host buffers copied back to back into d (one staging copy).
int ctx_h2d2(bpp_ctx* ctx, void* d, const void* h0, size_t n0, const void* h1, size_t n1);
// Two-step form for data produced straight into the pinned arena:
// ctx_h2d_stage hands out `bytes` of staging (valid until the next
// ctx_sync), ctx_h2d_staged enqueues its copy to d.
int ctx_h2d_stage(bpp_ctx* ctx, size_t bytes, uint8_t** p);
// Records [p, p + bytes) of the pinned arena as holding secrets (prove_wipe
// zeroes the recorded spans).  Overlapping or touching spans are merged: the
// arena is reused from offset 0 after every ctx_sync, so batches that are
// never wiped (the u64-seed entry points) leave one span per distinct
// region, not one per call.
void ctx_secret_span(bpp_ctx* ctx, uint8_t* p, size_t bytes);
int ctx_h2d_staged(bpp_ctx* ctx, void* d, const uint8_t* p, size_t bytes);
// ctx_h2d that skips the copy when workspace `name` (at d) already holds
// exactly these bytes: for arrays that repeat batch after batch (circuit
// CSR, generator indices).  Only for workspaces no kernel writes.
int ctx_h2d_const(bpp_ctx* ctx, const char* name, void* d, const void* h, size_t bytes);
// Device->host copy through the arena; synchronous (stream synchronised).
int ctx_d2h(bpp_ctx* ctx, void* h, const void* d, size_t bytes);
// Wait for ctx's stream (event poll with short sleeps, see ctx.hip) +
// recycle the upload arena.
int ctx_sync(bpp_ctx* ctx);
// ctx_sync for a latency-bound single call (a lone MSM, a batch
// verification's two round trips): polls the event without sleeping for up to
// spin_us first (a 5 us nanosleep sleeps ~55 us under the default timer
// slack, and these calls wait on the GPU twice or three times per result).
int ctx_sync_latency(bpp_ctx* ctx, unsigned spin_us = 400);
// Scoped latency mode: ctx_sync on ctx spins `us` before sleeping while the
// guard lives (a 5-us nanosleep oversleeps by the 50-us default timer slack,
// which a chain of short kernels and host steps pays at every sync).
// The completion flag of the next launch (latency paths): *ticket (device,
// zero between launches) and *word (coherent pinned host memory) for a
// kernel that ends with done_signal(ticket, word, *tag); ctx_wait_flag then
// waits for it -- ~6 us of a kernel -> host round trip where an event record
// and query took ~12.5 (tools/ubench/flagpoll).
int ctx_done_flag(bpp_ctx* ctx, uint32_t** ticket, uint32_t** word, uint32_t* tag);
// Waits for *word == tag: spins up to the context's sync_spin_us, then falls
// back to ctx_sync (which reports a failed launch) and resets the ticket if
// the flag never came (a launch cut short), so the flag is only ever a
// shortcut.  Clears nothing ctx_sync would (zc_live, the stage arena).
int ctx_wait_flag(bpp_ctx* ctx, const uint32_t* word, uint32_t tag);

struct SyncSpin {
  bpp_ctx* c;
  unsigned old;
  SyncSpin(bpp_ctx* ctx, unsigned us) : c(ctx), old(ctx->sync_spin_us) { ctx->sync_spin_us = us; }
  ~SyncSpin() { c->sync_spin_us = old; }
  SyncSpin(const SyncSpin&) = delete;
  SyncSpin& operator=(const SyncSpin&) = delete;
};
// i-th child context of ctx (created on first use, destroyed with ctx).
int ctx_child(bpp_ctx* ctx, size_t i, bpp_ctx** out);

// Profiling brackets around a launch on ctx->stream.
struct ProfScope {
  bpp_ctx* ctx;
  const char* name;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(bpp_ctx* c, const char* n);
  ~ProfScope();
};

// Wall-clock bracket around a host phase (includes any GPU work it waits
// for); accumulated under `name` when profiling is on.
struct HostScope {
  bpp_ctx* ctx;
  const char* name;
  std::chrono::steady_clock::time_point t0;
  HostScope(bpp_ctx* c, const char* n) : ctx(c), name(n) {
    if (ctx->prof) t0 = std::chrono::steady_clock::now();
  }
  ~HostScope() {
    if (!ctx->prof) return;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    auto& acc = ctx->prof_acc[name];
    acc.first += ms;
    acc.second += 1;
  }
};

int ctx_check_launch(bpp_ctx* ctx, const char* what);
// Adds to a work counter (see bpp_ctx::work).
inline void ctx_work(bpp_ctx* ctx, const char* name, uint64_t n) { ctx->work[name] += n; }

// scan.hip
int scan_exclusive_u32(bpp_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, size_t n);
