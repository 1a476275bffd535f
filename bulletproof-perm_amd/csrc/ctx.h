// Internal context / workspace / error plumbing shared by the HIP sources.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
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
  // profiling
  bool prof = false;
  struct Pend {
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<Pend> pending;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, std::pair<double, uint64_t>> prof_acc;
};

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

// Scratch buffer that grows on demand (never shrinks until ctx destroy).
int ctx_ws(bpp_ctx* ctx, const char* name, size_t bytes, void** out);
int ctx_pinned(bpp_ctx* ctx, size_t bytes, void** out);

// Profiling brackets around a launch on ctx->stream.
struct ProfScope {
  bpp_ctx* ctx;
  const char* name;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(bpp_ctx* c, const char* n);
  ~ProfScope();
};

int ctx_check_launch(bpp_ctx* ctx, const char* what);

// scan.hip
int scan_exclusive_u32(bpp_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, size_t n);
