// Exclusive prefix sum over uint32 (bucket histogram -> bucket offsets).
// Three-phase: per-block wave-shuffle scan (1024 elements / 256 lanes),
// recursive scan of block totals, uniform add.
#include "ctx.h"

#define SCAN_T 256
#define SCAN_PER 4
#define SCAN_TILE (SCAN_T * SCAN_PER)

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}

__global__ void __launch_bounds__(SCAN_T) k_scan_tile(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                     uint32_t* __restrict__ sums, size_t n) {
  __shared__ uint32_t wsum[SCAN_T / 64];
  const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_PER;
  uint32_t v[SCAN_PER];
  uint32_t tot = 0;
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    v[i] = (base + i < n) ? in[base + i] : 0u;
    tot += v[i];
  }
  uint32_t incl = wave_incl_scan(tot);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  uint32_t woff = 0;
  for (int w = 0; w < wid; ++w) woff += wsum[w];
  uint32_t run = woff + incl - tot;
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (threadIdx.x == SCAN_T - 1 && sums) sums[blockIdx.x] = run;
}

__global__ void k_scan_add(uint32_t* __restrict__ out, const uint32_t* __restrict__ sums, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += sums[i / SCAN_TILE];
}

static int scan_level(bpp_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, size_t n, int depth) {
  const size_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (tiles <= 1) {
    hipLaunchKernelGGL(k_scan_tile, dim3(1), dim3(SCAN_T), 0, ctx->stream, d_in, d_out, (uint32_t*)nullptr, n);
    return ctx_check_launch(ctx, "k_scan_tile");
  }
  void* sums = nullptr;
  void* sums_sc = nullptr;
  char nm[32];
  snprintf(nm, sizeof nm, "scan_sums%d", depth);
  BPP_TRY(ctx_ws(ctx, nm, tiles * sizeof(uint32_t), &sums));
  snprintf(nm, sizeof nm, "scan_sc%d", depth);
  BPP_TRY(ctx_ws(ctx, nm, tiles * sizeof(uint32_t), &sums_sc));
  hipLaunchKernelGGL(k_scan_tile, dim3((unsigned)tiles), dim3(SCAN_T), 0, ctx->stream, d_in, d_out, (uint32_t*)sums, n);
  BPP_TRY(ctx_check_launch(ctx, "k_scan_tile"));
  BPP_TRY(scan_level(ctx, (const uint32_t*)sums, (uint32_t*)sums_sc, tiles, depth + 1));
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, d_out,
                     (const uint32_t*)sums_sc, n);
  return ctx_check_launch(ctx, "k_scan_add");
}

int scan_exclusive_u32(bpp_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, size_t n) {
  return scan_level(ctx, d_in, d_out, n, 0);
}
