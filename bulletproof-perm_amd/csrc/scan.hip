// Exclusive prefix sum over uint32 (bucket histogram -> bucket offsets).
// Reduce-then-scan in two launches: k_scan_reduce sums each tile of
// SCAN_TILE elements; k_scan_apply recomputes the exclusive prefix of the
// tile sums in every block (a few hundred values: one strided pass and a
// block reduction) and scans its own tile.  The previous three-phase form
// (1024-element tiles, recursive scan of the tile sums, uniform add) took
// five launches at 2^20 x 16 windows of counts.
#include "ctx.h"

#define SCAN_T 256
#define SCAN_PER 32
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

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// block-wide sum (every thread gets it); ws holds SCAN_T / 64 words
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* ws) {
  v = wave_sum(v);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) ws[wid] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < SCAN_T / 64; ++w) t += ws[w];
  return t;
}

__global__ void __launch_bounds__(SCAN_T) k_scan_reduce(const uint32_t* __restrict__ in, uint32_t* __restrict__ sums,
                                                       size_t n) {
  __shared__ uint32_t ws[SCAN_T / 64];
  const size_t base = (size_t)blockIdx.x * SCAN_TILE;
  uint32_t t = 0;
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    const size_t j = base + (size_t)i * SCAN_T + threadIdx.x;  // coalesced
    t += j < n ? in[j] : 0u;
  }
  t = block_sum(t, ws);
  if (threadIdx.x == 0) sums[blockIdx.x] = t;
}

__global__ void __launch_bounds__(SCAN_T) k_scan_apply(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      const uint32_t* __restrict__ sums, size_t n) {
  __shared__ uint32_t ws[SCAN_T / 64];
  __shared__ uint32_t wsum[SCAN_T / 64];
  // exclusive prefix of the tile sums before this tile
  uint32_t pre = 0;
  for (uint32_t k = threadIdx.x; k < blockIdx.x; k += SCAN_T) pre += sums[k];
  pre = block_sum(pre, ws);
  // this tile: thread-contiguous runs of SCAN_PER elements
  const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_PER;
  uint32_t v[SCAN_PER];
  uint32_t tot = 0;
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    v[i] = (base + i < n) ? in[base + i] : 0u;
    tot += v[i];
  }
  const uint32_t incl = wave_incl_scan(tot);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  uint32_t woff = 0;
  for (int w = 0; w < wid; ++w) woff += wsum[w];
  uint32_t run = pre + woff + incl - tot;
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
}

int scan_exclusive_u32(bpp_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, size_t n) {
  if (!n) return BPP_OK;
  const size_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  void* sums = nullptr;
  BPP_TRY(ctx_ws(ctx, "scan_sums", tiles * sizeof(uint32_t), &sums));
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)tiles), dim3(SCAN_T), 0, ctx->stream, d_in, (uint32_t*)sums, n);
  BPP_TRY(ctx_check_launch(ctx, "k_scan_reduce"));
  hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)tiles), dim3(SCAN_T), 0, ctx->stream, d_in, d_out,
                     (const uint32_t*)sums, n);
  return ctx_check_launch(ctx, "k_scan_apply");
}
