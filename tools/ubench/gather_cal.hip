// FETCH_SIZE calibration for the MSM accumulate access pattern on gfx950
// (MI355X_MICROARCH.md: FETCH_SIZE is exact only up to a factor for wide
// streaming reads; other patterns must be calibrated on a known byte count).
//   k_stream   : 16 B per lane, fully coalesced, known bytes
//   k_gather96 : random 96-byte rows (6 x 16 B loads per lane, the layout of
//                an affine-Niels table entry) from a 100 MB table, like
//                k_msm_accumulate's point fetches
// Run under rocprofv3 --pmc FETCH_SIZE; tools/pmc_summary.py reads the
// per-kernel values and prints raw KB vs known bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_stream(const uint4* __restrict__ in, size_t n, uint4* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t j = i; j < n; j += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = in[j];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[i] = acc;
}

__global__ void k_gather96(const uint4* __restrict__ tbl, uint32_t nrows, uint32_t per_lane, uint4* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t h = i * 2654435761u + 12345u;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint32_t k = 0; k < per_lane; ++k) {
    h ^= h << 13; h ^= h >> 17; h ^= h << 5;
    const uint4* row = tbl + (size_t)(h % nrows) * 6;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const uint4 v = row[q];
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[i] = acc;
}

int main() {
  const uint32_t nrows = 1u << 20;  // 100 MB of 96-byte rows (the 2^20 MSM table)
  const size_t tbl_bytes = (size_t)nrows * 96;
  const size_t stream_bytes = 256ull << 20;
  uint4 *tbl, *big, *out;
  if (hipMalloc(&tbl, tbl_bytes) || hipMalloc(&big, stream_bytes) || hipMalloc(&out, 64 << 20)) return 1;
  if (hipMemset(tbl, 1, tbl_bytes) || hipMemset(big, 2, stream_bytes)) return 1;
  hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)big, stream_bytes / 16, out);
  const uint32_t lanes = 1u << 20, per_lane = 16;  // 16.8M row reads = the 2^20 x 16-window MSM
  hipLaunchKernelGGL(k_gather96, dim3(lanes / 256), dim3(256), 0, 0, (const uint4*)tbl, nrows, per_lane, out);
  if (hipDeviceSynchronize()) return 1;
  printf("k_stream known bytes %zu\n", stream_bytes);
  printf("k_gather96 rows %llu x 96 B = %llu bytes (table %zu bytes)\n", (unsigned long long)lanes * per_lane,
         (unsigned long long)lanes * per_lane * 96ull, tbl_bytes);
  return 0;
}
