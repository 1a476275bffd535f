// Scalar Montgomery multiply: radix-2^29 sc_mont vs the 8 x 32-bit CIOS
// sc_mont_cios (sc25519.cuh).  Checks equality on random inputs (canonical,
// and a < 2^256 against canonical b -- the precondition's edge), then
// measures the latency of a dependent chain on one wave and the throughput
// of a full grid.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench/scbench.hip -o /tmp/scbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../bulletproof-perm_amd/csrc/sc25519.cuh"

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

__global__ void k_check(const uint32_t* a, const uint32_t* b, uint32_t n, uint32_t* bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const sc x = sc_load(a + 8 * i), y = sc_load(b + 8 * i);
  const sc r1 = sc_mont(x, y), r2 = sc_mont_cios(x, y);
  bool eq = true;
  for (int k = 0; k < 8; ++k) eq &= r1.v[k] == r2.v[k];
  if (!eq) atomicAdd(bad, 1u);
}

template <int NEW>
__global__ void k_chain(uint32_t* io, const uint32_t* yv, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  sc x = sc_load(io + 8 * i), y = sc_load(yv + 8 * i);
  for (uint32_t t = 0; t < iters; ++t) x = NEW ? sc_mont(x, y) : sc_mont_cios(x, y);
  sc_store(io + 8 * i, x);
}

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint32_t r32() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)rng;
}
static const uint32_t L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0, 0, 0, 0x10000000u};
static void rand_canon(uint32_t* w) {  // < 2^252 < l
  for (int k = 0; k < 8; ++k) w[k] = r32();
  w[7] &= 0x0fffffffu;
}

template <int NEW>
static float time_chain(uint32_t* d, const uint32_t* y, uint32_t blocks, uint32_t threads, uint32_t iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_chain<NEW>, dim3(blocks), dim3(threads), 0, 0, d, y, iters);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_chain<NEW>, dim3(blocks), dim3(threads), 0, 0, d, y, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

int main() {
  const uint32_t n = 1 << 20;
  uint32_t* ha = (uint32_t*)malloc(32ull * n);
  uint32_t* hb = (uint32_t*)malloc(32ull * n);
  for (uint32_t i = 0; i < n; ++i) {
    rand_canon(hb + 8 * i);
    if (i % 4 == 0) {  // a anywhere below 2^256
      for (int k = 0; k < 8; ++k) ha[8 * i + k] = r32();
    } else if (i % 4 == 1) {  // a = l - 1 - small, b near l
      for (int k = 0; k < 8; ++k) ha[8 * i + k] = L[k];
      ha[8 * i] -= 1 + (r32() & 0xff);
      for (int k = 0; k < 8; ++k) hb[8 * i + k] = L[k];
      hb[8 * i] -= 1 + (r32() & 0xff);
    } else if (i % 4 == 2) {  // a = 2^256 - 1
      for (int k = 0; k < 8; ++k) ha[8 * i + k] = 0xffffffffu;
    } else {
      rand_canon(ha + 8 * i);
    }
  }
  uint32_t *da, *db, *dbad;
  CHECK(hipMalloc(&da, 32ull * n));
  CHECK(hipMalloc(&db, 32ull * n));
  CHECK(hipMalloc(&dbad, 4));
  CHECK(hipMemcpy(da, ha, 32ull * n, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, hb, 32ull * n, hipMemcpyHostToDevice));
  CHECK(hipMemset(dbad, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, da, db, n, dbad);
  uint32_t bad = 0;
  CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  printf("mismatches: %u of %u\n", bad, n);
  // latency: one wave, a dependent chain
  const uint32_t it = 2000;
  const float l_new = time_chain<1>(da, db, 1, 64, it), l_old = time_chain<0>(da, db, 1, 64, it);
  printf("lone wave: radix-29 %.0f ns, cios %.0f ns per multiply\n", l_new * 1e6 / it, l_old * 1e6 / it);
  // throughput: 4096 blocks x 256 lanes
  const uint32_t itt = 200, nb = 4096;
  const float t_new = time_chain<1>(da, db, nb, 256, itt), t_old = time_chain<0>(da, db, nb, 256, itt);
  const double ops = (double)nb * 256 * itt;
  printf("full grid: radix-29 %.2f, cios %.2f G multiplies/s\n", ops / (t_new * 1e6), ops / (t_old * 1e6));
  return bad ? 1 : 0;
}
