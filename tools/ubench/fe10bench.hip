// Prototype: radix-2^25.5 (10 x 32-bit limbs) field multiply built only from
// v_mad_u64_u32 column chains (tools/gen_fe10.py) vs the current 8-limb
// Comba (fe25519.cuh).  Checks equality on random inputs, then measures
// throughput and single-wave latency like tools/ubench/felat.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "fe8_ref.cuh"

namespace f10 {
struct fe {
  uint32_t v[10];
};
#define MAD64(a, b, c) ((uint64_t)(uint32_t)(a) * (uint64_t)(uint32_t)(b) + (uint64_t)(c))
#ifdef PLAIN
#define MADC(a, b, c) MAD64(a, b, c)
#else
FE_INLINE uint64_t fe_madc(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t d, unused;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(unused) : "v"(a), "v"(b), "v"(c));
  return d;
}
#define MADC(a, b, c) fe_madc((a), (b), (c))
#endif
#include "../../bulletproof-perm_amd/csrc/fe10_ops.inc"
__device__ __constant__ const int OFF[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
FE_INLINE fe from_words(const ::fe& a) {  // loose 8x32 (< 2^256) -> 10 limbs
  fe r;
  const uint32_t top = a.v[7] >> 31;  // bit 255 -> 19
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int o = OFF[i], w = (i & 1) ? 25 : 26;
    const int q = o >> 5, s = o & 31;
    uint64_t x = a.v[q];
    if (q + 1 < 8) x |= (uint64_t)a.v[q + 1] << 32;
    uint32_t limb = (uint32_t)(x >> s) & ((1u << w) - 1);
    if (i == 9) limb &= (1u << 25) - 1;
    r.v[i] = limb;
  }
  r.v[0] += 19u * top;
  return r;
}
FE_INLINE ::fe to_words(fe a) {  // full carry, then pack (< 2^256, loose)
  for (int rep = 0; rep < 2; ++rep) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int w = (i & 1) ? 25 : 26;
      a.v[i] += c;
      c = a.v[i] >> w;
      a.v[i] &= (1u << w) - 1;
    }
    a.v[0] += 19u * c;
  }
  ::fe r = fe_zero();
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int o = OFF[i], q = o >> 5, s = o & 31;
    const uint64_t x = (uint64_t)a.v[i] << s;
    r.v[q] |= (uint32_t)x;
    if (q + 1 < 8) r.v[q + 1] |= (uint32_t)(x >> 32);
  }
  return r;
}
}  // namespace f10

#define ITERS 4096

__global__ void k_check(const uint32_t* in, uint32_t* bad, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  ::fe a, b;
  for (int i = 0; i < 8; ++i) {
    a.v[i] = in[16 * t + i];
    b.v[i] = in[16 * t + 8 + i];
  }
  const f10::fe A = f10::from_words(a), B = f10::from_words(b);
  const ::fe m1 = fe_canon(fe_mul(a, b)), m2 = fe_canon(f10::to_words(f10::fe_mul(A, B)));
  const ::fe s1 = fe_canon(fe_sq(a)), s2 = fe_canon(f10::to_words(f10::fe_sq(A)));
  // chains: 20 squarings / multiplications
  ::fe c1 = a;
  f10::fe C2 = A;
  for (int i = 0; i < 20; ++i) {
    c1 = fe_mul(fe_sq(c1), b);
    C2 = f10::fe_mul(f10::fe_sq(C2), B);
  }
  const ::fe d1 = fe_canon(c1), d2 = fe_canon(f10::to_words(C2));
  for (int i = 0; i < 8; ++i)
    if (m1.v[i] != m2.v[i] || s1.v[i] != s2.v[i] || d1.v[i] != d2.v[i]) atomicAdd(bad, 1u);
}

__global__ void __launch_bounds__(64) k_mul8(uint32_t* out, uint32_t seed) {
  ::fe x, y;
  for (int i = 0; i < 8; ++i) {
    x.v[i] = seed * (i + 1) + threadIdx.x + blockIdx.x;
    y.v[i] = seed * (i + 3) + 7 * threadIdx.x;
  }
  for (int i = 0; i < ITERS; ++i) x = fe_mul(x, y);
  for (int i = 0; i < 8; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 10 + i] = x.v[i];
}
__global__ void __launch_bounds__(64) k_mul10(uint32_t* out, uint32_t seed) {
  f10::fe x, y;
  for (int i = 0; i < 10; ++i) {
    x.v[i] = (seed * (i + 1) + threadIdx.x + blockIdx.x) & 0x1ffffff;
    y.v[i] = (seed * (i + 3) + 7 * threadIdx.x) & 0x1ffffff;
  }
  for (int i = 0; i < ITERS; ++i) x = f10::fe_mul(x, y);
  for (int i = 0; i < 10; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 10 + i] = x.v[i];
}
__global__ void __launch_bounds__(64) k_sq8(uint32_t* out, uint32_t seed) {
  ::fe x;
  for (int i = 0; i < 8; ++i) x.v[i] = seed * (i + 1) + threadIdx.x + blockIdx.x;
  for (int i = 0; i < ITERS; ++i) x = fe_sq(x);
  for (int i = 0; i < 8; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 10 + i] = x.v[i];
}
__global__ void __launch_bounds__(64) k_sq10(uint32_t* out, uint32_t seed) {
  f10::fe x;
  for (int i = 0; i < 10; ++i) x.v[i] = (seed * (i + 1) + threadIdx.x + blockIdx.x) & 0x1ffffff;
  for (int i = 0; i < ITERS; ++i) x = f10::fe_sq(x);
  for (int i = 0; i < 10; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 10 + i] = x.v[i];
}

template <class K>
static void run(const char* name, K k, int blocks) {
  uint32_t* d;
  if (hipMalloc(&d, (size_t)blocks * 64 * 40)) exit(1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, 1u);
  if (hipDeviceSynchronize()) exit(1);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, 3u);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double per = ms * 1e6 / ITERS;
  printf("%-6s blocks=%6d  chain step %7.1f ns (%5.0f cyc)  throughput %7.2f Gop/s\n", name, blocks, per, per * 2.4,
         (double)blocks * 64 * ITERS / (ms * 1e6));
  (void)hipFree(d);
}

int main() {
  const int n = 1 << 20;
  uint32_t *in, *bad;
  uint32_t* h = (uint32_t*)malloc((size_t)n * 64);
  srand(7);
  for (size_t i = 0; i < (size_t)n * 16; ++i) h[i] = (uint32_t)rand() * 2654435761u ^ (uint32_t)rand();
  for (int t = 0; t < n; ++t)  // include edge values: all-ones words (>= p, loose)
    if (t % 97 == 0)
      for (int i = 0; i < 16; ++i) h[16 * t + i] = 0xffffffffu;
  if (hipMalloc(&in, (size_t)n * 64) || hipMalloc(&bad, 4)) return 1;
  (void)hipMemcpy(in, h, (size_t)n * 64, hipMemcpyHostToDevice);
  (void)hipMemset(bad, 0, 4);
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, in, bad, n);
  uint32_t nb = 0;
  (void)hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
  printf("mismatches: %u of %d (mul, sq, 20-step chains)\n", nb, n);
  for (int blocks : {1, 1024, 4096, 16384}) {
    run("mul8", k_mul8, blocks);
    run("mul10", k_mul10, blocks);
    run("sq8", k_sq8, blocks);
    run("sq10", k_sq10, blocks);
  }
  return nb ? 2 : 0;
}
