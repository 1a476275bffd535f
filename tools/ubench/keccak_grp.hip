// Latency of one Keccak-f[1600] permutation for the batch verifier's replay
// (one transcript chain per lane vs per 8-lane group, merlin_group.cuh), and
// the dependent-latency building blocks it is made of, for a lone wave per
// SIMD (the replay's regime).  s_memtime cycles per wave.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bulletproof-perm_amd/csrc \
//         tools/ubench/keccak_grp.hip -o /tmp/keccak_grp && /tmp/keccak_grp
#include <hip/hip_runtime.h>

#include <cstdio>

#include "merlin_group.cuh"

#define NPERM 64

__global__ void __launch_bounds__(64) k_lane(unsigned long long* cyc, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint64_t st[64 * 25];
  for (int i = 0; i < 25; ++i) st[threadIdx.x * 25 + i] = i * 0x9e3779b97f4a7c15ull + threadIdx.x;
  lds_u64* s = (lds_u64*)(st + threadIdx.x * 25);
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = clock64();
  for (int n = 0; n < NPERM; ++n) lane_keccak(s);
  const unsigned long long t1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = (uint32_t)s[0];
}

__global__ void __launch_bounds__(64) k_group(unsigned long long* cyc, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t sp[8 * GRP_BLOCK];
  const uint32_t g = threadIdx.x >> 3, gl = threadIdx.x & 7;
  uint8_t* st = sp + g * GRP_BLOCK;  // (merlin_group.cuh GRP_BLOCK / GRP_SCR_OFF)
  for (int i = gl; i < 25; i += 8) reinterpret_cast<uint64_t*>(st)[i] = i * 0x9e3779b97f4a7c15ull + g;
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = clock64();
  for (int n = 0; n < NPERM; ++n) grp_keccak((lds_u64*)st, (lds_u64*)(st + GRP_SCR_OFF), gl);
  const unsigned long long t1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = reinterpret_cast<uint32_t*>(st)[gl];
}

__global__ void __launch_bounds__(64) k_group16(unsigned long long* cyc, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t sp[4 * GRP_BLOCK];
  const uint32_t g = threadIdx.x >> 4, gl = threadIdx.x & 15;
  uint8_t* st = sp + g * GRP_BLOCK;
  for (int i = gl; i < 25; i += 16) reinterpret_cast<uint64_t*>(st)[i] = i * 0x9e3779b97f4a7c15ull + g;
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = clock64();
  for (int n = 0; n < NPERM; ++n) grp_keccak16((lds_u64*)st, (lds_u64*)(st + GRP_SCR_OFF), gl);
  const unsigned long long t1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = reinterpret_cast<uint32_t*>(st)[gl];
}

// the three permutations agree on the same inputs (8 states per block)
__global__ void __launch_bounds__(64) k_check(uint32_t* bad) {
  __shared__ __attribute__((aligned(16))) uint64_t ref[8 * 25];
  __shared__ __attribute__((aligned(16))) uint8_t s8[8 * GRP_BLOCK];
  __shared__ __attribute__((aligned(16))) uint8_t s16[4 * GRP_BLOCK];
  for (int i = threadIdx.x; i < 8 * 25; i += 64) ref[i] = (i % 25) * 0x9e3779b97f4a7c15ull + (i / 25) * 0x1234567ull;
  for (int i = threadIdx.x; i < 8 * 25; i += 64)
    reinterpret_cast<uint64_t*>(s8 + (i / 25) * GRP_BLOCK)[i % 25] = ref[i];
  for (int i = threadIdx.x; i < 4 * 25; i += 64)
    reinterpret_cast<uint64_t*>(s16 + (i / 25) * GRP_BLOCK)[i % 25] = ref[i];
  __syncthreads();
  if (threadIdx.x < 8) lane_keccak((lds_u64*)(ref + 25 * threadIdx.x));
  grp_keccak((lds_u64*)(s8 + (threadIdx.x >> 3) * GRP_BLOCK), (lds_u64*)(s8 + (threadIdx.x >> 3) * GRP_BLOCK + GRP_SCR_OFF),
             threadIdx.x & 7);
  grp_keccak16((lds_u64*)(s16 + (threadIdx.x >> 4) * GRP_BLOCK), (lds_u64*)(s16 + (threadIdx.x >> 4) * GRP_BLOCK + GRP_SCR_OFF),
               threadIdx.x & 15);
  __syncthreads();
  uint32_t nb = 0;
  for (int i = threadIdx.x; i < 8 * 25; i += 64) {
    nb += reinterpret_cast<uint64_t*>(s8 + (i / 25) * GRP_BLOCK)[i % 25] != ref[i];
    if (i < 4 * 25) nb += reinterpret_cast<uint64_t*>(s16 + (i / 25) * GRP_BLOCK)[i % 25] != ref[i];
  }
  atomicAdd(bad, nb);
}

// dependent VALU chain (v_xor) and dependent bitop3, DPP-fed chain, LDS round trip
__global__ void __launch_bounds__(64) k_lat(unsigned long long* cyc, uint32_t* sink) {
  __shared__ uint32_t l[64 * 16];
  uint32_t a = threadIdx.x, b = blockIdx.x + 7;
  unsigned long long t0 = clock64();
  for (int i = 0; i < 256; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
  unsigned long long t1 = clock64();
  cyc[blockIdx.x * 4 + 0] = t1 - t0;
  t0 = clock64();
  for (int i = 0; i < 256; ++i) a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(a ^ b), 0x101, 0xf, 0xf, false);
  t1 = clock64();
  cyc[blockIdx.x * 4 + 1] = t1 - t0;
  t0 = clock64();
  typedef __attribute__((address_space(3))) uint32_t lds32;
  lds32* L = (lds32*)l;
  for (int i = 0; i < 256; ++i) {
    L[threadIdx.x] = a;
    __asm__ volatile("" ::: "memory");
    a = L[(threadIdx.x + 1) & 63] ^ b;
    __asm__ volatile("" ::: "memory");
  }
  t1 = clock64();
  cyc[blockIdx.x * 4 + 2] = t1 - t0;
  t0 = clock64();
  for (int i = 0; i < 256; ++i) a = __builtin_amdgcn_alignbit(a, a ^ b, 31);
  t1 = clock64();
  cyc[blockIdx.x * 4 + 3] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = a;
}

// one wave-uniform scalar inversion (sc_inv_vartime, binary Euclid) as the
// replay runs it: on VGPRs (the value comes from a wave shuffle) or on SGPRs
// (readfirstlane: the compiler then runs the loop on the scalar unit)
template <bool SCALAR>
__global__ void __launch_bounds__(64) k_inv(unsigned long long* cyc, uint32_t* sink) {
  sc a;
  for (int i = 0; i < 8; ++i) a.v[i] = __shfl(0x9e3779b9u * (i + 1) + blockIdx.x, 5, 64);
  a.v[7] &= 0x0fffffffu;
  if (SCALAR)
    for (int i = 0; i < 8; ++i) a.v[i] = __builtin_amdgcn_readfirstlane(a.v[i]);
  const unsigned long long t0 = clock64();
  sc r = sc_inv_vartime(a);
  const unsigned long long t1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = r.v[threadIdx.x & 7];
}

// 64-byte challenge -> scalar (sc_from_wide_w), dependent chain of 16
__global__ void __launch_bounds__(64) k_wide(unsigned long long* cyc, uint32_t* sink) {
  uint32_t w[16];
  for (int i = 0; i < 16; ++i) w[i] = 0x85ebca6bu * (i + threadIdx.x + 1);
  const unsigned long long t0 = clock64();
  for (int n = 0; n < 16; ++n) {
    sc r = sc_from_wide_w(w);
    for (int i = 0; i < 8; ++i) w[i] ^= r.v[i];
  }
  const unsigned long long t1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = w[threadIdx.x & 15];
}

static void report(const char* name, void (*k)(unsigned long long*, uint32_t*), int blocks, double per) {
  unsigned long long* d;
  uint32_t* s;
  hipMalloc(&d, 8 * 4 * 2048);
  hipMalloc(&s, 4 * 64 * 2048);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, s);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, s);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[4];
  hipMemcpy(h, d, 8 * 4, hipMemcpyDeviceToHost);
  printf("%-28s blocks %4d: wave 0 %.1f cycles per unit, kernel %.3f us\n", name, blocks, h[0] / per, ms * 1e3);
  if (k == k_lat)
    printf("   xor chain %.1f  dpp+xor chain %.1f  lds write->read %.1f  alignbit chain %.1f cycles per step\n",
           h[0] / 256.0, h[1] / 256.0, h[2] / 256.0, h[3] / 256.0);
  hipFree(d);
  hipFree(s);
}

int main() {
  uint32_t* dbad;
  hipMalloc(&dbad, 4);
  hipMemset(dbad, 0, 4);
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, dbad);
  uint32_t hb = ~0u;
  hipMemcpy(&hb, dbad, 4, hipMemcpyDeviceToHost);
  printf("group permutations vs lane keccak: %u mismatching words\n", hb);
  for (int b : {1, 512}) {
    report("lane keccak (per perm)", k_lane, b, NPERM);
    report("group keccak (per perm)", k_group, b, NPERM);
    report("group16 keccak (per perm)", k_group16, b, NPERM);
  }
  report("latency", k_lat, 1, 1);
  report("sc_inv_vartime on VGPRs", k_inv<false>, 1, 1);
  report("sc_inv_vartime on SGPRs", k_inv<true>, 1, 1);
  report("sc_from_wide_w (per call)", k_wide, 1, 16);
  return 0;
}
