// Integer / fp64 instruction-throughput microbenchmark for gfx950 (inline asm,
// 8 independent chains per lane). Decides the limb representation of the
// curve25519 field multiply.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 2048
#define CH 8

__global__ void k_mad64(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 7 + seed + threadIdx.x;
  uint64_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c)
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x * 7 + seed + threadIdx.x;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x * 7 + seed + threadIdx.x;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_u24(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x * 7 + seed + threadIdx.x;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc[c]) : "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_hi24(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x * 7 + seed + threadIdx.x;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(uint64_t* out, uint32_t seed) {
  double b = 1.0000001 + seed * 1e-9;
  double acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x * 1e-3;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(acc[c]) : "v"(b));
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_add32(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x * 7 + seed + threadIdx.x;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x * 7 + seed + threadIdx.x;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[c]) : "v"(b) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add64(uint64_t* out, uint32_t seed) {
  uint64_t b = blockIdx.x * 7 + seed + threadIdx.x;
  uint64_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static double run(kfn k, uint64_t* d, int blocks, int threads) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double waveinstr = 5.0 * blocks * (threads / 64) * (double)ITERS * CH;
  // cycles per wave-instruction per SIMD at 2.4GHz: SIMDs*clk*time / instr
  double cyc = 1024.0 * 2.4e9 * (ms * 1e-3) / waveinstr;
  return cyc;
}

int main() {
  int blocks = 256 * 16, threads = 256;
  uint64_t* d; hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  printf("cycles per wave64 instruction per SIMD (assuming 2.4 GHz; full-rate = 2)\n");
  for (int rep = 0; rep < 2; ++rep) {
  printf("v_add_u32       : %.2f\n", run(k_add32, d, blocks, threads));
  printf("v_addc_co_u32   : %.2f\n", run(k_addc, d, blocks, threads));
  printf("v_lshl_add_u64  : %.2f\n", run(k_add64, d, blocks, threads));
  printf("v_mad_u64_u32   : %.2f\n", run(k_mad64, d, blocks, threads));
  printf("v_mul_lo_u32    : %.2f\n", run(k_mullo, d, blocks, threads));
  printf("v_mul_hi_u32    : %.2f\n", run(k_mulhi, d, blocks, threads));
  printf("v_mad_u32_u24   : %.2f\n", run(k_u24, d, blocks, threads));
  printf("v_mul_hi_u32_u24: %.2f\n", run(k_hi24, d, blocks, threads));
  printf("v_fma_f64       : %.2f\n", run(k_fma64, d, blocks, threads));
  }
  return 0;
}
