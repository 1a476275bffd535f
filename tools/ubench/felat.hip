// Field-multiply latency vs throughput on gfx950: a dependent chain of
// fe_sq / fe_mul per lane, launched with 1 wave, 1 wave per SIMD and 8 waves
// per SIMD.  Tells how latency-bound a one-lane-per-item kernel (point
// encoding, bucket reduction tails, fixed-base Pedersen) is.
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../../bulletproof-perm_amd/csrc/ge25519.cuh"

#define ITERS 4096

__global__ void __launch_bounds__(64) k_sq_chain(uint32_t* out, uint32_t seed) {
  fe x;
  for (int i = 0; i < FE_LIMBS; ++i) x.v[i] = (seed * (i + 1) + threadIdx.x + blockIdx.x) & FE_M25;
  for (int i = 0; i < ITERS; ++i) x = fe_sq(x);
  for (int i = 0; i < 8; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 8 + i] = x.v[i];
}

__global__ void __launch_bounds__(64) k_mul_chain(uint32_t* out, uint32_t seed) {
  fe x, y;
  for (int i = 0; i < FE_LIMBS; ++i) {
    x.v[i] = (seed * (i + 1) + threadIdx.x + blockIdx.x) & FE_M25;
    y.v[i] = (seed * (i + 3) + 7 * threadIdx.x) & FE_M25;
  }
  for (int i = 0; i < ITERS; ++i) x = fe_mul(x, y);
  for (int i = 0; i < 8; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 8 + i] = x.v[i];
}

// two independent chains per lane (ILP 2)
__global__ void __launch_bounds__(64) k_sq_chain2(uint32_t* out, uint32_t seed) {
  fe x, y;
  for (int i = 0; i < FE_LIMBS; ++i) {
    x.v[i] = (seed * (i + 1) + threadIdx.x + blockIdx.x) & FE_M25;
    y.v[i] = (seed * (i + 5) + threadIdx.x) & FE_M25;
  }
  for (int i = 0; i < ITERS; ++i) {
    x = fe_sq(x);
    y = fe_sq(y);
  }
  for (int i = 0; i < 8; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 8 + i] = x.v[i] ^ y.v[i];
}

// mixed additions (ge_madd: 7 field multiplies + the formula's additions and
// carries, exactly the MSM accumulate's per-entry arithmetic) on one
// dependent chain per lane, operand in registers: the ALU roofline of the
// bucket accumulation and the direct-table MSM
template <int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, 8))) k_madd_chain(uint32_t* out, uint32_t seed) {
  ge_p3 acc = ge_identity();
  ge_niels q;
  for (int i = 0; i < FE_LIMBS; ++i) {
    q.ypx.v[i] = (seed * (i + 1) + threadIdx.x + blockIdx.x) & FE_M25;
    q.ymx.v[i] = (seed * (i + 3) + 7 * threadIdx.x) & FE_M25;
    q.xy2d.v[i] = (seed * (i + 5) + threadIdx.x) & FE_M25;
  }
  for (int i = 0; i < ITERS / 8; ++i) acc = ge_madd(acc, q);
  for (int i = 0; i < 8; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 8 + i] = acc.X.v[i] ^ acc.T.v[i];
}

template <class K>
static void run(const char* name, K k, int blocks, int ops_per_iter) {
  uint32_t* d;
  hipMalloc(&d, (size_t)blocks * 64 * 32);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, 1u);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, 3u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const int iters = ops_per_iter < 0 ? ITERS / 8 : ITERS;
  if (ops_per_iter < 0) ops_per_iter = 1;
  const double per_op_ns = ms * 1e6 / iters;  // one lane's dependent op
  const double ops = (double)blocks * 64 * iters * ops_per_iter;
  printf("%-10s blocks=%6d  chain step %8.1f ns (%6.0f cyc @2.4GHz)  throughput %7.2f Gop/s\n", name, blocks,
         per_op_ns, per_op_ns * 2.4, ops / (ms * 1e6));
  hipFree(d);
}

int main() {
  for (int blocks : {1, 1024, 4096, 8192, 16384, 32768}) run("sq", k_sq_chain, blocks, 1);
  for (int blocks : {1, 1024, 4096, 8192, 16384, 32768, 65536, 131072, 262144}) run("mul", k_mul_chain, blocks, 1);
  for (int blocks : {1, 1024, 4096, 8192, 16384}) run("sq x2", k_sq_chain2, blocks, 2);
  // ops_per_iter -1: ITERS / 8 mixed additions per lane
  for (int blocks : {1, 1024, 4096, 8192, 16384, 32768, 65536}) run("madd w2", k_madd_chain<2>, blocks, -1);
  for (int blocks : {1, 1024, 4096, 8192, 16384, 32768, 65536}) run("madd w4", k_madd_chain<4>, blocks, -1);
  return 0;
}
