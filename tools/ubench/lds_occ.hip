// How many 256-lane workgroups with a given static LDS size one CU holds at
// once (k_msm_accumulate: 40960 B of LDS per workgroup, 4 x 40960 = 160 KiB
// exactly).  Every workgroup spins ~SPIN cycles; NWG workgroups then take
// ceil(NWG / (256 CUs x resident)) rounds, so the kernel time gives the
// number resident per CU.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/lds_occ.hip -o /tmp/lds_occ && /tmp/lds_occ
#include <hip/hip_runtime.h>

#include <cstdio>

#define SPIN 200000ull

template <int LDS>
__global__ void __launch_bounds__(256) k_occ(uint32_t* sink) {
  __shared__ uint32_t buf[LDS / 4];
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = clock64();
  uint32_t a = buf[(threadIdx.x + 1) & 255];
  while (clock64() - t0 < SPIN) a = a * 1664525u + 1013904223u;
  if (a == 0x12345678u) sink[blockIdx.x] = a + buf[threadIdx.x ^ 1];
}

template <int LDS>
static void run(int nwg, int ncu) {
  uint32_t* s;
  hipMalloc(&s, 4 * nwg);
  hipLaunchKernelGGL(k_occ<LDS>, dim3(nwg), dim3(256), 0, 0, s);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9f;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_occ<LDS>, dim3(nwg), dim3(256), 0, 0, s);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  hipLaunchKernelGGL(k_occ<LDS>, dim3(1), dim3(256), 0, 0, s);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_occ<LDS>, dim3(1), dim3(256), 0, 0, s);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float one;
  hipEventElapsedTime(&one, e0, e1);
  printf("LDS %6d B/WG: %5d WGs in %.3f ms, one WG %.3f ms -> %.2f rounds -> ~%.2f WGs per CU resident\n", LDS, nwg,
         best, one, best / one, (double)nwg / ncu / (best / one));
  hipFree(s);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs: %d\n", ncu);
  const int nwg = ncu * 12;
  run<32768>(nwg, ncu);
  run<40704>(nwg, ncu);
  run<40960>(nwg, ncu);
  run<41216>(nwg, ncu);
  run<53248>(nwg, ncu);
  return 0;
}
