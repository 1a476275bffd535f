// Kernel -> host completion latency, one small kernel per round trip on one
// stream: (a) hipEventRecord + hipEventQuery spin (ctx_sync_latency), (b) the
// kernel's last write a flag word in pinned host memory after a system-scope
// release fence, the host spinning on the word, (c) (b) plus the event, as a
// drop-in would keep it for the error path.  Is the event round trip what
// the IPA rounds' ~27 us host gaps are made of?
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/flagpoll.cpp -o tools/ubench/flagpoll
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>

__global__ void k_work(uint32_t* out, volatile uint32_t* flag, uint32_t v, int use_flag) {
  out[blockIdx.x * 64 + threadIdx.x] = v + threadIdx.x;
  if (use_flag) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence_system();
      __hip_atomic_store((uint32_t*)flag + blockIdx.x, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  uint32_t *out, *flag;
  hipHostMalloc((void**)&out, 64 * 64 * 4, hipHostMallocDefault);
  hipHostMalloc((void**)&flag, 64 * 4, hipHostMallocCoherent);
  for (int i = 0; i < 64; ++i) flag[i] = 0;
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  const char* names[3] = {"event spin", "flag spin", "flag spin + event record"};
  for (int blocks : {1, 64})
    for (int mode = 0; mode < 3; ++mode) {
      uint32_t v = 1000000u * (mode + 1) + 100000u * blocks;
      const int N = 3000;
      long bad = 0;
      const auto t0 = std::chrono::steady_clock::now();
      for (int it = 0; it < N; ++it) {
        ++v;
        hipLaunchKernelGGL(k_work, dim3(blocks), dim3(64), 0, s, out, flag, v, mode != 0);
        if (mode != 1) hipEventRecord(ev, s);
        if (mode == 0) {
          while (hipEventQuery(ev) == hipErrorNotReady) {
          }
        } else {
          const auto ts = std::chrono::steady_clock::now();
          for (int b = 0; b < blocks; ++b)
            while (__atomic_load_n(flag + b, __ATOMIC_ACQUIRE) != v) {
              if (std::chrono::steady_clock::now() - ts > std::chrono::milliseconds(200)) {
                ++bad;
                break;
              }
            }
        }
        if (out[(blocks - 1) * 64 + 5] != v + 5) ++bad;
      }
      hipStreamSynchronize(s);
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
      printf("%-26s blocks %2d: %6.2f us per round trip, bad %ld\n", names[mode], blocks, us, bad);
    }
  return 0;
}
