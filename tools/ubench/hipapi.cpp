// HIP runtime round trips from T host threads, each on its own stream:
// per iteration one small kernel, one 4 KB host<-device copy into pinned
// memory and a wait (event polled with 5 us sleeps, as ctx_sync).  Does the
// runtime serialise independent streams' round trips?  The prover runs ~20
// such round trips per batch on each of 8-12 streams.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/hipapi.cpp -o tools/ubench/hipapi
#include <hip/hip_runtime.h>

#include <sched.h>
#include <sys/prctl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void k_touch(uint32_t* p, uint32_t v) { p[threadIdx.x] = v + threadIdx.x; }

int main() {
  const char* names[4] = {"hipStreamSynchronize", "poll + 5 us sleep", "poll + sched_yield", "poll + 5 us sleep, timer slack 1 us"};
  for (int mode = 0; mode < 4; ++mode)
  for (int T : {1, 8, 16}) {
    std::vector<std::thread> th;
    std::atomic<long> total{0};
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < T; ++t)
      th.emplace_back([&] {
        hipStream_t s;
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        uint32_t *d, *h;
        hipMalloc(&d, 4096);
        hipHostMalloc((void**)&h, 4096);
        if (mode == 3) prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
        hipEvent_t ev;
        hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        long n = 0;
        while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(800)) {
          hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, d, (uint32_t)n);
          hipMemcpyAsync(h, d, 4096, hipMemcpyDeviceToHost, s);
          hipEventRecord(ev, s);
          if (mode == 0) {
            hipStreamSynchronize(s);
          } else {
            while (hipEventQuery(ev) == hipErrorNotReady) {
              if (mode == 2) sched_yield();
              else std::this_thread::sleep_for(std::chrono::microseconds(5));
            }
          }
          ++n;
        }
        total += n;
        hipEventDestroy(ev);
        hipHostFree(h);
        hipFree(d);
        hipStreamDestroy(s);
      });
    for (auto& x : th) x.join();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("%-36s threads %2d: %8.0f round trips/s total, %6.1f us per round trip per thread\n", names[mode], T, total / sec,
           1e6 * sec * T / total);
  }
  return 0;
}
