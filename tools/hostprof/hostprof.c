// Minimal in-process CPU sampling profiler for the host side of the prover
// (the GPU box has no perf / gdb): a sampler thread wakes `hz` times a
// second, and sends SIGPROF to every thread of the process that is running
// at that moment (state R in /proc/self/task/TID/stat); the handler records
// its instruction pointer.  (ITIMER_PROF delivered only ~15 samples a
// second to a 20-thread process.)  hp_stop() writes one line
// per sample: "<object path> <offset in object> <symbol or ?>" (dladdr), to
// be aggregated by tools/hostprof/report.py (nm resolves local symbols).
//   gcc -O2 -shared -fPIC tools/hostprof/hostprof.c -o tools/hostprof/libhostprof.so -ldl -lpthread
#define _GNU_SOURCE
#include <dlfcn.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/time.h>
#include <ucontext.h>
#include <dirent.h>
#include <pthread.h>
#include <stdlib.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#define MAXS (1u << 21)
static uintptr_t samples[MAXS];
static atomic_uint nsamp;

static void on_prof(int sig, siginfo_t* si, void* ucv) {
  (void)sig;
  (void)si;
  const ucontext_t* uc = (const ucontext_t*)ucv;
  const unsigned i = atomic_fetch_add(&nsamp, 1u);
  if (i < MAXS) samples[i] = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
}

static atomic_int running;
static pthread_t sampler;
static int period_us = 500;

static void* sampler_main(void* arg) {
  (void)arg;
  const pid_t pid = getpid(), self = (pid_t)syscall(SYS_gettid);
  char path[64], buf[256];
  while (atomic_load(&running)) {
    DIR* d = opendir("/proc/self/task");
    if (d) {
      struct dirent* e;
      while ((e = readdir(d))) {
        const pid_t tid = (pid_t)atoi(e->d_name);
        if (tid <= 0 || tid == self) continue;
        snprintf(path, sizeof path, "/proc/self/task/%d/stat", (int)tid);
        FILE* f = fopen(path, "r");
        if (!f) continue;
        const size_t n = fread(buf, 1, sizeof buf - 1, f);
        fclose(f);
        buf[n] = 0;
        const char* rp = strrchr(buf, ')');  // "tid (comm) S ..."
        if (rp && rp[1] == ' ' && rp[2] == 'R') syscall(SYS_tgkill, pid, tid, SIGPROF);
      }
      closedir(d);
    }
    struct timespec ts = {0, period_us * 1000L};
    nanosleep(&ts, NULL);
  }
  return NULL;
}

int hp_start(int hz) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, NULL)) return -1;
  atomic_store(&nsamp, 0u);
  period_us = 1000000 / (hz > 0 ? hz : 1000);
  atomic_store(&running, 1);
  return pthread_create(&sampler, NULL, sampler_main, NULL);
}

long hp_stop(const char* path) {
  atomic_store(&running, 0);
  pthread_join(sampler, NULL);
  unsigned n = atomic_load(&nsamp);
  if (n > MAXS) n = MAXS;
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  for (unsigned i = 0; i < n; ++i) {
    Dl_info di;
    if (dladdr((void*)samples[i], &di) && di.dli_fname) {
      fprintf(f, "%s %lx %s\n", di.dli_fname, (unsigned long)(samples[i] - (uintptr_t)di.dli_fbase),
              di.dli_sname ? di.dli_sname : "?");
    } else {
      fprintf(f, "? %lx ?\n", (unsigned long)samples[i]);
    }
  }
  fclose(f);
  return (long)n;
}
