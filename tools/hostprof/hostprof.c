// Minimal in-process CPU sampling profiler for the host side of the prover
// (the GPU box has no perf / gdb): a sampler thread wakes `hz` times a
// second, and sends SIGPROF to every thread of the process that is running
// at that moment (state R in /proc/self/task/TID/stat); the handler records
// its instruction pointer.  (ITIMER_PROF delivered only ~15 samples a
// second to a 20-thread process.)  hp_stop() writes one line
// per sample: "<object path> <offset> <caller offset in libbpperm> <symbol or ?>", to
// be aggregated by tools/hostprof/report.py (nm resolves local symbols);
// for every sample the first word of the interrupted stack that points into
// libbpperm.so's code is kept as a likely caller (libc / runtime samples).
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

#define MAXS (1u << 18)
#define STACKW 48  // words copied from the stack top (caller heuristics)
static uintptr_t samples[MAXS];
static uintptr_t stacks[MAXS][STACKW];
static int tids[MAXS];
static atomic_uint nsamp;

static void on_prof(int sig, siginfo_t* si, void* ucv) {
  (void)sig;
  (void)si;
  const ucontext_t* uc = (const ucontext_t*)ucv;
  const unsigned i = atomic_fetch_add(&nsamp, 1u);
  if (i < MAXS) {
    samples[i] = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
    tids[i] = (int)syscall(SYS_gettid);
    const uintptr_t* sp = (const uintptr_t*)uc->uc_mcontext.gregs[REG_RSP];
    for (int k = 0; k < STACKW; ++k) stacks[i][k] = sp[k];
  }
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

// executable mappings of libbpperm.so (caller candidates must point into code)
static uintptr_t xlo[8], xhi[8];
static int nx = 0;
static void load_exec_ranges(void) {
  FILE* m = fopen("/proc/self/maps", "r");
  if (!m) return;
  char line[512];
  while (nx < 8 && fgets(line, sizeof line, m)) {
    unsigned long lo, hi;
    char perms[8];
    if (sscanf(line, "%lx-%lx %7s", &lo, &hi, perms) == 3 && perms[2] == 'x' && strstr(line, "libbpperm")) {
      xlo[nx] = lo;
      xhi[nx] = hi;
      ++nx;
    }
  }
  fclose(m);
}
static int in_exec(uintptr_t a) {
  for (int i = 0; i < nx; ++i)
    if (a >= xlo[i] && a < xhi[i]) return 1;
  return 0;
}

long hp_stop(const char* path) {
  atomic_store(&running, 0);
  pthread_join(sampler, NULL);
  unsigned n = atomic_load(&nsamp);
  if (n > MAXS) n = MAXS;
  load_exec_ranges();
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  for (unsigned i = 0; i < n; ++i) {
    Dl_info di;
    // caller heuristic for samples outside libbpperm: the first stack word
    // that points into libbpperm.so's code
    unsigned long caller = 0;
    for (int k = 0; k < STACKW; ++k) {
      Dl_info dc;
      if (in_exec(stacks[i][k]) && dladdr((void*)stacks[i][k], &dc) && dc.dli_fname) {
        caller = (unsigned long)(stacks[i][k] - (uintptr_t)dc.dli_fbase);
        break;
      }
    }
    char comm[32] = "?";
    {
      char pth[64];
      snprintf(pth, sizeof pth, "/proc/self/task/%d/comm", tids[i]);
      FILE* c = fopen(pth, "r");
      if (c) {
        if (fgets(comm, sizeof comm, c)) comm[strcspn(comm, "\n ")] = 0;
        fclose(c);
      }
    }
    if (dladdr((void*)samples[i], &di) && di.dli_fname) {
      fprintf(f, "%s %lx %lx %s %s\n", di.dli_fname, (unsigned long)(samples[i] - (uintptr_t)di.dli_fbase), caller,
              comm, di.dli_sname ? di.dli_sname : "?");
    } else {
      fprintf(f, "? %lx %lx %s ?\n", (unsigned long)samples[i], caller, comm);
    }
  }
  fclose(f);
  return (long)n;
}
