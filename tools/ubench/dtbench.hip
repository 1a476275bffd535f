// Direct-table MSM (k_dt_msm) in isolation: the product kernel timed on
// random table rows / scalars (the instruction stream does not depend on the
// values), plus an instrumented copy that stamps s_memtime at its phase
// borders (first gather issued, main loop done, tree done) for lane 0 of
// every block.  Shapes: M MSMs of T terms (IPA round: 256 x 129; A_I/A_O/S:
// 384 x ~214), window c, lanes per MSM.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dtbench.hip -o dtbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../../bulletproof-perm_amd/csrc/msm_kernels.cuh"

static DtGeom geom(uint32_t c) {
  DtGeom g;
  g.c = c;
  g.W = (254 + c - 1) / c;
  g.H = 1u << (c - 1);
  for (int i = 0; i < 8; ++i) g.K[i] = 0;
  for (uint32_t w = 0; w + 1 < g.W; ++w) {
    const uint32_t pos = c * w + c - 1;
    g.K[pos >> 5] |= 1u << (pos & 31);
  }
  return g;
}

__global__ void k_fill(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = x & 0x1ffffffu;  // limb-sized words (tight field elements)
  }
}

__global__ void k_fix_scalars(uint32_t* s, size_t n) {  // < 2^252 (canonical)
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) s[8 * i + 7] &= 0x0fffffffu;
}

// instrumented copy of k_dt_msm (same walk, same tree)
__global__ void __launch_bounds__(DT_NT_MAX) k_dt_msm_stamped(const uint32_t* __restrict__ dt, DtGeom dg,
                                                            const uint32_t* __restrict__ scalars,
                                                            const uint32_t* __restrict__ pidx,
                                                            const uint32_t* __restrict__ off,
                                                            uint32_t* __restrict__ out_p3,
                                                            unsigned long long* __restrict__ stamps) {
  extern __shared__ uint32_t tl[];
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  const uint32_t nt = blockDim.x, TG = nt / dg.W;
  const uint32_t m = blockIdx.x;
  const uint32_t tg = threadIdx.x / dg.W;
  DtLane ln;
  ln.w = threadIdx.x % dg.W;
  ln.wi = (dg.c * ln.w) >> 5;
  ln.sh = (dg.c * ln.w) & 31;
  ln.fmask = (1u << dg.c) - 1u;
  ln.W = dg.W;
  ln.H = dg.H;
  ln.top = ln.w + 1 == dg.W;
  const uint32_t t1 = off[m + 1];
  uint32_t t = off[m] + tg;
  ge_p3 acc = ge_identity();
  unsigned long long t_first = 0;
  if (tg < TG && t < t1) {
    uint32_t sc[8];
    load_scalar(scalars, t, sc);
    uint32_t gen = pidx ? pidx[t] : t;
    uint32_t tn = t + TG;
    uint32_t scn[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t genn = 0;
    if (tn < t1) {
      load_scalar(scalars, tn, scn);
      genn = pidx ? pidx[tn] : tn;
    }
    uint32_t row;
    bool neg, zero;
    ln.row_of(dg, sc, gen, row, neg, zero);
    ge_niels q = load_niels(dt, row);
    t_first = __builtin_amdgcn_s_memtime();
    for (;;) {
      if (zero) q = ge_niels_identity();
      const ge_madd_mid mid = ge_madd_signed_h1(acc, q, neg);
      const bool more = tn < t1;
      bool neg2 = false, zero2 = false;
      if (more) {
        uint32_t row2;
        ln.row_of(dg, scn, genn, row2, neg2, zero2);
        q = load_niels(dt, row2);
        tn += TG;
        if (tn < t1) {
          load_scalar(scalars, tn, scn);
          genn = pidx ? pidx[tn] : tn;
        }
      }
      acc = ge_madd_h2(mid);
      if (!more) break;
      neg = neg2;
      zero = zero2;
    }
  }
  const unsigned long long t_loop = __builtin_amdgcn_s_memtime();
  store_p3(tl, threadIdx.x, acc);
  __syncthreads();
  const unsigned long long t_bar = __builtin_amdgcn_s_memtime();
  uint32_t p2 = 1;
  while (p2 < nt) p2 <<= 1;
  for (uint32_t s = p2 >> 1; s > 0; s >>= 1) {
    if (threadIdx.x < s && threadIdx.x + s < nt)
      store_p3(tl, threadIdx.x, ge_add(load_p3(tl, threadIdx.x), load_p3(tl, threadIdx.x + s)));
    __syncthreads();
  }
  const unsigned long long t_tree = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    store_p3(out_p3, m, load_p3(tl, 0));
    stamps[5 * m + 0] = t_start;
    stamps[5 * m + 1] = t_first;
    stamps[5 * m + 2] = t_loop;
    stamps[5 * m + 3] = t_bar;
    stamps[5 * m + 4] = t_tree;
  }
}

// Experiment (rejected): two accumulator chains per lane.
// (A depth-2 row prefetch was measured the same way: 74.0 vs 70.1 us for
// the IPA round shape, 154.7 vs 152.4 for A_I/A_O/S.)
// Two independent accumulator chains per lane (terms t, t + 2 TG, ... and
// t + TG, t + 3 TG, ...), advanced together so that a lone wave has two
// dependent instruction streams to interleave; summed at the end.
template <class Src>
FE_INLINE ge_p3 dt_walk_ilp2(const uint32_t* __restrict__ dt, const DtGeom& dg, const DtLane& ln, uint32_t t,
                             uint32_t t1, uint32_t TG, const Src& src) {
  ge_p3 a0 = ge_identity(), a1 = ge_identity();
  uint32_t sc[8];
  uint32_t gen, row;
  for (; t < t1; t += 2 * TG) {
    bool n0, z0, n1 = false, z1 = true;
    src(t, sc, gen);
    ln.row_of(dg, sc, gen, row, n0, z0);
    ge_niels q0 = load_niels(dt, row);
    ge_niels q1 = ge_niels_identity();
    if (t + TG < t1) {
      src(t + TG, sc, gen);
      ln.row_of(dg, sc, gen, row, n1, z1);
      q1 = load_niels(dt, row);
    }
    if (z0) q0 = ge_niels_identity();
    if (z1) q1 = ge_niels_identity();
    const ge_madd_mid m0 = ge_madd_signed_h1(a0, q0, n0);
    const ge_madd_mid m1 = ge_madd_signed_h1(a1, q1, n1);
    a0 = ge_madd_h2(m0);
    a1 = ge_madd_h2(m1);
  }
  return ge_add(a0, a1);
}

__global__ void __launch_bounds__(DT_NT_MAX) k_dt_msm2(const uint32_t* __restrict__ dt, DtGeom dg,
                                                     const uint32_t* __restrict__ scalars,
                                                     const uint32_t* __restrict__ pidx,
                                                     const uint32_t* __restrict__ off, uint32_t* __restrict__ out_p3) {
  extern __shared__ uint32_t tl[];
  const uint32_t nt = blockDim.x, TG = nt / dg.W;
  const uint32_t m = blockIdx.x;
  const DtLane ln = DtLane::make(dg, threadIdx.x % dg.W);
  const uint32_t tg = threadIdx.x / dg.W;
  const ge_p3 acc = tg < TG ? dt_walk_ilp2(dt, dg, ln, off[m] + tg, off[m + 1], TG,
                                       [&](uint32_t t, uint32_t s[8], uint32_t& gen) {
                                         load_scalar(scalars, t, s);
                                         gen = pidx ? pidx[t] : t;
                                       })
                            : ge_identity();
  dt_block_tree(tl, acc, nt, out_p3, m);
}

static float time_kernel(bool two, uint32_t M, uint32_t nt, const uint32_t* dt, DtGeom g, const uint32_t* sc,
                         const uint32_t* pidx, const uint32_t* off, uint32_t* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9;
  for (int rep = 0; rep < 7; ++rep) {
    hipEventRecord(a);
    if (two)
      hipLaunchKernelGGL(k_dt_msm2, dim3(M), dim3(nt), nt * 160, 0, dt, g, sc, pidx, off, out);
    else
      hipLaunchKernelGGL(k_dt_msm, dim3(M), dim3(nt), nt * 160, 0, dt, g, sc, pidx, off, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best;
}

static void run(uint32_t c, uint32_t M, uint32_t T, uint32_t nt_cap) {
  const DtGeom g = geom(c);
  const uint32_t ngen = 258;
  const size_t rows = (size_t)ngen * g.W * g.H;
  uint32_t *dt, *sc, *pidx, *off, *out;
  unsigned long long* st;
  hipMalloc(&dt, rows * 128);
  hipMalloc(&sc, (size_t)M * T * 32);
  hipMalloc(&pidx, (size_t)M * T * 4);
  hipMalloc(&off, (M + 1) * 4);
  hipMalloc(&out, (size_t)M * 160);
  hipMalloc(&st, (size_t)M * 5 * 8);
  k_fill<<<4096, 256>>>(dt, rows * 32, 1);
  k_fill<<<4096, 256>>>(sc, (size_t)M * T * 8, 2);
  k_fix_scalars<<<(M * T + 255) / 256, 256>>>(sc, (size_t)M * T);
  std::vector<uint32_t> hp((size_t)M * T), ho(M + 1);
  for (size_t i = 0; i < hp.size(); ++i) hp[i] = (uint32_t)((i * 7919) % ngen);
  for (uint32_t m = 0; m <= M; ++m) ho[m] = m * T;
  hipMemcpy(pidx, hp.data(), hp.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(off, ho.data(), ho.size() * 4, hipMemcpyHostToDevice);
  uint32_t TG = nt_cap / g.W;
  while (TG > 1 && (double)T < 2.0 * TG) TG >>= 1;
  const uint32_t nt = TG * g.W;
  hipFuncSetAttribute((const void*)k_dt_msm, hipFuncAttributeMaxDynamicSharedMemorySize, DT_NT_MAX * 160);
  hipFuncSetAttribute((const void*)k_dt_msm_stamped, hipFuncAttributeMaxDynamicSharedMemorySize, DT_NT_MAX * 160);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL(k_dt_msm, dim3(M), dim3(nt), nt * 160, 0, dt, g, sc, pidx, off, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  // same result from the depth-2 walk, and its time
  std::vector<uint32_t> r1((size_t)M * 40), r2((size_t)M * 40);
  hipMemcpy(r1.data(), out, r1.size() * 4, hipMemcpyDeviceToHost);
  const float t2 = time_kernel(true, M, nt, dt, g, sc, pidx, off, out);
  hipMemcpy(r2.data(), out, r2.size() * 4, hipMemcpyDeviceToHost);
  printf("  two chains per lane: %7.1f us (projective coordinates differ: %s)\n", t2 * 1e3, r1 == r2 ? "no" : "yes");
  hipLaunchKernelGGL(k_dt_msm_stamped, dim3(M), dim3(nt), nt * 160, 0, dt, g, sc, pidx, off, out, st);
  hipDeviceSynchronize();
  std::vector<unsigned long long> hs((size_t)M * 5);
  hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost);
  double ph[4] = {0, 0, 0, 0};
  unsigned long long t0 = ~0ull, t_end = 0;
  for (uint32_t m = 0; m < M; ++m) {
    for (int k = 0; k < 4; ++k) ph[k] += (double)(hs[5 * m + k + 1] - hs[5 * m + k]);
    t0 = hs[5 * m] < t0 ? hs[5 * m] : t0;
    t_end = hs[5 * m + 4] > t_end ? hs[5 * m + 4] : t_end;
  }
  // s_memtime counts shader cycles (MI355X_MICROARCH.md): us at ~2.4 GHz
  const double tick_us = 1.0 / 2400.0;
  const double madds = (double)M * T * g.W;
  printf("c=%2u W=%2u M=%4u T=%4u lanes=%3u  kernel %7.1f us  %6.2f G madd/s | per block (us): first-gather %6.1f"
         "  loop %6.1f  barrier-wait %6.1f  tree %6.1f  (span %7.1f)\n",
         c, g.W, M, T, nt, best * 1e3, madds / (best * 1e-3) / 1e9, ph[0] / M * tick_us, ph[1] / M * tick_us,
         ph[2] / M * tick_us, ph[3] / M * tick_us, (double)(t_end - t0) * tick_us);
  hipFree(dt);
  hipFree(sc);
  hipFree(pidx);
  hipFree(off);
  hipFree(out);
  hipFree(st);
}

int main(int argc, char** argv) {
  // IPA round (256 x 129) and A_I/A_O/S (384 x 214) at one batch, and 8
  // batches' IPA rounds at once (the throughput regime of 8 in flight)
  for (uint32_t c : {12u, 13u, 16u}) {
    run(c, 256, 129, 256);
    run(c, 384, 214, 256);
    run(c, 2048, 129, 256);
  }
  return 0;
}
