// Pippenger multiscalar multiplication kernels (gfx950).
//
// Replaces `RistrettoPoint::vartime_multiscalar_mul` (curve25519-dalek-ng
// 4.1.1 Straus/Pippenger, serial u64 backend) at the reference's 15 call
// sites (circuit_lib.rs:187,202,216,363,374,385,396,407,498,504,509,525,535,
// 552,568) with a batched, sort-based bucket method:
//
//   K1 msm_count      one lane per term: signed radix-2^c digits, per-bucket
//                     histogram (global atomics)
//   K2 scan           exclusive scan of the histogram -> bucket offsets
//   K3 msm_scatter    one lane per term: entries[] sorted by bucket
//                     (point index | sign bit)
//   K4 msm_accumulate one lane per bucket: sum of its points (mixed adds from
//                     the 96-byte affine-Niels table, gathered from HBM)
//   K5 msm_reduce     one workgroup per (msm, window) segment: per-lane
//                     running sums over a bucket range, LDS tree combine
//   K6 msm_horner     one lane per MSM: Horner over windows (batched MSMs);
//                     a single large MSM combines its W window sums on the
//                     host instead (240 serial doublings are latency-bound
//                     on one GPU lane).
//
// Work for an MSM of n terms, window c, W = ceil(254/c) windows:
//   n*W mixed adds (K4) + W*2^c full adds (K5) + (W-1)*c doublings (K6).
#pragma once
#include "ge_io.cuh"

// Bits [pos, pos+c) of a 256-bit little-endian scalar (c <= 24).
FE_INLINE uint32_t scalar_bits(const uint32_t s[8], int pos, int c) {
  const int wi = pos >> 5, sh = pos & 31;
  uint64_t lo = s[wi];
  uint64_t hi = (wi + 1 < 8) ? s[wi + 1] : 0u;
  uint64_t v = (lo | (hi << 32)) >> sh;
  return (uint32_t)v & ((1u << c) - 1u);
}

FE_INLINE void load_scalar(const uint32_t* __restrict__ sc, size_t t, uint32_t s[8]) {
  const uint4* p = reinterpret_cast<const uint4*>(sc + t * 8);
  uint4 a = p[0], b = p[1];
  s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
  s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
}

// Which MSM does term t belong to (offsets has M+1 entries).
FE_INLINE uint32_t msm_of_term(const uint32_t* __restrict__ offsets, uint32_t M, uint32_t t) {
  uint32_t lo = 0, hi = M;  // offsets[lo] <= t < offsets[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}

struct MsmGeom {
  uint32_t M;       // number of MSMs
  uint32_t T;       // total terms
  uint32_t c;       // window bits
  uint32_t W;       // windows of the full signed decomposition = ceil(254/c)
  uint32_t wb;      // first window handled by this launch (multi-GPU split)
  uint32_t Wn;      // windows handled by this launch
  uint32_t B;       // buckets per window = 2^(c-1)
};

// Signed digit loop: calls f(w - wb, digit) for every window in
// [wb, wb + Wn) whose signed radix-2^c digit is non-zero.  Digits lie in
// [-2^(c-1), 2^(c-1)]; scalars must be < 2^253 (canonical mod l).
template <typename F>
FE_INLINE void for_each_digit(const uint32_t s[8], const MsmGeom& g, F f) {
  uint32_t carry = 0;
  const uint32_t half = 1u << (g.c - 1);
  const uint32_t we = g.wb + g.Wn;
  for (uint32_t w = 0; w < we; ++w) {
    uint32_t v = scalar_bits(s, (int)(w * g.c), (int)g.c) + carry;
    int d;
    if (v >= half && w + 1 < g.W) {
      d = (int)v - (int)(1u << g.c);
      carry = 1;
    } else {
      d = (int)v;
      carry = 0;
    }
    if (d != 0 && w >= g.wb) f(w - g.wb, d);
  }
}

__global__ void k_msm_count(const uint32_t* __restrict__ scalars, const uint32_t* __restrict__ offsets,
                            MsmGeom g, uint32_t* __restrict__ cnt) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= g.T) return;
  uint32_t s[8];
  load_scalar(scalars, t, s);
  const uint32_t m = (g.M == 1) ? 0 : msm_of_term(offsets, g.M, t);
  const uint32_t base = m * g.Wn;
  for_each_digit(s, g, [&](uint32_t w, int d) {
    const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u;
    atomicAdd(&cnt[((base + w) << (g.c - 1)) + b], 1u);
  });
}

__global__ void k_msm_scatter(const uint32_t* __restrict__ scalars, const uint32_t* __restrict__ offsets,
                              const uint32_t* __restrict__ pidx, MsmGeom g,
                              const uint32_t* __restrict__ boff, uint32_t* __restrict__ cursor,
                              uint32_t* __restrict__ entries) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= g.T) return;
  uint32_t s[8];
  load_scalar(scalars, t, s);
  const uint32_t m = (g.M == 1) ? 0 : msm_of_term(offsets, g.M, t);
  const uint32_t base = m * g.Wn;
  const uint32_t pi = pidx ? pidx[t] : t;
  for_each_digit(s, g, [&](uint32_t w, int d) {
    const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u;
    const uint32_t gb = ((base + w) << (g.c - 1)) + b;
    const uint32_t pos = boff[gb] + atomicAdd(&cursor[gb], 1u);
    entries[pos] = pi | (d < 0 ? 0x80000000u : 0u);
  });
}

// One lane per bucket.
// Points with index < n0 come from tbl, the rest from tbl1[idx - n0] (so a
// proof's own points can join the resident generators without a copy).
__global__ void __launch_bounds__(256) k_msm_accumulate(const uint32_t* __restrict__ tbl,
                                                       const uint32_t* __restrict__ tbl1, uint32_t n0,
                                                       const uint32_t* __restrict__ entries,
                                                       const uint32_t* __restrict__ boff, uint32_t nbuckets,
                                                       uint32_t* __restrict__ bsum) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nbuckets) return;
  const uint32_t lo = boff[b], hi = boff[b + 1];
  ge_p3 acc = ge_identity();
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t e = entries[i];
    const uint32_t pi = e & 0x7fffffffu;
    ge_niels q = pi < n0 ? load_niels(tbl, pi) : load_niels(tbl1, pi - n0);
    if (e & 0x80000000u) q = ge_niels_neg(q);
    acc = ge_madd(acc, q);
  }
  store_p3(bsum, b, acc);
}

// One workgroup (RT lanes) per segment (msm, window): sum_b (b+1) * bsum[b].
template <int RT>
__global__ void __launch_bounds__(RT) k_msm_reduce(const uint32_t* __restrict__ bsum, MsmGeom g,
                                                  uint32_t* __restrict__ wsum) {
  __shared__ uint32_t lds[RT * 32];
  const uint32_t seg = blockIdx.x;
  const uint32_t per = (g.B + RT - 1) / RT;
  const uint32_t lo = threadIdx.x * per;
  const uint32_t hi = min(lo + per, g.B);
  const size_t base = (size_t)seg * g.B;
  ge_p3 run = ge_identity();
  ge_p3 acc = ge_identity();
  for (uint32_t b = hi; b > lo; --b) {
    run = ge_add(run, load_p3(bsum, base + b - 1));
    acc = ge_add(acc, run);
  }
  // acc = sum (b - lo + 1) B_b ; need + lo * run
  if (lo < hi && lo > 0) {
    ge_p3 m = ge_identity();
    bool started = false;
    for (int bit = 31; bit >= 0; --bit) {
      if (started) m = ge_dbl(m);
      if ((lo >> bit) & 1u) {
        m = started ? ge_add(m, run) : run;
        started = true;
      }
    }
    acc = ge_add(acc, m);
  }
  store_p3(lds, threadIdx.x, acc);
  __syncthreads();
  for (uint32_t s = RT / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      ge_p3 a = load_p3(lds, threadIdx.x);
      ge_p3 b = load_p3(lds, threadIdx.x + s);
      store_p3(lds, threadIdx.x, ge_add(a, b));
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) store_p3(wsum, seg, load_p3(lds, 0));
}

// One lane per MSM: Horner over its W window sums.
__global__ void k_msm_horner(const uint32_t* __restrict__ wsum, MsmGeom g, uint32_t* __restrict__ out) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= g.M) return;
  const size_t base = (size_t)m * g.Wn;
  ge_p3 acc = load_p3(wsum, base + g.Wn - 1);
  for (int w = (int)g.Wn - 2; w >= 0; --w) {
    acc = ge_dbl_n(acc, (int)g.c);
    acc = ge_add(acc, load_p3(wsum, base + w));
  }
  store_p3(out, m, acc);
}
