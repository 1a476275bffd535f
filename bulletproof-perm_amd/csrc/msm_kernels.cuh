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

// Bits [pos, pos + c) of a 256-bit scalar held in registers, with the word
// picked by selects (a runtime index into s[] would put it in scratch).
FE_INLINE uint32_t word_sel(const uint32_t s[8], uint32_t i) {
  uint32_t r = 0;
  _Pragma("unroll") for (uint32_t k = 0; k < 8; ++k) r = (i == k) ? s[k] : r;
  return r;
}
FE_INLINE uint32_t scalar_bits_sel(const uint32_t s[8], uint32_t pos, uint32_t c) {
  const uint32_t wi = pos >> 5, sh = pos & 31;
  const uint64_t v = ((uint64_t)word_sel(s, wi) | ((uint64_t)word_sel(s, wi + 1) << 32)) >> sh;
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
  uint32_t fb;      // fixed-base mode: point idx -> idx*W + w in a table of
                    // precomputed 2^(c*w) multiples; all windows of an MSM
                    // share one bucket set (no Horner combine)
  uint32_t K[8];     // sum_{w < W-1} 2^(c-1) 2^(cw), little-endian words (rs_signed_digit)
  uint32_t tfb = 7;  // radix sort: fine bits of the top window (RS_FINE_BITS
                    // unless it is narrow: see rs_fbits)
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
    const uint32_t seg = g.fb ? m : base + w;
    atomicAdd(&cnt[(seg << (g.c - 1)) + b], 1u);
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
    const uint32_t seg = g.fb ? m : base + w;
    const uint32_t gb = (seg << (g.c - 1)) + b;
    const uint32_t pos = boff[gb] + atomicAdd(&cursor[gb], 1u);
    entries[pos] = (g.fb ? pi * g.W + w : pi) | (d < 0 ? 0x80000000u : 0u);
  });
}

// 4 waves per SIMD (<= 128 VGPRs; the LDS piece buffer also allows 4):
// without the bound the post-barrier fold lifts the kernel to 187 VGPRs.
// (3 waves, with or without a software-pipelined row gather, measured equal
// alone and slower in the pipelined stream: DESIGN.md §4)
#ifndef ACC_WPE
#define ACC_WPE 4
#endif
#define ACC_ATTR __attribute__((amdgpu_waves_per_eu(ACC_WPE, 8)))

// Largest b with boff[b] <= i (boff non-decreasing, boff[0] = 0, i < boff[nb]).
FE_INLINE uint32_t bucket_of(const uint32_t* __restrict__ boff, uint32_t nb, uint32_t i) {
  uint32_t lo = 0, hi = nb;  // boff[lo] <= i < boff[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (boff[mid] <= i) lo = mid; else hi = mid;
  }
  return lo;
}

#ifndef ACC_ADDR_SWAP
#define ACC_ADDR_SWAP 1
#endif
#ifndef ACC_RESET_Z
#define ACC_RESET_Z 1
#endif
// Table row of entry e for ge_madd_fg: for a negative digit (-Q = (y-x,
// y+x, -2dxy)) the (y+x, y-x) fields are read swapped -- the swap is in the
// per-lane load addresses, so it costs no instruction -- and the sign of
// 2dxy is left to ge_madd_fg (F and G exchanged).  The two swapped fields sit
// at 40-byte offsets, so they are read as 8-byte loads.  This replaces the
// divergent negation branch below (a register swap and a carried fe_neg that
// the wave ran in almost every iteration).
FE_INLINE ge_niels fetch_entry_sw(const uint32_t* __restrict__ tbl, const uint32_t* __restrict__ tbl1, uint32_t n0,
                                  uint32_t e) {
  const uint32_t pi = e & 0x7fffffffu;
  const uint32_t neg = e >> 31;
  const uint32_t* row = pi < n0 ? tbl + (size_t)pi * MSM_NIELS_WORDS : tbl1 + (size_t)(pi - n0) * MSM_NIELS_WORDS;
  const uint2* pa = reinterpret_cast<const uint2*>(row + (neg ? 10u : 0u));  // -> ypx
  const uint2* pb = reinterpret_cast<const uint2*>(row + (neg ? 0u : 10u));  // -> ymx
  const uint4* pc = reinterpret_cast<const uint4*>(row + 20);
  uint2 a[5], b[5];
  _Pragma("unroll") for (int i = 0; i < 5; ++i) a[i] = pa[i];
  _Pragma("unroll") for (int i = 0; i < 5; ++i) b[i] = pb[i];
  const uint4 c0 = pc[0], c1 = pc[1];
  const uint2 c2 = *reinterpret_cast<const uint2*>(row + 28);
  ge_niels q;
  _Pragma("unroll") for (int i = 0; i < 5; ++i) {
    q.ypx.v[2 * i] = a[i].x;
    q.ypx.v[2 * i + 1] = a[i].y;
    q.ymx.v[2 * i] = b[i].x;
    q.ymx.v[2 * i + 1] = b[i].y;
  }
  q.xy2d.v[0] = c0.x; q.xy2d.v[1] = c0.y; q.xy2d.v[2] = c0.z; q.xy2d.v[3] = c0.w;
  q.xy2d.v[4] = c1.x; q.xy2d.v[5] = c1.y; q.xy2d.v[6] = c1.z; q.xy2d.v[7] = c1.w;
  q.xy2d.v[8] = c2.x; q.xy2d.v[9] = c2.y;
  return q;
}
// p + q (neg = false) or p - q (neg = true) for q from fetch_entry_sw (its
// (y+x, y-x) already swapped for a negative digit): the sign of 2dxy only
// exchanges F = D - C and G = D + C.
FE_INLINE ge_p3 ge_madd_fg(const ge_p3& p, const ge_niels& q, bool neg) {
  fe A = fe_mul(fe_sub_nc(p.Y, p.X), q.ymx);
  fe B = fe_mul(fe_add_nc(p.Y, p.X), q.ypx);
  fe C = fe_mul(p.T, q.xy2d);
  fe D = fe_add_nc(p.Z, p.Z);
  fe E = fe_sub_nc(B, A);
  fe H = fe_add_nc(B, A);
  const fe Dm = fe_sub(D, C), Dp = fe_add_nc(D, C);
  fe F, G;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    F.v[i] = neg ? Dp.v[i] : Dm.v[i];
    G.v[i] = neg ? Dm.v[i] : Dp.v[i];
  }
  ge_p3 r;
  r.X = fe_mul(E, F);
  r.Y = fe_mul(G, H);
  r.Z = fe_mul(G, F);  // F as the second operand in X and Z: its 19x limbs are shared
  r.T = fe_mul(E, H);
  return r;
}

// Table point of entry e, negated for a negative digit (in this kernel the
// branch measured 1.5 % faster than ge_madd_signed's operand selects).
FE_INLINE ge_niels fetch_entry(const uint32_t* __restrict__ tbl, const uint32_t* __restrict__ tbl1, uint32_t n0,
                               uint32_t e) {
#ifdef EXP_ACC_L2ROWS  // timing experiment only (wrong results): every gather from 1024 L2-resident rows
  const uint32_t pi = e & 0x3ffu;
#else
  const uint32_t pi = e & 0x7fffffffu;
#endif
  ge_niels q = pi < n0 ? load_niels(tbl, pi) : load_niels(tbl1, pi - n0);
#ifdef ACC_NEG_NC
  // (A/B only) -2dxy uncarried (2p - limb < 2^27.6, a valid multiplier
  // operand): 10 subtractions instead of a carried fe_neg, but the 2^20
  // stream ran 1.09 vs 0.85 ms per MSM (accumulate 0.85 vs 0.67 ms; more
  // spills around the branch), profiles/r04_acc_ab.txt
  if (e & 0x80000000u) {
    const fe t = q.ypx;
    q.ypx = q.ymx;
    q.ymx = t;
    q.xy2d = fe_sub_nc(fe_zero(), q.xy2d);
  }
#else
  if (e & 0x80000000u) q = ge_niels_neg(q);
#endif
  return q;
}

// A bucket spanning more than FIX_MAX chunks (bucket skew: the few buckets
// of a narrow top window, equal scalars) is listed in heavy[1..] (count in
// heavy[0]) by the lane where it starts and summed by a whole wave
// (k_msm_fixup_heavy) instead of one lane's serial chain.
#define FIX_MAX 8
#ifndef ACC_T
#define ACC_T 256
#endif
#ifndef ACC_PARK_SPLIT
#define ACC_PARK_SPLIT 1
#endif
#ifndef ACC_PARK_PRE
#define ACC_PARK_PRE 1
#endif

// Balanced bucket accumulation: lane l owns entries [l*K, (l+1)*K) of the
// bucket-sorted entry array, so every lane does exactly K mixed additions
// whatever the bucket-size distribution (the top window of a 253-bit scalar
// is 8x denser than the others at c = 16).  A run (a bucket's entries inside
// one chunk) that covers its whole bucket is written to bsum directly.  A
// bucket crossing chunk borders is finished inside the workgroup when it can
// be: the lanes holding its later pieces park them in LDS, and after a
// barrier the lane where it starts adds them and writes bsum.  Only buckets
// that leave the workgroup (or are heavy) keep global pieces -- the owner's
// partial in tail[l], later pieces in head[l] -- and are assembled by the
// bucket reduction (bucket_total); empty buckets are never written.
// Points with index < n0 come from tbl, the rest from tbl1[idx - n0] (so a
// proof's own points can join the resident generators without a copy).
__global__ void __launch_bounds__(ACC_T) ACC_ATTR k_msm_accumulate(const uint32_t* __restrict__ tbl,
                                                       const uint32_t* __restrict__ tbl1, uint32_t n0,
                                                       const uint32_t* __restrict__ entries,
                                                       const uint32_t* __restrict__ boff, uint32_t nbuckets,
                                                       uint32_t K, uint32_t* __restrict__ bsum,
                                                       uint32_t* __restrict__ head, uint32_t* __restrict__ tail,
                                                       uint32_t* __restrict__ heavy) {
  // K is a multiple of 4 (msm_engine); lane of entry e = e / K
  const uint32_t l = blockIdx.x * ACC_T + threadIdx.x;
  const uint32_t lane_first = blockIdx.x * ACC_T, lane_last = lane_first + ACC_T - 1;
  const uint32_t E = boff[nbuckets];
  const uint32_t i0 = l * K;
  const uint32_t i1 = min(i0 + K, E);
#if ACC_PIECE_GLOBAL
  // (A/B) every later piece to head[l], the owner folding this workgroup's
  // from there after the barrier (a workgroup's waves share the CU's L1, so
  // the barrier's release / acquire makes them visible): no LDS, so the
  // occupancy is the VGPRs' (8 waves per SIMD at 64) instead of 4 workgroups
  // of 40 KB per CU
  auto park = [&](const ge_p3& v, uint32_t, uint32_t) { store_p3(head, l, v); };
  const uint32_t* piece = head + (size_t)lane_first * P3_WORDS;
#else
  __shared__ __attribute__((aligned(16))) uint32_t piece[ACC_T * P3_WORDS];
  // a later piece of a bucket that started in an earlier chunk: to LDS when
  // its owner is in this workgroup and will fold it, else to head[l]
#if ACC_PARK_SPLIT && ACC_PARK_PRE
  // Only a lane's FIRST run can park (its bucket started in an earlier
  // chunk), so where it parks is decided once before the loop (park_lds0)
  // instead of by two divisions by the runtime K inside the divergent close
  // path, which the whole wave executed whenever any lane closed its first
  // run.  Two destinations as two stores (ds_write / global_store), as below.
  bool park_lds0 = false;
  auto park = [&](const ge_p3& v, uint32_t, uint32_t) {
    if (park_lds0)
      store_p3(piece, threadIdx.x, v);
    else
      store_p3(head, l, v);
  };
#elif ACC_PARK_SPLIT
  // the two destinations as two stores (ds_write / global_store) instead of
  // one through a selected generic pointer, which compiled to 10
  // flat_store_dwordx4 on every close: accumulate 0.715-0.735 vs 0.743-0.749
  // ms at 2^20, three interleaved passes (profiles/r05_acc_park_ab.txt)
  auto park = [&](const ge_p3& v, uint32_t s, uint32_t e) {
    const uint32_t l0 = s / K;
    if ((((e - 1) / K) - l0) < FIX_MAX && l0 >= lane_first)
      store_p3(piece, threadIdx.x, v);
    else
      store_p3(head, l, v);
  };
#else
  auto park = [&](const ge_p3& v, uint32_t s, uint32_t e) {
    const uint32_t l0 = s / K;
    uint32_t* dst = ((((e - 1) / K) - l0) < FIX_MAX && l0 >= lane_first) ? piece + threadIdx.x * P3_WORDS
                                                                           : head + (size_t)l * P3_WORDS;
    store_p3(dst, 0, v);
  };
#endif
#endif
  bool owner = false;
  uint32_t b = 0, bstart = 0, bend = 0;
  // a bucket is heavy when it ends FIX_MAX or more lanes past this one:
  // ((bend - 1) / K) - l >= FIX_MAX  <=>  bend - 1 >= (l + FIX_MAX) K (no
  // division by the runtime K in the loop's bucket-close path: accumulate
  // 0.668-0.671 vs 0.682-0.693 ms at 2^20, three interleaved passes,
  // profiles/r04_acc_ab.txt; ACC_HEAVY_DIV = the division, A/B)
  const uint32_t heavy_lim = (l + FIX_MAX) * K;
  ge_p3 acc = ge_identity();
  if (i0 < E) {
    b = bucket_of(boff, nbuckets, i0);
    bstart = boff[b];
    bend = boff[b + 1];
#if ACC_PARK_SPLIT && ACC_PARK_PRE && !ACC_PIECE_GLOBAL
    if (bstart < i0) {
      const uint32_t l0 = bstart / K;
      park_lds0 = (((bend - 1) / K) - l0) < FIX_MAX && l0 >= lane_first;
    }
#endif
    // the lane where a bucket starts lists it if it is heavy
#ifndef ACC_HEAVY_DIV
    if (bstart == i0 && bend - 1 >= heavy_lim) heavy[1 + atomicAdd(&heavy[0], 1u)] = b;
#else
    if (bstart == i0 && ((bend - 1) / K) - l >= FIX_MAX) heavy[1 + atomicAdd(&heavy[0], 1u)] = b;
#endif
    // entries are read 4 at a time (one 16-B load; K is a multiple of 4 and
    // the array is padded): a lane's chunk is contiguous, so per-entry 4-B
    // loads touch the same 128-B line K times across a long loop and
    // re-fetch it once the table gathers have evicted it
    uint4 e4 = make_uint4(0, 0, 0, 0);
#ifndef EXP_ACC_BOFF_CHAIN
    // end of bucket b + 1, loaded one bucket ahead: when b closes, the next
    // bucket (almost always non-empty: ~32 entries each at 2^20) starts at
    // bend and ends at nbend, so the wave does not wait on dependent boff
    // loads in the iteration that closes a run
    uint32_t nbend = boff[min(b + 2, nbuckets)];
#endif
#if ACC_PREFETCH
    // (A/B) one entry ahead: the next entry's table row is requested before
    // this entry's mixed addition, so its load latency hides behind ~5 K
    // cycles of arithmetic instead of stalling the next iteration
    e4 = *reinterpret_cast<const uint4*>(entries + i0);
    uint32_t e_next = e4.x;
    ge_niels q_next = fetch_entry_sw(tbl, tbl1, n0, e_next);
#endif
    for (uint32_t i = i0; i < i1; ++i) {
#if ACC_PREFETCH
      const uint32_t e = e_next;
      const ge_niels q_cur = q_next;
      if (i + 1 < i1) {
        const uint32_t j = i + 1 - i0;
        if ((j & 3u) == 0) e4 = *reinterpret_cast<const uint4*>(entries + i + 1);
        const uint32_t jq = j & 3u;
        e_next = jq == 0 ? e4.x : jq == 1 ? e4.y : jq == 2 ? e4.z : e4.w;
        q_next = fetch_entry_sw(tbl, tbl1, n0, e_next);
      }
#else
      if (((i - i0) & 3u) == 0) e4 = *reinterpret_cast<const uint4*>(entries + i);
      const uint32_t q = (i - i0) & 3u;
      const uint32_t e = q == 0 ? e4.x : q == 1 ? e4.y : q == 2 ? e4.z : e4.w;
#endif
      if (i == bend) {  // close the run of bucket b
        if (bstart >= i0) {
          store_p3(bsum, b, acc);  // whole bucket inside the chunk
        } else {
          park(acc, bstart, bend);  // first run, bucket started earlier
        }
#ifndef EXP_ACC_BOFF_CHAIN
        if (nbend > i) {  // bucket b + 1 is non-empty
          ++b;
          bstart = i;
          bend = nbend;
        } else {  // skip empty buckets
          do { ++b; } while (boff[b + 1] <= i);
          bstart = boff[b];
          bend = boff[b + 1];
        }
        nbend = boff[min(b + 2, nbuckets)];
#else
        do { ++b; } while (boff[b + 1] <= i);
        bstart = boff[b];
        bend = boff[b + 1];
#endif
#ifndef ACC_HEAVY_DIV
        if (bend - 1 >= heavy_lim) heavy[1 + atomicAdd(&heavy[0], 1u)] = b;
#else
        if (((bend - 1) / K) - l >= FIX_MAX) heavy[1 + atomicAdd(&heavy[0], 1u)] = b;
#endif
#if ACC_RESET_Z
        // the identity as (0 : Z : Z : 0) with the accumulator's own Z (never
        // zero): 30 moves instead of materialising (0 : 1 : 1 : 0)'s 40 words
        acc.Y = acc.Z;
        acc.X = fe_zero();
        acc.T = fe_zero();
#else
        acc = ge_identity();
#endif
      }
#if ACC_PREFETCH
      acc = ge_madd_fg(acc, q_cur, (e >> 31) != 0);
#elif ACC_ADDR_SWAP
      acc = ge_madd_fg(acc, fetch_entry_sw(tbl, tbl1, n0, e), (e >> 31) != 0);
#else
      acc = ge_madd(acc, fetch_entry(tbl, tbl1, n0, e));
#endif
    }
    // last run [max(bstart, i0), i1)
    if (bstart >= i0 && bend <= i1) {
      store_p3(bsum, b, acc);
    } else if (bstart < i0) {  // single run crossing both borders
      park(acc, bstart, bend);
    } else {  // bucket starts here and continues: its partial waits in
      owner = true;  // tail[l] (holding it in registers across the barrier
      store_p3(tail, l, acc);  // costs ~20 VGPRs in the main loop)
    }
  }
  __syncthreads();
  if (owner) {
    const uint32_t l1 = (bend - 1) / K;
    if (l1 - l >= FIX_MAX) {  // heavy: k_msm_fixup_heavy's piece convention
      if (bstart == i0) store_p3(head, l, load_p3(tail, l));
      return;
    }
    const uint32_t last = min(l1, lane_last);
    acc = load_p3(tail, l);
    for (uint32_t m = l + 1; m <= last; ++m) acc = ge_add(acc, load_p3(piece, m - lane_first));
    if (l1 <= lane_last) store_p3(bsum, b, acc);
    else store_p3(tail, l, acc);  // continues past this workgroup
  }
}

// Total of non-empty bucket b (global index) spanning entries [bs, be):
// bsum[b] unless the bucket left its owner's workgroup without being heavy
// (then the owner's partial tail[l0] plus the head pieces of the lanes of
// later workgroups).
FE_INLINE ge_p3 bucket_total(size_t b, uint32_t bs, uint32_t be, uint32_t K, const uint32_t* __restrict__ head,
                             const uint32_t* __restrict__ tail, const uint32_t* __restrict__ bsum) {
  const uint32_t l0 = bs / K, l1 = (be - 1) / K;
  const uint32_t next_wg = (l0 / ACC_T + 1) * ACC_T;
  if (l1 < next_wg || l1 - l0 >= FIX_MAX) return load_p3(bsum, b);
  ge_p3 v = load_p3(tail, l0);
  for (uint32_t l = next_wg; l <= l1; ++l) v = ge_add(v, load_p3(head, l));
  return v;
}

// Bucket reduction sum_b (b+1) * bsum[b] per segment (msm, window), in two
// launches so that enough lanes are in flight (the work is ~1/16 of the
// accumulation but latency-bound if given few lanes):
//   k_msm_reduce_partial: block (seg, j) of 64 lanes; lane t owns L buckets
//     [lo, lo+L) (bucket_total; empty ones are skipped): running sum from the top gives sum (b-lo+1) B_b and
//     run = sum B_b, plus lo*run by double-and-add; LDS tree over the wave.
//   k_msm_reduce_final: one 64-lane block per segment sums its BPS partials.
#define RED_T 64
FE_INLINE ge_p3 ge_shfl_xor(const ge_p3& a, int m) {
  ge_p3 o;
  _Pragma("unroll") for (int k = 0; k < FE_LIMBS; ++k) {
    o.X.v[k] = __shfl_xor(a.X.v[k], m, 64);
    o.Y.v[k] = __shfl_xor(a.Y.v[k], m, 64);
    o.Z.v[k] = __shfl_xor(a.Z.v[k], m, 64);
    o.T.v[k] = __shfl_xor(a.T.v[k], m, 64);
  }
  return o;
}
// value of lane (self + d) of the wave (d < 64; lanes past the end read their own)
FE_INLINE ge_p3 ge_shfl_down(const ge_p3& a, int d) {
  ge_p3 o;
  _Pragma("unroll") for (int k = 0; k < FE_LIMBS; ++k) {
    o.X.v[k] = __shfl_down(a.X.v[k], d, 64);
    o.Y.v[k] = __shfl_down(a.Y.v[k], d, 64);
    o.Z.v[k] = __shfl_down(a.Z.v[k], d, 64);
    o.T.v[k] = __shfl_down(a.T.v[k], d, 64);
  }
  return o;
}
#define RED_LMAX 8
FE_INLINE ge_p3 lds_tree_sum(uint32_t* lds, ge_p3 v) {
  store_p3(lds, threadIdx.x, v);
  __syncthreads();
  for (uint32_t s = RED_T / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) store_p3(lds, threadIdx.x, ge_add(load_p3(lds, threadIdx.x), load_p3(lds, threadIdx.x + s)));
    __syncthreads();
  }
  return load_p3(lds, 0);
}

__global__ void __launch_bounds__(RED_T) k_msm_reduce_partial(const uint32_t* __restrict__ boff, uint32_t K,
                                                             const uint32_t* __restrict__ head,
                                                             const uint32_t* __restrict__ tail,
                                                             const uint32_t* __restrict__ bsum, MsmGeom g,
                                                             uint32_t L, uint32_t BPS, uint32_t* __restrict__ part) {
  __shared__ uint32_t lds[RED_T * P3_WORDS];
  const uint32_t seg = blockIdx.x / BPS, j = blockIdx.x % BPS;
  const uint32_t lo = (j * RED_T + threadIdx.x) * L;
  const uint32_t hi = min(lo + L, g.B);
  const size_t base = (size_t)seg * g.B;
  ge_p3 run = ge_identity();
  ge_p3 acc = ge_identity();
  // bucket offsets of the lane's range up front (L <= RED_LMAX): the
  // bucket loads below then do not wait on them one by one
  const uint32_t nb = lo < hi ? hi - lo : 0u;
  uint32_t bo[RED_LMAX + 1];
  _Pragma("unroll") for (uint32_t k = 0; k <= RED_LMAX; ++k) bo[k] = (nb && k <= nb) ? boff[base + lo + k] : 0u;
  for (uint32_t b = hi; b > lo; --b) {
    const uint32_t bs = bo[b - 1 - lo], be = bo[b - lo];
    if (bs != be) run = ge_add(run, bucket_total(base + b - 1, bs, be, K, head, tail, bsum));
    acc = ge_add(acc, run);
  }
  if (lo < hi && lo > 0) {  // + lo * run
    ge_p3 m = run;
    const int top = 31 - __clz(lo);
    for (int bit = top - 1; bit >= 0; --bit) {
      m = ge_dbl(m);
      if ((lo >> bit) & 1u) m = ge_add(m, run);
    }
    acc = ge_add(acc, m);
  }
  const ge_p3 tot = lds_tree_sum(lds, acc);
  if (threadIdx.x == 0) store_p3(part, blockIdx.x, tot);
}

__global__ void __launch_bounds__(RED_T) k_msm_reduce_final(const uint32_t* __restrict__ part, uint32_t BPS,
                                                           uint32_t* __restrict__ wsum) {
  __shared__ uint32_t lds[RED_T * P3_WORDS];
  const uint32_t seg = blockIdx.x;
  ge_p3 acc = ge_identity();
  for (uint32_t j = threadIdx.x; j < BPS; j += RED_T) acc = ge_add(acc, load_p3(part, (size_t)seg * BPS + j));
  const ge_p3 tot = lds_tree_sum(lds, acc);
  if (threadIdx.x == 0) store_p3(wsum, seg, tot);
}

// Bucket reduction for one large MSM (B >= 1024 buckets per window) whose
// power-of-two weights are left to the host Horner, which doubles between
// windows anyway.  With L = RWAVE_L buckets per lane and
// b = 64 L w + L t + i (wave w, lane t, i < L):
//   sum_b (b+1) S_b = sum_{w,t} acc_{w,t}            acc = sum_i (i+1) S_b
//                   + L sum_w sum_{t>=1} suf_{w,t}    suf = suffix sum of the lanes' run = sum_i S_b
//                   + 64 L sum_w w R_w                R_w = suf_{w,0}
// k_msm_reduce_wave: one 64-lane wave per (segment, w): 2L running-sum
//   additions per lane, a 6-step suffix scan, v = acc + L suf (t >= 1), a
//   6-step butterfly; writes V_w = sum_t v and R_w.
// k_msm_reduce_bits: one wave per (segment, term): term 0 is X = sum_w V_w,
//   term 1 + j is Y_j = sum_{w : bit j of w} R_w, so that
//   sum_b (b+1) S_b = X + sum_j 2^(log2(64 L)+j) Y_j (horner_host_terms).
// In a stream of MSMs (bpp_msm_submit) L = 16 (32 waves per 2^15-bucket window): 2^20 three in flight 0.888 /
// 0.892 ms per MSM against 0.913 / 0.899 at L = 8 (whose reduce costs more
// issue slots: 12 scan / butterfly additions per 8 buckets instead of per
// 16); alone the reduce takes 0.233 vs 0.170 ms and L = 32 0.339 ms
// (0.899 / 0.904 pipelined).  An MSM that runs alone (bpp_msm, the verifier's
// single MSM) has idle SIMDs to spare and uses L = 8: twice the waves of the
// stream shape, 2/3 of its serial chain (msm_single_dev; config 5's 17 x 2^14
// buckets, two interleaved passes: reduce 0.159-0.166 ms at L = 8 against
// 0.205-0.209 at L = 4, 0.231-0.234 at 2, 0.228-0.231 at 16, 0.363-0.387 at
// 32 -- the 12 scan / butterfly additions per lane, not the chain, set the
// cost; profiles/r05_reduce_l_ab.txt).
#ifndef RWAVE_LOG
#define RWAVE_LOG 4  // log2 buckets per lane (MSM streams)
#endif
#ifndef RWAVE_LOG_LONE
#define RWAVE_LOG_LONE 3  // log2 buckets per lane when the MSM runs alone (latency)
#endif
#define RWAVE_L (1 << RWAVE_LOG)
#define RWAVE_SHIFT (RWAVE_LOG + 6)  // log2(RWAVE_L * 64)
#define RWAVE_NW_MAX 256             // waves per segment k_msm_reduce_bits folds
template <int LOG>
__global__ void __launch_bounds__(64) k_msm_reduce_wave(const uint32_t* __restrict__ boff, uint32_t K,
                                                       const uint32_t* __restrict__ head,
                                                       const uint32_t* __restrict__ tail,
                                                       const uint32_t* __restrict__ bsum, MsmGeom g,
                                                       uint32_t* __restrict__ part) {
  constexpr uint32_t L = 1u << LOG;
  const uint32_t nw = g.B >> (LOG + 6);
  const uint32_t seg = blockIdx.x / nw, w = blockIdx.x % nw;
  const uint32_t t = threadIdx.x;
  const uint32_t lo = (w * 64 + t) * L;
  const size_t base = (size_t)seg * g.B + lo;
  uint32_t bo[L + 1];
  _Pragma("unroll") for (uint32_t k = 0; k <= L; ++k) bo[k] = boff[base + k];
  ge_p3 run = ge_identity();
  ge_p3 acc = ge_identity();
  // a lane whose buckets are all empty (most of the narrow top window's)
  // keeps run = acc = identity without the additions
  if (bo[0] != bo[L])
    for (int i = (int)L - 1; i >= 0; --i) {
      if (bo[i] != bo[i + 1]) run = ge_add(run, bucket_total(base + i, bo[i], bo[i + 1], K, head, tail, bsum));
      acc = ge_add(acc, run);
    }
  ge_p3 suf = run;  // inclusive suffix sum over lanes t..63
  _Pragma("unroll") for (int d = 1; d < 64; d <<= 1) {
    const ge_p3 s2 = ge_add(suf, ge_shfl_down(suf, d));
    if (t + d < 64) suf = s2;
  }
  ge_p3 sufL = suf;  // L * suf
  _Pragma("unroll") for (int k = 0; k < LOG; ++k) sufL = ge_dbl(sufL);
  ge_p3 v = ge_add(acc, sufL);
  if (t == 0) v = acc;
  _Pragma("unroll") for (int k = 1; k < 64; k <<= 1) v = ge_add(v, ge_shfl_xor(v, k));
  if (t == 0) {
    store_p3(part, 2 * (size_t)blockIdx.x, v);
    store_p3(part, 2 * (size_t)blockIdx.x + 1, suf);  // lane 0: R_w
  }
}

// terms per segment = 1 + log2(nw); lane t folds waves t, t + 64, ...
template <int LOG>
__global__ void __launch_bounds__(64) k_msm_reduce_bits(const uint32_t* __restrict__ part, MsmGeom g,
                                                       uint32_t nterms, uint32_t* __restrict__ out) {
  const uint32_t nw = g.B >> (LOG + 6);
  const uint32_t seg = blockIdx.x / nterms, term = blockIdx.x % nterms;
  ge_p3 v = ge_identity();
  for (uint32_t w = threadIdx.x; w < nw; w += 64)
    if (term == 0 || ((w >> (term - 1)) & 1u)) v = ge_add(v, load_p3(part, 2 * ((size_t)seg * nw + w) + (term ? 1 : 0)));
  _Pragma("unroll") for (int k = 1; k < 64; k <<= 1) v = ge_add(v, ge_shfl_xor(v, k));
  if (threadIdx.x == 0) store_p3(out, blockIdx.x, v);
}

// One lane per MSM: Horner over its W window sums.
__global__ void __launch_bounds__(64) k_msm_horner(const uint32_t* __restrict__ wsum, MsmGeom g, uint32_t* __restrict__ out) {
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

// ---------------------------------------------------------------------------
// Single large MSM sort path (M == 1, c <= 16): digits are recoded once into
// a window-major array of 16-bit codes (below), widened in registers to
// sign << 31 | (|d| - 1) (~0 = zero digit), then one workgroup per (window,
// chunk of terms) builds the bucket
// histogram in LDS.  Global memory then sees one coalesced atomic per
// (block, bucket) instead of one scattered memory-side atomic per
// (term, window) — the global-atomic kernels above ran at ~26 G atomics/s.
#define DIG_ZERO 0xFFFFFFFFu
#define DIG_SIGN 0x80000000u
// In HBM the codes are 16-bit (sign << 15 | (|d| - 1); |d| - 1 < 2^15 for
// c <= 16, and 0x7FFF -- the code of d = +2^15, which signed recoding never
// produces -- marks a zero digit): half the digit traffic of the sort passes.
typedef uint16_t dig_t;
#define DIG16_ZERO 0x7FFFu
FE_INLINE uint32_t dig_expand(uint32_t c16) {
  return c16 == DIG16_ZERO ? DIG_ZERO : ((c16 & 0x7FFFu) | ((c16 & 0x8000u) << 16));
}
#define SORT_T 1024

__global__ void __launch_bounds__(256) k_msm_digits(const uint32_t* __restrict__ scalars, MsmGeom g,
                                                   dig_t* __restrict__ dig) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= g.T) return;
  uint32_t s[8];
  load_scalar(scalars, t, s);
  // for_each_digit's recoding, every window of [wb, wb + Wn) written once
  uint32_t carry = 0;
  const uint32_t half = 1u << (g.c - 1);
  for (uint32_t w = 0; w < g.wb + g.Wn; ++w) {
    const uint32_t v = scalar_bits(s, (int)(w * g.c), (int)g.c) + carry;
    int d;
    if (v >= half && w + 1 < g.W) {
      d = (int)v - (int)(1u << g.c);
      carry = 1;
    } else {
      d = (int)v;
      carry = 0;
    }
    if (w < g.wb) continue;
    const uint32_t code = d == 0 ? DIG16_ZERO : (((uint32_t)(d < 0 ? -d : d) - 1u) | (d < 0 ? 0x8000u : 0u));
    dig[(size_t)(w - g.wb) * g.T + t] = (dig_t)code;
  }
}

// grid = Wn * nchunk blocks; dynamic LDS = B * 4 bytes
__global__ void __launch_bounds__(SORT_T) k_msm_count_lds(const dig_t* __restrict__ dig, MsmGeom g, uint32_t chunk,
                                                         uint32_t nchunk, uint32_t* __restrict__ cnt) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const uint32_t w = blockIdx.x / nchunk, ch = blockIdx.x % nchunk;
  for (uint32_t b = threadIdx.x; b < g.B; b += SORT_T) hist[b] = 0;
  __syncthreads();
  const uint32_t t0 = ch * chunk, t1 = min(t0 + chunk, g.T);
  const dig_t* dw = dig + (size_t)w * g.T;
  for (uint32_t t = t0 + threadIdx.x; t < t1; t += SORT_T) {
    const uint32_t code = dig_expand(dw[t]);
    if (code != DIG_ZERO) atomicAdd(&hist[code & ~DIG_SIGN], 1u);
  }
  __syncthreads();
  uint32_t* cw = cnt + ((size_t)w << (g.c - 1));
  for (uint32_t b = threadIdx.x; b < g.B; b += SORT_T) {
    const uint32_t h = hist[b];
    if (h) atomicAdd(&cw[b], h);
  }
}

__global__ void __launch_bounds__(SORT_T) k_msm_scatter_lds(const dig_t* __restrict__ dig,
                                                           const uint32_t* __restrict__ pidx, MsmGeom g,
                                                           uint32_t chunk, uint32_t nchunk,
                                                           const uint32_t* __restrict__ boff,
                                                           uint32_t* __restrict__ cursor,
                                                           uint32_t* __restrict__ entries) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const uint32_t w = blockIdx.x / nchunk, ch = blockIdx.x % nchunk;
  for (uint32_t b = threadIdx.x; b < g.B; b += SORT_T) hist[b] = 0;
  __syncthreads();
  const uint32_t t0 = ch * chunk, t1 = min(t0 + chunk, g.T);
  const dig_t* dw = dig + (size_t)w * g.T;
  for (uint32_t t = t0 + threadIdx.x; t < t1; t += SORT_T) {
    const uint32_t code = dig_expand(dw[t]);
    if (code != DIG_ZERO) atomicAdd(&hist[code & ~DIG_SIGN], 1u);
  }
  __syncthreads();
  // reserve this block's slice of every bucket: hist[b] becomes a cursor
  const size_t gb0 = (size_t)w << (g.c - 1);
  for (uint32_t b = threadIdx.x; b < g.B; b += SORT_T) {
    const uint32_t h = hist[b];
    hist[b] = h ? boff[gb0 + b] + atomicAdd(&cursor[gb0 + b], h) : 0u;
  }
  __syncthreads();
  for (uint32_t t = t0 + threadIdx.x; t < t1; t += SORT_T) {
    const uint32_t code = dig_expand(dw[t]);
    if (code == DIG_ZERO) continue;
    const uint32_t pos = atomicAdd(&hist[code & ~DIG_SIGN], 1u);
    entries[pos] = (pidx ? pidx[t] : t) | (code & DIG_SIGN);
  }
}

// ---------------------------------------------------------------------------
// Two-pass (MSD) bucket sort for one large MSM, c >= 12.  The one-pass LDS
// scatter above writes every entry as an isolated 4-B store (2^15 buckets
// per window, ~1 entry per bucket per block: 9x write amplification
// measured); here both passes stage in LDS and write runs.
//   k_rsort_count   per (window, chunk of RS_CHUNK digits): histogram of the
//                   coarse bin = bucket >> RS_FINE_BITS (<= 256 bins) ->
//                   cntA[w][bin][chunk]
//   (exclusive scan of cntA: offA = where each block's run of each bin goes;
//    bins of a window and windows follow each other, the final order)
//   k_rsort_scatter coarse scatter of (point idx | fine bits << 24 | sign)
//   k_rsort_fine    one block per (window, coarse bin): LDS counting sort of
//                   its segment by the fine bits; writes the final entries
//                   and the bucket offsets boff of its 128 buckets
#define RS_FINE_BITS 7
#define RS_FINE_N (1u << RS_FINE_BITS)
#define RS_T 256
#define RS_CHUNK 4096  // digits per block in the coarse passes (LDS staging)
#define RS_FMASK (0x7fu << 24)

// Fine bits of window ww of a launch.  Bucket b of a window sorts into
// coarse bin b >> fbits and fine slot b & (2^fbits - 1).  The top window of
// a 253-bit scalar holds fewer bits than the others (13 at c = 16: buckets
// < 2^13, not 2^15), so with 7 fine bits it would fill only 64 of the 256
// coarse bins, each 4x as dense: at 2^23 terms (one rank's share of the
// N = 8 window split) its bins exceed the fine sort's one-tile capacity 16x
// and serialise in the multi-tile path.  Its fine bits are therefore
// g.tfb = top bits - log2(NC) (5 at c = 16), spreading it over all coarse
// bins; its buckets at and above NC << tfb are empty (canonical scalars).
FE_INLINE uint32_t rs_fbits(const MsmGeom& g, uint32_t ww) {
  return g.wb + ww + 1 == g.W ? g.tfb : RS_FINE_BITS;
}
// coarse bin of bucket b (clamped: a non-canonical device scalar gives a
// wrong result, never an out-of-range bin)
FE_INLINE uint32_t rs_bin(uint32_t b, uint32_t fbits, uint32_t NC) { return min(b >> fbits, NC - 1); }

// Digits of a chunk are loaded into registers in one batch of independent
// coalesced loads (RS_PER per thread) before any LDS atomic: a load-then-
// atomic loop leaves each load's latency exposed.
#define RS_PER (RS_CHUNK / RS_T)
FE_INLINE void rs_load_chunk(const dig_t* __restrict__ dw, uint32_t t0, uint32_t t1, uint32_t v[RS_PER]) {
  _Pragma("unroll") for (uint32_t k = 0; k < RS_PER; ++k) {
    const uint32_t t = t0 + k * RS_T + threadIdx.x;
    v[k] = t < t1 ? dig_expand(dw[t]) : DIG_ZERO;
  }
}

__global__ void __launch_bounds__(RS_T) k_rsort_count(const dig_t* __restrict__ dig, MsmGeom g, uint32_t chunk,
                                                     uint32_t nchunk, uint32_t NC, uint32_t* __restrict__ cntA) {
  __shared__ uint32_t h[256];
  const uint32_t w = blockIdx.x / nchunk, ch = blockIdx.x % nchunk;
  for (uint32_t b = threadIdx.x; b < NC; b += RS_T) h[b] = 0;
  const uint32_t t0 = ch * chunk, t1 = min(t0 + chunk, g.T);  // chunk == RS_CHUNK
  uint32_t v[RS_PER];
  rs_load_chunk(dig + (size_t)w * g.T, t0, t1, v);
  __syncthreads();
  _Pragma("unroll") for (uint32_t k = 0; k < RS_PER; ++k)
    if (v[k] != DIG_ZERO) atomicAdd(&h[rs_bin(v[k] & ~DIG_SIGN, rs_fbits(g, w), NC)], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < NC; b += RS_T) cntA[((size_t)w * NC + b) * nchunk + ch] = h[b];
}

// Digits and the coarse histogram in one pass over the scalars (the radix
// path's first kernel; replaces k_msm_digits + k_rsort_count, so the digit
// codes are written once and first read back by the scatter): block = one
// chunk of RS_CHUNK terms, every window of [wb, wb + Wn); LDS histogram of
// the Wn x NC coarse bins -> cntA[(w * NC + bin) * nchunk + ch].  Block 0
// also clears the two words later passes need zeroed (the scan's trailing
// count, the accumulation's heavy-bucket counter): no memset launches.
#define RS_DC_T 1024
#define RS_DC_HMAX 4096  // Wn * NC <= 16 * 256 for c <= 16
__global__ void __launch_bounds__(RS_DC_T) k_rsort_digits_count(const uint32_t* __restrict__ scalars, MsmGeom g,
                                                              uint32_t nchunk, uint32_t NC, dig_t* __restrict__ dig,
                                                              uint32_t* __restrict__ cntA, uint32_t* __restrict__ z0,
                                                              uint32_t* __restrict__ z1) {
  __shared__ uint32_t h[RS_DC_HMAX];
  const uint32_t ch = blockIdx.x, nh = g.Wn * NC;
  for (uint32_t i = threadIdx.x; i < nh; i += RS_DC_T) h[i] = 0;
  if (ch == 0 && threadIdx.x == 0) {
    *z0 = 0;
    *z1 = 0;
  }
  __syncthreads();
  const uint32_t half = 1u << (g.c - 1);
  for (uint32_t k = 0; k < RS_CHUNK / RS_DC_T; ++k) {
    const uint32_t t = ch * RS_CHUNK + k * RS_DC_T + threadIdx.x;
    if (t >= g.T) continue;
    uint32_t s[8];
    load_scalar(scalars, t, s);
    // Signed digits in closed form: with K = sum_{w < W-1} 2^(c-1) 2^(cw),
    // digit w = ((s + K) >> cw mod 2^c) - 2^(c-1) below the top window and
    // (s + K) >> c(W-1) at it -- the digits of the sequential recoding
    // (v >= 2^(c-1) -> v - 2^c, carry 1), but a window costs O(1) instead of
    // a carry walk from window 0 (the rank holding the top windows of a
    // window-split MSM walked all W)
    uint64_t acc = 0;
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      acc += (uint64_t)s[i] + g.K[i];
      s[i] = (uint32_t)acc;
      acc >>= 32;
    }
    for (uint32_t ww = 0; ww < g.Wn; ++ww) {
      const uint32_t w = g.wb + ww;
      const uint32_t v = scalar_bits_sel(s, w * g.c, g.c);
      const int d = w + 1 < g.W ? (int)v - (int)half : (int)v;
      uint32_t code = DIG16_ZERO;
      if (d != 0) {
        const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u;
        code = b | (d < 0 ? 0x8000u : 0u);
        atomicAdd(&h[ww * NC + rs_bin(b, rs_fbits(g, ww), NC)], 1u);
      }
      dig[(size_t)ww * g.T + t] = (dig_t)code;
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nh; i += RS_DC_T) cntA[(size_t)i * nchunk + ch] = h[i];
}

// In-place exclusive scan of a[0..64 * per) (per <= 4) by wave 0; the
// caller synchronises.  a[i] <- base + sum(a[0..i)).
__device__ __forceinline__ void lds_excl_scan_w0(uint32_t* a, uint32_t per, uint32_t base) {
  if (threadIdx.x >= 64) return;
  uint32_t v[4], tot = 0;
  for (uint32_t k = 0; k < per; ++k) {
    v[k] = a[threadIdx.x * per + k];
    tot += v[k];
  }
  uint32_t inc = tot;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(inc, d, 64);
    if ((int)threadIdx.x >= d) inc += u;
  }
  uint32_t run = base + inc - tot;
  for (uint32_t k = 0; k < per; ++k) {
    a[threadIdx.x * per + k] = run;
    run += v[k];
  }
}

// Coarse scatter with block-local staging: entries of the chunk are sorted
// by coarse bin in LDS, then written out bin-run by bin-run (consecutive
// lanes -> consecutive addresses).  (idx < 2^24 on this path.)
__global__ void __launch_bounds__(RS_T) k_rsort_scatter(const dig_t* __restrict__ dig,
                                                       const uint32_t* __restrict__ pidx, MsmGeom g, uint32_t nchunk,
                                                       uint32_t NC, const uint32_t* __restrict__ offA,
                                                       uint32_t* __restrict__ tmpA) {
  __shared__ uint32_t cnt[256], loc[256], gofs[256];
  __shared__ uint32_t stage[RS_CHUNK];
  __shared__ uint8_t sbin[RS_CHUNK];
  const uint32_t w = blockIdx.x / nchunk, ch = blockIdx.x % nchunk;
  const uint32_t fbits = rs_fbits(g, w);
  for (uint32_t b = threadIdx.x; b < 256; b += RS_T) cnt[b] = 0;
  __syncthreads();
  const uint32_t t0 = ch * RS_CHUNK, t1 = min(t0 + RS_CHUNK, g.T);
  uint32_t v[RS_PER];
  rs_load_chunk(dig + (size_t)w * g.T, t0, t1, v);
  _Pragma("unroll") for (uint32_t k = 0; k < RS_PER; ++k)
    if (v[k] != DIG_ZERO) atomicAdd(&cnt[rs_bin(v[k] & ~DIG_SIGN, fbits, NC)], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < 256; b += RS_T) {
    loc[b] = cnt[b];
    gofs[b] = b < NC ? offA[((size_t)w * NC + b) * nchunk + ch] : 0u;
  }
  __syncthreads();
  lds_excl_scan_w0(loc, 4, 0);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < 256; b += RS_T) cnt[b] = loc[b];  // cursors
  __syncthreads();
  _Pragma("unroll") for (uint32_t k = 0; k < RS_PER; ++k) {
    const uint32_t code = v[k];
    if (code == DIG_ZERO) continue;
    const uint32_t t = t0 + k * RS_T + threadIdx.x;
    const uint32_t b = code & ~DIG_SIGN, bin = rs_bin(b, fbits, NC);
    const uint32_t p = atomicAdd(&cnt[bin], 1u);
    stage[p] = (pidx ? pidx[t] : t) | (((b - (bin << fbits)) & (RS_FINE_N - 1)) << 24) | (code & DIG_SIGN);
    sbin[p] = (uint8_t)bin;
  }
  __syncthreads();
  const uint32_t n = cnt[255];  // end of the last bin = entries in this chunk
  for (uint32_t j = threadIdx.x; j < n; j += RS_T) {
    const uint32_t bin = sbin[j];
    tmpA[gofs[bin] + j - loc[bin]] = stage[j];
  }
}

// One block per (window, coarse bin): counting sort of its segment by the
// fine bits, in LDS tiles of RS_FTILE entries with coalesced output runs.
// A segment that fits one tile (all but the top window's, typically) is
// read twice; longer ones get a counting pass first.
#define RS_FTILE 8192
#define RS_FT 512  // 8 waves per block: 4 blocks (40 KB LDS each) = 32 waves per CU
#define RS_FPER (RS_FTILE / RS_FT)
__global__ void __launch_bounds__(RS_FT) k_rsort_fine(const uint32_t* __restrict__ tmpA, uint32_t nchunk,
                                                    const uint32_t* __restrict__ offA, uint32_t* __restrict__ boff,
                                                    uint32_t* __restrict__ entries, uint32_t* __restrict__ end_dst,
                                                    const uint32_t* __restrict__ end_src, MsmGeom g, uint32_t NC) {
  __shared__ uint32_t base[RS_FINE_N], lcnt[RS_FINE_N], lloc[RS_FINE_N];
  __shared__ uint32_t stage[RS_FTILE];
  __shared__ uint8_t sf[RS_FTILE];
  // w * NC + coarse bin, last first: the top window's dense bins (if any
  // take the multi-tile path) should not be the grid's tail
  const uint32_t seg = gridDim.x - 1 - blockIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) *end_dst = *end_src;  // boff[NB] = number of entries
  const uint32_t s = offA[(size_t)seg * nchunk], e = offA[(size_t)(seg + 1) * nchunk];
  // this segment's buckets: w * B + (coarse << fbits) + f, f < 2^fbits
  const uint32_t w = seg / NC, coarse = seg % NC, fbits = rs_fbits(g, w);
  const uint32_t nf = 1u << fbits;
  uint32_t* const sboff = boff + (size_t)w * g.B + (coarse << fbits);
  if (fbits < RS_FINE_BITS) {  // narrow top window: its buckets from NC << fbits up are empty
    const uint32_t wend = offA[(size_t)(w + 1) * NC * nchunk];
    const uint32_t lo = NC << fbits, per = (g.B - lo) / NC;
    for (uint32_t j = threadIdx.x; j < per; j += RS_FT) boff[(size_t)w * g.B + lo + coarse * per + j] = wend;
  }
  if (e - s <= RS_FTILE) {  // one tile, held in registers between the passes
    uint32_t v[RS_FPER];
    _Pragma("unroll") for (uint32_t k = 0; k < RS_FPER; ++k) {
      const uint32_t i = s + k * RS_FT + threadIdx.x;
      v[k] = i < e ? tmpA[i] : 0u;
    }
    if (threadIdx.x < RS_FINE_N) lcnt[threadIdx.x] = 0;
    __syncthreads();
    _Pragma("unroll") for (uint32_t k = 0; k < RS_FPER; ++k)
      if (k * RS_FT + threadIdx.x < e - s) atomicAdd(&lcnt[(v[k] >> 24) & 0x7fu], 1u);
    __syncthreads();
    if (threadIdx.x < RS_FINE_N) lloc[threadIdx.x] = lcnt[threadIdx.x];
    __syncthreads();
    lds_excl_scan_w0(lloc, 2, 0);
    __syncthreads();
    if (threadIdx.x < RS_FINE_N) {
      lcnt[threadIdx.x] = lloc[threadIdx.x];  // cursors
      if (threadIdx.x < nf) sboff[threadIdx.x] = s + lloc[threadIdx.x];
    }
    __syncthreads();
    _Pragma("unroll") for (uint32_t k = 0; k < RS_FPER; ++k) {
      if (k * RS_FT + threadIdx.x >= e - s) continue;
      const uint32_t f = (v[k] >> 24) & 0x7fu;
      stage[atomicAdd(&lcnt[f], 1u)] = v[k] & ~RS_FMASK;
    }
    __syncthreads();
    // stage is sorted by fine bin and the segment's entries are contiguous
    // in the output: one coalesced copy
    for (uint32_t j = threadIdx.x; j < e - s; j += RS_FT) entries[s + j] = stage[j];
    return;
  }
  const bool one_tile = false;
  if (!one_tile) {
    if (threadIdx.x < RS_FINE_N) base[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = s + threadIdx.x; i < e; i += RS_FT) atomicAdd(&base[(tmpA[i] >> 24) & 0x7fu], 1u);
    __syncthreads();
    lds_excl_scan_w0(base, 2, s);
    __syncthreads();
    if (threadIdx.x < nf) sboff[threadIdx.x] = base[threadIdx.x];
  }
  for (uint32_t ts = s; ts < e || (one_tile && ts == s); ts += RS_FTILE) {
    const uint32_t te = min(ts + RS_FTILE, e);
    if (threadIdx.x < RS_FINE_N) lcnt[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = ts + threadIdx.x; i < te; i += RS_FT) atomicAdd(&lcnt[(tmpA[i] >> 24) & 0x7fu], 1u);
    __syncthreads();
    if (threadIdx.x < RS_FINE_N) lloc[threadIdx.x] = lcnt[threadIdx.x];
    __syncthreads();
    lds_excl_scan_w0(lloc, 2, 0);
    __syncthreads();
    if (threadIdx.x < RS_FINE_N) {
      lcnt[threadIdx.x] = lloc[threadIdx.x];  // cursors
      if (one_tile) {
        base[threadIdx.x] = s + lloc[threadIdx.x];
        if (threadIdx.x < nf) sboff[threadIdx.x] = s + lloc[threadIdx.x];
      }
    }
    __syncthreads();
    for (uint32_t i = ts + threadIdx.x; i < te; i += RS_FT) {
      const uint32_t v = tmpA[i];
      const uint32_t f = (v >> 24) & 0x7fu;
      const uint32_t p = atomicAdd(&lcnt[f], 1u);
      stage[p] = v & ~RS_FMASK;
      sf[p] = (uint8_t)f;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < te - ts; j += RS_FT) {
      const uint32_t f = sf[j];
      entries[base[f] + j - lloc[f]] = stage[j];
    }
    __syncthreads();
    // advance the global cursors by this tile's counts (lcnt = lloc + count)
    if (threadIdx.x < RS_FINE_N) base[threadIdx.x] += lcnt[threadIdx.x] - lloc[threadIdx.x];
    __syncthreads();
    if (one_tile) break;
  }
}

// ---------------------------------------------------------------------------
// Direct fixed-base MSM over full radix-2^c tables (small MSMs over resident
// generators: A_I/A_O/S, IPA rounds, vector commitments).  With
// W = ceil(254 / c) windows and H = 2^(c-1) rows per window, table row
// (gen * W + w) * H + |d| - 1 holds d * 2^(c w) * G_gen (d = 1..H), so a term
// is at most W table additions and an MSM is one flat sum: no digit sort, no
// buckets, no bucket reduction.
//
// Digits in closed form: with K = sum_{w < W-1} 2^(c w + c - 1) (host,
// DtGeom::K), field w of s + K minus H is signed digit w in [-H, H) for
// w < W - 1 and field W - 1 the top digit (>= 0; s < 2^253 so s + K < 2^254),
// the digits of a carry-propagating signed recoding without the carry chain.
//
// One block per MSM, blockDim = W * TG lanes: lane (tg, w) owns WINDOW w of
// terms tg, tg + TG, tg + 2 TG, ... -- the window is fixed per lane, so the
// digit is a fixed bit field of s + K (no per-entry division or scan), and
// the W lanes sharing a term read the same 32 scalar bytes.  Then an LDS
// tree over the block's lanes.
#include "dt_walk.cuh"
#include "sc25519.cuh"

// smap (optional): term t's scalar is scalars[smap[t]] / 2 mod l (the
// prover's halved, compacted A_I/A_O/S terms without a gather pass).
// segs MSMs per block (1 or 2; M = the launch's MSM count): lanes
// [j nt / segs, (j + 1) nt / segs) walk MSM blockIdx.x * segs + j, and the
// segments' block trees run side by side (their narrow levels share waves).
__global__ void __launch_bounds__(DT_NT_MAX) k_dt_msm(const uint32_t* __restrict__ dt, DtGeom dg,
                                                    const uint32_t* __restrict__ scalars,
                                                    const uint32_t* __restrict__ pidx, const uint32_t* __restrict__ off,
                                                    uint32_t* __restrict__ out_p3, const uint32_t* __restrict__ smap,
                                                    uint32_t segs, uint32_t M) {
  extern __shared__ uint32_t tl[];  // blockDim.x extended points (40 KB at 256 lanes)
  const uint32_t nt = blockDim.x, ns = nt / segs, sg = threadIdx.x / ns, lt = threadIdx.x - sg * ns;
  const uint32_t TG = ns / dg.W;
  const uint32_t m0 = blockIdx.x * segs, m = m0 + sg;
  const DtLane ln = DtLane::make(dg, lt % dg.W);
  const uint32_t tg = lt / dg.W;
#ifdef EXP_DT_NOWALK  // timing experiment only (wrong results): no walk, no tree
  if (lt == 0 && m < M) store_p3(out_p3, m, ge_identity());
  return;
#endif
  const ge_p3 acc = tg < TG && m < M ? dt_walk(dt, dg, ln, off[m] + tg, off[m + 1], TG,
                                               [&](uint32_t t, uint32_t s[8], uint32_t& gen) {
                                                 if (smap) {
                                                   const sc h = sc_half(sc_load(scalars + 8 * (size_t)smap[t]));
                                                   _Pragma("unroll") for (int i = 0; i < 8; ++i) s[i] = h.v[i];
                                                 } else {
                                                   load_scalar(scalars, t, s);
                                                 }
                                                 gen = pidx ? pidx[t] : t;
                                               })
                                     : ge_identity();
  dt_block_tree_segs(tl, acc, nt, segs, out_p3, m0, 1, M);
}

// Direct tables from the window tables (wt[k * 32 + u] = 2^(8u) P_k): lane
// (k, w, d) -> d * 2^(c w) P_k = d * 2^r * wt[k * 32 + u], c w = 8u + r.
__global__ void __launch_bounds__(64) k_dt_build(const uint32_t* __restrict__ wt, uint32_t ngen, DtGeom dg,
                                                 uint32_t* __restrict__ dt) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)ngen * dg.W * dg.H) return;
  const uint32_t d = (uint32_t)(i & (dg.H - 1)) + 1u;
  const size_t kw = i >> (dg.c - 1);  // k * W + w
  const uint32_t k = (uint32_t)(kw / dg.W), w = (uint32_t)(kw % dg.W);
  const uint32_t bit = dg.c * w;
  ge_p3 Q = ge_from_niels(load_niels(wt, k * 32u + (bit >> 3)));
  for (uint32_t r = 0; r < (bit & 7u); ++r) Q = ge_dbl(Q);
  ge_p3 R = Q;
  const int top = 31 - __clz(d);
  for (int b = top - 1; b >= 0; --b) {
    R = ge_dbl(R);
    if ((d >> b) & 1u) R = ge_add(R, Q);
  }
  store_niels(dt, (uint32_t)i, ge_to_niels(R));
}

// The same rows, RPL consecutive digits per lane: d0 * Q by double-and-add,
// then d0 + 1 .. d0 + RPL - 1 by one addition each, and the RPL inverses of Z
// by one field inversion (Montgomery's trick).  A lane's chain -- not the row
// count -- sets a table build's time (one wave per SIMD or less: the Q slot
// of bpp_ipa_prove builds 20 x 4096 rows per call), and this chain is ~1/RPL
// of RPL separate double-and-adds and inversions.
template <int RPL>
__global__ void __launch_bounds__(64) k_dt_build_n(const uint32_t* __restrict__ wt, uint32_t ngen, DtGeom dg,
                                                   uint32_t* __restrict__ dt) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // lane: rows [RPL t, RPL t + RPL)
  const size_t i0 = t * RPL;
  if (i0 >= (size_t)ngen * dg.W * dg.H) return;
  const uint32_t d0 = (uint32_t)(i0 & (dg.H - 1)) + 1u;  // (H is a multiple of RPL: one window per lane)
  const size_t kw = i0 >> (dg.c - 1);
  const uint32_t k = (uint32_t)(kw / dg.W), w = (uint32_t)(kw % dg.W);
  const uint32_t bit = dg.c * w;
  ge_p3 Q = ge_from_niels(load_niels(wt, k * 32u + (bit >> 3)));
  for (uint32_t r = 0; r < (bit & 7u); ++r) Q = ge_dbl(Q);
  ge_p3 R[RPL];
  R[0] = Q;
  const int top = 31 - __clz(d0);
  for (int b = top - 1; b >= 0; --b) {
    R[0] = ge_dbl(R[0]);
    if ((d0 >> b) & 1u) R[0] = ge_add(R[0], Q);
  }
  _Pragma("unroll") for (int j = 1; j < RPL; ++j) R[j] = ge_add(R[j - 1], Q);
  fe pre[RPL];
  fe run = R[0].Z;
  pre[0] = fe_one();
  _Pragma("unroll") for (int j = 1; j < RPL; ++j) {
    pre[j] = run;
    run = fe_mul(run, R[j].Z);
  }
  fe inv = fe_invert(run);
  _Pragma("unroll") for (int j = RPL - 1; j >= 0; --j) {
    const fe zi = j ? fe_mul(inv, pre[j]) : inv;
    if (j) inv = fe_mul(inv, R[j].Z);
    store_niels(dt, (uint32_t)(i0 + j), ge_niels_from_affine(fe_mul(R[j].X, zi), fe_mul(R[j].Y, zi)));
  }
}

// One wave per heavy bucket: lane j sums pieces j, j+64, ... of the bucket's
// chunk sequence, then a 6-level shuffle tree.  Blocks past heavy[0] exit.
__global__ void __launch_bounds__(64) k_msm_fixup_heavy(const uint32_t* __restrict__ boff, uint32_t K,
                                                        const uint32_t* __restrict__ head,
                                                        const uint32_t* __restrict__ tail,
                                                        const uint32_t* __restrict__ heavy, uint32_t* __restrict__ bsum) {
  // grid-stride over the listed buckets (the grid is sized for the worst
  // case; most of it would otherwise be empty blocks)
  for (uint32_t hb = blockIdx.x; hb < heavy[0]; hb += gridDim.x) {
    const uint32_t b = heavy[1 + hb];
    const uint32_t s = boff[b], e = boff[b + 1];
    const uint32_t l0 = s / K, np = (e - 1) / K - l0 + 1;  // pieces
    auto piece = [&](uint32_t p) {
      return p ? load_p3(head, l0 + p) : (s == l0 * K ? load_p3(head, l0) : load_p3(tail, l0));
    };
    ge_p3 acc = threadIdx.x < np ? piece(threadIdx.x) : ge_identity();
    for (uint32_t p = threadIdx.x + 64; p < np; p += 64) acc = ge_add(acc, piece(p));
    // butterfly over the lanes that hold pieces only (np is wave-uniform):
    // 4 levels for the 9-16 pieces of a top-window bucket at 2^22 terms
    for (uint32_t k = 1; k < 64 && k < np; k <<= 1) acc = ge_add(acc, ge_shfl_xor(acc, k));
    if (threadIdx.x == 0) store_p3(bsum, b, acc);
  }
}
