// Inner-product argument on gfx950 (bulletproofs 4.0.0 InnerProductProof
// semantics; the reference's hook fields
// ACEssentials.G_factors / H_factors, circuit_lib.rs:62-63).
//
// MSM form.  bulletproofs folds G and H every round with one 2-term MSM per
// element (G'_i = u^-1 Gf_i G_i + u Gf_{i+h} G_{i+h}), a chain of dependent
// 253-bit scalar multiplications that would leave the GPU latency-bound.
// Here the generators never move: with m the current length and
// fG[k] = Gf_k * prod(u_r^{+-1}) the accumulated challenge factor of the
// ORIGINAL G_k, the folded G^{(j)}_r = sum_{k = r mod m} fG[k] G_k, so
//   L_j = sum_k [k mod m >= h] a_{(k mod m) ^ h} fG[k] G_k
//       + sum_k [k mod m <  h] b_{(k mod m) ^ h} fH[k] H_k + c_L Q
// (R_j symmetric) is one n+1-term MSM over the resident table, and a round
// is: scalar terms (k_ipa_terms), c_L / c_R (wave-shuffle reduction,
// k_ipa_cross), a 2-MSM batch through the Pippenger engine, the Fiat-Shamir
// challenge on the host, and the scalar fold (k_ipa_fold).  L, R, a, b are
// identical group elements / scalars to the folding form (same transcript).
#include <cstdlib>
#include <chrono>
#include <thread>
#include <condition_variable>
#include <mutex>
#include <memory>
#include <map>
#include <functional>
#include <cstring>

#include "ctx.h"
#include "dt_walk.cuh"
#include "ipa.h"
#include "merlin_dev.h"
#include "msm_engine.h"
#include "host/par.h"
#include "sc25519.cuh"

DtGeom dt_geom(uint32_t c);                                     // msm.hip
bool msm_use_dt(const MsmPoints& pts, uint32_t M, uint32_t T);  // msm.hip

static unsigned grid_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }


// All kernels run P independent instances of the same length n in lockstep
// (a batch of proofs); per-instance arrays are [P][n] scalars, the MSM term
// arrays [P][2n+2] (L terms then R terms of each instance).
__global__ void __launch_bounds__(256) k_ipa_init(uint32_t n, uint32_t P, const uint32_t* __restrict__ a,
                                                 const uint32_t* __restrict__ b, const uint32_t* __restrict__ gf,
                                                 const uint32_t* __restrict__ hf, uint32_t* __restrict__ am,
                                                 uint32_t* __restrict__ bm, uint32_t* __restrict__ fG,
                                                 uint32_t* __restrict__ fH) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (size_t)n * P) return;
  sc_store(am + 8 * k, sc_to_mont(sc_load(a + 8 * k)));
  sc_store(bm + 8 * k, sc_to_mont(sc_load(b + 8 * k)));
  sc one = sc_zero();
  one.v[0] = 1;
  sc_store(fG + 8 * k, gf ? sc_load(gf + 8 * k) : one);
  sc_store(fH + 8 * k, hf ? sc_load(hf + 8 * k) : one);
}

// terms of L at [0, n+1), of R at [n+1, 2n+2) of each instance; slots n and
// 2n+1 (Q) are written by k_ipa_cross_final.  Both write HALF the term
// scalars: the round's MSMs give L/2, R/2, encoded as L = 2 (L/2) on the host
// (msm_multi_enc), so no separate halving pass over the term array.
__global__ void __launch_bounds__(256) k_ipa_terms(uint32_t n, uint32_t lg_n, uint32_t P, uint32_t m, uint32_t lg_h,
                                                  const uint32_t* __restrict__ am, const uint32_t* __restrict__ bm,
                                                  const uint32_t* __restrict__ fG, const uint32_t* __restrict__ fH,
                                                  uint32_t gbase, uint32_t hbase, uint32_t* __restrict__ scal,
                                                  uint32_t* __restrict__ pidx, uint32_t* __restrict__ part) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)n * P) return;  // (n >= 64 when part is set: whole waves leave)
  const size_t inst = t >> lg_n;
  const uint32_t k = (uint32_t)(t & (n - 1));
  const uint32_t h = m >> 1;
  const uint32_t r = k & (m - 1);
  const bool hi = (r & h) != 0;
  const uint32_t p = r ^ h;
  const uint32_t cidx = ((k >> (lg_h + 1)) << lg_h) | (k & (h - 1));
  const size_t ib = inst << lg_n;  // instance base in [P][n]
  const sc sG = sc_mont(sc_load(am + 8 * (ib + p)), sc_load(fG + 8 * t));  // canonical a_p * fG_k
  const sc sH = sc_mont(sc_load(bm + 8 * (ib + p)), sc_load(fH + 8 * t));
  const size_t tb = inst * (2 * (size_t)n + 2);
  const size_t posG = tb + (hi ? cidx : (n + 1) + cidx);
  const size_t posH = tb + (hi ? (n + 1) + (n >> 1) + cidx : (n >> 1) + cidx);
  sc_store(scal + 8 * posG, sc_half(sG));
  sc_store(scal + 8 * posH, sc_half(sH));
  pidx[posG] = gbase + k;
  pidx[posH] = hbase + k;
  if (part) {
    // fused cross products (n >= 64, so a wave lies in one instance): lane k
    // < h adds a_k b_{k+h} to c_L and a_{k+h} b_k to c_R; one partial per
    // wave -> part[inst][k / 64], summed by k_ipa_cross_final
    sc cl = sc_zero(), cr = sc_zero();
    if (k < h) {
      const sc a0 = sc_load(am + 8 * (ib + k)), a1 = sc_load(am + 8 * (ib + k + h));
      const sc b0 = sc_load(bm + 8 * (ib + k)), b1 = sc_load(bm + 8 * (ib + k + h));
      cl = sc_mont(a0, b1);
      cr = sc_mont(a1, b0);
    }
    cl = sc_wave_sum(cl);
    cr = sc_wave_sum(cr);
    if ((threadIdx.x & 63u) == 0) {
      const size_t o = 16 * (inst * (size_t)(n >> 6) + (k >> 6));
      sc_store(part + o, cl);
      sc_store(part + o + 8, cr);
    }
  }
}

// grid (nb, P): block x of instance y sums its stride of
// <a_lo, b_hi> and <a_hi, b_lo> -> part[y][x] (16 words).
#define CROSS_T 256
__global__ void __launch_bounds__(CROSS_T) k_ipa_cross(uint32_t n, uint32_t h, const uint32_t* __restrict__ am,
                                                      const uint32_t* __restrict__ bm, uint32_t* __restrict__ part) {
  __shared__ uint32_t lds[2][CROSS_T / 64][8];
  const size_t ib = (size_t)blockIdx.y * n;
  sc cl = sc_zero(), cr = sc_zero();
  for (uint32_t i = blockIdx.x * CROSS_T + threadIdx.x; i < h; i += gridDim.x * CROSS_T) {
    const sc a0 = sc_load(am + 8 * (ib + i)), a1 = sc_load(am + 8 * (ib + i + h));
    const sc b0 = sc_load(bm + 8 * (ib + i)), b1 = sc_load(bm + 8 * (ib + i + h));
    cl = sc_add(cl, sc_mont(a0, b1));
    cr = sc_add(cr, sc_mont(a1, b0));
  }
  cl = sc_wave_sum(cl);
  cr = sc_wave_sum(cr);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      lds[0][wid][i] = cl.v[i];
      lds[1][wid][i] = cr.v[i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    sc sl = sc_zero(), sr = sc_zero();
    for (int w = 0; w < CROSS_T / 64; ++w) {
      sc t;
      _Pragma("unroll") for (int i = 0; i < 8; ++i) t.v[i] = lds[0][w][i];
      sl = sc_add(sl, t);
      _Pragma("unroll") for (int i = 0; i < 8; ++i) t.v[i] = lds[1][w][i];
      sr = sc_add(sr, t);
    }
    const size_t o = 16 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x);
    sc_store(part + o, sl);
    sc_store(part + o + 8, sr);
  }
}

// one lane per instance: c_L * qmul, c_R * qmul into the Q slots
__global__ void __launch_bounds__(64) k_ipa_cross_final(uint32_t nblk, uint32_t P, const uint32_t* __restrict__ part,
                                                       const uint32_t* __restrict__ qmul, uint32_t qidx, uint32_t n,
                                                       uint32_t* __restrict__ scal, uint32_t* __restrict__ pidx) {
  const uint32_t inst = blockIdx.x * blockDim.x + threadIdx.x;
  if (inst >= P) return;
  sc sl = sc_zero(), sr = sc_zero();
  for (uint32_t b = 0; b < nblk; ++b) {
    sl = sc_add(sl, sc_load(part + 16 * ((size_t)inst * nblk + b)));
    sr = sc_add(sr, sc_load(part + 16 * ((size_t)inst * nblk + b) + 8));
  }
  // Montgomery c * canonical qmul -> canonical c*qmul
  const sc q = sc_load(qmul + 8 * inst);
  const size_t tb = (size_t)inst * (2 * (size_t)n + 2);
  sc_store(scal + 8 * (tb + n), sc_half(sc_mont(sl, q)));
  sc_store(scal + 8 * (tb + 2 * n + 1), sc_half(sc_mont(sr, q)));
  pidx[tb + n] = qidx;
  pidx[tb + 2 * n + 1] = qidx;
}

// u: [P][16] = (u * R, u^-1 * R) per instance (Montgomery form)
__global__ void __launch_bounds__(256) k_ipa_fold(uint32_t n, uint32_t lg_n, uint32_t P, uint32_t m,
                                                 uint32_t* __restrict__ am, uint32_t* __restrict__ bm,
                                                 uint32_t* __restrict__ fG, uint32_t* __restrict__ fH,
                                                 const uint32_t* __restrict__ u) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)n * P) return;
  const size_t inst = t >> lg_n;
  const uint32_t k = (uint32_t)(t & (n - 1));
  const sc um = sc_load(u + 16 * inst), uim = sc_load(u + 16 * inst + 8);
  const uint32_t h = m >> 1;
  const bool hi = ((k & (m - 1)) & h) != 0;
  // G' = u^-1 G_lo + u G_hi ; H' = u H_lo + u^-1 H_hi
  sc_store(fG + 8 * t, sc_mont(sc_load(fG + 8 * t), hi ? um : uim));
  sc_store(fH + 8 * t, sc_mont(sc_load(fH + 8 * t), hi ? uim : um));
  if (k < h) {
    const size_t ib = inst << lg_n;
    const sc a0 = sc_load(am + 8 * (ib + k)), a1 = sc_load(am + 8 * (ib + k + h));
    const sc b0 = sc_load(bm + 8 * (ib + k)), b1 = sc_load(bm + 8 * (ib + k + h));
    sc_store(am + 8 * (ib + k), sc_add(sc_mont(a0, um), sc_mont(a1, uim)));
    sc_store(bm + 8 * (ib + k), sc_add(sc_mont(b0, uim), sc_mont(b1, um)));
  }
}

// The J partials of a split round's L / R (block b = MSM b, lane j = partial
// b J + j, J a power of two <= 64) summed by dt_block_tree_segs' tree and
// written to out[b] (pinned host memory) -- the host then encodes 2P points
// instead of adding 2P (J - 1) first.
__global__ void __launch_bounds__(64) k_ipa_jsum(const uint32_t* __restrict__ part, uint32_t J,
                                                uint32_t* __restrict__ out) {
  extern __shared__ uint32_t lds[];
  const ge_p3 p = load_p3(part, (size_t)blockIdx.x * J + threadIdx.x);
  dt_block_tree_segs(lds, p, J, 1, out, blockIdx.x, 0);
}

// The last fold of the fused path, for element 0 only (the proof's a, b):
// out[p] = (a_0 u + a_1 u^-1, b_0 u^-1 + b_1 u), Montgomery words, written
// in place into pinned host memory -- one launch where k_ipa_fold over all n
// elements and two copies stood.
__global__ void __launch_bounds__(64) k_ipa_final(uint32_t P, uint32_t n, const uint32_t* __restrict__ am,
                                                 const uint32_t* __restrict__ bm, const uint32_t* __restrict__ u,
                                                 uint32_t* __restrict__ out) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const size_t ib = (size_t)p * n;
  const sc um = sc_load(u + 16 * p), uim = sc_load(u + 16 * p + 8);
  sc_store(out + 16 * p, sc_add(sc_mont(sc_load(am + 8 * ib), um), sc_mont(sc_load(am + 8 * (ib + 1)), uim)));
  sc_store(out + 16 * p + 8, sc_add(sc_mont(sc_load(bm + 8 * ib), uim), sc_mont(sc_load(bm + 8 * (ib + 1)), um)));
}

// One whole IPA round per launch over the direct tables (the fused form of
// k_ipa_fold + k_ipa_terms + k_ipa_cross_final + k_dt_msm): block 2i + s is
// instance i's L (s = 0) or R (s = 1).  The block
//   1. folds the previous round's challenge into a, b (length 2m -> m) and
//      the generator factors fG, fH (all n) when `fold`, reading set *_in and
//      (side 0 only) writing set *_out -- the two sides compute the same
//      values, so the other side's reads of *_in never race with a write;
//   2. builds its n + 1 halved term scalars in LDS (as k_ipa_terms: L gets
//      a_lo fG_hi and b_hi fH_lo, R the mirror) and c_L or c_R (block
//      reduction of a_lo b_hi / a_hi b_lo) times qmul for the Q term;
//   3. runs the direct-table walk over those terms and the block tree
//      (dt_walk.cuh) -> out_p3[blockIdx.x] = L/2 or R/2 (halve: the host
//      encodes 2 (L/2)), or L / R (the device transcript path encodes them
//      on the GPU).
// One launch per round instead of four: the latency of three small kernels
// and their passes over the [P][n] arrays leave every round of a batch.
// (512-lane blocks, half the walk per lane: 73.9 vs 70.8 us per round -- a
// lone wave per SIMD already issues the walk at its rate)
// One batch's round as the fused kernel sees it (k_ipa_round_dt's
// arguments; k_ipa_round_dt_multi runs several batches' rounds in one launch).
struct IpaRoundArgs {
  const uint32_t *am_in, *bm_in, *fG_in, *fH_in;
  uint32_t *am_out, *bm_out, *fG_out, *fH_out;
  const uint32_t *u, *qmul;
  uint32_t* out_p3;
  const uint32_t *a0, *b0, *gf0, *hf0;
  uint32_t m, lg_h, fold, init, halve, gbase, hbase, qidx;
  uint32_t blocks;  // 2 P J (k_ipa_round_dt_multi)
  uint32_t split;   // J: blocks per L / R MSM, each walking a slice of its n + 1 terms
  const uint32_t* qpow;  // IpaGens::qpow (null: Q's term walked from its table rows)
  uint32_t qrow0;        // qpow's first row as a row of dt (the virtual terms' rows)
  uint32_t *done_ticket, *done_word;  // the launch's completion flag (null: none)
  uint32_t done_tag;
  // P = 1: the challenge's words u R, u^-1 R by value (kernel arguments)
  // instead of a load from pinned host memory at the head of the round
  uint32_t u1;
  sc u1m, u1im;
};

// u R, u^-1 R of a one-instance round, passed by value (IpaRoundArgs::u1)
struct IpaU1 {
  uint32_t w[16];
};

// QP (IpaGens::qpow): c Q for the Q term's scalar c with Q given as its 253
// doublings 2^j Q, Niels rows inside dt from row qrow0 (no per-call direct
// table for Q, whose build cost 152 us of bpp_ipa_prove in config 2): the
// Q term becomes V = ceil(253 / W) virtual terms carrying c, and lane w of
// virtual term v adds 2^(vW + w) Q when that bit of c is set
// (DtLane::row_of_q) -- walked like any other term.
// The launch's completion flag (ctx_done_flag / ctx_wait_flag): after the
// block's results are stored (all by wave 0, whose thread 0 runs this),
// each block counts itself on the device ticket behind a system-scope
// release; the last one re-zeroes the ticket and writes the tag to the
// host's word.  Vector atomics and stores only.
FE_INLINE void done_signal(uint32_t* ticket, uint32_t* word, uint32_t tag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    if (atomicAdd(ticket, 1u) == gridDim.x - 1) {
      atomicExch(ticket, 0u);
      __threadfence_system();
      __hip_atomic_store(word, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <bool QP>  // QP: Q by its doublings (A.qpow), a separate instantiation (VGPRs)
FE_INLINE void ipa_round_body(const uint32_t* __restrict__ dt, const DtGeom& dg, uint32_t n, uint32_t TG,
                              const IpaRoundArgs& A, uint32_t bidx, uint32_t* lds, uint32_t S) {
  const uint32_t m = A.m, lg_h = A.lg_h, fold = A.fold, init = A.init, halve = A.halve, gbase = A.gbase,
                 hbase = A.hbase, qidx = A.qidx, J = A.split;
  const uint32_t* __restrict__ am_in = A.am_in;
  const uint32_t* __restrict__ bm_in = A.bm_in;
  const uint32_t* __restrict__ fG_in = A.fG_in;
  const uint32_t* __restrict__ fH_in = A.fH_in;
  uint32_t* __restrict__ am_out = A.am_out;
  uint32_t* __restrict__ bm_out = A.bm_out;
  uint32_t* __restrict__ fG_out = A.fG_out;
  uint32_t* __restrict__ fH_out = A.fH_out;
  const uint32_t* __restrict__ u = A.u;
  const uint32_t* __restrict__ qmul = A.qmul;
  uint32_t* __restrict__ out_p3 = A.out_p3;
  const uint32_t* __restrict__ a0 = A.a0;
  const uint32_t* __restrict__ b0 = A.b0;
  const uint32_t* __restrict__ gf0 = A.gf0;
  const uint32_t* __restrict__ hf0 = A.hf0;
  const uint32_t VQ = QP ? (253u + dg.W - 1) / dg.W : 1u;  // Q term slots: 1, or QP's V virtual terms
  const uint32_t NS = n + VQ;                    // term slots per side
  uint32_t* tsc = lds;                           // S x (n + 1) x 8 words: halved term scalars
  uint32_t* tgen = lds + 8 * S * NS;             // S x (n + 1) generator indices
  uint32_t* sa = tgen + ((S * NS + 3) & ~3u);    // m x 8: a (Montgomery), this round
  uint32_t* sb = sa + 8 * m;                     // m x 8: b
  uint32_t* red = sb + 8 * m;                    // S x waves x 8 words
  const uint32_t nt = blockDim.x, tid = threadIdx.x, nwv = (nt + 63) / 64;
  // S = 1: block bidx is slice jp of J of MSM bidx / J = instance inst's L
  // (side 0) or R; S = 2: slice jp of instance bidx / J, both sides
  uint32_t inst, side0, jp;
  if (S == 2) {
    inst = bidx / J;
    jp = bidx - inst * J;
    side0 = 0;
  } else {
    const uint32_t msm = bidx / J;
    jp = bidx - msm * J;
    inst = msm >> 1;
    side0 = msm & 1u;
  }
  const size_t ib = (size_t)inst * n;
  // init (the first round, no fold): a, b and the generator factors come
  // from the caller's canonical arrays a0, b0, gf0, hf0 (null: all one), and
  // side 0 writes the Montgomery state that round 1 folds (k_ipa_init's work)
  const bool writer = (fold || init) && side0 == 0 && jp == 0;
  sc um = sc_zero(), uim = sc_zero();
  if (fold) {
    um = A.u1 ? A.u1m : sc_load(u + 16 * inst);
    uim = A.u1 ? A.u1im : sc_load(u + 16 * inst + 8);
  }
#ifndef IPA_SPLIT_PROLOGUE
#define IPA_SPLIT_PROLOGUE 1
#endif
  if (IPA_SPLIT_PROLOGUE && J > 1) {
    // A split round (J blocks per MSM: small batches, config 2): each block
    // computes only what its slice needs -- the term scalars of its n / J
    // slots per side, its J-th of the next state's writes and of the cross
    // product -- instead of every block folding the whole state and forming
    // all 2n term scalars (28 of a config-2 round's 64 us, EXP_IPA_NOWALK).
    // The Q term rides in every block with that block's share of
    // c = <a_lo, b_hi> (resp. <a_hi, b_lo>): the host adds the J partials,
    // and sum_jp c^(jp) Q = c Q.
    const uint32_t h = m >> 1;
    const uint32_t* __restrict__ gf0p = A.gf0;
    const uint32_t* __restrict__ hf0p = A.hf0;
    auto cur_ab = [&](bool isb, uint32_t p) -> sc {  // element p of this round's a or b (Montgomery)
      const uint32_t* in = isb ? bm_in : am_in;
      if (fold)
        return sc_add(sc_mont(sc_load(in + 8 * (ib + p)), isb ? uim : um),
                      sc_mont(sc_load(in + 8 * (ib + p + m)), isb ? um : uim));
      if (init) return sc_to_mont(sc_load((isb ? b0 : a0) + 8 * (ib + p)));
      return sc_load(in + 8 * (ib + p));
    };
    auto factor = [&](bool ish, uint32_t k) -> sc {  // generator k's factor this round (canonical)
      sc f;
      if (init) {
        const uint32_t* r = ish ? hf0p : gf0p;
        if (r) {
          f = sc_load(r + 8 * (ib + k));
        } else {
          f = sc_zero();
          f.v[0] = 1;
        }
      } else {
        f = sc_load((ish ? fH_in : fG_in) + 8 * (ib + k));
      }
      if (fold) {
        const bool hi_prev = (k & (2 * m - 1)) & m;
        f = sc_mont(f, hi_prev != ish ? um : uim);
      }
      return f;
    };
    // (ii) the slice's term scalars: side slots [t0, t1) of [0, n) (G terms
    // below n / 2, H terms above), local slot cnt = the Q term
    const uint32_t t0 = (uint32_t)((uint64_t)jp * n / J), t1 = (uint32_t)((uint64_t)(jp + 1) * n / J);
    const uint32_t cnt = t1 - t0, CS = cnt + VQ;
    uint32_t* tsl = lds;                            // S x CS x 8 words
    uint32_t* tgl = lds + 8 * S * CS;               // S x CS
    uint32_t* redl = tgl + ((S * CS + 3) & ~3u);    // S x waves x 8 words
    for (uint32_t q = tid; q < S * cnt; q += nt) {
      const uint32_t s = q / cnt, slot = t0 + (q - s * cnt);
      const uint32_t side = S == 2 ? s : side0;
      const bool ish = slot >= (n >> 1);
      const uint32_t cidx = slot - (ish ? (n >> 1) : 0u);
      const bool hi = ish != (side == 0);  // G_k on side 0 for hi k, H_k for lo k
      const uint32_t k = ((cidx >> lg_h) << (lg_h + 1)) | (hi ? h : 0u) | (cidx & (h - 1));
      const uint32_t p = (k & (m - 1)) ^ h;
      const sc x = sc_mont(cur_ab(ish, p), factor(ish, k));
      sc_store(tsl + 8 * (s * CS + (slot - t0)), halve ? sc_half(x) : x);
      tgl[s * CS + (slot - t0)] = (ish ? hbase : gbase) + k;
    }
    // (iii) this block's share of the cross product
    const uint32_t j0 = (uint32_t)((uint64_t)jp * h / J), j1 = (uint32_t)((uint64_t)(jp + 1) * h / J);
    for (uint32_t s = 0; s < S; ++s) {
      const uint32_t side = S == 2 ? s : side0;
      sc c = sc_zero();
      for (uint32_t j = j0 + tid; j < j1; j += nt)
        c = sc_add(c, side == 0 ? sc_mont(cur_ab(false, j), cur_ab(true, j + h))
                                : sc_mont(cur_ab(false, j + h), cur_ab(true, j)));
      c = sc_wave_sum(c);
      if ((tid & 63u) == 0) sc_store(redl + 8 * (s * nwv + (tid >> 6)), c);
    }
    __syncthreads();
    if (tid < S * VQ) {  // (QP: the same scalar in each of the V virtual terms)
      const uint32_t s = tid / VQ, v = tid - s * VQ;
      sc t = sc_zero();
      for (uint32_t wv = 0; wv < nwv; ++wv) t = sc_add(t, sc_load(redl + 8 * (s * nwv + wv)));
      const sc cq = sc_mont(t, sc_load(qmul + 8 * inst));
      sc_store(tsl + 8 * (s * CS + cnt + v), halve ? sc_half(cq) : cq);
      tgl[s * CS + cnt + v] = QP ? 0x80000000u | v : qidx;
    }
    __syncthreads();
    const uint32_t ns = nt / S, ls = tid / ns, lt = tid - ls * ns;
    const uint32_t tg = lt / dg.W;
    const DtLane ln = DtLane::make(dg, lt % dg.W);
    const uint32_t* __restrict__ tscs = tsl + 8 * ls * CS;
    const uint32_t* __restrict__ tgens = tgl + ls * CS;
#ifdef EXP_IPA_NOWALK  // timing experiment only (wrong results): no walk, no tree
    if (tid < S) store_p3(out_p3, (S == 2 ? 2 * inst * J + jp : bidx) + tid * J, ge_identity());
    return;
#endif
    // (QP: every slice walks its own share of c Q as the V virtual terms)
    const ge_p3 acc = tg < TG ? dt_walk<QP>(dt, dg, ln, tg, CS, TG,
                                            [&](uint32_t t, uint32_t sv[8], uint32_t& gen) {
                                              const sc v = sc_load(tscs + 8 * t);
                                              _Pragma("unroll") for (int i = 0; i < 8; ++i) sv[i] = v.v[i];
                                              gen = tgens[t];
                                            },
                                            ge_identity(), A.qrow0)
                              : ge_identity();
    __syncthreads();
#ifdef EXP_IPA_NOTREE  // timing experiment only (wrong results): no block tree
    if (lt == 0) store_p3(out_p3, (S == 2 ? 2 * inst * J + jp : bidx) + ls * J, acc);
    return;
#endif
    dt_block_tree_segs(lds, acc, nt, S, out_p3, S == 2 ? 2 * inst * J + jp : bidx, J);
    if (A.done_word) done_signal(A.done_ticket, A.done_word, A.done_tag);
    // (i) this block's share of the next state (the side-0 blocks of S = 1),
    // written after the block's L / R partial and the completion flag: the
    // next round reads it only after this launch has ended, so its loads and
    // multiplies overlap the host's round step instead of preceding it
    if ((fold || init) && (S == 2 || side0 == 0)) {
      const uint32_t q0 = (uint32_t)((uint64_t)jp * 2 * m / J), q1 = (uint32_t)((uint64_t)(jp + 1) * 2 * m / J);
      for (uint32_t q = q0 + tid; q < q1; q += nt) {
        const bool isb = q >= m;
        const uint32_t p = isb ? q - m : q;
        sc_store((isb ? bm_out : am_out) + 8 * (ib + p), cur_ab(isb, p));
      }
      const uint32_t f0 = (uint32_t)((uint64_t)jp * 2 * n / J), f1 = (uint32_t)((uint64_t)(jp + 1) * 2 * n / J);
      for (uint32_t q = f0 + tid; q < f1; q += nt) {
        const bool ish = q >= n;
        const uint32_t k = ish ? q - n : q;
        sc_store((ish ? fH_out : fG_out) + 8 * (ib + k), factor(ish, k));
      }
    }
    return;
  }
  // 1. a, b of this round (length m) into LDS: item q < m is a_q, q >= m is
  // b_{q-m} (one vector per lane, so a fold costs a lane two multiplies, not
  // four, while 2 m <= blockDim)
  for (uint32_t q = tid; q < 2 * m; q += nt) {
    const bool isb = q >= m;
    const uint32_t p = isb ? q - m : q;
    const uint32_t* in = isb ? bm_in : am_in;
    sc x;
    if (fold) {  // G' = u^-1 G_lo + u G_hi: a' = a_lo u + a_hi u^-1, b' = b_lo u^-1 + b_hi u
      x = sc_add(sc_mont(sc_load(in + 8 * (ib + p)), isb ? uim : um),
                 sc_mont(sc_load(in + 8 * (ib + p + m)), isb ? um : uim));
      if (writer) sc_store((isb ? bm_out : am_out) + 8 * (ib + p), x);
    } else if (init) {
      x = sc_to_mont(sc_load((isb ? b0 : a0) + 8 * (ib + p)));
      if (writer) sc_store((isb ? bm_out : am_out) + 8 * (ib + p), x);
    } else {
      x = sc_load(in + 8 * (ib + p));
    }
    sc_store((isb ? sb : sa) + 8 * p, x);
  }
  __syncthreads();
  // 2. term scalars: every k gives one G term and one H term, to side 0 or
  // side 1; item q < n is G_k, q >= n is H_{q-n}
  const uint32_t h = m >> 1;
  for (uint32_t q = tid; q < 2 * n; q += nt) {
    const bool ish = q >= n;
    const uint32_t k = ish ? q - n : q;
    sc f;
    if (init) {
      const uint32_t* r = ish ? hf0 : gf0;
      if (r) {
        f = sc_load(r + 8 * (ib + k));
      } else {
        f = sc_zero();
        f.v[0] = 1;
      }
      if (writer) sc_store((ish ? fH_out : fG_out) + 8 * (ib + k), f);
    } else {
      f = sc_load((ish ? fH_in : fG_in) + 8 * (ib + k));
    }
    if (fold) {
      const bool hi_prev = (k & (2 * m - 1)) & m;
      f = sc_mont(f, hi_prev != ish ? um : uim);
      if (writer) sc_store((ish ? fH_out : fG_out) + 8 * (ib + k), f);
    }
    const uint32_t r = k & (m - 1);
    const bool hi = (r & h) != 0;
    // G_k's term is on side 0 (L) for hi k, H_k's on side 0 for lo k
    const uint32_t side = hi != ish ? 0u : 1u;
    if (S == 2 || side == side0) {
      const uint32_t p = r ^ h;
      const uint32_t cidx = ((k >> (lg_h + 1)) << lg_h) | (k & (h - 1));
      const sc x = sc_mont(sc_load((ish ? sb : sa) + 8 * p), f);
      const uint32_t slot = (S == 2 ? side * NS : 0u) + (ish ? (n >> 1) : 0) + cidx;
      sc_store(tsc + 8 * slot, halve ? sc_half(x) : x);
      tgen[slot] = (ish ? hbase : gbase) + k;
    }
  }
  // c_L = <a_lo, b_hi> (L) or c_R = <a_hi, b_lo> (R), Montgomery form
  for (uint32_t s = 0; s < S; ++s) {
    const uint32_t side = S == 2 ? s : side0;
    sc c = sc_zero();
    for (uint32_t j = tid; j < h; j += nt)
      c = sc_add(c, side == 0 ? sc_mont(sc_load(sa + 8 * j), sc_load(sb + 8 * (j + h)))
                              : sc_mont(sc_load(sa + 8 * (j + h)), sc_load(sb + 8 * j)));
    c = sc_wave_sum(c);
    if ((tid & 63u) == 0) sc_store(red + 8 * (s * nwv + (tid >> 6)), c);
  }
  __syncthreads();
  if (tid < S * VQ) {  // (QP: the same scalar in each of the V virtual terms)
    const uint32_t s = tid / VQ, v = tid - s * VQ;
    sc t = sc_zero();
    for (uint32_t wv = 0; wv < nwv; ++wv) t = sc_add(t, sc_load(red + 8 * (s * nwv + wv)));
    const sc cq = sc_mont(t, sc_load(qmul + 8 * inst));  // Montgomery c * canonical q
    sc_store(tsc + 8 * (s * NS + n + v), halve ? sc_half(cq) : cq);
    tgen[s * NS + n + v] = QP ? 0x80000000u | v : qidx;
  }
  __syncthreads();
  // 3. direct-table walk over the LDS terms, then the block tree (reusing LDS)
  const uint32_t ns = nt / S, ls = tid / ns, lt = tid - ls * ns;  // lanes per side, this lane's side
  const uint32_t tg = lt / dg.W;
  const DtLane ln = DtLane::make(dg, lt % dg.W);
  const uint32_t* __restrict__ tscs = tsc + 8 * ls * NS;
  const uint32_t* __restrict__ tgens = tgen + ls * NS;
#ifdef EXP_IPA_NOWALK  // timing experiment only (wrong results): no walk, no tree
  if (tid < S) store_p3(out_p3, S == 2 ? (2 * inst + tid) * J + jp : bidx, ge_identity());
  return;
#endif
  const uint32_t t0 = (uint32_t)((uint64_t)jp * NS / J), t1 = (uint32_t)((uint64_t)(jp + 1) * NS / J);
  const ge_p3 acc = tg < TG ? dt_walk<QP>(dt, dg, ln, t0 + tg, t1, TG,
                                          [&](uint32_t t, uint32_t s[8], uint32_t& gen) {
                                            const sc v = sc_load(tscs + 8 * t);
                                            _Pragma("unroll") for (int i = 0; i < 8; ++i) s[i] = v.v[i];
                                            gen = tgens[t];
                                          },
                                          ge_identity(), A.qrow0)
                            : ge_identity();
  __syncthreads();
#ifdef EXP_IPA_NOTREE  // timing experiment only (wrong results): no block tree
  if (lt == 0) store_p3(out_p3, S == 2 ? (2 * inst + ls) * J + jp : bidx, acc);
  return;
#endif
  // result of side s: out_p3[(2 inst + s) J + jp] (= bidx for S = 1)
  dt_block_tree_segs(lds, acc, nt, S, out_p3, S == 2 ? 2 * inst * J + jp : bidx, J);
  if (A.done_word) done_signal(A.done_ticket, A.done_word, A.done_tag);
}

template <bool QP>
__global__ void __launch_bounds__(DT_NT_MAX) k_ipa_round_dt(
    const uint32_t* __restrict__ dt, DtGeom dg, uint32_t n, uint32_t m, uint32_t lg_h, uint32_t fold,
    const uint32_t* __restrict__ am_in, const uint32_t* __restrict__ bm_in, const uint32_t* __restrict__ fG_in,
    const uint32_t* __restrict__ fH_in, uint32_t* __restrict__ am_out, uint32_t* __restrict__ bm_out,
    uint32_t* __restrict__ fG_out, uint32_t* __restrict__ fH_out, const uint32_t* __restrict__ u,
    const uint32_t* __restrict__ qmul, uint32_t gbase, uint32_t hbase, uint32_t qidx, uint32_t TG, uint32_t halve,
    uint32_t* __restrict__ out_p3, const uint32_t* __restrict__ a0, const uint32_t* __restrict__ b0,
    const uint32_t* __restrict__ gf0, const uint32_t* __restrict__ hf0, uint32_t init, uint32_t J, uint32_t S,
    const uint32_t* __restrict__ qpow, uint32_t* done_ticket, uint32_t* done_word, uint32_t done_tag,
    uint32_t u1, IpaU1 u1w) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  IpaRoundArgs A;
  A.am_in = am_in; A.bm_in = bm_in; A.fG_in = fG_in; A.fH_in = fH_in;
  A.am_out = am_out; A.bm_out = bm_out; A.fG_out = fG_out; A.fH_out = fH_out;
  A.u = u; A.qmul = qmul; A.out_p3 = out_p3;
  A.a0 = a0; A.b0 = b0; A.gf0 = gf0; A.hf0 = hf0;
  A.m = m; A.lg_h = lg_h; A.fold = fold; A.init = init; A.halve = halve;
  A.gbase = gbase; A.hbase = hbase; A.qidx = qidx;
  A.split = J;
  A.qpow = qpow;
  A.qrow0 = qpow ? (uint32_t)((size_t)(qpow - dt) / MSM_NIELS_WORDS) : 0u;  // (qpow lies inside dt)
  A.done_ticket = done_ticket;
  A.done_word = done_word;
  A.done_tag = done_tag;
  A.u1 = u1;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    A.u1m.v[i] = u1w.w[i];
    A.u1im.v[i] = u1w.w[8 + i];
  }
  ipa_round_body<QP>(dt, dg, n, TG, A, blockIdx.x, lds, S);
}

// Several batches' rounds in one launch (BPP_IPA_MERGE, the shared-launch
// round scheduler below): block b runs block b - prefix of batch j.  args:
// nargs structs in pinned host memory, read once per block into LDS.
#define IPA_MERGE_MAX 16
__global__ void __launch_bounds__(DT_NT_MAX) k_ipa_round_dt_multi(const uint32_t* __restrict__ dt, DtGeom dg,
                                                                 uint32_t n, uint32_t TG,
                                                                 const IpaRoundArgs* __restrict__ args,
                                                                 uint32_t nargs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ IpaRoundArgs sA;
  __shared__ uint32_t sb;
  if (threadIdx.x == 0) {
    uint32_t b = blockIdx.x, j = 0;
    while (j + 1 < nargs && b >= args[j].blocks) b -= args[j++].blocks;
    sA = args[j];
    sb = b;
  }
  __syncthreads();
  ipa_round_body<false>(dt, dg, n, TG, sA, sb, lds, 1);  // (the merged launches never carry qpow)
}

// The shared-launch round scheduler (BPP_IPA_MERGE=1; an
// A/B switch): the batches in flight on one device hand their fused IPA
// rounds to one merger, which issues ONE k_ipa_round_dt_multi over every
// round pending at the time on its own stream, after each batch's stream has
// reached the round (an event per request).  Combining: the first thread to
// arrive leads -- it waits BPP_IPA_MERGE_US (default 0) for others, takes
// every pending request with the same shape (n, TG, tables), launches, and
// wakes them; each then waits for the launch's event.  A batch's round thus
// runs as part of a larger grid (more waves per SIMD for the latency-bound
// walk and tree) instead of on its own queue beside the others.
namespace {
struct IpaMergeReq {
  IpaRoundArgs a;
  hipEvent_t ready = nullptr;  // recorded on the batch's stream
  const uint32_t* dt = nullptr;
  DtGeom dg;
  uint32_t n = 0, TG = 0, nt = 0;
  size_t lds = 0;
  uint64_t gen = 0;            // set when launched
  hipEvent_t done = nullptr;   // the launch's completion
  int err = BPP_OK;
};
struct IpaMerger {
  std::mutex mu;
  std::condition_variable cv;
  bool leading = false;
  uint64_t gen = 0;
  std::vector<IpaMergeReq*> pending;
  hipStream_t stream = nullptr;
  static constexpr int RING = 64;
  IpaRoundArgs* ring = nullptr;  // pinned: RING x IPA_MERGE_MAX argument blocks
  hipEvent_t ring_ev[RING] = {};
  bool ring_used[RING] = {};
  int ring_pos = 0;
  uint64_t launches = 0, rounds = 0;
};
IpaMerger& ipa_merger(int dev) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<IpaMerger>> all;
  std::lock_guard<std::mutex> g(mu);
  auto& p = all[dev];
  if (!p) p.reset(new IpaMerger);
  return *p;
}
bool same_shape(const IpaMergeReq& a, const IpaMergeReq& b) {
  return a.dt == b.dt && a.n == b.n && a.TG == b.TG && a.nt == b.nt && a.dg.c == b.dg.c;
}
// the leader's launch of `reqs` (same shape); sets their gen / done
int merger_launch(bpp_ctx* ctx, IpaMerger& M, std::vector<IpaMergeReq*>& reqs) {
  if (!M.stream) BPP_HIP(hipStreamCreateWithFlags(&M.stream, hipStreamNonBlocking));
  if (!M.ring) BPP_HIP(hipHostMalloc((void**)&M.ring, sizeof(IpaRoundArgs) * IPA_MERGE_MAX * IpaMerger::RING));
  const int slot = M.ring_pos;
  M.ring_pos = (M.ring_pos + 1) % IpaMerger::RING;
  if (!M.ring_ev[slot]) BPP_HIP(hipEventCreateWithFlags(&M.ring_ev[slot], hipEventDisableTiming));
  if (M.ring_used[slot]) BPP_HIP(hipEventSynchronize(M.ring_ev[slot]));  // (its last launch has read the slot)
  IpaRoundArgs* args = M.ring + (size_t)slot * IPA_MERGE_MAX;
  uint32_t blocks = 0;
  for (size_t i = 0; i < reqs.size(); ++i) {
    args[i] = reqs[i]->a;
    blocks += reqs[i]->a.blocks;
    BPP_HIP(hipStreamWaitEvent(M.stream, reqs[i]->ready, 0));
  }
  const IpaMergeReq& r0 = *reqs[0];
  hipLaunchKernelGGL(k_ipa_round_dt_multi, dim3(blocks), dim3(r0.nt), r0.lds, M.stream, r0.dt, r0.dg, r0.n, r0.TG,
                     (const IpaRoundArgs*)args, (uint32_t)reqs.size());
  BPP_HIP(hipGetLastError());
  BPP_HIP(hipEventRecord(M.ring_ev[slot], M.stream));
  M.ring_used[slot] = true;
  ++M.launches;
  M.rounds += reqs.size();
  for (IpaMergeReq* r : reqs) r->done = M.ring_ev[slot];
  return BPP_OK;
}
// Blocks until the request's round has been launched; returns the event to
// wait for (or an error).
int merger_submit(bpp_ctx* ctx, IpaMergeReq& req) {
  IpaMerger& M = ipa_merger(ctx->device);
  static const int wait_us = [] {
    const char* e = getenv("BPP_IPA_MERGE_US");
    return e ? std::max(0, atoi(e)) : 0;
  }();
  std::unique_lock<std::mutex> lk(M.mu);
  M.pending.push_back(&req);
  for (;;) {
    if (req.gen) return req.err;
    if (!M.leading) break;
    M.cv.wait(lk);
  }
  // lead: gather, launch every pending request of this shape, wake them
  M.leading = true;
  if (wait_us > 0) {
    lk.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(wait_us));
    lk.lock();
  }
  std::vector<IpaMergeReq*> take{&req}, keep;  // (the leader's own request first)
  for (IpaMergeReq* r : M.pending)
    if (r != &req) (same_shape(*r, req) && take.size() < IPA_MERGE_MAX ? take : keep).push_back(r);
  M.pending.swap(keep);
  lk.unlock();
  const int rc = merger_launch(ctx, M, take);
  lk.lock();
  const uint64_t g = ++M.gen;
  for (IpaMergeReq* r : take) {
    r->gen = g;
    r->err = rc;
  }
  M.leading = false;
  M.cv.notify_all();
  return req.err;
}
}  // namespace

// LDS words of k_ipa_round_dt: terms + indices + a, b + wave partials, or
// the block tree, whichever is larger
static size_t ipa_round_lds_words(uint32_t n, uint32_t nt, uint32_t S = 1, uint32_t vq = 1) {
  const size_t NS = (size_t)S * (n + vq);  // (vq: the Q term's slots, ipa_round_body VQ)
  const size_t prologue = 8 * NS + ((NS + 3) & ~(size_t)3) + 16 * (size_t)n + 8 * (size_t)S * ((nt + 63) / 64);
  return std::max(prologue, (size_t)nt * P3_WORDS);
}

static sc to_dev_sc(const hsc::Sc& x) {
  sc r;
  for (int i = 0; i < 4; ++i) {
    r.v[2 * i] = (uint32_t)x.v[i];
    r.v[2 * i + 1] = (uint32_t)(x.v[i] >> 32);
  }
  return r;
}

static int ipa_hook_failed(bpp_ctx* ctx) {
  ctx->err = "ipa: a transcript hook returned an error";
  return BPP_ERR_CALLBACK;
}

static hsc::Sc from_dev_words(const uint32_t w[8]) {
  hsc::Sc r;
  for (int i = 0; i < 4; ++i) r.v[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  return r;
}

int ipa_prove_batch_dev(bpp_ctx* ctx, const std::vector<merlin::Transcript*>& trs, const IpaGens& g, uint32_t n,
                        const uint32_t* d_Gf, const uint32_t* d_Hf, const uint32_t* d_a, const uint32_t* d_b,
                        const std::vector<hsc::Sc>& qmul, std::vector<IpaProofHost>& out,
                        IpaTranscript* one) {
  const uint32_t P = one ? 1u : (uint32_t)trs.size();
  if (n == 0 || (n & (n - 1))) {
    ctx->err = "ipa: n must be a power of two";
    return BPP_ERR_LEN;
  }
  if (qmul.size() != P) return BPP_ERR_ARG;
  out.resize(P);  // (callers may pass vectors back for reuse: keep their capacity)
  for (auto& o : out) {
    o.L.clear();
    o.R.clear();
  }
  if (!P) return BPP_OK;
  uint32_t lg_n = 0;
  while ((1u << lg_n) < n) ++lg_n;
  if (one) {
    if (!one->domain_sep(n)) return ipa_hook_failed(ctx);
  } else {
    par::for_each(P, [&](size_t p) { trs[p]->innerproduct_domain_sep(n); });
  }
  const size_t PN = (size_t)P * n, PT = (size_t)P * (2 * n + 2);
  void *am, *bm, *fG, *fH, *scal, *pidx, *part, *d_q, *d_u;
  BPP_TRY(ctx_ws(ctx, "ipa_am", PN * 32, &am));
  BPP_TRY(ctx_ws(ctx, "ipa_bm", PN * 32, &bm));
  BPP_TRY(ctx_ws(ctx, "ipa_fG", PN * 32, &fG));
  BPP_TRY(ctx_ws(ctx, "ipa_fH", PN * 32, &fH));
  BPP_TRY(ctx_ws(ctx, "ipa_scal", PT * 32, &scal));
  BPP_TRY(ctx_ws(ctx, "ipa_pidx", PT * 4, &pidx));

  BPP_TRY(ctx_ws(ctx, "ipa_u", (size_t)P * 64, &d_u));
  // cross blocks per instance: enough lanes overall, at most 64
  const uint32_t cross_blocks =
      std::max<uint32_t>(1, std::min<uint32_t>({64u, grid_for(std::max<uint32_t>(n / 2, 1), CROSS_T),
                                                 std::max<uint32_t>(1, 512 / P)}));
  // cross products fused into k_ipa_terms (one partial per wave) when every
  // wave lies in one instance; k_ipa_cross otherwise
  const bool fuse_cross = n >= 64;
  BPP_TRY(ctx_ws(ctx, "ipa_part", (size_t)P * std::max<uint32_t>(cross_blocks, n / 64) * 64, &part));
  {
    std::vector<uint32_t> qw((size_t)P * 8);
    for (uint32_t p = 0; p < P; ++p) {
      const sc q = to_dev_sc(qmul[p]);
      memcpy(&qw[8 * (size_t)p], q.v, 32);
    }
    uint32_t* hq = nullptr;  // read in place from pinned host memory (ctx_zc_in)
    BPP_TRY(ctx_zc_in(ctx, "ipa_qmul_h", qw.data(), qw.size() * 4, &hq));
    d_q = hq;
  }
  std::vector<uint32_t> off(2 * (size_t)P + 1);
  for (uint32_t p = 0; p < P; ++p) {
    off[2 * p] = (uint32_t)(p * (2 * (size_t)n + 2));
    off[2 * p + 1] = off[2 * p] + n + 1;
  }
  off[2 * P] = (uint32_t)PT;
  std::vector<uint8_t> enc((size_t)2 * P * 32);
  std::vector<hsc::Sc> u(P), ui(P);
  std::vector<uint32_t> uw((size_t)P * 16);
  // One launch per round (k_ipa_round_dt) when the generators have direct
  // tables: the state (a, b, fG, fH) alternates between two sets so that a
  // round's blocks read the previous state while side 0 writes the next.
  const bool fused = n >= 2 && n <= IPA_FUSED_NMAX && !g.pts.tbl1 && msm_use_dt(g.pts, 2 * P, (uint32_t)PT);
  if (g.qpow && !fused) {  // (only the fused rounds add Q by its doublings)
    ctx->err = "ipa: Q as doublings needs the fused direct-table rounds";
    return BPP_ERR_ARG;
  }
  if (!fused) {  // (the fused first round converts the inputs itself)
    hipLaunchKernelGGL(k_ipa_init, dim3(grid_for(PN, 256)), dim3(256), 0, ctx->stream, n, P, d_a, d_b, d_Gf, d_Hf,
                       (uint32_t*)am, (uint32_t*)bm, (uint32_t*)fG, (uint32_t*)fH);
    BPP_TRY(ctx_check_launch(ctx, "k_ipa_init"));
  }
  uint32_t* S[2][4] = {{(uint32_t*)am, (uint32_t*)bm, (uint32_t*)fG, (uint32_t*)fH}, {nullptr, nullptr, nullptr, nullptr}};
  void* d_res = nullptr;
  DtGeom dg;
  uint32_t TG = 1, nt = 1;
  if (fused) {
    static const char* names[4] = {"ipa_am1", "ipa_bm1", "ipa_fG1", "ipa_fH1"};
    for (int i = 0; i < 4; ++i) {
      void* d = nullptr;
      BPP_TRY(ctx_ws(ctx, names[i], PN * 32, &d));
      S[1][i] = (uint32_t*)d;
    }
    BPP_TRY(ctx_ws(ctx, "ipa_res", (size_t)2 * P * P3_BYTES, &d_res));
    dg = dt_geom(g.pts.dt_c);
    TG = dt_term_groups(dg.W, (double)(n + 1), 2 * P);  // as msm_multi_dt_dev for (n + 1)-term MSMs
    static const int tg_env = [] {  // term groups per side (A/B switch)
      const char* e = getenv("BPP_IPA_TG");
      return e ? atoi(e) : 0;
    }();
    if (tg_env >= 1 && (uint32_t)tg_env * dg.W <= DT_NT_MAX) TG = (uint32_t)tg_env;
    nt = TG * dg.W;
  }
  // Both sides of an instance in one block (ipa_round_body S = 2) for batches
  // that fill the device with blocks anyway; BPP_IPA_LR=0 keeps one side per
  // block (A/B switch)
  static const bool lr_env = [] {
    const char* e = getenv("BPP_IPA_LR");
    return !e || atoi(e) != 0;
  }();
  uint32_t sides = 1;
  if (fused && lr_env && P >= 128 && 2 * nt <= DT_NT_MAX && ipa_round_lds_words(n, 2 * nt, 2) * 4 <= 65536) sides = 2;
  // Device transcript path (an A/B experiment: see
  // DESIGN.md): the rounds run back to back on the stream -- fused MSM,
  // k_compress_p3 of L and R, k_ipa_transcript_step (Merlin + u^-1) --
  // with no host round trip; L, R and the transcripts come back at the end.
  const char* dm_env = getenv("BPP_IPA_DEVICE_MERLIN");
  const bool dev_merlin = fused && !one && dm_env && atoi(dm_env) != 0;
  // Host round trip of the fused rounds without copy launches: the round
  // kernel writes L/2, R/2 straight into pinned host memory and reads the
  // challenges u, u^-1 from it (ctx_host_buf), where a device result buffer
  // and a staged upload cost a copy launch each way per round.
#ifdef EXP_IPA_NOZC
  const bool zc = false;
#else
  const bool zc = fused && !dev_merlin;
#endif
  // the shared-launch round scheduler (A/B switch, off by default)
  static const bool merge_env = [] {
    const char* e = getenv("BPP_IPA_MERGE");
    return e && atoi(e) != 0;
  }();
  const bool merge = merge_env && zc && !g.qpow;
  // J blocks per L / R MSM when the batch is small (config 2: P = 1, two
  // blocks of one wave per SIMD walking ~64 of the 1025 terms per lane in a
  // row): each block walks a slice of the terms and the host adds the J
  // partials before it encodes (zero-copy path only; BPP_IPA_SPLIT overrides).
  // Since each block folds only its own slice (IPA_SPLIT_PROLOGUE) a slice
  // may be as short as one term per lane group: config 2 J = 16 1.10-1.13 ms,
  // 32 1.06, 64 1.10 (profiles/r06_ipa_jsweep.txt)
  uint32_t J = 1;
  if (zc && nt) {
    static const int split_env = [] {
      const char* e = getenv("BPP_IPA_SPLIT");
      return e ? atoi(e) : -1;
    }();
    if (split_env >= 1) {
      J = (uint32_t)split_env;
    } else if (split_env < 0) {
#ifndef IPA_J_MAX
#define IPA_J_MAX 32
#endif
#ifndef IPA_J_SLICE_TG
#define IPA_J_SLICE_TG (IPA_SPLIT_PROLOGUE ? 1 : 2)
#endif
      const uint32_t per_slice = IPA_J_SLICE_TG * TG;
      while (J < IPA_J_MAX && 2 * P * (2 * J) <= 512 && (n + 1) / (2 * J) >= per_slice) J *= 2;
    }
  }
  // the J partials of each L / R summed on the device (k_ipa_jsum, one
  // block per MSM, a 5-level tree for J = 32) rather than by 2 (J - 1) host
  // additions between the rounds: an A/B switch, off (BPP_IPA_JSUM=1 on).
  // Config 2 measured 1.10-1.11 ms with it against 1.03-1.04 without: the
  // host's 62 additions take ~6.5 us a round, the extra launch and its tree
  // ~13 us of the round's wait (profiles/r06_ipa_jsum_ab.txt)
  static const bool jsum_env = [] {
    const char* e = getenv("BPP_IPA_JSUM");
    return e && atoi(e) != 0;
  }();
  const bool dev_jsum = zc && !merge && J > 1 && J <= 64 && (J & (J - 1)) == 0 && jsum_env;
  void* d_part = nullptr;  // dev_jsum: the round kernel's J partials per MSM
  // one IPA alone (bpp_ipa_prove: P = 1 on a spinning context) waits for
  // each round through the kernel's completion flag instead of an event
  // (ctx_wait_flag; BPP_IPA_FLAG=0 off): config 2 0.92-0.95 vs 0.96-0.99 ms.
  // Not for prover batches: with 8 sub-batches in flight the busy flag
  // waits cost the config-4 job 7.5-9.1 vs 7.0-7.2 ms (r06_ipa_flag_ab.txt)
  static const bool flag_env = [] {
    const char* e = getenv("BPP_IPA_FLAG");
    return !e || atoi(e) != 0;
  }();
  const bool use_flag = zc && !merge && !dev_jsum && P == 1 && ctx->sync_spin_us > 0 && flag_env;
  uint32_t *done_ticket = nullptr, *done_word = nullptr, done_tag = 0;
  uint32_t* h_uw = nullptr;  // zc: the challenges' device words, in place
  if (zc) {
    void *hr = nullptr, *hu = nullptr;
    BPP_TRY(ctx_host_buf(ctx, "ipa_res_h", (size_t)2 * P * (dev_jsum ? 1 : J) * P3_BYTES, &hr));
    BPP_TRY(ctx_host_buf(ctx, "ipa_u_h", (size_t)P * 64, &hu));
    d_res = hr;
    d_u = hu;
    h_uw = (uint32_t*)hu;
    if (dev_jsum) BPP_TRY(ctx_ws(ctx, "ipa_part", (size_t)2 * P * J * P3_BYTES, &d_part));
  }
  void *d_states = nullptr, *d_lr = nullptr;
  if (dev_merlin) {
    std::vector<uint8_t> stt((size_t)P * MERLIN_DEV_STATE_BYTES);
    for (uint32_t p = 0; p < P; ++p) merlin_state_export(*trs[p], &stt[(size_t)p * MERLIN_DEV_STATE_BYTES]);
    BPP_TRY(ctx_ws(ctx, "ipa_mstate", stt.size(), &d_states));
    BPP_TRY(ctx_h2d(ctx, d_states, stt.data(), stt.size()));
    BPP_TRY(ctx_ws(ctx, "ipa_lr", (size_t)lg_n * P * 64, &d_lr));
  }
  uint32_t* ab_host = nullptr;  // k_ipa_final's output (fused path)
  int cur = 0;  // set holding the state at the start of a round (before its fold)
  uint32_t m = n, round = 0;
  uint32_t lg_h = lg_n ? lg_n - 1 : 0;  // log2(m/2)
  while (m > 1) {
    const uint32_t h = m >> 1;
    if (fused) {
      const int in = cur, outs = cur ^ 1;
      if (merge) {  // one launch with the other batches' pending rounds (the merger's stream)
        static thread_local hipEvent_t ready = nullptr;
        if (!ready) BPP_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        IpaMergeReq req;
        IpaRoundArgs& A = req.a;
        A.am_in = S[in][0]; A.bm_in = S[in][1]; A.fG_in = S[in][2]; A.fH_in = S[in][3];
        A.am_out = S[round ? outs : in][0]; A.bm_out = S[round ? outs : in][1];
        A.fG_out = S[round ? outs : in][2]; A.fH_out = S[round ? outs : in][3];
        A.u = (const uint32_t*)d_u; A.qmul = (const uint32_t*)d_q; A.out_p3 = (uint32_t*)d_res;
        A.a0 = d_a; A.b0 = d_b; A.gf0 = d_Gf; A.hf0 = d_Hf;
        A.m = m; A.lg_h = lg_h; A.fold = round ? 1u : 0u; A.init = round ? 0u : 1u; A.halve = 1u;
        A.gbase = g.gbase; A.hbase = g.hbase; A.qidx = g.qidx;
        A.blocks = 2 * P * J;
        A.split = J;
        A.qpow = g.qpow;
        A.qrow0 = 0;  // (merged launches never carry qpow: merge is off with it)
        A.done_ticket = A.done_word = nullptr;
        A.done_tag = 0;
        A.u1 = 0;
        req.dt = g.pts.dt;
        req.dg = dg;
        req.n = n;
        req.TG = TG;
        req.nt = nt;
        req.lds = ipa_round_lds_words(n, nt) * 4;
        BPP_HIP(hipEventRecord(ready, ctx->stream));
        req.ready = ready;
        BPP_TRY(merger_submit(ctx, req));
        BPP_HIP(hipStreamWaitEvent(ctx->stream, req.done, 0));  // (ctx_sync below then covers the round)
      } else {
        ProfScope ps(ctx, "ipa_round_dt");  // (bench.py: this kernel's own roofline)
        if (use_flag) BPP_TRY(ctx_done_flag(ctx, &done_ticket, &done_word, &done_tag));
        // one instance: its u words as kernel arguments (the host wrote them
        // after the last round; BPP_IPA_U_ARG=0: read in place).  Config 2
        // best of four 0.795 vs 0.804 ms, within the run-to-run noise
        // (r06_ipa_uarg_ab.txt)
        static const bool u1_env = [] {
          const char* e = getenv("BPP_IPA_U_ARG");
          return !e || atoi(e) != 0;
        }();
        const bool u1 = P == 1 && zc && round > 0 && u1_env;
        IpaU1 u1w{};
        if (u1) memcpy(u1w.w, h_uw, sizeof u1w.w);
        hipLaunchKernelGGL(g.qpow ? k_ipa_round_dt<true> : k_ipa_round_dt<false>, dim3(2 / sides * P * J),
                           dim3(sides * nt),
                           ipa_round_lds_words(n, sides * nt, sides, g.qpow ? (253u + dg.W - 1) / dg.W : 1u) * 4,
                           ctx->stream,
                           g.pts.dt, dg, n, m, lg_h, round ? 1u : 0u, S[in][0], S[in][1], S[in][2], S[in][3],
                           S[round ? outs : in][0], S[round ? outs : in][1], S[round ? outs : in][2],
                           S[round ? outs : in][3], (const uint32_t*)d_u, (const uint32_t*)d_q, g.gbase, g.hbase,
                           g.qidx, TG, dev_merlin ? 0u : 1u, (uint32_t*)(dev_jsum ? d_part : d_res), d_a, d_b,
                           d_Gf, d_Hf, round ? 0u : 1u, J, sides, g.qpow, done_ticket,
                           use_flag ? done_word : nullptr, done_tag, u1 ? 1u : 0u, u1w);
        if (dev_jsum)
          hipLaunchKernelGGL(k_ipa_jsum, dim3(2 * P), dim3(J), (size_t)J * P3_BYTES, ctx->stream,
                             (const uint32_t*)d_part, J, (uint32_t*)d_res);
      }
      BPP_TRY(ctx_check_launch(ctx, "k_ipa_round_dt"));
      if (round) cur = outs;
      const uint64_t terms = (uint64_t)2 * P * (n + 1);
      ctx_work(ctx, "msm_terms", terms);
      ctx_work(ctx, "madds", terms * dg.W);
      ctx_work(ctx, "padds", (uint64_t)2 * P * J * (nt - 1));
      ctx_work(ctx, "msm_launches", 1);
      ctx_work(ctx, "dt_terms", terms);
      ctx_work(ctx, "dt_madds", terms * dg.W);
      ctx_work(ctx, "dt_launches", 1);
      ctx_work(ctx, "ipa_dt_terms", terms);  // k_ipa_round_dt's share of the dt_* totals
      ctx_work(ctx, "ipa_dt_madds", terms * dg.W);
      ctx_work(ctx, "ipa_dt_launches", 1);
      if (dev_merlin) {
        uint8_t* lr = (uint8_t*)d_lr + (size_t)round * P * 64;
        BPP_TRY(points_compress_p3_dev(ctx, (const uint32_t*)d_res, 2 * (size_t)P, lr));
        BPP_TRY(ipa_transcript_step_dev(ctx, P, (uint8_t*)d_states, lr, (uint32_t*)d_u));
      } else if (zc) {
        HostScope hs(ctx, "ipa_msm");
        {
          HostScope hw(ctx, "ipa_wait");
          // the kernel's L/2, R/2 are in host memory now
          if (use_flag && !merge)
            BPP_TRY(ctx_wait_flag(ctx, done_word, done_tag));
          else
            BPP_TRY(ctx_sync(ctx));
        }
        BPP_TRY(points_double_encode_host(ctx, (const uint32_t*)d_res, 2 * (size_t)P, enc.data(), dev_jsum ? 1 : J));
      } else {
        HostScope hs(ctx, "ipa_msm");
        BPP_TRY(points_double_encode_p3(ctx, (const uint32_t*)d_res, 2 * (size_t)P, enc.data()));
      }
    } else {
      {
        ProfScope ps(ctx, "ipa_terms");
        hipLaunchKernelGGL(k_ipa_terms, dim3(grid_for(PN, 256)), dim3(256), 0, ctx->stream, n, lg_n, P, m, lg_h,
                           (const uint32_t*)am, (const uint32_t*)bm, (const uint32_t*)fG, (const uint32_t*)fH,
                           g.gbase, g.hbase, (uint32_t*)scal, (uint32_t*)pidx, fuse_cross ? (uint32_t*)part : nullptr);
        uint32_t nb = n / 64;  // partials per instance (fused: one per wave)
        if (!fuse_cross) {
          nb = std::min<uint32_t>(cross_blocks, grid_for(h, CROSS_T));
          hipLaunchKernelGGL(k_ipa_cross, dim3(nb, P), dim3(CROSS_T), 0, ctx->stream, n, h, (const uint32_t*)am,
                             (const uint32_t*)bm, (uint32_t*)part);
        }
        hipLaunchKernelGGL(k_ipa_cross_final, dim3(grid_for(P, 64)), dim3(64), 0, ctx->stream, nb, P,
                           (const uint32_t*)part, (const uint32_t*)d_q, g.qidx, n, (uint32_t*)scal, (uint32_t*)pidx);
      }
      BPP_TRY(ctx_check_launch(ctx, "ipa round kernels"));
      HostScope hs(ctx, "ipa_msm");
      // L/2, R/2 from the halved term scalars (k_ipa_terms, k_ipa_cross_final),
      // encoded as L, R (msm_multi_enc)
      BPP_TRY(msm_multi_enc(ctx, (const uint32_t*)scal, (const uint32_t*)pidx, off, g.pts, enc.data(), true));
    }
    if (!dev_merlin) {
    HostScope hs(ctx, "ipa_host");
    if (one) {  // the caller's transcript (bpp_ipa_prove_cb), one instance
      if (!one->append("L", enc.data(), 32) || !one->append("R", enc.data() + 32, 32) ||
          !one->challenge_scalar("u", u[0]))
        return ipa_hook_failed(ctx);
    } else
    // L, R appends and the u challenge of eight proofs at a time on the
    // 8-way Keccak (their transcripts are in lockstep)
    merlin::lockstep_x8(
        trs, [](size_t n, const std::function<void(size_t)>& f) { par::for_each(n, f); },
        [&](merlin::TranscriptX8& X, const size_t* idx, size_t real) {
          const uint8_t *lm[8], *rm[8];
          for (int j = 0; j < 8; ++j) {
            lm[j] = enc.data() + 64 * idx[j];
            rm[j] = lm[j] + 32;
          }
          X.append("L", lm, 32);
          X.append("R", rm, 32);
          hsc::Sc u8[8];
          X.challenge_scalar("u", u8);
          for (size_t j = 0; j < real; ++j) u[idx[j]] = u8[j];
        },
        [&](size_t p) {
          trs[p]->append_point("L", enc.data() + 64 * p);
          trs[p]->append_point("R", enc.data() + 64 * p + 32);
          u[p] = trs[p]->challenge_scalar("u");
        });
    for (uint32_t p = 0; p < P; ++p) {
      Enc32 Le, Re;
      memcpy(Le.data(), enc.data() + 64 * p, 32);
      memcpy(Re.data(), enc.data() + 64 * p + 32, 32);
      out[p].L.push_back(Le);
      out[p].R.push_back(Re);
    }
    ui = u;
    {
      HostScope hi(ctx, "ipa_uinv");
      hsc::batch_invert(ui, false, true);  // (u: public challenges)
    }
    uint32_t* uwp = zc ? h_uw : uw.data();  // (zc: the device reads them in place)
    for (uint32_t p = 0; p < P; ++p) {  // device Montgomery forms u R, u^-1 R
      const sc um = to_dev_sc(hsc::to_mont(u[p]));
      const sc uim = to_dev_sc(hsc::to_mont(ui[p]));
      memcpy(&uwp[16 * (size_t)p], um.v, 32);
      memcpy(&uwp[16 * (size_t)p + 8], uim.v, 32);
    }
    if (!zc) BPP_TRY(ctx_h2d(ctx, d_u, uw.data(), uw.size() * 4));
    }
    // the fused rounds fold inside the next round's launch; the last
    // challenge (and every challenge of the unfused path) is folded here
    if (fused && h == 1 && n >= 2) {  // (the proof needs element 0 only)
      uint32_t* hab = nullptr;
      BPP_TRY(ctx_zc_out(ctx, "ipa_ab_h", (size_t)P * 64, &hab));
      hipLaunchKernelGGL(k_ipa_final, dim3(grid_for(P, 64)), dim3(64), 0, ctx->stream, P, n, S[cur][0], S[cur][1],
                         (const uint32_t*)d_u, hab);
      ab_host = hab;
    } else if (!fused || h == 1) {
      uint32_t** st = S[cur];
      ProfScope ps(ctx, "ipa_fold");
      hipLaunchKernelGGL(k_ipa_fold, dim3(grid_for(PN, 256)), dim3(256), 0, ctx->stream, n, lg_n, P, m, st[0], st[1],
                         st[2], st[3], (const uint32_t*)d_u);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_ipa_fold"));
    m = h;
    ++round;
    if (lg_h) --lg_h;
  }
  am = S[cur][0];
  bm = S[cur][1];
  if (dev_merlin) {  // L, R of every round and the transcripts back to the host
    std::vector<uint8_t> lr((size_t)lg_n * P * 64), stt((size_t)P * MERLIN_DEV_STATE_BYTES);
    BPP_TRY(ctx_d2h(ctx, lr.data(), d_lr, lr.size()));
    BPP_TRY(ctx_d2h(ctx, stt.data(), d_states, stt.size()));
    for (uint32_t p = 0; p < P; ++p) {
      merlin_state_import(*trs[p], &stt[(size_t)p * MERLIN_DEV_STATE_BYTES]);
      for (uint32_t j = 0; j < lg_n; ++j) {
        Enc32 Le, Re;
        memcpy(Le.data(), &lr[((size_t)j * P + p) * 64], 32);
        memcpy(Re.data(), &lr[((size_t)j * P + p) * 64 + 32], 32);
        out[p].L.push_back(Le);
        out[p].R.push_back(Re);
      }
    }
  }
  // a, b = element 0 of each instance
  std::vector<uint32_t> ab((size_t)P * 16);
  if (ab_host) {  // k_ipa_final wrote them into host memory
    BPP_TRY(ctx_sync(ctx));
    memcpy(ab.data(), ab_host, ab.size() * 4);
  } else {
    void* h = nullptr;
    BPP_TRY(ctx_pinned(ctx, ab.size() * 4, &h));
    BPP_HIP(hipMemcpy2DAsync(h, 64, am, (size_t)n * 32, 32, P, hipMemcpyDeviceToHost, ctx->stream));
    BPP_HIP(hipMemcpy2DAsync((uint8_t*)h + 32, 64, bm, (size_t)n * 32, 32, P, hipMemcpyDeviceToHost, ctx->stream));
    BPP_TRY(ctx_sync(ctx));
    memcpy(ab.data(), h, ab.size() * 4);
  }
  for (uint32_t p = 0; p < P; ++p) {
    out[p].a = hsc::mont(from_dev_words(&ab[16 * (size_t)p]), hsc::one());
    out[p].b = hsc::mont(from_dev_words(&ab[16 * (size_t)p + 8]), hsc::one());
  }
  return BPP_OK;
}

int ipa_prove_dev(bpp_ctx* ctx, IpaTranscript& tr, const IpaGens& g, uint32_t n, const uint32_t* d_Gf,
                  const uint32_t* d_Hf, const uint32_t* d_a, const uint32_t* d_b, IpaProofHost& out) {
  std::vector<IpaProofHost> o;
  BPP_TRY(ipa_prove_batch_dev(ctx, {}, g, n, d_Gf, d_Hf, d_a, d_b, {g.qmul}, o, &tr));
  out = std::move(o[0]);
  return BPP_OK;
}

bool ipa_verification_scalars(IpaTranscript& tr, uint32_t n, const std::vector<Enc32>& L,
                              const std::vector<Enc32>& R, std::vector<hsc::Sc>& u_sq,
                              std::vector<hsc::Sc>& uinv_sq, std::vector<hsc::Sc>& s, bool* hook_failed) {
  const size_t lg_n = L.size();
  if (hook_failed) *hook_failed = false;
  if (lg_n >= 32 || R.size() != lg_n || n != (1u << lg_n)) return false;
  auto failed = [&] {
    if (hook_failed) *hook_failed = true;
    return false;
  };
  if (!tr.domain_sep(n)) return failed();
  std::vector<hsc::Sc> u(lg_n);
  static const uint8_t zero[32] = {0};
  for (size_t j = 0; j < lg_n; ++j) {
    // validate_and_append_point (transcript_protocol.rs:48-60): the identity
    // encoding is a VerificationError before anything is appended
    if (!memcmp(L[j].data(), zero, 32)) return false;
    if (!tr.append("L", L[j].data(), 32)) return failed();
    if (!memcmp(R[j].data(), zero, 32)) return false;
    if (!tr.append("R", R[j].data(), 32)) return failed();
    if (!tr.challenge_scalar("u", u[j])) return failed();
  }
  std::vector<hsc::Sc> ui = u;
  const hsc::Sc allinv = hsc::batch_invert(ui, true, true);  // (u: public challenges)
  u_sq.resize(lg_n);
  uinv_sq.resize(lg_n);
  for (size_t j = 0; j < lg_n; ++j) {
    u_sq[j] = hsc::sq(u[j]);
    uinv_sq[j] = hsc::sq(ui[j]);
  }
  s.assign(n, hsc::zero());
  s[0] = allinv;
  for (uint32_t i = 1; i < n; ++i) {
    uint32_t lg_i = 31 - __builtin_clz(i);
    uint32_t k = 1u << lg_i;
    s[i] = hsc::mul(s[i - k], u_sq[lg_n - 1 - lg_i]);
  }
  return true;
}
