// Vector-polynomial stage of the batched permutation prover on the GPU
// (the reference's vm_mult / mv_mult /
// inner_product / VecPoly3 work, util.rs:6-94, poly.rs:39-76, batched over
// the proofs of a lockstep batch).  Host side: the transcript challenges
// (y, z, x) and scalar bookkeeping only.
//
// Per proof (one workgroup; lane i handles gates i, i + 256, ...; Montgomery domain,
// R = 2^256 as in sc25519.cuh and host/scalar.h):
//   k_poly_coef  y^i, y^-i, z^(q+1) (LDS), the sparse column sums
//                zW_L, zW_R, zW_O (column-CSR of the circuit matrices), the
//                coefficient vectors of l(X) = l1 X + l2 X^2 + l3 X^3 and
//                r(X) = r0 + r1 X + r3 X^3, and the six t_i = inner products
//                (workgroup reduction) -> host for the T commitments; also
//                <z^Q W_V, gamma> (the V columns of the same CSR against the
//                proof's blindings) -> host for tau_x
//   k_poly_x     l = l(x), r = r(x) straight into the IPA's input arrays,
//                t_hat = <l, r> -> host
// Identical values to the host formulas they replace (perm_api.hip history;
// oracle/bulletproofs.py prove()), hence identical proof bytes (tests).
#include <algorithm>
#include <cstring>

#include "ctx.h"
#include "poly.h"
#include "verify_dev.h"
#include "keccak_dev.cuh"
#include "sc25519.cuh"

#define POLY_SLOTS 7  // l1 r0 r1 r3 l2 l3 (Montgomery) per gate
#define POLY_T 256    // lanes per proof; lane i handles gates i, i + POLY_T, ...

// aR^e (Montgomery in, Montgomery out), e < 2^31
FE_INLINE sc sc_pow_small(const sc& aR, uint32_t e, const sc& oneR) {
  sc r = oneR;
  if (!e) return r;
  for (int b = 31 - __clz(e); b >= 0; --b) {
    r = sc_mont(r, r);
    if ((e >> b) & 1u) r = sc_mont(r, aR);
  }
  return r;
}

// Doubling tables in LDS (every lane calls; ends with a barrier).  Table t
// holds N_t >= 1 entries tab[e] = prod over the set bits b of e of f_b
// (Montgomery), from tab[0] = 1 and either tab[1] = x (powers, f_b = x^(2^b);
// pre = false) or every tab[2^b] = f_b written by the caller (pre = true);
// the step for s = 1, 2, 4, ... fills (s, 2s], or (s, 2s) when preloaded, as
// tab[e - s] tab[s] (e - s < s shares no bit with s).  A table costs log2(N)
// dependent multiplies where sc_pow_small spends up to 2 log2(N) on each
// entry, and all tables advance in the same steps.
struct ScTable {
  uint32_t* tab;
  uint32_t N;
  bool pre;
};
FE_INLINE void sc_tables3(const ScTable t0, const ScTable t1, const ScTable t2) {
  constexpr int T = 3;
  const ScTable tb[T] = {t0, t1, t2};
  uint32_t nmax = 0;
  _Pragma("unroll") for (int t = 0; t < T; ++t) nmax = max(nmax, tb[t].N);
  __syncthreads();  // the caller's preloads
  for (uint32_t s = 1; s + 1 < nmax; s <<= 1) {
    uint32_t cnt[T], tot = 0;
    _Pragma("unroll") for (int t = 0; t < T; ++t) {
      const uint32_t hi = min(2 * s - (tb[t].pre ? 1u : 0u), tb[t].N - 1);
      cnt[t] = hi > s ? hi - s : 0;
      tot += cnt[t];
    }
    for (uint32_t u = threadIdx.x; u < tot; u += blockDim.x) {
      uint32_t off = u, t = 0;
      _Pragma("unroll") for (int k = 0; k + 1 < T; ++k) if (t == (uint32_t)k && off >= cnt[k]) {
          off -= cnt[k];
          t = k + 1;
        }
      uint32_t* tab = tb[0].tab;
      _Pragma("unroll") for (int k = 1; k < T; ++k) tab = t == (uint32_t)k ? tb[k].tab : tab;
      const uint32_t e = s + 1 + off;
      sc_store(tab + 8 * e, sc_mont(sc_load(tab + 8 * (e - s)), sc_load(tab + 8 * s)));
    }
    __syncthreads();
  }
}

// Power-table preload (one lane): tab[0] = 1, tab[1] = x
FE_INLINE void sc_table_pow_init(uint32_t* tab, uint32_t N, const sc& xR, const sc& oneR) {
  sc_store(tab, oneR);
  if (N > 1) sc_store(tab + 8, xR);
}

// Gates beyond the first POW_LO: lane tid handles gate i = tid + POW_LO r
// (blockDim = POLY_T = POW_LO whenever n_p > POW_LO), so x^i = tab[tid]
// (x^POW_LO)^r with the second factor kept as a running product
#define POW_LO POLY_T
#define POW_LO_LG 8
static_assert(POW_LO == 1 << POW_LO_LG, "POW_LO");

// Sum over the workgroup of K Montgomery scalars per lane; valid in lane 0.
template <int K>
FE_INLINE void sc_block_sum(sc (&v)[K], uint32_t* lds) {
  _Pragma("unroll") for (int j = 0; j < K; ++j) v[j] = sc_wave_sum(v[j]);
  const uint32_t nw = blockDim.x >> 6, w = threadIdx.x >> 6;
  if (nw == 1) return;
  if ((threadIdx.x & 63u) == 0)
    _Pragma("unroll") for (int j = 0; j < K; ++j) sc_store(lds + (w * K + j) * 8, v[j]);
  __syncthreads();
  if (threadIdx.x == 0)
    for (uint32_t u = 1; u < nw; ++u)
      _Pragma("unroll") for (int j = 0; j < K; ++j) v[j] = sc_add(v[j], sc_load(lds + (u * K + j) * 8));
}

// sum over the column's entries of z^(q+1) * val (Montgomery)
FE_INLINE sc col_sum(const uint32_t* __restrict__ cp, const uint32_t* __restrict__ ce, uint32_t col,
                     const uint32_t* zp) {
  sc acc = sc_zero();
  for (uint32_t e = cp[col]; e < cp[col + 1]; ++e)
    acc = sc_add(acc, sc_mont(sc_load(zp + 8 * ce[9 * e]), sc_load(ce + 9 * e + 1)));
  return acc;
}

// Column sum split over the whole workgroup (every lane must call it): for
// the few columns with many entries -- W_V's x column holds one entry per
// a_L / a_R row using x (2k + 1 of them), which as one lane's serial chain
// doubled k_poly_coef (126 -> 292 us) and dominated k_verify_scalars.
// Valid in lane 0; `red` is the workgroup-sum scratch.
#define HEAVY_COL 8
FE_INLINE sc col_sum_block(const uint32_t* __restrict__ cp, const uint32_t* __restrict__ ce, uint32_t col,
                           const uint32_t* zp, uint32_t* red) {
  sc v[1] = {sc_zero()};
  for (uint32_t e = cp[col] + threadIdx.x; e < cp[col + 1]; e += blockDim.x)
    v[0] = sc_add(v[0], sc_mont(sc_load(zp + 8 * ce[9 * e]), sc_load(ce + 9 * e + 1)));
  sc_block_sum<1>(v, red);
  __syncthreads();  // red is reused by the next call
  return v[0];
}

// grid = P proofs, block = poly_block(max(n_p, m)); dynamic LDS = (Q + 1 + 2 min(n_p, POW_LO)) * 32 + (POLY_T / 64) * 7 * 32
// t_out[p] = t_1..t_6, <z^Q W_V, gamma_p> (gamma: [P][m] canonical)
#define POLY_NT 7
__global__ void __launch_bounds__(POLY_T) k_poly_coef(uint32_t n_p, uint32_t m, uint32_t Q, uint32_t per,
                                                   const uint32_t* __restrict__ sc_in,
                                                   const uint32_t* __restrict__ ch,
                                                   const uint32_t* __restrict__ cp, const uint32_t* __restrict__ ce,
                                                   const uint32_t* __restrict__ gamma, uint32_t* __restrict__ vec,
                                                   uint32_t* __restrict__ hf, uint32_t* __restrict__ t_out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t NY = min(n_p, (uint32_t)POW_LO);
  uint32_t* zt = lds;               // [Q + 1] z^e
  uint32_t* yt = zt + 8 * (Q + 1);  // [NY] y^i
  uint32_t* yit = yt + 8 * NY;      // [NY] y^-i
  uint32_t* red = yit + 8 * NY;     // reduction scratch
  const uint32_t* zp = zt + 8;      // z^(q+1)
  const uint32_t p = blockIdx.x;
  const sc oneR = sc_one_mont();
  const sc yR = sc_to_mont(sc_load(ch + 24 * p)), yiR = sc_to_mont(sc_load(ch + 24 * p + 8)),
           zR = sc_to_mont(sc_load(ch + 24 * p + 16));
  if (threadIdx.x == 0) {
    sc_table_pow_init(zt, Q + 1, zR, oneR);
    sc_table_pow_init(yt, NY, yR, oneR);
    sc_table_pow_init(yit, NY, yiR, oneR);
  }
  sc_tables3({zt, Q + 1, false}, {yt, NY, false}, {yit, NY, false});
  sc yhi = oneR, yihi = oneR, ystep = oneR, yistep = oneR;  // (y^POW_LO)^r
  if (n_p > POW_LO) {
    ystep = sc_mont(sc_load(yt + 8 * (POW_LO - 1)), yR);
    yistep = sc_mont(sc_load(yit + 8 * (POW_LO - 1)), yiR);
  }
  sc t[POLY_NT];
  _Pragma("unroll") for (int j = 0; j < POLY_NT; ++j) t[j] = sc_zero();
  for (uint32_t i = threadIdx.x; i < n_p; i += blockDim.x) {
    const uint32_t* s = sc_in + (size_t)p * per * 8;
    const sc aL = sc_to_mont(sc_load(s + 8 * (1 + i)));
    const sc aR = sc_to_mont(sc_load(s + 8 * (1 + n_p + i)));
    const sc l2 = sc_to_mont(sc_load(s + 8 * (2 + 2 * n_p + i)));  // a_O
    const sc l3 = sc_to_mont(sc_load(s + 8 * (3 + 3 * n_p + i)));  // s_L
    const sc sR = sc_to_mont(sc_load(s + 8 * (3 + 4 * n_p + i)));
    sc yp = sc_load(yt + 8 * (i % POW_LO)), yip = sc_load(yit + 8 * (i % POW_LO));
    if (i >= POW_LO) {
      yp = sc_mont(yp, yhi);
      yip = sc_mont(yip, yihi);
    }
    if (n_p > POW_LO) {
      yhi = sc_mont(yhi, ystep);
      yihi = sc_mont(yihi, yistep);
    }
#ifdef EXP_P_NOCS
    const sc zWL = aL, zWR = aR, zWO = l2;
#else
    const sc zWL = col_sum(cp, ce, i, zp), zWR = col_sum(cp + (n_p + 1), ce, i, zp),
             zWO = col_sum(cp + 2 * (n_p + 1), ce, i, zp);
#endif
    const sc l1 = sc_add(aL, sc_mont(zWR, yip));
    const sc r0 = sc_sub(zWO, yp);
    const sc r1 = sc_add(sc_mont(aR, yp), zWL);
    const sc r3 = sc_mont(sR, yp);
#ifndef EXP_P_NOT
    t[0] = sc_add(t[0], sc_mont(l1, r0));
    t[1] = sc_add(t[1], sc_add(sc_mont(l1, r1), sc_mont(l2, r0)));
    t[2] = sc_add(t[2], sc_add(sc_mont(l2, r1), sc_mont(l3, r0)));
    t[3] = sc_add(t[3], sc_add(sc_mont(l1, r3), sc_mont(l3, r1)));
    t[4] = sc_add(t[4], sc_mont(l2, r3));
    t[5] = sc_add(t[5], sc_mont(l3, r3));
#endif
    uint32_t* v = vec + ((size_t)p * n_p + i) * POLY_SLOTS * 8;
    sc_store(v + 0, l1);
    sc_store(v + 8, r0);
    sc_store(v + 16, r1);
    sc_store(v + 24, r3);
    sc_store(v + 32, l2);
    sc_store(v + 40, l3);
    sc_store(hf + ((size_t)p * n_p + i) * 8, sc_from_mont(yip));  // H factors y^-i
  }
  // tau_x's <z^Q W_V, gamma>: V column j of the fourth CSR block (Montgomery)
  // times gamma_j (canonical) is canonical z^Q W_V[j] gamma_j; to_mont keeps
  // the sum in the Montgomery domain of the other six
  const uint32_t* cpv = cp + 3 * (n_p + 1);
  const uint32_t* gam = gamma + 8 * (size_t)p * m;
#ifndef EXP_P_NOV
  for (uint32_t j = threadIdx.x; j < m; j += blockDim.x)
    if (cpv[j + 1] - cpv[j] <= HEAVY_COL) t[6] = sc_add(t[6], sc_mont(col_sum(cpv, ce, j, zp), sc_to_mont(sc_load(gam + 8 * j))));
  const uint32_t* heavy = cpv + m + 1;  // [count, columns...] (build_csr)
  for (uint32_t h = 0; h < heavy[0]; ++h) {
    const uint32_t j = heavy[1 + h];
    const sc cs = col_sum_block(cpv, ce, j, zp, red);
    if (threadIdx.x == 0) t[6] = sc_add(t[6], sc_mont(cs, sc_to_mont(sc_load(gam + 8 * j))));
  }
#endif
  sc_block_sum<POLY_NT>(t, red);
  if (threadIdx.x == 0)
    _Pragma("unroll") for (int j = 0; j < POLY_NT; ++j) sc_store(t_out + (POLY_NT * p + j) * 8, sc_from_mont(t[j]));
}

// grid = P, block = poly_block(n_p)
__global__ void __launch_bounds__(POLY_T) k_poly_x(uint32_t n_p, const uint32_t* __restrict__ xs,
                                                const uint32_t* __restrict__ vec, uint32_t* __restrict__ l_out,
                                                uint32_t* __restrict__ r_out, uint32_t* __restrict__ that_out) {
  __shared__ __attribute__((aligned(16))) uint32_t red[(POLY_T / 64) * 8];
  const uint32_t p = blockIdx.x;
  const sc xR = sc_to_mont(sc_load(xs + 8 * p));
  const sc x2R = sc_mont(xR, xR);
  sc th[1] = {sc_zero()};
  for (uint32_t i = threadIdx.x; i < n_p; i += blockDim.x) {
    const uint32_t* v = vec + ((size_t)p * n_p + i) * POLY_SLOTS * 8;
    const sc l1 = sc_load(v), r0 = sc_load(v + 8), r1 = sc_load(v + 16), r3 = sc_load(v + 24), l2 = sc_load(v + 32),
             l3 = sc_load(v + 40);
    const sc l = sc_mont(sc_add(l1, sc_mont(sc_add(l2, sc_mont(l3, xR)), xR)), xR);
    const sc r = sc_add(r0, sc_mont(sc_add(r1, sc_mont(r3, x2R)), xR));
    th[0] = sc_add(th[0], sc_mont(l, r));
    sc_store(l_out + ((size_t)p * n_p + i) * 8, sc_from_mont(l));
    sc_store(r_out + ((size_t)p * n_p + i) * 8, sc_from_mont(r));
  }
  sc_block_sum<1>(th, red);
  if (threadIdx.x == 0) sc_store(that_out + 8 * p, sc_from_mont(th[0]));
}

// ---------------------------------------------------------------------------
// Batch verifier's MSM scalars on the GPU (the verifier side of the same
// circuit algebra, circuit_lib.rs:478-585 in sound form; host restatement
// perm_api.hip verify_expand, which bpp_perm_verify_scalars still uses).
// One workgroup per proof; rec[p] = VREC_N canonical scalars:
// (VREC_* slots: verify_dev.h)
// Writes wt * (generator scalars) to gen[p][2 n_p + 2] (summed over proofs by
// k_verify_merge) and wt * (proof-point scalars) to sc_out[NG + p npt + j]
// (V_0..V_{m-1}, A_I, A_O, S, T1 T3 T4 T5 T6, L_0.., R_0..), canonical.
#ifdef VS_TIMING  // phase stamps of k_verify_scalars (timing variant only: tools/vs_phases.py)
__device__ unsigned long long vs_dbg[8192 * 8];
#define VS_T(k) \
  if (threadIdx.x == 0 && blockIdx.x < 8192) vs_dbg[blockIdx.x * 8 + (k)] = clock64()
extern "C" int bpp_debug_vs_timing(unsigned long long* out, size_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vs_dbg), n * 8) == hipSuccess ? 0 : 1;
}
#else
#define VS_T(k)
#endif
// Per-proof constants of k_verify_scalars (Montgomery form, VK_N x 8 words
// a proof): every product of two workgroup-uniform values is formed here, on
// the vector unit.  Inside k_verify_scalars such products ran on the scalar
// unit (uniform operands): 21 K SALU instructions per wave next to 15 K VALU,
// ~400 spilled SGPRs, and the CU's one scalar unit shared by its waves (r04
// PMC, tools/vs_phases.py).
//
// No inverses: proof p's check is scaled by F = U^2 Y, U = prod u_j, Y =
// y^(n_p - 1) (nonzero: a zero y or u_j rejects the proof in the replay), so
// that with s_i / s_0 = prod over the bits of i of u^2 (st below) and yr_i =
// y^(n_p - 1 - i):
//   G_i: st[i] U Y a - x zWR_i U^2 yr_i
//   H_i: st[n_p-1-i] U b yr_i - (x zWL_i + zWO_i) U^2 yr_i + F
//   B:   r F t_hat - r x^2 (delta' + F <z^Q, c>) + w F (a b - t_hat),
//        delta' = sum_i U^2 yr_i zWR_i zWL_i
//   B~:  F (r tau_x + mu)
//   V_j: -r x^2 F zWV_j;  A_I A_O S: -F x^(1,2,3);  T_k: -F r x^k
//   L_j: -F u_j^2;  R_j: -Y prod_{k != j} u_k^2
// (F times bulletproofs' verification_scalars / the t-check), all times the
// proof's batch weight w_p = perm::batch_weight(seed, first + p, r_p).
#define VK_Z 0       // z
#define VK_Y 1       // y
#define VK_X 2       // x
#define VK_WT 3      // w_p, the proof's batch weight
#define VK_UYA 4     // w_p U Y a
#define VK_UB 5      // w_p U b
#define VK_WRX2 6    // w_p r x^2
#define VK_WRFT 7    // w_p r F t_hat
#define VK_IB 8      // w_p w F (a b - t_hat)
#define VK_BB 9      // w_p F (r tau_x + mu)
#define VK_R 10      // r
#define VK_NXP 11    // -x_perm
#define VK_U2 12     // U^2
#define VK_F 13      // F
#define VK_WTF 14    // w_p F
#define VK_WRX2F 15  // w_p r x^2 F
#define VK_XU2 16    // w_p x U^2
#define VK_U2W 17    // w_p U^2
#define VK_N 18      // constants a proof

// k_verify_consts works on 16 lanes a proof, 4 proofs a wave, VC_W such
// waves and one Keccak wave a workgroup.  One lane a proof (round 5's first
// version) ran every product of a proof on one lane: ~100 dependent scalar
// multiplies plus the sponge, 67 us for 4096 proofs on 64 waves.  Here the
// proof's multiplies are spread over its 16 lanes in dependency levels: the
// R_j products prod_{k != j} u_k^2, U = prod u_k and Y = y^(2^lg - 1) as one
// lg-step loop (one lane each), the named constants in four levels of at most
// 10 independent products (a table of (op, dst, a, b) per lane), and the
// batch weight's SHAKE256 on the Keccak wave while the loop runs.  Values
// travel through LDS slots (VC_*), the first VK_N of which are the VK_*
// outputs.  The proof-point scalars that are per-proof constants -- A_I,
// A_O, S: -w F x^(1,2,3); T_k: -w F r x^k (k = 1, 3..6); L_j: -w F u_j^2;
// R_j: -w Y prod_{k != j} u_k^2 -- are finished here too and written
// straight to their MSM slots (sc_out[NG + p npt + m + j], canonical), so
// k_verify_scalars is left with the gate and V columns.
#define VC_W 2
#define VC_P (4 * VC_W)  // proofs a workgroup
#define VC_LGMAX 32
#define VC_T_U 18
#define VC_T_YR 19
#define VC_T_A 20
#define VC_T_B 21
#define VC_T_TH 22
#define VC_T_W 23
#define VC_T_TAUX 24
#define VC_T_MU 25
#define VC_T_WR 26
#define VC_T_X2 27
#define VC_T_AB 28
#define VC_T_RT 29
#define VC_T_WU 30
#define VC_T_WY 31
#define VC_T_WX 32
#define VC_T_RTH 33
#define VC_T_ABT 34
#define VC_T_RTM 35
#define VC_T_NWY 36
#define VC_T_WUA 37
#define VC_T_IBT 38
#define VC_NV 39
enum : uint8_t { VC_NOP = 0, VC_MUL, VC_ADD, VC_SUB, VC_NEG };
// level l, lane k: {op, dst, a, b}
__constant__ uint8_t vc_prog[4][16][4] = {
    {{VC_MUL, VK_U2, VC_T_U, VC_T_U},
     {VC_MUL, VC_T_WR, VK_WT, VK_R},
     {VC_MUL, VC_T_X2, VK_X, VK_X},
     {VC_MUL, VC_T_AB, VC_T_A, VC_T_B},
     {VC_MUL, VC_T_RT, VK_R, VC_T_TAUX},
     {VC_MUL, VC_T_WU, VK_WT, VC_T_U},
     {VC_MUL, VC_T_WY, VK_WT, VC_T_YR},
     {VC_MUL, VC_T_WX, VK_WT, VK_X},
     {VC_MUL, VC_T_RTH, VK_R, VC_T_TH}},
    {{VC_MUL, VK_F, VK_U2, VC_T_YR},
     {VC_MUL, VK_WRX2, VC_T_WR, VC_T_X2},
     {VC_MUL, VC_T_WUA, VC_T_WU, VC_T_A},
     {VC_MUL, VK_UB, VC_T_WU, VC_T_B},
     {VC_MUL, VK_XU2, VC_T_WX, VK_U2},
     {VC_MUL, VK_U2W, VK_WT, VK_U2},
     {VC_MUL, VK_WTF, VC_T_WY, VK_U2},
     {VC_SUB, VC_T_ABT, VC_T_AB, VC_T_TH},
     {VC_ADD, VC_T_RTM, VC_T_RT, VC_T_MU},
     {VC_NEG, VC_T_NWY, VC_T_WY, 0}},
    {{VC_MUL, VK_UYA, VC_T_WUA, VC_T_YR},
     {VC_MUL, VK_WRFT, VK_WTF, VC_T_RTH},
     {VC_MUL, VC_T_IBT, VC_T_W, VC_T_ABT},
     {VC_MUL, VK_BB, VK_WTF, VC_T_RTM},
     {VC_MUL, VK_WRX2F, VK_WRX2, VK_F}},
    {{VC_MUL, VK_IB, VK_WTF, VC_T_IBT}},
};
// (record slot, value slot) of the loaded proof values
__constant__ uint8_t vc_load[11][2] = {{VREC_Z, VK_Z},     {VREC_Y, VK_Y},         {VREC_X, VK_X},
                                       {VREC_R, VK_R},     {VREC_XPERM, VK_NXP},   {VREC_A, VC_T_A},
                                       {VREC_B, VC_T_B},   {VREC_THAT, VC_T_TH},   {VREC_W, VC_T_W},
                                       {VREC_TAUX, VC_T_TAUX}, {VREC_MU, VC_T_MU}};
__global__ void __launch_bounds__(64 * (VC_W + 1)) k_verify_consts(uint32_t count, uint32_t lg, uint64_t first,
                                                                   const uint32_t* __restrict__ seed,
                                                                   const uint32_t* __restrict__ rec,
                                                                   uint32_t* __restrict__ kc, uint32_t NG, uint32_t m,
                                                                   uint32_t npt, uint32_t* __restrict__ sc_out) {
  __builtin_amdgcn_s_setprio(3);  // (latency chain; the decompression runs beside it)
  __shared__ __attribute__((aligned(16))) uint32_t vs[VC_P][VC_NV * 8];
  __shared__ __attribute__((aligned(16))) uint32_t ut[VC_P][VC_LGMAX * 8], u2t[VC_P][VC_LGMAX * 8],
      pjt[VC_P][VC_LGMAX * 8];
  const uint32_t nrec = VREC_U + lg;
  const bool kwave = threadIdx.x >= 64 * VC_W;
  const uint32_t g = (threadIdx.x >> 4) & (VC_P - 1), l = threadIdx.x & 15u;
  const uint32_t p = blockIdx.x * VC_P + g;
  const bool live = !kwave && p < count;
  const uint32_t* R = rec + (size_t)p * nrec * 8;
  uint32_t* V = vs[g];
  const sc oneR = sc_one_mont();
  auto ldv = [&](uint32_t k) { return sc_load(V + 8 * k); };
  if (live) {
    if (l < 11) {
      sc v = sc_to_mont(sc_load(R + 8 * vc_load[l][0]));
      if (vc_load[l][1] == VK_NXP) v = sc_neg(v);
      sc_store(V + 8 * vc_load[l][1], v);
    }
    for (uint32_t j = l; j < lg; j += 16) {
      const sc u = sc_to_mont(sc_load(R + 8 * (VREC_U + j)));
      sc_store(ut[g] + 8 * j, u);
      sc_store(u2t[g] + 8 * j, sc_mont(u, u));
    }
  }
  __syncthreads();
  if (live) {
    // lanes j < lg: prod_{k != j} u_k^2; lane lg: U; lane lg + 1: Y
    const sc yR = ldv(VK_Y);
    for (uint32_t jj = l; jj < lg + 2; jj += 16) {
      const bool isY = jj == lg + 1, isU = jj == lg;
      sc v = oneR;
      for (uint32_t k = 0; k < lg; ++k) {
        const sc f = isY ? v : isU ? sc_load(ut[g] + 8 * k) : k == jj ? oneR : sc_load(u2t[g] + 8 * k);
        v = sc_mont(v, f);
        if (isY) v = sc_mont(v, yR);
      }
      sc_store(isY ? V + 8 * VC_T_YR : isU ? V + 8 * VC_T_U : pjt[g] + 8 * jj, v);
    }
  } else if (kwave && (threadIdx.x & 63u) < VC_P && blockIdx.x * VC_P + (threadIdx.x & 63u) < count) {
    // w_p = from_wide(SHAKE256("bp-perm-batch-wt" || seed || le64(first + p) ||
    // r_p)[0..64]): 88 bytes, one sponge block (perm::batch_weight)
    const uint32_t q = threadIdx.x & 63u, pq = blockIdx.x * VC_P + q;
    uint64_t a[25];
    _Pragma("unroll") for (int i = 0; i < 25; ++i) a[i] = 0;
    a[0] = 0x6d7265702d7062ull | (0x2dull << 56);  // "bp-perm-"
    a[1] = 0x74772d6863746162ull;                 // "batch-wt"
    _Pragma("unroll") for (int i = 0; i < 4; ++i) a[2 + i] = (uint64_t)seed[2 * i] | ((uint64_t)seed[2 * i + 1] << 32);
    a[6] = first + pq;
    const uint32_t* rp = rec + ((size_t)pq * nrec + VREC_R) * 8;
    _Pragma("unroll") for (int i = 0; i < 4; ++i) a[7 + i] = (uint64_t)rp[2 * i] | ((uint64_t)rp[2 * i + 1] << 32);
    a[11] = 0x1full;        // SHAKE domain byte at 88
    a[16] = 0x80ull << 56;  // last byte of the 136-byte rate
    keccak_f1600_dev(a);
    uint32_t o[16];
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      o[2 * i] = (uint32_t)a[i];
      o[2 * i + 1] = (uint32_t)(a[i] >> 32);
    }
    sc_store(vs[q] + 8 * VK_WT, sc_to_mont(sc_from_wide_w(o)));
  }
  __syncthreads();
  for (uint32_t lv = 0; lv < 4; ++lv) {
    if (live && vc_prog[lv][l][0] != VC_NOP) {
      const uint8_t op = vc_prog[lv][l][0];
      const sc x = ldv(vc_prog[lv][l][2]), y = ldv(vc_prog[lv][l][3]);
      const sc r = op == VC_MUL ? sc_mont(x, y) : op == VC_ADD ? sc_add(x, y) : op == VC_SUB ? sc_sub(x, y) : sc_neg(x);
      sc_store(V + 8 * vc_prog[lv][l][1], r);
    }
    __syncthreads();
  }
  if (live) {
    uint32_t* K = kc + (size_t)p * VK_N * 8;
    for (uint32_t w = l; w < VK_N * 8; w += 16) K[w] = V[w];
    // the proof-point scalars after V_0..V_{m-1}
    uint32_t* out = sc_out + 8 * ((size_t)NG + (size_t)p * npt + m);
    const sc xR = ldv(VK_X), nwtf = sc_neg(ldv(VK_WTF));
    for (uint32_t j = l; j < 8 + 2 * lg; j += 16) {
      sc v;
      if (j >= 8 + lg) {
        v = sc_mont(sc_load(pjt[g] + 8 * (j - 8 - lg)), ldv(VC_T_NWY));
      } else {
        if (j < 3) {
          v = sc_pow_small(xR, j + 1, oneR);
        } else if (j < 8) {
          v = sc_mont(ldv(VK_R), sc_pow_small(xR, j == 3 ? 1u : j - 1, oneR));  // T1, T3, T4, T5, T6
        } else {
          v = sc_load(u2t[g] + 8 * (j - 8));
        }
        v = sc_mont(v, nwtf);
      }
      sc_store(out + 8 * j, sc_from_mont(v));
    }
  }
}

// (at 4 waves per SIMD: 128 VGPRs instead of 148, 108 B of spills, 8
// workgroups per CU instead of 6 -- 2 rounds for 4096 proofs instead of 2.7;
// three interleaved passes 0.281-0.283 vs 0.294-0.297 ms with the constants
// and the merge, 0.309-0.312 at 5, profiles/r04_verify_vs_ab.txt)
#ifndef VS_WPE
#define VS_WPE 4
#endif
__global__ void __launch_bounds__(POLY_T) __attribute__((amdgpu_waves_per_eu(VS_WPE))) k_verify_scalars(
    uint32_t n_p, uint32_t m, uint32_t Q, uint32_t lg, const uint32_t* __restrict__ rec,
    const uint32_t* __restrict__ kc, const uint32_t* __restrict__ cp, const uint32_t* __restrict__ ce,
    const uint32_t* __restrict__ cR, uint32_t* __restrict__ gen, uint32_t* __restrict__ sc_out, uint32_t NG,
    uint32_t npt) {
  __builtin_amdgcn_s_setprio(2);  // (ahead of the proof-point decompression beside it)
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t NY = min(n_p, (uint32_t)POW_LO);
  uint32_t* zt = lds;                // [Q + 1] z^e, Montgomery
  uint32_t* yt = zt + 8 * (Q + 1);   // [NY] y^e
  uint32_t* st = yt + 8 * NY;        // [NY] s_i / s_0 (below)
  uint32_t* red = st + 8 * NY;       // reduction scratch
  const uint32_t* zp = zt + 8;       // z^(q+1)
  const uint32_t p = blockIdx.x, nrec = VREC_U + lg;
  const uint32_t* R = rec + (size_t)p * nrec * 8;
  const uint32_t* K = kc + (size_t)p * VK_N * 8;
  const sc oneR = sc_one_mont();
  auto ldm = [&](uint32_t k) { return sc_to_mont(sc_load(R + 8 * k)); };
  auto ldk = [&](uint32_t k) { return sc_load(K + 8 * k); };
  VS_T(0);
  // s_i = s_0 prod_{bit k of i} u_{lg-1-k}^2 (bulletproofs
  // verification_scalars): st[i] = s_i / s_0 for i < NY as a doubling table
  // over the factors u_{lg-1-k}^2, the bits from POW_LO_LG up per lane
  if (threadIdx.x == 0) {
    sc_table_pow_init(zt, Q + 1, ldk(VK_Z), oneR);
    sc_table_pow_init(yt, NY, ldk(VK_Y), oneR);
    sc_store(st, oneR);
  }
  for (uint32_t b = threadIdx.x; b < POW_LO_LG && (1u << b) < NY; b += blockDim.x) {
    const sc u = ldm(VREC_U + lg - 1 - b);
    sc_store(st + 8 * (1u << b), sc_mont(u, u));
  }
  sc_tables3({zt, Q + 1, false}, {yt, NY, false}, {st, NY, true});
  VS_T(1);
  auto s_of = [&](uint32_t i) {  // s_i / s_0
    sc v = sc_load(st + 8 * (i % POW_LO));
    for (uint32_t k = POW_LO_LG; k < lg; ++k)
      if ((i >> k) & 1u) {
        const sc u = ldm(VREC_U + lg - 1 - k);
        v = sc_mont(v, sc_mont(u, u));
      }
    return v;
  };
  // (weighted: w_p folded into the constants)
  const sc uyaR = ldk(VK_UYA), ubR = ldk(VK_UB), xu2R = ldk(VK_XU2), u2R = ldk(VK_U2W), fR = ldk(VK_WTF);
  // gate i = n_p - 1 - e with e ascending per lane: yr_i = y^e = yt[e mod
  // POW_LO] (y^POW_LO)^(e / POW_LO), the second factor a running product
  // (blockDim = POW_LO whenever n_p > POW_LO)
  sc yhi = oneR, ystep = oneR;
  if (n_p > POW_LO) ystep = sc_mont(sc_load(yt + 8 * (POW_LO - 1)), ldk(VK_Y));
  const size_t gb = (size_t)p * NG;
  // acc[0]: delta'' = sum yr_i zWR_i zWL_i (delta' = U^2 delta'', applied
  // once below); acc[1]: zc = <z^Q, c>
  sc acc[2] = {sc_zero(), sc_zero()};
  for (uint32_t e = threadIdx.x; e < n_p; e += blockDim.x) {
    const uint32_t i = n_p - 1 - e;
    sc yr = sc_load(yt + 8 * (e % POW_LO));
    if (e >= POW_LO) yr = sc_mont(yr, yhi);
    if (n_p > POW_LO) yhi = sc_mont(yhi, ystep);
    const sc zWL = col_sum(cp, ce, i, zp), zWR = col_sum(cp + (n_p + 1), ce, i, zp),
             zWO = col_sum(cp + 2 * (n_p + 1), ce, i, zp);
    const sc rw = sc_mont(zWR, yr);
    acc[0] = sc_add(acc[0], sc_mont(rw, zWL));
    // G_i: st[i] U Y a - (zWR yr) x U^2;  H_i: (st[e] U b - zWL x U^2 - zWO U^2) yr + F
    const sc gi = sc_sub(sc_mont(s_of(i), uyaR), sc_mont(rw, xu2R));
    const sc hi = sc_add(sc_mont(sc_sub(sc_sub(sc_mont(s_of(e), ubR), sc_mont(zWL, xu2R)), sc_mont(zWO, u2R)), yr),
                         fR);
    sc_store(gen + 8 * (gb + i), sc_from_mont(gi));
    sc_store(gen + 8 * (gb + n_p + i), sc_from_mont(hi));
  }
  VS_T(2);
  for (uint32_t q = threadIdx.x; q < Q; q += blockDim.x) {
    const sc c = q + 1 == Q ? ldk(VK_NXP) : sc_to_mont(sc_load(cR + 8 * q));
    acc[1] = sc_add(acc[1], sc_mont(sc_load(zp + 8 * q), c));
  }
  VS_T(3);
  const sc wrx2fR = ldk(VK_WRX2F);
  const size_t pb = NG + (size_t)p * npt;
  // V_j: -wt r x^2 F zWV_j (zWV from the fourth column-CSR, m columns; the
  // heavy x column summed by the whole workgroup)
  const uint32_t* cpv = cp + 3 * (n_p + 1);
  for (uint32_t j = threadIdx.x; j < m; j += blockDim.x)
    if (cpv[j + 1] - cpv[j] <= HEAVY_COL)
      sc_store(sc_out + 8 * (pb + j), sc_from_mont(sc_neg(sc_mont(col_sum(cpv, ce, j, zp), wrx2fR))));
  const uint32_t* heavy = cpv + m + 1;  // [count, columns...] (build_csr)
  for (uint32_t h = 0; h < heavy[0]; ++h) {
    const uint32_t j = heavy[1 + h];
    const sc cs = col_sum_block(cpv, ce, j, zp, red);
    if (threadIdx.x == 0) sc_store(sc_out + 8 * (pb + j), sc_from_mont(sc_neg(sc_mont(cs, wrx2fR))));
  }
  VS_T(4);
  // (A_I .. R_j: written by k_verify_consts)
  VS_T(5);
  sc_block_sum<2>(acc, red);
  VS_T(6);
  if (threadIdx.x == 0) {
    // B: wt (r F t_hat - r x^2 (delta' + F zc) + w F (a b - t_hat)); B_blinding: wt F (r tau_x + mu)
    const sc tB =
        sc_sub(ldk(VK_WRFT), sc_mont(ldk(VK_WRX2), sc_add(sc_mont(ldk(VK_U2), acc[0]), sc_mont(ldk(VK_F), acc[1]))));
    sc_store(gen + 8 * (gb + 2 * n_p), sc_from_mont(sc_add(tB, ldk(VK_IB))));
    sc_store(gen + 8 * (gb + 2 * n_p + 1), sc_from_mont(ldk(VK_BB)));
  }
  VS_T(7);
}

// sc_out[i] = sum_p gen[p][i] (one workgroup per generator column)
__global__ void __launch_bounds__(POLY_T) k_verify_merge(uint32_t count, uint32_t NG, const uint32_t* __restrict__ gen,
                                                      uint32_t* __restrict__ sc_out) {
  __shared__ __attribute__((aligned(16))) uint32_t red[(POLY_T / 64) * 8];
  const uint32_t i = blockIdx.x;
  sc acc[1] = {sc_zero()};
  for (uint32_t p = threadIdx.x; p < count; p += blockDim.x) acc[0] = sc_add(acc[0], sc_load(gen + 8 * ((size_t)p * NG + i)));
  sc_block_sum<1>(acc, red);
  if (threadIdx.x == 0) sc_store(sc_out + 8 * i, acc[0]);
}

// ---------------------------------------------------------------------------
// The prover's wide random draws reduced on the device.  stream = [P][len]
// bytes of each proof's SHAKE256 stream (host/perm.h draw order: pi's u64s,
// gamma[m], alpha beta rho, s_L[n_p], s_R[n_p], tau[5]); the host parses pi,
// alpha, beta, rho and tau itself and never needs gamma, s_L, s_R: gamma goes
// to [P][m] (V commitments, tau_x), s_L / s_R straight into their slots of the
// A_I/A_O/S scalar array ([P][per], per = 3 + 5 n_p: s_L at 3 + 3 n_p).
// The blinding draws (perm.h draw_scalar) of P proofs, one thread per draw:
// draw j's sponge block is the proof's template (tmpl [P][7] u64, host-built:
// domain || seed with the 0x1F pad byte after the index) plus le32 j at byte
// jo and the 0x80 that closes the 136-byte rate; one Keccak-f yields the 64
// bytes that from_wide reduces.  gamma -> [P][m]; alpha, beta, rho, s_L, s_R
// -> their slots of the A_I/A_O/S scalar array ([alpha, a_L, a_R, beta, a_O,
// rho, s_L, s_R], per words x 8 a proof); the host draws tau itself.
// With v (non-null) it also writes the V commitments' inputs (gamma_j's
// thread, j <= 2k): v[p][i] = i + 1 (i < k) or pi_p[i - k] + 1 (k <= i < 2k),
// g[p][i] = gamma_i, gx_half[p] = gamma_2k / 2 (V_2k is committed with halved
// scalars and encoded as 2 (C / 2) on the host) -- no launch of its own.
__global__ void __launch_bounds__(256) k_draws(uint32_t P, uint32_t m, uint32_t n_p, uint32_t per, uint32_t jo,
                                              const uint64_t* __restrict__ tmpl, uint32_t* __restrict__ gamma,
                                              uint32_t* __restrict__ sc_out, uint32_t k,
                                              const uint32_t* __restrict__ pi, uint32_t* __restrict__ v,
                                              uint32_t* __restrict__ g, uint32_t* __restrict__ gx_half) {
  const uint32_t nw = m + 3 + 2 * n_p;  // gamma[m], alpha, beta, rho, s_L[n_p], s_R[n_p]
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)P * nw) return;
  const uint32_t p = (uint32_t)(t / nw), j = (uint32_t)(t % nw);
  uint64_t a[25];
  _Pragma("unroll") for (int i = 0; i < 25; ++i) a[i] = i < 7 ? tmpl[7 * (size_t)p + i] : 0ull;
  a[16] ^= 0x8000000000000000ull;
  const uint32_t li = jo >> 3, sh = 8 * (jo & 7);
  _Pragma("unroll") for (uint32_t i = 0; i < 7; ++i) {  // (static indices: no scratch)
    if (i == li) a[i] ^= (uint64_t)j << sh;
    if (i == li + 1 && sh > 32) a[i] ^= (uint64_t)j >> (64 - sh);
  }
  keccak_f1600_dev(a);
  uint32_t w[16];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    w[2 * i] = (uint32_t)a[i];
    w[2 * i + 1] = (uint32_t)(a[i] >> 32);
  }
  const sc x = sc_from_wide_w(w);
  if (j < m) {
    sc_store(gamma + 8 * ((size_t)p * m + j), x);
    if (v) {
      if (j == 2 * k) {
        sc_store(gx_half + 8 * (size_t)p, sc_half(x));
      } else if (j < 2 * k) {
        sc vv = sc_zero();
        vv.v[0] = j < k ? j + 1 : pi[(size_t)p * k + (j - k)] + 1;
        sc_store(v + 8 * ((size_t)p * 2 * k + j), vv);
        sc_store(g + 8 * ((size_t)p * 2 * k + j), x);
      }
    }
    return;
  }
  const uint32_t q = j - m;
  const uint32_t pos = q == 0 ? 0u : q == 1 ? 1 + 2 * n_p : q == 2 ? 2 + 3 * n_p : 3 + 3 * n_p + (q - 3);
  sc_store(sc_out + 8 * ((size_t)p * per + pos), x);
}

// The sound create_a witness of one proof per workgroup (host restatement
// host/perm_circuit.cpp witness, weights.rs:63-113 fixed as SURVEY Q3):
// with d_A[i] = (i + 1) - x and d_B[i] = (pi_i + 1) - x (i < k) and their
// inclusive prefix products A, B, gates g < k - 1 are (A[g], d_A[g+1],
// A[g+1]), gates k-1+g' (g' < k-1) are (B[g'], d_B[g'+1], B[g'+1]), gate
// 2k-2 is (B[k-1], -1, -B[k-1]) and gate 2k-1 is (A[k-1] - B[k-1], 1, same);
// padding gates are zero.  a_L, a_R, a_O go straight into the A_I/A_O/S
// scalar array.  Prefix products: per-lane chunks, then a Hillis-Steele scan
// of the chunk products in LDS.  dynamic LDS = (2 k + 4 blockDim) x 32 B.
__global__ void __launch_bounds__(256) k_witness(uint32_t k, uint32_t n_p, uint32_t per, const uint32_t* __restrict__ pi,
                                                const uint32_t* __restrict__ xs, uint32_t* __restrict__ sc_out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* pref = lds;           // [2][k] prefix products (A then B): Montgomery, then canonical
  uint32_t* scan = lds + 16 * k;  // [2 buffers][2][blockDim] chunk products
  const uint32_t p = blockIdx.x, nt = blockDim.x, t = threadIdx.x;
  const sc x = sc_load(xs + 8 * (size_t)p);
  sc one = sc_zero();
  one.v[0] = 1;
  const sc oneR = sc_to_mont(one);
  // lane t owns elements [i0, i1) of both chains; nch lanes own any
  const uint32_t C = (k + nt - 1) / nt, nch = (k + C - 1) / C, i0 = t * C, i1 = min(i0 + C, k);
  auto dd = [&](uint32_t c, uint32_t i) {  // v_i - x: v = i + 1 (A) or pi(i) + 1 (B)
    sc v = sc_zero();
    v.v[0] = c == 0 ? i + 1 : pi[(size_t)p * k + i] + 1;
    return sc_sub(v, x);
  };
  sc run[2] = {oneR, oneR};
  for (uint32_t i = i0; i < i1; ++i)
    _Pragma("unroll") for (uint32_t c = 0; c < 2; ++c) {
      run[c] = sc_mont(run[c], sc_to_mont(dd(c, i)));
      sc_store(pref + 8 * (c * k + i), run[c]);
    }
  // inclusive Hillis-Steele scan of the chunk products, ping-pong buffers
  uint32_t cur = 0;
  _Pragma("unroll") for (uint32_t c = 0; c < 2; ++c) sc_store(scan + 8 * (c * nt + t), run[c]);
  __syncthreads();
  for (uint32_t d = 1; d < nch; d <<= 1) {
    const uint32_t* src = scan + 16 * nt * cur;
    uint32_t* dst = scan + 16 * nt * (cur ^ 1);
    if (t < nch)
      _Pragma("unroll") for (uint32_t c = 0; c < 2; ++c) {
        sc a = sc_load(src + 8 * (c * nt + t));
        if (t >= d) a = sc_mont(sc_load(src + 8 * (c * nt + t - d)), a);
        sc_store(dst + 8 * (c * nt + t), a);
      }
    cur ^= 1;
    __syncthreads();
  }
  // canonical prefixes: mont(e, P) for the canonical product e of the
  // earlier chunks and Montgomery P is e P canonical (one multiply each)
  if (t < nch)
    _Pragma("unroll") for (uint32_t c = 0; c < 2; ++c) {
      const sc e = t > 0 ? sc_from_mont(sc_load(scan + 16 * nt * cur + 8 * (c * nt + t - 1))) : one;
      for (uint32_t i = i0; i < i1; ++i) sc_store(pref + 8 * (c * k + i), sc_mont(e, sc_load(pref + 8 * (c * k + i))));
    }
  __syncthreads();
  uint32_t* o = sc_out + 8 * (size_t)p * per;
  auto pr = [&](uint32_t c, uint32_t i) { return sc_load(pref + 8 * (c * k + i)); };
  for (uint32_t g = t; g < n_p; g += nt) {
    sc aL = sc_zero(), aR = sc_zero(), aO = sc_zero();
    if (g + 1 < k) {
      aL = pr(0, g);
      aR = dd(0, g + 1);
      aO = pr(0, g + 1);
    } else if (g + 2 < 2 * k) {
      const uint32_t h = g - (k - 1);
      aL = pr(1, h);
      aR = dd(1, h + 1);
      aO = pr(1, h + 1);
    } else if (g == 2 * k - 2) {
      aL = pr(1, k - 1);
      aR = sc_neg(one);
      aO = sc_neg(aL);
    } else if (g == 2 * k - 1) {
      aL = sc_sub(pr(0, k - 1), pr(1, k - 1));
      aR = one;
      aO = aL;
    }
    sc_store(o + 8 * (1 + g), aL);
    sc_store(o + 8 * (1 + n_p + g), aR);
    sc_store(o + 8 * (2 + 2 * n_p + g), aO);
  }
}

int witness_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const uint32_t* d_pi, const uint32_t* d_x,
                uint32_t per, uint32_t* d_sc) {
  if (!P) return BPP_OK;
  // (256 lanes while the prefixes and both scan buffers fit 64 KB, else 128:
  // perm_api's dev_witness bound (2 k + 512) x 32 B)
  const unsigned nt = (2 * (size_t)C.k + 4 * 256) * 32 <= 64 * 1024 ? 256 : 128;
  const size_t lds = (2 * (size_t)C.k + 4 * nt) * 32;
  hipLaunchKernelGGL(k_witness, dim3(P), dim3(nt), lds, ctx->stream, C.k, C.n_p, per, d_pi, d_x, d_sc);
  return ctx_check_launch(ctx, "k_witness");
}

int draws_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const uint64_t* d_tmpl, uint32_t seed_len,
              uint32_t per, uint32_t* d_gamma, uint32_t* d_sc, const uint32_t* d_pi, uint32_t* d_v, uint32_t* d_g,
              uint32_t* d_gx_half) {
  if (!P) return BPP_OK;
  if (seed_len > 32) {
    ctx->err = "draws_dev: seed longer than 32 bytes";
    return BPP_ERR_ARG;
  }
  const size_t nt = (size_t)P * (C.m + 3 + 2 * C.n_p);
  hipLaunchKernelGGL(k_draws, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, ctx->stream, P, C.m, C.n_p, per,
                     (uint32_t)(BPP_DRAW_DOMAIN_LEN + seed_len), d_tmpl, d_gamma, d_sc, C.k, d_pi, d_v, d_g,
                     d_gx_half);
  return ctx_check_launch(ctx, "k_draws");
}

void draw_template(const perm::Seed& seed, uint64_t tmpl[7]) {
  uint8_t b[56] = {0};
  memcpy(b, BPP_DRAW_DOMAIN, BPP_DRAW_DOMAIN_LEN);
  memcpy(b + BPP_DRAW_DOMAIN_LEN, seed.b, seed.len);
  b[BPP_DRAW_DOMAIN_LEN + seed.len + 4] = 0x1F;  // SHAKE's pad byte after le32 j
  memcpy(tmpl, b, 56);
}


namespace {

// Column-CSR of WL, WR, WO over the n_p gate columns: cp[3][n_p + 1],
// entries (q, valR[8]) as 9 words; with_v appends WV over its m columns at
// cp[3 (n_p + 1)] (m + 1 offsets, the verifier's V scalars), then the count
// and list of its heavy columns.
void build_csr(const perm::Circuit& C, std::vector<uint32_t>& cp, std::vector<uint32_t>& ce, bool with_v = false) {
  const uint32_t n_p = C.n_p;
  cp.assign(3 * (n_p + 1) + (with_v ? C.m + 1 : 0), 0);
  ce.clear();
  const std::vector<perm::Entry>* Ws[4] = {&C.WL, &C.WR, &C.WO, &C.WV};
  uint32_t total = 0;
  for (int w = 0; w < (with_v ? 4 : 3); ++w) {
    const uint32_t ncol = w == 3 ? C.m : n_p;
    std::vector<std::vector<const perm::Entry*>> cols(ncol);
    for (const perm::Entry& e : *Ws[w]) cols[e.col].push_back(&e);
    for (uint32_t c = 0; c < ncol; ++c) {
      cp[w * (n_p + 1) + c] = total;
      for (const perm::Entry* e : cols[c]) {
        ce.push_back(e->q);
        uint32_t words[8];
        memcpy(words, e->valR.v, 32);
        ce.insert(ce.end(), words, words + 8);
        ++total;
      }
    }
    cp[w * (n_p + 1) + ncol] = total;
  }
  if (with_v) {  // then the V columns too long for one lane (col_sum_block)
    const uint32_t* cpv = &cp[3 * (n_p + 1)];
    std::vector<uint32_t> heavy;
    for (uint32_t j = 0; j < C.m; ++j)
      if (cpv[j + 1] - cpv[j] > HEAVY_COL) heavy.push_back(j);
    cp.push_back((uint32_t)heavy.size());
    cp.insert(cp.end(), heavy.begin(), heavy.end());
  }
}

unsigned poly_block(uint32_t n_p) { return n_p < 64 ? 64u : (n_p > POLY_T ? POLY_T : n_p); }

}  // namespace

int poly_coef_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const uint32_t* d_sc, uint32_t per,
                  const uint32_t* d_gamma, const std::vector<hsc::Sc>& ch, std::vector<hsc::Sc>& t) {
  std::vector<uint32_t> cp, ce;
  build_csr(C, cp, ce, true);
  void *d_cp, *d_ce, *d_ch, *d_vec, *d_hf, *d_t;
  BPP_TRY(ctx_ws(ctx, "poly_cp", cp.size() * 4, &d_cp));
  BPP_TRY(ctx_ws(ctx, "poly_ce", ce.size() * 4 + 4, &d_ce));

  BPP_TRY(ctx_ws(ctx, "poly_vec", (size_t)P * C.n_p * POLY_SLOTS * 32, &d_vec));
  BPP_TRY(ctx_ws(ctx, "poly_hf", (size_t)P * C.n_p * 32, &d_hf));
  {  // challenges in, t out: pinned host memory the kernel reads / writes in place
    uint32_t *hc = nullptr, *ht = nullptr;
    BPP_TRY(ctx_zc_in(ctx, "poly_ch_h", ch.data(), ch.size() * 32, &hc));
    BPP_TRY(ctx_zc_out(ctx, "poly_t_h", (size_t)P * POLY_NT * 32, &ht));
    d_ch = hc;
    d_t = ht;
  }
  BPP_TRY(ctx_h2d_const(ctx, "poly_cp", d_cp, cp.data(), cp.size() * 4));  // the circuit: same every batch
  BPP_TRY(ctx_h2d_const(ctx, "poly_ce", d_ce, ce.data(), ce.size() * 4));
  const unsigned nt = poly_block(std::max(C.n_p, C.m));
  const size_t lds = ((size_t)C.Q + 1 + 2 * std::min(C.n_p, (uint32_t)POW_LO)) * 32 + (POLY_T / 64) * POLY_NT * 32;
  {
    ProfScope ps(ctx, "poly_coef");
    hipLaunchKernelGGL(k_poly_coef, dim3(P), dim3(nt), lds, ctx->stream, C.n_p, C.m, C.Q, per, d_sc,
                       (const uint32_t*)d_ch, (const uint32_t*)d_cp, (const uint32_t*)d_ce, d_gamma,
                       (uint32_t*)d_vec, (uint32_t*)d_hf, (uint32_t*)d_t);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_poly_coef"));
  t.resize((size_t)P * POLY_NT);
  BPP_TRY(ctx_sync(ctx));
  memcpy(t.data(), d_t, (size_t)P * POLY_NT * 32);
  return BPP_OK;
}

int poly_x_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const std::vector<hsc::Sc>& x, uint32_t** d_l,
               uint32_t** d_r, uint32_t** d_hf, std::vector<hsc::Sc>& t_hat) {
  void *d_x, *d_vec, *d_lo, *d_ro, *d_th, *hf;

  BPP_TRY(ctx_ws(ctx, "poly_vec", (size_t)P * C.n_p * POLY_SLOTS * 32, &d_vec));
  BPP_TRY(ctx_ws(ctx, "poly_hf", (size_t)P * C.n_p * 32, &hf));
  BPP_TRY(ctx_ws(ctx, "pf_l", (size_t)P * C.n_p * 32 + 32, &d_lo));
  BPP_TRY(ctx_ws(ctx, "pf_r", (size_t)P * C.n_p * 32 + 32, &d_ro));
  {  // x in, t_hat out: in place in pinned host memory
    uint32_t *hx = nullptr, *hth = nullptr;
    BPP_TRY(ctx_zc_in(ctx, "poly_x_h", x.data(), (size_t)P * 32, &hx));
    BPP_TRY(ctx_zc_out(ctx, "poly_that_h", (size_t)P * 32, &hth));
    d_x = hx;
    d_th = hth;
  }
  {
    ProfScope ps(ctx, "poly_x");
    hipLaunchKernelGGL(k_poly_x, dim3(P), dim3(poly_block(C.n_p)), 0, ctx->stream, C.n_p, (const uint32_t*)d_x,
                       (const uint32_t*)d_vec, (uint32_t*)d_lo, (uint32_t*)d_ro, (uint32_t*)d_th);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_poly_x"));
  t_hat.resize(P);
  BPP_TRY(ctx_sync(ctx));
  memcpy(t_hat.data(), d_th, (size_t)P * 32);
  *d_l = (uint32_t*)d_lo;
  *d_r = (uint32_t*)d_ro;
  *d_hf = (uint32_t*)hf;
  return BPP_OK;
}

int verify_scalars_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const std::vector<uint32_t>& rec,
                       const uint8_t seed[32], uint64_t first, uint32_t* d_sc) {
  uint32_t *h = nullptr, *hs = nullptr;  // per-proof records read in place from pinned host memory (ctx_zc_in)
  BPP_TRY(ctx_zc_in(ctx, "vs_rec_h", rec.data(), rec.size() * 4, &h));
  BPP_TRY(ctx_zc_in(ctx, "vs_seed_h", seed, 32, &hs));
  return verify_scalars_dev_rec(ctx, C, count, h, hs, first, d_sc);
}

int verify_scalars_dev_rec(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_rec,
                           const uint32_t* seed, uint64_t first, uint32_t* d_sc) {
  std::vector<uint32_t> cp, ce;
  build_csr(C, cp, ce, true);
  std::vector<uint32_t> cw((size_t)C.Q * 8);
  for (uint32_t q = 0; q < C.Q; ++q) memcpy(&cw[8 * (size_t)q], C.c[q].v, 32);
  const uint32_t NG = 2 * C.n_p + 2, npt = C.m + 8 + 2 * C.lg;
  void *d_cp, *d_ce, *d_c, *d_gen;
  BPP_TRY(ctx_ws(ctx, "vs_cp", cp.size() * 4, &d_cp));
  BPP_TRY(ctx_ws(ctx, "vs_ce", ce.size() * 4 + 4, &d_ce));
  BPP_TRY(ctx_ws(ctx, "vs_c", cw.size() * 4, &d_c));

  BPP_TRY(ctx_ws(ctx, "vs_gen", (size_t)count * NG * 32, &d_gen));
  BPP_TRY(ctx_h2d_const(ctx, "vs_cp", d_cp, cp.data(), cp.size() * 4));  // the circuit: same every batch
  BPP_TRY(ctx_h2d_const(ctx, "vs_ce", d_ce, ce.data(), ce.size() * 4));
  BPP_TRY(ctx_h2d_const(ctx, "vs_c", d_c, cw.data(), cw.size() * 4));
  const unsigned nt = poly_block(std::max(C.n_p, C.m));
  const size_t lds = ((size_t)C.Q + 1 + 2 * std::min(C.n_p, (uint32_t)POW_LO)) * 32 + (POLY_T / 64) * 2 * 32;
  if (C.lg > VC_LGMAX) return BPP_ERR_LEN;  // (k_verify_consts' LDS tables)
  void* d_kc = nullptr;
  BPP_TRY(ctx_ws(ctx, "vs_kc", (size_t)count * VK_N * 32, &d_kc));
  {
    ProfScope ps(ctx, "verify_scalars");
    hipLaunchKernelGGL(k_verify_consts, dim3((count + VC_P - 1) / VC_P), dim3(64 * (VC_W + 1)), 0, ctx->stream, count,
                       C.lg, first, seed, d_rec, (uint32_t*)d_kc, NG, C.m, npt, d_sc);
    hipLaunchKernelGGL(k_verify_scalars, dim3(count), dim3(nt), lds, ctx->stream, C.n_p, C.m, C.Q, C.lg, d_rec,
                       (const uint32_t*)d_kc, (const uint32_t*)d_cp, (const uint32_t*)d_ce, (const uint32_t*)d_c,
                       (uint32_t*)d_gen, d_sc, NG, npt);
    hipLaunchKernelGGL(k_verify_merge, dim3(NG), dim3(POLY_T), 0, ctx->stream, count, NG, (const uint32_t*)d_gen,
                       d_sc);
  }
  return ctx_check_launch(ctx, "k_verify_scalars/merge");
}
