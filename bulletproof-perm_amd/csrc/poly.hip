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
//                (workgroup reduction) -> host for the T commitments
//   k_poly_x     l = l(x), r = r(x) straight into the IPA's input arrays,
//                t_hat = <l, r> -> host
// Identical values to the host formulas they replace (perm_api.hip history;
// oracle/bulletproofs.py prove()), hence identical proof bytes (tests).
#include <cstring>

#include "ctx.h"
#include "poly.h"
#include "sc25519.cuh"

#define POLY_SLOTS 7  // l1 r0 r1 r3 l2 l3 (Montgomery) per gate
#define POLY_T 256    // lanes per proof; lane i handles gates i, i + POLY_T, ...

FE_INLINE sc sc_one_mont() {
  sc one = sc_zero();
  one.v[0] = 1;
  return sc_to_mont(one);
}

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

// grid = P proofs, block = poly_block(n_p); dynamic LDS = Q * 32 + (POLY_T / 64) * 6 * 32
__global__ void __launch_bounds__(POLY_T) k_poly_coef(uint32_t n_p, uint32_t Q, uint32_t per,
                                                   const uint32_t* __restrict__ sc_in,
                                                   const uint32_t* __restrict__ ch,
                                                   const uint32_t* __restrict__ cp, const uint32_t* __restrict__ ce,
                                                   uint32_t* __restrict__ vec, uint32_t* __restrict__ hf,
                                                   uint32_t* __restrict__ t_out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* zp = lds;           // [Q] z^(q+1)
  uint32_t* red = lds + 8 * Q;  // reduction scratch
  const uint32_t p = blockIdx.x;
  const sc oneR = sc_one_mont();
  const sc yR = sc_to_mont(sc_load(ch + 24 * p)), yiR = sc_to_mont(sc_load(ch + 24 * p + 8)),
           zR = sc_to_mont(sc_load(ch + 24 * p + 16));
  for (uint32_t q = threadIdx.x; q < Q; q += blockDim.x) sc_store(zp + 8 * q, sc_pow_small(zR, q + 1, oneR));
  __syncthreads();
  sc t[6];
  _Pragma("unroll") for (int j = 0; j < 6; ++j) t[j] = sc_zero();
  for (uint32_t i = threadIdx.x; i < n_p; i += blockDim.x) {
    const uint32_t* s = sc_in + (size_t)p * per * 8;
    const sc aL = sc_to_mont(sc_load(s + 8 * (1 + i)));
    const sc aR = sc_to_mont(sc_load(s + 8 * (1 + n_p + i)));
    const sc l2 = sc_to_mont(sc_load(s + 8 * (2 + 2 * n_p + i)));  // a_O
    const sc l3 = sc_to_mont(sc_load(s + 8 * (3 + 3 * n_p + i)));  // s_L
    const sc sR = sc_to_mont(sc_load(s + 8 * (3 + 4 * n_p + i)));
    const sc yp = sc_pow_small(yR, i, oneR), yip = sc_pow_small(yiR, i, oneR);
    const sc zWL = col_sum(cp, ce, i, zp), zWR = col_sum(cp + (n_p + 1), ce, i, zp),
             zWO = col_sum(cp + 2 * (n_p + 1), ce, i, zp);
    const sc l1 = sc_add(aL, sc_mont(zWR, yip));
    const sc r0 = sc_sub(zWO, yp);
    const sc r1 = sc_add(sc_mont(aR, yp), zWL);
    const sc r3 = sc_mont(sR, yp);
    t[0] = sc_add(t[0], sc_mont(l1, r0));
    t[1] = sc_add(t[1], sc_add(sc_mont(l1, r1), sc_mont(l2, r0)));
    t[2] = sc_add(t[2], sc_add(sc_mont(l2, r1), sc_mont(l3, r0)));
    t[3] = sc_add(t[3], sc_add(sc_mont(l1, r3), sc_mont(l3, r1)));
    t[4] = sc_add(t[4], sc_mont(l2, r3));
    t[5] = sc_add(t[5], sc_mont(l3, r3));
    uint32_t* v = vec + ((size_t)p * n_p + i) * POLY_SLOTS * 8;
    sc_store(v + 0, l1);
    sc_store(v + 8, r0);
    sc_store(v + 16, r1);
    sc_store(v + 24, r3);
    sc_store(v + 32, l2);
    sc_store(v + 40, l3);
    sc_store(hf + ((size_t)p * n_p + i) * 8, sc_from_mont(yip));  // H factors y^-i
  }
  sc_block_sum<6>(t, red);
  if (threadIdx.x == 0)
    _Pragma("unroll") for (int j = 0; j < 6; ++j) sc_store(t_out + (6 * p + j) * 8, sc_from_mont(t[j]));
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

namespace {

// Column-CSR of WL, WR, WO over the n_p gate columns: cp[3][n_p + 1],
// entries (q, valR[8]) as 9 words.
void build_csr(const perm::Circuit& C, std::vector<uint32_t>& cp, std::vector<uint32_t>& ce) {
  const uint32_t n_p = C.n_p;
  cp.assign(3 * (n_p + 1), 0);
  ce.clear();
  const std::vector<perm::Entry>* Ws[3] = {&C.WL, &C.WR, &C.WO};
  uint32_t total = 0;
  for (int w = 0; w < 3; ++w) {
    std::vector<std::vector<const perm::Entry*>> cols(n_p);
    for (const perm::Entry& e : *Ws[w]) cols[e.col].push_back(&e);
    for (uint32_t c = 0; c < n_p; ++c) {
      cp[w * (n_p + 1) + c] = total;
      for (const perm::Entry* e : cols[c]) {
        ce.push_back(e->q);
        uint32_t words[8];
        memcpy(words, e->valR.v, 32);
        ce.insert(ce.end(), words, words + 8);
        ++total;
      }
    }
    cp[w * (n_p + 1) + n_p] = total;
  }
}

unsigned poly_block(uint32_t n_p) { return n_p < 64 ? 64u : (n_p > POLY_T ? POLY_T : n_p); }

}  // namespace

int poly_coef_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const uint32_t* d_sc, uint32_t per,
                  const std::vector<hsc::Sc>& ch, std::vector<hsc::Sc>& t) {
  std::vector<uint32_t> cp, ce;
  build_csr(C, cp, ce);
  void *d_cp, *d_ce, *d_ch, *d_vec, *d_hf, *d_t;
  BPP_TRY(ctx_ws(ctx, "poly_cp", cp.size() * 4, &d_cp));
  BPP_TRY(ctx_ws(ctx, "poly_ce", ce.size() * 4 + 4, &d_ce));
  BPP_TRY(ctx_ws(ctx, "poly_ch", ch.size() * 32, &d_ch));
  BPP_TRY(ctx_ws(ctx, "poly_vec", (size_t)P * C.n_p * POLY_SLOTS * 32, &d_vec));
  BPP_TRY(ctx_ws(ctx, "poly_hf", (size_t)P * C.n_p * 32, &d_hf));
  BPP_TRY(ctx_ws(ctx, "poly_t", (size_t)P * 6 * 32, &d_t));
  BPP_TRY(ctx_h2d_const(ctx, "poly_cp", d_cp, cp.data(), cp.size() * 4));  // the circuit: same every batch
  BPP_TRY(ctx_h2d_const(ctx, "poly_ce", d_ce, ce.data(), ce.size() * 4));
  BPP_TRY(ctx_h2d(ctx, d_ch, ch.data(), ch.size() * 32));
  const unsigned nt = poly_block(C.n_p);
  const size_t lds = (size_t)C.Q * 32 + (POLY_T / 64) * 6 * 32;
  {
    ProfScope ps(ctx, "poly_coef");
    hipLaunchKernelGGL(k_poly_coef, dim3(P), dim3(nt), lds, ctx->stream, C.n_p, C.Q, per, d_sc,
                       (const uint32_t*)d_ch, (const uint32_t*)d_cp, (const uint32_t*)d_ce, (uint32_t*)d_vec,
                       (uint32_t*)d_hf, (uint32_t*)d_t);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_poly_coef"));
  t.resize((size_t)P * 6);
  return ctx_d2h(ctx, t.data(), d_t, (size_t)P * 6 * 32);
}

int poly_x_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const std::vector<hsc::Sc>& x, uint32_t** d_l,
               uint32_t** d_r, uint32_t** d_hf, std::vector<hsc::Sc>& t_hat) {
  void *d_x, *d_vec, *d_lo, *d_ro, *d_th, *hf;
  BPP_TRY(ctx_ws(ctx, "poly_x", (size_t)P * 32, &d_x));
  BPP_TRY(ctx_ws(ctx, "poly_vec", (size_t)P * C.n_p * POLY_SLOTS * 32, &d_vec));
  BPP_TRY(ctx_ws(ctx, "poly_hf", (size_t)P * C.n_p * 32, &hf));
  BPP_TRY(ctx_ws(ctx, "pf_l", (size_t)P * C.n_p * 32 + 32, &d_lo));
  BPP_TRY(ctx_ws(ctx, "pf_r", (size_t)P * C.n_p * 32 + 32, &d_ro));
  BPP_TRY(ctx_ws(ctx, "poly_that", (size_t)P * 32, &d_th));
  BPP_TRY(ctx_h2d(ctx, d_x, x.data(), (size_t)P * 32));
  {
    ProfScope ps(ctx, "poly_x");
    hipLaunchKernelGGL(k_poly_x, dim3(P), dim3(poly_block(C.n_p)), 0, ctx->stream, C.n_p, (const uint32_t*)d_x,
                       (const uint32_t*)d_vec, (uint32_t*)d_lo, (uint32_t*)d_ro, (uint32_t*)d_th);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_poly_x"));
  t_hat.resize(P);
  BPP_TRY(ctx_d2h(ctx, t_hat.data(), d_th, (size_t)P * 32));
  *d_l = (uint32_t*)d_lo;
  *d_r = (uint32_t*)d_ro;
  *d_hf = (uint32_t*)hf;
  return BPP_OK;
}
