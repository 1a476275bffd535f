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
#include <cstring>

#include "ctx.h"
#include "ipa.h"
#include "msm_engine.h"
#include "sc25519.cuh"

static unsigned grid_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

__global__ void __launch_bounds__(256) k_ipa_init(uint32_t n, const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                           const uint32_t* __restrict__ gf, const uint32_t* __restrict__ hf, uint32_t* __restrict__ am,
                           uint32_t* __restrict__ bm, uint32_t* __restrict__ fG, uint32_t* __restrict__ fH) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  sc_store(am + 8 * k, sc_to_mont(sc_load(a + 8 * k)));
  sc_store(bm + 8 * k, sc_to_mont(sc_load(b + 8 * k)));
  sc one = sc_zero();
  one.v[0] = 1;
  sc_store(fG + 8 * k, gf ? sc_load(gf + 8 * k) : one);
  sc_store(fH + 8 * k, hf ? sc_load(hf + 8 * k) : one);
}

// terms of L at [0, n+1), of R at [n+1, 2n+2); slots n and 2n+1 (Q) are
// written by k_ipa_cross_final.
__global__ void __launch_bounds__(256) k_ipa_terms(uint32_t n, uint32_t m, uint32_t lg_h, const uint32_t* __restrict__ am,
                            const uint32_t* __restrict__ bm, const uint32_t* __restrict__ fG,
                            const uint32_t* __restrict__ fH, uint32_t gbase, uint32_t hbase,
                            uint32_t* __restrict__ scal, uint32_t* __restrict__ pidx) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t h = m >> 1;
  const uint32_t r = k & (m - 1);
  const bool hi = (r & h) != 0;
  const uint32_t p = r ^ h;
  const uint32_t cidx = ((k >> (lg_h + 1)) << lg_h) | (k & (h - 1));
  const sc sG = sc_mont(sc_load(am + 8 * p), sc_load(fG + 8 * k));  // canonical a_p * fG_k
  const sc sH = sc_mont(sc_load(bm + 8 * p), sc_load(fH + 8 * k));
  const uint32_t posG = hi ? cidx : (n + 1) + cidx;
  const uint32_t posH = hi ? (n + 1) + (n >> 1) + cidx : (n >> 1) + cidx;
  sc_store(scal + 8 * posG, sG);
  sc_store(scal + 8 * posH, sH);
  pidx[posG] = gbase + k;
  pidx[posH] = hbase + k;
}

#define CROSS_T 256
__global__ void __launch_bounds__(CROSS_T) k_ipa_cross(uint32_t h, const uint32_t* __restrict__ am,
                                                      const uint32_t* __restrict__ bm, uint32_t* __restrict__ part) {
  __shared__ uint32_t lds[2][CROSS_T / 64][8];
  sc cl = sc_zero(), cr = sc_zero();
  for (uint32_t i = blockIdx.x * CROSS_T + threadIdx.x; i < h; i += gridDim.x * CROSS_T) {
    const sc a0 = sc_load(am + 8 * i), a1 = sc_load(am + 8 * (i + h));
    const sc b0 = sc_load(bm + 8 * i), b1 = sc_load(bm + 8 * (i + h));
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
    sc_store(part + 16 * blockIdx.x, sl);
    sc_store(part + 16 * blockIdx.x + 8, sr);
  }
}

__global__ void __launch_bounds__(64) k_ipa_cross_final(uint32_t nblk, const uint32_t* __restrict__ part, sc qmul, uint32_t qidx, uint32_t n,
                                  uint32_t* __restrict__ scal, uint32_t* __restrict__ pidx) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  sc sl = sc_zero(), sr = sc_zero();
  for (uint32_t b = 0; b < nblk; ++b) {
    sl = sc_add(sl, sc_load(part + 16 * b));
    sr = sc_add(sr, sc_load(part + 16 * b + 8));
  }
  // Montgomery c * canonical qmul -> canonical c*qmul
  sc_store(scal + 8 * n, sc_mont(sl, qmul));
  sc_store(scal + 8 * (2 * n + 1), sc_mont(sr, qmul));
  pidx[n] = qidx;
  pidx[2 * n + 1] = qidx;
}

__global__ void __launch_bounds__(256) k_ipa_fold(uint32_t n, uint32_t m, uint32_t* __restrict__ am, uint32_t* __restrict__ bm,
                           uint32_t* __restrict__ fG, uint32_t* __restrict__ fH, sc um, sc uim) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t h = m >> 1;
  const bool hi = ((k & (m - 1)) & h) != 0;
  // G' = u^-1 G_lo + u G_hi ; H' = u H_lo + u^-1 H_hi
  sc_store(fG + 8 * k, sc_mont(sc_load(fG + 8 * k), hi ? um : uim));
  sc_store(fH + 8 * k, sc_mont(sc_load(fH + 8 * k), hi ? uim : um));
  if (k < h) {
    const sc a0 = sc_load(am + 8 * k), a1 = sc_load(am + 8 * (k + h));
    const sc b0 = sc_load(bm + 8 * k), b1 = sc_load(bm + 8 * (k + h));
    sc_store(am + 8 * k, sc_add(sc_mont(a0, um), sc_mont(a1, uim)));
    sc_store(bm + 8 * k, sc_add(sc_mont(b0, uim), sc_mont(b1, um)));
  }
}

static sc to_dev_sc(const hsc::Sc& x) {
  sc r;
  for (int i = 0; i < 4; ++i) {
    r.v[2 * i] = (uint32_t)x.v[i];
    r.v[2 * i + 1] = (uint32_t)(x.v[i] >> 32);
  }
  return r;
}

static hsc::Sc from_dev_words(const uint32_t w[8]) {
  hsc::Sc r;
  for (int i = 0; i < 4; ++i) r.v[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  return r;
}

int ipa_prove_dev(bpp_ctx* ctx, merlin::Transcript& tr, const IpaGens& g, uint32_t n, const uint32_t* d_Gf,
                  const uint32_t* d_Hf, const uint32_t* d_a, const uint32_t* d_b, IpaProofHost& out) {
  if (n == 0 || (n & (n - 1))) {
    ctx->err = "ipa: n must be a power of two";
    return BPP_ERR_LEN;
  }
  tr.innerproduct_domain_sep(n);
  out.L.clear();
  out.R.clear();
  void *am, *bm, *fG, *fH, *scal, *pidx, *part;
  BPP_TRY(ctx_ws(ctx, "ipa_am", (size_t)n * 32, &am));
  BPP_TRY(ctx_ws(ctx, "ipa_bm", (size_t)n * 32, &bm));
  BPP_TRY(ctx_ws(ctx, "ipa_fG", (size_t)n * 32, &fG));
  BPP_TRY(ctx_ws(ctx, "ipa_fH", (size_t)n * 32, &fH));
  BPP_TRY(ctx_ws(ctx, "ipa_scal", (size_t)(2 * n + 2) * 32, &scal));
  BPP_TRY(ctx_ws(ctx, "ipa_pidx", (size_t)(2 * n + 2) * 4, &pidx));
  const uint32_t cross_blocks = std::min<uint32_t>(64, grid_for(std::max<uint32_t>(n / 2, 1), CROSS_T));
  BPP_TRY(ctx_ws(ctx, "ipa_part", (size_t)cross_blocks * 64, &part));
  hipLaunchKernelGGL(k_ipa_init, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, n, d_a, d_b, d_Gf, d_Hf,
                     (uint32_t*)am, (uint32_t*)bm, (uint32_t*)fG, (uint32_t*)fH);
  BPP_TRY(ctx_check_launch(ctx, "k_ipa_init"));
  const sc qmul = to_dev_sc(g.qmul);
  uint32_t m = n;
  uint32_t lg_h = 0;
  while ((1u << (lg_h + 1)) < n) ++lg_h;  // log2(n/2)
  std::vector<h25519::ge> res;
  while (m > 1) {
    const uint32_t h = m >> 1;
    {
      ProfScope ps(ctx, "ipa_terms");
      hipLaunchKernelGGL(k_ipa_terms, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, n, m, lg_h,
                         (const uint32_t*)am, (const uint32_t*)bm, (const uint32_t*)fG, (const uint32_t*)fH, g.gbase,
                         g.hbase, (uint32_t*)scal, (uint32_t*)pidx);
      const uint32_t nb = std::min<uint32_t>(cross_blocks, grid_for(h, CROSS_T));
      hipLaunchKernelGGL(k_ipa_cross, dim3(nb), dim3(CROSS_T), 0, ctx->stream, h, (const uint32_t*)am,
                         (const uint32_t*)bm, (uint32_t*)part);
      hipLaunchKernelGGL(k_ipa_cross_final, dim3(1), dim3(64), 0, ctx->stream, nb, (const uint32_t*)part, qmul, g.qidx,
                         n, (uint32_t*)scal, (uint32_t*)pidx);
    }
    BPP_TRY(ctx_check_launch(ctx, "ipa round kernels"));
    const std::vector<uint32_t> off = {0, n + 1, 2 * n + 2};
    BPP_TRY(msm_multi(ctx, (const uint32_t*)scal, (const uint32_t*)pidx, off, g.d_tbl, g.d_tbl1, g.n0, res));
    Enc32 Le, Re;
    h25519::encode(Le.data(), res[0]);
    h25519::encode(Re.data(), res[1]);
    out.L.push_back(Le);
    out.R.push_back(Re);
    tr.append_point("L", Le.data());
    tr.append_point("R", Re.data());
    const hsc::Sc u = tr.challenge_scalar("u");
    const hsc::Sc ui = hsc::invert(u);
    const sc um = to_dev_sc(hsc::mul(u, SC_R_MOD_L));
    const sc uim = to_dev_sc(hsc::mul(ui, SC_R_MOD_L));
    {
      ProfScope ps(ctx, "ipa_fold");
      hipLaunchKernelGGL(k_ipa_fold, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, n, m, (uint32_t*)am,
                         (uint32_t*)bm, (uint32_t*)fG, (uint32_t*)fH, um, uim);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_ipa_fold"));
    m = h;
    if (lg_h) --lg_h;
  }
  uint32_t ab[16];
  BPP_HIP(hipMemcpyAsync(ab, am, 32, hipMemcpyDeviceToHost, ctx->stream));
  BPP_HIP(hipMemcpyAsync(ab + 8, bm, 32, hipMemcpyDeviceToHost, ctx->stream));
  BPP_HIP(hipStreamSynchronize(ctx->stream));
  out.a = hsc::mont(from_dev_words(ab), hsc::one());
  out.b = hsc::mont(from_dev_words(ab + 8), hsc::one());
  return BPP_OK;
}

bool ipa_verification_scalars(merlin::Transcript& tr, uint32_t n, const std::vector<Enc32>& L,
                              const std::vector<Enc32>& R, std::vector<hsc::Sc>& u_sq,
                              std::vector<hsc::Sc>& uinv_sq, std::vector<hsc::Sc>& s) {
  const size_t lg_n = L.size();
  if (lg_n >= 32 || R.size() != lg_n || n != (1u << lg_n)) return false;
  tr.innerproduct_domain_sep(n);
  std::vector<hsc::Sc> u(lg_n);
  for (size_t j = 0; j < lg_n; ++j) {
    if (!tr.validate_and_append_point("L", L[j].data())) return false;
    if (!tr.validate_and_append_point("R", R[j].data())) return false;
    u[j] = tr.challenge_scalar("u");
  }
  std::vector<hsc::Sc> ui = u;
  const hsc::Sc allinv = hsc::batch_invert(ui);
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
