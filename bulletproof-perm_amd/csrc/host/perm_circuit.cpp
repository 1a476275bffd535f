// Permutation circuit (sound mode) — see perm.h and oracle/bulletproofs.py
// perm_circuit / perm_witness (the checker this must agree with).
//
// Reference shape (weights.rs:63-113 create_a, weights.rs:130-204
// create_weights): n = 2k multiplication gates forming two product chains
// prod_i (v_i - x) and prod_i (v'_i - x), a negation gate and a final
// difference gate whose output is constrained to 0.  Fixes: the final gate
// combines the END of chain A (a_O[k-2]; weights.rs:106 used a_O[offset]),
// a_O[n-1] = a_L * a_R (weights.rs:108 squared a_L), and x is a transcript
// challenge bound to the committed v_2k by the last row (weights.rs:50 fixed
// x = 1).  Rows: a_L (2k), a_R (2k), a_O[n-1] = 0, v_2k = x  => Q = 4k + 2.
#include <errno.h>
#include <sys/random.h>
#include "par.h"
#include "perm.h"

namespace perm {

using hsc::Sc;

Circuit build(uint32_t k) {
  Circuit C;
  C.k = k;
  C.n = 2 * k;
  C.n_p = 1;
  while (C.n_p < C.n) C.n_p *= 2;
  while ((1u << C.lg) < C.n_p) ++C.lg;
  C.Q = 4 * k + 2;
  C.m = 2 * k + 1;
  const uint32_t X = 2 * k;
  const Sc one = hsc::one(), neg1 = hsc::neg(hsc::one());
  C.c.assign(C.Q, hsc::zero());
  for (uint32_t g = 0; g < C.n; ++g) {  // a_L rows
    C.WL.push_back({g, g, one});
    if (g == 0) {
      C.WV.push_back({g, 0, one});
      C.WV.push_back({g, X, neg1});
    } else if (g == k - 1) {
      C.WV.push_back({g, k, one});
      C.WV.push_back({g, X, neg1});
    } else if (g == 2 * k - 1) {
      C.WO.push_back({g, k - 2, neg1});
      C.WO.push_back({g, 2 * k - 2, neg1});
    } else {
      C.WO.push_back({g, g - 1, neg1});
    }
  }
  for (uint32_t g = 0; g < C.n; ++g) {  // a_R rows
    const uint32_t q = C.n + g;
    C.WR.push_back({q, g, one});
    if (g + 2 <= k) {  // g <= k-2
      C.WV.push_back({q, g + 1, one});
      C.WV.push_back({q, X, neg1});
    } else if (g + 3 <= 2 * k) {  // g <= 2k-3
      C.WV.push_back({q, g + 2, one});
      C.WV.push_back({q, X, neg1});
    } else if (g == 2 * k - 2) {
      C.c[q] = neg1;
    } else {
      C.c[q] = one;
    }
  }
  C.WO.push_back({4 * k, 2 * k - 1, one});
  C.WV.push_back({4 * k + 1, X, one});
  for (auto* W : {&C.WL, &C.WR, &C.WO, &C.WV})
    for (Entry& e : *W) e.valR = hsc::to_mont(e.val);
  return C;
}

void witness(const Circuit& C, const std::vector<uint32_t>& pi, const Sc& x, std::vector<Sc>& v, std::vector<Sc>& aL,
             std::vector<Sc>& aR, std::vector<Sc>& aO) {
  const uint32_t k = C.k, n = C.n;
  v.assign(C.m, hsc::zero());
  for (uint32_t i = 0; i < k; ++i) {
    v[i] = hsc::from_u64(i + 1);
    v[k + i] = hsc::from_u64(pi[i] + 1);
  }
  v[2 * k] = x;
  aL.assign(C.n_p, hsc::zero());
  aR.assign(C.n_p, hsc::zero());
  aO.assign(C.n_p, hsc::zero());
  for (uint32_t g = 0; g + 1 < k; ++g) {
    aL[g] = g == 0 ? hsc::sub(v[0], x) : aO[g - 1];
    aR[g] = hsc::sub(v[g + 1], x);
    aO[g] = hsc::mul(aL[g], aR[g]);
  }
  for (uint32_t g = k - 1; g + 2 < 2 * k; ++g) {
    aL[g] = g == k - 1 ? hsc::sub(v[k], x) : aO[g - 1];
    aR[g] = hsc::sub(v[g + 2], x);
    aO[g] = hsc::mul(aL[g], aR[g]);
  }
  uint32_t g = 2 * k - 2;
  aL[g] = aO[2 * k - 3];
  aR[g] = hsc::neg(hsc::one());
  aO[g] = hsc::mul(aL[g], aR[g]);
  g = n - 1;
  aL[g] = hsc::add(aO[k - 2], aO[2 * k - 2]);
  aR[g] = hsc::one();
  aO[g] = hsc::mul(aL[g], aR[g]);
}

std::vector<Sc> zW(const std::vector<Entry>& W, const std::vector<Sc>& zq, uint32_t ncols) {
  std::vector<Sc> out(ncols, hsc::zero());
  for (const Entry& e : W) out[e.col] = hsc::add(out[e.col], hsc::mulm(zq[e.q], e.valR));
  return out;
}

std::vector<uint32_t> fisher_yates(uint32_t k, Rng& rng) {
  std::vector<uint32_t> p(k);
  for (uint32_t i = 0; i < k; ++i) p[i] = i;
  for (uint32_t i = k - 1; i > 0; --i) {
    const uint32_t j = (uint32_t)(rng.u64() % (uint64_t)(i + 1));
    std::swap(p[i], p[j]);
  }
  return p;
}

Sc draw_scalar(const Seed& seed, uint32_t j) {
  merlin::Shake256 sh;
  sh.update((const uint8_t*)BPP_DRAW_DOMAIN, BPP_DRAW_DOMAIN_LEN);
  sh.update(seed.b, seed.len);
  const uint8_t jb[4] = {(uint8_t)j, (uint8_t)(j >> 8), (uint8_t)(j >> 16), (uint8_t)(j >> 24)};
  sh.update(jb, 4);
  uint8_t b[64];
  sh.read(b, 64);
  return hsc::from_wide(b);
}

void draw_prover_randomness(const Circuit& C, const Seed& seed, std::vector<uint32_t>& pi, std::vector<Sc>& gamma,
                            Sc& alpha, Sc& beta, Sc& rho, std::vector<Sc>& sL, std::vector<Sc>& sR,
                            std::vector<Sc>& taus) {
  Rng rng("bpperm-prove", seed);
  pi = fisher_yates(C.k, rng);
  uint32_t j = 0;
  gamma.resize(C.m);
  for (auto& g : gamma) g = draw_scalar(seed, j++);
  alpha = draw_scalar(seed, j++);
  beta = draw_scalar(seed, j++);
  rho = draw_scalar(seed, j++);
  sL.resize(C.n_p);
  sR.resize(C.n_p);
  taus.resize(5);
  for (auto& x : sL) x = draw_scalar(seed, j++);
  for (auto& x : sR) x = draw_scalar(seed, j++);
  for (auto& x : taus) x = draw_scalar(seed, j++);
}

size_t proof_len(uint32_t k) {
  Circuit C;
  uint32_t n_p = 1, lg = 0;
  while (n_p < 2 * k) n_p *= 2;
  while ((1u << lg) < n_p) ++lg;
  (void)C;
  // A_I A_O S T1 T3 T4 T5 T6 | tau_x mu t_hat | (L_j R_j) x lg | a b
  return 32 * (8 + 3 + 2 * lg + 2);
}

hsc::Sc batch_weight(const uint8_t seed[32], uint64_t p, const hsc::Sc& r) {
  merlin::Shake256 sh;
  sh.update((const uint8_t*)"bp-perm-batch-wt", 16);
  sh.update(seed, 32);
  sh.update((const uint8_t*)&p, 8);
  sh.update((const uint8_t*)&r, 32);  // (canonical Sc == its 32 bytes)
  uint8_t o[64];
  sh.read(o, 64);
  return hsc::from_wide(o);
}

bool verify_seed(uint8_t seed[32]) {
  size_t got = 0;
  while (got < 32) {
    const ssize_t n = getrandom(seed + got, 32 - got, 0);
    if (n > 0)
      got += (size_t)n;
    else if (n < 0 && errno != EINTR)
      return false;
  }
  return true;
}

}  // namespace perm
