// Inner-product argument (bulletproofs 4.0.0 InnerProductProof) — internal API.
#pragma once
#include <array>
#include <vector>

#include "ctx.h"
#include "host/merlin.h"
#include "host/scalar.h"
#include "msm_engine.h"

// widest IPA run as one launch per round (k_ipa_round_dt; its LDS holds the
// n + 1 terms and the round's a, b: 102 KB at n = 1024, within gfx950's 160 KB
// per workgroup; 0 builds the four-kernel rounds everywhere, for A/B runs)
#ifndef IPA_FUSED_NMAX
#define IPA_FUSED_NMAX 1024
#endif

struct IpaGens {
  MsmPoints pts;                      // generators (+ window tables), extra points from n0
  uint32_t gbase = 0, hbase = 0;     // G_i at gbase + i, H_i at hbase + i
  uint32_t qidx = 0;                 // Q = qmul * P[qidx]
  hsc::Sc qmul = hsc::one();
};

typedef std::array<uint8_t, 32> Enc32;

struct IpaProofHost {
  std::vector<Enc32> L, R;
  hsc::Sc a, b;
};

// a, b, Gf, Hf: device arrays of n canonical scalars (Gf/Hf may be null =
// all ones).  a and b are consumed.
int ipa_prove_dev(bpp_ctx* ctx, merlin::Transcript& tr, const IpaGens& g, uint32_t n, const uint32_t* d_Gf,
                  const uint32_t* d_Hf, const uint32_t* d_a, const uint32_t* d_b, IpaProofHost& out);

// P instances in lockstep (one per transcript): d_a, d_b, d_Gf, d_Hf are
// [P][n] (Gf/Hf may be null); Q_p = qmul[p] * P[g.qidx].
int ipa_prove_batch_dev(bpp_ctx* ctx, const std::vector<merlin::Transcript*>& trs, const IpaGens& g, uint32_t n,
                        const uint32_t* d_Gf, const uint32_t* d_Hf, const uint32_t* d_a, const uint32_t* d_b,
                        const std::vector<hsc::Sc>& qmul, std::vector<IpaProofHost>& out);

// Replays the verifier side of the transcript; returns false on malformed
// proof (identity L/R, wrong length).  Fills u^2, u^-2 and s (bulletproofs
// verification_scalars).
bool ipa_verification_scalars(merlin::Transcript& tr, uint32_t n, const std::vector<Enc32>& L,
                              const std::vector<Enc32>& R, std::vector<hsc::Sc>& u_sq,
                              std::vector<hsc::Sc>& uinv_sq, std::vector<hsc::Sc>& s);

static const hsc::Sc SC_R_MOD_L = {{0xd6ec31748d98951dULL, 0xc6ef5bf4737dcf70ULL, 0xfffffffffffffffeULL,
                                    0x0fffffffffffffffULL}};
