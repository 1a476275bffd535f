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
  // non-null: Q given as its 253 doublings 2^j Q (device P3 rows) instead of
  // a generator: the fused rounds add c Q bit by bit, one lane per bit, into
  // the block tree (no per-call Q table; qidx / qmul unused)
  const uint32_t* qpow = nullptr;
};

typedef std::array<uint8_t, 32> Enc32;

struct IpaProofHost {
  std::vector<Enc32> L, R;
  hsc::Sc a, b;
};

// The transcript of ONE inner-product argument, as bulletproofs 4.0.0 drives
// it: innerproduct_domain_sep(n) = append_message("dom-sep", "ipp v1") +
// append_u64("n", n); per round append_point("L"), append_point("R"),
// challenge_scalar("u") = 64 challenge bytes reduced wide
// (transcript_protocol.rs:26-67).  Two primitives are all it needs, so a
// caller-owned merlin::Transcript can sit behind C hooks (bpp_ipa_prove_cb);
// a false return (a hook failed) aborts the IPA.
struct IpaTranscript {
  virtual ~IpaTranscript() = default;
  virtual bool append(const char* label, const uint8_t* msg, size_t n) = 0;
  virtual bool challenge(const char* label, uint8_t* out, size_t n) = 0;
  bool domain_sep(uint64_t n) {
    uint8_t le[8];
    memcpy(le, &n, 8);
    return append("dom-sep", (const uint8_t*)"ipp v1", 6) && append("n", le, 8);
  }
  bool challenge_scalar(const char* label, hsc::Sc& out) {
    uint8_t buf[64];
    if (!challenge(label, buf, 64)) return false;
    out = hsc::from_wide(buf);
    return true;
  }
};

// The library's own Merlin behind that interface (bpp_transcript*).
struct IpaMerlin final : IpaTranscript {
  merlin::Transcript& t;
  explicit IpaMerlin(merlin::Transcript& tr) : t(tr) {}
  bool append(const char* label, const uint8_t* msg, size_t n) override {
    t.append(label, msg, n);
    return true;
  }
  bool challenge(const char* label, uint8_t* out, size_t n) override {
    t.challenge_bytes(label, out, n);
    return true;
  }
};

// a, b, Gf, Hf: device arrays of n canonical scalars (Gf/Hf may be null =
// all ones).  a and b are consumed.  BPP_ERR_CALLBACK when a transcript hook
// fails.
int ipa_prove_dev(bpp_ctx* ctx, IpaTranscript& tr, const IpaGens& g, uint32_t n, const uint32_t* d_Gf,
                  const uint32_t* d_Hf, const uint32_t* d_a, const uint32_t* d_b, IpaProofHost& out);

// P instances in lockstep (one per transcript): d_a, d_b, d_Gf, d_Hf are
// [P][n] (Gf/Hf may be null); Q_p = qmul[p] * P[g.qidx].  `one` (P = 1, trs
// ignored): the single instance's transcript behind the generic interface.
int ipa_prove_batch_dev(bpp_ctx* ctx, const std::vector<merlin::Transcript*>& trs, const IpaGens& g, uint32_t n,
                        const uint32_t* d_Gf, const uint32_t* d_Hf, const uint32_t* d_a, const uint32_t* d_b,
                        const std::vector<hsc::Sc>& qmul, std::vector<IpaProofHost>& out,
                        IpaTranscript* one = nullptr);

// Replays the verifier side of the transcript; returns false on malformed
// proof (identity L/R, wrong length) or a failed hook (*hook_failed set).
// Fills u^2, u^-2 and s (bulletproofs verification_scalars).
bool ipa_verification_scalars(IpaTranscript& tr, uint32_t n, const std::vector<Enc32>& L,
                              const std::vector<Enc32>& R, std::vector<hsc::Sc>& u_sq,
                              std::vector<hsc::Sc>& uinv_sq, std::vector<hsc::Sc>& s, bool* hook_failed = nullptr);

static const hsc::Sc SC_R_MOD_L = {{0xd6ec31748d98951dULL, 0xc6ef5bf4737dcf70ULL, 0xfffffffffffffffeULL,
                                    0x0fffffffffffffffULL}};
