// Permutation circuit + arithmetic-circuit proof (sound mode) — host side.
//
// Restates the reference's ACProof::ArithmeticCircuitProof
// (bp-perm/src/circuit_lib.rs:139-585) and the permutation circuit of
// weights.rs:26-204 in their sound form (SURVEY.md §2.2 defects Q1-Q10
// fixed; DESIGN.md "Protocol"), with every group operation dropped through
// the GPU (MSM engine, fixed-base Pedersen, IPA).  Matrices are sparse
// (the reference's dense Q x n matrices are 99.4 % zeros).
#pragma once
#include <stdint.h>

#include <array>
#include <vector>

#include "merlin.h"
#include "scalar.h"

namespace perm {

struct Entry {
  uint32_t q, col;
  hsc::Sc val;
  hsc::Sc valR;  // Montgomery form of val (zW products in one step)
};

struct Circuit {
  uint32_t k = 0, n = 0, n_p = 0, lg = 0, Q = 0, m = 0;
  std::vector<Entry> WL, WR, WO, WV;
  std::vector<hsc::Sc> c;  // c[Q-1] = -x set per proof
};

Circuit build(uint32_t k);

// v = [1..k, pi(1..k), x]; gate values (sound create_a)
void witness(const Circuit& C, const std::vector<uint32_t>& pi, const hsc::Sc& x, std::vector<hsc::Sc>& v,
             std::vector<hsc::Sc>& aL, std::vector<hsc::Sc>& aR, std::vector<hsc::Sc>& aO);

// (z^Q)^T W as a dense vector of length ncols
std::vector<hsc::Sc> zW(const std::vector<Entry>& W, const std::vector<hsc::Sc>& zq, uint32_t ncols);

// Prover seed: the 8-byte little-endian u64 of the deterministic test
// entry points (bpp_perm_prove / _batch) or 32 bytes of caller / OS entropy
// (bpp_perm_prove_batch_entropy), absorbed after the domain string.
struct Seed {
  uint8_t b[32] = {0};
  uint32_t len = 8;
  static Seed u64(uint64_t x) {
    Seed s;
    memcpy(s.b, &x, 8);
    s.len = 8;
    return s;
  }
  static Seed bytes32(const uint8_t* p) {
    Seed s;
    memcpy(s.b, p, 32);
    s.len = 32;
    return s;
  }
};

// SHAKE256(domain || seed bytes) byte stream (oracle/merlin.py Rng)
struct Rng {
  merlin::Shake256 sh;
  Rng(const char* domain, const Seed& seed) {
    sh.update((const uint8_t*)domain, strlen(domain));
    sh.update(seed.b, seed.len);
  }
  Rng(const char* domain, uint64_t seed) : Rng(domain, Seed::u64(seed)) {}
  void bytes(uint8_t* out, size_t n) { sh.read(out, n); }
  uint64_t u64() {
    uint8_t b[8];
    bytes(b, 8);
    uint64_t x;
    memcpy(&x, b, 8);
    return x;
  }
  hsc::Sc scalar() {
    uint8_t b[64];
    bytes(b, 64);
    return hsc::from_wide(b);
  }
};

std::vector<uint32_t> fisher_yates(uint32_t k, Rng& rng);

// The prover's random draws (the stand-in for thread_rng,
// circuit_lib.rs:175): pi by Fisher-Yates from the stream
// SHAKE256("bpperm-prove" || seed), one u64 per step; the blinding scalars
// by index j in the order gamma[m], alpha, beta, rho, s_L[n_p], s_R[n_p],
// tau[5], scalar j = from_wide(SHAKE256("bpperm-prove-sc" || seed ||
// le32 j)[0..64]) (draw_scalar; oracle/merlin.py indexed_scalar) -- one
// sponge block per draw, so the GPU makes every draw in its own thread
// (poly.h draws_dev).
void draw_prover_randomness(const Circuit& C, const Seed& seed, std::vector<uint32_t>& pi, std::vector<hsc::Sc>& gamma,
                            hsc::Sc& alpha, hsc::Sc& beta, hsc::Sc& rho, std::vector<hsc::Sc>& sL,
                            std::vector<hsc::Sc>& sR, std::vector<hsc::Sc>& taus);
#define BPP_DRAW_DOMAIN "bpperm-prove-sc"
#define BPP_DRAW_DOMAIN_LEN 15
hsc::Sc draw_scalar(const Seed& seed, uint32_t j);
inline uint32_t draw_alpha_index(const Circuit& C) { return C.m; }            // then beta, rho
inline uint32_t draw_tau_index(const Circuit& C) { return C.m + 3 + 2 * C.n_p; }  // tau[5]
inline uint32_t draw_count(const Circuit& C) { return C.m + 3 + 2 * C.n_p + 5; }

struct RandomDraws {
  std::vector<uint32_t> pi;
  std::vector<hsc::Sc> gamma, sL, sR, taus;
  hsc::Sc alpha, beta, rho;
};
// The draws of eight proofs at once: the eight pi streams and each index's
// eight scalar sponges run through an AVX-512 8-way Keccak
// (host/keccak_x8.cpp; scalar fallback without AVX-512), identical to
// draw_prover_randomness.  (the eight seeds must have the same length)
void draw_prover_randomness_x8(const Circuit& C, const Seed seeds[8], RandomDraws* const out[8]);
// As above, but only the host's share -- pi, alpha, beta, rho and tau: the
// GPU draws gamma, s_L and s_R (and alpha, beta, rho again, into its scalar
// arrays; poly.h draws_dev), and out[j]'s vectors for them are left empty.
void draw_prover_host_x8(const Circuit& C, const Seed seeds[8], RandomDraws* const out[8]);

size_t proof_len(uint32_t k);

// Batch-verification weight of proof p (its index in the batch) with weight
// challenge r_p (its own transcript's "t-check-weight"):
//   w_p = from_bytes_mod_order_wide(SHAKE256("bp-perm-batch-wt" || seed ||
//         le64 p || r_p)[0..64])
// seed = 32 bytes of the VERIFIER's randomness (getrandom; every rank of a
// split batch uses the same seed), mixed with the proof's own transcript
// challenge as bulletproofs' r1cs batch verifier mixes its external rng into
// each proof's TranscriptRng.  The weights need nothing from the other
// proofs, so they are made in each proof's own GPU lane right after its
// replay (DESIGN.md §5 "Batch weights").  A seed the provers can predict
// voids the batch's soundness.
hsc::Sc batch_weight(const uint8_t seed[32], uint64_t p, const hsc::Sc& r);
// 32 bytes from the OS CSPRNG (getrandom); false if it fails
bool verify_seed(uint8_t seed[32]);

}  // namespace perm
