// Internal view of bpp_gens (see gens.hip).
#pragma once
#include <stdint.h>

#include <mutex>
#include <vector>

#include "ctx.h"
#include "msm_engine.h"

#define FB_POS 64  // radix-16 positions per fixed base
#define GENS_DT_MAX 4096  // generators for which direct tables are kept (c >= 8: 2 GB at the limit)
// c = 16 (W = 16 windows, 17.3 GB for the 258 generators of a 52-card
// proof) against c = 13 (W = 20, 2.7 GB): 20 % fewer table additions per
// term; 12 batches in flight 141.5-146.8 K vs 120.7-137.5 K proofs/s, but one
// batch alone 4.6 vs 3.8 ms (a lone batch's row gathers into 17 GB miss the
// caches and TLBs with nothing to hide them)
#ifndef GENS_DT_BUDGET
#define GENS_DT_BUDGET (32ull << 30)  // HBM for one generator set's direct tables (288 GB per GPU)
#endif
#ifndef GENS_DT_TOTAL
#define GENS_DT_TOTAL (80ull << 30)  // all live generator sets' direct tables in one process
#endif
#ifndef GENS_DT_CMAX
#define GENS_DT_CMAX 16  // widest direct-table window (2^15 rows per window)
#endif

struct bpp_gens {
  bpp_ctx* ctx = nullptr;
  size_t n = 0;
  uint32_t* d_tbl = nullptr;  // (2n+2) affine Niels: G[0..n) H[n..2n) B[2n] Bb[2n+1]
  uint32_t* d_fb = nullptr;   // fixed-base tables for B and Bb: 2 x 64 x 8 Niels
  // window tables of every generator (FBW_W x 128 B each), built on first use
  mutable uint32_t* d_wt = nullptr;
  // direct tables d * 2^(c w) * P (d <= 2^(c-1), w < ceil(254 / c)), built
  // on first use when 2n+2 <= GENS_DT_MAX, c the widest window within
  // GENS_DT_BUDGET (gens_points)
  mutable uint32_t* d_dt = nullptr;
  mutable uint32_t dt_c = 8;
  // guards the first-use builds of d_wt / d_dt: contexts on other streams
  // (bpp_perm_prove_batch sub-batches, callers sharing one gens across
  // threads) may ask for the tables at the same time
  mutable std::mutex build_mu;
  // bpp_ipa_prove's Q (an arbitrary point): its Niels row at d_tbl[2n + 2]
  // and its direct-table rows at generator slot 2n + 2 of d_dt, written per
  // call under q_mu (ipa_api.hip ipa_q_slot), so that the IPA rounds run
  // fused over the direct tables like the prover's, whose Q is a multiple
  // of the resident B
  mutable std::mutex q_mu;
  uint32_t qslot() const { return (uint32_t)(2 * n + 2); }
  uint32_t gidx(size_t i) const { return (uint32_t)i; }
  uint32_t hidx(size_t i) const { return (uint32_t)(n + i); }
  uint32_t bidx() const { return (uint32_t)(2 * n); }
  uint32_t bbidx() const { return (uint32_t)(2 * n + 1); }
};

// Builds g->d_wt if needed; fills a MsmPoints view (tbl = generators,
// wt = their window tables).
int gens_points(bpp_ctx* ctx, const bpp_gens* g, MsmPoints* out);
// v_bound: 0, or a public bound every v is below (fewer positions for v)
int pedersen_dev(bpp_ctx* ctx, const bpp_gens* g, const uint32_t* d_v, const uint32_t* d_gam, size_t m,
                 uint32_t* d_out_enc, uint32_t* d_out_p3,
                 uint64_t v_bound = 0);
