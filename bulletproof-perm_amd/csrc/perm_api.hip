// Permutation proof: sound-mode arithmetic-circuit prover / verifier over
// the GPU primitives (C ABI bpp_perm_*).
//
// Restates ACProof::ArithmeticCircuitProof (bp-perm/src/circuit_lib.rs):
//   create                 :139-253  -> V (fixed-base Pedersen), A_I/A_O/S
//                                       (one 3-MSM batch)
//   challenge_wit_and_const:133-138  -> y, z
//   compute_per_challenges :256-302  -> y^n, y^-n (batch inversion), z^Q W
//                                       (sparse, host)
//   commit_Ts              :304-423  -> t_1..t_6 (host), T_i (fixed-base)
//   random_chall_x         :425-432  -> x
//   blinding_values        :434-476  -> l, r, t_hat, tau_x, mu; the clear
//                                       l, r of :466-467 replaced by an IPA
//   verify                 :478-585  -> ONE GPU MSM (t-check weighted by a
//                                       verifier challenge + the IPA check,
//                                       generator scalars merged)
// Transcript order and RNG draw order match oracle/bulletproofs.py
// ac_prove / ac_verify exactly (tests compare proof bytes).
#include <cerrno>
#include <cstring>
#include <cstdlib>
#include <sys/random.h>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>

#include "ctx.h"
#include "gens.h"
#include "host/par.h"
#include "host/perm.h"
#include "ipa.h"
#include "msm_engine.h"
#include "poly.h"
#include "layout.h"
#include "verify_dev.h"
#include "merlin_dev.h"

using hsc::Sc;

int decompress_ws(bpp_ctx* ctx, const uint8_t* enc, size_t count, const char* name, uint32_t** d_out);
// declared in points.hip
__global__ void k_decompress(const uint32_t* __restrict__ enc, size_t n, uint32_t* __restrict__ tbl,
                             unsigned long long* __restrict__ bad);

namespace {

struct Proof {
  std::vector<Enc32> V;
  Enc32 AI, AO, S, T[5];
  Sc tau_x, mu, t_hat;
  IpaProofHost ipa;
  std::vector<uint32_t> pi;  // prover side only
};

void put_sc(std::vector<uint8_t>& buf, const Sc& s) {
  uint8_t b[32];
  hsc::to_bytes(b, s);
  buf.insert(buf.end(), b, b + 32);
}

void serialize(const perm::Circuit& C, const Proof& P, uint8_t* out) {
  std::vector<uint8_t> b;
  b.reserve(perm::proof_len(C.k));
  for (const Enc32* e : {&P.AI, &P.AO, &P.S, &P.T[0], &P.T[1], &P.T[2], &P.T[3], &P.T[4]})
    b.insert(b.end(), e->begin(), e->end());
  put_sc(b, P.tau_x);
  put_sc(b, P.mu);
  put_sc(b, P.t_hat);
  for (uint32_t j = 0; j < C.lg; ++j) {
    b.insert(b.end(), P.ipa.L[j].begin(), P.ipa.L[j].end());
    b.insert(b.end(), P.ipa.R[j].begin(), P.ipa.R[j].end());
  }
  put_sc(b, P.ipa.a);
  put_sc(b, P.ipa.b);
  memcpy(out, b.data(), b.size());
}

bool deserialize(const perm::Circuit& C, const uint8_t* in, size_t len, const uint8_t* V, Proof& P) {
  if (len != perm::proof_len(C.k)) return false;
  size_t o = 0;
  auto pt = [&](Enc32& e) {
    memcpy(e.data(), in + o, 32);
    o += 32;
  };
  auto sc = [&](Sc& s) {
    bool ok = hsc::from_canonical(s, in + o);
    o += 32;
    return ok;
  };
  pt(P.AI);
  pt(P.AO);
  pt(P.S);
  for (int i = 0; i < 5; ++i) pt(P.T[i]);
  if (!sc(P.tau_x) || !sc(P.mu) || !sc(P.t_hat)) return false;
  P.ipa.L.resize(C.lg);
  P.ipa.R.resize(C.lg);
  for (uint32_t j = 0; j < C.lg; ++j) {
    pt(P.ipa.L[j]);
    pt(P.ipa.R[j]);
  }
  if (!sc(P.ipa.a) || !sc(P.ipa.b)) return false;
  P.V.resize(C.m);
  for (uint32_t j = 0; j < C.m; ++j) memcpy(P.V[j].data(), V + 32 * j, 32);
  return true;
}

std::vector<uint8_t> to_bytes(const std::vector<Sc>& v) {
  std::vector<uint8_t> b(v.size() * 32);
  for (size_t i = 0; i < v.size(); ++i) hsc::to_bytes(b.data() + 32 * i, v[i]);
  return b;
}

// Small vectors go to pinned host memory the kernels read in place (no copy
// launch, ctx_zc_in); large ones (vector commitments of many terms, whose
// scalars every window lane re-reads) are copied to the device.
#define UPLOAD_ZC_MAX (256u << 10)
int upload_sc(bpp_ctx* ctx, const std::vector<Sc>& v, const char* name, uint32_t** d) {
  static_assert(sizeof(Sc) == 32, "Sc is the 32-byte little-endian scalar");  // canonical Sc == its bytes
  if (v.size() * 32 <= UPLOAD_ZC_MAX) return ctx_zc_in(ctx, name, v.data(), v.size() * 32, d);
  void* p = nullptr;
  BPP_TRY(ctx_ws(ctx, name, v.size() * 32 + 32, &p));
  BPP_TRY(ctx_h2d(ctx, p, v.data(), v.size() * 32));
  *d = (uint32_t*)p;
  return BPP_OK;
}

// Fixed-base commitments v_i*B + g_i*Bb, returned compressed.
// Small batches (<= PED_DOUBLE_MAX) commit with halved scalars and encode
// C = 2 (C / 2) on the host (points_double_encode_p3): one inversion per
// chunk instead of a ~70 us per-point inverse-square-root chain on the GPU.
#define PED_DOUBLE_MAX 2048
int pedersen_host(bpp_ctx* ctx, const bpp_gens* g, const std::vector<Sc>& v, const std::vector<Sc>& gam,
                  std::vector<Enc32>& out) {
  const size_t m = v.size();
  // (encoding the 13 312 V commitments of a 128-proof batch this way too
  // measured slower at 8 batches in flight, 72-77 K vs 80-83 K proofs/s:
  // the host is loaded as well)
  const bool doubled = m <= PED_DOUBLE_MAX;
  uint32_t *d_v, *d_g;
  {
    HostScope hs(ctx, "ped_upload");
    if (doubled) {
      std::vector<Sc> hv(m), hg(m);
      for (size_t i = 0; i < m; ++i) {
        hv[i] = hsc::half(v[i]);
        hg[i] = hsc::half(gam[i]);
      }
      BPP_TRY(upload_sc(ctx, hv, "pp_v", &d_v));
      BPP_TRY(upload_sc(ctx, hg, "pp_g", &d_g));
    } else {
      BPP_TRY(upload_sc(ctx, v, "pp_v", &d_v));
      BPP_TRY(upload_sc(ctx, gam, "pp_g", &d_g));
    }
  }
  out.resize(m);
  if (doubled) {
    uint32_t* h_p3 = nullptr;  // written in place by the kernel (ctx_zc_out)
    BPP_TRY(ctx_zc_out(ctx, "pp_p3_h", m * P3_BYTES, &h_p3));
    {
      HostScope hs(ctx, "ped_kernels");
      BPP_TRY(pedersen_dev(ctx, g, d_v, d_g, m, nullptr, h_p3));
    }
    HostScope hs(ctx, "ped_d2h");
    BPP_TRY(ctx_sync(ctx));
    return points_double_encode_host(ctx, h_p3, m, out[0].data());
  }
  void* d_out = nullptr;
  BPP_TRY(ctx_ws(ctx, "pp_out", m * 32, &d_out));
  {
    HostScope hs(ctx, "ped_kernels");
    BPP_TRY(pedersen_dev(ctx, g, d_v, d_g, m, (uint32_t*)d_out, nullptr));
  }
  HostScope hs(ctx, "ped_d2h");
  BPP_TRY(ctx_d2h(ctx, out.data(), d_out, m * 32));
  return BPP_OK;
}

int msm_terms(bpp_ctx* ctx, const std::vector<Sc>& sc, const std::vector<uint32_t>& idx,
              const std::vector<uint32_t>& off, const MsmPoints& pts, std::vector<h25519::ge>& res) {
  uint32_t* d_s = nullptr;
  BPP_TRY(upload_sc(ctx, sc, "mt_s", &d_s));
  void* d_i = nullptr;
  BPP_TRY(ctx_ws(ctx, "mt_i", idx.size() * 4 + 4, &d_i));
  BPP_TRY(ctx_h2d_const(ctx, "mt_i", d_i, idx.data(), idx.size() * 4));
  return msm_multi(ctx, d_s, (const uint32_t*)d_i, off, pts, res);
}

// The prover's V transcript phase on the device (k_prove_v_transcript,
// BPP_PROVE_DEV_V=1) instead of the host's 8-way lockstep Keccak.  Off:
// measured 244-250 K vs 264-266 K proofs/s at 256 x 12 in flight (three
// interleaved passes, tools/gpu_ab_env_prove.sh) -- the host is not the
// bound (8 of 16 cores busy), and the 4-wave kernel's ~0.3 ms latency
// lands on every batch's critical path.
bool dev_v_transcript() {
  const char* e = getenv("BPP_PROVE_DEV_V");
  return e && atoi(e) != 0;
}

// Per-proof prover state carried between the lockstep phases.  The states
// (and their vectors) persist per driver thread across batches: a host
// profile of 8 batches in flight spent ~20 % of the host CPU in malloc /
// free and arena locks, largely vectors allocated by pool workers and freed
// by the driver thread at the end of every batch.
// Batch-sized host arrays, also reused batch after batch (resize to the same
// size neither allocates nor zero-fills; every element is written before use).
struct ProverScratch {
  std::vector<Enc32> V;
  // A_I/A_O/S MSM terms without the zero padding gates (a_L, a_R, a_O of
  // gates 2k..n_p-1): generator index and source slot in the [P][per]
  // scalar array per term, rebuilt when (P, k, generator set) changes: the
  // indices embed G->n (hidx(i) = n + i, bbidx() = 2n + 1), so one thread
  // proving the same (P, k) against generator sets of different sizes must
  // not reuse them
  std::vector<uint32_t> idx, map, off;
  size_t key_P = 0;
  uint32_t key_k = 0;
  const bpp_gens* key_G = nullptr;
  size_t key_n = 0;
};

struct ProverState {
  merlin::Transcript tr;
  perm::RandomDraws d;  // pi, gamma, alpha, beta, rho, s_L, s_R, tau
  std::vector<Sc> vals, aL, aR, aO;
  Sc x_perm, w;
  Sc t[7];
};

std::vector<std::unique_ptr<ProverState>>& prover_states_tl() {
  static thread_local std::vector<std::unique_ptr<ProverState>> S;
  return S;
}
std::vector<Proof>& proofs_tl();

// Wipes what the last batch proved on this thread and context left of its
// secrets: the pinned-arena spans the batch staged secrets in
// (draw templates and pi; the witness and blindings on the host-witness path,
// k > 768), the device workspaces holding blindings, witness and the l / r
// vectors, the host buffers of the T-commitment inputs, and the calling
// thread's reused prover states and proof objects (pi).  Called by the
// production entry point (bpp_perm_prove_batch_entropy) on its context, and
// by each sub-batch thread on its child context (BPP_PROVE_STREAMS > 1).
static const char* const kSecretWs[] = {"pb_rng_in", "pb_gamma", "mt_s",  "pv_v",   "pv_g",    "pv_gx",  "poly_vec",
                                        "poly_hf",   "pf_l",     "pf_r",  "ipa_am", "ipa_bm",  "ipa_am1", "ipa_bm1"};
static const char* const kSecretHost[] = {"pp_v", "pp_g", "ipa_zc_a", "ipa_zc_b"};  // (ipa_zc_*: bpp_ipa_prove zeroes them itself)
// The device workspaces of kSecretWs zeroed by ONE launch (blockIdx.y = span)
// instead of one hipMemsetAsync (a fill kernel each) per workspace.
#define WIPE_MAX 16
struct WipeSpans {
  uint8_t* p[WIPE_MAX];
  uint64_t n[WIPE_MAX];
};
static_assert(sizeof(kSecretWs) / sizeof(kSecretWs[0]) <= WIPE_MAX, "WipeSpans too small");
__global__ void __launch_bounds__(256) k_wipe_spans(WipeSpans w) {
  uint8_t* p = w.p[blockIdx.y];
  const uint64_t n = w.n[blockIdx.y], n16 = n >> 4;  // (hipMalloc'd: 16-B aligned)
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint4*>(p)[i] = make_uint4(0, 0, 0, 0);
  if (blockIdx.x == 0 && threadIdx.x < (n & 15)) p[n16 * 16 + threadIdx.x] = 0;
}
int prove_wipe(bpp_ctx* ctx) {
  WipeSpans w = {};
  uint32_t cnt = 0;
  uint64_t most = 0;
  for (const char* n : kSecretWs) {
    auto it = ctx->ws.find(n);
    if (it == ctx->ws.end() || !it->second.p || !it->second.bytes) continue;
    w.p[cnt] = (uint8_t*)it->second.p;
    w.n[cnt] = it->second.bytes;
    most = std::max<uint64_t>(most, it->second.bytes);
    ++cnt;
  }
  if (cnt) {
    const uint32_t bx = (uint32_t)std::min<uint64_t>(64, (most / 16 + 255) / 256 + 1);
    hipLaunchKernelGGL(k_wipe_spans, dim3(bx, cnt), dim3(256), 0, ctx->stream, w);
    BPP_TRY(ctx_check_launch(ctx, "k_wipe_spans"));
  }
  BPP_TRY(ctx_sync(ctx));
  for (const char* n : kSecretHost) {
    auto it = ctx->host_bufs.find(n);
    if (it != ctx->host_bufs.end() && it->second.first) memset(it->second.first, 0, it->second.second);
  }
  for (auto& st : ctx->secret_stage) memset(st.first, 0, st.second);
  ctx->wiped.swap(ctx->secret_stage);
  ctx->secret_stage.clear();
  for (auto& S : prover_states_tl()) {
    perm::RandomDraws& d = S->d;
    std::fill(d.pi.begin(), d.pi.end(), 0u);
    for (auto* v : {&d.gamma, &d.sL, &d.sR, &d.taus, &S->vals, &S->aL, &S->aR, &S->aO})
      std::fill(v->begin(), v->end(), hsc::zero());
    d.alpha = d.beta = d.rho = hsc::zero();
    for (Sc& t : S->t) t = hsc::zero();
  }
  for (Proof& P : proofs_tl()) std::fill(P.pi.begin(), P.pi.end(), 0u);
  return BPP_OK;
}

// Test hook (bpp_debug_secret_residue): nonzero bytes left in what prove_wipe
// zeroes on ctx and its child contexts (device workspaces, host buffers, the
// arena spans of the last wipe).
static int secret_residue(bpp_ctx* ctx, uint64_t* nz) {
  std::vector<uint8_t> h;
  for (const char* n : kSecretWs) {
    auto it = ctx->ws.find(n);
    if (it == ctx->ws.end() || !it->second.p) continue;
    h.resize(it->second.bytes);
    BPP_HIP(hipMemcpy(h.data(), it->second.p, h.size(), hipMemcpyDeviceToHost));
    for (uint8_t b : h) *nz += b != 0;
  }
  for (const char* n : kSecretHost) {
    auto it = ctx->host_bufs.find(n);
    if (it == ctx->host_bufs.end() || !it->second.first) continue;
    const uint8_t* b = (const uint8_t*)it->second.first;
    for (size_t i = 0; i < it->second.second; ++i) *nz += b[i] != 0;
  }
  for (auto& st : ctx->wiped)
    for (size_t i = 0; i < st.second; ++i) *nz += st.first[i] != 0;
  for (bpp_ctx* kid : ctx->children)
    if (kid) BPP_TRY(secret_residue(kid, nz));
  return BPP_OK;
}

// Proves `seeds.size()` permutation proofs in lockstep: every GPU step
// (Pedersen V, Pedersen V_2k, the A_I/A_O/S MSMs, Pedersen T, each IPA
// round) is ONE launch sequence for the whole batch, and the per-proof host
// work between them (transcripts, challenges, polynomial coefficients) runs
// on a thread pool.  Outputs are identical to proving one at a time.
int prove_batch(bpp_ctx* ctx, const bpp_gens* G, const perm::Circuit& C, const std::vector<perm::Seed>& seeds,
                const uint8_t* label, size_t llen, std::vector<Proof>& Ps) {
  const uint32_t k = C.k, n_p = C.n_p, m = C.m;
  const size_t P = seeds.size();
  Ps.resize(P);
  if (!P) return BPP_OK;
  // A small batch is a latency chain (a config-4 job's sub-batches): its
  // syncs spin before sleeping; the throughput shape (384 proofs, 32 in
  // flight) keeps the sleeping wait that frees the host cores
  // (BPP_SPIN_BATCH = the largest batch that spins, 0 = none)
  static const size_t spin_batch = [] {
    const char* e = getenv("BPP_SPIN_BATCH");
    return e ? (size_t)std::max(0, atoi(e)) : (size_t)128;
  }();
  SyncSpin spin(ctx, P <= spin_batch ? 300u : ctx->sync_spin_us);
  // (a plain reference: pool workers must reach THIS thread's states, a
  // thread_local named inside their lambdas would be their own)
  std::vector<std::unique_ptr<ProverState>>& S = prover_states_tl();
  while (S.size() < P) S.emplace_back(new ProverState());
  par::for_each(P, [&](size_t p) { S[p]->tr = merlin::Transcript(label, llen); });
  static thread_local ProverScratch scr_tl;
  ProverScratch& scr = scr_tl;
  std::vector<merlin::Transcript*> trs(P);  // this batch's transcripts (lockstep_x8)
  for (size_t p = 0; p < P; ++p) trs[p] = &S[p]->tr;
  const auto for_groups = [](size_t n, const std::function<void(size_t)>& f) { par::for_each(n, f); };

  const uint32_t per = 3 + 5 * n_p;  // A_I/A_O/S terms per proof
  // the witness on the device (k_witness) while its prefix products fit the
  // workgroup's LDS; the host restatement beyond that
  const bool dev_witness = (2 * (size_t)k + 512) * 32 <= 64 * 1024;
  // RNG draws (perm.h draw_prover_randomness): the host makes pi (its short
  // SHAKE256 streams, 8-way AVX-512 Keccak) and alpha, beta, rho, tau; the
  // GPU makes the 2 n_p + m + 3 indexed scalar draws its kernels use (k_draws:
  // gamma -> [P][m], alpha .. s_R -> their slots of the A_I/A_O/S scalar
  // array) from per-proof sponge templates written straight into the pinned
  // upload arena
  std::unique_ptr<HostScope> hs(new HostScope(ctx, "pb_rng"));
  uint32_t *d_gamma = nullptr, *d_s = nullptr, *d_pi = nullptr;
  {
    void *dg = nullptr, *dsc = nullptr, *dst = nullptr, *dpi = nullptr;
    const size_t tlen = 7 * sizeof(uint64_t);  // draw template per proof
    for (const perm::Seed& sd : seeds)
      if (sd.len != seeds[0].len) {
        ctx->err = "prove_batch: seeds of different lengths in one batch";
        return BPP_ERR_ARG;
      }
    BPP_TRY(ctx_ws(ctx, "pb_gamma", (size_t)P * m * 32, &dg));
    BPP_TRY(ctx_ws(ctx, "mt_s", (size_t)P * per * 32 + 32, &dsc));
    // templates then pi, one device buffer filled by one copy
    BPP_TRY(ctx_ws(ctx, "pb_rng_in", P * tlen + (size_t)P * k * 4, &dst));
    dpi = (uint8_t*)dst + P * tlen;
    d_gamma = (uint32_t*)dg;
    d_s = (uint32_t*)dsc;
    d_pi = (uint32_t*)dpi;
    // (one staging region: a second take could recycle the arena under the first;
    // read in place instead, by k_draws through LDS, measured within noise)
    uint8_t* stage = nullptr;
    BPP_TRY(ctx_h2d_stage(ctx, P * tlen + (size_t)P * k * 4, &stage));
    ctx_secret_span(ctx, stage, P * tlen + (size_t)P * k * 4);  // (prove_wipe)
    uint8_t* pis = stage + P * tlen;
    par::for_each((P + 7) / 8, [&](size_t gi) {
      perm::Seed sd[8];
      perm::RandomDraws* d[8];
      perm::RandomDraws spare;  // a short last group's padding lanes
      for (size_t j = 0; j < 8; ++j) {
        const bool real = 8 * gi + j < P;
        sd[j] = seeds[std::min(8 * gi + j, P - 1)];
        d[j] = real ? &S[8 * gi + j]->d : &spare;
      }
      perm::draw_prover_host_x8(C, sd, d);
      for (size_t j = 0; j < 8 && 8 * gi + j < P; ++j) {
        const size_t i = 8 * gi + j;
        S[i]->tr.arithmetic_domain_sep(n_p);
        uint64_t tm[7];
        draw_template(sd[j], tm);
        memcpy(stage + i * tlen, tm, tlen);
        memcpy(pis + i * 4 * (size_t)k, S[i]->d.pi.data(), 4 * (size_t)k);
      }
#ifdef EXP_HOST_BURN_US  // timing experiment only: extra host CPU per proof
      const auto t0 = std::chrono::steady_clock::now();
      while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(8 * EXP_HOST_BURN_US)) {
      }
#endif
    });
    BPP_TRY(ctx_h2d_staged(ctx, dst, stage, P * tlen + (size_t)P * k * 4));  // (pis follows the templates)
    // (the V commitments' inputs in the same launch: values 1..k and pi + 1,
    // gamma copies and gamma_2k / 2, into the V phase's workspaces)
    void *dv = nullptr, *dgv = nullptr, *dgx = nullptr;
    BPP_TRY(ctx_ws(ctx, "pv_v", (size_t)P * 2 * k * 32, &dv));
    BPP_TRY(ctx_ws(ctx, "pv_g", (size_t)P * 2 * k * 32, &dgv));
    BPP_TRY(ctx_ws(ctx, "pv_gx", (size_t)P * 32, &dgx));
    BPP_TRY(draws_dev(ctx, C, (uint32_t)P, (const uint64_t*)dst, P ? seeds[0].len : 0, per, d_gamma, d_s, d_pi,
                      (uint32_t*)dv, (uint32_t*)dgv, (uint32_t*)dgx));
  }
  // V_0..V_2k-1 of every proof: one fixed-base launch over device inputs
  // (values 1..k, pi + 1 and gamma, written by k_draws), encodings back to the host
  hs.reset(new HostScope(ctx, "pb_pedersen_V"));
  uint32_t* d_gx_half = nullptr;  // gamma_2k / 2 for V_2k
  {
    void *dv = nullptr, *dg = nullptr, *dgx = nullptr, *denc = nullptr;
    const size_t nv = (size_t)P * 2 * k;
    BPP_TRY(ctx_ws(ctx, "pv_v", nv * 32, &dv));
    BPP_TRY(ctx_ws(ctx, "pv_g", nv * 32, &dg));
    BPP_TRY(ctx_ws(ctx, "pv_gx", (size_t)P * 32, &dgx));
    {
      uint32_t* h = nullptr;  // encodings written in place by k_compress_p3 (ctx_zc_out)
      BPP_TRY(ctx_zc_out(ctx, "pv_enc_h", nv * 32, &h));
      denc = h;
    }
    d_gx_half = (uint32_t*)dgx;  // (filled by k_draws above)
    // the 2k V appends and x_perm on the device (k_prove_v_transcript, one
    // lane per proof; the host's share of a batch was ~10 us of CPU per
    // proof here, its largest transcript phase): encodings to the device,
    // copied back for the proofs, and the transcript states imported after
    const bool dev_v = dev_v_transcript();
    uint8_t* h_st = nullptr;
    uint32_t* h_xp = nullptr;
    {
      HostScope hk(ctx, "ped_kernels");
      void* dvenc = nullptr;
      if (dev_v) BPP_TRY(ctx_ws(ctx, "pv_enc_d", nv * 32, &dvenc));
      // (values 1..k and pi + 1 <= k: the public bound k + 1)
      BPP_TRY(pedersen_dev(ctx, G, (const uint32_t*)dv, (const uint32_t*)dg, nv,
                           dev_v ? (uint32_t*)dvenc : (uint32_t*)denc, nullptr, (uint64_t)k + 1));
      if (dev_v) {
        BPP_HIP(hipMemcpyAsync(denc, dvenc, nv * 32, hipMemcpyDeviceToHost, ctx->stream));
        uint32_t init[52], *h_init = nullptr;
        verify_init_state(C, label, llen, init);  // (the same shared prefix as the verifier's)
        BPP_TRY(ctx_zc_in(ctx, "pv_init", init, sizeof init, &h_init));
        uint32_t* hs_ = nullptr;
        BPP_TRY(ctx_zc_out(ctx, "pv_states", P * MERLIN_DEV_STATE_BYTES, &hs_));
        BPP_TRY(ctx_zc_out(ctx, "pv_xperm", P * 32, &h_xp));
        h_st = (uint8_t*)hs_;
        BPP_TRY(prove_v_transcript_dev(ctx, (uint32_t)P, k, h_init, (const uint32_t*)dvenc, h_st, h_xp));
      }
    }
    std::vector<Enc32>& V = scr.V;
    V.resize(nv);
    {
      HostScope hd(ctx, "ped_d2h");
      BPP_TRY(ctx_sync(ctx));
      memcpy(V.data(), denc, nv * 32);
    }
    par::for_each(P, [&](size_t p) {
      Ps[p].V.assign(V.begin() + p * 2 * k, V.begin() + (p + 1) * 2 * k);
      if (dev_v) {
        merlin_state_import(S[p]->tr, h_st + p * MERLIN_DEV_STATE_BYTES);
        memcpy(&S[p]->x_perm, h_xp + 8 * p, 32);  // (canonical Sc == its 32 bytes)
      }
    });
    if (!dev_v) {
      // the 2k "V" appends and x_perm of eight proofs at a time in lockstep
      // on the 8-way Keccak (byte-identical; 2.5x on this phase's ~26 us of
      // permutations per proof)
      merlin::lockstep_x8(
          trs, for_groups,
          [&](merlin::TranscriptX8& T8, const size_t* idx, size_t real) {
            const uint8_t* msg[8];
            for (uint32_t i = 0; i < 2 * k; ++i) {
              for (size_t j = 0; j < 8; ++j) msg[j] = V[idx[j] * 2 * k + i].data();
              T8.append("V", msg, 32);
            }
            hsc::Sc xp[8];
            T8.challenge_scalar("x_perm", xp);
            for (size_t j = 0; j < real; ++j) S[idx[j]]->x_perm = xp[j];
          },
          [&](size_t p) {
            for (auto& e : Ps[p].V) S[p]->tr.append_point("V", e.data());
            S[p]->x_perm = S[p]->tr.challenge_scalar("x_perm");
          });
    }
  }
  // V_2k = commit(x_perm, gamma_2k): halved scalars (x_perm / 2 from the
  // host, gamma_2k / 2 from k_draws), encoded as 2 (C / 2) on the host
  hs.reset(new HostScope(ctx, "pb_pedersen_Vx_witness"));
  {
    std::vector<Sc> vh(2 * P);  // x_perm / 2 (V_2k), then x_perm (the device witness)
    for (size_t p = 0; p < P; ++p) {
      vh[p] = hsc::half(S[p]->x_perm);
      vh[P + p] = S[p]->x_perm;
    }
    uint32_t* d_vh = nullptr;
    BPP_TRY(upload_sc(ctx, vh, "pv_vx", &d_vh));
    if (dev_witness) BPP_TRY(witness_dev(ctx, C, (uint32_t)P, d_pi, d_vh + 8 * P, per, d_s));
    uint32_t* h_p3 = nullptr;  // written in place by the kernel (ctx_zc_out)
    BPP_TRY(ctx_zc_out(ctx, "pv_p3_h", P * P3_BYTES, &h_p3));
    BPP_TRY(pedersen_dev(ctx, G, d_vh, d_gx_half, P, nullptr, h_p3));
    std::vector<Enc32> Vx(P);
    BPP_TRY(ctx_sync(ctx));
    BPP_TRY(points_double_encode_host(ctx, h_p3, P, Vx[0].data()));
    par::for_each(P, [&](size_t p) {
      Ps[p].V.push_back(Vx[p]);
      S[p]->tr.append_point("V", Vx[p].data());
      if (!dev_witness) perm::witness(C, S[p]->d.pi, S[p]->x_perm, S[p]->vals, S[p]->aL, S[p]->aR, S[p]->aO);
    });
  }
  MsmPoints pts;
  BPP_TRY(gens_points(ctx, G, &pts));
  // A_I, A_O, S of every proof: one batch of 3P MSMs over the [P][per]
  // scalar array that k_draws_reduce (alpha, beta, rho, s_L, s_R) and
  // k_witness (a_L, a_R, a_O) filled -- or, beyond the device witness's
  // size, the host writes its first 3 + 3 n_p scalars.  The MSMs skip the
  // padding gates' zero a_L, a_R, a_O (11 % of the terms at k = 52).
  hs.reset(new HostScope(ctx, "pb_msm_AI_AO_S"));
  {
    const uint32_t hostw = 3 + 3 * n_p;  // host-written scalars per proof
    std::vector<uint32_t>&idx = scr.idx, &map = scr.map, &off = scr.off;
    const uint32_t n = C.n;                       // real gates; n_p - n padding gates are zero
    const uint32_t per_c = 3 + 3 * n + 2 * n_p;  // MSM terms per proof
    if (scr.key_P != P || scr.key_k != k || scr.key_G != G || scr.key_n != G->n) {
      idx.resize((size_t)P * per_c);
      map.resize((size_t)P * per_c);
      off.resize(3 * P + 1);
      for (size_t p = 0; p < P; ++p) {
        size_t t = p * per_c;
        const uint32_t b = (uint32_t)(p * per);
        auto term = [&](uint32_t src, uint32_t gen) {
          map[t] = b + src;
          idx[t++] = gen;
        };
        off[3 * p] = (uint32_t)t;
        term(0, G->bbidx());                                                  // alpha
        for (uint32_t i = 0; i < n; ++i) term(1 + i, G->gidx(i));             // a_L
        for (uint32_t i = 0; i < n; ++i) term(1 + n_p + i, G->hidx(i));       // a_R
        off[3 * p + 1] = (uint32_t)t;
        term(1 + 2 * n_p, G->bbidx());                                        // beta
        for (uint32_t i = 0; i < n; ++i) term(2 + 2 * n_p + i, G->gidx(i));   // a_O
        off[3 * p + 2] = (uint32_t)t;
        term(2 + 3 * n_p, G->bbidx());                                        // rho
        for (uint32_t i = 0; i < n_p; ++i) term(3 + 3 * n_p + i, G->gidx(i));  // s_L
        for (uint32_t i = 0; i < n_p; ++i) term(3 + 4 * n_p + i, G->hidx(i));  // s_R
      }
      off[3 * P] = (uint32_t)(P * per_c);
      scr.key_P = P;
      scr.key_k = k;
      scr.key_G = G;
      scr.key_n = G->n;
    }
    uint8_t* stg = nullptr;  // (host witness only) written in place in the pinned arena
    if (!dev_witness) {
      BPP_TRY(ctx_h2d_stage(ctx, (size_t)P * hostw * 32, &stg));
      ctx_secret_span(ctx, stg, (size_t)P * hostw * 32);  // (prove_wipe)
      par::for_each(P, [&](size_t p) {
        ProverState& st = *S[p];
        Sc* o = reinterpret_cast<Sc*>(stg) + p * hostw;
        o[0] = st.d.alpha;
        std::copy(st.aL.begin(), st.aL.begin() + n_p, o + 1);
        std::copy(st.aR.begin(), st.aR.begin() + n_p, o + 1 + n_p);
        o[1 + 2 * n_p] = st.d.beta;
        std::copy(st.aO.begin(), st.aO.begin() + n_p, o + 2 + 2 * n_p);
        o[2 + 3 * n_p] = st.d.rho;
      });
      BPP_HIP(hipMemcpy2DAsync(d_s, (size_t)per * 32, stg, (size_t)hostw * 32, (size_t)hostw * 32, P,
                               hipMemcpyHostToDevice, ctx->stream));
    }
    void *d_i = nullptr, *d_map = nullptr;
    BPP_TRY(ctx_ws(ctx, "mt_i", idx.size() * 4 + 4, &d_i));
    BPP_TRY(ctx_h2d_const(ctx, "mt_i", d_i, idx.data(), idx.size() * 4));  // generator indices: same every batch
    BPP_TRY(ctx_ws(ctx, "mt_map", map.size() * 4 + 4, &d_map));
    BPP_TRY(ctx_h2d_const(ctx, "mt_map", d_map, map.data(), map.size() * 4));
    // MSMs of the halved, compacted scalars, encoded as 2 * result (msm_multi_enc)
    // (gathered and halved inside the direct-table kernel: d_map)
    std::vector<uint8_t> enc(3 * P * 32);
    BPP_TRY(msm_multi_enc(ctx, d_s, (const uint32_t*)d_i, off, pts, enc.data(), true, (const uint32_t*)d_map));
    par::for_each(P, [&](size_t p) {
      memcpy(Ps[p].AI.data(), &enc[96 * p], 32);
      memcpy(Ps[p].AO.data(), &enc[96 * p + 32], 32);
      memcpy(Ps[p].S.data(), &enc[96 * p + 64], 32);
    });
  }
  // challenges y, z (host transcripts), then the t(X) coefficients and
  // tau_x's <z^Q W_V, gamma> of every proof in one device launch (poly.hip)
  hs.reset(new HostScope(ctx, "pb_host_poly"));
  std::vector<Sc> zwvg(P);  // <z^Q W_V, gamma> per proof (k_poly_coef)
  {
    std::vector<Sc> ys(P), ch((size_t)P * 3), tco;
    merlin::lockstep_x8(
        trs, for_groups,
        [&](merlin::TranscriptX8& X, const size_t* idx, size_t real) {
          const uint8_t* m[8];
          for (int j = 0; j < 8; ++j) m[j] = Ps[idx[j]].AI.data();
          X.append("A_I", m, 32);
          for (int j = 0; j < 8; ++j) m[j] = Ps[idx[j]].AO.data();
          X.append("A_O", m, 32);
          for (int j = 0; j < 8; ++j) m[j] = Ps[idx[j]].S.data();
          X.append("S", m, 32);
          Sc y8[8], z8[8];
          X.challenge_scalar("y", y8);
          X.challenge_scalar("z", z8);
          for (size_t j = 0; j < real; ++j) {
            ys[idx[j]] = y8[j];
            ch[3 * idx[j]] = y8[j];
            ch[3 * idx[j] + 2] = z8[j];
          }
        },
        [&](size_t p) {
          ProverState& st = *S[p];
          Proof& Pf = Ps[p];
          st.tr.append_point("A_I", Pf.AI.data());
          st.tr.append_point("A_O", Pf.AO.data());
          st.tr.append_point("S", Pf.S.data());
          ys[p] = st.tr.challenge_scalar("y");
          ch[3 * p] = ys[p];
          ch[3 * p + 2] = st.tr.challenge_scalar("z");
        });
    std::vector<Sc> yinv = ys;
    hsc::batch_invert(yinv, false, true);  // (y: public challenges)
    for (size_t p = 0; p < P; ++p) ch[3 * p + 1] = yinv[p];
    BPP_TRY(poly_coef_dev(ctx, C, (uint32_t)P, d_s, per, d_gamma, ch, tco));
    for (size_t p = 0; p < P; ++p) {
      for (int j = 0; j < 6; ++j) S[p]->t[1 + j] = tco[7 * p + j];
      zwvg[p] = tco[7 * p + 6];
    }
  }
  // T1, T3..T6 of every proof: one fixed-base launch
  hs.reset(new HostScope(ctx, "pb_pedersen_T_lr"));
  uint32_t *d_l = nullptr, *d_r = nullptr, *d_hf = nullptr;  // IPA inputs, on the device
  {
    std::vector<Sc> v(5 * P), g(5 * P);
    static const int ti[5] = {1, 3, 4, 5, 6};
    for (size_t p = 0; p < P; ++p)
      for (int i = 0; i < 5; ++i) {
        v[5 * p + i] = S[p]->t[ti[i]];
        g[5 * p + i] = S[p]->d.taus[i];
      }
    std::vector<Enc32> T;
    {
      HostScope hs2(ctx, "pbT_pedersen");
      BPP_TRY(pedersen_host(ctx, G, v, g, T));
    }
    HostScope hs3(ctx, "pbT_host");
    std::vector<Sc> xs(P), t_hat;
    static const char* Tlab[5] = {"T1", "T3", "T4", "T5", "T6"};
    for (size_t p = 0; p < P; ++p)
      for (int i = 0; i < 5; ++i) Ps[p].T[i] = T[5 * p + i];
    merlin::lockstep_x8(
        trs, for_groups,
        [&](merlin::TranscriptX8& X, const size_t* idx, size_t real) {
          const uint8_t* msg[8];
          for (int i = 0; i < 5; ++i) {
            for (int j = 0; j < 8; ++j) msg[j] = Ps[idx[j]].T[i].data();
            X.append(Tlab[i], msg, 32);
          }
          Sc x8[8];
          X.challenge_scalar("x", x8);
          for (size_t j = 0; j < real; ++j) xs[idx[j]] = x8[j];
        },
        [&](size_t p) {
          for (int i = 0; i < 5; ++i) S[p]->tr.append_point(Tlab[i], Ps[p].T[i].data());
          xs[p] = S[p]->tr.challenge_scalar("x");
        });
    BPP_TRY(poly_x_dev(ctx, C, (uint32_t)P, xs, &d_l, &d_r, &d_hf, t_hat));
    par::for_each(P, [&](size_t p) {
      ProverState& st = *S[p];
      Proof& Pf = Ps[p];
      const Sc x = xs[p];
      Sc xp[7];
      xp[0] = hsc::one();
      for (int i = 1; i < 7; ++i) xp[i] = hsc::mul(xp[i - 1], x);
      const int tidx[5] = {1, 3, 4, 5, 6};
      using hsc::add;
      Sc tau_x = hsc::mul(xp[2], zwvg[p]);
      for (int i = 0; i < 5; ++i) tau_x = add(tau_x, hsc::mul(st.d.taus[i], xp[tidx[i]]));
      Pf.tau_x = tau_x;
      Pf.mu = add(add(hsc::mul(st.d.alpha, x), hsc::mul(st.d.beta, xp[2])), hsc::mul(st.d.rho, xp[3]));
      Pf.t_hat = t_hat[p];
    });
    merlin::lockstep_x8(
        trs, for_groups,
        [&](merlin::TranscriptX8& X, const size_t* idx, size_t real) {
          uint8_t b[3][8][32];
          const uint8_t* msg[8];
          for (int j = 0; j < 8; ++j) {
            hsc::to_bytes(b[0][j], Ps[idx[j]].tau_x);
            hsc::to_bytes(b[1][j], Ps[idx[j]].mu);
            hsc::to_bytes(b[2][j], Ps[idx[j]].t_hat);
          }
          static const char* lab[3] = {"TX", "mu", "t"};
          for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 8; ++j) msg[j] = b[i][j];
            X.append(lab[i], msg, 32);
          }
          Sc w8[8];
          X.challenge_scalar("w", w8);
          for (size_t j = 0; j < real; ++j) S[idx[j]]->w = w8[j];
        },
        [&](size_t p) {
          ProverState& st = *S[p];
          st.tr.append_scalar("TX", Ps[p].tau_x);
          st.tr.append_scalar("mu", Ps[p].mu);
          st.tr.append_scalar("t", Ps[p].t_hat);
          st.w = st.tr.challenge_scalar("w");
        });
  }
  // IPA of every proof in lockstep
  hs.reset(new HostScope(ctx, "pb_ipa"));
  {
    std::vector<Sc> qmul(P);
    for (size_t p = 0; p < P; ++p) qmul[p] = S[p]->w;
    IpaGens ig;
    ig.pts = pts;
    ig.gbase = 0;
    ig.hbase = (uint32_t)G->n;
    ig.qidx = G->bidx();
    static thread_local std::vector<IpaProofHost> ipas_tl;
    std::vector<IpaProofHost>& ipas = ipas_tl;
    BPP_TRY(ipa_prove_batch_dev(ctx, trs, ig, n_p, nullptr, d_hf, d_l, d_r, qmul, ipas));
    for (size_t p = 0; p < P; ++p) std::swap(Ps[p].ipa, ipas[p]);  // (both keep their capacity)
  }
  for (size_t p = 0; p < P; ++p) Ps[p].pi.assign(S[p]->d.pi.begin(), S[p]->d.pi.end());
  return BPP_OK;
}

// Verifier, phase 1: replay one proof's transcript (all Fiat-Shamir
// challenges; point validation as validate_and_append_point).
struct VerifyChallenges {
  Sc x_perm, y, z, x, w, r;
  std::vector<Sc> u;  // IPA round challenges
};

bool verify_replay(const perm::Circuit& C, const Proof& P, merlin::Transcript& tr, VerifyChallenges& ch) {
  const uint32_t k = C.k, n_p = C.n_p, m = C.m;
  if (P.V.size() != m || P.ipa.L.size() != C.lg || P.ipa.R.size() != C.lg) return false;
  tr.arithmetic_domain_sep(n_p);
  for (uint32_t j = 0; j < 2 * k; ++j) tr.append_point("V", P.V[j].data());
  ch.x_perm = tr.challenge_scalar("x_perm");
  tr.append_point("V", P.V[2 * k].data());
  if (!tr.validate_and_append_point("A_I", P.AI.data())) return false;
  if (!tr.validate_and_append_point("A_O", P.AO.data())) return false;
  if (!tr.validate_and_append_point("S", P.S.data())) return false;
  ch.y = tr.challenge_scalar("y");
  ch.z = tr.challenge_scalar("z");
  static const char* lab[5] = {"T1", "T3", "T4", "T5", "T6"};
  for (int i = 0; i < 5; ++i)
    if (!tr.validate_and_append_point(lab[i], P.T[i].data())) return false;
  ch.x = tr.challenge_scalar("x");
  tr.append_scalar("TX", P.tau_x);
  tr.append_scalar("mu", P.mu);
  tr.append_scalar("t", P.t_hat);
  ch.w = tr.challenge_scalar("w");
  // bulletproofs InnerProductProof::verification_scalars, transcript part
  tr.innerproduct_domain_sep(n_p);
  ch.u.resize(C.lg);
  for (uint32_t j = 0; j < C.lg; ++j) {
    if (!tr.validate_and_append_point("L", P.ipa.L[j].data())) return false;
    if (!tr.validate_and_append_point("R", P.ipa.R[j].data())) return false;
    ch.u[j] = tr.challenge_scalar("u");
  }
  ch.r = tr.challenge_scalar("t-check-weight");
  return true;
}

// Verifier, phase 2: the proof's unweighted MSM scalars from its
// challenges, scaled by F = U^2 Y (U = prod u_j, Y = y^(n_p - 1)) so that no
// inverse is needed -- the same scalars as k_verify_consts / k_verify_scalars
// (formulas there).  gen_sc (2n_p + 2: G, H, B, Bb) is set; proof-point
// scalars (m + 8 + 2lg, order V, A_I, A_O, S, T1..T6, L.., R..) are appended.
void verify_expand(const perm::Circuit& C, const Proof& P, const VerifyChallenges& ch, std::vector<Sc>& gen_sc,
                   std::vector<Sc>& pt_sc) {
  const uint32_t n_p = C.n_p, m = C.m, lg = C.lg;
  using hsc::add;
  using hsc::mul;
  using hsc::neg;
  using hsc::sub;
  // st[i] = s_i / s_0 = prod over the bits of i of u^2 (bulletproofs
  // verification_scalars' s_i with s_0 = prod u_j^-1 factored out)
  std::vector<Sc> u_sq(lg), st(n_p);
  Sc U = hsc::one();
  for (uint32_t j = 0; j < lg; ++j) {
    u_sq[j] = hsc::sq(ch.u[j]);
    U = mul(U, ch.u[j]);
  }
  st[0] = hsc::one();
  for (uint32_t i = 1; i < n_p; ++i) {
    const uint32_t lg_i = 31 - __builtin_clz(i), kk = 1u << lg_i;
    st[i] = mul(st[i - kk], u_sq[lg - 1 - lg_i]);
  }
  const Sc x = ch.x, r = ch.r, w = ch.w;
  std::vector<Sc> xp = hsc::powers(x, 7);
  std::vector<Sc> y_n = hsc::powers(ch.y, n_p);  // y^e, e < n_p
  const Sc Y = y_n[n_p - 1], U2 = hsc::sq(U), F = mul(U2, Y);
  std::vector<Sc> zq = hsc::powers(ch.z, C.Q + 1);
  zq.erase(zq.begin());
  const std::vector<Sc> zWL = perm::zW(C.WL, zq, n_p), zWR = perm::zW(C.WR, zq, n_p), zWO = perm::zW(C.WO, zq, n_p),
                        zWV = perm::zW(C.WV, zq, m);
  std::vector<Sc> c = C.c;
  c[C.Q - 1] = hsc::neg(ch.x_perm);
  const Sc a = P.ipa.a, b = P.ipa.b;
  const Sc uyaR = hsc::to_mont(mul(mul(U, Y), a)), ubR = hsc::to_mont(mul(U, b)), xR_ = hsc::to_mont(x),
           u2R = hsc::to_mont(U2);
  Sc delta = hsc::zero();  // sum_i U^2 yr_i zWR_i zWL_i (= F delta)
  for (uint32_t i = 0; i < n_p; ++i) {
    const Sc yr = y_n[n_p - 1 - i];  // y^(n_p - 1 - i) = Y y^-i
    const Sc yu = hsc::mulm(yr, u2R);
    const Sc yuR = hsc::to_mont(yu), yrR = hsc::to_mont(yr);
    delta = add(delta, mul(mul(yu, zWR[i]), zWL[i]));
    gen_sc[i] = sub(hsc::mulm(st[i], uyaR), hsc::mulm(hsc::mulm(zWR[i], xR_), yuR));
    gen_sc[n_p + i] = add(sub(hsc::mulm(hsc::mulm(st[n_p - 1 - i], ubR), yrR),
                              hsc::mulm(add(hsc::mulm(zWL[i], xR_), zWO[i]), yuR)),
                          F);
  }
  const Sc zc = hsc::inner_product(zq, c);
  const Sc tcheck_B = mul(r, sub(mul(F, P.t_hat), mul(xp[2], add(delta, mul(F, zc)))));
  const Sc ipa_B = mul(mul(w, F), sub(mul(a, b), P.t_hat));
  gen_sc[2 * n_p] = add(tcheck_B, ipa_B);
  gen_sc[2 * n_p + 1] = mul(F, add(mul(r, P.tau_x), P.mu));
  // proof points
  const Sc rx2FR = hsc::to_mont(mul(mul(r, xp[2]), F));
  for (uint32_t j = 0; j < m; ++j) pt_sc.push_back(neg(hsc::mulm(zWV[j], rx2FR)));
  pt_sc.push_back(neg(mul(F, x)));
  pt_sc.push_back(neg(mul(F, xp[2])));
  pt_sc.push_back(neg(mul(F, xp[3])));
  const int tidx[5] = {1, 3, 4, 5, 6};
  for (int i = 0; i < 5; ++i) pt_sc.push_back(neg(mul(F, mul(r, xp[tidx[i]]))));
  for (uint32_t j = 0; j < lg; ++j) pt_sc.push_back(neg(mul(F, u_sq[j])));
  for (uint32_t j = 0; j < lg; ++j) {  // -Y prod_{k != j} u_k^2 (= -F u_j^-2)
    Sc v = Y;
    for (uint32_t k = 0; k < lg; ++k)
      if (k != j) v = mul(v, u_sq[k]);
    pt_sc.push_back(neg(v));
  }
}

void proof_points(const Proof& P, std::vector<uint8_t>& enc) {
  auto add = [&](const Enc32& e) { enc.insert(enc.end(), e.begin(), e.end()); };
  for (auto& v : P.V) add(v);
  add(P.AI);
  add(P.AO);
  add(P.S);
  for (int i = 0; i < 5; ++i) add(P.T[i]);
  for (auto& l : P.ipa.L) add(l);
  for (auto& r : P.ipa.R) add(r);
}

}  // namespace

// A batch verification split into its host replay (begin) and its weighted
// MSM (partial), so that the MSM can be partitioned over GPUs: by bucket
// windows (every rank holds every proof) or by proofs (each rank holds a
// slice; only the r challenges are exchanged before the MSM).
struct bpp_verify_job {
  perm::Circuit C;
  size_t count = 0, npt = 0;
  std::vector<Proof> Ps;
  std::vector<Sc> rs;                 // per-proof weight challenges
  std::vector<VerifyChallenges> ch;   // every proof's transcript challenges
  // unweighted generator / proof-point scalars, expanded on the host only
  // when asked for (bpp_perm_verify_scalars); the GPU path expands them on
  // the device (k_verify_scalars)
  mutable std::mutex mu;
  mutable bool expanded = false;
  mutable std::vector<std::vector<Sc>> gen_p, pt_p;
  // device job (bpp_perm_verify_begin_dev): the replay ran on the GPU and the
  // records / decompressed proof points sit in dctx's "vj_*" workspaces
  // (generation dgen); Ps and ch stay empty.  An asynchronous begin
  // (verify_batch) leaves the replay's verdicts in bad_h (pinned, rcount
  // words) for the partial to check after its own synchronisation.
  const uint32_t* bad_h = nullptr;
  bool dev = false;
  bpp_ctx* dctx = nullptr;
  uint64_t dgen = 0;
  // sliced device job (bpp_perm_verify_begin_dev_slice): all `count` proofs
  // uploaded and their points decompressed, only [rfirst, rfirst + rcount)
  // replayed (records and rs of that slice); a whole job has rcount = count
  size_t rfirst = 0, rcount = 0;
};

namespace {

// pass 1 (parallel over chunks of proofs): parse and replay each transcript
// (all challenges and the proof's weight challenge r); a zero y or u_j
// rejects the proof (the checks are scaled by a product of them)
// (circuit_lib.rs:478-585 restated in sound mode)
int verify_begin(const perm::Circuit& C, const uint8_t* label, size_t llen, size_t count, const uint8_t* proofs,
                 size_t proof_stride, const uint8_t* V, std::unique_ptr<bpp_verify_job>& job) {
  job.reset(new bpp_verify_job);
  bpp_verify_job& J = *job;
  J.C = C;
  J.count = count;
  J.npt = (size_t)C.m + 8 + 2 * C.lg;
  J.Ps.resize(count);
  J.rs.resize(count);
  J.ch.resize(count);
  std::vector<uint8_t> ok(count, 0);
  par::for_each(count, [&](size_t p) {
    if (!deserialize(C, proofs + p * proof_stride, perm::proof_len(C.k), V + p * 32 * C.m, J.Ps[p])) return;
    merlin::Transcript tr(label, llen);
    VerifyChallenges& ch = J.ch[p];
    if (!verify_replay(C, J.Ps[p], tr, ch)) return;
    if (hsc::is_zero(ch.y)) return;
    for (const Sc& u : ch.u)
      if (hsc::is_zero(u)) return;
    J.rs[p] = ch.r;
    ok[p] = 1;
  });
  for (size_t p = 0; p < count; ++p)
    if (!ok[p]) return BPP_ERR_VERIFY;
  return BPP_OK;
}

// Host expansion of every proof's unweighted scalars (verify_expand), once.
void job_expand_host(const bpp_verify_job& J) {
  std::lock_guard<std::mutex> g(J.mu);
  if (J.expanded) return;
  const perm::Circuit& C = J.C;
  J.gen_p.assign(J.count, std::vector<Sc>());
  J.pt_p.assign(J.count, std::vector<Sc>());
  par::for_each(J.count, [&](size_t p) {
    J.gen_p[p].assign(2 * C.n_p + 2, hsc::zero());
    verify_expand(C, J.Ps[p], J.ch[p], J.gen_p[p], J.pt_p[p]);
  });
  J.expanded = true;
}

// Terms of the job's MSM: merged generators (G, H, B, Bb) + every proof point.
size_t verify_terms(const bpp_verify_job& J) { return 2 * (size_t)J.C.n_p + 2 + J.count * J.npt; }

// pass 2 (host): the job's MSM terms with proof p weighted by
// perm::batch_weight(seed, first + p, r_p) -- generator scalars merged across
// its proofs (G[0..n_p), H[0..n_p), B, Bb), then each proof's points (V,
// A_I, A_O, S, T1..T6, L.., R..) weighted by their proof's weight; enc =
// those points' encodings.
int verify_terms_weighted(const bpp_verify_job& J, const uint8_t seed[32], size_t first, std::vector<Sc>& sc,
                          std::vector<uint8_t>& enc) {
  const uint32_t n_p = J.C.n_p;
  const size_t count = J.count, npt = J.npt;
  job_expand_host(J);
  std::vector<Sc> wR(count);  // Montgomery form (one step per product)
  par::for_each(count, [&](size_t p) { wR[p] = hsc::to_mont(perm::batch_weight(seed, first + p, J.rs[p])); });
  const Sc* wts = wR.data();
  const size_t NG = 2 * (size_t)n_p + 2;
  sc.assign(NG + count * npt, hsc::zero());
  enc.assign(count * npt * 32, 0);
  // proof chunks with private generator accumulators (each reads its proofs'
  // rows contiguously), summed at the end
  const size_t chunks = std::max<size_t>(1, std::min<size_t>(count, 64));
  std::vector<std::vector<Sc>> acc(chunks, std::vector<Sc>(NG, hsc::zero()));
  par::for_each(chunks, [&](size_t ch) {
    std::vector<Sc>& a = acc[ch];
    std::vector<uint8_t> e;
    for (size_t p = ch * count / chunks; p < (ch + 1) * count / chunks; ++p) {
      const Sc& w = wts[p];
      for (size_t i = 0; i < NG; ++i) a[i] = hsc::add(a[i], hsc::mulm(J.gen_p[p][i], w));
      for (size_t j = 0; j < npt; ++j) sc[NG + p * npt + j] = hsc::mulm(J.pt_p[p][j], w);
      e.clear();
      proof_points(J.Ps[p], e);
      memcpy(&enc[p * npt * 32], e.data(), npt * 32);
    }
  });
  for (size_t ch = 0; ch < chunks; ++ch)
    for (size_t i = 0; i < NG; ++i) sc[i] = hsc::add(sc[i], acc[ch][i]);
  return BPP_OK;
}

// The batch's ONE MSM over windows [wb, we) of its c-bit signed digits (c =
// msm_choose_c(terms)) -> raw partial point: scalars d_sv (2 n_p + 2 merged
// generator scalars, then count x npt proof-point scalars), proof points d_x.
int verify_msm(bpp_ctx* ctx, const bpp_gens* G, const perm::Circuit& C, size_t count, const uint32_t* d_sv,
               const uint32_t* d_x, uint32_t wb, uint32_t we, h25519::ge* out) {
  const uint32_t n_p = C.n_p;
  const size_t NG = 2 * (size_t)n_p + 2, T = NG + count * vpts_n(C);
  // term t reads generator t of the resident table (G[0..n_p), H[0..n_p),
  // B, Bb) or proof point t - NG; the index list is needed only when the
  // generator set is longer than the padded circuit
  const uint32_t n0 = (uint32_t)(2 * G->n + 2);
  uint32_t* d_idx = nullptr;
  if (G->n != n_p) {
    std::vector<uint32_t> idx(T);
    for (uint32_t i = 0; i < n_p; ++i) {
      idx[i] = G->gidx(i);
      idx[n_p + i] = G->hidx(i);
    }
    idx[2 * n_p] = G->bidx();
    idx[2 * n_p + 1] = G->bbidx();
    for (size_t j = NG; j < T; ++j) idx[j] = n0 + (uint32_t)(j - NG);
    void* d = nullptr;
    BPP_TRY(ctx_ws(ctx, "pv_idx", idx.size() * 4 + 4, &d));
    BPP_TRY(ctx_h2d_const(ctx, "pv_idx", d, idx.data(), idx.size() * 4));
    d_idx = (uint32_t*)d;
  }
  const uint32_t c = msm_choose_c((double)T);
  return msm_single_dev(ctx, d_sv, d_idx, G->d_tbl, T, c, wb, we - wb, out, d_x, n0);
}

// pass 2 of a host job: per-proof records built on the host from the host
// replay, then the same device scalars and MSM as a device job.
int verify_partial(bpp_ctx* ctx, const bpp_gens* G, const bpp_verify_job& J, const uint8_t seed[32], size_t first,
                   uint32_t wb, uint32_t we, h25519::ge* out) {
  const uint32_t n_p = J.C.n_p;
  if (G->n < n_p) {
    ctx->err = "generators shorter than the padded circuit";
    return BPP_ERR_LEN;
  }
  const size_t NG = 2 * (size_t)n_p + 2, count = J.count, npt = J.npt, T = NG + count * npt;
  const uint32_t lg = J.C.lg, nrec = vrec_n(J.C);
  // per-proof records for k_verify_consts / k_verify_scalars and the proof
  // points' encodings
  std::vector<uint32_t> rec(count * nrec * 8);
  std::vector<uint8_t> enc(count * npt * 32);
  {
    HostScope hs(ctx, "verify_terms");
    par::for_each(count, [&](size_t p) {
      const VerifyChallenges& ch = J.ch[p];
      const Proof& P = J.Ps[p];
      uint32_t* r = &rec[p * nrec * 8];
      auto put = [&](uint32_t k, const Sc& v) { hsc::to_bytes((uint8_t*)(r + 8 * k), v); };
      put(VREC_XPERM, ch.x_perm);
      put(VREC_Y, ch.y);
      put(VREC_Z, ch.z);
      put(VREC_X, ch.x);
      put(VREC_W, ch.w);
      put(VREC_R, ch.r);
      put(VREC_A, P.ipa.a);
      put(VREC_B, P.ipa.b);
      put(VREC_THAT, P.t_hat);
      put(VREC_TAUX, P.tau_x);
      put(VREC_MU, P.mu);
      put(VREC_WT, hsc::zero());
      for (uint32_t j = 0; j < lg; ++j) put(VREC_U + j, ch.u[j]);
      std::vector<uint8_t> e;
      e.reserve(npt * 32);
      proof_points(P, e);
      memcpy(&enc[p * npt * 32], e.data(), npt * 32);
    });
  }
  void* d_sv = nullptr;
  BPP_TRY(ctx_ws(ctx, "pv_s", T * 32 + 32, &d_sv));
  BPP_TRY(verify_scalars_dev(ctx, J.C, (uint32_t)count, rec, seed, first, (uint32_t*)d_sv));
  uint32_t* d_x = nullptr;
  int rc = decompress_ws(ctx, enc.data(), enc.size() / 32, "pv_x", &d_x);
  if (rc == BPP_ERR_DECOMPRESS) return BPP_ERR_VERIFY;
  BPP_TRY(rc);
  // term t reads generator t of the resident table (G[0..n_p), H[0..n_p),
  // B, Bb) or proof point t - NG; the index list is needed only when the
  // generator set is longer than the padded circuit
  return verify_msm(ctx, G, J.C, count, (const uint32_t*)d_sv, d_x, wb, we, out);
}

// pass 1 on the device (bpp_perm_verify_begin_dev): upload the proofs and V,
// replay every transcript on the GPU (k_verify_replay_g, one 16-lane group per proof)
// and return the r challenges; meanwhile the proof points are decompressed
// on child stream VJ_CHILD into the "vj_x" workspace (k_verify_decompress,
// independent of the replay: the 64 replay waves are latency-bound, the
// decompression throughput-bound).  BPP_ERR_VERIFY if the replay rejects a
// proof; an undecodable point is reported by verify_partial_dev.
// rfirst / rcount: replay only that slice (the points of all count proofs
// are still decompressed; rcount = SIZE_MAX: all of them).
// sync = false (verify_batch): nothing waits here -- the replay's verdicts
// stay in J.bad_h for verify_partial_dev to check after its own
// synchronisation, so the weights, scalars and MSM are queued right behind
// the replay with no host round trip (J.rs stays empty).
int verify_begin_dev(bpp_ctx* ctx, const perm::Circuit& C, const uint8_t* label, size_t llen, size_t count,
                     const uint8_t* proofs, const uint8_t* V, std::unique_ptr<bpp_verify_job>& job,
                     size_t rfirst = 0, size_t rcount = SIZE_MAX, bool sync = true) {
  job.reset(new bpp_verify_job);
  bpp_verify_job& J = *job;
  if (rcount == SIZE_MAX) rcount = count;
  J.C = C;
  J.count = count;
  J.npt = vpts_n(C);
  J.rfirst = rfirst;
  J.rcount = rcount;
  J.rs.resize(rcount);
  J.dev = true;
  J.dctx = ctx;
  // (before the generation: a refused call supersedes nothing)
  if (count > (1u << 26) || rfirst > count || rcount > count - rfirst) return BPP_ERR_ARG;
  J.dgen = ++ctx->vjob_gen;
  if (!count) return BPP_OK;
  const size_t plen = perm::proof_len(C.k), vbytes = (size_t)C.m * 32, npts = count * J.npt;
  bpp_ctx* kid = nullptr;
  BPP_TRY(ctx_child(ctx, VJ_CHILD, &kid));
  if (!ctx->vj_ev_in) BPP_HIP(hipEventCreateWithFlags(&ctx->vj_ev_in, hipEventDisableTiming));
  if (!ctx->vj_ev_dec) BPP_HIP(hipEventCreateWithFlags(&ctx->vj_ev_dec, hipEventDisableTiming));
  // (the previous job's decompression may still read "vj_in")
  if (ctx->vj_dec_pending) BPP_HIP(hipStreamWaitEvent(ctx->stream, ctx->vj_ev_dec, 0));
  void *d_in = nullptr, *d_rec = nullptr, *d_x = nullptr, *d_dbad = nullptr;
  BPP_TRY(ctx_ws(ctx, "vj_in", count * (plen + vbytes), &d_in));
  const uint32_t* d_pf = (const uint32_t*)d_in;
  const uint32_t* d_V = (const uint32_t*)((uint8_t*)d_in + count * plen);
  // (+1: the pad record of the replay's groups past the batch)
  BPP_TRY(ctx_ws(ctx, "vj_rec", (count + 1) * vrec_n(C) * 32, &d_rec));
  BPP_TRY(ctx_ws(ctx, "vj_x", npts * MSM_NIELS_WORDS * 4, &d_x));
  BPP_TRY(ctx_ws(ctx, "vj_dbad", 8, &d_dbad));
  BPP_HIP(hipMemsetAsync(d_dbad, 0xff, 8, ctx->stream));
  // decompression order (BPP_VERIFY_DEC, A/B): 0 = per upload chunk, beside
  // the upload and then the replay, 1 = launched after the replay's launch
  // (beside it), 2 = after the replay completes (it then overlaps the host
  // weights and k_verify_scalars instead)
  static const int dec_order = [] {
    const char* e = getenv("BPP_VERIFY_DEC");
    return e ? atoi(e) : 0;
  }();
  auto launch_dec = [&]() -> int {
    BPP_HIP(hipEventRecord(ctx->vj_ev_in, ctx->stream));
    BPP_HIP(hipStreamWaitEvent(kid->stream, ctx->vj_ev_in, 0));
    BPP_TRY(verify_decompress_dev(kid, C, (uint32_t)count, d_pf, d_V, (uint32_t*)d_x, (unsigned long long*)d_dbad));
    BPP_HIP(hipEventRecord(ctx->vj_ev_dec, kid->stream));
    ctx->vj_dec_pending = true;
    return BPP_OK;
  };
  // BPP_VERIFY_SPLIT=1 (whole jobs): the V bytes of every chunk go up first
  // and the transcripts run their V part (2k V appends, x_perm, V_2k: ~60 %
  // of a transcript's permutations) on a second child stream as soon as the
  // last V byte lands, while the proof bytes are still being copied; the
  // proof part follows the last copy.  Each chunk's V points and then its
  // proof points are decompressed as they land.
  static const bool split_env = [] {
    const char* e = getenv("BPP_VERIFY_SPLIT");
    return e && atoi(e) != 0;
  }();
  const bool split = split_env && dec_order == 0 && rfirst == 0 && rcount == count && count >= 256;
  uint32_t* d_stt = nullptr;
  uint32_t* h_init = nullptr;  // the shared transcript prefix, read in place (zero copy)
  ReplayEarly early{};
  bool use_early = false;
  if (split) {
    void* d = nullptr;
    BPP_TRY(ctx_ws(ctx, "vj_stt", count * 52 * 4, &d));
    d_stt = (uint32_t*)d;
  }
  {
    HostScope hs(ctx, "verify_upload");
    if (split) {
      bpp_ctx* kv = nullptr;
      BPP_TRY(ctx_child(ctx, VJ_CHILD + 1, &kv));
      {
        uint32_t init[52];
        verify_init_state(C, label, llen, init);
        BPP_TRY(ctx_zc_in(ctx, "vj_init", init, sizeof init, &h_init));
      }
      static const size_t nchunk_env = [] {
        const char* e = getenv("BPP_VERIFY_CHUNKS");
        return (size_t)std::max(1, e ? atoi(e) : 4);
      }();
      const size_t nchunk = std::min(nchunk_env, std::max<size_t>(1, count / 256));
      for (auto* evs : {&ctx->vj_ev_chunk, &ctx->vj_ev_chunk2})
        while (evs->size() < nchunk) {
          hipEvent_t e = nullptr;
          BPP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
          evs->push_back(e);
        }
      if (!ctx->vj_ev_vrep) BPP_HIP(hipEventCreateWithFlags(&ctx->vj_ev_vrep, hipEventDisableTiming));
      const bool direct = host_is_pinned(proofs, count * plen) && host_is_pinned(V, count * vbytes);
      uint8_t* stg = nullptr;
      if (!direct) BPP_TRY(ctx_h2d_stage(ctx, count * (plen + vbytes), &stg));
      auto up = [&](size_t off, const uint8_t* src, size_t n) -> int {
        if (direct) {
          BPP_HIP(hipMemcpyAsync((uint8_t*)d_in + off, src, n, hipMemcpyHostToDevice, ctx->stream));
        } else {
          ctx_stage_copy(stg + off, src, n);
          BPP_TRY(ctx_h2d_staged(ctx, (uint8_t*)d_in + off, stg + off, n));
        }
        return BPP_OK;
      };
      const uint32_t m = C.m, npt = (uint32_t)J.npt;
      // (the V parts as ONE launch once every V byte is up: a transcript is a
      // latency chain, so per-chunk launches in a row on one stream cost a
      // chain each -- 4 x 185 us, measured)
      for (size_t q = 0; q < nchunk; ++q) {  // V bytes, V points
        const size_t p0 = count * q / nchunk, p1 = count * (q + 1) / nchunk;
        BPP_TRY(up(count * plen + p0 * vbytes, V + p0 * vbytes, (p1 - p0) * vbytes));
        BPP_HIP(hipEventRecord(ctx->vj_ev_chunk[q], ctx->stream));
        BPP_HIP(hipStreamWaitEvent(kid->stream, ctx->vj_ev_chunk[q], 0));
        BPP_TRY(verify_decompress_dev(kid, C, (uint32_t)count, d_pf, d_V, (uint32_t*)d_x, (unsigned long long*)d_dbad,
                                      (uint32_t)p0, (uint32_t)p1, 0, m));
      }
      BPP_HIP(hipStreamWaitEvent(kv->stream, ctx->vj_ev_chunk[nchunk - 1], 0));
      BPP_TRY(verify_replay_v_dev(ctx, kv->stream, C, 0, (uint32_t)count, (uint32_t)count, h_init, d_V, d_stt));
      BPP_HIP(hipEventRecord(ctx->vj_ev_vrep, kv->stream));
      for (size_t q = 0; q < nchunk; ++q) {  // proof bytes, proof points
        const size_t p0 = count * q / nchunk, p1 = count * (q + 1) / nchunk;
        BPP_TRY(up(p0 * plen, proofs + p0 * plen, (p1 - p0) * plen));
        BPP_HIP(hipEventRecord(ctx->vj_ev_chunk2[q], ctx->stream));
        BPP_HIP(hipStreamWaitEvent(kid->stream, ctx->vj_ev_chunk2[q], 0));
        BPP_TRY(verify_decompress_dev(kid, C, (uint32_t)count, d_pf, d_V, (uint32_t*)d_x, (unsigned long long*)d_dbad,
                                      (uint32_t)p0, (uint32_t)p1, m, npt - m));
      }
      BPP_HIP(hipEventRecord(ctx->vj_ev_dec, kid->stream));
      ctx->vj_dec_pending = true;
      BPP_HIP(hipStreamWaitEvent(ctx->stream, ctx->vj_ev_vrep, 0));
    } else if (dec_order == 0) {
      // The proofs and V go up in chunks of proofs (each chunk's proof bytes
      // and V bytes to their places in the [proofs][V] layout), and each
      // chunk's points are decompressed on the child stream as soon as its
      // copies land, so the decompression -- the longest stage beside the
      // replay -- starts while later chunks are still being staged and copied
      // (BPP_VERIFY_CHUNKS, default 4; 1 = one decompression after the whole
      // upload).
      static const size_t nchunk_env = [] {
        const char* e = getenv("BPP_VERIFY_CHUNKS");
        return (size_t)std::max(1, e ? atoi(e) : 4);
      }();
      // (chunks of >= 1024 proofs: a decompression launch is a per-lane
      // latency chain of ~50-80 us however few points it has, and the
      // launches of one stream run in turn -- a 512-proof slice in two
      // chunks waited 0.32 ms for its points, tools/shard_model.py)
      const size_t nchunk = std::min(nchunk_env, std::max<size_t>(1, count / 1024));
      while (ctx->vj_ev_chunk.size() < nchunk) {
        hipEvent_t e = nullptr;
        BPP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->vj_ev_chunk.push_back(e);
      }
      // proofs and V already in pinned host memory (bpp_host_alloc; memory
      // the caller registered itself with BPP_PIN_QUERY=1) go up by DMA from
      // where they are; pageable buffers are staged through the pinned arena
      // first (the host copy then paces the upload)
      const bool direct = host_is_pinned(proofs, count * plen) && host_is_pinned(V, count * vbytes);
      uint8_t* stg = nullptr;
      if (!direct) BPP_TRY(ctx_h2d_stage(ctx, count * (plen + vbytes), &stg));
      static const size_t stage_piece = [] {  // (BPP_VERIFY_PIECE_KB, A/B; 0 = whole parts, the default)
        const char* e = getenv("BPP_VERIFY_PIECE_KB");
        const long kb = e ? atol(e) : 0;
        return kb > 0 ? (size_t)kb << 10 : SIZE_MAX;
      }();
      // BPP_VERIFY_EARLY=1 (A/B, off): the first nchunk - 1 chunks'
      // transcripts start on a side stream once their bytes are up, beside
      // the last chunk's upload.  It does not pay: a replay launch is a
      // latency chain of ~0.26-0.28 ms however few transcripts it holds, so
      // the last chunk's replay ends when the whole one did (1.84-1.89 vs
      // 1.80-1.86 ms per batch, profiles/r05_verify_ab.txt)
      static const bool early_env = [] {
        const char* e = getenv("BPP_VERIFY_EARLY");
        return e && atoi(e) != 0;
      }();
      if (early_env && nchunk >= 2 && rfirst == 0 && rcount == count) {
        bpp_ctx* kv = nullptr;
        BPP_TRY(ctx_child(ctx, VJ_CHILD + 1, &kv));
        if (!ctx->vj_ev_vrep) BPP_HIP(hipEventCreateWithFlags(&ctx->vj_ev_vrep, hipEventDisableTiming));
        early = ReplayEarly{kv->stream, ctx->vj_ev_chunk[nchunk - 2], ctx->vj_ev_vrep,
                            (uint32_t)(count * (nchunk - 1) / nchunk)};
        use_early = true;
        uint32_t init[52];
        verify_init_state(C, label, llen, init);
        BPP_TRY(ctx_zc_in(ctx, "vj_init", init, sizeof init, &h_init));
      }
      for (size_t q = 0; q < nchunk; ++q) {
        const size_t p0 = count * q / nchunk, p1 = count * (q + 1) / nchunk;
        const size_t po = p0 * plen, pn = (p1 - p0) * plen, vo = count * plen + p0 * vbytes, vn = (p1 - p0) * vbytes;
        if (direct) {
          BPP_HIP(hipMemcpyAsync((uint8_t*)d_in + po, proofs + po, pn, hipMemcpyHostToDevice, ctx->stream));
          BPP_HIP(hipMemcpyAsync((uint8_t*)d_in + vo, V + p0 * vbytes, vn, hipMemcpyHostToDevice, ctx->stream));
        } else {
          // (in pieces, each piece's DMA behind its host copy, with
          // BPP_VERIFY_PIECE_KB: measured slower, r05_verify_ab.txt)
          auto staged = [&](size_t o, const uint8_t* src, size_t n) -> int {
            for (size_t a = 0; a < n; a += stage_piece) {
              const size_t b = std::min(n, a + stage_piece);
              ctx_stage_copy(stg + o + a, src + a, b - a);
              BPP_TRY(ctx_h2d_staged(ctx, (uint8_t*)d_in + o + a, stg + o + a, b - a));
            }
            return BPP_OK;
          };
          BPP_TRY(staged(po, proofs + po, pn));
          BPP_TRY(staged(vo, V + p0 * vbytes, vn));
        }
        BPP_HIP(hipEventRecord(ctx->vj_ev_chunk[q], ctx->stream));
        BPP_HIP(hipStreamWaitEvent(kid->stream, ctx->vj_ev_chunk[q], 0));
        BPP_TRY(verify_decompress_dev(kid, C, (uint32_t)count, d_pf, d_V, (uint32_t*)d_x,
                                      (unsigned long long*)d_dbad, (uint32_t)p0, (uint32_t)p1));
        if (use_early && q + 2 == nchunk)
          BPP_TRY(verify_replay_early_dev(ctx, C, (uint32_t)count, h_init, d_pf, d_V, early));
      }
      BPP_HIP(hipEventRecord(ctx->vj_ev_dec, kid->stream));
      ctx->vj_dec_pending = true;
    } else {
      BPP_TRY(ctx_h2d2(ctx, d_in, proofs, count * plen, V, count * vbytes));
    }
  }
  HostScope hs(ctx, "verify_replay");
  if (dec_order != 0 && !rcount) BPP_TRY(launch_dec());
  uint32_t *h_r = nullptr, *h_bad = nullptr;
  if (!h_init) {
    uint32_t init[52];
    verify_init_state(C, label, llen, init);
    BPP_TRY(ctx_zc_in(ctx, "vj_init", init, sizeof init, &h_init));
  }
  if (!rcount) return ctx_sync(ctx);
  BPP_TRY(ctx_zc_out(ctx, "vj_r", rcount * 32, &h_r));
  BPP_TRY(ctx_zc_out(ctx, "vj_bad", rcount * 4, &h_bad));
  if (dec_order == 1) {  // (the event is recorded before the replay: the decompression waits for the upload only)
    BPP_HIP(hipEventRecord(ctx->vj_ev_in, ctx->stream));
  }
  BPP_TRY(verify_replay_dev(ctx, C, (uint32_t)rcount, h_init, d_pf + rfirst * (plen / 4),
                            d_V + rfirst * (vbytes / 4), (uint32_t*)d_rec, h_r, h_bad, d_stt,
                            use_early ? &early : nullptr));
  if (dec_order == 1) {
    BPP_HIP(hipStreamWaitEvent(kid->stream, ctx->vj_ev_in, 0));
    BPP_TRY(verify_decompress_dev(kid, C, (uint32_t)count, d_pf, d_V, (uint32_t*)d_x, (unsigned long long*)d_dbad));
    BPP_HIP(hipEventRecord(ctx->vj_ev_dec, kid->stream));
    ctx->vj_dec_pending = true;
  } else if (dec_order == 2) {
    BPP_TRY(launch_dec());
  }
  if (!sync) {
    J.bad_h = h_bad;
    J.rs.clear();
    return BPP_OK;
  }
  BPP_TRY(ctx_sync_latency(ctx));
  uint32_t any = 0;
  for (size_t p = 0; p < rcount; ++p) any |= h_bad[p];
  if (any) return BPP_ERR_VERIFY;
  memcpy(J.rs.data(), h_r, rcount * 32);
  return BPP_OK;
}

// A sliced job's scalars (bpp_perm_verify_slice_scalars): the slice's
// proofs weighted by perm::batch_weight(seed, rfirst + p, r_p), the generator
// scalars summed over the slice and the slice's proof-point scalars ->
// d_out = [NG | rcount x npt] x 32 B (device memory).
int verify_slice_scalars_dev(bpp_ctx* ctx, const bpp_verify_job& J, const uint8_t seed[32], size_t first,
                             uint32_t* d_out) {
  if (J.dctx != ctx || J.dgen != ctx->vjob_gen) {
    ctx->err = "device verify job belongs to another context or was superseded by a later begin";
    return BPP_ERR_ARG;
  }
  if (!J.rcount) {  // an empty slice adds nothing to the generator scalars
    BPP_HIP(hipMemsetAsync(d_out, 0, (2 * (size_t)J.C.n_p + 2) * 32, ctx->stream));
    return ctx_sync(ctx);
  }
  void* d_rec = nullptr;
  BPP_TRY(ctx_ws(ctx, "vj_rec", (J.rcount + 1) * vrec_n(J.C) * 32, &d_rec));
  uint32_t* h_seed = nullptr;
  BPP_TRY(ctx_zc_in(ctx, "vj_seed", seed, 32, &h_seed));
  BPP_TRY(verify_scalars_dev_rec(ctx, J.C, (uint32_t)J.rcount, (const uint32_t*)d_rec, h_seed, first + J.rfirst,
                                 d_out));
  BPP_TRY(ctx_sync(ctx));
  if (J.bad_h) {  // an asynchronous begin's replay verdicts (the stream has passed them)
    uint32_t any = 0;
    for (size_t p = 0; p < J.rcount; ++p) any |= J.bad_h[p];
    if (any) {
      ctx->err = "a proof's transcript replay rejected it";
      return BPP_ERR_VERIFY;
    }
  }
  return BPP_OK;
}

// A job's decompressed proof points (bpp_perm_verify_slice_points): count x
// npt extended-Niels records (MSM_NIELS_WORDS words each, proof-major) ->
// d_out, after the job's decompression; BPP_ERR_VERIFY if a point did not
// decode.  Synchronises ctx.
int verify_slice_points_dev(bpp_ctx* ctx, const bpp_verify_job& J, void* d_out) {
  if (J.dctx != ctx || J.dgen != ctx->vjob_gen) {
    ctx->err = "device verify job belongs to another context or was superseded by a later begin";
    return BPP_ERR_ARG;
  }
  if (!J.count) return BPP_OK;
  // on the decompression's own (child) stream, behind the decompression:
  // an asynchronous begin's replay may still be running on ctx's stream
  bpp_ctx* kid = nullptr;
  BPP_TRY(ctx_child(ctx, VJ_CHILD, &kid));
  void *d_x = nullptr, *d_dbad = nullptr;
  BPP_TRY(ctx_ws(ctx, "vj_x", J.count * J.npt * MSM_NIELS_WORDS * 4, &d_x));
  BPP_TRY(ctx_ws(ctx, "vj_dbad", 8, &d_dbad));
  uint64_t* h_dbad = nullptr;
  BPP_TRY(ctx_zc_out(kid, "sp_dbad_h", 8, (uint32_t**)&h_dbad));
  BPP_HIP(hipStreamWaitEvent(kid->stream, ctx->vj_ev_dec, 0));
  BPP_HIP(hipMemcpyAsync(h_dbad, d_dbad, 8, hipMemcpyDeviceToHost, kid->stream));
  BPP_HIP(hipMemcpyAsync(d_out, d_x, J.count * J.npt * MSM_NIELS_WORDS * 4, hipMemcpyDeviceToDevice, kid->stream));
  BPP_TRY(ctx_sync(kid));
  if (*h_dbad != ~0ull) {
    ctx->err = "undecodable proof point at index " + std::to_string(*h_dbad);
    return BPP_ERR_VERIFY;
  }
  return BPP_OK;
}

// Gathered slice blocks -> one contiguous array in ONE launch (a
// hipMemcpyAsync per slice cost ~5 us of launch gap each: 8 slices of
// scalars took 50 us before config 5's rank MSM, tools/shard_model.py):
// slice r's n_r elements of `ew` 16-B units sit at src + r stride + off, and
// land at dst in slice order.
#define GB_MAX 64
struct GatherTab {
  uint32_t n;                // slices
  uint32_t pre[GB_MAX + 1];  // element prefix counts
};
__global__ void __launch_bounds__(256) k_gather_blocks(const uint8_t* __restrict__ src, size_t stride, size_t off,
                                                       uint32_t ew, GatherTab tab, uint4* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // 16-B unit
  const size_t e = i / ew;
  if (e >= tab.pre[tab.n]) return;
  uint32_t lo = 0, hi = tab.n;  // slice r: pre[r] <= e < pre[r + 1]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (tab.pre[mid] <= e) lo = mid;
    else hi = mid;
  }
  const uint4* s = reinterpret_cast<const uint4*>(src + lo * stride + off);
  dst[i] = s[(e - tab.pre[lo]) * ew + i % ew];
}

static int gather_blocks_dev(bpp_ctx* ctx, const uint8_t* src, size_t stride, size_t off, size_t elem_bytes,
                             const size_t* counts, size_t nslices, uint8_t* dst) {
  if (nslices > GB_MAX || elem_bytes % 16 || stride % 16 || off % 16) {
    size_t o = 0;
    for (size_t r = 0; r < nslices; ++r) {
      if (counts[r])
        BPP_HIP(hipMemcpyAsync(dst + o * elem_bytes, src + r * stride + off, counts[r] * elem_bytes,
                               hipMemcpyDeviceToDevice, ctx->stream));
      o += counts[r];
    }
    return BPP_OK;
  }
  GatherTab tab;
  tab.n = (uint32_t)nslices;
  tab.pre[0] = 0;
  for (size_t r = 0; r < nslices; ++r) tab.pre[r + 1] = tab.pre[r] + (uint32_t)counts[r];
  const uint32_t ew = (uint32_t)(elem_bytes / 16);
  const size_t units = (size_t)tab.pre[nslices] * ew;
  if (!units) return BPP_OK;
  hipLaunchKernelGGL(k_gather_blocks, dim3((unsigned)((units + 255) / 256)), dim3(256), 0, ctx->stream, src, stride,
                     off, ew, tab, (uint4*)dst);
  return ctx_check_launch(ctx, "k_gather_blocks");
}

// The MSM of a sharded batch over windows [wb, we) (bpp_perm_verify_partial_sharded):
// slice s's scalar block at d_blocks + s stride ([NG | counts[s] x npt]:
// the generator scalars summed over the slice, then its proof-point scalars)
// and its decompressed points at d_pblocks + s
// pstride (counts[s] x npt Niels records, bpp_perm_verify_slice_points); J is
// this rank's job over its own slice, batch proofs [first, first + J.count).
int verify_partial_sharded_dev(bpp_ctx* ctx, const bpp_gens* G, const bpp_verify_job& J, size_t first,
                               const uint8_t* d_blocks, size_t stride, const uint8_t* d_pblocks, size_t pstride,
                               const size_t* counts, size_t nslices, uint32_t wb, uint32_t we, h25519::ge* out) {
  if (J.dctx != ctx || J.dgen != ctx->vjob_gen) {
    ctx->err = "device verify job belongs to another context or was superseded by a later begin";
    return BPP_ERR_ARG;
  }
  if (J.rcount != J.count) {
    ctx->err = "a sharded batch takes one whole job per slice (bpp_perm_verify_begin_dev on the slice)";
    return BPP_ERR_ARG;
  }
  if (G->n < J.C.n_p) {
    ctx->err = "generators shorter than the padded circuit";
    return BPP_ERR_LEN;
  }
  const size_t NG = 2 * (size_t)J.C.n_p + 2, npt = J.npt, prec = (size_t)MSM_NIELS_WORDS * 4;
  size_t total = 0;
  bool mine = false, tight = true;  // (tight: the point blocks already lie end to end)
  for (size_t r = 0; r < nslices; ++r) {
    if ((NG + counts[r] * npt) * 32 > stride || counts[r] * npt * prec > pstride) return BPP_ERR_ARG;
    mine |= total == first && counts[r] == J.count;
    tight &= r + 1 == nslices || counts[r] * npt * prec == pstride;
    total += counts[r];
  }
  if (stride % 16 || pstride % 16 || total > (1u << 26)) return BPP_ERR_ARG;
  if (!mine) {
    ctx->err = "the gathered blocks do not hold this job's slice at its proof offset";
    return BPP_ERR_ARG;
  }
  const size_t T = NG + total * npt;
  void* d_sv = nullptr;
  BPP_TRY(ctx_ws(ctx, "pv_s", T * 32 + 32, &d_sv));
  BPP_TRY(verify_sum_blocks_dev(ctx, (uint32_t)nslices, (uint32_t)NG, (const uint32_t*)d_blocks,
                                (uint32_t)(stride / 4), (uint32_t*)d_sv));
  const uint8_t* d_x = d_pblocks;
  if (!tight) {
    void* d = nullptr;
    BPP_TRY(ctx_ws(ctx, "vj_xg", total * npt * prec, &d));
    d_x = (const uint8_t*)d;
  }
  // the slices' proof-point scalars (and, when padded, points) in proof order
  BPP_TRY(gather_blocks_dev(ctx, d_blocks, stride, NG * 32, npt * 32, counts, nslices, (uint8_t*)d_sv + NG * 32));
  if (!tight) BPP_TRY(gather_blocks_dev(ctx, d_pblocks, pstride, 0, npt * prec, counts, nslices, (uint8_t*)d_x));
  BPP_TRY(verify_msm(ctx, G, J.C, total, (const uint32_t*)d_sv, (const uint32_t*)d_x, wb, we, out));
  return ctx_sync(ctx);
}

// pass 2 of a device job: each proof's weight perm::batch_weight(seed,
// first + p, r_p) and constants (k_verify_consts), the weighted scalars
// (k_verify_scalars) and the MSM over windows [wb, we); BPP_ERR_VERIFY if a
// proof point did not decode or (an asynchronous begin) the replay rejected a
// proof.
int verify_partial_dev(bpp_ctx* ctx, const bpp_gens* G, const bpp_verify_job& J, const uint8_t seed[32],
                       size_t first, uint32_t wb, uint32_t we, h25519::ge* out) {
  if (J.dctx != ctx || J.dgen != ctx->vjob_gen) {
    ctx->err = "device verify job belongs to another context or was superseded by a later begin";
    return BPP_ERR_ARG;
  }
  if (J.rcount != J.count) {
    ctx->err = "a partially replayed job has no whole-batch partial";
    return BPP_ERR_ARG;
  }
  if (G->n < J.C.n_p) {
    ctx->err = "generators shorter than the padded circuit";
    return BPP_ERR_LEN;
  }
  const size_t count = J.count, T = 2 * (size_t)J.C.n_p + 2 + count * J.npt;
  void *d_rec = nullptr, *d_x = nullptr, *d_sv = nullptr, *d_dbad = nullptr;
  BPP_TRY(ctx_ws(ctx, "vj_rec", (count + 1) * vrec_n(J.C) * 32, &d_rec));
  BPP_TRY(ctx_ws(ctx, "vj_x", count * J.npt * MSM_NIELS_WORDS * 4, &d_x));
  BPP_TRY(ctx_ws(ctx, "vj_dbad", 8, &d_dbad));
  BPP_TRY(ctx_ws(ctx, "pv_s", T * 32 + 32, &d_sv));
  {
    HostScope hs(ctx, "verify_terms");
    uint32_t* h_seed = nullptr;
    BPP_TRY(ctx_zc_in(ctx, "vj_seed", seed, 32, &h_seed));
    BPP_TRY(verify_scalars_dev_rec(ctx, J.C, (uint32_t)count, (const uint32_t*)d_rec, h_seed, first,
                                   (uint32_t*)d_sv));
  }
  uint64_t* h_dbad = nullptr;  // the decompression's verdict, copied behind the MSM
  BPP_TRY(ctx_zc_out(ctx, "vj_dbad_h", 8, (uint32_t**)&h_dbad));
  BPP_HIP(hipStreamWaitEvent(ctx->stream, ctx->vj_ev_dec, 0));
  BPP_HIP(hipMemcpyAsync(h_dbad, d_dbad, 8, hipMemcpyDeviceToHost, ctx->stream));
  BPP_TRY(verify_msm(ctx, G, J.C, count, (const uint32_t*)d_sv, (const uint32_t*)d_x, wb, we, out));
  BPP_TRY(ctx_sync_latency(ctx));  // (msm_single_dev has synchronised; this keeps h_dbad's contract)
  if (J.bad_h) {  // an asynchronous begin's replay verdicts (the stream has passed them)
    uint32_t any = 0;
    for (size_t p = 0; p < J.rcount; ++p) any |= J.bad_h[p];
    if (any) {
      ctx->err = "a proof's transcript replay rejected it";
      return BPP_ERR_VERIFY;
    }
  }
  if (*h_dbad != ~0ull) {
    ctx->err = "undecodable proof point at index " + std::to_string(*h_dbad);
    return BPP_ERR_VERIFY;
  }
  return BPP_OK;
}

// Verify `count` proofs with ONE MSM: generator scalars summed across proofs
// with per-proof weights derived from every proof's r challenge; the
// transcripts are replayed on the device.
int verify_batch(bpp_ctx* ctx, const bpp_gens* G, const perm::Circuit& C, const uint8_t* label, size_t llen,
                 size_t count, const uint8_t* proofs, const uint8_t* V) {
  uint8_t seed[32];  // the verifier's own randomness for the batch weights
  if (!perm::verify_seed(seed)) {
    ctx->err = "getrandom failed";
    return BPP_ERR_DEVICE;
  }
  std::unique_ptr<bpp_verify_job> job;
  BPP_TRY(verify_begin_dev(ctx, C, label, llen, count, proofs, V, job, 0, SIZE_MAX, false));
  const uint32_t c = msm_choose_c((double)verify_terms(*job));
  h25519::ge res;
  BPP_TRY(verify_partial_dev(ctx, G, *job, seed, 0, 0, (254 + c - 1) / c, &res));
  uint8_t e[32];
  h25519::encode(e, res);
  static const uint8_t zero[32] = {0};
  return memcmp(e, zero, 32) == 0 ? BPP_OK : BPP_ERR_VERIFY;
}

}  // namespace

extern "C" {

size_t bpp_perm_proof_len(uint32_t k) { return k >= 2 && k <= (1u << 20) ? perm::proof_len(k) : 0; }

int bpp_perm_prove(bpp_ctx* ctx, const bpp_gens* G, uint32_t k, uint64_t seed, const uint8_t* label, size_t llen,
                   uint8_t* proof_out, uint8_t* V_out, uint32_t* perm_out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !G || !proof_out || !V_out || (!label && llen) || k < 2 || k > (1u << 20)) return BPP_ERR_ARG;
    const perm::Circuit C = perm::build(k);
    if (G->n < C.n_p) {
      ctx->err = "generators shorter than the padded circuit";
      return BPP_ERR_LEN;
    }
    BPP_HIP(hipSetDevice(ctx->device));
    std::vector<Proof> Ps;
    BPP_TRY(prove_batch(ctx, G, C, {perm::Seed::u64(seed)}, label, llen, Ps));
    serialize(C, Ps[0], proof_out);
    for (uint32_t j = 0; j < C.m; ++j) memcpy(V_out + 32 * j, Ps[0].V[j].data(), 32);
    if (perm_out) memcpy(perm_out, Ps[0].pi.data(), 4 * k);
    return BPP_OK;
  });
}

namespace {
std::vector<Proof>& proofs_tl() {
  static thread_local std::vector<Proof> Ps;
  return Ps;
}
}  // namespace

// wipe: prove_wipe after the batch, on ctx (this thread) and on every child
// context inside its sub-batch thread (whose prover states are its own)
static int prove_batch_api(bpp_ctx* ctx, const bpp_gens* G, uint32_t k, const std::vector<perm::Seed>& seeds,
                           const uint8_t* label, size_t llen, uint8_t* proofs_out, uint8_t* V_out,
                           bool wipe = false) {
  const size_t count = seeds.size();
  if (!count) return BPP_OK;
  const perm::Circuit C = perm::build(k);
  if (G->n < C.n_p) {
    ctx->err = "generators shorter than the padded circuit";
    return BPP_ERR_LEN;
  }
  BPP_HIP(hipSetDevice(ctx->device));
  const size_t pl = perm::proof_len(k);
  std::vector<Proof>& Ps = proofs_tl();  // reused batch after batch (ProverState note; the workers see this thread's)
  Ps.resize(count);
  // Sub-batches in flight on S streams (child contexts), one host thread
  // each: while one sub-batch waits on transcripts / challenges on the host,
  // the others' MSM and Pedersen kernels fill the GPU (a lockstep batch of
  // 128 proofs leaves most SIMDs idle in its latency-bound launch tails).
  // (default 1 until the concurrent path measures faster)
  size_t S = 1;
  if (const char* e = getenv("BPP_PROVE_STREAMS")) S = std::max<size_t>(1, std::min<size_t>(count, atoi(e)));
  {
    MsmPoints warm;  // build the window tables once, before the threads
    BPP_TRY(gens_points(ctx, G, &warm));
  }
  if (S <= 1) {
    BPP_TRY(prove_batch(ctx, G, C, seeds, label, llen, Ps));
  } else {
    std::vector<bpp_ctx*> kids(S);
    for (size_t s = 0; s < S; ++s) BPP_TRY(ctx_child(ctx, s, &kids[s]));
    std::vector<int> rcs(S, BPP_OK);
    std::vector<std::thread> th;
    for (size_t s = 0; s < S; ++s)
      th.emplace_back([&, s] {
        const size_t b = count * s / S, e = count * (s + 1) / S;
        bpp_ctx* kc = kids[s];
        kc->prof = ctx->prof;
        if (hipSetDevice(ctx->device) != hipSuccess) {
          rcs[s] = BPP_ERR_DEVICE;
          return;
        }
        std::vector<Proof> sub;
        std::vector<perm::Seed> part(seeds.begin() + b, seeds.begin() + e);
        rcs[s] = prove_batch(kc, G, C, part, label, llen, sub);
        if (rcs[s] == BPP_OK)
          for (size_t i = b; i < e; ++i) Ps[i] = std::move(sub[i - b]);
        if (wipe) {
          for (perm::Seed& x : part) memset(x.b, 0, sizeof x.b);
          for (Proof& q : sub) std::fill(q.pi.begin(), q.pi.end(), 0u);
          const int w = prove_wipe(kc);
          if (rcs[s] == BPP_OK) rcs[s] = w;
        }
      });
    for (auto& t : th) t.join();
    // (the children's stage times fold into ctx's on its next profile query)
    for (size_t s = 0; s < S; ++s)
      if (rcs[s] != BPP_OK) {
        ctx->err = kids[s]->err;
        return rcs[s];
      }
  }
  par::for_each(count, [&](size_t p) {
    serialize(C, Ps[p], proofs_out + p * pl);
    for (uint32_t j = 0; j < C.m; ++j) memcpy(V_out + (p * C.m + j) * 32, Ps[p].V[j].data(), 32);
  });
  return BPP_OK;
}

int bpp_perm_prove_batch(bpp_ctx* ctx, const bpp_gens* G, uint32_t k, size_t count, const uint64_t* seeds,
                         const uint8_t* label, size_t llen, uint8_t* proofs_out, uint8_t* V_out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !G || (!seeds && count) || ((!proofs_out || !V_out) && count) || (!label && llen) || k < 2 ||
        k > (1u << 20))
      return BPP_ERR_ARG;
    std::vector<perm::Seed> sd(count);
    for (size_t i = 0; i < count; ++i) sd[i] = perm::Seed::u64(seeds[i]);
    return prove_batch_api(ctx, G, k, sd, label, llen, proofs_out, V_out);
  });
}

int bpp_perm_prove_batch_entropy(bpp_ctx* ctx, const bpp_gens* G, uint32_t k, size_t count, const uint8_t* seeds32,
                                 const uint8_t* label, size_t llen, uint8_t* proofs_out, uint8_t* V_out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !G || ((!proofs_out || !V_out) && count) || (!label && llen) || k < 2 || k > (1u << 20))
      return BPP_ERR_ARG;
    std::vector<uint8_t> ent;
    if (!seeds32 && count) {  // the OS CSPRNG, the reference's thread_rng() (circuit_lib.rs:175)
      ent.resize(32 * count);
      size_t got = 0;
      while (got < ent.size()) {
        const ssize_t r = getrandom(ent.data() + got, ent.size() - got, 0);
        if (r < 0) {
          if (errno == EINTR) continue;
          ctx->err = "getrandom failed";
          return BPP_ERR_DEVICE;
        }
        got += (size_t)r;
      }
      seeds32 = ent.data();
    }
    std::vector<perm::Seed> sd(count);
    for (size_t i = 0; i < count; ++i) sd[i] = perm::Seed::bytes32(seeds32 + 32 * i);
    int rc = prove_batch_api(ctx, G, k, sd, label, llen, proofs_out, V_out, true);
    if (!ent.empty()) memset(ent.data(), 0, ent.size());
    for (perm::Seed& x : sd) memset(x.b, 0, sizeof x.b);
    const int wrc = prove_wipe(ctx);
    return rc ? rc : wrc;
  });
}

int bpp_debug_secret_residue(bpp_ctx* ctx, uint64_t* nonzero_bytes) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !nonzero_bytes) return BPP_ERR_ARG;
    BPP_HIP(hipSetDevice(ctx->device));
    BPP_TRY(ctx_sync(ctx));
    *nonzero_bytes = 0;
    return secret_residue(ctx, nonzero_bytes);
  });
}

int bpp_perm_verify(bpp_ctx* ctx, const bpp_gens* G, uint32_t k, const uint8_t* label, size_t llen,
                    const uint8_t* proof, size_t proof_len, const uint8_t* V) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !G || !proof || !V || (!label && llen) || k < 2 || k > (1u << 20)) return BPP_ERR_ARG;
    if (proof_len != perm::proof_len(k)) return BPP_ERR_VERIFY;
    BPP_HIP(hipSetDevice(ctx->device));
    const perm::Circuit C = perm::build(k);
    return verify_batch(ctx, G, C, label, llen, 1, proof, V);
  });
}

int bpp_perm_verify_batch(bpp_ctx* ctx, const bpp_gens* G, uint32_t k, size_t count, const uint8_t* label, size_t llen,
                          const uint8_t* proofs, const uint8_t* V) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !G || ((!proofs || !V) && count) || (!label && llen) || k < 2 || k > (1u << 20)) return BPP_ERR_ARG;
    if (!count) return BPP_OK;
    // (BPP_VERIFY_SPIN_US > 0: its syncs spin before sleeping, an A/B
    // switch, off: the verifier's waits already spin where they sit on the
    // critical path (ctx_sync_latency), and 300 us measured within noise,
    // profiles/r06_sync_spin_ab.txt)
    static const unsigned vspin = [] {
      const char* e = getenv("BPP_VERIFY_SPIN_US");
      return e ? (unsigned)std::max(0, atoi(e)) : 0u;
    }();
    SyncSpin spin(ctx, vspin ? vspin : ctx->sync_spin_us);
    BPP_HIP(hipSetDevice(ctx->device));
    const perm::Circuit C = perm::build(k);
    return verify_batch(ctx, G, C, label, llen, count, proofs, V);
  });
}

int bpp_perm_verify_begin(uint32_t k, size_t count, const uint8_t* label, size_t llen, const uint8_t* proofs,
                          const uint8_t* V, uint8_t* r_out, bpp_verify_job** out) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!out || ((!proofs || !V) && count) || (!label && llen) || k < 2 || k > (1u << 20)) return BPP_ERR_ARG;
    *out = nullptr;
    const perm::Circuit C = perm::build(k);
    std::unique_ptr<bpp_verify_job> job;
    BPP_TRY(verify_begin(C, label, llen, count, proofs, perm::proof_len(k), V, job));
    if (r_out)
      for (size_t p = 0; p < count; ++p) hsc::to_bytes(r_out + 32 * p, job->rs[p]);
    *out = job.release();
    return BPP_OK;
  });
}

int bpp_perm_verify_begin_dev(bpp_ctx* ctx, uint32_t k, size_t count, const uint8_t* label, size_t llen,
                              const uint8_t* proofs, const uint8_t* V, uint8_t* r_out, bpp_verify_job** out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !out || ((!proofs || !V) && count) || (!label && llen) || k < 2 || k > (1u << 20)) return BPP_ERR_ARG;
    *out = nullptr;
    BPP_HIP(hipSetDevice(ctx->device));
    const perm::Circuit C = perm::build(k);
    std::unique_ptr<bpp_verify_job> job;
    BPP_TRY(verify_begin_dev(ctx, C, label, llen, count, proofs, V, job));
    if (r_out && count) memcpy(r_out, job->rs.data(), 32 * count);
    *out = job.release();
    return BPP_OK;
  });
}

int bpp_perm_verify_begin_dev_async(bpp_ctx* ctx, uint32_t k, size_t count, const uint8_t* label, size_t llen,
                                    const uint8_t* proofs, const uint8_t* V, bpp_verify_job** out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !out || ((!proofs || !V) && count) || (!label && llen) || k < 2 || k > (1u << 20)) return BPP_ERR_ARG;
    *out = nullptr;
    BPP_HIP(hipSetDevice(ctx->device));
    const perm::Circuit C = perm::build(k);
    std::unique_ptr<bpp_verify_job> job;
    BPP_TRY(verify_begin_dev(ctx, C, label, llen, count, proofs, V, job, 0, SIZE_MAX, false));
    *out = job.release();
    return BPP_OK;
  });
}

int bpp_perm_verify_terms(const bpp_verify_job* job, size_t* terms) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!job || !terms) return BPP_ERR_ARG;
    *terms = verify_terms(*job);
    return BPP_OK;
  });
}

int bpp_verify_seed(uint8_t seed[32]) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!seed) return BPP_ERR_ARG;
    return perm::verify_seed(seed) ? BPP_OK : BPP_ERR_DEVICE;
  });
}

int bpp_perm_verify_scalars(const bpp_verify_job* job, const uint8_t seed[32], size_t first, uint8_t* scalars_out,
                            uint8_t* points_out) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!job || !seed || !scalars_out || (!points_out && job->count)) return BPP_ERR_ARG;
    if (job->dev) return BPP_ERR_ARG;  // (a device job keeps no host replay to expand)
    std::vector<Sc> sc;
    std::vector<uint8_t> enc;
    BPP_TRY(verify_terms_weighted(*job, seed, first, sc, enc));
    for (size_t i = 0; i < sc.size(); ++i) hsc::to_bytes(scalars_out + 32 * i, sc[i]);
    if (!enc.empty()) memcpy(points_out, enc.data(), enc.size());
    return BPP_OK;
  });
}

size_t bpp_perm_verify_slice_bytes(const bpp_verify_job* job) {
  return job ? (2 * (size_t)job->C.n_p + 2 + job->rcount * job->npt) * 32 : 0;
}

int bpp_perm_verify_slice_scalars_at(bpp_ctx* ctx, const bpp_verify_job* job, const uint8_t seed[32], size_t first,
                                     void* d_out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !job || !d_out || !seed || !job->dev || first > (1u << 26)) return BPP_ERR_ARG;
    BPP_HIP(hipSetDevice(ctx->device));
    return verify_slice_scalars_dev(ctx, *job, seed, first, (uint32_t*)d_out);
  });
}

size_t bpp_perm_verify_slice_point_bytes(const bpp_verify_job* job) {
  return job ? job->count * job->npt * MSM_NIELS_WORDS * 4 : 0;
}

int bpp_perm_verify_slice_points(bpp_ctx* ctx, const bpp_verify_job* job, void* d_out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !job || (!d_out && job->count) || !job->dev) return BPP_ERR_ARG;
    BPP_HIP(hipSetDevice(ctx->device));
    return verify_slice_points_dev(ctx, *job, d_out);
  });
}

int bpp_perm_verify_partial_sharded(bpp_ctx* ctx, const bpp_gens* G, const bpp_verify_job* job, size_t first,
                                    const void* d_blocks, size_t stride, const void* d_pblocks, size_t pstride,
                                    const size_t* counts, size_t nslices, uint32_t w_begin, uint32_t w_end,
                                    uint8_t partial[128]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !G || !job || !partial || !job->dev || !nslices || !d_blocks || !d_pblocks || !counts)
      return BPP_ERR_ARG;
    size_t total = 0;
    for (size_t r = 0; r < nslices; ++r) total += counts[r];
    const uint32_t c = msm_choose_c((double)(2 * (size_t)job->C.n_p + 2 + total * job->npt));
    if (w_begin > w_end || w_end > (254 + c - 1) / c) return BPP_ERR_ARG;
    BPP_HIP(hipSetDevice(ctx->device));
    h25519::ge r = h25519::ge_identity();
    if (total)
      BPP_TRY(verify_partial_sharded_dev(ctx, G, *job, first, (const uint8_t*)d_blocks, stride,
                                         (const uint8_t*)d_pblocks, pstride, counts, nslices, w_begin, w_end, &r));
    h25519::ge_to_words((uint32_t*)partial, r);
    return BPP_OK;
  });
}

int bpp_perm_verify_partial(bpp_ctx* ctx, const bpp_gens* G, const bpp_verify_job* job, const uint8_t seed[32],
                            size_t first, uint32_t w_begin, uint32_t w_end, uint8_t partial[128]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !G || !job || !partial || !seed) return BPP_ERR_ARG;
    const uint32_t c = msm_choose_c((double)verify_terms(*job));
    if (w_begin > w_end || w_end > (254 + c - 1) / c) return BPP_ERR_ARG;
    BPP_HIP(hipSetDevice(ctx->device));
    h25519::ge r = h25519::ge_identity();
    if (job->count) {
      if (job->dev)
        BPP_TRY(verify_partial_dev(ctx, G, *job, seed, first, w_begin, w_end, &r));
      else
        BPP_TRY(verify_partial(ctx, G, *job, seed, first, w_begin, w_end, &r));
    }
    h25519::ge_to_words((uint32_t*)partial, r);
    return BPP_OK;
  });
}

void bpp_perm_verify_end(bpp_verify_job* job) { delete job; }

int bpp_partials_is_identity(const uint8_t* partials, size_t count) {
  return bpp_guard(nullptr, [&]() -> int {
    uint8_t e[32];
    const int rc = bpp_partials_finish(partials, count, e);
    if (rc == BPP_ERR_ARG && partials) return BPP_ERR_VERIFY;  // a partial with Z = 0: never a pass
    BPP_TRY(rc);
    static const uint8_t zero[32] = {0};
    return memcmp(e, zero, 32) == 0 ? BPP_OK : BPP_ERR_VERIFY;
  });
}

}  // extern "C"
