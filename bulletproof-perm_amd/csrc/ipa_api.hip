// C ABI: Merlin transcript handles, vector commitments and the inner-product
// argument (bpp_transcript_*, bpp_vec_commit, bpp_ipa_prove, bpp_ipa_verify).
#include <cstring>
#include <mutex>
#include <vector>

#include "ctx.h"
#include "gens.h"
#include "ge_io.cuh"
#include "ipa.h"
#include "msm_engine.h"
#include "host/par.h"

struct bpp_transcript {
  merlin::Transcript t;
};

// declared in points.hip
__global__ void k_decompress(const uint32_t* __restrict__ enc, size_t n, uint32_t* __restrict__ tbl,
                             unsigned long long* __restrict__ bad);

static unsigned grid_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// Decompress `count` host encodings into workspace `name`; BPP_ERR_DECOMPRESS
// on any invalid encoding.
int decompress_ws(bpp_ctx* ctx, const uint8_t* enc, size_t count, const char* name, uint32_t** d_out) {
  void *d_tbl, *d_enc, *d_bad;
  BPP_TRY(ctx_ws(ctx, name, (count ? count : 1) * MSM_NIELS_WORDS * 4, &d_tbl));
  *d_out = (uint32_t*)d_tbl;
  if (!count) return BPP_OK;
  {  // encodings read in place from pinned host memory (ctx_zc_in)
    uint32_t* h = nullptr;
    BPP_TRY(ctx_zc_in(ctx, "dws_enc_h", enc, count * 32, &h));
    d_enc = h;
  }
  BPP_TRY(ctx_ws(ctx, "dws_bad", 8, &d_bad));
  unsigned long long bad = ~0ull;
  BPP_TRY(ctx_h2d(ctx, d_bad, &bad, 8));
  hipLaunchKernelGGL(k_decompress, dim3(grid_for(count, 64)), dim3(64), 0, ctx->stream, (const uint32_t*)d_enc, count,
                     (uint32_t*)d_tbl, (unsigned long long*)d_bad);
  BPP_TRY(ctx_check_launch(ctx, "k_decompress"));
  BPP_TRY(ctx_d2h(ctx, &bad, d_bad, 8));
  if (bad != ~0ull) {
    ctx->err = "invalid point encoding at index " + std::to_string(bad);
    return BPP_ERR_DECOMPRESS;
  }
  return BPP_OK;
}

// One commitment or one IPA is a chain of short kernels and host steps:
// its syncs spin before sleeping (SyncSpin; BPP_IPA_SPIN_US, 0 = sleep at
// once as the throughput paths do)
static unsigned ipa_spin_us() {
  static const unsigned v = [] {
    const char* e = getenv("BPP_IPA_SPIN_US");
    return e ? (unsigned)std::max(0, atoi(e)) : 400u;
  }();
  return v;
}

// Canonical host scalars into the pinned buffer `name`, which the kernels
// read in place (null s: *d = null, all ones); a non-canonical scalar fails
// with its index before anything is queued.
static int zc_scalars(bpp_ctx* ctx, const uint8_t* s, size_t n, const char* name, uint32_t** d) {
  *d = nullptr;
  if (!s) return BPP_OK;
  for (size_t i = 0; i < n; ++i)
    if (!scalar_is_canonical(s + 32 * i)) {
      ctx->err = "non-canonical scalar at index " + std::to_string(i);
      return BPP_ERR_NONCANONICAL;
    }
  BPP_TRY(ctx_zc_out(ctx, name, 32 * n + 32, d));
  memcpy(*d, s, 32 * n);
  memset((uint8_t*)*d + 32 * n, 0, 32);
  return BPP_OK;
}

// Zeroes the pinned copies of the witness (a, b) when the call returns,
// error paths included (after their drain): no secret residue in pinned
// host memory once bpp_ipa_prove(_cb) is back.
struct IpaZcWipe {
  bpp_ctx* ctx;
  std::vector<std::pair<void*, size_t>> spans;
  explicit IpaZcWipe(bpp_ctx* c) : ctx(c) {}
  void add(void* p, size_t n) {
    if (p) spans.emplace_back(p, n);
  }
  ~IpaZcWipe() {
    for (auto& sp : spans) memset(sp.first, 0, sp.second);  // (persistent buffers: not a dead store)
  }
};

static int upload_opt(bpp_ctx* ctx, const uint8_t* s, size_t n, const char* name, uint32_t** d) {
  if (!s) {
    *d = nullptr;
    return BPP_OK;
  }
  return upload_scalars(ctx, s, n, name, d);
}

extern "C" {

bpp_transcript* bpp_transcript_new(const uint8_t* label, size_t len) {
  bpp_transcript* t = new bpp_transcript();
  t->t = merlin::Transcript(label, len);
  return t;
}
bpp_transcript* bpp_transcript_clone(const bpp_transcript* t) { return t ? new bpp_transcript(*t) : nullptr; }
void bpp_transcript_destroy(bpp_transcript* t) { delete t; }
int bpp_transcript_append_message(bpp_transcript* t, const uint8_t* label, size_t llen, const uint8_t* msg,
                                  size_t mlen) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!t || (!label && llen) || (!msg && mlen)) return BPP_ERR_ARG;
    t->t.append_message(label, llen, msg, mlen);
    return BPP_OK;
  });
}
int bpp_transcript_append_u64(bpp_transcript* t, const uint8_t* label, size_t llen, uint64_t x) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!t || (!label && llen)) return BPP_ERR_ARG;
    uint8_t b[8];
    memcpy(b, &x, 8);
    t->t.append_message(label, llen, b, 8);
    return BPP_OK;
  });
}
int bpp_transcript_challenge_bytes(bpp_transcript* t, const uint8_t* label, size_t llen, uint8_t* out, size_t n) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!t || (!label && llen) || (!out && n)) return BPP_ERR_ARG;
    std::string lab((const char*)label, llen);
    t->t.challenge_bytes(lab.c_str(), out, n);
    return BPP_OK;
  });
}
int bpp_transcript_challenge_scalar(bpp_transcript* t, const uint8_t* label, size_t llen, uint8_t out[32]) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!t || (!label && llen) || !out) return BPP_ERR_ARG;
    std::string lab((const char*)label, llen);
    hsc::to_bytes(out, t->t.challenge_scalar(lab.c_str()));
    return BPP_OK;
  });
}

int bpp_scalar_invert(const uint8_t x[32], uint8_t out[32]) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!x || !out) return BPP_ERR_ARG;
    hsc::Sc v;
    if (!hsc::from_canonical(v, x)) return BPP_ERR_NONCANONICAL;
    if (hsc::is_zero(v)) return BPP_ERR_ARG;
    hsc::to_bytes(out, hsc::invert(v));
    return BPP_OK;
  });
}

int bpp_scalar_powers(const uint8_t x[32], size_t n, uint8_t* out) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!x || (!out && n)) return BPP_ERR_ARG;
    hsc::Sc v;
    if (!hsc::from_canonical(v, x)) return BPP_ERR_NONCANONICAL;
    const std::vector<hsc::Sc> p = hsc::powers(v, n);
    for (size_t i = 0; i < n; ++i) hsc::to_bytes(out + 32 * i, p[i]);
    return BPP_OK;
  });
}

int bpp_vec_commit(bpp_ctx* ctx, const bpp_gens* g, const uint8_t blind[32], const uint8_t* a, const uint8_t* b,
                   size_t n, uint8_t out[32]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !g || !blind || !a || !out) return BPP_ERR_ARG;
    if (n > g->n) return BPP_ERR_LEN;
    SyncSpin spin(ctx, ipa_spin_us());
    BPP_HIP(hipSetDevice(ctx->device));
    const size_t T = 1 + n + (b ? n : 0);
    std::vector<uint8_t> sc(T * 32);
    std::vector<uint32_t> idx(T);
    memcpy(sc.data(), blind, 32);
    idx[0] = g->bbidx();
    memcpy(sc.data() + 32, a, 32 * n);
    for (size_t i = 0; i < n; ++i) idx[1 + i] = g->gidx(i);
    if (b) {
      memcpy(sc.data() + 32 * (1 + n), b, 32 * n);
      for (size_t i = 0; i < n; ++i) idx[1 + n + i] = g->hidx(i);
    }
    uint32_t* d_s = nullptr;
    BPP_TRY(upload_scalars(ctx, sc.data(), T, "vc_s", &d_s));
    void* d_i = nullptr;
    BPP_TRY(ctx_ws(ctx, "vc_i", T * 4, &d_i));
    BPP_TRY(ctx_h2d(ctx, d_i, idx.data(), T * 4));
    std::vector<h25519::ge> res;
    MsmPoints pts;
    BPP_TRY(gens_points(ctx, g, &pts));
    // one long MSM alone runs as one block (one wave per SIMD walking ~T/16
    // terms per lane in a row): cut it into J slices of >= 32 terms, J blocks
    // side by side, and add the J results here (ge_sum_auto) -- config 2's
    // 2049 terms: BPP_VC_SPLIT caps J (default 64; config 2 at 16 / 32 / 64
    // slices 1.016-1.024 / 0.996-1.004 / 0.979-0.996 ms, r06_vc_split_ab.txt)
    static const size_t vc_split = [] {
      const char* e = getenv("BPP_VC_SPLIT");
      return (size_t)std::max(1, e ? atoi(e) : 64);
    }();
    const uint32_t J = (uint32_t)std::max<size_t>(1, std::min<size_t>(vc_split, T / 32));
    std::vector<uint32_t> off(J + 1);
    for (uint32_t j = 0; j <= J; ++j) off[j] = (uint32_t)((uint64_t)T * j / J);
    BPP_TRY(msm_multi(ctx, d_s, (const uint32_t*)d_i, off, pts, res));
    h25519::ge acc;
    h25519::ge_sum_auto(res.data(), 1, J, &acc);
    h25519::encode(out, acc);
    return BPP_OK;
  });
}

}  // extern "C" (C++ helpers below)

bool msm_use_dt(const MsmPoints& pts, uint32_t M, uint32_t T);  // msm.hip

namespace {
// host extended point -> the device's 128-B Niels row (y + x, y - x, 2 d x y
// in 10 limbs at bit offsets ceil(25.5 i), ge_io.cuh store_niels); zi = 1 / Z
void niels_row_host(const h25519::ge& p, const h25519::fe& zi, uint32_t w[MSM_NIELS_WORDS]) {
  namespace H = h25519;
  const H::fe x = H::fe_mul(p.X, zi), y = H::fe_mul(p.Y, zi);
  const H::fe f[3] = {H::fe_add(y, x), H::fe_sub(y, x), H::fe_mul(H::fe_mul(x, y), H::FE_D2)};
  for (int e = 0; e < 3; ++e) {
    const H::fe c = H::fe_canon(f[e]);
    for (int k = 0; k < 5; ++k) {
      w[10 * e + 2 * k] = (uint32_t)(c.v[k] & 0x3ffffffu);
      w[10 * e + 2 * k + 1] = (uint32_t)(c.v[k] >> 26);
    }
  }
  w[30] = w[31] = 0;
}

// Q into the generators' Q slot (gens.h): its window points 2^(8u) Q, u <
// 32, on the host (248 doublings: ~35 us, where one GPU lane's chain took
// ~0.5 ms), their Niels rows uploaded as a window table, then Q's direct-table
// rows built on the device into slot 2n + 2 and its Niels row into d_tbl.
// The caller holds g->q_mu until the IPA using the slot has completed.
int ipa_q_slot(bpp_ctx* ctx, const bpp_gens* g, const uint8_t Q[32], uint32_t dt_c) {
  h25519::ge P;
  if (!h25519::decode(P, Q)) {
    ctx->err = "Q does not decode";
    return BPP_ERR_DECOMPRESS;
  }
  std::vector<uint32_t> wt((size_t)FBW_W * MSM_NIELS_WORDS);
  std::vector<h25519::ge> pts(FBW_W);
  h25519::ge cur = P;
  for (uint32_t u = 0; u < FBW_W; ++u) {
    pts[u] = cur;
    for (uint32_t i = 0; i < FBW_C; ++i) cur = h25519::ge_dbl(cur);
  }
  // the FBW_W inverses of Z by one field inversion (Montgomery's trick): the
  // latency of bpp_ipa_prove on a fresh Q (config 2: ~75 -> ~15 us of host time)
  std::vector<h25519::fe> pre(FBW_W);
  h25519::fe run = h25519::fe_one();
  for (uint32_t u = 0; u < FBW_W; ++u) {
    pre[u] = run;
    run = h25519::fe_mul(run, pts[u].Z);  // (Z is never zero for a decoded point)
  }
  h25519::fe inv = h25519::fe_invert(run);
  for (uint32_t u = FBW_W; u-- > 0;) {
    const h25519::fe zi = h25519::fe_mul(inv, pre[u]);
    inv = h25519::fe_mul(inv, pts[u].Z);
    niels_row_host(pts[u], zi, &wt[(size_t)u * MSM_NIELS_WORDS]);
  }
  void* d_wt = nullptr;
  BPP_TRY(ctx_ws(ctx, "ipa_q_wt", wt.size() * 4, &d_wt));
  BPP_TRY(ctx_h2d(ctx, d_wt, wt.data(), wt.size() * 4));
  // (slot rows start after the 2n + 2 generators' rows: dt_bytes per point)
  uint32_t* slot = g->d_dt + dt_bytes(g->qslot(), dt_c) / 4;
  BPP_TRY(dt_build(ctx, (const uint32_t*)d_wt, 1, dt_c, slot));
  BPP_HIP(hipMemcpyAsync(g->d_tbl + (size_t)g->qslot() * MSM_NIELS_WORDS, d_wt, MSM_NIELS_WORDS * 4,
                         hipMemcpyDeviceToDevice, ctx->stream));
  return BPP_OK;
}
// Q as its doublings 2^j Q, j < 253 (IpaGens::qpow): 253 doublings on the
// host (the window points of a Q-slot table took 248), their Z inverses by
// one field inversion, and the 253 Niels rows written over the start of g's
// Q slot (the caller holds g->q_mu until the IPA has completed).  The fused
// rounds then add c Q bit by bit (ipa.hip q_bits_*, DtLane::row_of_q): no
// direct table is built for Q, where its build was 152 us of config 2.
int ipa_q_powers(bpp_ctx* ctx, const bpp_gens* g, const uint8_t Q[32], uint32_t dt_c, const uint32_t** d_out) {
  h25519::ge P;
  if (!h25519::decode(P, Q)) {
    ctx->err = "Q does not decode";
    return BPP_ERR_DECOMPRESS;
  }
  constexpr uint32_t NB = 253;
  std::vector<h25519::ge> pts(NB);
  for (uint32_t j = 0; j < NB; ++j) {
    pts[j] = P;
    P = h25519::ge_dbl(P);
  }
  // the Niels rows in four chunks on the pool, one field inversion per chunk
  // (Montgomery's trick): ~3/4 of the conversion's ~30 us off this thread
  std::vector<uint32_t> rows((size_t)NB * MSM_NIELS_WORDS);
  constexpr uint32_t NCH = 4;
  par::for_each(NCH, [&](size_t c) {
    const uint32_t j0 = (uint32_t)(NB * c / NCH), j1 = (uint32_t)(NB * (c + 1) / NCH);
    std::vector<h25519::fe> pre(j1 - j0);
    h25519::fe run = h25519::fe_one();
    for (uint32_t j = j0; j < j1; ++j) {
      pre[j - j0] = run;
      run = h25519::fe_mul(run, pts[j].Z);  // (Z is never zero for a decoded point)
    }
    h25519::fe inv = h25519::fe_invert(run);
    for (uint32_t j = j1; j-- > j0;) {
      const h25519::fe zi = h25519::fe_mul(inv, pre[j - j0]);
      inv = h25519::fe_mul(inv, pts[j].Z);
      niels_row_host(pts[j], zi, &rows[(size_t)j * MSM_NIELS_WORDS]);
    }
  });
  uint32_t* slot = g->d_dt + dt_bytes(g->qslot(), dt_c) / 4;
  BPP_TRY(ctx_h2d(ctx, slot, rows.data(), rows.size() * 4));
  *d_out = slot;
  return BPP_OK;
}
}  // namespace

static int ipa_prove_api(bpp_ctx* ctx, const bpp_gens* g, IpaTranscript* tr, const uint8_t Q[32],
                         const uint8_t* G_factors, const uint8_t* H_factors, const uint8_t* a, const uint8_t* b,
                         size_t n, uint8_t* L_out, uint8_t* R_out, uint8_t a_out[32], uint8_t b_out[32]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !g || !tr || !Q || !a || !b || !a_out || !b_out || ((!L_out || !R_out) && n > 1)) return BPP_ERR_ARG;
    if (n == 0 || (n & (n - 1)) || n > g->n) return BPP_ERR_LEN;
    SyncSpin spin(ctx, ipa_spin_us());
    BPP_HIP(hipSetDevice(ctx->device));
    uint32_t *d_a, *d_b, *d_gf, *d_hf, *d_q;
    IpaGens ig;
    BPP_TRY(gens_points(ctx, g, &ig.pts));
    ig.gbase = 0;
    ig.hbase = (uint32_t)g->n;
    // Q in the generators' slot when they have direct tables and the rounds
    // can run fused (BPP_IPA_QSLOT=0: Q as an extra point, the four-kernel
    // rounds over the generic engine)
    static const bool qslot_env = [] {
      const char* e = getenv("BPP_IPA_QSLOT");
      return !e || atoi(e) != 0;
    }();
    std::unique_lock<std::mutex> qlock;
    // (exactly the fused rounds' condition, ipa.hip: the slot has direct-table
    // rows and a Niels row only, no window-table rows for the other engines)
    const bool qslot =
        qslot_env && n >= 2 && n <= IPA_FUSED_NMAX && msm_use_dt(ig.pts, 2, (uint32_t)(2 * n + 2));
    // the fused path: Q's table build is queued first, and a, b and the
    // factors are read in place by round 0 from pinned host memory (each
    // element once) -- the inputs' staging copies and H2D enqueues, ~40 us
    // of host time, run beside the build instead of before it
    bool zc_in = false;
    IpaZcWipe wipe(ctx);  // (destroyed before qlock: the drain below runs first)
    IpaProofHost pf;
    // Q in the fused rounds: by its doublings (IpaGens::qpow, default) or in
    // g's Q slot with a per-call direct table (BPP_IPA_QPOW=0)
    static const bool qpow_env = [] {
      const char* e = getenv("BPP_IPA_QPOW");
      return !e || atoi(e) != 0;
    }();
    auto body = [&]() -> int {
      if (qslot) {
        qlock = std::unique_lock<std::mutex>(g->q_mu);
        if (qpow_env)
          BPP_TRY(ipa_q_powers(ctx, g, Q, ig.pts.dt_c, &ig.qpow));
        else
          BPP_TRY(ipa_q_slot(ctx, g, Q, ig.pts.dt_c));
        ig.qidx = g->qslot();
        static const bool zc_env = [] {
          const char* e = getenv("BPP_IPA_ZC_IN");
          return !e || atoi(e) != 0;
        }();
        zc_in = zc_env;
      } else {
        BPP_TRY(decompress_ws(ctx, Q, 1, "ipa_q", &d_q));
        BPP_TRY(msm_points_extra(ctx, &ig.pts, d_q, 1, (uint32_t)(2 * g->n + 2), "ipa_q_wt", (double)(n + 1)));
        ig.qidx = ig.pts.n0;
      }
      if (zc_in) {
        BPP_TRY(zc_scalars(ctx, a, n, "ipa_zc_a", &d_a));
        wipe.add(d_a, 32 * n);
        BPP_TRY(zc_scalars(ctx, b, n, "ipa_zc_b", &d_b));
        wipe.add(d_b, 32 * n);
        BPP_TRY(zc_scalars(ctx, G_factors, n, "ipa_zc_gf", &d_gf));
        BPP_TRY(zc_scalars(ctx, H_factors, n, "ipa_zc_hf", &d_hf));
      } else {
        BPP_TRY(upload_scalars(ctx, a, n, "ipa_in_a", &d_a));
        BPP_TRY(upload_scalars(ctx, b, n, "ipa_in_b", &d_b));
        BPP_TRY(upload_opt(ctx, G_factors, n, "ipa_in_gf", &d_gf));
        BPP_TRY(upload_opt(ctx, H_factors, n, "ipa_in_hf", &d_hf));
      }
      return ipa_prove_dev(ctx, *tr, ig, (uint32_t)n, d_gf, d_hf, d_a, d_b, pf);
    };
    int rc;
    try {
      rc = body();
    } catch (const std::bad_alloc&) {
      rc = BPP_ERR_NOMEM;
    } catch (...) {
      rc = BPP_ERR_DEVICE;
    }
    // a failed call (a non-canonical input, a hook error, a device error)
    // may leave this context's kernels queued on the Q slot (its build is
    // queued first) or reading the pinned inputs: drain them before the
    // slot's lock goes and the inputs are wiped
    if (rc != BPP_OK && (qlock.owns_lock() || zc_in)) (void)hipStreamSynchronize(ctx->stream);
    BPP_TRY(rc);
    for (size_t j = 0; j < pf.L.size(); ++j) {
      memcpy(L_out + 32 * j, pf.L[j].data(), 32);
      memcpy(R_out + 32 * j, pf.R[j].data(), 32);
    }
    hsc::to_bytes(a_out, pf.a);
    hsc::to_bytes(b_out, pf.b);
    return BPP_OK;
  });
}

static int ipa_verify_api(bpp_ctx* ctx, const bpp_gens* g, IpaTranscript* tr, size_t n, const uint8_t* G_factors,
                          const uint8_t* H_factors, const uint8_t P[32], const uint8_t Q[32], const uint8_t* L,
                          const uint8_t* R, const uint8_t a[32], const uint8_t b[32]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !g || !tr || !P || !Q || !a || !b || ((!L || !R) && n > 1)) return BPP_ERR_ARG;
    if (n == 0 || (n & (n - 1)) || n > g->n) return BPP_ERR_LEN;
    SyncSpin spin(ctx, ipa_spin_us());
    BPP_HIP(hipSetDevice(ctx->device));
    uint32_t lg = 0;
    while ((1u << lg) < n) ++lg;
    std::vector<Enc32> Lv(lg), Rv(lg);
    for (uint32_t j = 0; j < lg; ++j) {
      memcpy(Lv[j].data(), L + 32 * j, 32);
      memcpy(Rv[j].data(), R + 32 * j, 32);
    }
    hsc::Sc as, bs;
    if (!hsc::from_canonical(as, a) || !hsc::from_canonical(bs, b)) return BPP_ERR_NONCANONICAL;
    std::vector<hsc::Sc> gf(n, hsc::one()), hf(n, hsc::one());
    for (size_t i = 0; i < n; ++i) {
      if (G_factors && !hsc::from_canonical(gf[i], G_factors + 32 * i)) return BPP_ERR_NONCANONICAL;
      if (H_factors && !hsc::from_canonical(hf[i], H_factors + 32 * i)) return BPP_ERR_NONCANONICAL;
    }
    std::vector<hsc::Sc> u_sq, uinv_sq, s;
    bool hook_failed = false;
    if (!ipa_verification_scalars(*tr, (uint32_t)n, Lv, Rv, u_sq, uinv_sq, s, &hook_failed)) {
      if (hook_failed) ctx->err = "ipa: a transcript hook returned an error";
      return hook_failed ? BPP_ERR_CALLBACK : BPP_ERR_VERIFY;
    }
    // extra points: Q, L_0.., R_0.., P
    std::vector<uint8_t> extra((2 + 2 * lg) * 32);
    memcpy(extra.data(), Q, 32);
    memcpy(extra.data() + 32, L, 32 * lg);
    memcpy(extra.data() + 32 * (1 + lg), R, 32 * lg);
    memcpy(extra.data() + 32 * (1 + 2 * lg), P, 32);
    uint32_t* d_x = nullptr;
    int rc = decompress_ws(ctx, extra.data(), extra.size() / 32, "ipav_x", &d_x);
    if (rc == BPP_ERR_DECOMPRESS) return BPP_ERR_VERIFY;
    BPP_TRY(rc);
    const uint32_t n0 = (uint32_t)(2 * g->n + 2);
    const size_t T = 1 + 2 * n + 2 * lg + 1;
    std::vector<uint8_t> sc(T * 32);
    std::vector<uint32_t> idx(T);
    size_t t = 0;
    auto put = [&](const hsc::Sc& x, uint32_t i) {
      hsc::to_bytes(sc.data() + 32 * t, x);
      idx[t++] = i;
    };
    put(hsc::mul(as, bs), n0);
    for (size_t i = 0; i < n; ++i) put(hsc::mul(hsc::mul(as, s[i]), gf[i]), g->gidx(i));
    for (size_t i = 0; i < n; ++i) put(hsc::mul(hsc::mul(bs, s[n - 1 - i]), hf[i]), g->hidx(i));
    for (uint32_t j = 0; j < lg; ++j) put(hsc::neg(u_sq[j]), n0 + 1 + j);
    for (uint32_t j = 0; j < lg; ++j) put(hsc::neg(uinv_sq[j]), n0 + 1 + lg + j);
    put(hsc::neg(hsc::one()), n0 + 1 + 2 * lg);
    uint32_t* d_s = nullptr;
    BPP_TRY(upload_scalars(ctx, sc.data(), T, "ipav_s", &d_s));
    void* d_i = nullptr;
    BPP_TRY(ctx_ws(ctx, "ipav_i", T * 4, &d_i));
    BPP_TRY(ctx_h2d(ctx, d_i, idx.data(), T * 4));
    std::vector<h25519::ge> res;
    MsmPoints pts;
    BPP_TRY(gens_points(ctx, g, &pts));
    BPP_TRY(msm_points_extra(ctx, &pts, d_x, (uint32_t)(2 + 2 * lg), n0, "ipav_x_wt", (double)T));
    BPP_TRY(msm_multi(ctx, d_s, (const uint32_t*)d_i, {0, (uint32_t)T}, pts, res));
    uint8_t e[32];
    h25519::encode(e, res[0]);
    static const uint8_t zero[32] = {0};
    return memcmp(e, zero, 32) == 0 ? BPP_OK : BPP_ERR_VERIFY;
  });
}

namespace {
// the caller's transcript behind C hooks (bpp_transcript_hooks)
struct IpaHooks final : IpaTranscript {
  const bpp_transcript_hooks& h;
  explicit IpaHooks(const bpp_transcript_hooks& hooks) : h(hooks) {}
  bool append(const char* label, const uint8_t* msg, size_t n) override {
    return h.append_message(h.user, (const uint8_t*)label, strlen(label), msg, n) == 0;
  }
  bool challenge(const char* label, uint8_t* out, size_t n) override {
    return h.challenge_bytes(h.user, (const uint8_t*)label, strlen(label), out, n) == 0;
  }
};
bool hooks_ok(const bpp_transcript_hooks* h) { return h && h->append_message && h->challenge_bytes; }
}  // namespace

extern "C" {

int bpp_ipa_prove_cb(bpp_ctx* ctx, const bpp_gens* g, const bpp_transcript_hooks* tr, const uint8_t Q[32],
                     const uint8_t* G_factors, const uint8_t* H_factors, const uint8_t* a, const uint8_t* b, size_t n,
                     uint8_t* L_out, uint8_t* R_out, uint8_t a_out[32], uint8_t b_out[32]) {
  if (!hooks_ok(tr)) return BPP_ERR_ARG;
  IpaHooks t(*tr);
  return ipa_prove_api(ctx, g, &t, Q, G_factors, H_factors, a, b, n, L_out, R_out, a_out, b_out);
}

int bpp_ipa_verify_cb(bpp_ctx* ctx, const bpp_gens* g, const bpp_transcript_hooks* tr, size_t n,
                      const uint8_t* G_factors, const uint8_t* H_factors, const uint8_t P[32], const uint8_t Q[32],
                      const uint8_t* L, const uint8_t* R, const uint8_t a[32], const uint8_t b[32]) {
  if (!hooks_ok(tr)) return BPP_ERR_ARG;
  IpaHooks t(*tr);
  return ipa_verify_api(ctx, g, &t, n, G_factors, H_factors, P, Q, L, R, a, b);
}

// the library's own Merlin behind the same code path
int bpp_ipa_prove(bpp_ctx* ctx, const bpp_gens* g, bpp_transcript* tr, const uint8_t Q[32], const uint8_t* G_factors,
                  const uint8_t* H_factors, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* L_out,
                  uint8_t* R_out, uint8_t a_out[32], uint8_t b_out[32]) {
  if (!tr) return BPP_ERR_ARG;
  IpaMerlin t(tr->t);
  return ipa_prove_api(ctx, g, &t, Q, G_factors, H_factors, a, b, n, L_out, R_out, a_out, b_out);
}

int bpp_ipa_verify(bpp_ctx* ctx, const bpp_gens* g, bpp_transcript* tr, size_t n, const uint8_t* G_factors,
                   const uint8_t* H_factors, const uint8_t P[32], const uint8_t Q[32], const uint8_t* L,
                   const uint8_t* R, const uint8_t a[32], const uint8_t b[32]) {
  if (!tr) return BPP_ERR_ARG;
  IpaMerlin t(tr->t);
  return ipa_verify_api(ctx, g, &t, n, G_factors, H_factors, P, Q, L, R, a, b);
}

}  // extern "C"
