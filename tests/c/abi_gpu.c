/* A C caller of include/bpperm.h's GPU entry points -- what a Rust
 * `extern "C"` shim under bp-perm would call at the reference's call sites
 * (circuit_lib.rs:187-229 vector commitments, :363-413 commitments, the IPA
 * the reference leaves as hook fields :62-63, and verify :478-585).  Compiled
 * and run by tests/test_gpu_abi_c.py on a GPU box; no ctypes in between.
 *
 * argv[1]: a text file of "name hex" lines written by the test from the
 * committed golden vectors (tests/golden/msm.json, protocol.json config2) and
 * the oracle (k = 4 permutation proofs from 32-byte seeds, the IPA verifier's P
 * scalars).  Checks, in order:
 *   bpp_ctx_create; bpp_msm against msm.json (64 and 1024 terms);
 *   bpp_gens_create(1024); bpp_vec_commit == config2 A;
 *   Merlin y; bpp_ipa_prove == config2 L, R, a, b;
 *   bpp_gens_export + bpp_msm for P; bpp_ipa_verify accepts, rejects a
 *   tampered a;
 *   the same IPA through bpp_ipa_prove_cb / bpp_ipa_verify_cb with a
 *   caller-owned C Merlin (merlin_min.h) behind the hooks: L, R, a, b equal
 *   config2, the hooks are called 2 + 2 lg / lg times, a tampered a is
 *   refused, a failing hook gives BPP_ERR_CALLBACK;
 *   bpp_perm_prove_batch_entropy (caller seeds) == oracle proofs and V;
 *   bpp_debug_secret_residue == 0; bpp_perm_verify_batch accepts, rejects a
 *   tampered proof; OS-entropy proofs verify; bpp_perm_verify (one proof).
 * Prints "ok" and exits 0 on success. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bpperm.h"
#include "merlin_min.h"

#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      fprintf(stderr, "FAILED line %d: %s\n", __LINE__, #c); \
      return 1;                                               \
    }                                                         \
  } while (0)

static char* g_text = NULL;

static int load(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  g_text = malloc((size_t)n + 1);
  if (fread(g_text, 1, (size_t)n, f) != (size_t)n) return -1;
  g_text[n] = 0;
  fclose(f);
  return 0;
}

/* bytes of the line "name hex"; *len receives the byte count (NULL if absent) */
static uint8_t* get(const char* name, size_t* len) {
  const size_t nl = strlen(name);
  for (char* p = g_text; p && *p;) {
    char* e = strchr(p, '\n');
    if (!strncmp(p, name, nl) && p[nl] == ' ') {
      const char* h = p + nl + 1;
      size_t hl = e ? (size_t)(e - h) : strlen(h);
      uint8_t* out = malloc(hl / 2 + 1);
      for (size_t i = 0; i < hl / 2; ++i) sscanf(h + 2 * i, "%2hhx", &out[i]);
      *len = hl / 2;
      return out;
    }
    p = e ? e + 1 : NULL;
  }
  *len = 0;
  return NULL;
}

/* bpp_transcript_hooks over the caller's transcript; fail_at > 0 makes the
 * fail_at-th call (1-based) fail */
struct hook_log {
  mm_transcript* t;
  int appends, challenges;
  int fail_at;
};
static int hook_append(void* user, const uint8_t* label, size_t llen, const uint8_t* msg, size_t mlen) {
  struct hook_log* h = (struct hook_log*)user;
  if (h->fail_at && h->appends + h->challenges + 1 == h->fail_at) return -1;
  ++h->appends;
  mm_append_message(h->t, label, llen, msg, mlen);
  return 0;
}
static int hook_challenge(void* user, const uint8_t* label, size_t llen, uint8_t* out, size_t n) {
  struct hook_log* h = (struct hook_log*)user;
  if (h->fail_at && h->appends + h->challenges + 1 == h->fail_at) return -1;
  ++h->challenges;
  mm_challenge_bytes(h->t, label, llen, out, n);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2 || load(argv[1])) {
    fprintf(stderr, "usage: abi_gpu INPUTS\n");
    return 2;
  }
  size_t len = 0, len2 = 0, len3 = 0;
  bpp_ctx* ctx = NULL;
  CHECK(bpp_ctx_create(0, &ctx) == BPP_OK && ctx);

  /* ---- vartime_multiscalar_mul (circuit_lib.rs:187 ...): msm.json cases */
  const char* cases[] = {"msm64", "msm1024"};
  for (int c = 0; c < 2; ++c) {
    char nm[64];
    snprintf(nm, sizeof nm, "%s_scalars", cases[c]);
    uint8_t* sc = get(nm, &len);
    snprintf(nm, sizeof nm, "%s_points", cases[c]);
    uint8_t* pts = get(nm, &len2);
    snprintf(nm, sizeof nm, "%s_result", cases[c]);
    uint8_t* want = get(nm, &len3);
    CHECK(sc && pts && want && len == len2 && len3 == 32);
    uint8_t out[32];
    CHECK(bpp_msm(ctx, sc, pts, len / 32, out) == BPP_OK);
    CHECK(memcmp(out, want, 32) == 0);
    /* dalek panics on a length mismatch; the ABI returns BPP_ERR_LEN or
     * BPP_ERR_ARG, never a result */
    CHECK(bpp_msm(ctx, sc, NULL, len / 32, out) != BPP_OK);
    free(sc);
    free(pts);
    free(want);
  }

  /* ---- config 2: A = alpha B~ + <aL, G> + <aR, H>, then the IPA */
  uint8_t* c2n = get("c2_n", &len);
  CHECK(c2n && len == 4);
  const size_t n = (size_t)c2n[0] | ((size_t)c2n[1] << 8) | ((size_t)c2n[2] << 16);
  uint8_t* aL = get("c2_aL", &len);
  uint8_t* aR = get("c2_aR", &len2);
  CHECK(aL && aR && len == 32 * n && len2 == 32 * n);
  uint8_t* alpha = get("c2_alpha", &len);
  uint8_t* q64 = get("c2_q64", &len2);
  CHECK(alpha && len == 32 && q64 && len2 == 64);
  bpp_gens* g = NULL;
  CHECK(bpp_gens_create(ctx, n, &g) == BPP_OK && bpp_gens_len(g) == n);
  uint8_t A[32];
  CHECK(bpp_vec_commit(ctx, g, alpha, aL, aR, n, A) == BPP_OK);
  uint8_t* wantA = get("c2_A", &len);
  CHECK(wantA && memcmp(A, wantA, 32) == 0);
  bpp_points* qp = NULL;
  CHECK(bpp_points_from_uniform(ctx, q64, 1, &qp) == BPP_OK);
  uint8_t Q[32];
  CHECK(bpp_points_compress(ctx, qp, Q) == BPP_OK);
  bpp_points_destroy(qp);
  bpp_transcript* tr = bpp_transcript_new((const uint8_t*)"config2", 7);
  CHECK(bpp_transcript_append_message(tr, (const uint8_t*)"A", 1, A, 32) == BPP_OK);
  uint8_t y[32];
  CHECK(bpp_transcript_challenge_scalar(tr, (const uint8_t*)"y", 1, y) == BPP_OK);
  uint8_t* wanty = get("c2_y", &len);
  CHECK(wanty && memcmp(y, wanty, 32) == 0);
  uint8_t* hf = get("c2_hf", &len); /* y^-i, i < n (scalar algebra on the caller's side) */
  CHECK(hf && len == 32 * n);
  size_t lg = 0;
  while (((size_t)1 << lg) < n) ++lg;
  uint8_t* Lo = malloc(32 * lg);
  uint8_t* Ro = malloc(32 * lg);
  uint8_t a[32], b[32];
  CHECK(bpp_ipa_prove(ctx, g, tr, Q, NULL, hf, aL, aR, n, Lo, Ro, a, b) == BPP_OK);
  uint8_t* wL = get("c2_L", &len);
  uint8_t* wR = get("c2_R", &len2);
  CHECK(wL && wR && len == 32 * lg && len2 == 32 * lg);
  CHECK(memcmp(Lo, wL, 32 * lg) == 0 && memcmp(Ro, wR, 32 * lg) == 0);
  uint8_t* wa = get("c2_a", &len);
  uint8_t* wb = get("c2_b", &len2);
  CHECK(wa && wb && memcmp(a, wa, 32) == 0 && memcmp(b, wb, 32) == 0);
  bpp_transcript_destroy(tr);

  /* ---- InnerProductProof::verify: P = <aL, G> + <aR o hf, H> + <aL, aR> Q
   * over the exported generators (scalars from the caller, one GPU MSM) */
  uint8_t* gexp = malloc(32 * (2 * n + 2));
  CHECK(bpp_gens_export(ctx, g, gexp) == BPP_OK);
  uint8_t* psc = get("c2_P_scalars", &len);
  CHECK(psc && len == 32 * (2 * n + 1));
  uint8_t* ppts = malloc(32 * (2 * n + 1));
  memcpy(ppts, gexp, 32 * 2 * n);
  memcpy(ppts + 32 * 2 * n, Q, 32);
  uint8_t P[32];
  CHECK(bpp_msm(ctx, psc, ppts, 2 * n + 1, P) == BPP_OK);
  for (int tamper = 0; tamper < 2; ++tamper) {
    bpp_transcript* tv = bpp_transcript_new((const uint8_t*)"config2", 7);
    CHECK(bpp_transcript_append_message(tv, (const uint8_t*)"A", 1, A, 32) == BPP_OK);
    CHECK(bpp_transcript_challenge_scalar(tv, (const uint8_t*)"y", 1, y) == BPP_OK);
    uint8_t av[32];
    memcpy(av, a, 32);
    av[0] ^= (uint8_t)tamper;
    const int rc = bpp_ipa_verify(ctx, g, tv, n, NULL, hf, P, Q, Lo, Ro, av, b);
    CHECK(rc == (tamper ? BPP_ERR_VERIFY : BPP_OK));
    bpp_transcript_destroy(tv);
  }

  /* ---- the same IPA over the CALLER's transcript (bpp_ipa_prove_cb): an
   * independent C Merlin (merlin_min.h) behind the hooks, as the Rust crate's
   * merlin::Transcript would be; A and y go through it before the IPA */
  {
    mm_transcript ct;
    struct hook_log lg0 = {&ct, 0, 0, 0};
    bpp_transcript_hooks hk = {&lg0, hook_append, hook_challenge};
    mm_new(&ct, (const uint8_t*)"config2", 7);
    mm_append_message(&ct, (const uint8_t*)"A", 1, A, 32);
    uint8_t ywide[64];
    mm_challenge_bytes(&ct, (const uint8_t*)"y", 1, ywide, 64); /* (y itself comes with the inputs) */
    uint8_t Lc[32 * 16], Rc[32 * 16], ac[32], bc[32];
    CHECK(lg <= 16);
    CHECK(bpp_ipa_prove_cb(ctx, g, &hk, Q, NULL, hf, aL, aR, n, Lc, Rc, ac, bc) == BPP_OK);
    CHECK(memcmp(Lc, wL, 32 * lg) == 0 && memcmp(Rc, wR, 32 * lg) == 0);
    CHECK(memcmp(ac, wa, 32) == 0 && memcmp(bc, wb, 32) == 0);
    /* dom-sep, n, then L, R, u per round */
    CHECK(lg0.appends == 2 + 2 * lg && lg0.challenges == lg);
    for (int tamper = 0; tamper < 2; ++tamper) {
      mm_transcript cv;
      struct hook_log lv = {&cv, 0, 0, 0};
      bpp_transcript_hooks hv = {&lv, hook_append, hook_challenge};
      mm_new(&cv, (const uint8_t*)"config2", 7);
      mm_append_message(&cv, (const uint8_t*)"A", 1, A, 32);
      mm_challenge_bytes(&cv, (const uint8_t*)"y", 1, ywide, 64);
      uint8_t av[32];
      memcpy(av, ac, 32);
      av[0] ^= (uint8_t)tamper;
      CHECK(bpp_ipa_verify_cb(ctx, g, &hv, n, NULL, hf, P, Q, Lc, Rc, av, bc) == (tamper ? BPP_ERR_VERIFY : BPP_OK));
    }
    /* a hook that fails aborts the call */
    mm_transcript cf;
    struct hook_log lf = {&cf, 0, 0, 3};
    bpp_transcript_hooks hf2 = {&lf, hook_append, hook_challenge};
    mm_new(&cf, (const uint8_t*)"config2", 7);
    CHECK(bpp_ipa_prove_cb(ctx, g, &hf2, Q, NULL, hf, aL, aR, n, Lc, Rc, ac, bc) == BPP_ERR_CALLBACK);
    CHECK(bpp_ipa_prove_cb(ctx, g, NULL, Q, NULL, hf, aL, aR, n, Lc, Rc, ac, bc) == BPP_ERR_ARG);
  }
  bpp_gens_destroy(g);

  /* ---- permutation proofs: production entry point with caller entropy */
  uint8_t* kb = get("perm_k", &len);
  uint8_t* seeds = get("perm_seeds32", &len2);
  CHECK(kb && len == 4 && seeds);
  const uint32_t k = kb[0];
  const size_t cnt = len2 / 32, plen = bpp_perm_proof_len(k), vlen = 32 * (2 * (size_t)k + 1);
  uint8_t* wantp = get("perm_proofs", &len);
  uint8_t* wantv = get("perm_V", &len2);
  CHECK(wantp && wantv && len == cnt * plen && len2 == cnt * vlen);
  bpp_gens* g2 = NULL;
  CHECK(bpp_gens_create(ctx, 128, &g2) == BPP_OK);
  uint8_t* pf = malloc(cnt * plen);
  uint8_t* V = malloc(cnt * vlen);
  const uint8_t* lab = (const uint8_t*)"bp-perm";
  CHECK(bpp_perm_prove_batch_entropy(ctx, g2, k, cnt, seeds, lab, 7, pf, V) == BPP_OK);
  CHECK(memcmp(pf, wantp, cnt * plen) == 0);
  CHECK(memcmp(V, wantv, cnt * vlen) == 0);
  uint64_t nz = 1;
  CHECK(bpp_debug_secret_residue(ctx, &nz) == BPP_OK && nz == 0);
  CHECK(bpp_perm_verify_batch(ctx, g2, k, cnt, lab, 7, pf, V) == BPP_OK);
  CHECK(bpp_perm_verify(ctx, g2, k, lab, 7, pf, plen, V) == BPP_OK);
  pf[plen + 40] ^= 1; /* proof 1's A_O */
  CHECK(bpp_perm_verify_batch(ctx, g2, k, cnt, lab, 7, pf, V) == BPP_ERR_VERIFY);
  pf[plen + 40] ^= 1;
  /* seeds32 = NULL: the OS CSPRNG */
  CHECK(bpp_perm_prove_batch_entropy(ctx, g2, k, cnt, NULL, lab, 7, pf, V) == BPP_OK);
  CHECK(memcmp(pf, wantp, cnt * plen) != 0);
  CHECK(bpp_perm_verify_batch(ctx, g2, k, cnt, lab, 7, pf, V) == BPP_OK);
  bpp_gens_destroy(g2);
  bpp_ctx_destroy(ctx);
  printf("ok\n");
  return 0;
}
