/*
 * perm_cpu.c — serial C restatement of the permutation prover as the
 * reference would run it on a CPU.  TEST INFRASTRUCTURE / CPU BASELINE ONLY.
 *
 * Same protocol as oracle/bulletproofs.py ac_prove (sound mode, DESIGN.md
 * §2; reference circuit_lib.rs:139-253, weights.rs:26-204) with the
 * reference's *algorithms* for every piece the GPU build replaces:
 *   - MSMs through dalek-ng's vartime dispatch (dalek_port.c: Straus below
 *     190 terms, Pippenger above), Pedersen commits as 2-term MSMs
 *     (bulletproofs PedersenGens::commit, weights.rs:58-61)
 *   - bulletproofs 4.0.0 InnerProductProof::create in its FOLDING form: each
 *     round folds G and H with one 2-term MSM per element
 *   - merlin 3.0.0 transcript (STROBE-128 over Keccak-f[1600]), Scalar mod l
 *     (4 x u64 Montgomery), sparse circuit matrices (the reference's are
 *     dense, util.rs:22-56; sparse is the faster, fairer baseline)
 * It is an independent second implementation of the proof bytes: tests
 * compare it with the Python oracle and the GPU product.  Single-threaded;
 * the bench times it on 1 core and on all cores (one proof per thread).
 */
#include "dalek_port.c"

/* ================================================================ scalars */
typedef struct { uint64_t v[4]; } sc_t;
static const sc_t SC_L = {{0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0x0ULL, 0x1000000000000000ULL}};
static const sc_t SC_R2 = {{0xa40611e3449c0f01ULL, 0xd00e1ba768859347ULL, 0xceec73d217f5be65ULL, 0x0399411b7c309a3dULL}};
static const sc_t SC_R3 = {{0x2a9e49687b83a2dbULL, 0x278324e6aef7f3ecULL, 0x8065dc6c04ec5b65ULL, 0x0e530b773599cec7ULL}};
static const uint64_t SC_LINV = 0xd2b51da312547e1bULL;
static const sc_t SC_ZERO = {{0, 0, 0, 0}}, SC_ONE = {{1, 0, 0, 0}};

static int sc_geq(const sc_t* a, const sc_t* b) {
  for (int i = 3; i >= 0; --i)
    if (a->v[i] != b->v[i]) return a->v[i] > b->v[i];
  return 1;
}
static sc_t sc_subraw(sc_t a, const sc_t* b, uint64_t* bo) {
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a.v[i] - b->v[i] - br;
    a.v[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (bo) *bo = br;
  return a;
}
static sc_t sc_add(sc_t a, sc_t b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c = (u128)a.v[i] + b.v[i] + (uint64_t)(c >> 64);
    a.v[i] = (uint64_t)c;
  }
  if (sc_geq(&a, &SC_L)) a = sc_subraw(a, &SC_L, 0);
  return a;
}
static sc_t sc_sub(sc_t a, sc_t b) {
  uint64_t br;
  sc_t r = sc_subraw(a, &b, &br);
  if (br) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
      c = (u128)r.v[i] + SC_L.v[i] + (uint64_t)(c >> 64);
      r.v[i] = (uint64_t)c;
    }
  }
  return r;
}
static sc_t sc_neg(sc_t a) { return sc_sub(SC_ZERO, a); }
static sc_t sc_mont(sc_t a, sc_t b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c = (u128)a.v[i] * b.v[j] + t[j] + (uint64_t)(c >> 64);
      t[j] = (uint64_t)c;
    }
    c = (u128)t[4] + (uint64_t)(c >> 64);
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * SC_LINV;
    c = (u128)m * SC_L.v[0] + t[0];
    for (int j = 1; j < 4; ++j) {
      c = (u128)m * SC_L.v[j] + t[j] + (uint64_t)(c >> 64);
      t[j - 1] = (uint64_t)c;
    }
    c = (u128)t[4] + (uint64_t)(c >> 64);
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  sc_t r = {{t[0], t[1], t[2], t[3]}};
  if (t[4] || sc_geq(&r, &SC_L)) r = sc_subraw(r, &SC_L, 0);
  return r;
}
static sc_t sc_mul(sc_t a, sc_t b) { return sc_mont(sc_mont(a, b), SC_R2); }
static sc_t sc_u64(uint64_t x) { sc_t r = {{x, 0, 0, 0}}; return r; }
static sc_t sc_from_wide(const uint8_t b[64]) {
  sc_t lo, hi;
  memcpy(lo.v, b, 32);
  memcpy(hi.v, b + 32, 32);
  return sc_mont(sc_add(sc_mont(lo, SC_R2), sc_mont(hi, SC_R3)), SC_ONE);
}
static sc_t sc_inv(sc_t a) {
  sc_t e = sc_subraw(SC_L, &(sc_t){{2, 0, 0, 0}}, 0), r = SC_ONE;
  for (int i = 255; i >= 0; --i) {
    r = sc_mul(r, r);
    if ((e.v[i >> 6] >> (i & 63)) & 1) r = sc_mul(r, a);
  }
  return r;
}
static sc_t sc_inner(const sc_t* a, const sc_t* b, size_t n) {
  sc_t r = SC_ZERO;
  for (size_t i = 0; i < n; ++i) r = sc_add(r, sc_mul(a[i], b[i]));
  return r;
}
static void sc_powers(sc_t x, sc_t* out, size_t n) {
  sc_t c = SC_ONE;
  for (size_t i = 0; i < n; ++i) { out[i] = c; c = sc_mul(c, x); }
}

/* ================================================================ Keccak / XOFs */
static uint64_t k_rol(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }
static void keccakf(uint64_t s[25]) {
  static const uint64_t RC[24] = {
      0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
      0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
      0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
      0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
      0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
      0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
  static const int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  for (int round = 0; round < 24; ++round) {
    uint64_t C[5], D[5], B[25];
    for (int x = 0; x < 5; ++x) C[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
    for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ k_rol(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) s[i] ^= D[i % 5];
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = k_rol(s[x + 5 * y], R[x + 5 * y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) s[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]);
    s[0] ^= RC[round];
  }
}

/* sponge with rate r and domain byte ds (SHAKE256: 136, 0x1F; SHA3-512: 72, 0x06) */
typedef struct { uint64_t s[25]; size_t rate, pos; uint8_t ds; int squeezing; } sponge_t;
static void sp_init(sponge_t* p, size_t rate, uint8_t ds) { memset(p, 0, sizeof *p); p->rate = rate; p->ds = ds; }
static void sp_absorb(sponge_t* p, const uint8_t* d, size_t n) {
  uint8_t* st = (uint8_t*)p->s;
  for (size_t i = 0; i < n; ++i) {
    st[p->pos++] ^= d[i];
    if (p->pos == p->rate) { keccakf(p->s); p->pos = 0; }
  }
}
static void sp_squeeze(sponge_t* p, uint8_t* out, size_t n) {
  uint8_t* st = (uint8_t*)p->s;
  if (!p->squeezing) {
    st[p->pos] ^= p->ds;
    st[p->rate - 1] ^= 0x80;
    keccakf(p->s);
    p->pos = 0;
    p->squeezing = 1;
  }
  for (size_t i = 0; i < n; ++i) {
    if (p->pos == p->rate) { keccakf(p->s); p->pos = 0; }
    out[i] = st[p->pos++];
  }
}

/* ================================================================ STROBE-128 / Merlin */
#define STROBE_R 166
typedef struct { uint64_t s[25]; uint8_t pos, pos_begin, cur_flags; } strobe_t;
static void st_runf(strobe_t* t) {
  uint8_t* b = (uint8_t*)t->s;
  b[t->pos] ^= t->pos_begin;
  b[t->pos + 1] ^= 0x04;
  b[STROBE_R + 1] ^= 0x80;
  keccakf(t->s);
  t->pos = 0;
  t->pos_begin = 0;
}
static void st_absorb(strobe_t* t, const uint8_t* d, size_t n) {
  uint8_t* b = (uint8_t*)t->s;
  for (size_t i = 0; i < n; ++i) {
    b[t->pos++] ^= d[i];
    if (t->pos == STROBE_R) st_runf(t);
  }
}
static void st_squeeze(strobe_t* t, uint8_t* out, size_t n) {
  uint8_t* b = (uint8_t*)t->s;
  for (size_t i = 0; i < n; ++i) {
    out[i] = b[t->pos];
    b[t->pos++] = 0;
    if (t->pos == STROBE_R) st_runf(t);
  }
}
#define FLAG_I 1
#define FLAG_A 2
#define FLAG_C 4
#define FLAG_M 16
static void st_begin(strobe_t* t, uint8_t flags, int more) {
  if (more) return;
  uint8_t hdr[2] = {t->pos_begin, flags};
  t->pos_begin = (uint8_t)(t->pos + 1);
  t->cur_flags = flags;
  st_absorb(t, hdr, 2);
  if ((flags & FLAG_C) && t->pos != 0) st_runf(t);
}
static void st_meta_ad(strobe_t* t, const uint8_t* d, size_t n, int more) { st_begin(t, FLAG_M | FLAG_A, more); st_absorb(t, d, n); }
static void st_ad(strobe_t* t, const uint8_t* d, size_t n) { st_begin(t, FLAG_A, 0); st_absorb(t, d, n); }
static void st_prf(strobe_t* t, uint8_t* out, size_t n) { st_begin(t, FLAG_I | FLAG_A | FLAG_C, 0); st_squeeze(t, out, n); }

typedef struct { strobe_t st; } transcript_t;
static void tr_append(transcript_t* t, const char* label, const uint8_t* msg, size_t n) {
  uint32_t len = (uint32_t)n;
  st_meta_ad(&t->st, (const uint8_t*)label, strlen(label), 0);
  st_meta_ad(&t->st, (const uint8_t*)&len, 4, 1);
  st_ad(&t->st, msg, n);
}
static void tr_init(transcript_t* t, const uint8_t* label, size_t llen) {
  memset(t, 0, sizeof *t);
  uint8_t* b = (uint8_t*)t->st.s;
  const uint8_t hdr[6] = {1, STROBE_R + 2, 1, 0, 1, 96};
  memcpy(b, hdr, 6);
  memcpy(b + 6, "STROBEv1.0.2", 12);
  keccakf(t->st.s);
  st_meta_ad(&t->st, (const uint8_t*)"Merlin v1.0", 11, 0);
  tr_append(t, "dom-sep", label, llen);
}
static void tr_u64(transcript_t* t, const char* label, uint64_t x) { tr_append(t, label, (const uint8_t*)&x, 8); }
static void tr_challenge(transcript_t* t, const char* label, uint8_t* out, size_t n) {
  uint32_t len = (uint32_t)n;
  st_meta_ad(&t->st, (const uint8_t*)label, strlen(label), 0);
  st_meta_ad(&t->st, (const uint8_t*)&len, 4, 1);
  st_prf(&t->st, out, n);
}
static sc_t tr_scalar(transcript_t* t, const char* label) {
  uint8_t w[64];
  tr_challenge(t, label, w, 64);
  return sc_from_wide(w);
}
static void tr_sc(transcript_t* t, const char* label, sc_t s) { tr_append(t, label, (const uint8_t*)s.v, 32); }

/* ================================================================ MSM helpers */
/* dalek vartime dispatch over decoded points; scalars as sc_t (== bytes) */
static ge_ext msm(const sc_t* s, const ge_ext* P, size_t n) {
  return n < 190 ? straus_vartime((const uint8_t*)s, P, n) : pippenger_vartime((const uint8_t*)s, P, n);
}

/* ================================================================ generators */
typedef struct {
  uint32_t n_p;
  ge_ext *G, *H, B, Bb;
} gens_t;
static void gens_chain(const char* label, uint32_t n, ge_ext* out) {
  sponge_t x;
  sp_init(&x, 136, 0x1F);
  sp_absorb(&x, (const uint8_t*)"GeneratorsChain", 15);
  uint8_t lab[5] = {(uint8_t)label[0], 0, 0, 0, 0};
  sp_absorb(&x, lab, 5);
  uint8_t u[64];
  for (uint32_t i = 0; i < n; ++i) {
    sp_squeeze(&x, u, 64);
    out[i] = from_uniform(u);
  }
}
static const uint8_t B_ENC[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9,
                                  0x61, 0xc5, 0x00, 0x51, 0x5f, 0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82,
                                  0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
static void gens_make(gens_t* g, uint32_t n_p) {
  init_consts();
  g->n_p = n_p;
  g->G = (ge_ext*)malloc(sizeof(ge_ext) * n_p);
  g->H = (ge_ext*)malloc(sizeof(ge_ext) * n_p);
  gens_chain("G", n_p, g->G);
  gens_chain("H", n_p, g->H);
  ristretto_decode(&g->B, B_ENC);
  sponge_t h;
  sp_init(&h, 72, 0x06);
  sp_absorb(&h, B_ENC, 32);
  uint8_t d[64];
  sp_squeeze(&h, d, 64);
  g->Bb = from_uniform(d);
}

/* ================================================================ circuit */
typedef struct { uint32_t q, col; sc_t val; } entry_t;
typedef struct {
  uint32_t k, n, n_p, lg, Q, m;
  entry_t *WL, *WR, *WO, *WV;
  size_t nWL, nWR, nWO, nWV;
  sc_t* c;
} circuit_t;
static void ent(entry_t* W, size_t* nw, uint32_t q, uint32_t col, sc_t v) { W[(*nw)++] = (entry_t){q, col, v}; }
static void circuit_make(circuit_t* C, uint32_t k) {
  const sc_t one = SC_ONE, neg1 = sc_neg(SC_ONE);
  C->k = k; C->n = 2 * k; C->n_p = 1; C->lg = 0;
  while (C->n_p < C->n) { C->n_p *= 2; C->lg++; }
  C->Q = 4 * k + 2; C->m = 2 * k + 1;
  const uint32_t n = C->n, X = 2 * k;
  C->WL = calloc(2 * n + 4, sizeof(entry_t)); C->WR = calloc(2 * n + 4, sizeof(entry_t));
  C->WO = calloc(2 * n + 4, sizeof(entry_t)); C->WV = calloc(4 * n + 8, sizeof(entry_t));
  C->nWL = C->nWR = C->nWO = C->nWV = 0;
  C->c = calloc(C->Q, sizeof(sc_t));
  for (uint32_t g = 0; g < n; ++g) {
    ent(C->WL, &C->nWL, g, g, one);
    if (g == 0) { ent(C->WV, &C->nWV, g, 0, one); ent(C->WV, &C->nWV, g, X, neg1); }
    else if (g == k - 1) { ent(C->WV, &C->nWV, g, k, one); ent(C->WV, &C->nWV, g, X, neg1); }
    else if (g == 2 * k - 1) { ent(C->WO, &C->nWO, g, k - 2, neg1); ent(C->WO, &C->nWO, g, 2 * k - 2, neg1); }
    else ent(C->WO, &C->nWO, g, g - 1, neg1);
  }
  for (uint32_t g = 0; g < n; ++g) {
    const uint32_t q = n + g;
    ent(C->WR, &C->nWR, q, g, one);
    if (g + 2 <= k) { ent(C->WV, &C->nWV, q, g + 1, one); ent(C->WV, &C->nWV, q, X, neg1); }
    else if (g + 3 <= 2 * k) { ent(C->WV, &C->nWV, q, g + 2, one); ent(C->WV, &C->nWV, q, X, neg1); }
    else if (g == 2 * k - 2) C->c[q] = neg1;
    else C->c[q] = one;
  }
  ent(C->WO, &C->nWO, 4 * k, 2 * k - 1, one);
  ent(C->WV, &C->nWV, 4 * k + 1, X, one);
}
static void zW(const entry_t* W, size_t nw, const sc_t* zq, uint32_t ncols, sc_t* out) {
  for (uint32_t i = 0; i < ncols; ++i) out[i] = SC_ZERO;
  for (size_t i = 0; i < nw; ++i) out[W[i].col] = sc_add(out[W[i].col], sc_mul(zq[W[i].q], W[i].val));
}

/* ================================================================ RNG */
typedef struct { sponge_t x; } rng_t;
static void rng_init(rng_t* r, uint64_t seed) {
  sp_init(&r->x, 136, 0x1F);
  sp_absorb(&r->x, (const uint8_t*)"bpperm-prove", 12);
  sp_absorb(&r->x, (const uint8_t*)&seed, 8);
}
static uint64_t rng_u64(rng_t* r) { uint64_t v; sp_squeeze(&r->x, (uint8_t*)&v, 8); return v; }
/* blinding scalar j: from_wide(SHAKE256("bpperm-prove-sc" || seed || le32 j)[0..64])
 * (oracle/merlin.py indexed_scalar) */
static sc_t draw_sc(uint64_t seed, uint32_t j) {
  sponge_t x;
  uint8_t b[64], jb[4] = {(uint8_t)j, (uint8_t)(j >> 8), (uint8_t)(j >> 16), (uint8_t)(j >> 24)};
  sp_init(&x, 136, 0x1F);
  sp_absorb(&x, (const uint8_t*)"bpperm-prove-sc", 15);
  sp_absorb(&x, (const uint8_t*)&seed, 8);
  sp_absorb(&x, jb, 4);
  sp_squeeze(&x, b, 64);
  return sc_from_wide(b);
}

static void enc_pt(uint8_t out[32], const ge_ext* p) { ristretto_encode(out, p); }

/* ================================================================ IPA */
/* bulletproofs 4.0.0 InnerProductProof::create, folding form, G_factors = 1,
 * H_factors = hf applied in the first round (App. B2).  a, b (n entries) are
 * folded in place; writes L_0 R_0 ... L_{lg-1} R_{lg-1} a b (32 B each) to lr. */
static void ipa_create(transcript_t* tr, const ge_ext* Qp, const ge_ext* G0, const ge_ext* H0, sc_t* a, sc_t* b,
                       const sc_t* hf, uint32_t n_p, uint8_t* lr) {
  const ge_ext Q = *Qp;
  uint32_t nn = n_p;
  ge_ext* Gv = malloc(sizeof(ge_ext) * n_p);
  ge_ext* Hv = malloc(sizeof(ge_ext) * n_p);
  memcpy(Gv, G0, sizeof(ge_ext) * n_p);
  memcpy(Hv, H0, sizeof(ge_ext) * n_p);
  sc_t* sv = malloc(sizeof(sc_t) * (n_p + 1));
  ge_ext* pv = malloc(sizeof(ge_ext) * (n_p + 1));
  tr_append(tr, "dom-sep", (const uint8_t*)"ipp v1", 6);
  tr_u64(tr, "n", n_p);
  int first = 1;
  while (nn != 1) {
    nn /= 2;
    const sc_t cL = sc_inner(a, b + nn, nn), cR = sc_inner(a + nn, b, nn);
    /* L = <a_lo, G_hi> + <b_hi * hf_lo, H_lo> + c_L Q */
    for (uint32_t i = 0; i < nn; ++i) {
      sv[i] = a[i];
      pv[i] = Gv[nn + i];
      sv[nn + i] = first ? sc_mul(b[nn + i], hf[i]) : b[nn + i];
      pv[nn + i] = Hv[i];
    }
    sv[2 * nn] = cL;
    pv[2 * nn] = Q;
    ge_ext Lp = msm(sv, pv, 2 * nn + 1);
    for (uint32_t i = 0; i < nn; ++i) {
      sv[i] = a[nn + i];
      pv[i] = Gv[i];
      sv[nn + i] = first ? sc_mul(b[i], hf[nn + i]) : b[i];
      pv[nn + i] = Hv[nn + i];
    }
    sv[2 * nn] = cR;
    ge_ext Rp = msm(sv, pv, 2 * nn + 1);
    enc_pt(lr, &Lp);
    enc_pt(lr + 32, &Rp);
    tr_append(tr, "L", lr, 32);
    tr_append(tr, "R", lr + 32, 32);
    lr += 64;
    const sc_t u = tr_scalar(tr, "u"), ui = sc_inv(u);
    for (uint32_t i = 0; i < nn; ++i) {
      a[i] = sc_add(sc_mul(a[i], u), sc_mul(ui, a[nn + i]));
      b[i] = sc_add(sc_mul(b[i], ui), sc_mul(u, b[nn + i]));
      /* G'_i = u^-1 G_lo + u G_hi ; H'_i = u hf_lo H_lo + u^-1 hf_hi H_hi */
      sc_t s2[2] = {ui, u};
      ge_ext p2[2] = {Gv[i], Gv[nn + i]};
      Gv[i] = msm(s2, p2, 2);
      sc_t h2[2] = {first ? sc_mul(u, hf[i]) : u, first ? sc_mul(ui, hf[nn + i]) : ui};
      ge_ext q2[2] = {Hv[i], Hv[nn + i]};
      Hv[i] = msm(h2, q2, 2);
    }
    first = 0;
  }
  memcpy(lr, a[0].v, 32);
  memcpy(lr + 32, b[0].v, 32);
  free(Gv); free(Hv); free(sv); free(pv);
}

/* ================================================================ prover */
static ge_ext commit2(const gens_t* g, sc_t v, sc_t gam) {
  sc_t s[2] = {v, gam};
  ge_ext P[2] = {g->B, g->Bb};
  return msm(s, P, 2);
}

/* proof layout (perm_api.hip serialize): A_I A_O S T1 T3 T4 T5 T6 | tau_x mu
 * t_hat | L_j R_j ... | a b; V: m encodings */
static int prove(const gens_t* G, const circuit_t* C, uint64_t seed, const uint8_t* label, size_t llen,
                 uint8_t* proof, uint8_t* Vout) {
  const uint32_t k = C->k, n_p = C->n_p, m = C->m, n = C->n;
  rng_t rng;
  rng_init(&rng, seed);
  uint32_t* pi = malloc(4 * k);
  for (uint32_t i = 0; i < k; ++i) pi[i] = i;
  for (uint32_t i = k - 1; i > 0; --i) {
    uint32_t j = (uint32_t)(rng_u64(&rng) % (uint64_t)(i + 1));
    uint32_t t = pi[i]; pi[i] = pi[j]; pi[j] = t;
  }
  /* blinding scalars by index: gamma[m], alpha, beta, rho, s_L[n_p], s_R[n_p], tau[5] */
  sc_t* gamma = malloc(sizeof(sc_t) * m);
  for (uint32_t i = 0; i < m; ++i) gamma[i] = draw_sc(seed, i);
  sc_t alpha = draw_sc(seed, m), beta = draw_sc(seed, m + 1), rho = draw_sc(seed, m + 2);
  sc_t* buf = calloc((size_t)n_p * 24 + 4 * C->Q + 64, sizeof(sc_t));
  sc_t *sL = buf, *sR = sL + n_p, *aL = sR + n_p, *aR = aL + n_p, *aO = aR + n_p, *y_n = aO + n_p,
       *y_inv = y_n + n_p, *zWL = y_inv + n_p, *zWR = zWL + n_p, *zWO = zWR + n_p, *l1 = zWO + n_p, *r0 = l1 + n_p,
       *r1 = r0 + n_p, *r3 = r1 + n_p, *l = r3 + n_p, *r = l + n_p, *zq = r + n_p, *zWV = zq + C->Q + 1;
  for (uint32_t i = 0; i < n_p; ++i) sL[i] = draw_sc(seed, m + 3 + i);
  for (uint32_t i = 0; i < n_p; ++i) sR[i] = draw_sc(seed, m + 3 + n_p + i);
  sc_t taus[5];
  for (int i = 0; i < 5; ++i) taus[i] = draw_sc(seed, m + 3 + 2 * n_p + (uint32_t)i);

  transcript_t tr;
  tr_init(&tr, label, llen);
  tr_append(&tr, "dom-sep", (const uint8_t*)"acp v1", 6);
  tr_u64(&tr, "n", n_p);
  for (uint32_t j = 0; j < 2 * k; ++j) {
    const sc_t v = sc_u64(j < k ? j + 1 : pi[j - k] + 1);
    ge_ext P = commit2(G, v, gamma[j]);
    enc_pt(Vout + 32 * j, &P);
    tr_append(&tr, "V", Vout + 32 * j, 32);
  }
  const sc_t x_perm = tr_scalar(&tr, "x_perm");
  {
    ge_ext P = commit2(G, x_perm, gamma[2 * k]);
    enc_pt(Vout + 32 * 2 * k, &P);
    tr_append(&tr, "V", Vout + 32 * 2 * k, 32);
  }
  /* witness (oracle perm_witness) */
  {
    sc_t* v = malloc(sizeof(sc_t) * m);
    for (uint32_t i = 0; i < k; ++i) { v[i] = sc_u64(i + 1); v[k + i] = sc_u64(pi[i] + 1); }
    v[2 * k] = x_perm;
    for (uint32_t g = 0; g + 1 < k; ++g) {
      aL[g] = g == 0 ? sc_sub(v[0], x_perm) : aO[g - 1];
      aR[g] = sc_sub(v[g + 1], x_perm);
      aO[g] = sc_mul(aL[g], aR[g]);
    }
    for (uint32_t g = k - 1; g < 2 * k - 2; ++g) {
      aL[g] = g == k - 1 ? sc_sub(v[k], x_perm) : aO[g - 1];
      aR[g] = sc_sub(v[g + 2], x_perm);
      aO[g] = sc_mul(aL[g], aR[g]);
    }
    uint32_t g = 2 * k - 2;
    aL[g] = aO[2 * k - 3]; aR[g] = sc_neg(SC_ONE); aO[g] = sc_mul(aL[g], aR[g]);
    g = 2 * k - 1;
    aL[g] = sc_add(aO[k - 2], aO[2 * k - 2]); aR[g] = SC_ONE; aO[g] = sc_mul(aL[g], aR[g]);
    free(v);
  }
  (void)n;
  /* A_I, A_O, S */
  uint8_t* out = proof;
  {
    const size_t T = 1 + 2 * (size_t)n_p;
    sc_t* s = malloc(sizeof(sc_t) * T);
    ge_ext* P = malloc(sizeof(ge_ext) * T);
    P[0] = G->Bb;
    for (uint32_t i = 0; i < n_p; ++i) { P[1 + i] = G->G[i]; P[1 + n_p + i] = G->H[i]; }
    s[0] = alpha;
    for (uint32_t i = 0; i < n_p; ++i) { s[1 + i] = aL[i]; s[1 + n_p + i] = aR[i]; }
    ge_ext A = msm(s, P, T);
    enc_pt(out, &A);
    s[0] = beta;
    for (uint32_t i = 0; i < n_p; ++i) s[1 + i] = aO[i];
    A = msm(s, P, 1 + n_p);
    enc_pt(out + 32, &A);
    s[0] = rho;
    for (uint32_t i = 0; i < n_p; ++i) { s[1 + i] = sL[i]; s[1 + n_p + i] = sR[i]; }
    A = msm(s, P, T);
    enc_pt(out + 64, &A);
    free(s);
    free(P);
  }
  tr_append(&tr, "A_I", out, 32);
  tr_append(&tr, "A_O", out + 32, 32);
  tr_append(&tr, "S", out + 64, 32);
  const sc_t y = tr_scalar(&tr, "y"), z = tr_scalar(&tr, "z");
  sc_powers(y, y_n, n_p);
  sc_powers(sc_inv(y), y_inv, n_p);
  sc_powers(z, zq, C->Q + 1);
  zW(C->WL, C->nWL, zq + 1, n_p, zWL);
  zW(C->WR, C->nWR, zq + 1, n_p, zWR);
  zW(C->WO, C->nWO, zq + 1, n_p, zWO);
  zW(C->WV, C->nWV, zq + 1, m, zWV);
  for (uint32_t i = 0; i < n_p; ++i) {
    l1[i] = sc_add(aL[i], sc_mul(y_inv[i], zWR[i]));
    r0[i] = sc_sub(zWO[i], y_n[i]);
    r1[i] = sc_add(sc_mul(y_n[i], aR[i]), zWL[i]);
    r3[i] = sc_mul(y_n[i], sR[i]);
  }
  sc_t t[7];
  t[1] = sc_inner(l1, r0, n_p);
  t[2] = sc_add(sc_inner(l1, r1, n_p), sc_inner(aO, r0, n_p));
  t[3] = sc_add(sc_inner(aO, r1, n_p), sc_inner(sL, r0, n_p));
  t[4] = sc_add(sc_inner(l1, r3, n_p), sc_inner(sL, r1, n_p));
  t[5] = sc_inner(aO, r3, n_p);
  t[6] = sc_inner(sL, r3, n_p);
  static const char* TL[5] = {"T1", "T3", "T4", "T5", "T6"};
  static const int TI[5] = {1, 3, 4, 5, 6};
  for (int i = 0; i < 5; ++i) {
    ge_ext P = commit2(G, t[TI[i]], taus[i]);
    enc_pt(out + 96 + 32 * i, &P);
    tr_append(&tr, TL[i], out + 96 + 32 * i, 32);
  }
  const sc_t x = tr_scalar(&tr, "x");
  sc_t xp[7];
  sc_powers(x, xp, 7);
  sc_t tau_x = sc_mul(xp[2], sc_inner(zWV, gamma, m));
  for (int i = 0; i < 5; ++i) tau_x = sc_add(tau_x, sc_mul(taus[i], xp[TI[i]]));
  const sc_t mu = sc_add(sc_add(sc_mul(alpha, x), sc_mul(beta, xp[2])), sc_mul(rho, xp[3]));
  for (uint32_t i = 0; i < n_p; ++i) {
    l[i] = sc_mul(x, sc_add(l1[i], sc_mul(x, sc_add(aO[i], sc_mul(x, sL[i])))));
    r[i] = sc_add(r0[i], sc_mul(x, sc_add(r1[i], sc_mul(xp[2], r3[i]))));
  }
  const sc_t t_hat = sc_inner(l, r, n_p);
  tr_sc(&tr, "TX", tau_x);
  tr_sc(&tr, "mu", mu);
  tr_sc(&tr, "t", t_hat);
  memcpy(out + 256, tau_x.v, 32);
  memcpy(out + 288, mu.v, 32);
  memcpy(out + 320, t_hat.v, 32);
  const sc_t w = tr_scalar(&tr, "w");
  /* IPA, folding form (bulletproofs 4.0.0 InnerProductProof::create):
   * Q = w * B; G_factors = 1, H_factors = y^-i applied in the first round */
  {
    sc_t wq[1] = {w};
    ge_ext Bp[1] = {G->B};
    const ge_ext Q = msm(wq, Bp, 1);
    ipa_create(&tr, &Q, G->G, G->H, l, r, y_inv, n_p, out + 352);
  }
  free(pi); free(gamma); free(buf);
  return 0;
}

/* ================================================================ exported */
static gens_t g_gens;
static circuit_t g_circ;
static uint32_t g_k = 0;

/* one-time setup for k cards (not thread-safe; call before threads) */
int cpu_perm_setup(uint32_t k) {
  if (k < 2) return -1;
  if (g_k == k) return 0;
  circuit_make(&g_circ, k);
  gens_make(&g_gens, g_circ.n_p);
  g_k = k;
  return 0;
}
size_t cpu_perm_proof_len(uint32_t k) {
  uint32_t n_p = 1, lg = 0;
  while (n_p < 2 * k) { n_p *= 2; lg++; }
  return 32 * (8 + 3 + 2 * lg + 2);
}
int cpu_perm_prove(uint32_t k, uint64_t seed, const uint8_t* label, size_t llen, uint8_t* proof, uint8_t* V) {
  if (g_k != k) return -1;
  return prove(&g_gens, &g_circ, seed, label, llen, proof, V);
}
/* count proofs from seed0, timed (setup excluded); returns seconds */
double cpu_perm_time(uint32_t k, uint64_t seed0, int count, const uint8_t* label, size_t llen) {
  if (g_k != k) return -1.0;
  const size_t pl = cpu_perm_proof_len(k);
  uint8_t* proof = malloc(pl);
  uint8_t* V = malloc(32 * (2 * k + 1));
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int i = 0; i < count; ++i) prove(&g_gens, &g_circ, seed0 + (uint64_t)i, label, llen, proof, V);
  clock_gettime(CLOCK_MONOTONIC, &b);
  free(proof);
  free(V);
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

/* Config 2: A = alpha B~ + <aL, G> + <aR, H> over GeneratorsChain(n),
 * transcript `label` absorbs A ("A"), y = challenge "y", then the IPA on
 * (aL, aR) with G_factors = 1, H_factors = y^-i and Q = from_uniform(q64)
 * (tests/golden/make_golden.py config2_golden; bench.py bench_config2).
 * sc: aL[n] || aR[n] || alpha, 32 B each.  out: A || L/R pairs || a || b. */
static gens_t g_c2;
static uint32_t g_c2_n = 0;
int cpu_config2_setup(uint32_t n) {
  if (n < 2 || (n & (n - 1))) return -1;
  if (g_c2_n == n) return 0;
  gens_make(&g_c2, n);
  g_c2_n = n;
  return 0;
}
int cpu_config2(uint32_t n, const uint8_t* sc, const uint8_t q64[64], const uint8_t* label, size_t llen,
                uint8_t* out) {
  if (g_c2_n != n) return -1;
  const size_t T = 2 * (size_t)n + 1;
  sc_t* s = malloc(sizeof(sc_t) * (T + 2 * (size_t)n));
  ge_ext* P = malloc(sizeof(ge_ext) * T);
  s[0] = *(const sc_t*)(sc + 64 * (size_t)n);  /* alpha */
  P[0] = g_c2.Bb;
  for (uint32_t i = 0; i < n; ++i) {
    memcpy(&s[1 + i], sc + 32 * (size_t)i, 32);
    memcpy(&s[1 + n + i], sc + 32 * ((size_t)n + i), 32);
    P[1 + i] = g_c2.G[i];
    P[1 + n + i] = g_c2.H[i];
  }
  ge_ext A = msm(s, P, T);
  enc_pt(out, &A);
  transcript_t tr;
  tr_init(&tr, label, llen);
  tr_append(&tr, "A", out, 32);
  const sc_t y = tr_scalar(&tr, "y");
  sc_t* a = s + T;
  sc_t* b = a + n;
  sc_t* hf = malloc(sizeof(sc_t) * n);
  sc_powers(sc_inv(y), hf, n);
  for (uint32_t i = 0; i < n; ++i) { a[i] = s[1 + i]; b[i] = s[1 + n + i]; }
  const ge_ext Q = from_uniform(q64);
  ipa_create(&tr, &Q, g_c2.G, g_c2.H, a, b, hf, n, out + 32);
  free(s); free(P); free(hf);
  return 0;
}
/* count config-2 runs on the same inputs; returns seconds */
double cpu_config2_time(uint32_t n, const uint8_t* sc, const uint8_t q64[64], const uint8_t* label, size_t llen,
                        int count) {
  if (g_c2_n != n) return -1.0;
  uint32_t lg = 0;
  while ((1u << lg) < n) ++lg;
  uint8_t* out = malloc(32 * (1 + 2 * (size_t)lg + 2));
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int i = 0; i < count; ++i) cpu_config2(n, sc, q64, label, llen, out);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(out);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
