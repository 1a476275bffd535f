/*
 * bpperm.h — C ABI of the MI355X-native Bulletproof permutation hot path.
 *
 * Drop-in boundary for the three operations the reference
 * (ercembu/bulletproof-perm, Rust crate `bp-perm`) delegates to
 * curve25519-dalek-ng 4.1.1 / bulletproofs 4.0.0 / merlin 3.0.0:
 *
 *   Ristretto MSM      `VartimeMultiscalarMul::vartime_multiscalar_mul`
 *                      bp-perm/src/circuit_lib.rs:187,202,216,363,374,385,396,
 *                      407,498,504,509,525,535,552,568
 *   Pedersen commit    `PedersenGens::commit` weights.rs:58-61,
 *                      vector commitments A_I / A_O / S circuit_lib.rs:187-229
 *   point codec        `RistrettoPoint::compress` circuit_lib.rs:231-233,
 *                      `CompressedRistretto::decompress` circuit_lib.rs:532
 *   inner-product arg  `InnerProductProof::{create,verify}` (bulletproofs
 *                      4.0.0; hook fields ACEssentials.G_factors/H_factors,
 *                      circuit_lib.rs:62-63)
 *   transcript         merlin `Transcript` + TranscriptProtocol,
 *                      transcript_protocol.rs:26-67
 *   AC proof           `ACProof::ArithmeticCircuitProof`, circuit_lib.rs:139-585
 *
 * Conventions (inherited from the reference):
 *   - every function returns an int status (BPP_OK = 0); nothing unwinds;
 *   - scalars are 32-byte little-endian canonical integers mod l
 *     (dalek `Scalar::as_bytes`); points are 32-byte compressed ristretto255
 *     (dalek `CompressedRistretto`);
 *   - buffers are caller-owned; the library keeps no pointer after a call
 *     returns, except to the opaque objects it creates;
 *   - a context is bound to one GPU and one HIP stream; calls on one context
 *     must not overlap (the reference is single-threaded, `&mut Transcript`).
 *   - length mismatches are BPP_ERR_LEN where dalek panics (size-hint
 *     asserts); an undecodable point is BPP_ERR_DECOMPRESS where the
 *     reference `unwrap()`s (circuit_lib.rs:532); a failed check is
 *     BPP_ERR_VERIFY where the reference returns
 *     `ProofError::VerificationError` (circuit_lib.rs:519,543).
 */
#ifndef BPPERM_H
#define BPPERM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Return codes.  No C++ exception leaves the library: a host allocation that
 * cannot be met returns BPP_ERR_NOMEM, any other internal exception
 * BPP_ERR_DEVICE (text in bpp_ctx_last_error when the call has a context). */
enum {
  BPP_OK = 0,
  BPP_ERR_ARG = 1,
  BPP_ERR_LEN = 2,
  BPP_ERR_DECOMPRESS = 3,
  BPP_ERR_NONCANONICAL = 4,
  BPP_ERR_DEVICE = 5,
  BPP_ERR_VERIFY = 6,
  BPP_ERR_NOMEM = 7,
  BPP_ERR_CALLBACK = 8, /* a caller's transcript hook returned nonzero */
};

typedef struct bpp_ctx bpp_ctx;
typedef struct bpp_points bpp_points;

/* ------------------------------------------------------------- context */
int bpp_ctx_create(int device, bpp_ctx** out);
void bpp_ctx_destroy(bpp_ctx* ctx);
/* Last error text for this context ("" if none). */
const char* bpp_ctx_last_error(const bpp_ctx* ctx);
/* The hipStream_t every kernel of this context is launched on. */
void* bpp_ctx_stream(bpp_ctx* ctx);
/* Per-kernel timing with HIP events on the context stream (0 = off). */
int bpp_ctx_profile(bpp_ctx* ctx, int enable);
/* Accumulated time (ms) and launch count of a named kernel stage
 * ("msm_accumulate", "msm_reduce", "msm_count", "msm_scatter", ...). */
int bpp_ctx_profile_get(bpp_ctx* ctx, const char* stage, double* ms, uint64_t* launches);
void bpp_ctx_profile_reset(bpp_ctx* ctx);
/* Algorithmic work issued on this context (and its child streams) since the
 * last reset, counted at launch time: "msm_terms" (scalar-point terms of every
 * MSM and Pedersen commitment), "madds" (mixed additions of a table point:
 * direct-table MSMs count every window of every term), "padds" (additions of
 * two extended points in trees and bucket reductions), "msm_launches", and
 * the direct-table kernel's own "dt_terms" / "dt_madds" / "dt_launches".  The
 * roofline of the proof path (96 B x terms) reads these. */
int bpp_ctx_work_get(bpp_ctx* ctx, const char* name, uint64_t* value);
void bpp_ctx_work_reset(bpp_ctx* ctx);

/* Opt-in host-process tuning (process-wide, so never done implicitly):
 * BPP_TUNE_MALLOC fixes glibc's mmap threshold at 64 MB, disables heap
 * trimming and pads arena growth by 64 MB, which keeps the prover's
 * per-batch host vectors in the arenas
 * (measured in a host profile of 8 batches in flight).
 * BPP_TUNE_HW_QUEUES asks HIP for 8 hardware queues per process
 * (GPU_MAX_HW_QUEUES=8 unless the caller set it): a prover keeping many
 * batches in flight, one context and stream each, needs more than HIP's
 * default 4.  HIP reads the variable once, when it starts, so this flag must
 * come before the first bpp_ctx_create and any other HIP use in the process.
 * BPP_ERR_ARG for unknown flags. */
#define BPP_TUNE_MALLOC 1u
#define BPP_TUNE_HW_QUEUES 2u
int bpp_host_tuning(uint32_t flags);
/* Threads of the library's host pool (transcripts, scalar bookkeeping),
 * calling threads included: BPP_HOST_THREADS, else a quarter of this
 * process's share of the granted CPUs (cgroup quota / LOCAL_WORLD_SIZE),
 * at most 4. */
uint32_t bpp_host_threads(void);

/* Device memory helpers, so callers can stage inputs resident in HBM. */
int bpp_dev_alloc(bpp_ctx* ctx, size_t bytes, void** dptr);
int bpp_dev_free(bpp_ctx* ctx, void* dptr);
int bpp_memcpy_htod(bpp_ctx* ctx, void* dst, const void* src, size_t bytes);
int bpp_memcpy_dtoh(bpp_ctx* ctx, void* dst, const void* src, size_t bytes);
int bpp_synchronize(bpp_ctx* ctx);

/* ------------------------------------------------ resident point tables */
/* Decompress n 32-byte encodings into a table kept in HBM.
 * BPP_ERR_DECOMPRESS if any encoding is invalid (*bad_index set when
 * bad_index != NULL).  Replaces CompressedRistretto::decompress. */
int bpp_points_decompress(bpp_ctx* ctx, const uint8_t* enc, size_t n, bpp_points** out, size_t* bad_index);
/* n points RistrettoPoint::from_uniform_bytes(64 bytes each), on the GPU. */
int bpp_points_from_uniform(bpp_ctx* ctx, const uint8_t* bytes64, size_t n, bpp_points** out);
/* Compress every point of the table (RistrettoPoint::compress). */
int bpp_points_compress(bpp_ctx* ctx, const bpp_points* pts, uint8_t* out);
size_t bpp_points_len(const bpp_points* pts);
void bpp_points_destroy(bpp_points* pts);

/* ------------------------------------------------------------------ MSM */
/* out = sum_i scalars[i] * points[i]; host scalars, host compressed points.
 * `RistrettoPoint::vartime_multiscalar_mul(scalars, points).compress()`. */
int bpp_msm(bpp_ctx* ctx, const uint8_t* scalars, const uint8_t* points, size_t n, uint8_t out[32]);
/* Same over the first n points of a resident table; host scalars. */
int bpp_msm_table(bpp_ctx* ctx, const uint8_t* scalars, const bpp_points* tbl, size_t n, uint8_t out[32]);
/* Same with the scalars already resident in HBM (n x 32 bytes at d_scalars,
 * canonical).  The throughput entry point used by bench.py. */
int bpp_msm_table_dev(bpp_ctx* ctx, const void* d_scalars, const bpp_points* tbl, size_t n, uint8_t out[32]);
/* Window-partitioned MSM for multi-GPU: computes the partial sum over
 * windows [w_begin, w_end) of the signed radix-2^c decomposition the
 * library picks for size n (bpp_msm_windows reports c and the window
 * count).  Partial results are raw extended points (128 bytes) so that
 * partials from different GPUs can be added exactly (bpp_point_add_raw). */
int bpp_msm_windows(size_t n, uint32_t* c, uint32_t* windows);
int bpp_msm_table_dev_partial(bpp_ctx* ctx, const void* d_scalars, const bpp_points* tbl, size_t n,
                              uint32_t w_begin, uint32_t w_end, uint8_t partial[128]);
/* Asynchronous single MSMs over a resident table, for a stream of
 * independent MSMs (e.g. successive batch verifications): submit enqueues
 * the whole device pipeline of one MSM (windows [w_begin, w_end); w_end = 0
 * means all windows) on its own stream and returns at once; collect waits
 * for that MSM, runs its host window combine and returns the compressed
 * result (`out`, full MSMs) and/or the raw 128-byte partial (`partial`, as
 * bpp_msm_table_dev_partial).  At most BPP_MSM_INFLIGHT MSMs may be
 * outstanding (submit fails with BPP_ERR_ARG otherwise), so the device runs
 * MSM i+1's digit sort beside MSM i's latency-bound bucket reduction while
 * the host combines MSM i-1's windows (two in flight measured best).  d_scalars must stay valid until
 * collect; each outstanding MSM needs its own scalar buffer contents.
 * Same-result guarantee: collect(submit(s)) == bpp_msm_table_dev(s). */
#define BPP_MSM_INFLIGHT 4
int bpp_msm_submit(bpp_ctx* ctx, const void* d_scalars, const bpp_points* tbl, size_t n, uint32_t w_begin,
                   uint32_t w_end, uint64_t* ticket);
int bpp_msm_collect(bpp_ctx* ctx, uint64_t ticket, uint8_t out[32], uint8_t partial[128]);
/* The same with host scalars (the shape of the reference's
 * vartime_multiscalar_mul(scalars, points), circuit_lib.rs:187): the n x 32
 * bytes are copied to the device on the MSM's own stream, so in a stream of
 * submits the upload of one MSM overlaps the others' kernels.  From pinned memory (bpp_host_alloc)
 * the copy is a direct DMA; pageable memory goes through a staging copy
 * first (host memcpy inside the call).  h_scalars must stay valid and
 * unchanged until collect. */
int bpp_msm_submit_host(bpp_ctx* ctx, const void* h_scalars, const bpp_points* tbl, size_t n, uint32_t w_begin,
                        uint32_t w_end, uint64_t* ticket);
/* Pinned (page-locked) host memory for bpp_msm_submit_host and
 * bpp_perm_verify_* inputs: the library recognises these buffers (a range
 * inside one goes up by direct DMA) from its own registry; other host memory
 * is looked up in the HIP runtime (memory the caller pinned itself also goes
 * by DMA) and otherwise staged as pageable. */
int bpp_host_alloc(bpp_ctx* ctx, size_t bytes, void** hptr);
int bpp_host_free(bpp_ctx* ctx, void* hptr);
/* Sum raw extended partial points (count x 128 bytes) and compress.
 * BPP_ERR_ARG for a partial whose Z coordinate is zero (not a point: e.g. an
 * all-zero buffer a failed rank never wrote). */
int bpp_partials_finish(const uint8_t* partials, size_t count, uint8_t out[32]);
/* Host batch encoding of doubled points: out[i] = compress(2 * P_i) for raw
 * extended points P_i (count x 128 bytes), one field inversion per call
 * instead of one inverse square root per point (the prover computes C / 2
 * from halved scalars and encodes C this way).  Replaces the per-point
 * RistrettoPoint::compress of the reference's commitments and IPA L/R
 * (circuit_lib.rs:231-233) where batches are small; host-only. */
int bpp_points_double_compress(const uint8_t* raw, size_t count, uint8_t* out);
/* count independent MSMs; MSM j covers terms [offsets[j], offsets[j+1]) of
 * `scalars` (32 bytes each) and `point_idx` (indices into tbl). */
int bpp_msm_batch(bpp_ctx* ctx, size_t count, const uint64_t* offsets, const uint8_t* scalars,
                  const uint32_t* point_idx, const bpp_points* tbl, uint8_t* out);

/* ----------------------------------------------------------- generators */
typedef struct bpp_gens bpp_gens;
/* BulletproofGens::new(n, 1) (G, H from the SHAKE256 GeneratorsChain) plus
 * PedersenGens::default() (B, B_blinding), generated on the GPU and kept
 * resident with fixed-base tables for B and B_blinding.
 * Reference: lib.rs:163 (BulletproofGens::new), weights.rs:58 (PedersenGens). */
int bpp_gens_create(bpp_ctx* ctx, size_t n, bpp_gens** out);
/* Explicit generators (the reference's test draws random G, H and a random
 * PedersenGens, lib.rs:164-180).  G_enc, H_enc: n x 32 bytes. */
int bpp_gens_from_points(bpp_ctx* ctx, const uint8_t* G_enc, const uint8_t* H_enc, size_t n,
                         const uint8_t B_enc[32], const uint8_t Bb_enc[32], bpp_gens** out);
size_t bpp_gens_len(const bpp_gens* g);
/* Compressed G[0..n), H[0..n), B, B_blinding: (2n + 2) x 32 bytes. */
int bpp_gens_export(bpp_ctx* ctx, const bpp_gens* g, uint8_t* out);
void bpp_gens_destroy(bpp_gens* g);

/* ------------------------------------------------- Pedersen commitments */
/* V_j = v_j * B + gamma_j * B_blinding for j < m (PedersenGens::commit,
 * weights.rs:58-61), fixed-base on the GPU. */
int bpp_pedersen_commit_batch(bpp_ctx* ctx, const bpp_gens* g, const uint8_t* v, const uint8_t* gamma, size_t m,
                              uint8_t* out);
/* blind * B_blinding + <a, G[0..n)> (+ <b, H[0..n)> when b != NULL):
 * A_I / A_O / S of circuit_lib.rs:187-229. */
int bpp_vec_commit(bpp_ctx* ctx, const bpp_gens* g, const uint8_t blind[32], const uint8_t* a, const uint8_t* b,
                   size_t n, uint8_t out[32]);

/* ------------------------------------------------------ Merlin transcript */
typedef struct bpp_transcript bpp_transcript;
/* merlin 3.0.0 Transcript::new(label); byte-exact (transcript_protocol.rs). */
bpp_transcript* bpp_transcript_new(const uint8_t* label, size_t len);
bpp_transcript* bpp_transcript_clone(const bpp_transcript* t);
void bpp_transcript_destroy(bpp_transcript* t);
int bpp_transcript_append_message(bpp_transcript* t, const uint8_t* label, size_t llen, const uint8_t* msg,
                                  size_t mlen);
int bpp_transcript_append_u64(bpp_transcript* t, const uint8_t* label, size_t llen, uint64_t x);
int bpp_transcript_challenge_bytes(bpp_transcript* t, const uint8_t* label, size_t llen, uint8_t* out, size_t n);
/* challenge_scalar: 64 challenge bytes -> Scalar::from_bytes_mod_order_wide
 * (transcript_protocol.rs:62-67). */
int bpp_transcript_challenge_scalar(bpp_transcript* t, const uint8_t* label, size_t llen, uint8_t out[32]);

/* ------------------------------------------------- scalar helpers (host) */
/* The caller-side scalar algebra the IPA's factors need: Scalar::invert
 * (circuit_lib.rs:274; BPP_ERR_ARG for zero) and x^0 .. x^(n-1) (util.rs:
 * 138-157 exp_iter; e.g. H_factors = powers of y^-1).  Canonical 32-byte
 * scalars in and out (BPP_ERR_NONCANONICAL otherwise). */
int bpp_scalar_invert(const uint8_t x[32], uint8_t out[32]);
int bpp_scalar_powers(const uint8_t x[32], size_t n, uint8_t* out);

/* ------------------------------------------------ inner-product argument */
/* bulletproofs 4.0.0 InnerProductProof::create over G[0..n), H[0..n) of g
 * (n a power of two, n <= bpp_gens_len): L_out, R_out receive log2(n)
 * compressed points each; G_factors / H_factors may be NULL (all ones).
 * Q may be any point: it is written into g's spare generator slot for the
 * call (BPP_ERR_DECOMPRESS if it does not decode), so concurrent
 * bpp_ipa_prove calls on one g (from several contexts) run one at a time.
 * On that path the kernels read a, b and the factors in place from ctx's
 * pinned host buffers (copied in at the call; the copies of a and b are
 * zeroed before it returns, on error paths too); the folded a, b stay in
 * ctx's device workspaces (the entropy prover's wipe zeroes them). */
int bpp_ipa_prove(bpp_ctx* ctx, const bpp_gens* g, bpp_transcript* tr, const uint8_t Q[32], const uint8_t* G_factors,
                  const uint8_t* H_factors, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* L_out,
                  uint8_t* R_out, uint8_t a_out[32], uint8_t b_out[32]);
/* InnerProductProof::verify: BPP_OK or BPP_ERR_VERIFY.  One GPU MSM of
 * 2n + 2log2(n) + 2 terms checked against the identity. */
int bpp_ipa_verify(bpp_ctx* ctx, const bpp_gens* g, bpp_transcript* tr, size_t n, const uint8_t* G_factors,
                   const uint8_t* H_factors, const uint8_t P[32], const uint8_t Q[32], const uint8_t* L,
                   const uint8_t* R, const uint8_t a[32], const uint8_t b[32]);

/* The same two calls over the CALLER's transcript (north_star: the bp-perm
 * crate keeps its merlin::Transcript; bulletproofs'
 * InnerProductProof::create(transcript: &mut Transcript, ..) and verify).
 * The library never owns the transcript: it calls back, on the calling
 * thread and in this order, exactly where bulletproofs 4.0.0 touches it
 * (transcript_protocol.rs:26-67):
 *   append_message("dom-sep", "ipp v1"), append_message("n", le64(n))
 *                                  -- innerproduct_domain_sep(n)
 *   per round j < log2(n):
 *     append_message("L", L_j), append_message("R", R_j)
 *                                  -- append_point / validate_and_append_point
 *     challenge_bytes("u", 64 B)   -- challenge_scalar("u"): the library
 *                                     reduces the 64 bytes mod l (from_bytes_mod_order_wide)
 * Labels are exactly those byte strings (no NUL counted in llen).  The
 * verifier refuses an identity L_j / R_j (BPP_ERR_VERIFY) before appending
 * it, as validate_and_append_point does.  A hook returning nonzero aborts
 * the call with BPP_ERR_CALLBACK (the transcript is then in an unspecified
 * state).  bpp_ipa_prove / bpp_ipa_verify are these with the library's own
 * Merlin (bpp_transcript) behind the hooks. */
typedef struct bpp_transcript_hooks {
  void* user;
  int (*append_message)(void* user, const uint8_t* label, size_t llen, const uint8_t* msg, size_t mlen);
  int (*challenge_bytes)(void* user, const uint8_t* label, size_t llen, uint8_t* out, size_t n);
} bpp_transcript_hooks;
int bpp_ipa_prove_cb(bpp_ctx* ctx, const bpp_gens* g, const bpp_transcript_hooks* tr, const uint8_t Q[32],
                     const uint8_t* G_factors, const uint8_t* H_factors, const uint8_t* a, const uint8_t* b, size_t n,
                     uint8_t* L_out, uint8_t* R_out, uint8_t a_out[32], uint8_t b_out[32]);
int bpp_ipa_verify_cb(bpp_ctx* ctx, const bpp_gens* g, const bpp_transcript_hooks* tr, size_t n,
                      const uint8_t* G_factors, const uint8_t* H_factors, const uint8_t P[32], const uint8_t Q[32],
                      const uint8_t* L, const uint8_t* R, const uint8_t a[32], const uint8_t b[32]);

/* ------------------------------------------- permutation proof (sound) */
/* Arithmetic-circuit proof that the second half of v = [1..k, pi(1..k), x]
 * is a permutation of the first (ACProof::ArithmeticCircuitProof,
 * circuit_lib.rs:139-585 over the circuit of weights.rs:26-204), in sound
 * form (SURVEY.md §2.2 defects fixed; DESIGN.md "Protocol").  Gates are
 * padded to n_p = next_pow2(2k) <= bpp_gens_len(g).  Every entry point takes
 * 2 <= k <= 2^20 (BPP_ERR_ARG otherwise).
 *
 * Proof bytes (bpp_perm_proof_len(k)): A_I A_O S T1 T3 T4 T5 T6 | tau_x mu
 * t_hat | L_0 R_0 .. L_{lg-1} R_{lg-1} | a b.  The 2k+1 Pedersen
 * commitments V go to V_out (public inputs, 32 bytes each).  All prover
 * randomness comes from the seed, the injected stand-in for the reference's
 * thread_rng (circuit_lib.rs:175): pi from SHAKE256("bpperm-prove" || seed)
 * (Fisher-Yates, one u64 per step), blinding scalar j (order gamma[2k+1],
 * alpha, beta, rho, s_L[n_p], s_R[n_p], tau[5]) from the first 64 bytes of
 * SHAKE256("bpperm-prove-sc" || seed || le32 j), reduced mod l. */
size_t bpp_perm_proof_len(uint32_t k);
int bpp_perm_prove(bpp_ctx* ctx, const bpp_gens* g, uint32_t k, uint64_t seed, const uint8_t* label, size_t llen,
                   uint8_t* proof_out, uint8_t* V_out, uint32_t* perm_out);
int bpp_perm_prove_batch(bpp_ctx* ctx, const bpp_gens* g, uint32_t k, size_t count, const uint64_t* seeds,
                         const uint8_t* label, size_t llen, uint8_t* proofs_out, uint8_t* V_out);
/* The u64 seeds above are deterministic TEST hooks (64 bits of entropy, so
 * a guessable seed reveals the witness).  Production proofs: 32 bytes of
 * entropy per proof from the caller (seeds32, count x 32 B), or seeds32 =
 * NULL to draw them from the OS CSPRNG (getrandom), as the reference draws
 * from thread_rng (circuit_lib.rs:175, weights.rs:39,59).  The draws are
 * those above with the 32-byte seed32 in place of the 8-byte seed.
 * Secret lifetime: after the batch the library zeroes what it kept of it --
 * the device workspaces holding draws, witness, blindings and the l / r
 * vectors, the staged draw templates, pi and (k > 768) host-path witness,
 * the T-commitment inputs, and the calling thread's reused prover states and
 * permutations; with BPP_PROVE_STREAMS > 1 each sub-batch thread does the same
 * on its child context before it exits (the caller's own seeds32 buffer is
 * the caller's to wipe). */
int bpp_perm_prove_batch_entropy(bpp_ctx* ctx, const bpp_gens* g, uint32_t k, size_t count, const uint8_t* seeds32,
                                 const uint8_t* label, size_t llen, uint8_t* proofs_out, uint8_t* V_out);
/* Test hook for the secret lifetime above: the number of nonzero bytes left
 * in what the last bpp_perm_prove_batch_entropy zeroed on ctx and its child
 * contexts (device workspaces, pinned buffers and staging spans, including
 * the sub-batch contexts of BPP_PROVE_STREAMS > 1 and the host-witness
 * staging of k > 768).  Synchronises ctx. */
int bpp_debug_secret_residue(bpp_ctx* ctx, uint64_t* nonzero_bytes);
/* BPP_OK or BPP_ERR_VERIFY (ProofError::VerificationError). One GPU MSM. */
int bpp_perm_verify(bpp_ctx* ctx, const bpp_gens* g, uint32_t k, const uint8_t* label, size_t llen,
                    const uint8_t* proof, size_t proof_len, const uint8_t* V);
/* Batch verification: all proofs' checks folded into ONE MSM (generator
 * scalars merged across proofs) with random weights w_p =
 * from_wide(SHAKE256("bp-perm-batch-wt" || seed || le64 p || r_p)[0..64]):
 * seed = 32 bytes of the verifier's own randomness (getrandom), mixed with
 * each proof's transcript challenge r_p as bulletproofs' r1cs batch verifier
 * mixes its rng into a TranscriptRng.  The transcripts are replayed on the
 * GPU and the whole batch runs with no host round trip (DESIGN.md §5 "Batch
 * weights", "No inversions"). */
int bpp_perm_verify_batch(bpp_ctx* ctx, const bpp_gens* g, uint32_t k, size_t count, const uint8_t* label,
                          size_t llen, const uint8_t* proofs, const uint8_t* V);

/* Batch verification split for several GPUs (north_star: "the single large
 * verifier MSM partitions its bucket windows across GPUs"; reference verify
 * circuit_lib.rs:478-585).  Host phase, no GPU: parse `count` proofs, replay
 * their transcripts and return each proof's weight challenge r (count x 32
 * B, may be NULL).  BPP_ERR_VERIFY if a proof is malformed or its transcript
 * rejects a point encoding. */
typedef struct bpp_verify_job bpp_verify_job;
int bpp_perm_verify_begin(uint32_t k, size_t count, const uint8_t* label, size_t llen, const uint8_t* proofs,
                          const uint8_t* V, uint8_t* r_out, bpp_verify_job** out);
/* The same host interface with the replay on the GPU of ctx (one Merlin
 * transcript per 16-lane group, k_verify_replay_g): uploads the proofs and V, replays every
 * transcript, decompresses the proof points and returns r (count x 32 B, may
 * be NULL).  r is byte-identical to bpp_perm_verify_begin's.  The job keeps
 * its records and points in ctx's workspaces: it is valid for
 * bpp_perm_verify_partial on the same ctx until the next verification on
 * that ctx -- bpp_perm_verify_begin_dev, bpp_perm_verify or
 * bpp_perm_verify_batch, which all replay through the same workspaces
 * (BPP_ERR_ARG after that; a call refused for its arguments supersedes
 * nothing) -- and
 * bpp_perm_verify_scalars rejects it (BPP_ERR_ARG).  The proof points are
 * decompressed beside the replay; one that does not decode makes
 * bpp_perm_verify_partial return BPP_ERR_VERIFY. */
int bpp_perm_verify_begin_dev(bpp_ctx* ctx, uint32_t k, size_t count, const uint8_t* label, size_t llen,
                              const uint8_t* proofs, const uint8_t* V, uint8_t* r_out, bpp_verify_job** out);
/* Terms of the job's MSM: 2 n_p + 2 merged generators + count x (m + 8 +
 * 2 log2 n_p) proof points.  bpp_msm_windows(terms) gives c and W. */
int bpp_perm_verify_terms(const bpp_verify_job* job, size_t* terms);
/* 32 bytes of verifier randomness for a batch (the OS CSPRNG).  Every job,
 * slice and rank of ONE batch takes the same seed (rank 0 draws it and
 * broadcasts the 32 bytes); a seed the provers can predict voids the batch's
 * soundness. */
int bpp_verify_seed(uint8_t seed[32]);
/* The job's MSM terms (host): proof p of the job is batch proof first + p,
 * weighted by w = from_wide(SHAKE256("bp-perm-batch-wt" || seed || le64(first
 * + p) || r_p)[0..64]) (bpp_perm_verify_batch).  scalars_out: terms x 32 B
 * (G[0..n_p), H[0..n_p), B, B_blinding, then the proof points'); points_out:
 * the proof points' encodings ((terms - 2 n_p - 2) x 32 B).  Every proof's
 * check is scaled by (prod u_j)^2 y^(n_p - 1), so no inverse is formed. */
int bpp_perm_verify_scalars(const bpp_verify_job* job, const uint8_t seed[32], size_t first, uint8_t* scalars_out,
                            uint8_t* points_out);
/* The job's MSM over bucket windows [w_begin, w_end) on this GPU -> 128-B
 * raw partial point, its proofs being batch proofs [first, first + count)
 * weighted from `seed` as bpp_perm_verify_scalars.  The batch verifies iff
 * the partials of every window range (window split: every rank's job holds
 * all proofs) or of every proof slice (proof split: all windows each, no
 * exchange before the MSM) sum to the identity (bpp_partials_is_identity). */
int bpp_perm_verify_partial(bpp_ctx* ctx, const bpp_gens* g, const bpp_verify_job* job, const uint8_t seed[32],
                            size_t first, uint32_t w_begin, uint32_t w_end, uint8_t partial[128]);
/* Window split with the upload and decompression sharded too (config 5
 * over N GPUs, "windows_sharded").  Rank r of N, slice
 * [first, first + n) of the batch:
 *   1. bpp_perm_verify_begin_dev(_async) over the slice's proofs and V only
 *      (each rank uploads, decompresses and replays 1/N of the batch);
 *   2. bpp_perm_verify_slice_points copies the slice's decompressed points
 *      (bpp_perm_verify_slice_point_bytes(job): n x npt records of 128 B,
 *      proof-major) to device memory d_out; BPP_ERR_VERIFY if one did not
 *      decode; returns once d_out is complete (it waits for the
 *      decompression, not for an asynchronous begin's replay), so the point
 *      blocks' all-gather can run beside the replay and step 3;
 *   3. bpp_perm_verify_slice_scalars_at(job, seed, first) writes the slice's
 *      scalar block to device memory d_out (bpp_perm_verify_slice_bytes(job)
 *      bytes): the 2 n_p + 2 generator scalars summed over the slice, then
 *      the slice's n x (m + 8 + 2 lg) proof-point scalars (32 B each,
 *      canonical), the proofs weighted as batch proofs first + p; it
 *      synchronises ctx, so d_out is complete for a collective on return;
 *   4. the point blocks (pstride bytes apart) and the scalar blocks (stride
 *      apart) of all slices are all-gathered into device memory (RCCL
 *      all_gather over xGMI), slices contiguous and in proof order;
 *   5. bpp_perm_verify_partial_sharded runs the MSM of ALL proofs over windows
 *      [w_begin, w_end) from the gathered blocks (job: this rank's slice job,
 *      which must sit at proof offset `first` among counts[]);
 *   6. the 128-B partials are exchanged as for bpp_perm_verify_partial;
 *      a replay reject or an undecodable point on any rank vetoes the batch. */
/* bpp_perm_verify_begin_dev without waiting for the replay (no r_out): the
 * replay's verdicts are checked by the job's next synchronising call
 * (bpp_perm_verify_slice_scalars_at and bpp_perm_verify_partial return
 * BPP_ERR_VERIFY for a rejected proof); bpp_perm_verify_slice_points can run
 * meanwhile (it waits for the decompression only).  Pinned input buffers --
 * bpp_host_alloc's and any memory the caller page-locked itself
 * (hipHostRegister / hipHostMalloc), which the library also sends by DMA --
 * are read after the return: keep them alive and unchanged until that next
 * synchronising call; pageable ones are staged before it returns. */
int bpp_perm_verify_begin_dev_async(bpp_ctx* ctx, uint32_t k, size_t count, const uint8_t* label, size_t llen,
                                    const uint8_t* proofs, const uint8_t* V, bpp_verify_job** out);
size_t bpp_perm_verify_slice_bytes(const bpp_verify_job* job);
int bpp_perm_verify_slice_scalars_at(bpp_ctx* ctx, const bpp_verify_job* job, const uint8_t seed[32], size_t first,
                                     void* d_out);
size_t bpp_perm_verify_slice_point_bytes(const bpp_verify_job* job);
int bpp_perm_verify_slice_points(bpp_ctx* ctx, const bpp_verify_job* job, void* d_out);
int bpp_perm_verify_partial_sharded(bpp_ctx* ctx, const bpp_gens* g, const bpp_verify_job* job, size_t first,
                                    const void* d_blocks, size_t stride, const void* d_pblocks, size_t pstride,
                                    const size_t* counts, size_t nslices, uint32_t w_begin, uint32_t w_end,
                                    uint8_t partial[128]);
void bpp_perm_verify_end(bpp_verify_job* job);
/* BPP_OK if the partials add up to the identity, else BPP_ERR_VERIFY (also
 * for any partial with Z = 0, so an unwritten all-zero partial never passes;
 * callers still exchange a per-rank ok flag). */
int bpp_partials_is_identity(const uint8_t* partials, size_t count);

#ifdef __cplusplus
}
#endif
#endif
