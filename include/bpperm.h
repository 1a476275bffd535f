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

enum {
  BPP_OK = 0,
  BPP_ERR_ARG = 1,
  BPP_ERR_LEN = 2,
  BPP_ERR_DECOMPRESS = 3,
  BPP_ERR_NONCANONICAL = 4,
  BPP_ERR_DEVICE = 5,
  BPP_ERR_VERIFY = 6,
  BPP_ERR_NOMEM = 7,
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
/* Sum raw extended partial points (count x 128 bytes) and compress. */
int bpp_partials_finish(const uint8_t* partials, size_t count, uint8_t out[32]);
/* count independent MSMs; MSM j covers terms [offsets[j], offsets[j+1]) of
 * `scalars` (32 bytes each) and `point_idx` (indices into tbl). */
int bpp_msm_batch(bpp_ctx* ctx, size_t count, const uint64_t* offsets, const uint8_t* scalars,
                  const uint32_t* point_idx, const bpp_points* tbl, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
