// Batch verification on the device (verify_dev.hip, poly.hip k_verify_scalars).
#pragma once
#include <stdint.h>

#include "ctx.h"
#include "host/perm.h"

// Per-proof verifier record: [12 + lg] canonical scalars (8 words each).
// The verifier needs no inverse (DESIGN.md §5 "No inversions"): every
// proof's check is scaled by F = (u_0 .. u_{lg-1})^2 y^(n_p - 1), so y^-i,
// s_0 = prod u_j^-1 and u_j^-2 become y^(n_p-1-i), prod u_j and
// prod_{k != j} u_k^2.
#define VREC_XPERM 0
#define VREC_Y 1
#define VREC_Z 2
#define VREC_X 3
#define VREC_W 4
#define VREC_R 5
#define VREC_A 6
#define VREC_B 7
#define VREC_THAT 8
#define VREC_TAUX 9
#define VREC_MU 10
#define VREC_WT 11  // (unused: the weight is made by k_verify_consts)
#define VREC_U 12   // u_j (lg)
inline uint32_t vrec_n(const perm::Circuit& C) { return VREC_U + C.lg; }
// proof points per proof in MSM order: V_0..V_{m-1}, A_I, A_O, S, T1 T3 T4
// T5 T6, L_0.., R_0..
inline uint32_t vpts_n(const perm::Circuit& C) { return C.m + 8 + 2 * C.lg; }

// Replays `count` transcripts on the device, one per 16-lane group
// (k_verify_replay_g, then k_verify_reduce and k_verify_replay_post): d_proofs [count][proof_len] and d_V [count][m][32] on
// the device; init = the 52-word transcript state every proof shares (the
// label's Transcript::new and arithmetic_domain_sep(n_p); verify_init_state).
// Writes d_rec (the challenges and the proof's scalars), r_out ([count][32],
// the t-check weight challenges) and bad ([count] u32, nonzero where a point
// is the identity encoding, a scalar is not canonical or a challenge is
// zero).  r_out and bad may be pinned host memory (written in place).
// d_stt (optional): the transcripts' V parts already replayed by
// verify_replay_v_dev into d_stt ([count][52] words); the replay then starts
// from each proof's state there and reads only the proof bytes.
// early (optional): proofs [0, early->split) replay on early->st once
// early->ready has fired (their bytes are up), the rest on ctx's stream,
// which then waits for early->done.
struct ReplayEarly {
  hipStream_t st;
  hipEvent_t ready, done;
  uint32_t split;
};
int verify_replay_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_init,
                      const uint32_t* d_proofs, const uint32_t* d_V, uint32_t* d_rec, uint32_t* r_out, uint32_t* bad,
                      const uint32_t* d_stt = nullptr, const ReplayEarly* early = nullptr);
// The early part: launches proofs [0, e.split) on e.st behind e.ready and
// records e.done (call it as soon as those proofs' copies are enqueued).
int verify_replay_early_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_init,
                            const uint32_t* d_proofs, const uint32_t* d_V, const ReplayEarly& e);
// The V part of the transcripts of proofs [p0, p1) of a batch of `total`
// (2k V appends, x_perm, V_2k): needs only their V bytes; leaves each
// proof's sponge in d_stt[p] (52 words) and its x_perm challenge bytes in
// the replay's challenge workspace.
// Launched on stream st (the workspaces are ctx's).
int verify_replay_v_dev(bpp_ctx* ctx, hipStream_t st, const perm::Circuit& C, uint32_t p0, uint32_t p1,
                        uint32_t total, const uint32_t* d_init, const uint32_t* d_V, uint32_t* d_stt);
// Decompresses the proof points of proofs [p0, p1) (p1 = ~0u: count) of the
// uploaded proofs / V into d_tbl ([count * vpts_n] Niels rows in MSM order);
// *d_bad = the smallest index of an undecodable encoding (set to ~0 by the
// caller first).  Independent of the replay (launched on another stream, one
// launch per upload chunk).
// [jlo, jlo + jn): the points of each proof to decode (V_0..V_{m-1} are
// points 0..m-1, the proof's own m..npt-1; default all of them).
int verify_decompress_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_proofs,
                          const uint32_t* d_V, uint32_t* d_tbl, unsigned long long* d_bad, uint32_t p0 = 0,
                          uint32_t p1 = ~0u, uint32_t jlo = 0, uint32_t jn = ~0u);
// The 52-word shared transcript prefix for verify_replay_dev.
void verify_init_state(const perm::Circuit& C, const uint8_t* label, size_t llen, uint32_t out[52]);
// out[i] = sum over the nb blocks (stride words apart) of block[b][i], i < n
// (the generator scalars of a gathered sliced verification).
int verify_sum_blocks_dev(bpp_ctx* ctx, uint32_t nb, uint32_t n, const uint32_t* d_blocks, uint32_t stride,
                          uint32_t* d_out);
// k_verify_consts (each proof's weight perm::batch_weight(seed, first + p,
// r_p) and its constants) + k_verify_scalars + k_verify_merge over device
// records (poly.hip).  seed: 8 words, may be pinned host memory.
int verify_scalars_dev_rec(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_rec,
                           const uint32_t* seed, uint64_t first, uint32_t* d_sc);
