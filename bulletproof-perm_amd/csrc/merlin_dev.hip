// Device-side Merlin for the IPA rounds: one lane
// per proof runs the round's transcript step
//   append_point("L", L); append_point("R", R); u = challenge_scalar("u")
// (merlin 3.0.0 / STROBE-128 over Keccak-f[1600]; the reference's
// TranscriptProtocol, transcript_protocol.rs:45-47,62-67, and bulletproofs'
// InnerProductProof round) and then u^-1 (one variable-time inversion per
// wave: u is public), writing (u R, u^-1 R) in the layout k_ipa_round_dt
// folds with.  Byte-exact with host/merlin.h (tests/test_gpu_merlin.py).
//
// The proofs of a batch perform the same transcript operations with the same
// lengths, so their STROBE positions agree: pos / pos_begin / cur_flags are
// wave-uniform and only the 200-byte sponge states differ (merlin_lane.cuh).
#include "ctx.h"
#include "merlin_dev.h"
#include "merlin_lane.cuh"

// One IPA round's transcript step for P proofs, one lane each
// (merlin_lane.cuh's LaneStrobe: the sponge in LDS, 32-byte appends as
// dwords, the permutation out of line), u^-1 by one inversion per wave.
// states: [P][MERLIN_DEV_STATE_BYTES] (200-byte sponge, pos, pos_begin,
// cur_flags); enc: [P][64] (L then R encodings); u_out: [P][16] words =
// (u R, u^-1 R).
__global__ void __launch_bounds__(64) k_ipa_transcript_step(uint32_t P, uint8_t* __restrict__ states,
                                                            const uint8_t* __restrict__ enc,
                                                            uint32_t* __restrict__ u_out) {
  __shared__ __attribute__((aligned(16))) uint8_t st_lds[64 * LANE_ST_BYTES];
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = p < P;
  const uint32_t q = live ? p : P - 1;  // tail lanes shadow the last proof (the wave inversion needs every lane)
  uint8_t* g = states + (size_t)q * MERLIN_DEV_STATE_BYTES;
  LaneStrobe s;
  s.st = st_lds + threadIdx.x * LANE_ST_BYTES;
  {
    const uint2* src = reinterpret_cast<const uint2*>(g);  // 25 x 8 B (LDS rows are 8-B aligned)
    uint2* dst = reinterpret_cast<uint2*>(s.st);
    for (int i = 0; i < 25; ++i) dst[i] = src[i];
    s.pos = g[200];
    s.pos_begin = g[201];
  }
  uint32_t L[8], R[8];
  {
    const uint4* e = reinterpret_cast<const uint4*>(enc + (size_t)q * 64);
    const uint4 l0 = e[0], l1 = e[1], r0 = e[2], r1 = e[3];
    L[0] = l0.x; L[1] = l0.y; L[2] = l0.z; L[3] = l0.w; L[4] = l1.x; L[5] = l1.y; L[6] = l1.z; L[7] = l1.w;
    R[0] = r0.x; R[1] = r0.y; R[2] = r0.z; R[3] = r0.w; R[4] = r1.x; R[5] = r1.y; R[6] = r1.z; R[7] = r1.w;
  }
  s.append32("L", 1, L);
  s.append32("R", 1, R);
  const sc uR = sc_to_mont(s.challenge_scalar("u", 1));
  const sc uiR = sc_wave_inverse_mont(uR);
  if (!live) return;
  {
    const uint2* src = reinterpret_cast<const uint2*>(s.st);
    uint2* dst = reinterpret_cast<uint2*>(g);
    for (int i = 0; i < 25; ++i) dst[i] = src[i];
    g[200] = (uint8_t)s.pos;
    g[201] = (uint8_t)s.pos_begin;
    g[202] = 1u | 2u | 4u;  // cur_flags of the last op (the challenge's prf: I | A | C)
  }
  sc_store(u_out + 16 * (size_t)p, uR);
  sc_store(u_out + 16 * (size_t)p + 8, uiR);
}

// The prover's V phase for P proofs, one lane each: from the shared state
// after Transcript::new(label) + arithmetic_domain_sep(n_p) (init: 50 state
// words + pos + pos_begin), append_point("V", V_i) for i < 2k and
// x_perm = challenge_scalar("x_perm") (perm_api.hip prove_batch; the
// reference's create, circuit_lib.rs:139-186, in sound form).  venc: [P][2k]
// encodings on the device.  states_out: [P][MERLIN_DEV_STATE_BYTES],
// xperm_out: [P][8] canonical words (both may be pinned host memory).
__global__ void __launch_bounds__(64) k_prove_v_transcript(uint32_t P, uint32_t k, const uint32_t* __restrict__ init,
                                                           const uint32_t* __restrict__ venc,
                                                           uint8_t* __restrict__ states_out,
                                                           uint32_t* __restrict__ xperm_out) {
  __shared__ __attribute__((aligned(16))) uint8_t st_lds[64 * LANE_ST_BYTES];
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;  // (no LDS or shuffle shared between lanes)
  LaneStrobe s;
  s.st = st_lds + threadIdx.x * LANE_ST_BYTES;
  {
    uint32_t* d = reinterpret_cast<uint32_t*>(s.st);
    for (int i = 0; i < 50; ++i) d[i] = init[i];
    s.pos = init[50];
    s.pos_begin = init[51];
  }
  const uint32_t* V = venc + (size_t)p * 2 * k * 8;
  for (uint32_t j = 0; j < 2 * k; ++j) {
    const uint4 a = reinterpret_cast<const uint4*>(V + 8 * j)[0], b = reinterpret_cast<const uint4*>(V + 8 * j)[1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    s.append32("V", 1, w);
  }
  const sc x = s.challenge_scalar("x_perm", 6);
  uint8_t* g = states_out + (size_t)p * MERLIN_DEV_STATE_BYTES;
  const uint2* src = reinterpret_cast<const uint2*>(s.st);
  uint2* dst = reinterpret_cast<uint2*>(g);
  for (int i = 0; i < 25; ++i) dst[i] = src[i];
  reinterpret_cast<uint32_t*>(g)[50] = s.pos | (s.pos_begin << 8) | ((1u | 2u | 4u) << 16);  // pos, pos_begin, cur_flags
  sc_store(xperm_out + 8 * (size_t)p, x);
}

int prove_v_transcript_dev(bpp_ctx* ctx, uint32_t P, uint32_t k, const uint32_t* init, const uint32_t* d_venc,
                           uint8_t* states_out, uint32_t* xperm_out) {
  if (!P) return BPP_OK;
  {
    ProfScope ps(ctx, "prove_v_transcript");
    hipLaunchKernelGGL(k_prove_v_transcript, dim3((P + 63) / 64), dim3(64), 0, ctx->stream, P, k, init, d_venc,
                       states_out, xperm_out);
  }
  return ctx_check_launch(ctx, "k_prove_v_transcript");
}

static unsigned grid_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

int ipa_transcript_step_dev(bpp_ctx* ctx, uint32_t P, uint8_t* d_states, const uint8_t* d_enc, uint32_t* d_u) {
  if (!P) return BPP_OK;
  {
    ProfScope ps(ctx, "ipa_merlin");
    hipLaunchKernelGGL(k_ipa_transcript_step, dim3(grid_for(P, 64)), dim3(64), 0, ctx->stream, P, d_states, d_enc,
                       d_u);
  }
  return ctx_check_launch(ctx, "k_ipa_transcript_step");
}

void merlin_state_export(const merlin::Transcript& t, uint8_t* out) {
  memcpy(out, t.s.st, 200);
  out[200] = t.s.pos;
  out[201] = t.s.pos_begin;
  out[202] = t.s.cur_flags;
  memset(out + 203, 0, MERLIN_DEV_STATE_BYTES - 203);
}

void merlin_state_import(merlin::Transcript& t, const uint8_t* in) {
  memcpy(t.s.st, in, 200);
  t.s.pos = in[200];
  t.s.pos_begin = in[201];
  t.s.cur_flags = in[202];
}
