#include <algorithm>
// Batch verifier, device side: every proof's Fiat-Shamir replay on the GPU,
// one lane (one Merlin transcript) per proof, and the batch weights.
//
// Restates the verifier's transcript of ACProof::verify
// (bp-perm/src/circuit_lib.rs:478-585 in sound form; point validation as
// TranscriptProtocol::validate_and_append_point, transcript_protocol.rs:48-60)
// exactly as the host replay does (perm_api.hip verify_replay; byte-equal r
// challenges are tested, tests/test_gpu_verify_dev.py).  A batch's
// transcripts perform the same operations with the same lengths, so one
// wave-uniform schedule drives 64 sponges (merlin_lane.cuh).  The replay was
// the host's largest share of a 4096-proof batch verification (21.6 of 32.3
// ms on the round-2 box, 4 host threads); here 4096 proofs are 64 waves.
#include "ctx.h"
#include "ge_io.cuh"
#include "merlin_group.cuh"
#include "merlin_lane.cuh"
#include "verify_dev.h"

FE_INLINE void ld8(const uint32_t* __restrict__ src, uint32_t w[8]) {
  const uint4 a = reinterpret_cast<const uint4*>(src)[0], b = reinterpret_cast<const uint4*>(src)[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
FE_INLINE void st8(uint32_t* __restrict__ dst, const uint32_t w[8]) {
  reinterpret_cast<uint4*>(dst)[0] = make_uint4(w[0], w[1], w[2], w[3]);
  reinterpret_cast<uint4*>(dst)[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
FE_INLINE bool w8_zero(const uint32_t w[8]) {
  uint32_t o = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) o |= w[i];
  return o == 0;
}

// Proof layout (perm_api.hip serialize, bpp_perm_proof_len): A_I A_O S T1 T3
// T4 T5 T6 (points), tau_x mu t_hat, L_0 R_0 .. L_{lg-1} R_{lg-1}, a b;
// 8 words each.
// ---------------------------------------------------------------------------
// Group replay (round 4, the default): one transcript per 8 lanes
// (merlin_group.cuh), 8 transcripts per 64-lane block, so a 4096-proof batch
// is 512 waves whose permutations cost ~65 instructions a round instead of
// ~190 (GRP_LANES = 16: 16 lanes, 4 transcripts per block, ~45).  The replay keeps only the transcript chain: every challenge's 64
// squeezed bytes go to ch ([count + 1][6 + lg][16] words, the last a pad for
// groups past the batch) and the proof's encoding / canonical-scalar checks to
// okw[p]; k_verify_replay_post reduces the challenges, inverts y and the u_j
// and writes the records, one lane per proof.  STAGED: the group's proof and
// V bytes are first copied into LDS by its 8 lanes (one load latency instead
// of one per absorbed item).
#define RG_GROUPS (64 / GRP_LANES)
// A group's sponge (200 B) and pi scratch (GRP_SCR_BYTES) at a stride of
// GRP_BLOCK: 736 B = 184 dwords (24 mod 32) with the default half-column chi
// layout (GRP_CHI128), whose reads are one 16-B and one 4-B read per column;
// the former dword layout used 576 B = 144 dwords (16 mod 32), chosen with
// tools/lds_banks.py so that the two groups of a 32-lane half hit disjoint
// banks in every chi load (2 extra LDS cycles a round against 20 at 480 B).
// The 736-B stride has not been re-modelled: the replay measured the same
// with the conflicts gone (r04_verify_pmc_final.json), it is not LDS-bound.
#ifndef RG_GS  // (A/B: -DGRP_CHI128=0 -DRG_GS=480 -DRG_SCR_OFF=240 -DGRP_TRASH=50 is the round-3 layout)
#define RG_GS GRP_BLOCK
#define RG_SCR_OFF GRP_SCR_OFF
#endif
// PH: 0 = the whole transcript; 1 = its V part (the 2k V appends, x_perm,
// V_2k), the sponge left in stt[p] (52 words: state, pos, pos_begin); 2 =
// the rest, from stt[p].  The split lets the V part of a chunk of proofs run
// as soon as that chunk's V bytes land (verify_begin_dev, BPP_VERIFY_SPLIT),
// while the proof bytes are still on their way.  Proofs [p0, p1) of a batch
// of `total` (ch and okw indexed by batch proof; ch[total] is the pad).
template <bool STAGED, int PH>
__global__ void __launch_bounds__(64) k_verify_replay_g(uint32_t p0, uint32_t p1, uint32_t total, uint32_t k,
                                                        uint32_t lg, uint32_t n_p, const uint32_t* __restrict__ init,
                                                        const uint32_t* __restrict__ proofs, uint32_t pw,
                                                        const uint32_t* __restrict__ V, uint32_t* __restrict__ ch,
                                                        uint32_t* __restrict__ okw, uint32_t* __restrict__ stt) {
  __shared__ __attribute__((aligned(16))) uint8_t sp[RG_GROUPS * RG_GS];
  extern __shared__ __attribute__((aligned(16))) uint32_t stage[];  // STAGED: [8][pw + 8 m]
  // the replay is a latency chain and the proof-point decompression runs
  // beside it on the same SIMDs: win the issue arbitration
  __builtin_amdgcn_s_setprio(3);
  const uint32_t g = threadIdx.x / GRP_LANES, gl = threadIdx.x % GRP_LANES;
  const uint32_t pg = p0 + blockIdx.x * RG_GROUPS + g;
  const bool live = pg < p1;
  const uint32_t p = live ? pg : p1 - 1;
  const uint32_t m = 2 * k + 1, nch = 6 + lg;
  GroupStrobe t;
  t.st = sp + g * RG_GS;
  t.scr = t.st + RG_SCR_OFF;
  t.gl = gl;
  t.leader = gl == GRP_LEADER;
  {
    const uint32_t* src = PH == 2 ? stt + (size_t)p * 52 : init;
    uint32_t* d = reinterpret_cast<uint32_t*>(t.st);
    for (uint32_t i = gl; i < 50; i += GRP_LANES) d[i] = src[i];
    t.pos = src[50];
    t.pos_begin = src[51];
  }
  const uint32_t* PV = nullptr;
  const uint32_t* PP = nullptr;
  if (STAGED) {
    const uint32_t pwh = PH == 1 ? 0u : pw, vw = PH == 2 ? 0u : 8 * m;  // the words this phase reads
    uint32_t* sg = stage + (size_t)g * (pwh + vw);
    const uint4* sp4 = reinterpret_cast<const uint4*>(proofs + (size_t)p * pw);
    for (uint32_t i = gl; i < pwh / 4; i += GRP_LANES) reinterpret_cast<uint4*>(sg)[i] = sp4[i];
    const uint4* sv4 = reinterpret_cast<const uint4*>(V + (size_t)p * m * 8);
    for (uint32_t i = gl; i < vw / 4; i += GRP_LANES) reinterpret_cast<uint4*>(sg + pwh)[i] = sv4[i];
    PP = sg;
    PV = sg + pwh;
  } else {
    PP = proofs + (size_t)p * pw;
    PV = V + (size_t)p * m * 8;
  }
  GRP_FENCE();
#if GRP_PAR_APPEND
#define APPEND32(lab, ln, w, src) \
  if (!t.append32_par(lab, ln, src)) t.append32(lab, ln, w)
#else
#define APPEND32(lab, ln, w, src) t.append32(lab, ln, w)
#endif
  uint32_t* CH = ch + (size_t)(live ? p : total) * nch * 16;
  uint32_t w[8];
  bool ok = true;
  if (PH != 2) {
    for (uint32_t j = 0; j < 2 * k; ++j) {
      ld8(PV + 8 * j, w);
      APPEND32("V", 1, w, PV + 8 * j);
    }
    t.challenge64_to("x_perm", 6, CH, true);
    ld8(PV + 16 * k, w);
    APPEND32("V", 1, w, PV + 16 * k);
  }
  if (PH == 1) {
    if (live) {
      const uint32_t* d = reinterpret_cast<const uint32_t*>(t.st);
      uint32_t* o = stt + (size_t)p * 52;
      for (uint32_t i = gl; i < 50; i += GRP_LANES) o[i] = d[i];
      if (t.leader) {
        o[50] = t.pos;
        o[51] = t.pos_begin;
      }
    }
    return;
  }
  ld8(PP, w);
  ok &= !w8_zero(w);
  APPEND32("A_I", 3, w, PP);
  ld8(PP + 8, w);
  ok &= !w8_zero(w);
  APPEND32("A_O", 3, w, PP + 8);
  ld8(PP + 16, w);
  ok &= !w8_zero(w);
  APPEND32("S", 1, w, PP + 16);
  t.challenge64_to("y", 1, CH + 16, true);
  t.challenge64_to("z", 1, CH + 32, true);
  auto T_i = [&](int i, const char* lab) {
    ld8(PP + 24 + 8 * i, w);
    ok &= !w8_zero(w);
    APPEND32(lab, 2, w, PP + 24 + 8 * i);
  };
  T_i(0, "T1");
  T_i(1, "T3");
  T_i(2, "T4");
  T_i(3, "T5");
  T_i(4, "T6");
  t.challenge64_to("x", 1, CH + 48, true);
  ld8(PP + 64, w);
  ok &= !sc_geq_l(w);
  APPEND32("TX", 2, w, PP + 64);
  ld8(PP + 72, w);
  ok &= !sc_geq_l(w);
  APPEND32("mu", 2, w, PP + 72);
  ld8(PP + 80, w);
  ok &= !sc_geq_l(w);
  APPEND32("t", 1, w, PP + 80);
  t.challenge64_to("w", 1, CH + 64, true);
  t.append_bytes("dom-sep", 7, reinterpret_cast<const uint8_t*>("ipp v1"), 6);
  t.append_u64("n", 1, n_p);
  const uint32_t* PL = PP + 88;
  for (uint32_t j = 0; j < lg; ++j) {
    ld8(PL + 16 * j, w);
    ok &= !w8_zero(w);
    APPEND32("L", 1, w, PL + 16 * j);
    ld8(PL + 16 * j + 8, w);
    ok &= !w8_zero(w);
    APPEND32("R", 1, w, PL + 16 * j + 8);
    t.challenge64_to("u", 1, CH + 16 * (5 + j), true);
  }
  ld8(PL + 16 * lg, w);
  ok &= !sc_geq_l(w);
  ld8(PL + 16 * lg + 8, w);
  ok &= !sc_geq_l(w);
  t.challenge64_to("t-check-weight", 14, CH + 16 * (5 + lg), true);
  if (live && t.leader) okw[p] = ok ? 1u : 0u;
}

// One lane per (proof, challenge): the 64 squeezed bytes of k_verify_replay_g
// reduced mod l (the verifier's challenge_scalar, transcript_protocol.rs:62-67)
// into the proof's record -- x_perm, y, z, x, w, u_j, r in their slots -- and
// r to r_out.  (One lane per proof ran the 6 + lg reductions in a row, ~2.4 K
// cycles each.)
__global__ void __launch_bounds__(64) k_verify_reduce(uint32_t count, uint32_t lg, const uint32_t* __restrict__ ch,
                                                      uint32_t* __restrict__ rec, uint32_t* __restrict__ r_out) {
  __builtin_amdgcn_s_setprio(3);  // (latency chain; the decompression runs beside it)
  const uint32_t nch = 6 + lg, nrec = VREC_U + lg;
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (t >= (size_t)count * nch) return;
  const uint32_t p = (uint32_t)(t / nch), c = (uint32_t)(t % nch);
  const sc v = sc_from_wide_w(ch + t * 16);
  const uint32_t slot = c == 0   ? VREC_XPERM
                        : c == 1 ? VREC_Y
                        : c == 2 ? VREC_Z
                        : c == 3 ? VREC_X
                        : c == 4 ? VREC_W
                        : c < 5 + lg ? VREC_U + (c - 5)
                                     : VREC_R;
  sc_store(rec + ((size_t)p * nrec + slot) * 8, v);
  if (c == 5 + lg) sc_store(r_out + 8 * (size_t)p, v);
}

// One lane per proof, after k_verify_reduce: the checks (a zero y or u_j
// rejects the proof: the verifier's scaling by (prod u_j)^2 y^(n_p - 1) must
// not vanish) and the record's proof scalars.  No inversions: the checks are
// scaled instead (poly.hip k_verify_consts).
__global__ void __launch_bounds__(64) k_verify_replay_post(uint32_t count, uint32_t lg,
                                                           const uint32_t* __restrict__ okw,
                                                           const uint32_t* __restrict__ proofs, uint32_t pw,
                                                           uint32_t* __restrict__ rec, uint32_t* __restrict__ bad) {
  __builtin_amdgcn_s_setprio(3);  // (latency chain; the decompression runs beside it)
  const uint32_t p = blockIdx.x * 64 + threadIdx.x;
  if (p >= count) return;
  const uint32_t nrec = VREC_U + lg;
  uint32_t* __restrict__ R = rec + (size_t)p * nrec * 8;
  const uint32_t* __restrict__ PP = proofs + (size_t)p * pw;
  bool ok = okw[p] != 0;
  uint32_t w[8];
  ld8(R + 8 * VREC_Y, w);
  ok &= !w8_zero(w);
  for (uint32_t j = 0; j < lg; ++j) {
    ld8(R + 8 * (VREC_U + j), w);
    ok &= !w8_zero(w);
  }
  ld8(PP + 88 + 16 * lg, w);
  st8(R + 8 * VREC_A, w);
  ld8(PP + 88 + 16 * lg + 8, w);
  st8(R + 8 * VREC_B, w);
  ld8(PP + 80, w);
  st8(R + 8 * VREC_THAT, w);
  ld8(PP + 64, w);
  st8(R + 8 * VREC_TAUX, w);
  ld8(PP + 72, w);
  st8(R + 8 * VREC_MU, w);
  bad[p] = ok ? 0u : 1u;
}

// Decompress every proof point straight from the uploaded proofs and V into
// the MSM's Niels table (point i = p npt + j in vpts_n order), so that it
// needs nothing from the replay and runs beside it on another stream.
// *bad = the smallest index of an undecodable encoding (~0 if none).
// (VD_WPE waves per SIMD: unconstrained, the compiler takes 244 VGPRs for the
// inverse square root, 2 waves per SIMD; config 5, interleaved A/B passes:
// 0.594-0.607 ms unconstrained, 0.554-0.559 at 3 (167 VGPRs, spills outside
// the squaring loops only), 0.62 at 4, 0.58-0.59 at 6; with the chunked
// upload, 4 -- so that a replay wave fits beside three decompression waves --
// shortened the replay stage but not the batch: 2.11-2.15 vs 2.06-2.12 ms,
// profiles/r04_verify_vd4_ab.txt)
#ifndef VD_WPE
#define VD_WPE 3
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(VD_WPE)))
k_verify_decompress(size_t i0, size_t i1, uint32_t jlo, uint32_t jn, uint32_t m, uint32_t lg, uint32_t npt,
                    const uint32_t* __restrict__ proofs, uint32_t pw, const uint32_t* __restrict__ V,
                    uint32_t* __restrict__ tbl, unsigned long long* __restrict__ bad) {
#ifdef VD_PRIO  // (A/B: issue priority against the expansion's s_setprio(2))
  __builtin_amdgcn_s_setprio(VD_PRIO);
#endif
  // lane -> (proof p, point j = jlo + j' with j' < jn): the V points (jlo =
  // 0, jn = m) or the proof's own points (jlo = m) can go separately
  const size_t t = i0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= i1) return;
  const uint32_t p = (uint32_t)(t / jn), j = jlo + (uint32_t)(t % jn);
  const size_t i = (size_t)p * npt + j;
  const uint32_t* src;
  if (j < m)
    src = V + ((size_t)p * m + j) * 8;
  else if (j < m + 8)
    src = proofs + (size_t)p * pw + 8 * (j - m);  // A_I A_O S T1 T3..T6
  else if (j < m + 8 + lg)
    src = proofs + (size_t)p * pw + 88 + 16 * (j - m - 8);  // L_j
  else
    src = proofs + (size_t)p * pw + 96 + 16 * (j - m - 8 - lg);  // R_j
  uint32_t w[8];
  ld8(src, w);
  ge_p3 P;
  if (!ge_ristretto_decode(w, P)) {
    atomicMin(bad, (unsigned long long)i);
    P = ge_identity();
  }
  store_niels(tbl, (uint32_t)i, ge_niels_from_affine(P.X, P.Y));  // (Z = 1 after decode)
}

static unsigned grid_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

void verify_init_state(const perm::Circuit& C, const uint8_t* label, size_t llen, uint32_t out[52]) {
  merlin::Transcript tr(label, llen);
  tr.arithmetic_domain_sep(C.n_p);
  memcpy(out, tr.s.st, 200);
  out[50] = tr.s.pos;
  out[51] = tr.s.pos_begin;
}

template <int PH>
static void launch_replay(hipStream_t st, const perm::Circuit& C, uint32_t p0, uint32_t p1, uint32_t total,
                          const uint32_t* d_init, const uint32_t* d_proofs, const uint32_t* d_V, uint32_t* d_ch,
                          uint32_t* d_ok, uint32_t* d_stt) {
  const uint32_t pw = (uint32_t)(perm::proof_len(C.k) / 4);
  // the bytes the phase reads, of the block's groups, staged in LDS while they fit
  const size_t words = (PH == 1 ? 0 : pw) + (PH == 2 ? 0 : 8 * (size_t)C.m);
  const size_t stage = (size_t)RG_GROUPS * words * 4;
  if (stage <= 48 * 1024)
    hipLaunchKernelGGL((k_verify_replay_g<true, PH>), dim3(grid_for(p1 - p0, RG_GROUPS)), dim3(64), stage, st,
                       p0, p1, total, C.k, C.lg, C.n_p, d_init, d_proofs, pw, d_V, d_ch, d_ok, d_stt);
  else
    hipLaunchKernelGGL((k_verify_replay_g<false, PH>), dim3(grid_for(p1 - p0, RG_GROUPS)), dim3(64), 0, st,
                       p0, p1, total, C.k, C.lg, C.n_p, d_init, d_proofs, pw, d_V, d_ch, d_ok, d_stt);
}

int verify_replay_v_dev(bpp_ctx* ctx, hipStream_t st, const perm::Circuit& C, uint32_t p0, uint32_t p1,
                        uint32_t total, const uint32_t* d_init, const uint32_t* d_V, uint32_t* d_stt) {
  if (p0 >= p1) return BPP_OK;
  const uint32_t nch = 6 + C.lg;
  void *d_ch = nullptr, *d_ok = nullptr;
  BPP_TRY(ctx_ws(ctx, "vj_ch", ((size_t)total + 1) * nch * 64, &d_ch));
  BPP_TRY(ctx_ws(ctx, "vj_ok", (size_t)total * 4, &d_ok));
  launch_replay<1>(st, C, p0, p1, total, d_init, nullptr, d_V, (uint32_t*)d_ch, (uint32_t*)d_ok, d_stt);
  return ctx_check_launch(ctx, "k_verify_replay_g<V>");
}

int verify_replay_early_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_init,
                            const uint32_t* d_proofs, const uint32_t* d_V, const ReplayEarly& e) {
  if (!e.split || e.split >= count) return BPP_OK;
  const uint32_t nch = 6 + C.lg;
  void *d_ch = nullptr, *d_ok = nullptr;
  BPP_TRY(ctx_ws(ctx, "vj_ch", ((size_t)count + 1) * nch * 64, &d_ch));
  BPP_TRY(ctx_ws(ctx, "vj_ok", (size_t)count * 4, &d_ok));
  // proofs [0, split) as soon as their bytes are up (e.ready): a latency
  // chain of ~0.25-0.3 ms beside the last chunk's upload and the rest's replay
  BPP_HIP(hipStreamWaitEvent(e.st, e.ready, 0));
  launch_replay<0>(e.st, C, 0, e.split, count, d_init, d_proofs, d_V, (uint32_t*)d_ch, (uint32_t*)d_ok, nullptr);
  BPP_HIP(hipEventRecord(e.done, e.st));
  return ctx_check_launch(ctx, "k_verify_replay_g<early>");
}

int verify_replay_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_init,
                      const uint32_t* d_proofs, const uint32_t* d_V, uint32_t* d_rec, uint32_t* r_out, uint32_t* bad,
                      const uint32_t* d_stt, const ReplayEarly* early) {
  if (!count) return BPP_OK;
  const uint32_t pw = (uint32_t)(perm::proof_len(C.k) / 4);
  const uint32_t nch = 6 + C.lg;
  void *d_ch = nullptr, *d_ok = nullptr;
  BPP_TRY(ctx_ws(ctx, "vj_ch", ((size_t)count + 1) * nch * 64, &d_ch));
  BPP_TRY(ctx_ws(ctx, "vj_ok", (size_t)count * 4, &d_ok));
  {
    ProfScope ps(ctx, "verify_replay_dev");
    if (d_stt) {
      launch_replay<2>(ctx->stream, C, 0, count, count, nullptr, d_proofs, d_V, (uint32_t*)d_ch, (uint32_t*)d_ok,
                       (uint32_t*)d_stt);
    } else if (early && early->split > 0 && early->split < count) {
      // proofs [0, split) went on early->st already (verify_replay_early_dev);
      // the rest here after the last copy, then the join
      launch_replay<0>(ctx->stream, C, early->split, count, count, d_init, d_proofs, d_V, (uint32_t*)d_ch,
                       (uint32_t*)d_ok, nullptr);
      BPP_HIP(hipStreamWaitEvent(ctx->stream, early->done, 0));
    } else {
      launch_replay<0>(ctx->stream, C, 0, count, count, d_init, d_proofs, d_V, (uint32_t*)d_ch, (uint32_t*)d_ok,
                       nullptr);
    }
  }
  BPP_TRY(ctx_check_launch(ctx, "k_verify_replay_g"));
  {
    ProfScope ps(ctx, "verify_replay_post");
    hipLaunchKernelGGL(k_verify_reduce, dim3(grid_for((size_t)count * nch, 64)), dim3(64), 0, ctx->stream, count,
                       C.lg, (const uint32_t*)d_ch, d_rec, r_out);
    hipLaunchKernelGGL(k_verify_replay_post, dim3(grid_for(count, 64)), dim3(64), 0, ctx->stream, count, C.lg,
                       (const uint32_t*)d_ok, d_proofs, pw, d_rec, bad);
  }
  return ctx_check_launch(ctx, "k_verify_reduce/post");
}

// out[i] = sum_b blocks[b * stride + 8 i] (mod l, canonical in and out)
__global__ void __launch_bounds__(64) k_verify_sum_blocks(uint32_t nb, uint32_t n, const uint32_t* __restrict__ blocks,
                                                          uint32_t stride, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  sc acc = sc_zero();
  for (uint32_t b = 0; b < nb; ++b) acc = sc_add(acc, sc_load(blocks + (size_t)b * stride + 8 * (size_t)i));
  sc_store(out + 8 * (size_t)i, acc);
}

int verify_sum_blocks_dev(bpp_ctx* ctx, uint32_t nb, uint32_t n, const uint32_t* d_blocks, uint32_t stride,
                          uint32_t* d_out) {
  if (!n) return BPP_OK;
  hipLaunchKernelGGL(k_verify_sum_blocks, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, nb, n, d_blocks, stride,
                     d_out);
  return ctx_check_launch(ctx, "k_verify_sum_blocks");
}


int verify_decompress_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_proofs,
                          const uint32_t* d_V, uint32_t* d_tbl, unsigned long long* d_bad, uint32_t p0, uint32_t p1,
                          uint32_t jlo, uint32_t jn) {
  p1 = std::min(p1, count);
  const uint32_t npt = vpts_n(C);
  if (jlo >= npt) return BPP_OK;
  jn = std::min(jn, npt - jlo);
  if (p0 >= p1 || !jn) return BPP_OK;
  const size_t i0 = (size_t)p0 * jn, i1 = (size_t)p1 * jn;
  {
    ProfScope ps(ctx, "verify_decompress");
    hipLaunchKernelGGL(k_verify_decompress, dim3(grid_for(i1 - i0, 64)), dim3(64), 0, ctx->stream, i0, i1, jlo, jn, C.m,
                       C.lg, npt, d_proofs, (uint32_t)(perm::proof_len(C.k) / 4), d_V, d_tbl, d_bad);
  }
  return ctx_check_launch(ctx, "k_verify_decompress");
}
