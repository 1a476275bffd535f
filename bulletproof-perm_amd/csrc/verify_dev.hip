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
__global__ void __launch_bounds__(64) k_verify_replay(uint32_t count, uint32_t k, uint32_t lg, uint32_t n_p,
                                                      const uint32_t* __restrict__ init,
                                                      const uint32_t* __restrict__ proofs, uint32_t pw,
                                                      const uint32_t* __restrict__ V, uint32_t* __restrict__ rec,
                                                      uint32_t* __restrict__ r_out, uint32_t* __restrict__ bad) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[64 * LANE_ST_BYTES];
  // every lane stays active for the wave-wide inversion below: lanes past
  // the batch shadow the last proof and write nothing
  const bool live = blockIdx.x * 64 + threadIdx.x < count;
  const uint32_t p = live ? blockIdx.x * 64 + threadIdx.x : count - 1;
  LaneStrobe t;
  t.st = lds + threadIdx.x * LANE_ST_BYTES;
  {
    uint32_t* d = reinterpret_cast<uint32_t*>(t.st);
    for (int i = 0; i < 50; ++i) d[i] = init[i];
    t.pos = init[50];
    t.pos_begin = init[51];
  }
  const uint32_t m = 2 * k + 1, nrec = VREC_U + 2 * lg;
  uint32_t* __restrict__ R = rec + (size_t)p * nrec * 8;
  const uint32_t* __restrict__ PV = V + (size_t)p * m * 8;
  const uint32_t* __restrict__ PP = proofs + (size_t)p * pw;
  uint32_t w[8];
  bool ok = true;
  // V_0 .. V_{2k-1}, x_perm, V_2k
  for (uint32_t j = 0; j < 2 * k; ++j) {
    ld8(PV + 8 * j, w);
    t.append32("V", 1, w);
  }
  const sc x_perm = t.challenge_scalar("x_perm", 6);
  ld8(PV + 16 * k, w);
  t.append32("V", 1, w);
  // A_I, A_O, S (validated), y, z
  ld8(PP, w);
  ok &= !w8_zero(w);
  t.append32("A_I", 3, w);
  ld8(PP + 8, w);
  ok &= !w8_zero(w);
  t.append32("A_O", 3, w);
  ld8(PP + 16, w);
  ok &= !w8_zero(w);
  t.append32("S", 1, w);
  const sc y = t.challenge_scalar("y", 1);
  const sc z = t.challenge_scalar("z", 1);
  // T1, T3..T6 (validated), x
  auto T_i = [&](int i, const char* lab) {
    ld8(PP + 24 + 8 * i, w);
    ok &= !w8_zero(w);
    t.append32(lab, 2, w);
  };
  T_i(0, "T1");
  T_i(1, "T3");
  T_i(2, "T4");
  T_i(3, "T5");
  T_i(4, "T6");
  const sc x = t.challenge_scalar("x", 1);
  // tau_x, mu, t_hat (canonical scalars), w
  sc taux, mu, that;
  ld8(PP + 64, taux.v);
  ld8(PP + 72, mu.v);
  ld8(PP + 80, that.v);
  ok &= !sc_geq_l(taux.v) && !sc_geq_l(mu.v) && !sc_geq_l(that.v);
  t.append32("TX", 2, taux.v);
  t.append32("mu", 2, mu.v);
  t.append32("t", 1, that.v);
  const sc wch = t.challenge_scalar("w", 1);
  // bulletproofs InnerProductProof::verification_scalars, transcript part
  t.append_bytes("dom-sep", 7, reinterpret_cast<const uint8_t*>("ipp v1"), 6);
  t.append_u64("n", 1, n_p);
  const uint32_t* PL = PP + 88;
  for (uint32_t j = 0; j < lg; ++j) {
    ld8(PL + 16 * j, w);
    ok &= !w8_zero(w);
    t.append32("L", 1, w);
    ld8(PL + 16 * j + 8, w);
    ok &= !w8_zero(w);
    t.append32("R", 1, w);
    const sc u = t.challenge_scalar("u", 1);
    ok &= !w8_zero(u.v);  // (a zero challenge would fail the batch inversion)
    sc_store(R + 8 * (VREC_U + j), u);
  }
  sc a, b;
  ld8(PL + 16 * lg, a.v);
  ld8(PL + 16 * lg + 8, b.v);
  ok &= !sc_geq_l(a.v) && !sc_geq_l(b.v);
  const sc r = t.challenge_scalar("t-check-weight", 14);
  ok &= !w8_zero(y.v);
  // y^-1 and u_j^-1: Montgomery's trick over the lane's own values (the u^-1
  // slots hold the prefix products meanwhile), then over the wave's 64 lane
  // products, so the wave runs ONE inversion with uniform control flow (a
  // per-lane binary-Euclid inversion diverged and took 0.43 of the kernel's
  // 1.08 ms at 4096 proofs)
  sc acc = sc_to_mont(y);
  for (uint32_t j = 0; j < lg; ++j) {
    if (live) sc_store(R + 8 * (VREC_U + lg + j), acc);
    acc = sc_mont(acc, sc_to_mont(sc_load(R + 8 * (VREC_U + j))));
  }
  sc inv = sc_wave_inverse_mont(acc);
  for (uint32_t j = lg; j-- > 0;) {
    const sc pre = j ? sc_load(R + 8 * (VREC_U + lg + j)) : sc_to_mont(y);
    const sc ui = sc_from_mont(sc_mont(inv, pre));
    inv = sc_mont(inv, sc_to_mont(sc_load(R + 8 * (VREC_U + j))));
    if (live) sc_store(R + 8 * (VREC_U + lg + j), ui);
  }
  if (!live) return;
  sc_store(R + 8 * VREC_XPERM, x_perm);
  sc_store(R + 8 * VREC_YINV, sc_from_mont(inv));
  sc_store(R + 8 * VREC_Z, z);
  sc_store(R + 8 * VREC_X, x);
  sc_store(R + 8 * VREC_W, wch);
  sc_store(R + 8 * VREC_R, r);
  sc_store(R + 8 * VREC_A, a);
  sc_store(R + 8 * VREC_B, b);
  sc_store(R + 8 * VREC_THAT, that);
  sc_store(R + 8 * VREC_TAUX, taux);
  sc_store(R + 8 * VREC_MU, mu);
  sc_store(R + 8 * VREC_WT, sc_zero());
  sc_store(r_out + 8 * (size_t)p, r);
  bad[p] = ok ? 0u : 1u;
}

// w_p = from_wide(SHAKE256("bp-perm-batch-wt" || seed || le64(first + p))
// [0..64]) (perm::batch_weight): 56 bytes, one sponge block.
__global__ void __launch_bounds__(64) k_verify_weights(uint32_t count, uint64_t first, uint64_t total,
                                                       const uint32_t* __restrict__ seed, uint32_t* __restrict__ rec,
                                                       uint32_t nrec) {
  const uint32_t p = blockIdx.x * 64 + threadIdx.x;
  if (p >= count) return;
  sc wt = sc_zero();
  if (total <= 1) {
    wt.v[0] = 1;
  } else {
    uint64_t a[25];
    _Pragma("unroll") for (int i = 0; i < 25; ++i) a[i] = 0;
    a[0] = 0x6d7265702d7062ull | (0x2dull << 56);  // "bp-perm-"
    a[1] = 0x74772d6863746162ull;                 // "batch-wt"
    _Pragma("unroll") for (int i = 0; i < 4; ++i) a[2 + i] = (uint64_t)seed[2 * i] | ((uint64_t)seed[2 * i + 1] << 32);
    a[6] = first + p;
    a[7] = 0x1full;              // SHAKE domain byte at 56
    a[16] = 0x80ull << 56;       // last byte of the 136-byte rate
    keccak_f1600_dev(a);
    uint32_t o[16];
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      o[2 * i] = (uint32_t)a[i];
      o[2 * i + 1] = (uint32_t)(a[i] >> 32);
    }
    wt = sc_from_wide_w(o);
  }
  sc_store(rec + ((size_t)p * nrec + VREC_WT) * 8, wt);
}

// Decompress every proof point straight from the uploaded proofs and V into
// the MSM's Niels table (point i = p npt + j in vpts_n order), so that it
// needs nothing from the replay and runs beside it on another stream.
// *bad = the smallest index of an undecodable encoding (~0 if none).
__global__ void __launch_bounds__(64) k_verify_decompress(uint32_t count, uint32_t m, uint32_t lg, uint32_t npt,
                                                          const uint32_t* __restrict__ proofs, uint32_t pw,
                                                          const uint32_t* __restrict__ V, uint32_t* __restrict__ tbl,
                                                          unsigned long long* __restrict__ bad) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)count * npt) return;
  const uint32_t p = (uint32_t)(i / npt), j = (uint32_t)(i % npt);
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

int verify_replay_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_init,
                      const uint32_t* d_proofs, const uint32_t* d_V, uint32_t* d_rec, uint32_t* r_out,
                      uint32_t* bad) {
  if (!count) return BPP_OK;
  const uint32_t pw = (uint32_t)(perm::proof_len(C.k) / 4);
  {
    ProfScope ps(ctx, "verify_replay_dev");
    hipLaunchKernelGGL(k_verify_replay, dim3(grid_for(count, 64)), dim3(64), 0, ctx->stream, count, C.k, C.lg, C.n_p,
                       d_init, d_proofs, pw, d_V, d_rec, r_out, bad);
  }
  return ctx_check_launch(ctx, "k_verify_replay");
}

int verify_weights_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, uint64_t first, uint64_t total,
                       const uint32_t* seed, uint32_t* d_rec) {
  if (!count) return BPP_OK;
  {
    ProfScope ps(ctx, "verify_weights");
    hipLaunchKernelGGL(k_verify_weights, dim3(grid_for(count, 64)), dim3(64), 0, ctx->stream, count, first, total,
                       seed, d_rec, vrec_n(C));
  }
  return ctx_check_launch(ctx, "k_verify_weights");
}

int verify_decompress_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const uint32_t* d_proofs,
                          const uint32_t* d_V, uint32_t* d_tbl, unsigned long long* d_bad) {
  const size_t n = (size_t)count * vpts_n(C);
  if (!n) return BPP_OK;
  {
    ProfScope ps(ctx, "verify_decompress");
    hipLaunchKernelGGL(k_verify_decompress, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, count, C.m, C.lg,
                       vpts_n(C), d_proofs, (uint32_t)(perm::proof_len(C.k) / 4), d_V, d_tbl, d_bad);
  }
  return ctx_check_launch(ctx, "k_verify_decompress");
}
