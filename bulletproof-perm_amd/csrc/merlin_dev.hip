// Device-side Merlin for the IPA rounds: one lane
// per proof runs the round's transcript step
//   append_point("L", L); append_point("R", R); u = challenge_scalar("u")
// (merlin 3.0.0 / STROBE-128 over Keccak-f[1600]; the reference's
// TranscriptProtocol, transcript_protocol.rs:45-47,62-67, and bulletproofs'
// InnerProductProof round) and then u^-1 (binary extended Euclid, variable
// time: u is public), writing (u R, u^-1 R) in the layout k_ipa_round_dt
// folds with.  Byte-exact with host/merlin.h (tests/test_gpu_merlin.py).
//
// The proofs of a batch perform the same transcript operations with the same
// lengths, so their STROBE positions agree: pos / pos_begin / cur_flags are
// wave-uniform and only the 200-byte sponge states differ (one per lane, in
// LDS so that the byte-wise absorb/squeeze index them cheaply).
#include "ctx.h"
#include "merlin_dev.h"
#include "merlin_lane.cuh"  // (sc_inv_vartime)

#define STROBE_R_DEV 166
#define ST_STRIDE 200  // bytes of one lane's sponge state in LDS (8-byte aligned)

// STROBE-128 with the sponge state of this lane at `st` (LDS) and the
// wave-uniform position registers.
struct DevStrobe {
  uint8_t* st;
  uint32_t pos, pos_begin, cur_flags;
  FE_INLINE void run_f() {
    st[pos] ^= (uint8_t)pos_begin;
    st[pos + 1] ^= 0x04;
    st[STROBE_R_DEV + 1] ^= 0x80;
    uint64_t a[25];
    const uint64_t* w = reinterpret_cast<const uint64_t*>(st);
    _Pragma("unroll") for (int i = 0; i < 25; ++i) a[i] = w[i];
    keccak_f1600_dev(a);
    uint64_t* o = reinterpret_cast<uint64_t*>(st);
    _Pragma("unroll") for (int i = 0; i < 25; ++i) o[i] = a[i];
    pos = 0;
    pos_begin = 0;
  }
  FE_INLINE void absorb_byte(uint8_t b) {
    st[pos] ^= b;
    if (++pos == STROBE_R_DEV) run_f();
  }
  FE_INLINE void absorb(const uint8_t* d, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) absorb_byte(d[i]);
  }
  FE_INLINE void begin_op(uint32_t flags) {
    const uint32_t old_begin = pos_begin;
    pos_begin = pos + 1;
    cur_flags = flags;
    absorb_byte((uint8_t)old_begin);
    absorb_byte((uint8_t)flags);
    if ((flags & (4u | 32u)) && pos != 0) run_f();  // FLAG_C | FLAG_K
  }
  // merlin append_message(label, msg[n]): meta_ad(label), meta_ad(le32(n),
  // more), ad(msg)
  FE_INLINE void append_message(const uint8_t* label, uint32_t ln, const uint8_t* msg, uint32_t n) {
    begin_op(16u | 2u);  // FLAG_M | FLAG_A
    absorb(label, ln);
    absorb_byte((uint8_t)n);
    absorb_byte((uint8_t)(n >> 8));
    absorb_byte((uint8_t)(n >> 16));
    absorb_byte((uint8_t)(n >> 24));
    begin_op(2u);  // FLAG_A
    absorb(msg, n);
  }
  // merlin challenge_bytes(label, out[n])
  FE_INLINE void challenge_bytes(const uint8_t* label, uint32_t ln, uint8_t* out, uint32_t n) {
    begin_op(16u | 2u);
    absorb(label, ln);
    absorb_byte((uint8_t)n);
    absorb_byte((uint8_t)(n >> 8));
    absorb_byte((uint8_t)(n >> 16));
    absorb_byte((uint8_t)(n >> 24));
    begin_op(1u | 2u | 4u);  // FLAG_I | FLAG_A | FLAG_C
    for (uint32_t i = 0; i < n; ++i) {
      out[i] = st[pos];
      st[pos] = 0;
      if (++pos == STROBE_R_DEV) run_f();
    }
  }
};

__device__ __constant__ static const uint32_t SC_R3[8] = {0x7b83a2dbu, 0x2a9e4968u, 0xaef7f3ecu, 0x278324e6u,
                                                           0x04ec5b65u, 0x8065dc6cu, 0x3599cec7u, 0x0e530b77u};

// Scalar::from_bytes_mod_order_wide in Montgomery form: x = lo + hi 2^256,
// mont(lo, R^2) + mont(hi, R^3) = (lo + hi R) R = x R (mod l)
FE_INLINE sc sc_from_wide_mont(const uint8_t b[64]) {
  sc lo, hi, r2, r3;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    lo.v[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
              ((uint32_t)b[4 * i + 3] << 24);
    hi.v[i] = (uint32_t)b[32 + 4 * i] | ((uint32_t)b[33 + 4 * i] << 8) | ((uint32_t)b[34 + 4 * i] << 16) |
              ((uint32_t)b[35 + 4 * i] << 24);
    r2.v[i] = SC_R2[i];
    r3.v[i] = SC_R3[i];
  }
  return sc_add(sc_mont(lo, r2), sc_mont(hi, r3));
}

// One IPA round's transcript step for P proofs, one lane each.
// states: [P][MERLIN_DEV_STATE_BYTES] (200-byte sponge, pos, pos_begin,
// cur_flags); enc: [P][64] (L then R encodings); u_out: [P][16] words =
// (u R, u^-1 R); u_canon: [P][8] canonical u (for the host's record).
__global__ void __launch_bounds__(64) k_ipa_transcript_step(uint32_t P, uint8_t* __restrict__ states,
                                                            const uint8_t* __restrict__ enc,
                                                            uint32_t* __restrict__ u_out) {
  __shared__ __attribute__((aligned(16))) uint8_t st_lds[64 * ST_STRIDE];
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t q = p < P ? p : P - 1;  // tail lanes shadow the last proof (results dropped)
  uint8_t* g = states + (size_t)q * MERLIN_DEV_STATE_BYTES;
  DevStrobe s;
  s.st = st_lds + threadIdx.x * ST_STRIDE;
  {
    const uint2* src = reinterpret_cast<const uint2*>(g);  // 25 x 8 B (LDS rows are 8-B aligned)
    uint2* dst = reinterpret_cast<uint2*>(s.st);
    for (int i = 0; i < 25; ++i) dst[i] = src[i];
    const uint8_t* meta = g + 200;
    s.pos = meta[0];
    s.pos_begin = meta[1];
    s.cur_flags = meta[2];
  }
  uint8_t L[32], R[32];
  {
    const uint4* e = reinterpret_cast<const uint4*>(enc + (size_t)q * 64);
    uint4* l4 = reinterpret_cast<uint4*>(L);
    uint4* r4 = reinterpret_cast<uint4*>(R);
    l4[0] = e[0];
    l4[1] = e[1];
    r4[0] = e[2];
    r4[1] = e[3];
  }
  const uint8_t lab_L = 'L', lab_R = 'R', lab_u = 'u';
  s.append_message(&lab_L, 1, L, 32);
  s.append_message(&lab_R, 1, R, 32);
  uint8_t ch[64];
  s.challenge_bytes(&lab_u, 1, ch, 64);
  const sc uR = sc_from_wide_mont(ch);
  const sc u = sc_from_mont(uR);
  const sc uiR = sc_to_mont(sc_inv_vartime(u));
  if (p >= P) return;
  {
    const uint2* src = reinterpret_cast<const uint2*>(s.st);
    uint2* dst = reinterpret_cast<uint2*>(g);
    for (int i = 0; i < 25; ++i) dst[i] = src[i];
    uint8_t* meta = g + 200;
    meta[0] = (uint8_t)s.pos;
    meta[1] = (uint8_t)s.pos_begin;
    meta[2] = (uint8_t)s.cur_flags;
  }
  sc_store(u_out + 16 * (size_t)p, uR);
  sc_store(u_out + 16 * (size_t)p + 8, uiR);
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
