// Generators resident in HBM + fixed-base Pedersen commitments.
//
// bpp_gens = BulletproofGens::new(n, 1) (G_vec, H_vec from SHAKE256
// GeneratorsChain "G"||0u32 / "H"||0u32) + PedersenGens::default() (B, B_blinding
// = hash_from_bytes::<Sha3_512>(B.compress())), or explicit points as the
// reference's test builds them (lib.rs:163-180, random G/H and a random
// PedersenGens).  Table layout (affine Niels): G[0..n) H[n..2n) B[2n] Bb[2n+1].
//
// Pedersen commitments V = v*B + gamma*Bb (weights.rs:58-61,
// PedersenGens::commit) and T_i = t_i*g + tau_i*h (circuit_lib.rs:363-413) are
// fixed-base: per base a table of d*16^i*P (i < 64, d = 1..8) turns each
// commitment into 2 x 64 mixed additions with signed radix-16 digits and no
// doublings; one lane per commitment.
#include <cstdlib>
#include <cstring>

#include "ctx.h"
#include "gens.h"
#include "ge_io.cuh"
#include "host/merlin.h"

static unsigned grid_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// declared in points.hip
__global__ void k_decompress(const uint32_t* __restrict__ enc, size_t n, uint32_t* __restrict__ tbl,
                             unsigned long long* __restrict__ bad);
__global__ void k_from_uniform(const uint32_t* __restrict__ bytes, size_t n, uint32_t* __restrict__ tbl);

// thread t: base = t / 512, pos = (t / 8) % 64, d = t % 8 + 1 -> d * 16^pos * P_base
__global__ void __launch_bounds__(64) k_fb_tables(const uint32_t* __restrict__ tbl, uint32_t b0, uint32_t b1, uint32_t* __restrict__ fb) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * FB_POS * 8) return;
  const uint32_t base = t / (FB_POS * 8), pos = (t / 8) % FB_POS, d = t % 8 + 1;
  const ge_niels P = load_niels(tbl, base ? b1 : b0);
  ge_p3 acc = ge_identity();
  for (uint32_t i = 0; i < d; ++i) acc = ge_madd(acc, P);
  for (uint32_t i = 0; i < 4 * pos; ++i) acc = ge_dbl(acc);
  store_niels(fb, t, ge_to_niels(acc));
}

// Bits [16q, 16q + 16) of s + K, K = 8 * sum_{i<63} 16^i: nibble i of s + K
// minus 8 is signed radix-16 digit i of s (i < 63, digits in [-8, 8)) and
// nibble 63 the top digit (s < 2^253: at most 2), the same digits as a
// carry-propagating recoding, in closed form and without a data-dependent
// index (the word is picked by selects).
FE_INLINE uint32_t ped_digit_bits(const uint32_t* __restrict__ sp, uint32_t q) {
  uint64_t c = 0;
  uint32_t word = 0;
  _Pragma("unroll") for (uint32_t i = 0; i < 8; ++i) {
    c += (uint64_t)sp[i] + (i < 7 ? 0x88888888u : 0x08888888u);
    word = (q >> 1) == i ? (uint32_t)c : word;
    c >>= 32;
  }
  return (word >> (16 * (q & 1))) & 0xffffu;
}

// Constant-time table lookup (dalek's LookupTable::select, which
// PedersenGens::commit's constant-time multiscalar_mul uses): all eight
// rows d * 16^pos * P (d = 1..8) are loaded and the one for |d| is kept by
// masks; d = 0 keeps the Niels identity.  The loads and the instruction
// stream do not depend on the digit.
FE_INLINE ge_niels ped_select_ct(const uint32_t* __restrict__ fb, uint32_t row0, uint32_t ad) {
  ge_niels r = ge_niels_identity();
  _Pragma("unroll 2") for (uint32_t j = 1; j <= 8; ++j) {
    const ge_niels t = load_niels(fb, row0 + j - 1);
    const uint32_t mask = 0u - (uint32_t)(ad == j);
    _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
      r.ypx.v[i] ^= (r.ypx.v[i] ^ t.ypx.v[i]) & mask;
      r.ymx.v[i] ^= (r.ymx.v[i] ^ t.ymx.v[i]) & mask;
      r.xy2d.v[i] ^= (r.xy2d.v[i] ^ t.xy2d.v[i]) & mask;
    }
  }
  return r;
}

// P_j = v_j * B + g_j * Bb (PedersenGens::commit, weights.rs:58-61), PED_G
// lanes per commitment: lane q adds the table entries of radix-16 positions
// [4q, 4q+4) of both scalars (always 8 mixed additions: no zero skip), then
// the 16 partial sums are combined with 4 xor-shuffle levels.  Constant time
// in v and gamma like the reference's commit: digits in closed form,
// ped_select_ct over all eight rows, signs by operand selects
// (ge_madd_signed).  A one-lane-per-commitment kernel would chain 128
// additions (the GPU's per-lane field-multiply latency is ~0.3 us,
// profiles/r01_felat.txt).
#define PED_G 16
#define PED_PER (FB_POS / PED_G)  // radix-16 digits per lane and scalar
__global__ void __launch_bounds__(256) k_pedersen(const uint32_t* __restrict__ fb, const uint32_t* __restrict__ v,
                                                  const uint32_t* __restrict__ gam, size_t m,
                                                  uint32_t* __restrict__ out_p3) {
  const size_t gt = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t j = gt / PED_G;
  const uint32_t q = (uint32_t)(gt % PED_G);
  ge_p3 acc = ge_identity();
  if (j < m) {
    _Pragma("unroll 1") for (uint32_t which = 0; which < 2; ++which) {
      const uint32_t bits = ped_digit_bits((which ? gam : v) + 8 * j, q);
      _Pragma("unroll 1") for (uint32_t b = 0; b < PED_PER; ++b) {
        const uint32_t pos = PED_PER * q + b;
        const int nib = (int)((bits >> (4 * b)) & 15u);
        const int d = pos < FB_POS - 1 ? nib - 8 : nib;
        const int sg = d >> 31;  // 0 or -1
        const uint32_t ad = (uint32_t)((d ^ sg) - sg);
        const ge_niels t = ped_select_ct(fb, (which * FB_POS + pos) * 8, ad);
        acc = ge_madd_signed(acc, t, sg != 0);
      }
    }
  }
  _Pragma("unroll") for (int off = 1; off < PED_G; off <<= 1) {
    ge_p3 o;
    _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
      o.X.v[i] = __shfl_xor(acc.X.v[i], off, 64);
      o.Y.v[i] = __shfl_xor(acc.Y.v[i], off, 64);
      o.Z.v[i] = __shfl_xor(acc.Z.v[i], off, 64);
      o.T.v[i] = __shfl_xor(acc.T.v[i], off, 64);
    }
    acc = ge_add(acc, o);
  }
  if (j < m && q == 0) store_p3(out_p3, j, acc);
}

// declared in points.hip
__global__ void k_compress_p3(const uint32_t* __restrict__ pts, size_t n, uint32_t* __restrict__ out);

static int gens_alloc(bpp_ctx* ctx, size_t n, bpp_gens** out) {
  bpp_gens* g = new bpp_gens();
  g->ctx = ctx;
  g->n = n;
  if (hipMalloc(&g->d_tbl, (2 * n + 2) * MSM_NIELS_WORDS * 4) != hipSuccess ||
      hipMalloc(&g->d_fb, 2 * FB_POS * 8 * MSM_NIELS_WORDS * 4) != hipSuccess) {
    if (g->d_tbl) hipFree(g->d_tbl);
    delete g;
    ctx->err = "hipMalloc generators";
    return BPP_ERR_NOMEM;
  }
  *out = g;
  return BPP_OK;
}

static int gens_finish(bpp_ctx* ctx, bpp_gens* g) {
  {
    ProfScope ps(ctx, "fb_tables");
    hipLaunchKernelGGL(k_fb_tables, dim3(grid_for(2 * FB_POS * 8, 64)), dim3(64), 0, ctx->stream, g->d_tbl,
                       (uint32_t)(2 * g->n), (uint32_t)(2 * g->n + 1), g->d_fb);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_fb_tables"));
  BPP_HIP(hipStreamSynchronize(ctx->stream));
  return BPP_OK;
}

int pedersen_dev(bpp_ctx* ctx, const bpp_gens* g, const uint32_t* d_v, const uint32_t* d_gam, size_t m,
                 uint32_t* d_out_enc, uint32_t* d_out_p3) {
  if (!m) return BPP_OK;
  uint32_t* p3 = d_out_p3;
  if (!p3) {
    void* w = nullptr;
    BPP_TRY(ctx_ws(ctx, "ped_p3", m * P3_BYTES, &w));
    p3 = (uint32_t*)w;
  }
  // (commitments as 2-term MSMs over B / B~'s radix-256 direct tables, 8
  // lanes each, halve the table additions but measured slower with 8 proof
  // batches in flight, 68-79 K vs 80-82 K proofs/s: their 1 MB of rows
  // compete in L2 with the concurrent direct-table MSMs, while this kernel's
  // 128 KB radix-16 table stays resident)
  {
    ProfScope ps(ctx, "pedersen");
    hipLaunchKernelGGL(k_pedersen, dim3(grid_for(m * PED_G, 256)), dim3(256), 0, ctx->stream, g->d_fb, d_v, d_gam, m,
                       p3);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_pedersen"));
  if (d_out_enc) {
    {
      ProfScope ps(ctx, "compress");
      hipLaunchKernelGGL(k_compress_p3, dim3(grid_for(m, 64)), dim3(64), 0, ctx->stream, (const uint32_t*)p3, m,
                         d_out_enc);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_compress_p3"));
  }
  return BPP_OK;
}

int gens_points(bpp_ctx* ctx, const bpp_gens* g, MsmPoints* out) {
  const uint32_t np = (uint32_t)(2 * g->n + 2);
  // First use builds the tables on this context's stream.  They are
  // published only after that stream has finished them (hipStreamSynchronize),
  // under the gens' lock, so a context on another stream never reads a
  // half-built table and two first users cannot both build one.
  std::lock_guard<std::mutex> lock(g->build_mu);
  if (!g->d_wt) {
    uint32_t* d = nullptr;
    if (hipMalloc(&d, (size_t)np * FBW_W * MSM_NIELS_WORDS * 4) != hipSuccess) {
      ctx->err = "hipMalloc generator window tables";
      return BPP_ERR_NOMEM;
    }
    int rc = fbw_build(ctx, g->d_tbl, np, d);
    if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) {
      ctx->err = "window-table build failed";
      rc = BPP_ERR_DEVICE;
    }
    if (rc) {
      hipFree(d);
      return rc;
    }
    g->d_wt = d;
  }
  if (!g->d_dt && np <= GENS_DT_MAX) {
    // c = 8: 16-bit windows halve the table additions but measured no
    // faster (0.94 vs 0.91 ms of direct-table time per 128-proof batch;
    // 16.5 GB of tables gathered at random)
    const uint32_t c = 8;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, dt_bytes(np, c)) != hipSuccess) {
      ctx->err = "hipMalloc generator direct tables";
      return BPP_ERR_NOMEM;
    }
    int rc = dt_build(ctx, g->d_wt, np, c, d);
    if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) {
      ctx->err = "direct-table build failed";
      rc = BPP_ERR_DEVICE;
    }
    if (rc) {
      hipFree(d);
      return rc;
    }
    g->d_dt = d;
    g->dt_c = c;
  }
  *out = MsmPoints();
  out->tbl = g->d_tbl;
  out->wt = g->d_wt;
  out->dt = g->d_dt;
  out->dt_c = g->dt_c;
  return BPP_OK;
}

void gens_chain_bytes(const char* label, uint32_t party, size_t n, uint8_t* out64) {
  merlin::Shake256 sh;
  sh.update((const uint8_t*)"GeneratorsChain", 15);
  uint8_t lab[5] = {(uint8_t)label[0], 0, 0, 0, 0};
  memcpy(lab + 1, &party, 4);
  sh.update(lab, 5);
  sh.read(out64, 64 * n);
}

extern "C" {

int bpp_gens_create(bpp_ctx* ctx, size_t n, bpp_gens** out) {
  if (!ctx || !out || n == 0 || n >= (1u << 28)) return BPP_ERR_ARG;
  *out = nullptr;
  BPP_HIP(hipSetDevice(ctx->device));
  bpp_gens* g = nullptr;
  BPP_TRY(gens_alloc(ctx, n, &g));
  // uniform bytes: G chain, H chain, then B_blinding's SHA3-512(B) (as 64 B)
  std::vector<uint8_t> uni((2 * n + 1) * 64);
  gens_chain_bytes("G", 0, n, uni.data());
  gens_chain_bytes("H", 0, n, uni.data() + 64 * n);
  static const uint8_t B_ENC[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9,
                                    0x61, 0xc5, 0x00, 0x51, 0x5f, 0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82,
                                    0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
  merlin::sha3_512(B_ENC, 32, uni.data() + 64 * 2 * n);
  void *d_uni, *d_b, *d_bad;
  int rc = ctx_ws(ctx, "gens_uni", uni.size(), &d_uni);
  if (!rc) rc = ctx_ws(ctx, "gens_b", 32, &d_b);
  if (!rc) rc = ctx_ws(ctx, "gens_bad", 8, &d_bad);
  if (rc) {
    bpp_gens_destroy(g);
    return rc;
  }
  unsigned long long init = ~0ull;
  BPP_HIP(hipMemcpyAsync(d_uni, uni.data(), uni.size(), hipMemcpyHostToDevice, ctx->stream));
  BPP_HIP(hipMemcpyAsync(d_b, B_ENC, 32, hipMemcpyHostToDevice, ctx->stream));
  BPP_HIP(hipMemcpyAsync(d_bad, &init, 8, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_from_uniform, dim3(grid_for(2 * n, 64)), dim3(64), 0, ctx->stream, (const uint32_t*)d_uni, 2 * n,
                     g->d_tbl);
  hipLaunchKernelGGL(k_from_uniform, dim3(1), dim3(64), 0, ctx->stream, (const uint32_t*)d_uni + 16 * 2 * n, (size_t)1,
                     g->d_tbl + (2 * n + 1) * MSM_NIELS_WORDS);
  hipLaunchKernelGGL(k_decompress, dim3(1), dim3(64), 0, ctx->stream, (const uint32_t*)d_b, (size_t)1,
                     g->d_tbl + 2 * n * MSM_NIELS_WORDS, (unsigned long long*)d_bad);
  rc = ctx_check_launch(ctx, "gens kernels");
  if (!rc) rc = gens_finish(ctx, g);
  if (rc) {
    bpp_gens_destroy(g);
    return rc;
  }
  *out = g;
  return BPP_OK;
}

int bpp_gens_from_points(bpp_ctx* ctx, const uint8_t* G_enc, const uint8_t* H_enc, size_t n, const uint8_t B_enc[32],
                         const uint8_t Bb_enc[32], bpp_gens** out) {
  if (!ctx || !out || !G_enc || !H_enc || !B_enc || !Bb_enc || n == 0) return BPP_ERR_ARG;
  *out = nullptr;
  BPP_HIP(hipSetDevice(ctx->device));
  bpp_gens* g = nullptr;
  BPP_TRY(gens_alloc(ctx, n, &g));
  std::vector<uint8_t> enc((2 * n + 2) * 32);
  memcpy(enc.data(), G_enc, 32 * n);
  memcpy(enc.data() + 32 * n, H_enc, 32 * n);
  memcpy(enc.data() + 64 * n, B_enc, 32);
  memcpy(enc.data() + 64 * n + 32, Bb_enc, 32);
  void *d_enc, *d_bad;
  int rc = ctx_ws(ctx, "gens_enc", enc.size(), &d_enc);
  if (!rc) rc = ctx_ws(ctx, "gens_bad", 8, &d_bad);
  if (rc) {
    bpp_gens_destroy(g);
    return rc;
  }
  unsigned long long bad = ~0ull;
  BPP_HIP(hipMemcpyAsync(d_enc, enc.data(), enc.size(), hipMemcpyHostToDevice, ctx->stream));
  BPP_HIP(hipMemcpyAsync(d_bad, &bad, 8, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_decompress, dim3(grid_for(2 * n + 2, 64)), dim3(64), 0, ctx->stream, (const uint32_t*)d_enc,
                     2 * n + 2, g->d_tbl, (unsigned long long*)d_bad);
  BPP_HIP(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, ctx->stream));
  BPP_HIP(hipStreamSynchronize(ctx->stream));
  if (bad != ~0ull) {
    ctx->err = "invalid generator encoding at index " + std::to_string(bad);
    bpp_gens_destroy(g);
    return BPP_ERR_DECOMPRESS;
  }
  rc = gens_finish(ctx, g);
  if (rc) {
    bpp_gens_destroy(g);
    return rc;
  }
  *out = g;
  return BPP_OK;
}

size_t bpp_gens_len(const bpp_gens* g) { return g ? g->n : 0; }

int bpp_gens_export(bpp_ctx* ctx, const bpp_gens* g, uint8_t* out) {
  if (!ctx || !g || !out) return BPP_ERR_ARG;
  bpp_points view;
  view.ctx = ctx;
  view.d = g->d_tbl;
  view.n = 2 * g->n + 2;
  return bpp_points_compress(ctx, &view, out);
}

void bpp_gens_destroy(bpp_gens* g) {
  if (!g) return;
  hipSetDevice(g->ctx->device);
  if (g->d_tbl) hipFree(g->d_tbl);
  if (g->d_fb) hipFree(g->d_fb);
  if (g->d_wt) hipFree(g->d_wt);
  if (g->d_dt) hipFree(g->d_dt);
  delete g;
}

int bpp_pedersen_commit_batch(bpp_ctx* ctx, const bpp_gens* g, const uint8_t* v, const uint8_t* gamma, size_t m,
                              uint8_t* out) {
  if (!ctx || !g || ((!v || !gamma || !out) && m)) return BPP_ERR_ARG;
  if (!m) return BPP_OK;
  BPP_HIP(hipSetDevice(ctx->device));
  uint32_t *d_v, *d_g;
  BPP_TRY(upload_scalars(ctx, v, m, "ped_v", &d_v));
  BPP_TRY(upload_scalars(ctx, gamma, m, "ped_g", &d_g));
  void* d_out = nullptr;
  BPP_TRY(ctx_ws(ctx, "ped_out", m * 32, &d_out));
  BPP_TRY(pedersen_dev(ctx, g, d_v, d_g, m, (uint32_t*)d_out, nullptr));
  BPP_TRY(ctx_d2h(ctx, out, d_out, m * 32));
  return BPP_OK;
}

}  // extern "C"
