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

#include <atomic>

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

// Pedersen commitments P_j = v_j * B + g_j * Bb (PedersenGens::commit,
// weights.rs:58-61), constant time in v and gamma like the reference's
// commit (a constant-time 2-term multiscalar_mul).
//
// Signed radix-16 digits in closed form: nibble i of s + K, K = 8 * sum_{i<63}
// 16^i, minus 8 is digit i (i < 63, in [-8, 8)) and nibble 63 the top digit
// (s < 2^253: at most 2) -- the digits of a carry-propagating recoding,
// without a data-dependent branch or index.  Table row (which * 64 + pos) * 8
// + |d| - 1 of fb holds |d| * 16^pos * (B, Bb)[which].
//
// The work is split by POSITION GROUP, not by commitment: block (x, g) handles
// positions [Pg, Pg + P) of both scalars (P = 64 / G) for 256 commitments, one
// commitment per lane (2P mixed additions each).  Every lane of the block
// reads the same 16P table rows, staged once in LDS (16 KB at G = 8), so each
// lookup is a broadcast LDS read; the lookup is dalek's LookupTable::select -- all eight rows of a
// position read, the one for |d| kept by masks, d = 0 keeping the Niels
// identity -- and signs are operand selects (ge_madd_signed).  Loads and
// instruction stream are independent of the digits.  The G partial sums of
// a commitment are added by k_pedersen_sum (G lanes, log2 G butterfly levels).
// G = 8 for large batches (13 312 V commitments per 128 proofs: fewest
// partials), G = 32 for small ones (latency: 4 additions per lane).
#define PED_T 256
// v_groups: position groups that can hold nonzero digits of v (G in
// general; 1 when a PUBLIC bound puts every v below 2^(4 P - 1), e.g. the V
// commitments' values 1..k and pi + 1 <= k: their digits beyond group 0 are
// all zero for every v under the bound, so skipping those groups depends on
// k only, not on the secret values -- 72 instead of 128 table additions per
// V commitment at G = 8, 66 with v_npos below).  (Spreading v's P positions one per group, so no
// group adds more than P + 1 rows, measured slower: 124 vs 117 us alone and
// 206-218 K vs 208-222 K proofs/s at 256 x 8 -- the blocks are scheduled
// dynamically, so group 0's longer blocks were not the kernel's tail.)
template <int G>
__global__ void __launch_bounds__(PED_T) k_pedersen(const uint32_t* __restrict__ fb, const uint32_t* __restrict__ v,
                                                    const uint32_t* __restrict__ gam, size_t m, uint32_t v_groups,
                                                    uint32_t v_npos, uint32_t* __restrict__ part) {
  constexpr uint32_t PED_GPOS = FB_POS / G;    // positions per group
  constexpr uint32_t PED_ROWS = 2 * PED_GPOS * 8;  // table rows one block needs
  __shared__ __attribute__((aligned(16))) uint32_t rows[PED_ROWS * MSM_NIELS_WORDS];
  const uint32_t g = blockIdx.y;
  // stage rows (which, b, d) = fb row (which * 64 + 8g + b) * 8 + d - 1
  for (uint32_t i = threadIdx.x; i < PED_ROWS * (MSM_NIELS_WORDS / 4); i += PED_T) {
    const uint32_t r = i / (MSM_NIELS_WORDS / 4), c = i % (MSM_NIELS_WORDS / 4);
    const uint32_t which = r / (PED_GPOS * 8), rem = r % (PED_GPOS * 8);
    const uint32_t src = (which * FB_POS + PED_GPOS * g) * 8 + rem;
    reinterpret_cast<uint4*>(rows)[i] = reinterpret_cast<const uint4*>(fb + (size_t)src * MSM_NIELS_WORDS)[c];
  }
  __syncthreads();
  const size_t j = (size_t)blockIdx.x * PED_T + threadIdx.x;
  if (j >= m) return;
  ge_p3 acc = ge_identity();
  _Pragma("unroll 1") for (uint32_t which = g < v_groups ? 0 : 1; which < 2; ++which) {
    // word Pg / 8 of s + K holds the nibbles of positions [Pg, Pg + P)
    const uint32_t* sp = (which ? gam : v) + 8 * j;
    const uint32_t wsel = PED_GPOS * g / 8, sh = 4 * (PED_GPOS * g % 8);
    uint64_t c = 0;
    uint32_t word = 0;
    _Pragma("unroll") for (uint32_t i = 0; i < 8; ++i) {
      c += (uint64_t)sp[i] + (i < 7 ? 0x88888888u : 0x08888888u);
      word = wsel == i ? (uint32_t)c : word;
      c >>= 32;
    }
    word >>= sh;
    // (v: only the positions the public bound can reach, v_npos <= PED_GPOS)
    const uint32_t npos = which == 0 ? v_npos : PED_GPOS;
    _Pragma("unroll 1") for (uint32_t b = 0; b < npos; ++b) {
      const int nib = (int)((word >> (4 * b)) & 15u);
      const int d = PED_GPOS * g + b < FB_POS - 1 ? nib - 8 : nib;
      const int sg = d >> 31;  // 0 or -1
      const uint32_t ad = (uint32_t)((d ^ sg) - sg);
      const uint32_t r0 = (which * PED_GPOS + b) * 8;
      ge_niels t = ge_niels_identity();
      _Pragma("unroll 2") for (uint32_t k = 1; k <= 8; ++k) {
        const ge_niels e = load_niels(rows, r0 + k - 1);
        const bool hit = ad == k;
        _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
          t.ypx.v[i] = hit ? e.ypx.v[i] : t.ypx.v[i];
          t.ymx.v[i] = hit ? e.ymx.v[i] : t.ymx.v[i];
          t.xy2d.v[i] = hit ? e.xy2d.v[i] : t.xy2d.v[i];
        }
      }
      acc = ge_madd_signed(acc, t, sg != 0);
    }
  }
  store_p3(part, (size_t)g * m + j, acc);
}

// P_j = sum of its G partials: G lanes per commitment, log2 G levels.
template <int G>
__global__ void __launch_bounds__(256) k_pedersen_sum(const uint32_t* __restrict__ part, size_t m,
                                                      uint32_t* __restrict__ out_p3) {
  const size_t gt = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t j = gt / G;
  const uint32_t q = (uint32_t)(gt % G);
  ge_p3 acc = j < m ? load_p3(part, (size_t)q * m + j) : ge_identity();
  _Pragma("unroll") for (int off = 1; off < G; off <<= 1) {
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
  if (hipMalloc(&g->d_tbl, (2 * n + 3) * MSM_NIELS_WORDS * 4) != hipSuccess ||  // (+1: the Q slot, gens.h)
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
                 uint32_t* d_out_enc, uint32_t* d_out_p3, uint64_t v_bound) {
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
  const uint32_t G = m <= 2048 ? 32 : 8;
  // group 0 (P = FB_POS / G nibble positions) carries every v of the bound
  // when v + 8 (16^P - 1) / 15 (the recoding offset K's low P nibbles) does
  // not carry out of it: v < (7 16^P + 8) / 15 (2004318072 at P = 8, 120 at
  // P = 2); nibble 63's top digit never sits in group 0
  const uint32_t PG = FB_POS / G;
  const uint64_t v_lim = PG < 16 ? (7 * (1ull << (4 * PG)) + 8) / 15 : 0;
  const uint32_t v_groups = v_bound && v_bound <= v_lim ? 1u : G;
  // and within group 0 only the first v_npos positions: the least P' with
  // v_bound < (7 16^P' + 8) / 15 (e.g. 2 for the 52-card values <= 53,
  // 8 + 2 instead of 8 + 8 additions for v; still fixed by k alone)
  uint32_t v_npos = PG;
  if (v_groups == 1)
    for (uint32_t q = 1; q < PG; ++q)
      if (v_bound <= (7 * (1ull << (4 * q)) + 8) / 15) {
        v_npos = q;
        break;
      }
  ctx_work(ctx, "msm_terms", 2 * (uint64_t)m);
  // constant time: every position of gamma, every possible position of v
  ctx_work(ctx, "madds", (uint64_t)(FB_POS + (v_groups == 1 ? v_npos : FB_POS)) * m);
  ctx_work(ctx, "padds", (uint64_t)(G - 1) * m);
  ctx_work(ctx, "msm_launches", 1);
  void* part = nullptr;
  BPP_TRY(ctx_ws(ctx, "ped_part", m * G * P3_BYTES, &part));
  {
    ProfScope ps(ctx, "pedersen");
    if (G == 32) {
      hipLaunchKernelGGL(k_pedersen<32>, dim3(grid_for(m, PED_T), 32), dim3(PED_T), 0, ctx->stream, g->d_fb, d_v,
                         d_gam, m, v_groups, v_npos, (uint32_t*)part);
      hipLaunchKernelGGL(k_pedersen_sum<32>, dim3(grid_for(m * 32, 256)), dim3(256), 0, ctx->stream,
                         (const uint32_t*)part, m, p3);
    } else {
      hipLaunchKernelGGL(k_pedersen<8>, dim3(grid_for(m, PED_T), 8), dim3(PED_T), 0, ctx->stream, g->d_fb, d_v,
                         d_gam, m, v_groups, v_npos, (uint32_t*)part);
      hipLaunchKernelGGL(k_pedersen_sum<8>, dim3(grid_for(m * 8, 256)), dim3(256), 0, ctx->stream,
                         (const uint32_t*)part, m, p3);
    }
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

static std::atomic<size_t> g_dt_total{0};  // direct-table bytes of the live generator sets

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
    // The widest window (fewest table additions per term: W = ceil(254 / c))
    // whose tables fit GENS_DT_BUDGET: c = 13 (W = 20, 2.7 GB) for the
    // 258 generators of a 52-card proof, against W = 32 at c = 8.  Measured
    // in isolation (tools/ubench/dtbench, 8 batches' IPA rounds in one
    // launch): 446 / 376 / 337 / 312 / 294 us at c = 8 / 11 / 12 / 13 / 16.
    // (and within what the process's other live generator sets leave of
    // GENS_DT_TOTAL, so many sets -- tests, one per context -- fall back to
    // narrower tables instead of exhausting HBM)
    const size_t used = g_dt_total.load();
    const size_t budget = std::min<size_t>(GENS_DT_BUDGET, used < GENS_DT_TOTAL ? GENS_DT_TOTAL - used : 0);
    // (np + 1 generator slots: the last is bpp_ipa_prove's Q, gens.h)
    uint32_t c = 8;
    while (c < GENS_DT_CMAX && dt_bytes(np + 1, c + 1) <= budget) ++c;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, dt_bytes(np + 1, c)) != hipSuccess) {
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
    g_dt_total += dt_bytes(np + 1, c);
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
  return bpp_guard(ctx, [&]() -> int {
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
  });
}

int bpp_gens_from_points(bpp_ctx* ctx, const uint8_t* G_enc, const uint8_t* H_enc, size_t n, const uint8_t B_enc[32],
                         const uint8_t Bb_enc[32], bpp_gens** out) {
  return bpp_guard(ctx, [&]() -> int {
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
  });
}

size_t bpp_gens_len(const bpp_gens* g) { return g ? g->n : 0; }

int bpp_gens_export(bpp_ctx* ctx, const bpp_gens* g, uint8_t* out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !g || !out) return BPP_ERR_ARG;
    bpp_points view;
    view.ctx = ctx;
    view.d = g->d_tbl;
    view.n = 2 * g->n + 2;
    return bpp_points_compress(ctx, &view, out);
  });
}

void bpp_gens_destroy(bpp_gens* g) {
  if (!g) return;
  hipSetDevice(g->ctx->device);
  if (g->d_tbl) hipFree(g->d_tbl);
  if (g->d_fb) hipFree(g->d_fb);
  if (g->d_wt) hipFree(g->d_wt);
  if (g->d_dt) {
    hipFree(g->d_dt);
    g_dt_total -= dt_bytes((uint32_t)(2 * g->n + 3), g->dt_c);
  }
  delete g;
}

int bpp_pedersen_commit_batch(bpp_ctx* ctx, const bpp_gens* g, const uint8_t* v, const uint8_t* gamma, size_t m,
                              uint8_t* out) {
  return bpp_guard(ctx, [&]() -> int {
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
  });
}

}  // extern "C"
