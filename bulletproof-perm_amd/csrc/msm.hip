// MSM engine (host orchestration of msm_kernels.cuh) and its C-ABI entry
// points: bpp_msm, bpp_msm_table, bpp_msm_table_dev, bpp_msm_batch and the
// window-partitioned variants used for multi-GPU.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ctx.h"
#include "host/fe64.h"
#include "host/par.h"
#include "msm_kernels.cuh"
#include "msm_engine.h"

// Scalar field order l, little-endian 32-bit words.
static const uint32_t L_WORDS[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                                    0x00000000u, 0x00000000u, 0x00000000u, 0x10000000u};

bool scalar_is_canonical(const uint8_t* s) {
  uint32_t w[8];
  memcpy(w, s, 32);
  for (int i = 7; i >= 0; --i) {
    if (w[i] < L_WORDS[i]) return true;
    if (w[i] > L_WORDS[i]) return false;
  }
  return false;  // == l
}

uint32_t msm_choose_c(double n_per_msm) {
  static const int c_env = [] {  // (A/B runs: one window size for every MSM)
    const char* e = getenv("BPP_MSM_C");
    return e ? atoi(e) : 0;
  }();
  if (c_env >= 2 && c_env <= 16) return (uint32_t)c_env;
  uint32_t best = 4;
  double bestc = 1e300;
  // c <= 16: a window's bucket histogram (2^(c-1) x 4 B) fits in LDS
  // (128 KB at c = 16, which also gives W = 16 windows: an even split over
  // 1, 2, 4 and 8 GPUs).
  for (uint32_t c = 2; c <= 16; ++c) {
    const uint32_t W = (254 + c - 1) / c;
    const double cost = (double)W * (7.0 * n_per_msm + 9.0 * (double)(1u << c)) + 8.0 * c * (W - 1);
    if (cost < bestc) {
      bestc = cost;
      best = c;
    }
  }
  return best;
}

static unsigned grid_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// MSM offsets to the "multi_off" workspace, skipped when it already holds
// exactly these (same stream, nothing else writes it; ctx.h off_cache)
static int upload_offsets(bpp_ctx* ctx, const std::vector<uint32_t>& off, void** d_off) {
  BPP_TRY(ctx_ws(ctx, "multi_off", off.size() * 4, d_off));
  if (*d_off != ctx->off_cache_ptr || off != ctx->off_cache) {
    BPP_TRY(ctx_h2d(ctx, *d_off, off.data(), off.size() * 4));
    ctx->off_cache_ptr = *d_off;
    ctx->off_cache = off;
  }
  return BPP_OK;
}

int msm_engine(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const uint32_t* d_off, uint32_t M,
               uint32_t T, uint32_t c, uint32_t wb, uint32_t Wn, const uint32_t* d_tbl, uint32_t** d_wsum_out,
               const uint32_t* d_tbl1, uint32_t n0, bool fb, uint32_t* terms_out, uint32_t rlog,
               uint32_t* rshift_out) {
  if (terms_out) *terms_out = 1;
  if (rshift_out) *rshift_out = rlog + 6;
  MsmGeom g;
  g.M = M;
  g.T = T;
  g.c = c;
  g.W = (254 + c - 1) / c;
  g.wb = wb;
  g.Wn = Wn;
  g.B = 1u << (c - 1);
  g.fb = fb ? 1u : 0u;
  {
    // radix sort: the top window holds 253 - c (W - 1) bits (canonical
    // scalars < l < 2^253), i.e. buckets < 2^top; spread them over all
    // NC = B / 2^RS_FINE_BITS coarse bins (rs_fbits)
    const int top = 253 - (int)(c * (g.W - 1)), lognc = (int)c - 1 - RS_FINE_BITS;
    g.tfb = (top >= (int)c - 1 || lognc < 0) ? RS_FINE_BITS : (uint32_t)std::max(0, top - lognc);
    for (int i = 0; i < 8; ++i) g.K[i] = 0;
    for (uint32_t w = 0; w + 1 < g.W; ++w) {  // bit c w + c - 1 (< 256)
      const uint32_t pos = c * w + c - 1;
      g.K[pos >> 5] |= 1u << (pos & 31);
    }
  }
  const size_t nseg = fb ? (size_t)M : (size_t)M * Wn;
  const size_t NB = nseg * g.B;
  ctx_work(ctx, "msm_terms", T);
  ctx_work(ctx, "madds", (uint64_t)T * Wn);
  ctx_work(ctx, "padds", (uint64_t)2 * NB);  // running sums of the bucket reduction
  ctx_work(ctx, "msm_launches", 1);
  void *cnt, *cur, *boff, *entries, *bsum, *wsum;
  BPP_TRY(ctx_ws(ctx, "msm_cnt", (NB + 1) * 4, &cnt));
  BPP_TRY(ctx_ws(ctx, "msm_cur", NB * 4, &cur));
  BPP_TRY(ctx_ws(ctx, "msm_boff", (NB + 1) * 4, &boff));
  BPP_TRY(ctx_ws(ctx, "msm_entries", (size_t)T * Wn * 4 + 48, &entries));  // +48: 16-B reads (and the next group's) past the end
  BPP_TRY(ctx_ws(ctx, "msm_bsum", NB * P3_BYTES, &bsum));
  BPP_TRY(ctx_ws(ctx, "msm_wsum", nseg * P3_BYTES, &wsum));
  // (tmpA packs the point index in 24 bits)
  const bool radix_sort = !fb && (M == 1) && (c >= 12) && (c <= 16) && (T >= 16384) && (T <= (1u << 24)) &&
                          (!d_pidx) && (size_t)Wn * (g.B >> RS_FINE_BITS) <= RS_DC_HMAX &&
                          !getenv("BPP_MSM_LDS_SORT");
  const bool lds_sort = !fb && !radix_sort && (M == 1) && (c <= 16) && (T >= 16384);
  // entries per lane: enough lanes to fill the chip several times over
  const uint32_t E_max = T * Wn;
  // K = entries per lane (a multiple of 4, for the 16-B entry reads): at most
  // one round of lanes at the accumulate's occupancy (4 workgroups of 256
  // lanes per CU, LDS-bound: 256 K lanes on 256 CUs), since every lane does
  // the same K additions and a partial second round of waves runs after the
  // first as a tail (config 5's 8.85 M entries: K = 32 gave 4320 waves,
  // 224 past the round; K = 36 gives 3841).  Fewer chunk borders also mean
  // fewer head/tail pieces (2^20: K = 64 measured best of 32/64/128).
  static const size_t round_lanes = [] {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    return (size_t)std::max(1, ncu) * 4 * ACC_T;
  }();
  uint32_t K = (uint32_t)std::min<size_t>(128, std::max<size_t>(4, ((E_max + round_lanes - 1) / round_lanes + 3) & ~(size_t)3));
  // an MSM alone on the device (the lone reduction shape) with K >= 32 takes
  // K >= 48: fewer buckets cross lane borders, so its latency-bound reduction
  // assembles fewer pieces (config 5, K 36 -> 48, three interleaved passes:
  // reduce 0.216-0.218 -> 0.194-0.195 ms, accumulate 0.399 -> 0.394-0.398;
  // profiles/r04_verify_k_ab.txt)
  if (rlog == RWAVE_LOG_LONE && K >= 32) K = std::max<uint32_t>(K, 48);
  // ... and K >= 16 in any case: a window range of a large MSM (the window
  // split's partial: config 5 over 8 GPUs is 2 windows x 520 K terms, K = 4
  // by the round rule) otherwise spends its time closing buckets and joining
  // lane pieces (tools/shard_model.py, rank 0's partial: 0.857 ms at K = 4,
  // 0.377 at 16, 0.393 at 32, 0.431 at 48; 4 windows: 0.502 at K = 8, 0.421 at
  // 16, 0.405 at 32; profiles/r05_partial_k_ab.txt)
  if (rlog == RWAVE_LOG_LONE) K = std::max<uint32_t>(K, 16);
  if (const char* ek = getenv("BPP_MSM_ACC_K")) K = (uint32_t)std::min(128, std::max(4, atoi(ek) & ~3));  // A/B runs
  const size_t lanes = (E_max + K - 1) / K + 1;
  // a heavy bucket spans > FIX_MAX chunks, so holds > (FIX_MAX - 1) K
  // entries: at most E / ((FIX_MAX - 1) K) + 1 of them
  const size_t max_heavy = std::min<size_t>(NB, E_max / ((size_t)(FIX_MAX - 1) * K) + 1);
  void *head, *tail, *heavy;
  BPP_TRY(ctx_ws(ctx, "msm_head", lanes * P3_BYTES, &head));
  BPP_TRY(ctx_ws(ctx, "msm_tail", lanes * P3_BYTES, &tail));
  BPP_TRY(ctx_ws(ctx, "msm_heavy", (max_heavy + 1) * 4, &heavy));
  if (!radix_sort) {
    BPP_HIP(hipMemsetAsync(cnt, 0, (NB + 1) * 4, ctx->stream));
    BPP_HIP(hipMemsetAsync(cur, 0, NB * 4, ctx->stream));
  }
  if (radix_sort) {
    void *dig, *cntA, *offA, *tmpA;
    BPP_TRY(ctx_ws(ctx, "msm_dig", (size_t)T * Wn * sizeof(dig_t) + 16, &dig));
    const uint32_t nchunk = (T + RS_CHUNK - 1) / RS_CHUNK;
    const uint32_t NC = g.B >> RS_FINE_BITS;  // <= 256 coarse bins per window
    const size_t nA = (size_t)Wn * NC * nchunk;
    BPP_TRY(ctx_ws(ctx, "msm_cntA", (nA + 1) * 4, &cntA));
    BPP_TRY(ctx_ws(ctx, "msm_offA", (nA + 1) * 4, &offA));
    BPP_TRY(ctx_ws(ctx, "msm_tmpA", (size_t)T * Wn * 4 + 16, &tmpA));
    {
      ProfScope ps(ctx, "msm_digits");  // digits + coarse counts
      hipLaunchKernelGGL(k_rsort_digits_count, dim3(nchunk), dim3(RS_DC_T), 0, ctx->stream, d_scal, g, nchunk, NC,
                         (dig_t*)dig, (uint32_t*)cntA, (uint32_t*)cntA + nA, (uint32_t*)heavy);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_rsort_digits_count"));
    {
      ProfScope ps(ctx, "msm_scan");
      BPP_TRY(scan_exclusive_u32(ctx, (const uint32_t*)cntA, (uint32_t*)offA, nA + 1));
    }
    {
      ProfScope ps(ctx, "msm_scatter");
      hipLaunchKernelGGL(k_rsort_scatter, dim3(Wn * nchunk), dim3(RS_T), 0, ctx->stream, (const dig_t*)dig, d_pidx,
                         g, nchunk, NC, (const uint32_t*)offA, (uint32_t*)tmpA);
      hipLaunchKernelGGL(k_rsort_fine, dim3(Wn * NC), dim3(RS_FT), 0, ctx->stream, (const uint32_t*)tmpA, nchunk,
                         (const uint32_t*)offA, (uint32_t*)boff, (uint32_t*)entries, (uint32_t*)boff + NB,
                         (const uint32_t*)offA + nA, g, NC);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_rsort_scatter/fine"));
  } else if (lds_sort && T) {
    void* dig = nullptr;
    BPP_TRY(ctx_ws(ctx, "msm_dig", (size_t)T * Wn * sizeof(dig_t) + 16, &dig));
    {
      ProfScope ps(ctx, "msm_digits");
      hipLaunchKernelGGL(k_msm_digits, dim3(grid_for(T, 256)), dim3(256), 0, ctx->stream, d_scal, g, (dig_t*)dig);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_msm_digits"));
    // ~2 blocks per CU in total
    uint32_t nchunk = std::max<uint32_t>(1, (512 + Wn - 1) / Wn);
    nchunk = std::min<uint32_t>(nchunk, std::max<uint32_t>(1, T / 4096));
    const uint32_t chunk = (T + nchunk - 1) / nchunk;
    const size_t lds = (size_t)g.B * 4;
    static bool lds_attr = false;
    if (!lds_attr) {  // > 64 KB dynamic LDS (128 KB at c = 16; 160 KB per CU on gfx950)
      BPP_HIP(hipFuncSetAttribute((const void*)k_msm_count_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
      BPP_HIP(hipFuncSetAttribute((const void*)k_msm_scatter_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
      lds_attr = true;
    }
    {
      ProfScope ps(ctx, "msm_count");
      hipLaunchKernelGGL(k_msm_count_lds, dim3(Wn * nchunk), dim3(SORT_T), lds, ctx->stream, (const dig_t*)dig, g,
                         chunk, nchunk, (uint32_t*)cnt);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_msm_count_lds"));
    {
      ProfScope ps(ctx, "msm_scan");
      BPP_TRY(scan_exclusive_u32(ctx, (const uint32_t*)cnt, (uint32_t*)boff, NB + 1));
    }
    {
      ProfScope ps(ctx, "msm_scatter");
      hipLaunchKernelGGL(k_msm_scatter_lds, dim3(Wn * nchunk), dim3(SORT_T), lds, ctx->stream, (const dig_t*)dig,
                         d_pidx, g, chunk, nchunk, (const uint32_t*)boff, (uint32_t*)cur, (uint32_t*)entries);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_msm_scatter_lds"));
  } else {
    if (T) {
      ProfScope ps(ctx, "msm_count");
      hipLaunchKernelGGL(k_msm_count, dim3(grid_for(T, 256)), dim3(256), 0, ctx->stream, d_scal, d_off, g,
                         (uint32_t*)cnt);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_msm_count"));
    {
      ProfScope ps(ctx, "msm_scan");
      BPP_TRY(scan_exclusive_u32(ctx, (const uint32_t*)cnt, (uint32_t*)boff, NB + 1));
    }
    if (T) {
      ProfScope ps(ctx, "msm_scatter");
      hipLaunchKernelGGL(k_msm_scatter, dim3(grid_for(T, 256)), dim3(256), 0, ctx->stream, d_scal, d_off, d_pidx, g,
                         (const uint32_t*)boff, (uint32_t*)cur, (uint32_t*)entries);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_msm_scatter"));
  }
  {
    if (!radix_sort) BPP_HIP(hipMemsetAsync(heavy, 0, 4, ctx->stream));  // (radix: cleared by its first kernel)
    {
      ProfScope ps(ctx, "msm_accumulate");
      hipLaunchKernelGGL(k_msm_accumulate, dim3(grid_for(lanes, ACC_T)), dim3(ACC_T), ctx->acc_lds_pad, ctx->stream,
                         d_tbl, d_tbl1,
                         n0, (const uint32_t*)entries, (const uint32_t*)boff, (uint32_t)NB, K, (uint32_t*)bsum,
                         (uint32_t*)head, (uint32_t*)tail, (uint32_t*)heavy);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_msm_accumulate"));
    {
      ProfScope ps(ctx, "msm_fixup");
      hipLaunchKernelGGL(k_msm_fixup_heavy, dim3((unsigned)std::min<size_t>(max_heavy, 4096)), dim3(64), 0, ctx->stream,
                         (const uint32_t*)boff, K, (const uint32_t*)head, (const uint32_t*)tail,
                         (const uint32_t*)heavy, (uint32_t*)bsum);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_msm_fixup_heavy"));
    if (rlog != RWAVE_LOG && rlog != RWAVE_LOG_LONE) rlog = RWAVE_LOG;
    uint32_t rl = rlog;
    if (rlog == RWAVE_LOG_LONE) {
      // an MSM alone: 2^rl buckets a lane with rl <= RWAVE_LOG_LONE, as few as
      // keep >= 512 waves in flight (a window range of the split verifier
      // MSM, 2 x 2^14 buckets, ran k_msm_reduce_wave<3> on 64 waves: 124 us
      // of latency chain, tools/shard_model.py) and nw <= RWAVE_NW_MAX
      while (rl > 0 && (((size_t)nseg * g.B) >> (6 + rl)) < 512 && (g.B >> (6 + rl - 1)) <= RWAVE_NW_MAX) --rl;
    }
    const uint32_t rshift = rl + 6;
    if (terms_out && M == 1 && !fb && g.B >= (1u << rshift) && g.B <= ((uint32_t)RWAVE_NW_MAX << rshift)) {
      // power-of-two weights left to the host Horner (k_msm_reduce_wave)
      const uint32_t nw = g.B >> rshift;
      uint32_t J = 0;
      while ((1u << J) < nw) ++J;
      void* part = nullptr;
      BPP_TRY(ctx_ws(ctx, "msm_rpart", nseg * nw * 2 * P3_BYTES, &part));
      BPP_TRY(ctx_ws(ctx, "msm_wsum_terms", nseg * (1 + J) * P3_BYTES, &wsum));
      ProfScope ps(ctx, "msm_reduce");
#ifndef EXP_NO_REDUCE  // (timing experiment only: results are wrong without it)
      if (rlog == RWAVE_LOG) {
        hipLaunchKernelGGL(k_msm_reduce_wave<RWAVE_LOG>, dim3((unsigned)(nseg * nw)), dim3(64), 0, ctx->stream,
                           (const uint32_t*)boff, K, (const uint32_t*)head, (const uint32_t*)tail,
                           (const uint32_t*)bsum, g, (uint32_t*)part);
        hipLaunchKernelGGL(k_msm_reduce_bits<RWAVE_LOG>, dim3((unsigned)(nseg * (1 + J))), dim3(64), 0, ctx->stream,
                           (const uint32_t*)part, g, 1 + J, (uint32_t*)wsum);
      } else {
        auto launch = [&](auto kw, auto kb) {
          hipLaunchKernelGGL(kw, dim3((unsigned)(nseg * nw)), dim3(64), 0, ctx->stream, (const uint32_t*)boff, K,
                             (const uint32_t*)head, (const uint32_t*)tail, (const uint32_t*)bsum, g, (uint32_t*)part);
          hipLaunchKernelGGL(kb, dim3((unsigned)(nseg * (1 + J))), dim3(64), 0, ctx->stream, (const uint32_t*)part, g,
                             1 + J, (uint32_t*)wsum);
        };
        static_assert(RWAVE_LOG_LONE == 3, "lone reduce shapes 0..3");
        switch (rl) {
          case 0: launch(k_msm_reduce_wave<0>, k_msm_reduce_bits<0>); break;
          case 1: launch(k_msm_reduce_wave<1>, k_msm_reduce_bits<1>); break;
          case 2: launch(k_msm_reduce_wave<2>, k_msm_reduce_bits<2>); break;
          default: launch(k_msm_reduce_wave<3>, k_msm_reduce_bits<3>); break;
        }
      }
#endif
      BPP_TRY(ctx_check_launch(ctx, "k_msm_reduce_wave/bits"));
      *terms_out = 1 + J;
      if (rshift_out) *rshift_out = rshift;
      *d_wsum_out = (uint32_t*)wsum;
      return BPP_OK;
    }
    const uint32_t L = g.B >= 512 ? 8 : (g.B >= 64 ? 4 : (g.B >= 8 ? 2 : 1));  // <= RED_LMAX
    const uint32_t BPS = (g.B + RED_T * L - 1) / (RED_T * L);
    void* part = wsum;  // one block per segment: its partial is the sum
    if (BPS > 1) BPP_TRY(ctx_ws(ctx, "msm_rpart", nseg * BPS * P3_BYTES, &part));
    ProfScope ps(ctx, "msm_reduce");
    hipLaunchKernelGGL(k_msm_reduce_partial, dim3((unsigned)(nseg * BPS)), dim3(RED_T), 0, ctx->stream,
                       (const uint32_t*)boff, K, (const uint32_t*)head, (const uint32_t*)tail, (const uint32_t*)bsum,
                       g, L, BPS, (uint32_t*)part);
    if (BPS > 1)
      hipLaunchKernelGGL(k_msm_reduce_final, dim3((unsigned)nseg), dim3(RED_T), 0, ctx->stream,
                         (const uint32_t*)part, BPS, (uint32_t*)wsum);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_msm_reduce"));
  *d_wsum_out = (uint32_t*)wsum;
  return BPP_OK;
}

// Window j = term 0 + sum_k 2^(rshift + k) term 1+k: one Horner pass
// over all terms in descending bit position (the term offsets < c fall
// between the doublings the window combine does anyway).
h25519::ge horner_host_terms(const uint32_t* ws_words, uint32_t Wn, uint32_t nterms, uint32_t c, uint32_t wb,
                             uint32_t rshift) {
  using namespace h25519;
  ge acc = ge_identity();
  bool started = false;
  uint32_t pos = 0;  // bit position acc is currently scaled to
  for (int j = (int)Wn - 1; j >= 0; --j) {
    for (int k = (int)nterms - 1; k >= 0; --k) {
      const uint32_t off = c * (uint32_t)j + (k ? rshift + (uint32_t)(k - 1) : 0u);
      const ge v = ge_from_dev(ws_words + ((size_t)j * nterms + (size_t)k) * P3_WORDS);
      if (started)
        for (; pos > off; --pos) acc = ge_dbl(acc);
      acc = started ? ge_add(acc, v) : v;
      started = true;
      pos = off;
    }
  }
  for (uint32_t k = 0; k < pos + c * wb; ++k) acc = ge_dbl(acc);
  return acc;
}

// Single MSM over device scalars + resident table(s), windows [wb, wb+Wn).
// Point index i < n0 reads d_tbl[i], otherwise d_tbl1[i - n0].
int msm_single_dev(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const uint32_t* d_tbl, size_t n,
                   uint32_t c, uint32_t wb, uint32_t Wn, h25519::ge* out, const uint32_t* d_tbl1, uint32_t n0) {
  if (n == 0 || Wn == 0) {
    *out = h25519::ge_identity();
    return BPP_OK;
  }
  // (window groups pipelined over two child streams measured slower: G = 2
  // 1.38 ms, G = 4 1.70 ms vs 1.26 ms at 2^20 -- the reduce and fixup are
  // latency-bound and would run G times)
  // alone on the device: the latency-shaped bucket reduction (RWAVE_LOG_LONE;
  // BPP_MSM_LONE_RLOG=4 selects the stream shape, for A/B runs)
  static const uint32_t rlog = [] {
    const char* e = getenv("BPP_MSM_LONE_RLOG");
    return (e && atoi(e) == RWAVE_LOG) ? (uint32_t)RWAVE_LOG : (uint32_t)RWAVE_LOG_LONE;
  }();
  uint32_t* d_ws = nullptr;
  uint32_t nterms = 1, rshift = rlog + 6;
  BPP_TRY(msm_engine(ctx, d_scal, d_pidx, nullptr, 1, (uint32_t)n, c, wb, Wn, d_tbl, &d_ws, d_tbl1, n0, false,
                     &nterms, rlog, &rshift));
  void* h = nullptr;
  BPP_TRY(ctx_pinned(ctx, (size_t)Wn * nterms * P3_BYTES, &h));
  BPP_HIP(hipMemcpyAsync(h, d_ws, (size_t)Wn * nterms * P3_BYTES, hipMemcpyDeviceToHost, ctx->stream));
  BPP_TRY(ctx_sync_latency(ctx));
  *out = horner_host_terms((const uint32_t*)h, Wn, nterms, c, wb, rshift);
  return BPP_OK;
}

// Host scalars -> device d on ctx's stream: staged into ctx's pinned arena by
// the pool in pieces of 2^17 scalars (4 MB; BPP_UP_PIECE_SC overrides, for
// A/B), each piece checked for canonical scalars while it is in cache (when
// `check`) and its DMA queued as soon as it is staged, so the copy engine
// moves piece k while the pool stages piece k + 1.  Returns the index of the
// first non-canonical scalar, or n.  (2^20 one at a time: one serial check
// pass, a parallel copy and then the whole DMA took ~1.7 ms before the MSM.)
static int upload_pieces(bpp_ctx* ctx, void* d, const uint8_t* scalars, size_t n, bool check, size_t* bad_out) {
  static const size_t PIECE = [] {
    const char* e = getenv("BPP_UP_PIECE_SC");
    const long v = e ? atol(e) : 0;
    return v > 0 ? ((size_t)v + 4095) & ~(size_t)4095 : (size_t)1 << 17;
  }();
  constexpr size_t SUB = 4096;  // scalars per pool task
  *bad_out = n;
  if (!n) return BPP_OK;
  uint8_t* p = nullptr;
  BPP_TRY(ctx_h2d_stage(ctx, n * 32, &p));
  std::atomic<size_t> bad{n};
  for (size_t p0 = 0; p0 < n; p0 += PIECE) {
    const size_t pn = std::min(PIECE, n - p0);
    par::for_each((pn + SUB - 1) / SUB, [&](size_t t) {
      const size_t i0 = p0 + t * SUB, i1 = std::min(i0 + SUB, p0 + pn);
      memcpy(p + 32 * i0, scalars + 32 * i0, 32 * (i1 - i0));
      if (check)
        for (size_t i = i0; i < i1; ++i)
          if (!scalar_is_canonical(p + 32 * i)) {
            size_t cur = bad.load();
            while (i < cur && !bad.compare_exchange_weak(cur, i)) {
            }
            break;
          }
    });
    BPP_TRY(ctx_h2d_staged(ctx, (uint8_t*)d + 32 * p0, p + 32 * p0, 32 * pn));
  }
  *bad_out = bad.load();
  return BPP_OK;
}

// Host scalars -> workspace `name`; a non-canonical scalar fails the call
// (after the queued copies, which only touch the workspace) with its index.
int upload_scalars(bpp_ctx* ctx, const uint8_t* scalars, size_t n, const char* name, uint32_t** d_out) {
  void* d = nullptr;
  BPP_TRY(ctx_ws(ctx, name, n * 32 + 32, &d));
  size_t bad = n;
  BPP_TRY(upload_pieces(ctx, d, scalars, n, true, &bad));
  if (bad < n) {
    ctx->err = "non-canonical scalar at index " + std::to_string(bad);
    return BPP_ERR_NONCANONICAL;
  }
  *d_out = (uint32_t*)d;
  return BPP_OK;
}

extern "C" {

int bpp_msm_windows(size_t n, uint32_t* c, uint32_t* windows) {
  return bpp_guard(nullptr, [&]() -> int {
    uint32_t cc = msm_choose_c((double)(n ? n : 1));
    if (c) *c = cc;
    if (windows) *windows = (254 + cc - 1) / cc;
    return BPP_OK;
  });
}

int bpp_msm_table_dev(bpp_ctx* ctx, const void* d_scalars, const bpp_points* tbl, size_t n, uint8_t out[32]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !tbl || !out || (!d_scalars && n)) return BPP_ERR_ARG;
    if (n > tbl->n || n >= 0x80000000ull) return BPP_ERR_LEN;
    BPP_HIP(hipSetDevice(ctx->device));
    const uint32_t c = msm_choose_c((double)n);
    const uint32_t W = (254 + c - 1) / c;
    h25519::ge r;
    BPP_TRY(msm_single_dev(ctx, (const uint32_t*)d_scalars, nullptr, tbl->d, n, c, 0, W, &r));
    h25519::encode(out, r);
    return BPP_OK;
  });
}

int bpp_msm_table_dev_partial(bpp_ctx* ctx, const void* d_scalars, const bpp_points* tbl, size_t n, uint32_t w_begin,
                              uint32_t w_end, uint8_t partial[128]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !tbl || !partial || (!d_scalars && n)) return BPP_ERR_ARG;
    if (n > tbl->n || n >= 0x80000000ull) return BPP_ERR_LEN;
    const uint32_t c = msm_choose_c((double)n);
    const uint32_t W = (254 + c - 1) / c;
    if (w_begin > w_end || w_end > W) return BPP_ERR_ARG;
    BPP_HIP(hipSetDevice(ctx->device));
    h25519::ge r;
    BPP_TRY(msm_single_dev(ctx, (const uint32_t*)d_scalars, nullptr, tbl->d, n, c, w_begin, w_end - w_begin, &r));
    h25519::ge_to_words((uint32_t*)partial, r);
    return BPP_OK;
  });
}

static int msm_submit(bpp_ctx* ctx, const void* d_scalars, const void* h_scalars, const bpp_points* tbl, size_t n,
                      uint32_t w_begin, uint32_t w_end, uint64_t* ticket);

int bpp_msm_submit(bpp_ctx* ctx, const void* d_scalars, const bpp_points* tbl, size_t n, uint32_t w_begin,
                   uint32_t w_end, uint64_t* ticket) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !tbl || !ticket || (!d_scalars && n)) return BPP_ERR_ARG;
    return msm_submit(ctx, d_scalars, nullptr, tbl, n, w_begin, w_end, ticket);
  });
}

int bpp_msm_submit_host(bpp_ctx* ctx, const void* h_scalars, const bpp_points* tbl, size_t n, uint32_t w_begin,
                        uint32_t w_end, uint64_t* ticket) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !tbl || !ticket || (!h_scalars && n)) return BPP_ERR_ARG;
    return msm_submit(ctx, nullptr, h_scalars, tbl, n, w_begin, w_end, ticket);
  });
}

int bpp_host_alloc(bpp_ctx* ctx, size_t bytes, void** hptr) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !hptr) return BPP_ERR_ARG;
    BPP_HIP(hipSetDevice(ctx->device));
    BPP_HIP(hipHostMalloc(hptr, bytes ? bytes : 1));
    host_pinned_add(*hptr, bytes ? bytes : 1);
    return BPP_OK;
  });
}

int bpp_host_free(bpp_ctx* ctx, void* hptr) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx) return BPP_ERR_ARG;
    host_pinned_remove(hptr);
    BPP_HIP(hipHostFree(hptr));
    return BPP_OK;
  });
}

// d_scalars (device) or h_scalars (host: copied on the slot's stream, so the
// upload of MSM i+1 overlaps MSM i's kernels; a direct DMA from pinned
// memory, through the slot's staging arena from pageable memory)
static int msm_submit(bpp_ctx* ctx, const void* d_scalars, const void* h_scalars, const bpp_points* tbl, size_t n,
                      uint32_t w_begin, uint32_t w_end, uint64_t* ticket) {
  if (n > tbl->n || n >= 0x80000000ull) return BPP_ERR_LEN;
  const uint32_t c = msm_choose_c((double)(n ? n : 1));
  const uint32_t W = (254 + c - 1) / c;
  if (w_end == 0) w_end = W;
  if (w_begin > w_end || w_end > W) return BPP_ERR_ARG;
  const uint64_t t = ctx->msm_next_ticket;
  // lowest free slot: k MSMs kept in flight reuse the same k child contexts
  // (and their warm workspaces)
  size_t s = BPP_MSM_INFLIGHT;
  for (size_t i = BPP_MSM_INFLIGHT; i-- > 0;)
    if (!ctx->msm_slot[i].busy) s = i;
  if (s == BPP_MSM_INFLIGHT) {
    ctx->err = "bpp_msm_submit: " + std::to_string(BPP_MSM_INFLIGHT) + " MSMs already in flight (collect one first)";
    return BPP_ERR_ARG;
  }
  bpp_ctx::MsmSlot& sl = ctx->msm_slot[s];
  BPP_HIP(hipSetDevice(ctx->device));
  bpp_ctx* ch = nullptr;
  BPP_TRY(ctx_child(ctx, s, &ch));
  ch->prof = ctx->prof;
  // Another MSM in flight: hold this accumulation to 3 workgroups per CU
  // (LDS 40 + 13 KB each) so the other MSM's sort runs beside it rather than
  // after it -- 2^20, two in flight: 0.97 -> 0.945 ms per MSM; alone it
  // would cost the accumulation ~8 % (BPP_ACC_LDS_PAD overrides the pad).
  bool others = false;
  for (size_t i = 0; i < BPP_MSM_INFLIGHT; ++i) others |= ctx->msm_slot[i].busy;
  static const long pad_env = [] {
    const char* e = getenv("BPP_ACC_LDS_PAD");
    return e ? atol(e) : -1L;
  }();
  ch->acc_lds_pad = others ? (pad_env >= 0 ? (size_t)pad_env : (size_t)13000) : 0;
  if (!sl.done) BPP_HIP(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
  // inputs written on ctx's stream before this call are visible to the child
  BPP_HIP(hipEventRecord(sl.done, ctx->stream));
  BPP_HIP(hipStreamWaitEvent(ch->stream, sl.done, 0));
  sl.c = c;
  sl.wb = w_begin;
  sl.Wn = w_end - w_begin;
  sl.nterms = 1;
  if (h_scalars && n && sl.Wn) {
    int rc = BPP_OK;
    if (ch->up_sc_bytes < n * 32) {
      if (ch->up_sc) BPP_HIP(hipFree(ch->up_sc));
      ch->up_sc = nullptr;
      ch->up_sc_bytes = 0;
      // (BPP_MSM_UP_CACHED=1: an ordinary allocation; by default uncached,
      // so that the upload's 32 B x n writes do not evict the point table
      // the other MSMs' accumulations gather from the caches; the digit
      // kernel reads each scalar once)
      const bool cached = getenv("BPP_MSM_UP_CACHED") && atoi(getenv("BPP_MSM_UP_CACHED"));
      if (cached) {
        BPP_HIP(hipMalloc(&ch->up_sc, n * 32));
      } else {
        BPP_HIP(hipExtMallocWithFlags(&ch->up_sc, n * 32, hipDeviceMallocUncached));
      }
      ch->up_sc_bytes = n * 32;
    }
    void* d = ch->up_sc;
    {
      const bool pinned = host_is_pinned(h_scalars, n * 32);
      // (pinned read in place by the digit kernel, zero copy, measured 1.397
      // vs 0.875 ms per resident MSM: its PCIe-bound blocks held CUs the
      // other MSMs' accumulations needed)
      // The copy runs on the slot's own stream.  BPP_MSM_UP_STREAMS=k (1-4)
      // splits it into k chunks on k upload streams of the parent that the
      // slot's stream waits for by event (an A/B switch): the standalone
      // probe (tools/host_msm_probe.py, 2^20 pinned, 3 in flight, three
      // interleaved passes) measured 1.53-1.77 ms per MSM on the slot's
      // stream, 1.11-1.24 with one upload stream and 1.10-1.12 with two,
      // against 0.99 resident -- but inside bench.py (three interleaved full
      // runs) two upload streams measured 1.35-1.82x resident vs 1.21-1.61x,
      // the pageable leg 1.25-1.55x vs 1.16-1.22x, and the later prover leg
      // 270-273 K vs 282-287 K proofs/s, so the default stays 0.  Pageable
      // scalars go piece by piece (upload_pieces): 1.16-1.30x resident vs
      // 1.22-1.52x staged whole, within the box's noise.  The slot's previous
      // MSM has been collected, so nothing still reads up_sc.
      const char* se = getenv("BPP_MSM_UP_STREAMS");
      const int ns = se ? std::max(0, std::min(4, atoi(se))) : 0;
      const size_t bytes = n * 32;
      uint8_t* src = (uint8_t*)h_scalars;
      if (!pinned && ns == 0) {  // staged through the slot's arena (recycled
        // only by a sync of the slot's stream, which waits for the copies)
        // piece by piece, each piece's DMA queued on the slot's stream as
        // soon as it is staged (the stream's scalars are not checked here:
        // the submit contract, as for device scalars)
        size_t bad = n;
        rc = upload_pieces(ch, d, (const uint8_t*)h_scalars, n, false, &bad);
      } else if (!pinned) {
        uint8_t* p = nullptr;
        rc = ctx_h2d_stage(ch, bytes, &p);
        if (!rc) {
          ctx_stage_copy(p, h_scalars, bytes);
          src = p;
        }
      }
      if (pinned && !rc && ns == 0) {
        if (hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, ch->stream) != hipSuccess) rc = BPP_ERR_DEVICE;
      } else if (!rc && ns > 0) {
        const size_t part = ((bytes + ns - 1) / ns + 255) & ~(size_t)255;
        for (int k = 0; k < ns && !rc; ++k) {
          const size_t o = (size_t)k * part;
          if (o >= bytes) break;
          if (!ctx->up_stream[k]) BPP_HIP(hipStreamCreateWithFlags(&ctx->up_stream[k], hipStreamNonBlocking));
          if (!ch->up_ev[k]) BPP_HIP(hipEventCreateWithFlags(&ch->up_ev[k], hipEventDisableTiming));
          BPP_HIP(hipStreamWaitEvent(ctx->up_stream[k], sl.done, 0));  // (inputs written on ctx's stream)
          if (hipMemcpyAsync((uint8_t*)d + o, src + o, std::min(part, bytes - o), hipMemcpyHostToDevice,
                             ctx->up_stream[k]) != hipSuccess) {
            rc = BPP_ERR_DEVICE;
            break;
          }
          BPP_HIP(hipEventRecord(ch->up_ev[k], ctx->up_stream[k]));
          BPP_HIP(hipStreamWaitEvent(ch->stream, ch->up_ev[k], 0));
        }
      }
    }
    if (rc) {
      ctx->err = ch->err.empty() ? "bpp_msm_submit_host: scalar upload failed" : ch->err;
      return rc;
    }
    d_scalars = d;
  }
  if (n && sl.Wn) {
    // (in-flight MSMs share the device freely: serialising their
    // accumulations measured slower, 1.17 vs 1.04 ms per 2^20 MSM)
    uint32_t* d_ws = nullptr;
    const int rc = msm_engine(ch, (const uint32_t*)d_scalars, nullptr, nullptr, 1, (uint32_t)n, c, w_begin, sl.Wn,
                              tbl->d, &d_ws, nullptr, 0xffffffffu, false, &sl.nterms);
    if (rc) {
      ctx->err = ch->err;
      return rc;
    }
    const size_t bytes = (size_t)sl.Wn * sl.nterms * P3_BYTES;
    int prc = ctx_pinned(ch, bytes, &sl.h);
    if (prc) {
      ctx->err = ch->err;
      return prc;
    }
    BPP_HIP(hipMemcpyAsync(sl.h, d_ws, bytes, hipMemcpyDeviceToHost, ch->stream));
  }
  BPP_HIP(hipEventRecord(sl.done, ch->stream));
  sl.busy = true;
  sl.ticket = t;
  *ticket = t;
  ++ctx->msm_next_ticket;
  return BPP_OK;
}

int bpp_msm_collect(bpp_ctx* ctx, uint64_t ticket, uint8_t out[32], uint8_t partial[128]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx) return BPP_ERR_ARG;
    size_t s = BPP_MSM_INFLIGHT;
    for (size_t i = 0; i < BPP_MSM_INFLIGHT; ++i)
      if (ctx->msm_slot[i].busy && ctx->msm_slot[i].ticket == ticket) s = i;
    if (s == BPP_MSM_INFLIGHT) {
      ctx->err = "bpp_msm_collect: unknown or already collected ticket";
      return BPP_ERR_ARG;
    }
    bpp_ctx::MsmSlot& sl = ctx->msm_slot[s];
    BPP_HIP(hipSetDevice(ctx->device));
    // the slot (its child stream and pinned buffer) is released only once the
    // child's copies are known to be done; on a failed wait the child stream
    // is drained before the slot can be reused
    if (hipEventSynchronize(sl.done) != hipSuccess) {
      bpp_ctx* ch = s < ctx->children.size() ? ctx->children[s] : nullptr;
      if (ch) hipStreamSynchronize(ch->stream);
      sl.busy = false;
      sl.h = nullptr;
      ctx->err = "bpp_msm_collect: device error while waiting for the MSM";
      return BPP_ERR_DEVICE;
    }
    sl.busy = false;
    h25519::ge r = h25519::ge_identity();
    if (sl.h && sl.Wn) r = horner_host_terms((const uint32_t*)sl.h, sl.Wn, sl.nterms, sl.c, sl.wb);
    sl.h = nullptr;
    if (out) h25519::encode(out, r);
    if (partial) h25519::ge_to_words((uint32_t*)partial, r);
    return BPP_OK;
  });
}

int bpp_partials_finish(const uint8_t* partials, size_t count, uint8_t out[32]) {
  return bpp_guard(nullptr, [&]() -> int {
    if (!out || (!partials && count)) return BPP_ERR_ARG;
    h25519::ge acc = h25519::ge_identity();
    for (size_t i = 0; i < count; ++i) {
      uint32_t w[32];
      memcpy(w, partials + 128 * i, 128);
      const h25519::ge p = h25519::ge_from_words(w);
      // Z = 0 is no extended point (e.g. a partial a failed rank never
      // wrote): it would absorb the sum and encode as the identity, so it
      // is refused rather than accepted as one
      if (h25519::fe_iszero(p.Z)) return BPP_ERR_ARG;
      acc = h25519::ge_add(acc, p);
    }
    h25519::encode(out, acc);
    return BPP_OK;
  });
}

int bpp_points_double_compress(const uint8_t* raw, size_t count, uint8_t* out) {
  return bpp_guard(nullptr, [&]() -> int {
    if ((!raw || !out) && count) return BPP_ERR_ARG;
    std::vector<h25519::ge> pts(count);
    for (size_t i = 0; i < count; ++i) {
      uint32_t w[32];
      memcpy(w, raw + 128 * i, 128);
      pts[i] = h25519::ge_from_words(w);
    }
    h25519::encode_double_batch_auto(pts.data(), count, out);
    return BPP_OK;
  });
}

int bpp_msm_table(bpp_ctx* ctx, const uint8_t* scalars, const bpp_points* tbl, size_t n, uint8_t out[32]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !tbl || !out || (!scalars && n)) return BPP_ERR_ARG;
    if (n > tbl->n) return BPP_ERR_LEN;
    BPP_HIP(hipSetDevice(ctx->device));
    uint32_t* d_s = nullptr;
    BPP_TRY(upload_scalars(ctx, scalars, n, "msm_scal", &d_s));
    return bpp_msm_table_dev(ctx, d_s, tbl, n, out);
  });
}

int bpp_msm(bpp_ctx* ctx, const uint8_t* scalars, const uint8_t* points, size_t n, uint8_t out[32]) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !out || ((!scalars || !points) && n)) return BPP_ERR_ARG;
    bpp_points* tbl = nullptr;
    size_t bad = 0;
    BPP_TRY(bpp_points_decompress(ctx, points, n, &tbl, &bad));
    int rc = bpp_msm_table(ctx, scalars, tbl, n, out);
    bpp_points_destroy(tbl);
    return rc;
  });
}

int bpp_msm_batch(bpp_ctx* ctx, size_t count, const uint64_t* offsets, const uint8_t* scalars,
                  const uint32_t* point_idx, const bpp_points* tbl, uint8_t* out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !offsets || !tbl || (!out && count)) return BPP_ERR_ARG;
    if (count == 0) return BPP_OK;
    const uint64_t T = offsets[count];
    if (offsets[0] != 0 || T >= 0x80000000ull) return BPP_ERR_LEN;
    for (size_t j = 0; j < count; ++j)
      if (offsets[j + 1] < offsets[j]) return BPP_ERR_LEN;
    for (uint64_t t = 0; t < T; ++t)
      if (point_idx[t] >= tbl->n) return BPP_ERR_LEN;
    BPP_HIP(hipSetDevice(ctx->device));
    uint32_t* d_s = nullptr;
    BPP_TRY(upload_scalars(ctx, scalars, T, "msmb_scal", &d_s));
    void *d_idx, *d_off, *d_res;
    BPP_TRY(ctx_ws(ctx, "msmb_idx", T * 4 + 4, &d_idx));
    BPP_TRY(ctx_ws(ctx, "msmb_off", (count + 1) * 4, &d_off));
    BPP_TRY(ctx_ws(ctx, "msmb_res", count * P3_BYTES, &d_res));
    std::vector<uint32_t> off32(count + 1);
    for (size_t j = 0; j <= count; ++j) off32[j] = (uint32_t)offsets[j];
    if (T) BPP_HIP(hipMemcpyAsync(d_idx, point_idx, T * 4, hipMemcpyHostToDevice, ctx->stream));
    BPP_HIP(hipMemcpyAsync(d_off, off32.data(), (count + 1) * 4, hipMemcpyHostToDevice, ctx->stream));
    const uint32_t c = msm_choose_c((double)T / (double)count);
    const uint32_t W = (254 + c - 1) / c;
    MsmGeom g;
    g.M = (uint32_t)count;
    g.T = (uint32_t)T;
    g.c = c;
    g.W = W;
    g.wb = 0;
    g.Wn = W;
    g.B = 1u << (c - 1);
    g.fb = 0;
    uint32_t* d_ws = nullptr;
    BPP_TRY(msm_engine(ctx, d_s, (const uint32_t*)d_idx, (const uint32_t*)d_off, g.M, g.T, c, 0, W, tbl->d, &d_ws));
    {
      ProfScope ps(ctx, "msm_horner");
      hipLaunchKernelGGL(k_msm_horner, dim3(grid_for(count, 64)), dim3(64), 0, ctx->stream, (const uint32_t*)d_ws, g,
                         (uint32_t*)d_res);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_msm_horner"));
    return points_compress_p3(ctx, (const uint32_t*)d_res, count, out);
  });
}

}  // extern "C"

// thread t: w = t / npts, k = t % npts (a wave shares w, so every lane does
// the same c*w doublings) -> dst[k*W + w] = 2^(c*w) * src[k].
__global__ void __launch_bounds__(64) k_fbw_tables(const uint32_t* __restrict__ src, uint32_t npts,
                                                   uint32_t* __restrict__ dst) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)npts * FBW_W) return;
  const uint32_t w = (uint32_t)(t / npts), k = (uint32_t)(t % npts);
  const ge_niels P = load_niels(src, k);
  if (w == 0) {
    store_niels(dst, (size_t)k * FBW_W, P);
    return;
  }
  ge_p3 a = ge_from_niels(P);
  for (uint32_t i = 0; i < FBW_C * w; ++i) a = ge_dbl(a);
  store_niels(dst, (size_t)k * FBW_W + w, ge_to_niels(a));
}

int fbw_build(bpp_ctx* ctx, const uint32_t* d_src, uint32_t npts, uint32_t* d_dst) {
  if (!npts) return BPP_OK;
  {
    ProfScope ps(ctx, "fbw_tables");
    hipLaunchKernelGGL(k_fbw_tables, dim3(grid_for((size_t)npts * FBW_W, 64)), dim3(64), 0, ctx->stream, d_src, npts,
                       d_dst);
  }
  return ctx_check_launch(ctx, "k_fbw_tables");
}

static int fb_policy();
static bool fb_wins(double terms_per_msm);

int msm_points_extra(bpp_ctx* ctx, MsmPoints* pts, const uint32_t* d_x, uint32_t nx, uint32_t n0,
                     const char* ws_name, double terms_per_msm) {
  pts->tbl1 = d_x;
  pts->n0 = n0;
  pts->wt1 = nullptr;
  // Building a window table is a ~250-doubling chain per point plus an
  // inversion: it pays for resident generators, not for points used once
  // (measured: verify 1.1 ms without, 1.7 ms with), so only BPP_MSM_FB=1
  // builds them.
  if (!pts->wt || !nx || fb_policy() != 1 || !fb_wins(terms_per_msm)) return BPP_OK;
  void* d = nullptr;
  BPP_TRY(ctx_ws(ctx, ws_name, (size_t)nx * FBW_W * MSM_NIELS_WORDS * 4, &d));
  BPP_TRY(fbw_build(ctx, d_x, nx, (uint32_t*)d));
  pts->wt1 = (const uint32_t*)d;
  return BPP_OK;
}

// BPP_MSM_FB: unset = cost model, 0 = never, 1 = always (tests cover both)
static int fb_policy() {
  const char* e = getenv("BPP_MSM_FB");
  return e ? atoi(e) : -1;
}

// Fixed-base costs FBW_W = 32 mixed additions per term against ~W = 254/c
// for the variable-base engine plus its per-window bucket reduction and
// Horner combine; below ~16K terms per MSM the fixed cost dominates.
static bool fb_wins(double terms_per_msm) {
  const int pol = fb_policy();
  return pol == 1 || (pol == -1 && terms_per_msm <= 16384.0);
}

DtGeom dt_geom(uint32_t c) {
  DtGeom g;
  g.c = c;
  g.W = (254 + c - 1) / c;
  g.H = 1u << (c - 1);
  for (int i = 0; i < 8; ++i) g.K[i] = 0;
  for (uint32_t w = 0; w + 1 < g.W; ++w) {  // bit c w + c - 1 (< 253)
    const uint32_t pos = c * w + c - 1;
    g.K[pos >> 5] |= 1u << (pos & 31);
  }
  return g;
}

size_t dt_bytes(uint32_t npts, uint32_t c) {
  const DtGeom g = dt_geom(c);
  return (size_t)npts * g.W * g.H * MSM_NIELS_WORDS * 4;
}

int dt_build(bpp_ctx* ctx, const uint32_t* d_wt, uint32_t npts, uint32_t c, uint32_t* d_dt) {
  if (!npts) return BPP_OK;
  // (c <= 17: the top window's digit field of s + K < 2^254 stays below
  // H = 2^(c-1) rows, and the row index below 2^32 for the generator sets)
  if (c < 8 || c > 17) {
    ctx->err = "dt_build: window width must be 8..17";
    return BPP_ERR_ARG;
  }
  const DtGeom g = dt_geom(c);
  const size_t rows = (size_t)npts * g.W * g.H;
  if (rows >= 0x100000000ull) {
    ctx->err = "dt_build: table too large";
    return BPP_ERR_LEN;
  }
  // 4 rows a lane (k_dt_build_n: one double-and-add and one inversion per 4
  // rows; BPP_DT_BUILD_RPL=1 keeps one row a lane, an A/B switch)
  static const int rpl = [] {
    const char* e = getenv("BPP_DT_BUILD_RPL");
    return e ? atoi(e) : 4;
  }();
  {
    ProfScope ps(ctx, "dt_tables");
    if (rpl == 4 && g.H % 4 == 0)
      hipLaunchKernelGGL(k_dt_build_n<4>, dim3(grid_for(rows / 4, 64)), dim3(64), 0, ctx->stream, d_wt, npts, g, d_dt);
    else if (rpl == 2)
      hipLaunchKernelGGL(k_dt_build_n<2>, dim3(grid_for(rows / 2, 64)), dim3(64), 0, ctx->stream, d_wt, npts, g, d_dt);
    else
      hipLaunchKernelGGL(k_dt_build, dim3(grid_for(rows, 64)), dim3(64), 0, ctx->stream, d_wt, npts, g, d_dt);
  }
  return ctx_check_launch(ctx, "k_dt_build");
}

// Direct-table engine: one block per MSM (BPP_MSM_DT=0 disables, =1 forces).
bool msm_use_dt(const MsmPoints& pts, uint32_t M, uint32_t T) {
  if (!pts.dt || pts.tbl1 || M == 0) return false;
  const char* e = getenv("BPP_MSM_DT");
  const int pol = e ? atoi(e) : -1;
  return pol == 1 || (pol == -1 && (double)T <= 16384.0 * (double)M);
}

static int msm_multi_dt_dev(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx,
                            const std::vector<uint32_t>& off, const MsmPoints& pts, uint32_t** d_res,
                            uint32_t* res_out = nullptr, const uint32_t* d_smap = nullptr) {
  const uint32_t M = (uint32_t)off.size() - 1;
  const uint32_t T = off[M];
  void *d_off, *res;
  BPP_TRY(upload_offsets(ctx, off, &d_off));
  if (res_out)
    res = res_out;
  else
    BPP_TRY(ctx_ws(ctx, "dt_res", (size_t)M * P3_BYTES, &res));
  const DtGeom dg = dt_geom(pts.dt_c);
  // W lanes per term group: the largest multiple of W within DT_NT_MAX lanes
  // whose groups each still get about two terms (small MSMs: fewer lanes,
  // a shallower tree); ~512 lanes measured slower at 8 proof batches in
  // flight
  const double t_avg = (double)T / (double)M;
  const uint32_t TG = dt_term_groups(dg.W, t_avg, M);
  const uint32_t nt = TG * dg.W;
  // two MSMs per block (k_dt_msm segs = 2, BPP_DT_PAIR=1) for launches with
  // blocks to spare, an A/B switch, off: round 6 re-ran the A/B at the bench's
  // prover shape (384 x 32 in flight, 8 queues): proofs/s equal (363-365 K
  // vs 364-366 K), but one MSM per block issues more (k_dt_msm VALU issue
  // 0.359 vs 0.314, wait_any 0.368 vs 0.456) and misses the UTCL1 less (5.2 %
  // vs 8.3 % of requests); profiles/r06_dt_pair_ab.txt, r06_tlb_prover.json
  static const bool pair_env = [] {
    const char* e = getenv("BPP_DT_PAIR");
    return e && atoi(e) != 0;
  }();
  const uint32_t segs = pair_env && M >= 512 && 2 * nt <= DT_NT_MAX ? 2u : 1u;
  ctx_work(ctx, "msm_terms", T);
  ctx_work(ctx, "madds", (uint64_t)T * dg.W);
  ctx_work(ctx, "padds", (uint64_t)M * (nt - 1));
  ctx_work(ctx, "msm_launches", 1);
  ctx_work(ctx, "dt_terms", T);  // the direct-table kernel's own share
  ctx_work(ctx, "dt_madds", (uint64_t)T * dg.W);
  ctx_work(ctx, "dt_launches", 1);
  {
    ProfScope ps(ctx, "msm_direct");
    hipLaunchKernelGGL(k_dt_msm, dim3((M + segs - 1) / segs), dim3(segs * nt), (size_t)segs * nt * P3_BYTES,
                       ctx->stream, pts.dt, dg, d_scal, d_pidx, (const uint32_t*)d_off, (uint32_t*)res, d_smap, segs,
                       M);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_dt_msm"));
  *d_res = (uint32_t*)res;
  return BPP_OK;
}

static bool use_fb(const MsmPoints& pts, uint32_t M, uint32_t T) {
  const bool have_fb = pts.wt && (!pts.tbl1 || pts.wt1);
  return have_fb && M > 0 && fb_wins((double)T / (double)M);
}

// Fixed-base engine: device array of the M results (extended, 32 words each).
static int msm_multi_fb_dev(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx,
                            const std::vector<uint32_t>& off, const MsmPoints& pts, uint32_t** d_res) {
  const uint32_t M = (uint32_t)off.size() - 1;
  const uint32_t T = off[M];
  if ((uint64_t)(pts.n0 == 0xffffffffu ? 0 : pts.n0) * FBW_W >= 0x80000000ull ||
      (uint64_t)T * FBW_W >= 0x80000000ull) {
    ctx->err = "fixed-base MSM too large";
    return BPP_ERR_LEN;
  }
  void* d_off = nullptr;
  BPP_TRY(upload_offsets(ctx, off, &d_off));
  const uint32_t n0w = pts.n0 == 0xffffffffu ? 0xffffffffu : pts.n0 * FBW_W;
  return msm_engine(ctx, d_scal, d_pidx, (const uint32_t*)d_off, M, T, FBW_C, 0, FBW_W, pts.wt, d_res, pts.wt1, n0w,
                    true);
}

int msm_multi(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const std::vector<uint32_t>& off,
              const MsmPoints& pts, std::vector<h25519::ge>& out) {
  const uint32_t M = (uint32_t)off.size() - 1;
  const uint32_t T = off[M];
  const bool dt = msm_use_dt(pts, M, T);
  if (!dt && !use_fb(pts, M, T)) return msm_multi(ctx, d_scal, d_pidx, off, pts.tbl, pts.tbl1, pts.n0, out);
  out.assign(M, h25519::ge_identity());
  if (M == 0 || T == 0) return BPP_OK;
  uint32_t* d_ws = nullptr;
  if (dt) BPP_TRY(msm_multi_dt_dev(ctx, d_scal, d_pidx, off, pts, &d_ws));
  else BPP_TRY(msm_multi_fb_dev(ctx, d_scal, d_pidx, off, pts, &d_ws));
  void* h = nullptr;
  BPP_TRY(ctx_pinned(ctx, (size_t)M * P3_BYTES, &h));
  BPP_HIP(hipMemcpyAsync(h, d_ws, (size_t)M * P3_BYTES, hipMemcpyDeviceToHost, ctx->stream));
  BPP_TRY(ctx_sync(ctx));
  for (uint32_t m = 0; m < M; ++m) out[m] = h25519::ge_from_dev((const uint32_t*)h + (size_t)m * P3_WORDS);
  return BPP_OK;
}

int msm_multi_enc(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const std::vector<uint32_t>& off,
                  const MsmPoints& pts, uint8_t* out_enc, bool doubled, const uint32_t* d_smap) {
  const uint32_t M = (uint32_t)off.size() - 1;
  const uint32_t T = off[M];
  if (M == 0) return BPP_OK;
  if (d_smap && !(doubled && M > 16 && T > 0 && msm_use_dt(pts, M, T))) {
    // (only the direct-table kernel gathers and halves in place)
    void* d_sh = nullptr;
    BPP_TRY(ctx_ws(ctx, "mt_s_half", (size_t)T * 32 + 32, &d_sh));
    BPP_TRY(sc_halve_gather_dev(ctx, d_scal, d_smap, (uint32_t*)d_sh, T));
    return msm_multi_enc(ctx, (const uint32_t*)d_sh, d_pidx, off, pts, out_enc, doubled, nullptr);
  }
  // Few results: host encoding beats a latency-bound GPU launch; many: one
  // GPU lane per result, or (doubled) the host batch encoding of 2 R_m.
  if (M > 16 && T > 0 && (msm_use_dt(pts, M, T) || use_fb(pts, M, T))) {
    uint32_t* d_ws = nullptr;
    if (msm_use_dt(pts, M, T) && doubled) {  // results written in place in host memory (ctx_zc_out)
      uint32_t* h = nullptr;
      BPP_TRY(ctx_zc_out(ctx, "multi_res_h", (size_t)M * P3_BYTES, &h));
      BPP_TRY(msm_multi_dt_dev(ctx, d_scal, d_pidx, off, pts, &d_ws, h, d_smap));
      BPP_TRY(ctx_sync(ctx));
      return points_double_encode_host(ctx, h, M, out_enc);
    }
    if (msm_use_dt(pts, M, T))
      BPP_TRY(msm_multi_dt_dev(ctx, d_scal, d_pidx, off, pts, &d_ws));
    else
      BPP_TRY(msm_multi_fb_dev(ctx, d_scal, d_pidx, off, pts, &d_ws));
    return doubled ? points_double_encode_p3(ctx, d_ws, M, out_enc) : points_compress_p3(ctx, d_ws, M, out_enc);
  }
  std::vector<h25519::ge> res;
  BPP_TRY(msm_multi(ctx, d_scal, d_pidx, off, pts, res));
  if (doubled)
    h25519::encode_double_batch_auto(res.data(), M, out_enc);
  else
    for (uint32_t m = 0; m < M; ++m) h25519::encode(out_enc + 32 * (size_t)m, res[m]);
  return BPP_OK;
}

// M independent MSMs (host offsets, M+1 entries) over device scalars and
// point indices; results returned as host points.  Few MSMs: window sums are
// combined on the host; many: one GPU lane per MSM runs the Horner chain.
int msm_multi(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const std::vector<uint32_t>& off,
              const uint32_t* d_tbl, const uint32_t* d_tbl1, uint32_t n0, std::vector<h25519::ge>& out) {
  const uint32_t M = (uint32_t)off.size() - 1;
  const uint32_t T = off[M];
  out.assign(M, h25519::ge_identity());
  if (M == 0 || T == 0) return BPP_OK;
  void* d_off = nullptr;
  BPP_TRY(upload_offsets(ctx, off, &d_off));
  const uint32_t c = msm_choose_c((double)T / (double)M);
  const uint32_t W = (254 + c - 1) / c;
  uint32_t* d_ws = nullptr;
  uint32_t nterms = 1;
  BPP_TRY(msm_engine(ctx, d_scal, d_pidx, (const uint32_t*)d_off, M, T, c, 0, W, d_tbl, &d_ws, d_tbl1, n0, false,
                     M == 1 ? &nterms : nullptr));
  if (M <= 8) {
    void* h = nullptr;
    BPP_TRY(ctx_pinned(ctx, (size_t)M * W * nterms * P3_BYTES, &h));
    BPP_HIP(hipMemcpyAsync(h, d_ws, (size_t)M * W * nterms * P3_BYTES, hipMemcpyDeviceToHost, ctx->stream));
    BPP_TRY(ctx_sync(ctx));
    for (uint32_t m = 0; m < M; ++m)
      out[m] = horner_host_terms((const uint32_t*)h + (size_t)m * W * nterms * P3_WORDS, W, nterms, c, 0);
    return BPP_OK;
  }
  MsmGeom g;
  g.M = M;
  g.T = T;
  g.c = c;
  g.W = W;
  g.wb = 0;
  g.Wn = W;
  g.B = 1u << (c - 1);
  g.fb = 0;
  void* d_res = nullptr;
  BPP_TRY(ctx_ws(ctx, "multi_res", (size_t)M * P3_BYTES, &d_res));
  {
    ProfScope ps(ctx, "msm_horner");
    hipLaunchKernelGGL(k_msm_horner, dim3(grid_for(M, 64)), dim3(64), 0, ctx->stream, (const uint32_t*)d_ws, g,
                       (uint32_t*)d_res);
  }
  BPP_TRY(ctx_check_launch(ctx, "k_msm_horner"));
  std::vector<uint32_t> h((size_t)M * P3_WORDS);
  BPP_TRY(ctx_d2h(ctx, h.data(), d_res, (size_t)M * P3_BYTES));
  for (uint32_t m = 0; m < M; ++m) out[m] = h25519::ge_from_dev(h.data() + (size_t)m * P3_WORDS);
  return BPP_OK;
}
