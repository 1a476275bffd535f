// Internal MSM engine interface shared by msm.hip and the proof-level code.
#pragma once
#include <stdint.h>

#include "ctx.h"
#include "host/fe64.h"

bool scalar_is_canonical(const uint8_t* s);
// Buckets per lane of the single-MSM bucket reduction (k_msm_reduce_wave):
// 2^RWAVE_LOG in MSM streams, 2^RWAVE_LOG_LONE for an MSM that runs alone
#ifndef RWAVE_LOG
#define RWAVE_LOG 4
#endif
#ifndef RWAVE_LOG_LONE
#define RWAVE_LOG_LONE 3  // (msm_kernels.cuh holds the same value; msm.hip asserts it)
#endif
uint32_t msm_choose_c(double n_per_msm);
// Runs K1..K5 for M MSMs over T terms; returns the device array of M*Wn
// window sums (extended points, 32 words each).
int msm_engine(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const uint32_t* d_off, uint32_t M,
               uint32_t T, uint32_t c, uint32_t wb, uint32_t Wn, const uint32_t* d_tbl, uint32_t** d_wsum_out,
               const uint32_t* d_tbl1 = nullptr, uint32_t n0 = 0xffffffffu, bool fb = false,
               uint32_t* terms_out = nullptr, uint32_t rlog = RWAVE_LOG, uint32_t* rshift_out = nullptr);
// With terms_out (single MSMs only) the engine may return, per window, 1 + J
// terms instead of one sum: the window sum is term 0 + sum_j 2^(rshift+j)
// term 1+j (k_msm_reduce_wave); *terms_out = terms per window (1 = plain sums),
// *rshift_out = rshift (rlog + 6 for the stream shape; the lone shape picks
// its own buckets per lane).
// Host Horner over such terms: sum_j 2^(c (wb + j)) * window_j.
h25519::ge horner_host_terms(const uint32_t* ws_words, uint32_t Wn, uint32_t nterms, uint32_t c, uint32_t wb,
                             uint32_t rshift = RWAVE_LOG + 6);
int msm_single_dev(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const uint32_t* d_tbl, size_t n,
                   uint32_t c, uint32_t wb, uint32_t Wn, h25519::ge* out, const uint32_t* d_tbl1 = nullptr,
                   uint32_t n0 = 0xffffffffu);
int upload_scalars(bpp_ctx* ctx, const uint8_t* scalars, size_t n, const char* name, uint32_t** d_out);
int points_compress_p3(bpp_ctx* ctx, const uint32_t* d_p3, size_t n, uint8_t* out_host);
// same, encodings left on the device (d_out: n x 32 B)
int points_compress_p3_dev(bpp_ctx* ctx, const uint32_t* d_p3, size_t n, uint8_t* d_out);
// out = encodings of 2 * P_i (host batch encoding; see points.hip)
int points_double_encode_p3(bpp_ctx* ctx, const uint32_t* d_p3, size_t n, uint8_t* out_host);
// same for n points already in host memory (P3 words)
// raw: n x J device-layout points; point i = the sum of raw[i J .. i J + J)
int points_double_encode_host(bpp_ctx* ctx, const uint32_t* raw, size_t n, uint8_t* out_host, uint32_t J = 1);
// d_out[i] = d_in[i] / 2 mod l (canonical scalars; in place allowed)
int sc_halve_dev(bpp_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, size_t n);
// d_out[t] = d_in[d_map[t]] / 2 for t < n
int sc_halve_gather_dev(bpp_ctx* ctx, const uint32_t* d_in, const uint32_t* d_map, uint32_t* d_out, size_t n);
#include <vector>
// Fixed-base window tables: entry k*FBW_W + w = 2^(FBW_C*w) * P_k (affine
// Niels).  An MSM over such points needs no per-window Horner combine: all
// windows share one bucket set.
#define FBW_C 8
#define FBW_W 32
int fbw_build(bpp_ctx* ctx, const uint32_t* d_src, uint32_t npts, uint32_t* d_dst);
// Point sources of an MSM: index < n0 -> tbl, else tbl1[idx - n0]; wt / wt1
// are the matching window tables (null: not available).
struct MsmPoints {
  const uint32_t* tbl = nullptr;
  const uint32_t* tbl1 = nullptr;
  uint32_t n0 = 0xffffffffu;
  const uint32_t* wt = nullptr;
  const uint32_t* wt1 = nullptr;
  const uint32_t* dt = nullptr;  // direct radix-2^dt_c tables of tbl (msm_kernels.cuh k_dt_msm), or null
  uint32_t dt_c = 8;
};
// d * 2^(c w) * P for every table point, w < 256 / c, d = 1..2^(c-1)
// (128-B rows; c = 8 or 16)
int dt_build(bpp_ctx* ctx, const uint32_t* d_wt, uint32_t npts, uint32_t c, uint32_t* d_dt);
// bytes of the direct tables of npts points at window width c
size_t dt_bytes(uint32_t npts, uint32_t c);
// Adds nx extra points (device Niels table d_x) at indices n0.. to *pts,
// building their window tables in workspace `ws_name` when pts has tables
// and MSMs of `terms_per_msm` terms would take the fixed-base engine.
int msm_points_extra(bpp_ctx* ctx, MsmPoints* pts, const uint32_t* d_x, uint32_t nx, uint32_t n0, const char* ws_name,
                     double terms_per_msm);
// M independent MSMs; picks the fixed-base engine when window tables exist
// and the MSMs are small enough for it to win (BPP_MSM_FB=0/1 forces).
int msm_multi(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const std::vector<uint32_t>& off,
              const MsmPoints& pts, std::vector<h25519::ge>& out);
// Same, results compressed (M x 32 B).
// doubled: d_scal holds halved scalars s/2 and out_enc gets the encodings of
// 2 * result (host batch encoding, one inversion instead of a per-point
// inverse square root)
// d_smap (optional, with doubled): term t's scalar is d_scal[d_smap[t]] / 2
// (gathered and halved inside the direct-table kernel; a gather pass first
// on the other engines)
int msm_multi_enc(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const std::vector<uint32_t>& off,
                  const MsmPoints& pts, uint8_t* out_enc,
                  bool doubled = false, const uint32_t* d_smap = nullptr);
int msm_multi(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const std::vector<uint32_t>& off,
              const uint32_t* d_tbl, const uint32_t* d_tbl1, uint32_t n0, std::vector<h25519::ge>& out);
