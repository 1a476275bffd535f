// Internal MSM engine interface shared by msm.hip and the proof-level code.
#pragma once
#include <stdint.h>

#include "ctx.h"
#include "host/fe64.h"

bool scalar_is_canonical(const uint8_t* s);
uint32_t msm_choose_c(double n_per_msm);
// Runs K1..K5 for M MSMs over T terms; returns the device array of M*Wn
// window sums (extended points, 32 words each).
int msm_engine(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const uint32_t* d_off, uint32_t M,
               uint32_t T, uint32_t c, uint32_t wb, uint32_t Wn, const uint32_t* d_tbl, uint32_t** d_wsum_out,
               const uint32_t* d_tbl1 = nullptr, uint32_t n0 = 0xffffffffu);
int msm_single_dev(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const uint32_t* d_tbl, size_t n,
                   uint32_t c, uint32_t wb, uint32_t Wn, h25519::ge* out);
int upload_scalars(bpp_ctx* ctx, const uint8_t* scalars, size_t n, const char* name, uint32_t** d_out);
int points_compress_p3(bpp_ctx* ctx, const uint32_t* d_p3, size_t n, uint8_t* out_host);
#include <vector>
int msm_multi(bpp_ctx* ctx, const uint32_t* d_scal, const uint32_t* d_pidx, const std::vector<uint32_t>& off,
              const uint32_t* d_tbl, const uint32_t* d_tbl1, uint32_t n0, std::vector<h25519::ge>& out);
