// Batched point codec kernels: ristretto255 decompress / compress and
// RistrettoPoint::from_uniform_bytes, one lane per point, into the resident
// affine-Niels table format the MSM kernels gather from.
//
// Reference sites: compress circuit_lib.rs:231-233,368-412; decompress
// circuit_lib.rs:532 (`unwrap()` -> BPP_ERR_DECOMPRESS here);
// RistrettoPoint::random lib.rs:165-180 (from_uniform_bytes of rng bytes).
#include <algorithm>
#include <cstring>
#include <vector>

#include "ctx.h"
#include "sc25519.cuh"
#include "host/fe64.h"
#include "host/par.h"
#include "ge_io.cuh"

__global__ void __launch_bounds__(64) k_decompress(const uint32_t* __restrict__ enc, size_t n, uint32_t* __restrict__ tbl,
                             unsigned long long* __restrict__ bad) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  const uint4* p = reinterpret_cast<const uint4*>(enc + i * 8);
  uint4 a = p[0], b = p[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
  ge_p3 P;
  if (!ge_ristretto_decode(w, P)) {
    atomicMin(bad, (unsigned long long)i);
    P = ge_identity();
  }
  // Z = 1 after decode: Niels directly from (x, y)
  store_niels(tbl, (uint32_t)i, ge_niels_from_affine(P.X, P.Y));
}

__global__ void __launch_bounds__(64) k_from_uniform(const uint32_t* __restrict__ bytes, size_t n, uint32_t* __restrict__ tbl) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[16];
  const uint4* p = reinterpret_cast<const uint4*>(bytes + i * 16);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint4 q = p[k];
    w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
  }
  ge_p3 P = ge_from_uniform(w);
  store_niels(tbl, (uint32_t)i, ge_to_niels(P));
}

__global__ void __launch_bounds__(64) k_compress_niels(const uint32_t* __restrict__ tbl, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ge_p3 P = ge_from_niels(load_niels(tbl, (uint32_t)i));
  uint32_t w[8];
  ge_ristretto_encode(P, w);
  uint4* o = reinterpret_cast<uint4*>(out + i * 8);
  o[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__global__ void __launch_bounds__(64) k_compress_p3(const uint32_t* __restrict__ pts, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ge_p3 P = load_p3(pts, i);
  uint32_t w[8];
  ge_ristretto_encode(P, w);
  uint4* o = reinterpret_cast<uint4*>(out + i * 8);
  o[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

static unsigned grid_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

int points_compress_p3_dev(bpp_ctx* ctx, const uint32_t* d_p3, size_t n, uint8_t* d_out) {
  if (!n) return BPP_OK;
  {
    ProfScope ps(ctx, "compress");
    hipLaunchKernelGGL(k_compress_p3, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, d_p3, n, (uint32_t*)d_out);
  }
  return ctx_check_launch(ctx, "k_compress_p3");
}

int points_compress_p3(bpp_ctx* ctx, const uint32_t* d_p3, size_t n, uint8_t* out_host) {
  void* d_out = nullptr;
  BPP_TRY(ctx_ws(ctx, "compress_out", n * 32, &d_out));
  BPP_TRY(points_compress_p3_dev(ctx, d_p3, n, (uint8_t*)d_out));
  BPP_TRY(ctx_d2h(ctx, out_host, d_out, n * 32));
  return BPP_OK;
}

// Encodings of 2*P_i for n device points (P3 layout): the raw points come
// back to the host and are encoded in chunks with one field inversion each
// (h25519::encode_double_batch).  For small batches this beats the
// per-point inverse-square-root chain of k_compress_p3 (~70 us of serial
// field ops on one lane); callers compute P_i = C_i / 2 from halved scalars.
int points_double_encode_host(bpp_ctx* ctx, const uint32_t* raw, size_t n, uint8_t* out_host, uint32_t J = 1);
int points_double_encode_p3(bpp_ctx* ctx, const uint32_t* d_p3, size_t n, uint8_t* out_host) {
  if (!n) return BPP_OK;
  std::vector<uint32_t> raw(n * P3_WORDS);
  BPP_TRY(ctx_d2h(ctx, raw.data(), d_p3, n * P3_BYTES));
  return points_double_encode_host(ctx, raw.data(), n, out_host);
}

int points_double_encode_host(bpp_ctx* ctx, const uint32_t* raw, size_t n, uint8_t* out_host, uint32_t J) {
  if (!n) return BPP_OK;
  HostScope hs(ctx, "double_encode");
  const size_t chunks = std::min<size_t>(par::threads(), (n + 7) / 8);
  par::for_each(chunks, [&](size_t c) {
    const size_t b = n * c / chunks, e = n * (c + 1) / chunks;
    std::vector<h25519::ge> pts(e - b);
    if (J == 1) {
      for (size_t i = b; i < e; ++i) pts[i - b] = h25519::ge_from_dev(raw + i * P3_WORDS);
    } else {  // the J partials of each point summed eight additions a vector (ge_sum_auto)
      std::vector<h25519::ge> parts((e - b) * J);
      for (size_t k = 0; k < parts.size(); ++k) parts[k] = h25519::ge_from_dev(raw + (b * J + k) * P3_WORDS);
      h25519::ge_sum_auto(parts.data(), e - b, J, pts.data());
    }
    h25519::encode_double_batch_auto(pts.data(), e - b, out_host + 32 * b);
  });
  return BPP_OK;
}

// s / 2 mod l for canonical scalars: s even -> s >> 1, odd -> (s + l) >> 1
__global__ void __launch_bounds__(256) k_sc_halve(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                 size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  static constexpr uint32_t Lw[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0, 0, 0, 0x10000000u};
  uint32_t s[8];
  _Pragma("unroll") for (int k = 0; k < 8; ++k) s[k] = in[8 * i + k];
  const uint32_t odd = s[0] & 1u;
  uint64_t c = 0;
  _Pragma("unroll") for (int k = 0; k < 8; ++k) {
    c += (uint64_t)s[k] + (odd ? Lw[k] : 0u);
    s[k] = (uint32_t)c;
    c >>= 32;
  }
  _Pragma("unroll") for (int k = 0; k < 7; ++k) s[k] = (s[k] >> 1) | (s[k + 1] << 31);
  s[7] >>= 1;  // s + l < 2^254: no carry out
  _Pragma("unroll") for (int k = 0; k < 8; ++k) out[8 * i + k] = s[k];
}

// out[t] = in[map[t]] / 2: halving with a gather (drops terms known to be zero)
__global__ void __launch_bounds__(256) k_sc_halve_gather(const uint32_t* __restrict__ in,
                                                        const uint32_t* __restrict__ map, uint32_t* __restrict__ out,
                                                        size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sc_store(out + 8 * i, sc_half(sc_load(in + 8 * (size_t)map[i])));
}

int sc_halve_gather_dev(bpp_ctx* ctx, const uint32_t* d_in, const uint32_t* d_map, uint32_t* d_out, size_t n) {
  if (!n) return BPP_OK;
  hipLaunchKernelGGL(k_sc_halve_gather, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, d_in, d_map, d_out, n);
  return ctx_check_launch(ctx, "k_sc_halve_gather");
}

int sc_halve_dev(bpp_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, size_t n) {
  if (!n) return BPP_OK;
  hipLaunchKernelGGL(k_sc_halve, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, d_in, d_out, n);
  return ctx_check_launch(ctx, "k_sc_halve");
}

extern "C" {

int bpp_points_decompress(bpp_ctx* ctx, const uint8_t* enc, size_t n, bpp_points** out, size_t* bad_index) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !out || (!enc && n)) return BPP_ERR_ARG;
    *out = nullptr;
    BPP_HIP(hipSetDevice(ctx->device));
    bpp_points* P = new bpp_points();
    P->ctx = ctx;
    P->n = n;
    if (hipMalloc(&P->d, (n ? n : 1) * MSM_NIELS_WORDS * 4) != hipSuccess) {
      delete P;
      ctx->err = "hipMalloc point table";
      return BPP_ERR_NOMEM;
    }
    void* d_enc = nullptr;
    void* d_bad = nullptr;
    int rc = BPP_OK;
    if (n) {
      rc = ctx_ws(ctx, "dec_in", n * 32, &d_enc);
      if (!rc) rc = ctx_ws(ctx, "dec_bad", 8, &d_bad);
      if (!rc) {
        unsigned long long init = ~0ull;
        hipMemcpyAsync(d_enc, enc, n * 32, hipMemcpyHostToDevice, ctx->stream);
        hipMemcpyAsync(d_bad, &init, 8, hipMemcpyHostToDevice, ctx->stream);
        {
          ProfScope ps(ctx, "decompress");
          hipLaunchKernelGGL(k_decompress, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, (const uint32_t*)d_enc, n,
                             P->d, (unsigned long long*)d_bad);
        }
        rc = ctx_check_launch(ctx, "k_decompress");
        unsigned long long bad = ~0ull;
        if (!rc && hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) rc = BPP_ERR_DEVICE;
        if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = BPP_ERR_DEVICE;
        if (!rc && bad != ~0ull) {
          if (bad_index) *bad_index = (size_t)bad;
          ctx->err = "invalid ristretto encoding at index " + std::to_string(bad);
          rc = BPP_ERR_DECOMPRESS;
        }
      }
    }
    if (rc) {
      hipFree(P->d);
      delete P;
      return rc;
    }
    *out = P;
    return BPP_OK;
  });
}

int bpp_points_from_uniform(bpp_ctx* ctx, const uint8_t* bytes64, size_t n, bpp_points** out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !out || (!bytes64 && n)) return BPP_ERR_ARG;
    *out = nullptr;
    BPP_HIP(hipSetDevice(ctx->device));
    bpp_points* P = new bpp_points();
    P->ctx = ctx;
    P->n = n;
    if (hipMalloc(&P->d, (n ? n : 1) * MSM_NIELS_WORDS * 4) != hipSuccess) {
      delete P;
      ctx->err = "hipMalloc point table";
      return BPP_ERR_NOMEM;
    }
    if (n) {
      void* d_in = nullptr;
      int rc = ctx_ws(ctx, "uni_in", n * 64, &d_in);
      if (rc) {
        hipFree(P->d);
        delete P;
        return rc;
      }
      BPP_HIP(hipMemcpyAsync(d_in, bytes64, n * 64, hipMemcpyHostToDevice, ctx->stream));
      {
        ProfScope ps(ctx, "from_uniform");
        hipLaunchKernelGGL(k_from_uniform, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, (const uint32_t*)d_in, n,
                           P->d);
      }
      BPP_TRY(ctx_check_launch(ctx, "k_from_uniform"));
      BPP_TRY(ctx_sync(ctx));
    }
    *out = P;
    return BPP_OK;
  });
}

int bpp_points_compress(bpp_ctx* ctx, const bpp_points* pts, uint8_t* out) {
  return bpp_guard(ctx, [&]() -> int {
    if (!ctx || !pts || (!out && pts->n)) return BPP_ERR_ARG;
    if (!pts->n) return BPP_OK;
    void* d_out = nullptr;
    BPP_TRY(ctx_ws(ctx, "compress_out", pts->n * 32, &d_out));
    {
      ProfScope ps(ctx, "compress");
      hipLaunchKernelGGL(k_compress_niels, dim3(grid_for(pts->n, 64)), dim3(64), 0, ctx->stream, pts->d, pts->n,
                         (uint32_t*)d_out);
    }
    BPP_TRY(ctx_check_launch(ctx, "k_compress_niels"));
    BPP_HIP(hipMemcpyAsync(out, d_out, pts->n * 32, hipMemcpyDeviceToHost, ctx->stream));
    BPP_TRY(ctx_sync(ctx));
    return BPP_OK;
  });
}

size_t bpp_points_len(const bpp_points* pts) { return pts ? pts->n : 0; }

void bpp_points_destroy(bpp_points* pts) {
  if (!pts) return;
  hipSetDevice(pts->ctx->device);
  hipFree(pts->d);
  delete pts;
}

}  // extern "C"
