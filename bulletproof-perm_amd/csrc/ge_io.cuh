// Load / store of table points (affine Niels, 96 B) and extended points
// (128 B) with 16-byte vector accesses.
#pragma once
#include "ge25519.cuh"

// A table point is 96 bytes of affine Niels (y+x, y-x, 2dxy) stored at a
// 128-byte stride: one 128-B memory request per gather instead of 1.5 on
// average for packed 96-B rows (tools/ubench/gather_cal: 184 B fetched per
// packed row).
#define MSM_NIELS_WORDS 32

FE_INLINE ge_niels load_niels(const uint32_t* __restrict__ tbl, uint32_t idx) {
  const uint4* p = reinterpret_cast<const uint4*>(tbl + (size_t)idx * MSM_NIELS_WORDS);
  uint4 q[6];
  _Pragma("unroll") for (int i = 0; i < 6; ++i) q[i] = p[i];
  ge_niels n;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(q);
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    n.ypx.v[i] = w[i];
    n.ymx.v[i] = w[8 + i];
    n.xy2d.v[i] = w[16 + i];
  }
  return n;
}

FE_INLINE void store_niels(uint32_t* __restrict__ tbl, uint32_t idx, const ge_niels& n) {
  uint32_t w[24];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    w[i] = n.ypx.v[i];
    w[8 + i] = n.ymx.v[i];
    w[16 + i] = n.xy2d.v[i];
  }
  uint4* p = reinterpret_cast<uint4*>(tbl + (size_t)idx * MSM_NIELS_WORDS);
  const uint4* q = reinterpret_cast<const uint4*>(w);
  _Pragma("unroll") for (int i = 0; i < 6; ++i) p[i] = q[i];
}

FE_INLINE ge_p3 load_p3(const uint32_t* __restrict__ buf, size_t idx) {
  const uint4* p = reinterpret_cast<const uint4*>(buf + idx * 32);
  uint4 q[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) q[i] = p[i];
  const uint32_t* w = reinterpret_cast<const uint32_t*>(q);
  ge_p3 r;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    r.X.v[i] = w[i];
    r.Y.v[i] = w[8 + i];
    r.Z.v[i] = w[16 + i];
    r.T.v[i] = w[24 + i];
  }
  return r;
}

FE_INLINE void store_p3(uint32_t* __restrict__ buf, size_t idx, const ge_p3& r) {
  uint32_t w[32];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    w[i] = r.X.v[i];
    w[8 + i] = r.Y.v[i];
    w[16 + i] = r.Z.v[i];
    w[24 + i] = r.T.v[i];
  }
  uint4* p = reinterpret_cast<uint4*>(buf + idx * 32);
  const uint4* q = reinterpret_cast<const uint4*>(w);
  _Pragma("unroll") for (int i = 0; i < 8; ++i) p[i] = q[i];
}

