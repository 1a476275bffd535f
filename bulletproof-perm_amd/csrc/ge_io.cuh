// Load / store of table points (affine Niels) and extended points with
// 16-byte vector accesses (layout.h).
#pragma once
#include "ge25519.cuh"
#include "layout.h"

FE_INLINE ge_niels load_niels(const uint32_t* __restrict__ tbl, uint32_t idx) {
  const uint4* p = reinterpret_cast<const uint4*>(tbl + (size_t)idx * MSM_NIELS_WORDS);
  uint4 q[8];  // the whole 128-B row (words 30, 31 are padding)
  _Pragma("unroll") for (int i = 0; i < 8; ++i) q[i] = p[i];
  const uint32_t* w = reinterpret_cast<const uint32_t*>(q);
  ge_niels n;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    n.ypx.v[i] = w[i];
    n.ymx.v[i] = w[10 + i];
    n.xy2d.v[i] = w[20 + i];
  }
  return n;
}

FE_INLINE void store_niels(uint32_t* __restrict__ tbl, uint32_t idx, const ge_niels& n) {
  uint32_t w[32];
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    w[i] = n.ypx.v[i];
    w[10 + i] = n.ymx.v[i];
    w[20 + i] = n.xy2d.v[i];
  }
  w[30] = 0;
  w[31] = 0;
  uint4* p = reinterpret_cast<uint4*>(tbl + (size_t)idx * MSM_NIELS_WORDS);
  const uint4* q = reinterpret_cast<const uint4*>(w);
  _Pragma("unroll") for (int i = 0; i < 8; ++i) p[i] = q[i];
}

FE_INLINE ge_p3 load_p3(const uint32_t* __restrict__ buf, size_t idx) {
  const uint4* p = reinterpret_cast<const uint4*>(buf + idx * P3_WORDS);
  uint4 q[10];
  _Pragma("unroll") for (int i = 0; i < 10; ++i) q[i] = p[i];
  const uint32_t* w = reinterpret_cast<const uint32_t*>(q);
  ge_p3 r;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    r.X.v[i] = w[i];
    r.Y.v[i] = w[10 + i];
    r.Z.v[i] = w[20 + i];
    r.T.v[i] = w[30 + i];
  }
  return r;
}

FE_INLINE void store_p3(uint32_t* __restrict__ buf, size_t idx, const ge_p3& r) {
  uint32_t w[40];
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    w[i] = r.X.v[i];
    w[10 + i] = r.Y.v[i];
    w[20 + i] = r.Z.v[i];
    w[30 + i] = r.T.v[i];
  }
  uint4* p = reinterpret_cast<uint4*>(buf + idx * P3_WORDS);
  const uint4* q = reinterpret_cast<const uint4*>(w);
  _Pragma("unroll") for (int i = 0; i < 10; ++i) p[i] = q[i];
}
