// Direct-table MSM lane walk and block tree (shared by k_dt_msm,
// msm_kernels.cuh, and the fused IPA round, ipa.hip).
//
// Digits in closed form: with K = sum_{w < W-1} 2^(c w + c - 1) (host,
// DtGeom::K), field w of s + K minus H is signed digit w in [-H, H) for
// w < W - 1 and field W - 1 the top digit (>= 0; s < 2^253 so s + K < 2^254),
// the digits of a carry-propagating signed recoding without the carry chain.
//
// One block per MSM, blockDim = W * TG lanes: lane (tg, w) owns WINDOW w of
// terms tg, tg + TG, tg + 2 TG, ... -- the window is fixed per lane, so the
// digit is a fixed bit field of s + K (no per-entry division or scan), and
// the W lanes sharing a term read the same 32 scalar bytes.  Then an LDS
// tree over the block's lanes.
#pragma once
#include "ge_io.cuh"

struct DtGeom {
  uint32_t c, W, H;  // window bits, windows, rows per window (2^(c-1))
  uint32_t K[8];     // sum_{w < W-1} 2^(c w + c - 1), little-endian words
};
#define DT_NT_MAX 256
// (145 VGPRs, 3 waves per SIMD; capping the direct-table kernels at 128 for
// a fourth spilled 124 B per lane and measured 104-120 K vs 147-151 K
// proofs/s at 12 batches in flight)

// Term groups per block (TG, lanes = TG * W) for a launch of `nmsm` MSMs:
// at most DT_TG_DEFAULT (8: 128 lanes at c = 16) when the launch has blocks
// enough to fill the device (>= 256 MSMs; a few long MSMs keep 16 groups for
// latency), fewer for short MSMs; BPP_DT_TG_MAX overrides the cap (an A/B
// switch).  Fewer lanes per MSM mean a shallower block tree and
// less issue per MSM but a longer walk per lane.  256-proof batches, 52-card
// proofs (tools/prove_inflight_exp.py): at 12 in flight with the host the
// bottleneck, 16 / 8 / 4 / 2 groups measured 263-265 / 265 / 244 / 168-171 K
// proofs/s; once the IFMA host encoder made the prover GPU-bound (16 in
// flight), 8 groups beat 16 in three of three interleaved pairs (321-324 vs
// 310-317 K) and 4 lost (285-287 K).
#define DT_TG_DEFAULT 8
static inline uint32_t dt_term_groups(uint32_t W, double terms_per_msm, uint32_t nmsm) {
  uint32_t TG = DT_NT_MAX / W;
  if (nmsm >= 256 && TG > DT_TG_DEFAULT) TG = DT_TG_DEFAULT;
  if (const char* e = getenv("BPP_DT_TG_MAX")) {
    const int v = atoi(e);
    if (v >= 1 && (uint32_t)v <= DT_NT_MAX / W) TG = (uint32_t)v;
  }
  while (TG > 1 && terms_per_msm < 2.0 * TG) TG >>= 1;
  return TG;
}

FE_INLINE uint32_t sel8(const uint32_t v[8], uint32_t i) {  // v[i], 0 for i >= 8 (no scratch)
  uint32_t r = 0;
  _Pragma("unroll") for (uint32_t k = 0; k < 8; ++k) r = i == k ? v[k] : r;
  return r;
}

// Table row of window w of a term (scalar s, generator gen); d = 0 gives
// row of |d| = 1 and zero = true (the caller adds the identity instead).
struct DtLane {
  uint32_t w, wi, sh, fmask, W, H;
  bool top;
  FE_INLINE static DtLane make(const DtGeom& g, uint32_t w) {
    DtLane ln;
    ln.w = w;
    ln.wi = (g.c * w) >> 5;
    ln.sh = (g.c * w) & 31;
    ln.fmask = (1u << g.c) - 1u;
    ln.W = g.W;
    ln.H = g.H;
    ln.top = w + 1 == g.W;
    return ln;
  }
  FE_INLINE void row_of(const DtGeom& g, const uint32_t sc[8], uint32_t gen, uint32_t& row, bool& neg,
                        bool& zero) const {
    uint32_t s[8];
    uint64_t c = 0;
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {
      c += (uint64_t)sc[i] + g.K[i];
      s[i] = (uint32_t)c;
      c >>= 32;
    }
    const uint32_t lo = sel8(s, wi), hi = sel8(s, wi + 1);
    const uint32_t f = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & fmask;
    const int d = top ? (int)f : (int)f - (int)H;
    const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
    zero = ad == 0;
    neg = d < 0;
    row = (gen * W + w) * H + (zero ? 0u : ad - 1u);
  }
  // (VQ walks) a virtual term gen = 2^31 | v: lane w adds row qrow0 + b,
  // b = v W + w, when bit b of the term's scalar is set -- the 253 doublings
  // 2^b Q of a point with no direct table, as Niels rows from qrow0
  FE_INLINE void row_of_q(const uint32_t sc[8], uint32_t gen, uint32_t qrow0, uint32_t& row, bool& neg,
                          bool& zero) const {
    const uint32_t b = (gen & 0xffffu) * W + w;
    zero = b >= 253u || !((sel8(sc, b >> 5) >> (b & 31)) & 1u);
    neg = false;
    row = qrow0 + (b < 253u ? b : 0u);
  }
  template <bool VQ>
  FE_INLINE void row_any(const DtGeom& g, const uint32_t sc[8], uint32_t gen, uint32_t qrow0, uint32_t& row,
                         bool& neg, bool& zero) const {
    if (VQ && (gen >> 31))
      row_of_q(sc, gen, qrow0, row, neg, zero);
    else
      row_of(g, sc, gen, row, neg, zero);
  }
};

// One lane's walk over terms t, t + TG, ... < t1 (src(t, s, gen) supplies
// a term's scalar words and generator index).  Software pipeline: the scalar
// and generator index of the term after next are loaded one whole addition
// ahead, and the next term's 128-B table row is gathered between the two
// halves of the current addition (the operand is dead after its first three
// multiplies).  A zero digit adds the identity (no divergent skip).
// VQ: terms may be virtual (DtLane::row_of_q, rows from qrow0).
template <bool VQ = false, class Src>
FE_INLINE ge_p3 dt_walk(const uint32_t* __restrict__ dt, const DtGeom& dg, const DtLane& ln, uint32_t t, uint32_t t1,
                        uint32_t TG, const Src& src, const ge_p3& acc0 = ge_identity(), uint32_t qrow0 = 0) {
  ge_p3 acc = acc0;  // (a lane's starting point: the identity, or an extra term's point)
  if (t >= t1) return acc;
  uint32_t sc[8];
  uint32_t gen;
  src(t, sc, gen);
  uint32_t tn = t + TG;
  uint32_t scn[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t genn = 0;
  if (tn < t1) src(tn, scn, genn);
  uint32_t row;
  bool neg, zero;
  ln.row_any<VQ>(dg, sc, gen, qrow0, row, neg, zero);
  ge_niels q = load_niels(dt, row);
  for (;;) {
    if (zero) q = ge_niels_identity();
    const ge_madd_mid mid = ge_madd_signed_h1(acc, q, neg);
    const bool more = tn < t1;
    bool neg2 = false, zero2 = false;
    if (more) {
      uint32_t row2;
      ln.row_any<VQ>(dg, scn, genn, qrow0, row2, neg2, zero2);
      q = load_niels(dt, row2);
      tn += TG;
      if (tn < t1) src(tn, scn, genn);
    }
    acc = ge_madd_h2(mid);
    if (!more) break;
    neg = neg2;
    zero = zero2;
  }
  return acc;
}

// Extended points in LDS as 10 planes of 16-byte chunks (chunk i of slot j
// at plane i, position j): consecutive lanes touch consecutive 16 B, where
// the 160-B-per-point layout of store_p3 put 4 lanes on the same banks (PMC:
// ~2.7 LDS bank conflicts per LDS instruction in the trees).
FE_INLINE void lds_store_p3(uint32_t* tl, uint32_t nslots, uint32_t j, const ge_p3& r) {
  uint32_t w[40];
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    w[i] = r.X.v[i];
    w[10 + i] = r.Y.v[i];
    w[20 + i] = r.Z.v[i];
    w[30 + i] = r.T.v[i];
  }
  uint4* p = reinterpret_cast<uint4*>(tl);
  const uint4* q = reinterpret_cast<const uint4*>(w);
  _Pragma("unroll") for (int i = 0; i < 10; ++i) p[(size_t)i * nslots + j] = q[i];
}
FE_INLINE ge_p3 lds_load_p3(const uint32_t* tl, uint32_t nslots, uint32_t j) {
  const uint4* p = reinterpret_cast<const uint4*>(tl);
  uint4 q[10];
  _Pragma("unroll") for (int i = 0; i < 10; ++i) q[i] = p[(size_t)i * nslots + j];
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

// Quad exchange: lane l reads lane (l & ~3) | ((l & 3) ^ X) of its own quad
// (DPP quad_perm, no LDS round trip).
template <int X>
FE_INLINE fe fe_quad_xor(const fe& a) {
  constexpr int ctrl = ((0 ^ X) << 0) | ((1 ^ X) << 2) | ((2 ^ X) << 4) | ((3 ^ X) << 6);
  fe r;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) r.v[i] =
      (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], ctrl, 0xf, 0xf, false);
  return r;
}
FE_INLINE fe fe_pick(bool c, const fe& a, const fe& b) {
  fe r;
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// p + q by the four lanes of a quad, lane c = lane & 3 returning coordinate c
// (X, Y, Z, T) of the sum.  ge_add's nine multiplies are two rounds of four
// independent products plus 2d * T1T2: lane c forms product c of the first
// round (A = (Y1-X1)(Y2-X2), B = (Y1+X1)(Y2+X2), T1 T2, Z1 Z2), DPP hands each
// lane the other three, every lane forms C = 2d T1T2 and E, F, G, H, and lane
// c forms product c of the second round (EF, GH, GF, EH).  A wave spends 3
// multiplies per addition instead of 9, with every lane on the same
// instruction stream (the operands are selected, not branched on).  The
// formulas and their bounds are ge_add_cached's.
FE_INLINE fe ge_add_quad(const ge_p3& p, const ge_p3& q, uint32_t c) {
  const fe a0 = fe_pick(c == 0, fe_sub_nc(p.Y, p.X), fe_pick(c == 1, fe_add_nc(p.Y, p.X), fe_pick(c == 2, p.T, p.Z)));
  const fe b0 = fe_pick(c == 0, fe_sub_nc(q.Y, q.X), fe_pick(c == 1, fe_add_nc(q.Y, q.X), fe_pick(c == 2, q.T, q.Z)));
  const fe m0 = fe_mul(a0, b0);
  const fe m1 = fe_quad_xor<1>(m0), m2 = fe_quad_xor<2>(m0), m3 = fe_quad_xor<3>(m0);
  // product of lane t = the exchange with lane distance t ^ c
  auto prod = [&](uint32_t t) {
    const uint32_t d = t ^ c;
    return fe_pick(d == 0, m0, fe_pick(d == 1, m1, fe_pick(d == 2, m2, m3)));
  };
  const fe A = prod(0), B = prod(1), ZZ = prod(3);
  const fe C = fe_mul(prod(2), fe_const(FE_D2));
  const fe D = fe_add_nc(ZZ, ZZ);
  const fe E = fe_sub_nc(B, A), F = fe_sub(D, C), G = fe_add_nc(D, C), H = fe_add_nc(B, A);
  return fe_mul(fe_pick(c == 0 || c == 3, E, G), fe_pick(c == 0 || c == 2, F, H));
}

// Coordinate c (10 words) of slot j in lds_store_p3's layout.
FE_INLINE void lds_store_coord(uint32_t* tl, uint32_t nslots, uint32_t j, uint32_t c, const fe& v) {
  _Pragma("unroll") for (int i = 0; i < FE_LIMBS; ++i) {
    const uint32_t w = 10 * c + i;
    tl[((w >> 2) * nslots + j) * 4 + (w & 3)] = v.v[i];
  }
}

// Block tree in LDS (tl: blockDim.x extended points) over `segs` segments
// of nt / segs lanes each; lane i < segs writes segment i's sum to
// out_p3[m0 + i * mstride] when that index is below mend.  A level of s additions per segment runs one
// lane per addition while 4 segs s exceeds the block, then four lanes per
// addition (ge_add_quad): a narrow level's latency is one wave's instruction
// stream, which the quads cut by ~3x (the 8-level tree was ~29 us of each
// 80-us IPA round at 256 lanes, measured with EXP_IPA_NOTREE).  Segments
// side by side share the narrow levels' waves (the two-sided IPA round).
FE_INLINE void dt_block_tree_segs(uint32_t* tl, const ge_p3& acc, uint32_t nt, uint32_t segs,
                                  uint32_t* __restrict__ out_p3, uint32_t m0, uint32_t mstride,
                                  uint32_t mend = 0xffffffffu) {
  lds_store_p3(tl, nt, threadIdx.x, acc);
  __syncthreads();
  const uint32_t ns = nt / segs;  // lanes per segment (segs divides nt)
  uint32_t p2 = 1, lp = 0;
  while (p2 < ns) {
    p2 <<= 1;
    ++lp;
  }
  for (uint32_t s = p2 >> 1, l = lp - (lp ? 1u : 0u); s > 0; s >>= 1, --l) {
    const uint32_t na = segs * s;  // additions at this level
    if (4 * na > nt) {
      if (threadIdx.x < na) {
        const uint32_t g = threadIdx.x >> l, j = threadIdx.x & (s - 1u), a = g * ns + j;
        if (j + s < ns) lds_store_p3(tl, nt, a, ge_add(lds_load_p3(tl, nt, a), lds_load_p3(tl, nt, a + s)));
      }
    } else if ((threadIdx.x & ~63u) < 4 * na) {  // wave-uniform: whole waves run the DPP exchange
      const uint32_t i = threadIdx.x >> 2, c = threadIdx.x & 3;
      const uint32_t g = i >> l, j = i & (s - 1u), a = g * ns + j;
      const bool live = i < na && j + s < ns;
      const fe r = ge_add_quad(lds_load_p3(tl, nt, live ? a : 0), lds_load_p3(tl, nt, live ? a + s : 0), c);
      if (live) lds_store_coord(tl, nt, a, c, r);
    }
    __syncthreads();
  }
  if (threadIdx.x < segs && m0 + threadIdx.x * mstride < mend)
    store_p3(out_p3, m0 + threadIdx.x * mstride, lds_load_p3(tl, nt, threadIdx.x * ns));
}
FE_INLINE void dt_block_tree(uint32_t* tl, const ge_p3& acc, uint32_t nt, uint32_t* __restrict__ out_p3, uint32_t m) {
  dt_block_tree_segs(tl, acc, nt, 1, out_p3, m, 0);
}
