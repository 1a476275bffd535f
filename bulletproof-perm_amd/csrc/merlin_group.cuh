// Merlin transcripts on the device, one transcript per GROUP of 8 lanes
// (merlin 3.0.0 / STROBE-128 over Keccak-f[1600]; the reference's
// TranscriptProtocol, transcript_protocol.rs:26-67).  Byte-exact with
// host/merlin.h and merlin_lane.cuh.
//
// Why groups: a batch of P proofs replays P independent transcripts of ~53
// permutations each.  With one transcript per lane (merlin_lane.cuh) the
// 4096 transcripts of config 5 are 64 waves, so the replay's time is one
// wave's instruction stream: 24 rounds x ~190 VALU instructions per
// permutation.  Here the five lanes of a group each own one column of the
// state (Keccak lanes A[x][0..4], as lo / hi halves), so a round costs a lane
// ~45 VALU and ~20 LDS instructions:
//   theta   the column parity is the lane's own five words; C[x+1] and
//           C[x-1] come from the neighbouring lanes by DPP (row_shl:1 /
//           row_shr:1, no LDS);
//   rho/pi  the lane rotates its five words by its own offsets (v_alignbit
//           with per-lane shift registers; a rotation by >= 32 is a swap of
//           the halves, folded into the LDS store addresses) and stores them
//           at their pi destinations in the group's scratch (the copies'
//           lanes into trash words past the state, so no branch);
//   chi     the lane reads back columns x, x+1, x+2 of the permuted state
//           (ds_read2_b64) and forms its new column;
//   iota    the lane of column 0 folds in the round constant.
// Group lane gl holds column x = (gl + 4) mod 5 (gl 0..7 -> 4 0 1 2 3 4 0 1):
// lanes 1..5 are the state's owners ("canonical", the only ones whose stores land)
// and every canonical lane finds C[x+1] at gl + 1 and C[x-1] at gl - 1 inside
// the same 8-lane group, so the DPP row shifts never leave the group for
// them; lanes 0, 6, 7 compute copies that nobody reads.
// The 8 lanes of a group are in one wave and LDS instructions of one wave
// execute in order, so the scratch needs no barrier -- only compiler fences
// (the cross-lane dependence is invisible to the compiler).
//
// The STROBE byte operations (absorbs, the begin_op flags, the squeeze) are
// the schedule of merlin_lane.cuh executed by the group's leader lane (GRP_LEADER)
// on the group's sponge in LDS; every lane runs the same control flow (the
// positions are uniform: a batch's transcripts have the same lengths), so the
// whole wave enters each permutation together.
#pragma once
#include "keccak_dev.cuh"
#include "merlin_lane.cuh"

#ifndef GRP_LANES
#define GRP_LANES 16  // lanes per transcript: 16 (grp_keccak16) or 8 (grp_keccak, A/B)
#endif
#define GRP_ST_BYTES 200
#ifndef GRP_TRASH
#define GRP_TRASH 60  // first trash dword of grp_keccak16 (50: the former layout, A/B)
#endif
#ifndef GRP_K16_FULL
#define GRP_K16_FULL 1  // grp_keccak16 fully unrolled (0: the rolled loop, A/B)
#endif
#ifndef GRP_PAR_APPEND
#define GRP_PAR_APPEND 0  // append32 as one parallel XOR over the group (A/B)
#endif
#ifndef GRP_CHI128
#define GRP_CHI128 1  // chi reads half-columns as 16-B + 4-B reads (0: the former dword layout, A/B)
#endif
#if GRP_CHI128 && !GRP_K16_FULL
#error "GRP_CHI128 is implemented in the unrolled grp_keccak16 only"
#endif
#if GRP_CHI128
#define GRP_SCR_OFF 208  // the pi scratch's offset in a group's block (16-B aligned for the chi reads)
#define GRP_BLOCK 736    // a group's sponge + scratch block (130 scratch dwords)
#else
#define GRP_SCR_OFF 200
#define GRP_BLOCK 576
#endif
// the pi scratch: GRP_BLOCK - GRP_SCR_OFF bytes (CHI128: 528 = 130
// half-column dwords (12 (2X + h) + row, X < 5, h < 2) + pad; the former
// dword layout: 200 bytes of state + the copies' trash words, dwords 60..69)
#define GRP_SCR_BYTES (GRP_BLOCK - GRP_SCR_OFF)

// rho offsets r[x][y] packed per y (6 bits per x) and the pi destination row
// (2x + 3y) mod 5 packed per y (3 bits per x); pi's destination column is y
__device__ __constant__ static const uint32_t GRP_RHO[5] = {
    (0u << 0) | (1u << 6) | (62u << 12) | (28u << 18) | (27u << 24),
    (36u << 0) | (44u << 6) | (6u << 12) | (55u << 18) | (20u << 24),
    (3u << 0) | (10u << 6) | (43u << 12) | (25u << 18) | (39u << 24),
    (41u << 0) | (45u << 6) | (15u << 12) | (21u << 18) | (8u << 24),
    (18u << 0) | (2u << 6) | (61u << 12) | (56u << 18) | (14u << 24)};

// (mov_dpp with bound_ctrl: lanes whose source is outside the row read 0,
// so no "old" value has to be materialised first)
FE_INLINE uint32_t grp_dpp_next(uint32_t v) {  // lane i <- lane i + 1 (row_shl:1)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xf, 0xf, true);
}
FE_INLINE uint32_t grp_dpp_prev(uint32_t v) {  // lane i <- lane i - 1 (row_shr:1)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, true);
}
#define GRP_FENCE() __asm__ volatile("" ::: "memory")

// Keccak-f[1600] on the group's sponge st (25 x u64 in the standard x + 5y
// order, LDS), with scr (200 B, LDS) as the pi scratch; called by all 8 lanes
// of the group (gl = lane within the group).
__device__ __noinline__ static void grp_keccak(lds_u64* st, lds_u64* scr, uint32_t gl) {
  const uint32_t x = (gl + 4) % 5;
  const bool canon = gl - 1u < 5u;
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  lds_u32* scr32 = (lds_u32*)scr;
  uint32_t lo[5], hi[5], c[5], wl[5], wh[5];
  _Pragma("unroll") for (int y = 0; y < 5; ++y) {
    const uint64_t v = st[x + 5 * y];
    lo[y] = (uint32_t)v;
    hi[y] = (uint32_t)(v >> 32);
    const uint32_t n = (GRP_RHO[y] >> (6 * x)) & 63u;
    const uint32_t s = n & 31u, sw = (n >> 5) ^ (s == 0 ? 1u : 0u);
    c[y] = (32u - s) & 31u;
    const uint32_t Y = (2 * x + 3 * y) % 5;
    // dword index of the destination word (column y, row Y); the copies'
    // lanes store into the trash words past the state (no branch per round)
    const uint32_t off = canon ? 2 * (5 * y + Y) : 50 + 2 * y;
    wl[y] = off + sw;
    wh[y] = off + (sw ^ 1u);
  }
  const uint32_t c0 = 5 * x, c1 = 5 * ((x + 1) % 5), c2 = 5 * ((x + 2) % 5);  // u64 index of columns
  const uint32_t ms = x == 0 ? ~0u : 0u;
  _Pragma("unroll 2") for (int r = 0; r < 24; ++r) {
    // theta
    const uint32_t cl = xor3(xor3(lo[0], lo[1], lo[2]), lo[3], lo[4]);
    const uint32_t ch = xor3(xor3(hi[0], hi[1], hi[2]), hi[3], hi[4]);
    const uint32_t nl = grp_dpp_next(cl), nh = grp_dpp_next(ch);
    const uint32_t pl = grp_dpp_prev(cl), ph = grp_dpp_prev(ch);
    const uint32_t dl = pl ^ __builtin_amdgcn_alignbit(nl, nh, 31);
    const uint32_t dh = ph ^ __builtin_amdgcn_alignbit(nh, nl, 31);
    // rho + pi: rotated words to their destinations (halves swapped there
    // for rotations by >= 32)
    GRP_FENCE();
    _Pragma("unroll") for (int y = 0; y < 5; ++y) {
      const uint32_t a = lo[y] ^ dl, b = hi[y] ^ dh;
      scr32[wl[y]] = __builtin_amdgcn_alignbit(a, b, c[y]);
      scr32[wh[y]] = __builtin_amdgcn_alignbit(b, a, c[y]);
    }
    GRP_FENCE();
    // chi over columns x, x + 1, x + 2 of the permuted state
    _Pragma("unroll") for (int y = 0; y < 5; ++y) {
      const uint64_t b0 = scr[c0 + y], b1 = scr[c1 + y], b2 = scr[c2 + y];
      const uint32_t b0l = (uint32_t)b0, b0h = (uint32_t)(b0 >> 32), b1l = (uint32_t)b1, b1h = (uint32_t)(b1 >> 32),
                     b2l = (uint32_t)b2, b2h = (uint32_t)(b2 >> 32);
      lo[y] = b0l ^ (~b1l & b2l);
      hi[y] = b0h ^ (~b1h & b2h);
    }
    GRP_FENCE();
    // iota (column 0's lanes)
    lo[0] ^= (uint32_t)KECCAK_RC[r] & ms;
    hi[0] ^= (uint32_t)(KECCAK_RC[r] >> 32) & ms;
  }
  if (canon) {
    _Pragma("unroll") for (int y = 0; y < 5; ++y) st[x + 5 * y] = ((uint64_t)hi[y] << 32) | lo[y];
  }
}

// The same permutation on 16-lane groups, each of the five columns on a PAIR
// of lanes (lane 2j + h holds half h -- lo / hi -- of column x = (j + 4) mod
// 5, pairs j = 1..5 canonical): a round costs a lane ~45 instructions instead
// of ~68 (5 words' halves instead of 10 dwords; the rotation takes the other
// half from the partner lane by DPP quad_perm), one transcript per 16 lanes.
template <int CTRL>
FE_INLINE uint32_t grp_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}
__device__ __noinline__ static void grp_keccak16(lds_u64* st, lds_u64* scr, uint32_t gl) {
  const uint32_t j = gl >> 1, h = gl & 1u;
  const uint32_t x = (j + 4) % 5;
  const bool canon = j - 1u < 5u;
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  lds_u32* scr32 = (lds_u32*)scr;
  const lds_u32* st32 = (const lds_u32*)st;
  uint32_t a[5], c[5], w[5], rd[3];
  const uint32_t cm = canon ? ~0u : 0u, hm = h ? ~0u : 0u;
  _Pragma("unroll") for (int y = 0; y < 5; ++y) {
    a[y] = st32[2 * (x + 5 * y) + h];
    const uint32_t n = (GRP_RHO[y] >> (6 * x)) & 63u;
    const uint32_t s = n & 31u, sw = (n >> 5) ^ (s == 0 ? 1u : 0u);
    c[y] = (32u - s) & 31u;
    const uint32_t Y = (2 * x + 3 * y) % 5;
    // (copies: trash dwords 60..69, placed so that they share no bank with
    // the same instruction's state stores, tools/lds_banks.py)
#if GRP_CHI128
    // (half-column layout: half h of column X at dwords 12 (2 X + h) + row;
    // the copies' trash words past them)
    const uint32_t wc = 12 * (2 * y + (sw ^ h)) + Y, wt = 120 + 2 * y + h;
#else
    const uint32_t wc = 2 * (5 * y + Y) + (sw ^ h), wt = GRP_TRASH + 2 * y + h;
#endif
    w[y] = (wc & cm) | (wt & ~cm);
  }
#if GRP_CHI128
  rd[0] = 12 * (2 * x + h);
  rd[1] = 12 * (2 * ((x + 1) % 5) + h);
  rd[2] = 12 * (2 * ((x + 2) % 5) + h);
#else
  rd[0] = 10 * x + h;
  rd[1] = 10 * ((x + 1) % 5) + h;
  rd[2] = 10 * ((x + 2) % 5) + h;
#endif
  const uint32_t ms = x == 0 ? ~0u : 0u;
#if GRP_K16_FULL
  // All 24 rounds unrolled with the round constants as literals: iota is one
  // XOR on the chain (its lane-dependent constant is formed off the chain),
  // and the rounds carry no scalar-memory load of KECCAK_RC -- whose
  // s_load shared the lgkmcnt wait of the chi reads -- and no loop counter;
  // rho/pi issues the five XORs, then the five DPP moves, then the rotates
  // and stores, so no DPP waits on the XOR just before it (s_nop 1 each).
  constexpr uint64_t RC[24] = {
      0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
      0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
      0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
      0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
      0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
      0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
  _Pragma("unroll") for (int r = 0; r < 24; ++r) {
    const uint32_t cc = xor3(xor3(a[0], a[1], a[2]), a[3], a[4]);
    const uint32_t cp_same = grp_dpp<0x102>(cc);
    const uint32_t o1 = grp_dpp<0x101>(cc), o3 = grp_dpp<0x103>(cc);
    const uint32_t cp_other = o3 ^ ((o1 ^ o3) & hm);
    const uint32_t cm_same = grp_dpp<0x112>(cc);
    const uint32_t d = cm_same ^ __builtin_amdgcn_alignbit(cp_same, cp_other, 31);
    uint32_t v[5], pv[5];
    _Pragma("unroll") for (int y = 0; y < 5; ++y) v[y] = a[y] ^ d;
    _Pragma("unroll") for (int y = 0; y < 5; ++y) pv[y] = grp_dpp<0xB1>(v[y]);
    GRP_FENCE();
    _Pragma("unroll") for (int y = 0; y < 5; ++y) scr32[w[y]] = __builtin_amdgcn_alignbit(v[y], pv[y], c[y]);
    GRP_FENCE();
#if GRP_CHI128
    {
      // each half-column as one 16-B read (rows 0..3) and one dword (row 4)
      typedef uint32_t grp_v4 __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(3))) grp_v4 lds_v4;
      uint32_t b[3][5];
      _Pragma("unroll") for (int k = 0; k < 3; ++k) {
        const grp_v4 q = *(const lds_v4*)(scr32 + rd[k]);
        b[k][0] = q.x;
        b[k][1] = q.y;
        b[k][2] = q.z;
        b[k][3] = q.w;
        b[k][4] = scr32[rd[k] + 4];
      }
      _Pragma("unroll") for (int y = 0; y < 5; ++y) a[y] = b[0][y] ^ (~b[1][y] & b[2][y]);
    }
#else
    _Pragma("unroll") for (int y = 0; y < 5; ++y) {
      const uint32_t b0 = scr32[rd[0] + 2 * y], b1 = scr32[rd[1] + 2 * y], b2 = scr32[rd[2] + 2 * y];
      a[y] = b0 ^ (~b1 & b2);
    }
#endif
    GRP_FENCE();
    const uint32_t rl = (uint32_t)RC[r], rh = (uint32_t)(RC[r] >> 32);
    a[0] ^= (rl ^ ((rl ^ rh) & hm)) & ms;
  }
#else
  _Pragma("unroll 2") for (int r = 0; r < 24; ++r) {
    // theta: this half's column parity; the neighbours' from the pairs beside
    const uint32_t cc = xor3(xor3(a[0], a[1], a[2]), a[3], a[4]);
    const uint32_t cp_same = grp_dpp<0x102>(cc);                      // lane + 2: C[x+1], this half
    const uint32_t o1 = grp_dpp<0x101>(cc), o3 = grp_dpp<0x103>(cc);
    const uint32_t cp_other = o3 ^ ((o1 ^ o3) & hm);  // C[x+1], the other half (lane + 1 or + 3)
    const uint32_t cm_same = grp_dpp<0x112>(cc);                      // lane - 2: C[x-1], this half
    const uint32_t d = cm_same ^ __builtin_amdgcn_alignbit(cp_same, cp_other, 31);
    GRP_FENCE();
    _Pragma("unroll") for (int y = 0; y < 5; ++y) {
      const uint32_t v = a[y] ^ d;
      const uint32_t pv = grp_dpp<0xB1>(v);  // the partner lane's half (quad_perm 1,0,3,2)
      scr32[w[y]] = __builtin_amdgcn_alignbit(v, pv, c[y]);
    }
    GRP_FENCE();
    _Pragma("unroll") for (int y = 0; y < 5; ++y) {
      const uint32_t b0 = scr32[rd[0] + 2 * y], b1 = scr32[rd[1] + 2 * y], b2 = scr32[rd[2] + 2 * y];
      a[y] = b0 ^ (~b1 & b2);
    }
    GRP_FENCE();
    const uint64_t rc = KECCAK_RC[r];
    const uint32_t rl = (uint32_t)rc, rh = (uint32_t)(rc >> 32);
    a[0] ^= (rl ^ ((rl ^ rh) & hm)) & ms;
  }
#endif
  if (canon) {
    lds_u32* stw = (lds_u32*)st;
    _Pragma("unroll") for (int y = 0; y < 5; ++y) stw[2 * (x + 5 * y) + h] = a[y];
  }
}

#define GRP_LEADER 2  // a canonical lane of either layout (8: gl 1..5, 16: gl 2..11)

// The STROBE-128 schedule of LaneStrobe (merlin_lane.cuh) for a group: byte
// operations by the leader lane, permutations by the whole group.
struct GroupStrobe {
  uint8_t* st;   // the group's 200-byte sponge (LDS)
  uint8_t* scr;  // the group's pi scratch (LDS)
  uint32_t gl;   // lane within the group
  bool leader;   // gl == GRP_LEADER
  uint32_t pos, pos_begin;

  FE_INLINE void run_f() {
    if (leader) {
      st[pos] ^= (uint8_t)pos_begin;
      st[pos + 1] ^= 0x04;
      st[LANE_STROBE_R + 1] ^= 0x80;
    }
#if GRP_LANES == 16
    grp_keccak16((lds_u64*)st, (lds_u64*)scr, gl);
#else
    grp_keccak((lds_u64*)st, (lds_u64*)scr, gl);
#endif
    pos = 0;
    pos_begin = 0;
  }
  FE_INLINE void absorb_byte(uint32_t b) {
    if (leader) st[pos] ^= (uint8_t)b;
    if (++pos == LANE_STROBE_R) run_f();
  }
  FE_INLINE void absorb_bytes(const uint8_t* d, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) absorb_byte(d[i]);
  }
  FE_INLINE void absorb_le32(uint32_t x) {
    absorb_byte(x & 0xffu);
    absorb_byte((x >> 8) & 0xffu);
    absorb_byte((x >> 16) & 0xffu);
    absorb_byte(x >> 24);
  }
  // 32 bytes as 8 little-endian words (valid in the leader lane)
  FE_INLINE void absorb32(const uint32_t w[8]) {
    if (pos + 32 < LANE_STROBE_R) {
      if (leader) {
        uint32_t* d = reinterpret_cast<uint32_t*>(st) + (pos >> 2);
        const uint32_t sh = 8 * (pos & 3);
        if (sh == 0) {
          _Pragma("unroll") for (int i = 0; i < 8; ++i) d[i] ^= w[i];
        } else {
          d[0] ^= w[0] << sh;
          _Pragma("unroll") for (int i = 1; i < 8; ++i) d[i] ^= __builtin_amdgcn_alignbit(w[i], w[i - 1], 32 - sh);
          d[8] ^= w[7] >> (32 - sh);
        }
      }
      pos += 32;
      return;
    }
    _Pragma("unroll") for (int i = 0; i < 8; ++i) absorb_le32(w[i]);
  }
  FE_INLINE void begin_op(uint32_t flags) {
    const uint32_t old_begin = pos_begin;
    pos_begin = pos + 1;
    absorb_byte(old_begin);
    absorb_byte(flags);
    if ((flags & (4u | 32u)) && pos != 0) run_f();  // FLAG_C | FLAG_K
  }
  FE_INLINE void meta(const char* label, uint32_t ln, uint32_t n) {
    begin_op(16u | 2u);  // FLAG_M | FLAG_A
    absorb_bytes(reinterpret_cast<const uint8_t*>(label), ln);
    absorb_le32(n);
  }
  // the framing bytes of append_message(label, n-byte message) before the
  // message: begin_op(M | A), the label, le32(n), begin_op(A) -- when they
  // and the message end before the rate, one branch-free run of byte XORs
  // (the leader's LDS read-modify-writes then pipeline instead of paying the
  // LDS latency byte by byte between the rate checks)
  // (flags2: the second begin_op's flags, FLAG_A for a message; FLAG_I |
  // FLAG_A | FLAG_C for a challenge, whose permutation the caller runs)
  FE_INLINE bool frame_fast(const char* label, uint32_t ln, uint32_t n, uint32_t flags2 = 2u) {
    const uint32_t fl = 2 + ln + 4 + 2;
    if (pos + fl + (flags2 == 2u ? n : 0u) >= LANE_STROBE_R) return false;
    if (leader) {
      uint8_t* d = st + pos;
      d[0] ^= (uint8_t)pos_begin;
      d[1] ^= 18u;  // FLAG_M | FLAG_A
      for (uint32_t i = 0; i < ln; ++i) d[2 + i] ^= (uint8_t)label[i];
      d[2 + ln] ^= (uint8_t)n;
      d[3 + ln] ^= (uint8_t)(n >> 8);
      d[4 + ln] ^= (uint8_t)(n >> 16);
      d[5 + ln] ^= (uint8_t)(n >> 24);
      d[6 + ln] ^= (uint8_t)(pos + 1);  // the second begin_op: the old begin is this meta's
      d[7 + ln] ^= (uint8_t)flags2;
    }
    pos_begin = pos + 7 + ln;  // (the second begin_op at byte pos + 6 + ln)
    pos += fl;
    return true;
  }
#if GRP_PAR_APPEND
  // append_message(label, 32 bytes) when the framing and the message end
  // before the rate, as ONE XOR of the 8 + ln framing bytes and the message
  // into the sponge by the group's lanes, a dword each (lane gl: sponge dword
  // (pos >> 2) + gl), instead of the leader's byte and dword read-modify-
  // writes one after another; msg = the message's 8 words, readable by every
  // lane (the staged proof bytes).  Byte-identical to frame_fast + absorb32.
  FE_INLINE bool append32_par(const char* label, uint32_t ln, const uint32_t* msg) {
    const uint32_t fl = 8 + ln;
    if (pos + fl + 32 >= LANE_STROBE_R) return false;
    uint32_t FD[3] = {0u, 0u, 0u};  // the framing bytes, little-endian
    auto putb = [&](uint32_t i, uint32_t v) { FD[i >> 2] |= (v & 0xffu) << (8 * (i & 3)); };
    putb(0, pos_begin);
    putb(1, 18u);  // FLAG_M | FLAG_A
    for (uint32_t i = 0; i < ln; ++i) putb(2 + i, (uint8_t)label[i]);
    putb(2 + ln, 32u);   // le32(32)
    putb(6 + ln, pos + 1);  // the second begin_op: the old begin is this meta's
    putb(7 + ln, 2u);       // FLAG_A
    const uint32_t o = pos & 3u, g = gl;
    const uint32_t fcur = g == 0 ? FD[0] : g == 1 ? FD[1] : g == 2 ? FD[2] : 0u;
    const uint32_t fprev = g == 1 ? FD[0] : g == 2 ? FD[1] : g == 3 ? FD[2] : 0u;
    uint32_t M = o ? __builtin_amdgcn_alignbit(fcur, fprev, 32 - 8 * o) : fcur;
    // the message bytes v .. v + 3 of this lane's dword (v may be negative)
    const int v = (int)(4 * g) - (int)o - (int)fl;
    const int qd = v >> 2;
    const uint32_t r = (uint32_t)v & 3u;
    const uint32_t lo = (qd >= 0 && qd < 8) ? msg[qd] : 0u;
    const uint32_t hi = (qd + 1 >= 0 && qd + 1 < 8) ? msg[qd + 1] : 0u;
    M |= __builtin_amdgcn_alignbit(hi, lo, 8 * r);
    if (g < 12) {  // (8 + 3 + 32 bytes from offset pos & 3: at most 12 dwords)
      typedef __attribute__((address_space(3))) uint32_t lds_u32;
      lds_u32* d = (lds_u32*)st + (pos >> 2) + g;
      *d ^= M;
    }
    pos_begin = pos + 7 + ln;
    pos += fl + 32;
    return true;
  }
#endif
  FE_INLINE void append32(const char* label, uint32_t ln, const uint32_t w[8]) {
    if (frame_fast(label, ln, 32)) {
      absorb32(w);
      return;
    }
    meta(label, ln, 32);
    begin_op(2u);  // FLAG_A
    absorb32(w);
  }
  FE_INLINE void append_bytes(const char* label, uint32_t ln, const uint8_t* msg, uint32_t n) {
    meta(label, ln, n);
    begin_op(2u);
    absorb_bytes(msg, n);
  }
  FE_INLINE void append_u64(const char* label, uint32_t ln, uint64_t x) {
    meta(label, ln, 8);
    begin_op(2u);
    absorb_le32((uint32_t)x);
    absorb_le32((uint32_t)(x >> 32));
  }
  // challenge_bytes(label, 64): the 16 squeezed words to out (16 x u32,
  // written by the leader; global memory), the rate's first 64 bytes cleared
  FE_INLINE void challenge64_to(const char* label, uint32_t ln, uint32_t* __restrict__ out, bool store) {
    if (frame_fast(label, ln, 64, 1u | 2u | 4u)) {
      run_f();  // (begin_op(C) with pos != 0)
    } else {
      meta(label, ln, 64);
      begin_op(1u | 2u | 4u);  // FLAG_I | FLAG_A | FLAG_C
    }
    if (leader) {
      uint4* d = reinterpret_cast<uint4*>(st);
      _Pragma("unroll") for (int i = 0; i < 4; ++i) {
        const uint4 v = d[i];
        if (store) reinterpret_cast<uint4*>(out)[i] = v;
        d[i] = make_uint4(0, 0, 0, 0);
      }
    }
    pos = 64;
  }
};
