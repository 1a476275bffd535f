// Host-side code of libbpperm under AddressSanitizer + UBSan and under
// ThreadSanitizer ("Host C++ under ASan/UBSan"), built and run
// by tests/test_host_sanitizers.py on the CPU.  Exercises what the GPU path
// leans on between launches:
//   - merlin / STROBE transcripts (the KAT), the 8-way AVX-512 Keccak and
//     TranscriptX8 against eight scalar transcripts, SHAKE256 x8;
//   - the prover's random draws (x8 vs scalar, u64 and 32-byte seeds);
//   - scalar arithmetic mod l (invert, batch_invert, from_wide);
//   - the host field / group (encode, decode, encode_double_batch);
//   - the circuit build and sparse z^Q W;
//   - the persistent thread pool (host/par.h): nested and concurrent callers.
// Exit 0 and "ok" on success.
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "host/fe64.h"
#include "host/merlin.h"
#include "host/par.h"
#include "host/perm.h"
#include "host/scalar.h"

#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      fprintf(stderr, "FAILED line %d: %s\n", __LINE__, #c); \
      return 1;                                               \
    }                                                         \
  } while (0)

static bool hexeq(const uint8_t* b, size_t n, const char* hex) {
  char buf[256];
  for (size_t i = 0; i < n; ++i) snprintf(buf + 2 * i, 3, "%02x", b[i]);
  return strcmp(buf, hex) == 0;
}

static int test_transcripts() {
  merlin::Transcript t((const uint8_t*)"test protocol", 13);
  t.append("some label", (const uint8_t*)"some data", 9);
  uint8_t ch[32];
  t.challenge_bytes("challenge", ch, 32);
  CHECK(hexeq(ch, 32, "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"));
  if (!merlin::keccak_x8_available()) return 0;
  // eight transcripts in lockstep vs alone, messages longer than the rate
  std::vector<merlin::Transcript> a, b;
  for (int j = 0; j < 8; ++j) {
    a.emplace_back((const uint8_t*)"x8", 2);
    b.emplace_back((const uint8_t*)"x8", 2);
  }
  std::vector<uint8_t> msg(8 * 300);
  for (size_t i = 0; i < msg.size(); ++i) msg[i] = (uint8_t)(i * 131 + 7);
  merlin::Transcript* tp[8];
  const uint8_t* mp[8];
  for (int j = 0; j < 8; ++j) {
    tp[j] = &b[j];
    mp[j] = msg.data() + 300 * j;
  }
  merlin::TranscriptX8 x;
  CHECK(x.load(tp));
  for (int r = 0; r < 3; ++r) x.append("V", mp, 300);
  hsc::Sc sx[8];
  x.challenge_scalar("c", sx);
  x.store(tp);
  for (int j = 0; j < 8; ++j) {
    for (int r = 0; r < 3; ++r) a[j].append("V", mp[j], 300);
    const hsc::Sc s1 = a[j].challenge_scalar("c");
    CHECK(memcmp(&s1, &sx[j], 32) == 0);
    uint8_t c1[40], c2[40];
    a[j].challenge_bytes("d", c1, 40);
    b[j].challenge_bytes("d", c2, 40);
    CHECK(memcmp(c1, c2, 40) == 0);
  }
  // SHAKE256 x8 vs one at a time
  uint8_t in[8][37], out8[8][500], out1[500];
  const uint8_t* ip[8];
  uint8_t* op[8];
  for (int j = 0; j < 8; ++j) {
    for (int i = 0; i < 37; ++i) in[j][i] = (uint8_t)(j * 37 + i);
    ip[j] = in[j];
    op[j] = out8[j];
  }
  merlin::shake256_x8(ip, 37, op, 500);
  for (int j = 0; j < 8; ++j) {
    merlin::Shake256 sh;
    sh.update(in[j], 37);
    sh.read(out1, 500);
    CHECK(memcmp(out1, out8[j], 500) == 0);
  }
  return 0;
}

static int test_draws() {
  const perm::Circuit C = perm::build(52);
  for (int kind = 0; kind < 2; ++kind) {
    perm::Seed sd[8];
    for (int j = 0; j < 8; ++j) {
      uint8_t b[32];
      for (int i = 0; i < 32; ++i) b[i] = (uint8_t)(j + 3 * i);
      sd[j] = kind ? perm::Seed::bytes32(b) : perm::Seed::u64(1000 + j);
    }
    perm::RandomDraws d[8];
    perm::RandomDraws* dp[8];
    for (int j = 0; j < 8; ++j) dp[j] = &d[j];
    perm::draw_prover_randomness_x8(C, sd, dp);
    for (int j = 0; j < 8; ++j) {
      std::vector<uint32_t> pi;
      std::vector<hsc::Sc> gamma, sL, sR, taus;
      hsc::Sc al, be, rh;
      perm::draw_prover_randomness(C, sd[j], pi, gamma, al, be, rh, sL, sR, taus);
      CHECK(pi == d[j].pi);
      CHECK(gamma.size() == d[j].gamma.size() && memcmp(gamma.data(), d[j].gamma.data(), 32 * gamma.size()) == 0);
      CHECK(memcmp(taus.data(), d[j].taus.data(), 32 * taus.size()) == 0);
      CHECK(memcmp(&rh, &d[j].rho, 32) == 0);
    }
    perm::RandomDraws h[8];
    perm::RandomDraws* hp[8];
    for (int j = 0; j < 8; ++j) hp[j] = &h[j];
    perm::draw_prover_host_x8(C, sd, hp);  // the host's share of the same draws
    for (int j = 0; j < 8; ++j) {
      CHECK(h[j].pi == d[j].pi);
      CHECK(memcmp(&h[j].alpha, &d[j].alpha, 32) == 0 && memcmp(&h[j].beta, &d[j].beta, 32) == 0);
      CHECK(memcmp(&h[j].rho, &d[j].rho, 32) == 0);
      CHECK(h[j].taus.size() == 5 && memcmp(h[j].taus.data(), d[j].taus.data(), 32 * 5) == 0);
      CHECK(h[j].gamma.empty() && h[j].sL.empty());
    }
  }
  // sparse z^Q W over the circuit
  std::vector<hsc::Sc> zq(C.Q);
  hsc::Sc z = hsc::from_u64(7), acc = z;
  for (auto& v : zq) {
    v = acc;
    acc = hsc::mul(acc, z);
  }
  const auto zWL = perm::zW(C.WL, zq, C.n_p);
  CHECK(zWL.size() == C.n_p);
  return 0;
}

static int test_scalars() {
  std::vector<hsc::Sc> xs;
  uint8_t w[64];
  for (int i = 0; i < 37; ++i) {
    for (int b = 0; b < 64; ++b) w[b] = (uint8_t)(i * 64 + b * 13 + 1);
    xs.push_back(hsc::from_wide(w));
  }
  std::vector<hsc::Sc> inv = xs;
  hsc::batch_invert(inv);
  for (size_t i = 0; i < xs.size(); ++i) {
    const hsc::Sc prod = hsc::mul(xs[i], inv[i]), one = hsc::one();
    CHECK(memcmp(&prod, &one, 32) == 0);
    const hsc::Sc i2 = hsc::invert(xs[i]);
    CHECK(memcmp(&i2, &inv[i], 32) == 0);
  }
  return 0;
}

static int test_group() {
  using namespace h25519;
  // basepoint encoding (RFC 9496 multiple 1) -> decode -> multiples
  uint8_t e1[32];
  const char* B1 = "e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76";
  for (int i = 0; i < 32; ++i) sscanf(B1 + 2 * i, "%2hhx", &e1[i]);
  ge B;
  CHECK(decode(B, e1));
  uint8_t e[32];
  encode(e, B);
  CHECK(memcmp(e, e1, 32) == 0);
  std::vector<ge> pts;
  ge P = B;
  for (int i = 0; i < 19; ++i) {
    pts.push_back(P);
    P = ge_add(P, B);
  }
  std::vector<uint8_t> dbl(32 * pts.size());
  encode_double_batch(pts.data(), pts.size(), dbl.data());
  for (size_t i = 0; i < pts.size(); ++i) {
    encode(e, ge_dbl(pts[i]));
    CHECK(memcmp(e, dbl.data() + 32 * i, 32) == 0);
  }
  encode(e, ge_dbl(B));
  CHECK(hexeq(e, 32, "6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919"));
  uint8_t bad[32];
  memset(bad, 0xff, 32);
  bad[31] = 0x7f;
  ge Q;
  CHECK(!decode(Q, bad));
  return 0;
}

static int test_pool() {
  // concurrent callers (batches in flight each drive the pool), each with
  // nested for_each inside a task (runs inline)
  std::vector<std::thread> th;
  std::vector<int> rc(4, 0);
  for (int c = 0; c < 4; ++c)
    th.emplace_back([&, c] {
      for (int rep = 0; rep < 20; ++rep) {
        std::vector<uint64_t> v(1000, 0);
        par::for_each(v.size(), [&](size_t i) {
          uint64_t s = 0;
          par::for_each(4, [&](size_t k) { s += k; });  // inline (same thread)
          v[i] = i * 3 + s;
        });
        for (size_t i = 0; i < v.size(); ++i)
          if (v[i] != i * 3 + 6) rc[c] = 1;
      }
    });
  for (auto& t : th) t.join();
  for (int r : rc) CHECK(r == 0);
  return 0;
}

int main() {
  if (test_transcripts() || test_draws() || test_scalars() || test_group() || test_pool()) return 1;
  printf("ok\n");
  return 0;
}
