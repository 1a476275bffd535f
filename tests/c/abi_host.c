/* A C caller of include/bpperm.h (what a Rust `extern "C"` shim or any other
 * FFI binds), compiled and run by tests/test_abi_c.py on the CPU: only the
 * host-side entry points are called (no GPU in the test container).
 *   - bpp_transcript_*: the merlin 3.0.0 "simple transcript" KAT
 *     (transcript_protocol.rs:26-67 builds on it)
 *   - bpp_points_double_compress: 2 * basepoint = RFC 9496 multiple 2
 *   - bpp_partials_finish / bpp_partials_is_identity: the multi-GPU combine
 *   - bpp_msm_windows, bpp_perm_proof_len: geometry queries
 *   - argument errors: NULL handles, bad k -> BPP_ERR_ARG (no crash)
 * Prints "ok" and exits 0 on success. */
#include <stdio.h>
#include <string.h>

#include "bpperm.h"

static int hexeq(const uint8_t* b, size_t n, const char* hex) {
  char buf[256];
  for (size_t i = 0; i < n; ++i) sprintf(buf + 2 * i, "%02x", b[i]);
  return strcmp(buf, hex) == 0;
}

static void unhex(const char* h, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n; ++i) sscanf(h + 2 * i, "%2hhx", &out[i]);
}

#define CHECK(c)                                               \
  do {                                                         \
    if (!(c)) {                                                \
      fprintf(stderr, "FAILED line %d: %s\n", __LINE__, #c);  \
      return 1;                                                \
    }                                                          \
  } while (0)

int main(void) {
  /* merlin: Transcript::new(b"test protocol"); append_message(b"some label",
   * b"some data"); challenge_bytes(b"challenge", 32) */
  bpp_transcript* t = bpp_transcript_new((const uint8_t*)"test protocol", 13);
  CHECK(t != NULL);
  CHECK(bpp_transcript_append_message(t, (const uint8_t*)"some label", 10, (const uint8_t*)"some data", 9) == BPP_OK);
  bpp_transcript* t2 = bpp_transcript_clone(t);
  uint8_t ch[32], ch2[32];
  CHECK(bpp_transcript_challenge_bytes(t, (const uint8_t*)"challenge", 9, ch, 32) == BPP_OK);
  CHECK(hexeq(ch, 32, "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"));
  CHECK(bpp_transcript_challenge_bytes(t2, (const uint8_t*)"challenge", 9, ch2, 32) == BPP_OK);
  CHECK(memcmp(ch, ch2, 32) == 0); /* a clone continues identically */
  uint8_t sc[32];
  CHECK(bpp_transcript_challenge_scalar(t, (const uint8_t*)"x", 1, sc) == BPP_OK);
  CHECK(sc[31] <= 0x10); /* reduced mod l < 2^253 */
  bpp_transcript_destroy(t);
  bpp_transcript_destroy(t2);

  /* raw extended basepoint X||Y||Z||T (little-endian integers) */
  uint8_t B[128];
  unhex("1ad5258f602d56c9b2a7259560c72c695cdcd6fd31e2a4c0fe536ecdd3366921"
        "5866666666666666666666666666666666666666666666666666666666666666"
        "0100000000000000000000000000000000000000000000000000000000000000"
        "a3ddb7a5b38ade6df5525177809ff0207de3ab648e4eea6665768bd70f5f8767",
        B, 128);
  uint8_t enc[32];
  CHECK(bpp_points_double_compress(B, 1, enc) == BPP_OK);
  CHECK(hexeq(enc, 32, "6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919"));
  /* B + B via the partial combine = 2B; B alone is not the identity */
  uint8_t two[256];
  memcpy(two, B, 128);
  memcpy(two + 128, B, 128);
  CHECK(bpp_partials_finish(two, 2, enc) == BPP_OK);
  CHECK(hexeq(enc, 32, "6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919"));
  CHECK(bpp_partials_is_identity(B, 1) == BPP_ERR_VERIFY);
  CHECK(bpp_partials_is_identity(NULL, 0) == BPP_OK); /* empty sum */

  uint32_t c = 0, W = 0;
  CHECK(bpp_msm_windows((size_t)1 << 20, &c, &W) == BPP_OK);
  CHECK(c == 16 && W == 16);
  CHECK(bpp_perm_proof_len(52) == 32 * (8 + 3 + 2 * 7 + 2));
  CHECK(bpp_perm_proof_len(1) == 0);

  bpp_verify_job* job = NULL;
  CHECK(bpp_perm_verify_begin(1, 0, NULL, 0, NULL, NULL, NULL, &job) == BPP_ERR_ARG);
  CHECK(bpp_perm_verify_begin(4, 1, NULL, 0, NULL, NULL, NULL, &job) == BPP_ERR_ARG);
  CHECK(job == NULL);
  CHECK(bpp_transcript_append_message(NULL, NULL, 0, NULL, 0) != BPP_OK);
  CHECK(bpp_partials_finish(NULL, 1, enc) == BPP_ERR_ARG);
  printf("ok\n");
  return 0;
}
