/* merlin_min.h against merlin's "simple transcript" known answer (merlin
 * 3.0.0 src/transcript.rs test) -- run by tests/test_abi_c.py on the CPU. */
#include <stdio.h>

#include "merlin_min.h"

int main(void) {
  mm_transcript t;
  mm_new(&t, (const uint8_t*)"test protocol", 13);
  mm_append_message(&t, (const uint8_t*)"some label", 10, (const uint8_t*)"some data", 9);
  uint8_t out[32];
  mm_challenge_bytes(&t, (const uint8_t*)"challenge", 9, out, 32);
  for (int i = 0; i < 32; ++i) printf("%02x", out[i]);
  printf("\n");
  return 0;
}
