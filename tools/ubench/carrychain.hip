// Does a VALU carry chain need wait states on gfx950?  hipcc pads
// v_add_co/v_addc (VCC carry) with s_nop 1; this kernel runs 256-bit add
// chains in inline asm with NO padding, carry in an explicit SGPR pair
// (VOP3) and in VCC (VOP2), and compares against a 64-bit reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ uint32_t rnd(uint64_t& s) { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return (uint32_t)(s >> 33) ^ (uint32_t)s; }

__global__ void k(unsigned long long* bad, int iters, uint32_t seed) {
  uint64_t st = (uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B97F4A7C15ULL + seed;
  unsigned long long nbad = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t a[8], b[8], r1[8], r2[8], ref[8];
    for (int i = 0; i < 8; ++i) { a[i] = rnd(st); b[i] = rnd(st); if (rnd(st) & 1) a[i] = 0xffffffffu; }
    uint64_t c = 0;
    for (int i = 0; i < 8; ++i) { c = (uint64_t)a[i] + b[i] + (c >> 32); ref[i] = (uint32_t)c; }
    uint64_t cc;
    asm volatile(
        "v_add_co_u32 %[r0], %[c], %[a0], %[b0]\n\t"
        "v_addc_co_u32 %[r1], %[c], %[a1], %[b1], %[c]\n\t"
        "v_addc_co_u32 %[r2], %[c], %[a2], %[b2], %[c]\n\t"
        "v_addc_co_u32 %[r3], %[c], %[a3], %[b3], %[c]\n\t"
        "v_addc_co_u32 %[r4], %[c], %[a4], %[b4], %[c]\n\t"
        "v_addc_co_u32 %[r5], %[c], %[a5], %[b5], %[c]\n\t"
        "v_addc_co_u32 %[r6], %[c], %[a6], %[b6], %[c]\n\t"
        "v_addc_co_u32 %[r7], %[c], %[a7], %[b7], %[c]\n\t"
        : [r0] "=&v"(r1[0]), [r1] "=&v"(r1[1]), [r2] "=&v"(r1[2]), [r3] "=&v"(r1[3]), [r4] "=&v"(r1[4]), [r5] "=&v"(r1[5]), [r6] "=&v"(r1[6]), [r7] "=&v"(r1[7]), [c] "=&s"(cc)
        : [a0] "v"(a[0]), [b0] "v"(b[0]), [a1] "v"(a[1]), [b1] "v"(b[1]), [a2] "v"(a[2]), [b2] "v"(b[2]), [a3] "v"(a[3]), [b3] "v"(b[3]), [a4] "v"(a[4]), [b4] "v"(b[4]), [a5] "v"(a[5]), [b5] "v"(b[5]), [a6] "v"(a[6]), [b6] "v"(b[6]), [a7] "v"(a[7]), [b7] "v"(b[7]));
    asm volatile(
        "v_add_co_u32_e32 %0, vcc, %8, %16\n\t"
        "v_addc_co_u32_e32 %1, vcc, %9, %17, vcc\n\t"
        "v_addc_co_u32_e32 %2, vcc, %10, %18, vcc\n\t"
        "v_addc_co_u32_e32 %3, vcc, %11, %19, vcc\n\t"
        "v_addc_co_u32_e32 %4, vcc, %12, %20, vcc\n\t"
        "v_addc_co_u32_e32 %5, vcc, %13, %21, vcc\n\t"
        "v_addc_co_u32_e32 %6, vcc, %14, %22, vcc\n\t"
        "v_addc_co_u32_e32 %7, vcc, %15, %23, vcc\n\t"
        : "=&v"(r2[0]), "=&v"(r2[1]), "=&v"(r2[2]), "=&v"(r2[3]), "=&v"(r2[4]), "=&v"(r2[5]), "=&v"(r2[6]), "=&v"(r2[7])
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
          "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
        : "vcc");
    for (int i = 0; i < 8; ++i) { nbad += (r1[i] != ref[i]) ? 1 : 0; nbad += (r2[i] != ref[i]) ? (1ull << 32) : 0; }
  }
  atomicAdd(bad, nbad);
}

int main() {
  unsigned long long* d; hipMalloc(&d, 8); hipMemset(d, 0, 8);
  int blocks = 2048, threads = 256, iters = 200;
  for (int r = 0; r < 4; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, iters, (uint32_t)r * 7919u);
  unsigned long long h; hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("words checked: %llu per variant\n", 4ull * blocks * threads * iters * 8);
  printf("mismatches sgpr-carry(VOP3): %llu  vcc-carry(VOP2): %llu\n", h & 0xffffffffull, h >> 32);
  return 0;
}
