// Device memory layout of points (shared by kernels and host code).
//
// Field elements are 10 limbs of radix 2^25.5 (fe25519.cuh), stored as 10
// little-endian u32 words.
//   table point   affine Niels (y+x, y-x, 2dxy): 30 words at a 32-word
//                 (128 B) stride, i.e. one 128-B memory request per gather
//   extended pt   (X, Y, Z, T): 40 words (160 B)
// The C ABI's 128-byte raw partial points (bpp_msm_table_dev_partial) are a
// separate host format: X, Y, Z, T as 32-byte little-endian integers.
#pragma once

#define FE_DEV_WORDS 10
#define MSM_NIELS_WORDS 32
#define P3_WORDS 40
#define P3_BYTES (P3_WORDS * 4)
