// Device vector-polynomial stage of the batched prover (poly.hip).
#pragma once
#include <vector>

#include "ctx.h"
#include "host/perm.h"

// t_1, t_3..t_6 inputs: for P proofs, with d_sc the A_I/A_O/S scalar array
// ([P][per], per = 3 + 5 n_p: alpha, a_L, a_R, beta, a_O, rho, s_L, s_R,
// canonical), d_gamma the V blindings ([P][m], canonical) and ch =
// [P][y, y^-1, z] (canonical): t = [P][t_1..t_6, <z^Q W_V, gamma>].
// Keeps the l(X), r(X) coefficient vectors and the H factors y^-i on the
// device for poly_x_dev.
int poly_coef_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const uint32_t* d_sc, uint32_t per,
                  const uint32_t* d_gamma, const std::vector<hsc::Sc>& ch, std::vector<hsc::Sc>& t);

// l = l(x), r = r(x) ([P][n_p], canonical, on the device for the IPA), the
// H factors, and t_hat = <l, r> per proof.
int poly_x_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const std::vector<hsc::Sc>& x, uint32_t** d_l,
               uint32_t** d_r, uint32_t** d_hf, std::vector<hsc::Sc>& t_hat);

// The batch verifier's MSM scalars for `count` proofs (k_verify_consts +
// k_verify_scalars + k_verify_merge): rec = [count][12 + lg] canonical
// scalars (x_perm, y, z, x, w, r, a, b, t_hat, tau_x, mu, -, u_j..); proof p
// is weighted by perm::batch_weight(seed, first + p, r_p); d_sc (device)
// receives the 2 n_p + 2 merged generator scalars then count x (m + 8 + 2 lg)
// weighted proof-point scalars, every proof's check scaled by
// (prod u_j)^2 y^(n_p - 1) (verify_dev.h).
int verify_scalars_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t count, const std::vector<uint32_t>& rec,
                       const uint8_t seed[32], uint64_t first, uint32_t* d_sc);

// The prover's blinding draws on the device (perm.h draw_scalar, one
// thread each) from per-proof sponge templates (d_tmpl [P][7] u64,
// draw_template; seed_len uniform over the batch, <= 32) -> gamma ([P][m],
// canonical) and alpha, beta, rho, s_L, s_R into their slots of the
// A_I/A_O/S scalar array d_sc ([P][per]).
// With d_v non-null, also the V commitment inputs from pi ([P][k] u32):
// d_v, d_g [P][2k] (values 1..k and pi + 1; gamma_0..2k-1) and d_gx_half [P]
// = gamma_2k / 2, in the same launch.
int draws_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const uint64_t* d_tmpl, uint32_t seed_len,
              uint32_t per, uint32_t* d_gamma, uint32_t* d_sc, const uint32_t* d_pi = nullptr,
              uint32_t* d_v = nullptr, uint32_t* d_g = nullptr, uint32_t* d_gx_half = nullptr);
void draw_template(const perm::Seed& seed, uint64_t tmpl[7]);


// The witness a_L, a_R, a_O of every proof (x = x_perm [P] canonical, pi
// [P][k]) into their slots of d_sc.
int witness_dev(bpp_ctx* ctx, const perm::Circuit& C, uint32_t P, const uint32_t* d_pi, const uint32_t* d_x,
                uint32_t per, uint32_t* d_sc);
