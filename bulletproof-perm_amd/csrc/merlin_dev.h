// Device-side Merlin transcript step of the IPA rounds (merlin_dev.hip).
#pragma once
#include <stdint.h>

#include "ctx.h"
#include "host/merlin.h"

// bytes per transcript state on the device: 200-byte sponge + pos,
// pos_begin, cur_flags (+ padding to 16-B alignment)
#define MERLIN_DEV_STATE_BYTES 208

// d_states: [P][MERLIN_DEV_STATE_BYTES]; d_enc: [P][64] (L then R);
// d_u: [P][16] words = (u R, u^-1 R), the layout k_ipa_round_dt folds with.
int ipa_transcript_step_dev(bpp_ctx* ctx, uint32_t P, uint8_t* d_states, const uint8_t* d_enc, uint32_t* d_u);
// The prover's V appends and x_perm challenge on the device, one lane per
// proof (k_prove_v_transcript): init = the 52-word state every proof shares
// (50 state words, pos, pos_begin); d_venc [P][2k][32]; states_out
// [P][MERLIN_DEV_STATE_BYTES] (merlin_state_import), xperm_out [P][8] words.
int prove_v_transcript_dev(bpp_ctx* ctx, uint32_t P, uint32_t k, const uint32_t* init, const uint32_t* d_venc,
                           uint8_t* states_out, uint32_t* xperm_out);
void merlin_state_export(const merlin::Transcript& t, uint8_t* out);
void merlin_state_import(merlin::Transcript& t, const uint8_t* in);
