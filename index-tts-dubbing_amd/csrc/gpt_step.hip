// The whole GPT decode step behind one C-ABI call (itts_gpt_decode_step): the launch sequence of
// the bf16 product path (engine.HipGPT._decode_step_fold) in C++, so a host without Python (cgo,
// JNI, plain C) can run the decode loop through the ABI alone, and so the hipGraph capture of a step
// is one call.
//
// Reference: one KV-cached step of UnifiedVoice.inference_speech's generate (gpt/model.py:85-192 ->
// HF GPT2Block, modeling_gpt2.py:246-306: ln_1 -> c_attn -> attention (:54-72, :185-225) -> c_proj
// -> ln_2 -> c_fc -> gelu -> mlp.c_proj), then ln_f + final_norm -> mel_head (Q5) and the token
// selection (HF generation/utils.py).
//
// Measured and removed (profiles/ubench_fused_r02.txt, per layer at C3): c_attn + attention as ONE
// multi-role launch (producer workgroups publish q/k/v write-through and count per head, attention
// workgroups request their K/V first and then wait) 24.9 us vs 20.6 us for the two launches, and
// c_fc + mlp.c_proj + the split-K reduce as one launch (last-arriver reduce) 23.4 vs 14.5 us -- the
// producers' weight loads queue behind the consumers' streams and every in-launch hand-off (sc1
// stores, drain, counter, poll) cost more than the kernel boundary it replaced; K/V read ahead into
// the Infinity Cache on a side stream: attention with cache-resident K/V is 9.7 vs 12.7 us, but the
// side stream slowed the whole step from 830 to 1327 us; each kernel requesting a later kernel's
// weights into the Infinity Cache in-kernel (profiles/prefetch_ab_r02.txt): every plan slower.
#include <cstdlib>

#include "common.h"

namespace {
constexpr int kHD = 64;       // head size
constexpr int kMlpSplit = 8;  // mlp.c_proj split-K factor (reduced by itts_residual_reduce_ln)
}  // namespace

extern "C" int itts_gpt_decode_state_bytes(const ItTsGptWeights* w, int rows, int max_kv, int max_new,
                                           int64_t* bytes) {
  if (!w || !bytes || rows <= 0 || max_kv <= 0 || max_new <= 0 || w->n_layer <= 0 || w->d_model <= 0) return -1;
  const int64_t D = w->d_model, R = rows, Rp = (R + 31) / 32 * 32, P = w->logits_pitch;
  const int64_t kv = (int64_t)w->n_layer * R * w->n_head * max_kv * kHD * 2;
  const int64_t b[ITTS_GPT_STATE_NBUF] = {R * D * 4,     Rp * D * 2,       R * 3 * D * 4, Rp * D * 2,
                                          Rp * 4 * D * 2, kMlpSplit * R * D * 4, R * P * 4, kv,
                                          kv,            R * 4,            4 * 4,         R * P,
                                          R,             R * (int64_t)max_new * 4};
  for (int i = 0; i < ITTS_GPT_STATE_NBUF; ++i) bytes[i] = b[i];
  return 0;
}

namespace {
// ITTS_OPROJ_EPI=1: attn.c_proj as one 16-column launch with the residual epilogue (round 3) instead of
// split-K 8 + reduce (the persistent layer's arithmetic)
bool oproj_epi() {
  static const bool on = [] {
    const char* e = getenv("ITTS_OPROJ_EPI");
    return e && e[0] == '1';
  }();
  return on;
}
// one decode step without the step-counter advance; step k of a multi-step call reads key
// kv_base + tstate[0] + k and writes code column tstate[0] + 1 + k (so ONE advance by n follows n
// steps: the advance kernel is a whole dependent launch per step otherwise)
int decode_step_impl(const ItTsGptWeights* w, const ItTsGptDecodeState* st, const ItTsSampling* smp, int k,
                     void* stream) {
  const char* fn = "itts_gpt_decode_step";
  ITTS_REQUIRE(w && st && smp && w->layers, fn, "null pointer");
  const int L = w->n_layer, D = w->d_model, H = w->n_head, R = st->rows;
  ITTS_REQUIRE(L > 0 && D == H * kHD && D % 256 == 0, fn, "d_model must be 64 * n_head and a multiple of 256");
  ITTS_REQUIRE(R > 0, fn, "rows must be positive");
  ITTS_REQUIRE(smp->mode >= 0 && smp->mode <= 2, fn, "sampling mode must be 0 (greedy), 1 (sample) or 2 (logits)");
  ITTS_REQUIRE(st->x && st->xh && st->qkv && st->o && st->f && st->part && st->logits && st->k_cache && st->v_cache &&
                   st->tstate,
               fn, "null state buffer");
  ITTS_REQUIRE(w->layers[0].o_w, fn, "ItTsGptLayerW.o_w (attn.c_proj, 32-column fragments) missing");
  ITTS_REQUIRE(smp->mode == 2 || (st->seen && st->done && st->codes), fn, "sampler state missing");
  const float eps = 1e-5f;
  const int64_t cache_hs = (int64_t)st->max_kv * kHD, cache_bs = (int64_t)H * cache_hs;
  const int64_t layer_cache = (int64_t)R * cache_bs;
  int rc = 0;
  for (int l = 0; l < L && rc == 0; ++l) {
    const ItTsGptLayerW& ly = w->layers[l];
    uint16_t* kc = static_cast<uint16_t*>(st->k_cache) + l * layer_cache;
    uint16_t* vc = static_cast<uint16_t*>(st->v_cache) + l * layer_cache;
    const bool last = l + 1 == L;
    // ln_1 (folded) + c_attn -> q|k|v f32
    rc = itts_decode_gemm16x(st->xh, D, ly.qkv_w16, D, 3 * D, R, ly.qkv_c, ly.qkv_u, eps, 0, 0, st->qkv, 3 * D,
                             ITTS_F32, nullptr, 0, 8, stream);
    // attention (appends this step's k/v); beams read their keys through the lineage table
    if (rc == 0 && st->kv_rows)
      rc = itts_attn_decode_rows(st->qkv, 3 * D, 1, (int64_t)R * 3 * D, nullptr, kc, vc, cache_bs, cache_hs,
                                 st->max_kv, st->pad, st->kv_base + k, st->tstate, st->o, D, R, H, ITTS_BF16, ITTS_BF16,
                                 st->kv_rows, st->ld_rows, stream);
    else if (rc == 0)
      rc = itts_attn_decode(st->qkv, 3 * D, 1, (int64_t)R * 3 * D, nullptr, kc, vc, cache_bs, cache_hs, st->max_kv,
                            st->pad, st->kv_base + k, st->tstate, st->o, D, R, H, ITTS_BF16, ITTS_BF16, stream);
    // attn.c_proj: split-K 8 partials (one per head pair), then x += b_o + sum, x^ = bf16(x) -- the
    // persistent layer's arithmetic (gpt_layer.hip: each cluster of 32 CUs owns two heads), so both
    // paths give the same bits (round 3: one 16-column residual-epilogue launch, 5.4 us)
    if (oproj_epi()) {  // one 16-column launch with the residual epilogue (A/B)
      if (rc == 0)
        rc = itts_decode_gemm16x(st->o, D, ly.o_w16, D, D, R, ly.o_c, nullptr, eps, 0, 1, st->x, D, ITTS_F32, st->xh, D,
                                 8, stream);
    } else {
      if (rc == 0)
        rc = itts_decode_gemm(st->o, D, ly.o_w, D, D, R, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 2, st->part,
                              D, ITTS_F32, (int64_t)R * D, kMlpSplit, stream);
      if (rc == 0)
        rc = itts_residual_reduce_ln(st->x, D, st->part, kMlpSplit, (int64_t)R * D, D, ly.o_c, st->xh, D, R, D, nullptr,
                                     nullptr, nullptr, nullptr, ITTS_BF16, stream);
    }
    // ln_2 (folded) + c_fc + gelu -> f bf16
    if (rc == 0)
      rc = itts_decode_gemm16x(st->xh, D, ly.fc_w16, D, 4 * D, R, ly.fc_c, ly.fc_u, eps, 1, 0, st->f, 4 * D, ITTS_BF16,
                               nullptr, 0, 8, stream);
    // mlp.c_proj split-K partials, then x += b + sum (x^ = bf16 x; after the last layer LN(LN(x)), Q5)
    if (rc == 0)
      rc = itts_decode_gemm(st->f, 4 * D, ly.proj_w, 4 * D, D, R, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 2,
                            st->part, D, ITTS_F32, (int64_t)R * D, kMlpSplit, stream);
    if (rc == 0)
      rc = itts_residual_reduce_ln(st->x, D, st->part, kMlpSplit, (int64_t)R * D, D, ly.proj_b, st->xh, D, R, D,
                                   last ? w->ln_f_g : nullptr, last ? w->ln_f_b : nullptr, last ? w->final_g : nullptr,
                                   last ? w->final_b : nullptr, ITTS_BF16, stream);
  }
  if (rc) return rc;
  return itts::gpt_head_sample(w, st, smp, k, stream);
}
}  // namespace

// mel_head over x^ = final_norm(ln_f(x)) and the step's token selection + next embedding (shared by
// the launch chain and the persistent layers)
int itts::gpt_head_sample(const ItTsGptWeights* w, const ItTsGptDecodeState* st, const ItTsSampling* smp, int k,
                          void* stream) {
  const int D = w->d_model, R = st->rows;
  int rc = itts_decode_gemm(st->xh, D, w->head_w, D, w->n_mel_codes, R, w->head_b, nullptr, nullptr, nullptr, nullptr,
                            0, 0, 0, st->logits, w->logits_pitch, ITTS_F32, (int64_t)R * w->n_mel_codes, 1, stream);
  if (rc) return rc;
  if (smp->mode == 0) {
    rc = itts_sample_embed(st->logits, w->logits_pitch, w->n_mel_codes, st->seen, st->done, st->codes, st->max_new,
                           st->tstate, 1 + k, smp->min_new, w->stop_mel, smp->rep_penalty, w->mel_emb, w->mel_pos, 2, D,
                           nullptr, nullptr, st->x, st->xh, ITTS_BF16, R, st->forced, stream);
  } else if (smp->mode == 1) {
    rc = itts_sample_topk_embed(st->logits, w->logits_pitch, w->n_mel_codes, st->seen, st->done, st->codes,
                                st->max_new, st->tstate, 1 + k, smp->min_new, w->stop_mel, smp->rep_penalty,
                                smp->temperature, smp->top_k, smp->top_p, w->mel_emb, w->mel_pos, 2, D, nullptr,
                                nullptr, st->x, st->xh, ITTS_BF16, R, st->forced, stream);
  }
  return rc;
}

extern "C" int itts_gpt_decode_step(const ItTsGptWeights* w, const ItTsGptDecodeState* st, const ItTsSampling* smp,
                                    void* stream) {
  int rc = decode_step_impl(w, st, smp, 0, stream);
  if (rc == 0 && smp->mode != 2) rc = itts_step_advance(st->tstate, 1, stream);
  return rc;
}

extern "C" int itts_gpt_decode_steps(const ItTsGptWeights* w, const ItTsGptDecodeState* st, const ItTsSampling* smp,
                                     int nsteps, void* stream) {
  const char* fn = "itts_gpt_decode_steps";
  ITTS_REQUIRE(w && st && smp, fn, "null pointer");
  ITTS_REQUIRE(nsteps >= 1 && nsteps <= 64, fn, "nsteps must be in [1, 64]");
  ITTS_REQUIRE(nsteps == 1 || smp->mode != 2, fn, "beam decoding (mode 2) runs one step per call");
  int rc = 0;
  for (int k = 0; k < nsteps && rc == 0; ++k) rc = decode_step_impl(w, st, smp, k, stream);
  if (rc == 0 && smp->mode != 2) rc = itts_step_advance(st->tstate, nsteps, stream);
  return rc;
}
