// Full-sequence GPT passes behind the C ABI (no Python needed to produce the decode KV cache or the
// vocoder latents):
//   * itts_gpt_forward_rows: every GPT-2 block over packed variable-length sequences (x in place),
//     optionally writing the decode KV cache, then out[i] = final_norm(ln_f(x[idx[i]])) for selected
//     rows -- the teacher-forced latent pass of UnifiedVoice.forward(return_latent=True)
//     (gpt/model.py:521-578 -> get_logits :462-477) and the prefill of inference_speech's generate;
//   * itts_gpt_prefill: the prompt block [cond | text | start_mel] of every row through the layers
//     into a decode state's KV cache, then mel_head on the last position and the first token's
//     selection + next-token embedding (HF generate's first iteration; gpt/model.py:85-192 prefill
//     branch), after which itts_gpt_decode_step(s) continue the loop.
// The launch sequence is HipGPT._forward_rows_py / _start_lane's (indextts/gpt/engine.py):
// LayerNorm -> c_attn -> causal attention -> attn.c_proj (+x) -> LayerNorm -> c_fc + gelu ->
// mlp.c_proj (+x) per layer (HF modeling_gpt2.py:246-306); bf16 mode runs the GEMMs on the MFMA
// implicit GEMM (itts_igemm_fwd, 1-tap), f32 mode on the exact-f32 GEMM.
#include "common.h"

namespace {
constexpr int kHD = 64;

int64_t align16(int64_t b) { return (b + 255) / 256 * 256; }

struct SeqWs {
  void *h, *o, *f;
  float* qkv;
};

SeqWs carve(void* ws, int64_t M, int D, int act_bytes) {
  char* p = static_cast<char*>(ws);
  SeqWs w;
  w.h = p;
  p += align16(M * D * act_bytes);
  w.qkv = reinterpret_cast<float*>(p);
  p += align16(M * 3 * D * 4);
  w.o = p;
  p += align16(M * D * act_bytes);
  w.f = p;
  return w;
}

// Y = act(A @ W^T + bias) (+ Y when residual), A [M][K] (bf16 in bf16 mode, f32 in f32 mode)
int seq_gemm(const ItTsGptSeqWeights* w, const void* A, const void* W, const float* bias, int64_t M, int K, int N,
             bool gelu, bool residual, void* Y, int y_dtype, void* stream) {
  if (w->dtype == ITTS_F32)
    return itts_gemm_f32(static_cast<const float*>(A), K, static_cast<const float*>(W), K, (int)M, N, K, bias,
                         gelu ? 1 : 0, residual ? static_cast<const float*>(Y) : nullptr, static_cast<float*>(Y), N,
                         stream);
  static const int32_t tap0 = 0;
  return itts_igemm_fwd(A, M * K, K, W, bias, nullptr, residual ? Y : nullptr, nullptr, Y, M * N, N, nullptr, 1,
                        (int)M, K, N, 1, &tap0, 1, 0, 1.0f, gelu ? 1 : 0, y_dtype, stream);
}

int forward_rows(const ItTsGptSeqWeights* w, float* x, int64_t M, const int32_t* seq_start, const int32_t* seq_len,
                 const int32_t* seq_pad, int nseq, int max_len, void* cache_k, void* cache_v, int64_t cache_bs,
                 int64_t cache_hs, int64_t cache_ls, int cache_dtype, void* workspace, void* stream) {
  const int D = w->d_model, H = w->n_head;
  const int act = w->dtype == ITTS_F32 ? ITTS_F32 : ITTS_BF16;
  SeqWs ws = carve(workspace, M, D, act == ITTS_F32 ? 4 : 2);
  const int esz = cache_dtype == ITTS_F32 ? 4 : 2;
  int rc = 0;
  for (int l = 0; l < w->n_layer && rc == 0; ++l) {
    const ItTsGptSeqLayerW& ly = w->layers[l];
    rc = itts_layernorm_rows(x, D, nullptr, ws.h, D, (int)M, D, ly.ln1_g, ly.ln1_b, nullptr, nullptr, act, stream);
    if (rc == 0) rc = seq_gemm(w, ws.h, ly.qkv_w, ly.qkv_b, M, D, 3 * D, false, false, ws.qkv, ITTS_F32, stream);
    void* ck = cache_k ? static_cast<char*>(cache_k) + (int64_t)l * cache_ls * esz : nullptr;
    void* cv = cache_v ? static_cast<char*>(cache_v) + (int64_t)l * cache_ls * esz : nullptr;
    if (rc == 0)
      rc = itts_attn_prefill(ws.qkv, 3 * D, seq_start, seq_len, seq_pad, nseq, max_len, ck, cv, cache_bs, cache_hs,
                             ws.o, D, H, cache_k ? cache_dtype : act, act, stream);
    if (rc == 0) rc = seq_gemm(w, ws.o, ly.o_w, ly.o_b, M, D, D, false, true, x, ITTS_F32, stream);
    if (rc == 0)
      rc = itts_layernorm_rows(x, D, nullptr, ws.h, D, (int)M, D, ly.ln2_g, ly.ln2_b, nullptr, nullptr, act, stream);
    if (rc == 0) rc = seq_gemm(w, ws.h, ly.fc_w, ly.fc_b, M, D, 4 * D, true, false, ws.f, act, stream);
    if (rc == 0) rc = seq_gemm(w, ws.f, ly.proj_w, ly.proj_b, M, 4 * D, D, false, true, x, ITTS_F32, stream);
  }
  return rc;
}

bool seq_weights_ok(const ItTsGptSeqWeights* w) {
  if (!w || !w->layers || w->n_layer <= 0 || w->n_head <= 0 || w->d_model != w->n_head * kHD) return false;
  if (w->dtype != ITTS_F32 && w->dtype != ITTS_BF16) return false;
  for (int l = 0; l < w->n_layer; ++l) {
    const ItTsGptSeqLayerW& y = w->layers[l];
    if (!y.qkv_w || !y.o_w || !y.fc_w || !y.proj_w || !y.ln1_g || !y.ln1_b || !y.ln2_g || !y.ln2_b) return false;
  }
  return w->ln_f_g && w->ln_f_b && w->final_g && w->final_b;
}
}  // namespace

extern "C" int64_t itts_gpt_forward_rows_workspace_bytes(const ItTsGptSeqWeights* w, int64_t M) {
  if (!w || M < 0 || w->d_model <= 0) return -1;
  const int64_t D = w->d_model, ab = w->dtype == ITTS_F32 ? 4 : 2;
  return align16(M * D * ab) + align16(M * 3 * D * 4) + align16(M * D * ab) + align16(M * 4 * D * ab);
}

extern "C" int itts_gpt_forward_rows(const ItTsGptSeqWeights* w, float* x, int64_t M, const int32_t* seq_start,
                                     const int32_t* seq_len, const int32_t* seq_pad, int nseq, int max_len,
                                     void* cache_k, void* cache_v, int64_t cache_bs, int64_t cache_hs,
                                     int64_t cache_layer_stride, int cache_dtype, const int32_t* out_idx, int n_out,
                                     void* out, int out_dtype, void* workspace, void* stream) {
  const char* fn = "itts_gpt_forward_rows";
  ITTS_REQUIRE(seq_weights_ok(w), fn, "incomplete ItTsGptSeqWeights (d_model = 64 * n_head, dtype f32 / bf16)");
  ITTS_REQUIRE(M >= 0 && nseq >= 0 && max_len >= 0 && n_out >= 0, fn, "bad sizes");
  if (M == 0) return 0;
  ITTS_REQUIRE(x && seq_start && seq_len && workspace, fn, "null pointer");
  ITTS_REQUIRE(!cache_k == !cache_v, fn, "cache_k and cache_v go together");
  ITTS_REQUIRE(n_out == 0 || out, fn, "out required for n_out > 0");
  int rc = forward_rows(w, x, M, seq_start, seq_len, seq_pad, nseq, max_len, cache_k, cache_v, cache_bs, cache_hs,
                        cache_layer_stride, cache_dtype, workspace, stream);
  if (rc || n_out == 0) return rc;
  return itts_layernorm_rows(x, w->d_model, out_idx, out, w->d_model, n_out, w->d_model, w->ln_f_g, w->ln_f_b,
                             w->final_g, w->final_b, out_dtype, stream);
}

extern "C" int itts_gpt_prefill(const ItTsGptSeqWeights* ws, const ItTsGptWeights* w, const ItTsGptDecodeState* st,
                                float* emb, int s, const int32_t* seq_start, const int32_t* seq_len,
                                const int32_t* last_idx, const ItTsSampling* smp, void* workspace, void* stream) {
  const char* fn = "itts_gpt_prefill";
  ITTS_REQUIRE(seq_weights_ok(ws) && w && st && smp && emb && seq_start && seq_len && last_idx && workspace, fn,
               "null pointer or incomplete weights");
  ITTS_REQUIRE(w->d_model == ws->d_model && w->n_head == ws->n_head && w->n_layer == ws->n_layer, fn,
               "decode and sequence weights disagree");
  ITTS_REQUIRE(s >= 1 && s + 1 <= st->max_kv, fn, "prompt longer than the KV capacity");
  ITTS_REQUIRE(smp->mode >= 0 && smp->mode <= 2, fn, "sampling mode must be 0, 1 or 2");
  // the decode steps read key kv_base + t: the prompt block fills keys 0 .. s, so the first decode key is s + 1
  ITTS_REQUIRE(st->kv_base == s + 1, fn, "state kv_base must equal s + 1 (the prompt block's length)");
  ITTS_REQUIRE(ws->dtype == ITTS_F32 || w->head_w, fn, "bf16 mode needs head_w (mel_head, 32-column fragments)");
  ITTS_REQUIRE(st->xh && st->logits && st->k_cache && st->v_cache && st->tstate, fn, "null state buffer");
  ITTS_REQUIRE(smp->mode == 2 || (st->seen && st->done && st->codes && st->x && w->mel_emb && w->mel_pos), fn,
               "sampler state missing (seen / done / codes / x / mel embeddings)");
  const int R = st->rows, D = w->d_model, H = w->n_head;
  const int64_t cache_hs = (int64_t)st->max_kv * kHD, cache_bs = (int64_t)H * cache_hs;
  const int64_t M = (int64_t)R * (s + 1);
  const int cdt = ws->dtype == ITTS_F32 ? ITTS_F32 : ITTS_BF16;
  int rc = forward_rows(ws, emb, M, seq_start, seq_len, st->pad, R, s + 1, st->k_cache, st->v_cache, cache_bs, cache_hs,
                        (int64_t)R * cache_bs, cdt, workspace, stream);
  if (rc) return rc;
  // the head's input: final_norm(ln_f(x)) of every row's last position, into xh (the decode GEMMs' A)
  rc = itts_layernorm_rows(emb, D, last_idx, st->xh, D, R, D, w->ln_f_g, w->ln_f_b, w->final_g, w->final_b, cdt,
                           stream);
  if (rc) return rc;
  if (ws->dtype == ITTS_F32) {
    ITTS_REQUIRE(ws->head_w_f32, fn, "f32 mode needs head_w_f32");
    rc = itts_gemm_f32(static_cast<const float*>(st->xh), D, ws->head_w_f32, D, R, w->n_mel_codes, D, w->head_b, 0,
                       nullptr, st->logits, w->logits_pitch, stream);
  } else {
    rc = itts_decode_gemm(st->xh, D, w->head_w, D, w->n_mel_codes, R, w->head_b, nullptr, nullptr, nullptr, nullptr, 0,
                          0, 0, st->logits, w->logits_pitch, ITTS_F32, (int64_t)R * w->n_mel_codes, 1, stream);
  }
  if (rc || smp->mode == 2) return rc;
  const int hdt = cdt;
  if (smp->mode == 0)
    return itts_sample_embed(st->logits, w->logits_pitch, w->n_mel_codes, st->seen, st->done, st->codes, st->max_new,
                             st->tstate, 0, smp->min_new, w->stop_mel, smp->rep_penalty, w->mel_emb, w->mel_pos, 2, D,
                             ws->dtype == ITTS_F32 ? ws->layers[0].ln1_g : nullptr,
                             ws->dtype == ITTS_F32 ? ws->layers[0].ln1_b : nullptr, st->x, st->xh, hdt, R, st->forced,
                             stream);
  return itts_sample_topk_embed(st->logits, w->logits_pitch, w->n_mel_codes, st->seen, st->done, st->codes,
                                st->max_new, st->tstate, 0, smp->min_new, w->stop_mel, smp->rep_penalty,
                                smp->temperature, smp->top_k, smp->top_p, w->mel_emb, w->mel_pos, 2, D,
                                ws->dtype == ITTS_F32 ? ws->layers[0].ln1_g : nullptr,
                                ws->dtype == ITTS_F32 ? ws->layers[0].ln1_b : nullptr, st->x, st->xh, hdt, R,
                                st->forced, stream);
}
