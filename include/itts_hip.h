/* libitts_hip.so -- C ABI of the MI355X (gfx950) IndexTTS hot path:
 *   GPT speech-token decode (reference indextts/gpt/model.py + HF GPT-2) and the BigVGAN2 vocoder
 *   (reference indextts/BigVGAN/).
 *
 * Conventions (all entry points):
 *   - plain pointers to DEVICE memory allocated by the caller (the library never allocates or
 *     frees on the hot path); sizes / strides in elements; `stream` is a hipStream_t (NULL = the
 *     legacy default stream); launches are asynchronous, no host synchronisation;
 *   - return 0 on success, nonzero on an argument error or a HIP launch error; the message is in
 *     itts_last_error() (thread-local); no C++ exception crosses the ABI;
 *   - dtype codes: ITTS_F32 = 0, ITTS_BF16 = 1, ITTS_F16 = 2 (f16: the activation op only);
 *   - "channel-last" vocoder activations are [B][T][C] with per-sequence lengths[B] (ragged batch):
 *     rows t >= lengths[b] are never read as data (edge handling equals the reference's padding);
 *   - callable from any host thread; ctypes releases the GIL around every call.
 *
 * The reference's only native boundary on this path is the fused anti-alias activation extension
 * (anti_alias_activation_cuda.forward, BigVGAN/alias_free_activation/cuda/anti_alias_activation.cpp:19-23,
 * anti_alias_activation_cuda.cu:214-256); everything else in the reference is PyTorch / HF
 * transformers modules.  Each function below cites the reference code it replaces.
 */
#ifndef ITTS_HIP_H_
#define ITTS_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ITTS_DTYPE_F32 = 0, ITTS_DTYPE_BF16 = 1, ITTS_DTYPE_F16 = 2 };

/* ---- runtime -------------------------------------------------------------------------------- */
const char* itts_last_error(void);
int itts_abi_version(void);
const char* itts_build_target(void); /* "gfx950" */
/* sizeof of the ABI structs below (0 ItTsGptLayerW, 1 ItTsGptWeights, 2 ItTsGptDecodeState,
 * 3 ItTsSampling, 4 ItTsConv, 5 ItTsAct, 6 ItTsAmpLayer, 7 ItTsBigvganStage, 8 ItTsBigvganWeights,
 * 9 ItTsGptSeqLayerW, 10 ItTsGptSeqWeights, 11 ItTsGptPlLayerW),
 * -1 otherwise: lets a binding check its struct layouts. */
int64_t itts_struct_size(int which);

/* ---- BigVGAN2 vocoder ----------------------------------------------------------------------- */

/* Fused Activation1d(SnakeBeta): 2x upsample (replicate pad 5/5, 12-tap kaiser-sinc transposed conv,
 * crop 15/15) -> x + 1/(exp(beta)+1e-9) * sin^2(x*exp(alpha)) -> 2x downsample (replicate pad 5/6,
 * 12-tap lowpass, stride 2).  Replaces anti_alias_activation_cuda.forward
 * (anti_alias_activation_cuda.cu:214-256) and its torch path Activation1d.forward
 * (alias_free_torch/act.py:24-29, resample.py:25-49, filter.py:87-96, activations.py:109-122);
 * the parity target is the torch path (quirk Q7: the CUDA kernel differs on the first/last 3 samples).
 * Arbitrary strides (x_sb/x_st/x_sc = batch/time/channel strides); lengths may be NULL (all T).
 * dtypes: f32 / bf16 in any in-out combination, or f16 -> f16 (the reference op's float / bf16 / half
 * dispatch, type_shim.h:20-43); the arithmetic is f32 throughout, outputs rounded to nearest even. */
int itts_aa_snakebeta_fwd(const void* x, void* y, const float* up12, const float* down12, const float* log_alpha,
                          const float* log_beta, const int32_t* lengths, int B, int C, int T, int64_t x_sb,
                          int64_t x_st, int64_t x_sc, int64_t y_sb, int64_t y_st, int64_t y_sc, int dtype_in,
                          int dtype_out, void* stream);
/* Same, for contiguous [B][C][T] tensors -- exactly the reference extension's argument list
 * (input, up_filter, down_filter, alpha, beta; anti_alias_activation.cpp:19-23), caller-owned output. */
int itts_aa_snakebeta_bct(const void* x, void* y, const float* up12, const float* down12, const float* log_alpha,
                          const float* log_beta, int B, int C, int T, int dtype, void* stream);

/* Padded channel counts of the packed conv weights (K chunk of 32/64, N tile of 32/128). */
int itts_igemm_pack_dims(int Cin, int Cout, int* ci_pad, int* co_pad);
/* Implicit-GEMM 1-D convolution on MFMA (bf16 operands, f32 accumulate), channel-last, ragged:
 *   y[b][t*y_row_mul + y_row_off][:] = alpha * (act(sum_k x[b][t + tap_off[k]][:] @ W_k + bias + bias_b[b]) + r1 + r2)
 * with zero padding outside [0, lengths[b]).  Covers every Conv1d of the generator (conv_pre,
 * AMPBlock1 dilated convs with the residual add and the /num_kernels average fused in,
 * models.py:65-74,224-243), the polyphase ConvTranspose1d upsamplers (models.py:155-161,228-231)
 * and the GPT sequence GEMMs (HF Conv1D, pytorch_utils.py:119, as 1-tap convolutions).
 * act: gelu = 1 -> gelu_tanh, 2 -> SiLU (the conditioning encoder's feed-forward).
 * tap_off is a HOST array of ntaps offsets. */
int itts_igemm_fwd(const void* x, int64_t x_sb, int64_t ldx, const void* w_packed, const float* bias,
                   const float* bias_b, const void* r1, const void* r2, void* y, int64_t y_sb, int64_t ldy,
                   const int32_t* lengths, int B, int Tmax, int Cin, int Cout, int ntaps, const int32_t* tap_off,
                   int y_row_mul, int y_row_off, float alpha, int gelu, int out_dtype, void* stream);
/* Split-K form of the 1-tap igemm for long reductions over few rows (the conditioning encoder's
 * Linear(C * F -> D) after Conv2dSubsampling2, K = 25088): x bf16 [M][ldx] (K columns), w_chunks =
 * nsplit consecutive packed weights of the K / nsplit column chunks (each itts_igemm_pack_dims(K / nsplit,
 * N) sized), partials f32 [nsplit][M][N] workspace, y f32 [M][N] = bias + sum of the partials in chunk
 * order (row-independent, run-to-run identical). */
int itts_igemm_splitk(const void* x, int64_t ldx, int M, int K, const void* w_chunks, int nsplit, int N,
                      const float* bias, float* partials, float* y, void* stream);
/* One AMPBlock1 conv of the narrow stages (C in {24, 48, 96} after padding to 32/64/96) with the
 * preceding Activation1d fused in (log_alpha == NULL: no activation):
 *   y[b][t][:] = alpha * (sum_j W_j . act(x)[b][t + tap_off[j]][:] + bias + r1[b][t][:] + r2[b][t][:])
 * (models.py:65-74 `xt = c1(a1(x)); xt = c2(a2(xt)); x = xt + x`, :237-243 block mean).  bf16
 * channel-last, 16-B aligned, channels / strides multiples of 8; weights in the igemm packing. */
int itts_amp_conv_fwd(const void* x, int64_t x_sb, int64_t ldx, const float* up12, const float* down12,
                      const float* log_alpha, const float* log_beta, const void* w_packed, const float* bias,
                      const void* r1, const void* r2, void* y, int64_t y_sb, int64_t ldy, const int32_t* lengths,
                      int B, int Tmax, int Cin, int Cout, int ntaps, const int32_t* tap_off, float alpha,
                      void* stream);
/* conv_post (Conv1d(C->1, K, pad K/2), bias) + tanh (models.py:246-248), optionally also the int16
 * PCM of infer.py:627,653 (clamp(32767*wav, +-32767) truncated toward zero, quirk Q8). */
int itts_conv_post_tanh(const void* x, int64_t x_sb, int64_t ldx, const float* w, float bias, int C, int K,
                        const int32_t* lengths, int B, int Tmax, float* wav, int16_t* pcm, int64_t y_sb,
                        int dtype_in, void* stream);
/* activation_post (Activation1d, models.py:245; filters / log_alpha / log_beta as itts_aa_snakebeta_fwd) fused in
 * front of conv_post + tanh (+ int16): bf16 channel-last x, C a multiple of 8 and at most 32, K odd <= 15.  The
 * activation output never leaves the chip; results bit-identical to itts_aa_snakebeta_fwd (bf16) followed by
 * itts_conv_post_tanh on its output. */
int itts_act_conv_post_tanh(const void* x, int64_t x_sb, int64_t ldx, const float* up12, const float* down12,
                            const float* log_alpha, const float* log_beta, const float* w, float bias, int C, int K,
                            const int32_t* lengths, int B, int Tmax, float* wav, int16_t* pcm, int64_t y_sb,
                            void* stream);

/* The whole generator (BigVGAN.forward, models.py:201-250, + the int16 conversion of infer.py:627-631)
 * as one call.  Weights in the packings above: every conv as an igemm-packed tap list. */
typedef struct ItTsConv {
  const void* w;          /* [ntaps][co_pad][ci_pad] bf16 (itts_igemm_pack_dims) */
  const float* bias;      /* [cout] */
  int cin, cout, ntaps;
  int32_t tap_off[16];    /* y[t] = sum_j W_j x[t + tap_off[j]] */
} ItTsConv;
typedef struct ItTsAct {  /* Activation1d(SnakeBeta): 12-tap filters, log-scale alpha / beta [C] */
  const float *up12, *down12, *log_alpha, *log_beta;
} ItTsAct;
typedef struct ItTsAmpLayer {  /* one AMPBlock1 dilation: x' = c2(a2(c1(a1(x)))) + x */
  ItTsAct a1;
  ItTsConv c1;
  ItTsAct a2;
  ItTsConv c2;
} ItTsAmpLayer;
typedef struct ItTsBigvganStage {
  int up_rate;                 /* ConvTranspose1d stride u */
  const ItTsConv* phases;      /* [up_rate] polyphase convs (phase rho writes rows q*u + rho), OR [1]: one
                                  conv with cout = u * C (C = layers' channels) whose output column block
                                  rho is phase rho -- row q of its [T][u*C] output = rows q*u .. q*u+u-1 */
  const float* cond_w;         /* conds[i] (1x1 on the speaker embedding): [phases[0].cout][spk_dim] f32
                                  (the fused form repeats the C rows u times) */
  const float* cond_b;         /* [phases[0].cout] */
  int n_blocks, n_layers;      /* resblocks (kernel sizes) x dilations */
  const ItTsAmpLayer* layers;  /* [n_blocks][n_layers] */
  int amp_mode;                /* 0: act kernel + implicit-GEMM conv; 1: act fused into itts_amp_conv_fwd;
                                  2: act kernel + itts_amp_conv_fwd without activation */
} ItTsBigvganStage;
typedef struct ItTsBigvganWeights {
  int n_stages, gpt_dim, spk_dim;
  ItTsConv conv_pre;
  const float* cond_pre_w;     /* cond_layer: [conv_pre.cout][spk_dim] f32 */
  const float* cond_pre_b;
  const ItTsBigvganStage* stages;  /* HOST array [n_stages] */
  ItTsAct act_post;
  const float* post_w;         /* conv_post [C][post_k] f32 */
  float post_b;
  int post_k;
} ItTsBigvganWeights;
/* Workspace bytes of itts_bigvgan_forward for B utterances of at most T latent frames, or -1. */
int64_t itts_bigvgan_workspace_bytes(const ItTsBigvganWeights* w, int B, int T);
/* latent [B][T][gpt_dim] bf16 (rows >= lengths[b] ignored), lengths [B] frames (device), spk [B][spk_dim]
 * f32 -> wav [B][T*hop] f32 (tanh output) and, if pcm != NULL, pcm [B][T*hop] int16 (Q8); samples past
 * lengths[b]*hop undefined.  Per utterance exactly as at batch 1 (ragged-exact edges; speaker biases on
 * the exact-f32 GEMM).  Replaces BigVGAN.forward (models.py:201-250) with weight norm folded. */
int itts_bigvgan_forward(const ItTsBigvganWeights* w, const void* latent, const int32_t* lengths, const float* spk,
                         int B, int T, void* workspace, float* wav, int16_t* pcm, void* stream);

/* ---- prompt front-end ------------------------------------------------------------------------- */

/* log-mel spectrogram of B prompts (audio f32 [B][ld_audio], L samples each): center reflect padding
 * by n_fft/2, hop, caller's window [n_fft] (periodic Hann), |STFT| (power 1) @ mel_fb [n_fft/2+1][n_mels]
 * -> log(clamp(., 1e-7)) into out [B][n_mels][L/hop + 1].  Replaces torchaudio MelSpectrogram +
 * safe_log (indextts/utils/feature_extractors.py:24-50, indextts/utils/common.py:110-121,
 * infer.py:509-514).  n_fft a power of two <= 2048, L > n_fft/2. */
int itts_log_mel(const float* audio, int64_t ld_audio, int B, int L, const float* window, const float* mel_fb,
                 int n_fft, int hop, int n_mels, float* out, void* stream);
/* Band-limited resampling of the prompt (torchaudio.functional.resample, sinc_interp_hann: the
 * reference's Resample(sr, 24000), infer.py:509-514): rates reduced by their gcd to orig : new_rate,
 * kern [new_rate][2*width + orig] the windowed-sinc table (f32), y[b][i] for i < Lout,
 * y[new*f + p] = sum_k x[orig*f + k - width] * kern[p][k] (zero outside [0, L)). */
int itts_resample_sinc(const float* x, int64_t ldx, int B, int L, const float* kern, int orig, int new_rate,
                       int width, float* y, int64_t ldy, int Lout, void* stream);

/* Conditioning encoder, bf16 product path (HipGPT.conditioning(fast=True)):
 * itts_cond_subsample -- Conv2dSubsampling2 (gpt/conformer/subsampling.py:164-190): conv2d(1 -> C, 3x3,
 * stride 2) + ReLU of the image x[time][bin] = mel[b][bin][time] (mel strides mel_sb / mel_ld, unit time
 * stride), out bf16 y[B][To][Fo][C], To = (T - 3) / 2 + 1, Fo = (n_bins - 3) / 2 + 1; w [C][3][3], bias [C].
 * itts_cond_glu_dwconv -- ConvolutionModule middle (gpt/conformer_encoder.py:108-167): a [B][T][lda]
 * (pointwise_conv1 output, 2C channels) -> GLU -> depthwise conv1d w [C][K] (+w_bias, zero padding K/2)
 * -> LayerNorm(ln_g, ln_b, eps) -> SiLU -> bf16 y [B][T][ldy].  w_t (optional, 16-B aligned): w transposed
 * [K][C], enables the LDS-tiled form for C = 256, 512 or 1024. */
/* ECAPA speaker encoder, bf16 product path (channel-last, vocoder/ecapa.py speaker_embedding_cl):
 * itts_pad_rows_bf16 -- y bf16 [B][T + 2 pad][Cp] = x (+ x2, optional) rows, reflect (speechbrain "same"
 * padding, nnet/CNN.py:411-488) or zero padded in time, channels [C, Cp) zero; x / x2 f32 with batch and row
 * strides.  itts_relu_affine_rows -- y = relu(x) * scale + shift per channel (TDNNBlock's ReLU + eval
 * BatchNorm1d folded, BigVGAN/ECAPA_TDNN.py TDNNBlock), y may alias x. */
int itts_pad_rows_bf16(const float* x, int64_t x_sb, int64_t ldx, const float* x2, int64_t x2_sb, int64_t ldx2, int B,
                       int T, int C, int pad, int reflect, int Cp, void* y, void* stream);
int itts_relu_affine_rows(const float* x, int64_t x_sb, int64_t ldx, int B, int T, int C, const float* scale,
                          const float* shift, float* y, int64_t y_sb, int64_t ldy, void* stream);
/* itts_time_stats -- ECAPA pooling statistics (BigVGAN/ECAPA_TDNN.py AttentiveStatisticsPooling /
 * SEBlock means): per (b, c), w[t] = softmax_t(logits[b][t][c]) or 1/T (logits null); mean[b][c] =
 * sum_t w x[b][t][c], std[b][c] = sqrt(max(sum_t w (x - mean)^2, eps)) (std may be null).  t in order:
 * an utterance's statistics do not depend on the batch. */
int itts_time_stats(const float* x, int64_t x_sb, int64_t ldx, const float* logits, int64_t l_sb, int64_t ldl, int B,
                    int T, int C, float eps, float* mean, float* stdv, void* stream);
/* PerceiverResampler cross-attention (gpt/perceiver.py:111-150 Attend, :296-317 Attention) of 32 latent
 * queries q [B][32][ldq] over keys / values [B][nk][ldkv] (head h at columns 64h .. 64h+63, f32),
 * key_mask [B][nk] u8 (0 = masked, NULL = none): out[b][i][64h + d] f32, row-independent. */
int itts_cross_attn(const float* q, int64_t q_sb, int64_t ldq, const float* k, const float* v, int64_t kv_sb,
                    int64_t ldkv, const uint8_t* key_mask, int B, int nq, int nk, int heads, float scale, float* out,
                    int64_t o_sb, int64_t ldo, void* stream);
/* itts_cond_rel_attn -- RelPositionMultiHeadedAttention (gpt/conformer/attention.py:235-312, no rel_shift),
 * head dim 64, H heads (C = 64 H): qkv f32 [B][T][ld_qkv] = (q | k | v) linear outputs, pos f32 [T][ld_pos]
 * = linear_pos(pos_emb), bias_u / bias_v [H][64]; score = ((q+u).k + (q+v).p) * scale over keys t < lens[b]
 * (lens may be null = T; an all-masked row gives 0), softmax, @ v -> out [B][T][ld_out] (f32 or bf16). */
int itts_cond_rel_attn(const float* qkv, int64_t ld_qkv, const float* pos, int64_t ld_pos, const float* bias_u,
                       const float* bias_v, const int32_t* lens, int B, int T, int H, float scale, void* out,
                       int64_t ld_out, int out_dtype, void* stream);
int itts_cond_subsample(const float* mel, int64_t mel_sb, int64_t mel_ld, int B, int n_bins, int T, const float* w,
                        const float* bias, int C, void* y, void* stream);
int itts_cond_glu_dwconv(const float* a, int64_t lda, int B, int T, int C, const float* w, const float* w_bias, int K,
                         const float* ln_g, const float* ln_b, float eps, void* y, int64_t ldy, const float* w_t,
                         void* stream);

/* ---- GPT (UnifiedVoice + HF GPT-2) ------------------------------------------------------------ */

/* y[r] = LN2(LN1(x[row_idx ? row_idx[r] : r])) (LN2 optional; eps 1e-5).  ln_1 / ln_2 / ln_f and
 * the double norm before mel_head (HF modeling_gpt2.py:620 ln_f, gpt/model.py:48 final_norm; Q5). */
int itts_layernorm_rows(const float* x, int64_t ldx, const int32_t* row_idx, void* y, int64_t ldy, int M, int D,
                        const float* g1, const float* b1, const float* g2, const float* b2, int out_dtype,
                        void* stream);
/* x[m] += bias + sum_s part[s][m] (fixed order), then h[m] = LN2(LN1(x[m])): the residual add of
 * attn.c_proj / mlp.c_proj (HF modeling_gpt2.py:246-306) fused with the next LayerNorm. */
int itts_residual_reduce_ln(float* x, int64_t ldx, const float* part, int nsplit, int64_t split_stride, int64_t ldp,
                            const float* bias, void* h, int64_t ldh, int M, int D, const float* g1, const float* b1,
                            const float* g2, const float* b2, int out_dtype, void* stream);
/* Exact-f32 GEMM (one fmaf chain per output in k order): the f32 verification mode of every GPT
 * linear layer (HF Conv1D). */
int itts_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw, int M, int N, int K, const float* bias,
                  int gelu, const float* r1, float* Y, int64_t ldy, void* stream);
/* Decode-step GEMM for M <= 32 rows on MFMA with weights prepacked in fragment order; epi 0:
 * y = act(acc + bias), 1: y += acc + bias, 2: split-K partials y[ks][m][n] (reduced by
 * itts_residual_reduce_ln).  lnmode 1/2 normalises f32 rows of `a` in the prologue.  c_attn / c_proj /
 * c_fc / mlp.c_proj and mel_head of the KV-cached decode (gpt/model.py:85-192, HF :185-243). */
int itts_decode_gemm(const void* a, int64_t lda, const void* w_packed, int K, int N, int M, const float* bias,
                     const float* g1, const float* b1, const float* g2, const float* b2, int lnmode, int gelu, int epi,
                     void* y, int64_t ldy, int out_dtype, int64_t split_stride, int ksplit, void* stream);
/* The same store-epilogue GEMM on 16-column tiles (v_mfma_f32_16x16x32_bf16): y = act(a @ W^T + bias)
 * as out_dtype, act = gelu_tanh when gelu; weights prepacked [N/16][K/32][64][8] bf16 (lane 16q + c
 * holds W^T[16nt + c][32s + 8q : +8]); a bf16 with rows padded to whole 32-row tiles.  c_fc + gelu and
 * mel_head of the KV-cached decode (HF modeling_gpt2.py:229-243; gpt/model.py:180): twice the
 * workgroups of itts_decode_gemm, half the weight bytes each. */
int itts_decode_gemm16(const void* a, int64_t lda, const void* w_packed16, int K, int N, int M, const float* bias,
                       int gelu, void* y, int64_t ldy, int out_dtype, void* stream);
/* 16-column decode GEMM with the LayerNorm FOLDED in and a residual epilogue (product decode step:
 * five launches per layer).  With u != NULL: y = rstd * (a @ W'^T - mean * u) + c, where the row
 * statistics (mean, rstd with eps) of `a` are taken from the same A fragments the MFMAs consume,
 * W' = diag(ln.g) W (bf16), u = column sums of W', c = ln.b^T W + bias: exactly LN(a) @ W + bias
 * (HF ln_1 -> c_attn / ln_2 -> c_fc, modeling_gpt2.py:246-306).  With u == NULL: y = a @ W^T + c.
 * epi 0: store act(y) (gelu_tanh if gelu) as out_dtype; epi 1 (attn.c_proj / mlp.c_proj): residual,
 * y is the f32 stream x[M][ldy]: x += y, and xh[M][ldxh] = bf16(x) (the next A operand).
 * nwaves = 8 or 16 per workgroup. */
int itts_decode_gemm16x(const void* a, int64_t lda, const void* w_packed16, int K, int N, int M, const float* c,
                        const float* u, float eps, int gelu, int epi, void* y, int64_t ldy, int out_dtype, void* xh,
                        int64_t ldxh, int nwaves, void* stream);
/* One decode step of 16x64 causal attention per row: appends this step's k/v at position
 * kv_base + tstate[0] of the cache [B][H][smax][64] and attends over the valid (pad-masked,
 * quirk Q2) prefix.  HF modeling_gpt2.py:54-72,185-225 with the additive padding mask. */
/* q/k/v = qkv_bias (nullable) + sum of `nsplit` slabs qkv + s*split_stride (split-K partials of
 * c_attn, so that GEMM needs no reduce pass; nsplit = 1 with a finished qkv row is the plain case). */
int itts_attn_decode(const float* qkv, int64_t ldqkv, int nsplit, int64_t split_stride, const float* qkv_bias,
                     void* cache_k, void* cache_v, int64_t cache_bs, int64_t cache_hs, int smax, const int32_t* pad,
                     int kv_base, const int32_t* tstate, void* out, int64_t ldo, int B, int H, int cache_dtype,
                     int out_dtype, void* stream);
/* Beam variant (num_beams > 1): key position p of row b is read from cache row kv_rows[b*ld_rows + p]
 * (the beams' shared-prefix lineage; replaces HF's per-step _reorder_cache index_select of every
 * layer's K/V, gpt/model.py:194-207); this step's k/v are appended to row b. */
int itts_attn_decode_rows(const float* qkv, int64_t ldqkv, int nsplit, int64_t split_stride, const float* qkv_bias,
                          void* cache_k, void* cache_v, int64_t cache_bs, int64_t cache_hs, int smax,
                          const int32_t* pad, int kv_base, const int32_t* tstate, void* out, int64_t ldo, int B,
                          int H, int cache_dtype, int out_dtype, const int32_t* kv_rows, int64_t ld_rows,
                          void* stream);
/* Attention with attn.c_proj fused (bf16 product decode; kv_rows nullable, as itts_attn_decode_rows):
 * per (row b, head h) the f32 head output o_h [64] times rows 64h .. 64h+63 of w_proj (the c_proj
 * weight in HF Conv1D [in = H*64][out = N] order, bf16) is written as the split-K partial
 * part[h*part_stride + b*ldp + n], n < N (N % 8 == 0, N <= 1024); itts_residual_reduce_ln with
 * nsplit = H sums the heads with the bias and the residual.  HF modeling_gpt2.py:185-225. */
int itts_attn_decode_proj(const float* qkv, int64_t ldqkv, int nsplit, int64_t split_stride, const float* qkv_bias,
                          void* cache_k, void* cache_v, int64_t cache_bs, int64_t cache_hs, int smax,
                          const int32_t* pad, int kv_base, const int32_t* tstate, const void* w_proj, int N,
                          float* part, int64_t part_stride, int64_t ldp, int B, int H, int cache_dtype,
                          const int32_t* kv_rows, int64_t ld_rows, void* stream);
/* Causal attention over packed variable-length sequences (prefill and latent pass); optionally
 * writes K/V into the decode cache.  seq_pad[b] leading rows are masked (left padding, Q2). */
int itts_attn_prefill(const float* qkv, int64_t ldqkv, const int32_t* seq_start, const int32_t* seq_len,
                      const int32_t* seq_pad, int nseq, int max_len, void* cache_k, void* cache_v, int64_t cache_bs,
                      int64_t cache_hs, void* out, int64_t ldo, int H, int cache_dtype, int out_dtype, void* stream);
/* Greedy token selection + next-token embedding, per row:
 * RepetitionPenalty over all seen ids incl. the fake prefix ids (Q4; HF logits_process.py:409-412),
 * min_new_tokens, first-index argmax (HF generation/utils.py:2894-2925), finished rows -> stop,
 * x = mel_embedding(tok) + mel_pos[col + pos_delta] (Q1, gpt/model.py:151-155), h = ln_1(x).
 * col = tstate[0] + col_delta (device counter: graph-replayable).  forced (tests): feed these ids.
 * logits [B][ldl] f32 and seen [B][ldl] u8 share the row pitch ldl >= V (ldl % 4 == 0 with 16-B
 * aligned rows takes the vectorised path). */
int itts_sample_embed(const float* logits, int64_t ldl, int V, uint8_t* seen, uint8_t* done, int32_t* codes,
                      int64_t ldc, const int32_t* tstate, int col_delta, int min_new, int stop, float penalty,
                      const float* emb, const float* pos_emb, int pos_delta, int D, const float* ln_g,
                      const float* ln_b, float* x, void* h, int h_dtype, int B, const int32_t* forced, void* stream);
/* do_sample=True variant: Temperature -> TopK (any k >= 1, ties at the k-th value kept; 0 = off) ->
 * TopP (any top_p, also without TopK) warpers and a multinomial draw (HF 4.36 `sample`; infer.py:535-543
 * defaults top_k 30 / top_p 0.8).  k <= 64: candidate extraction by repeated block argmax; otherwise
 * exact thresholds (radix select for TopK, bitwise search of the cumulative mass for TopP) and a
 * Gumbel-max draw among the survivors.  top_k == 0 and top_p == 1: draw from the full softmax.  RNG: counter hash of
 * (seed = tstate[2] | tstate[3] << 32, row + tstate[1], column) -- statistical parity with
 * torch.multinomial; tstate[1] = global index of this launch's row 0 (row chunks on several streams). */
int itts_sample_topk_embed(const float* logits, int64_t ldl, int V, uint8_t* seen, uint8_t* done, int32_t* codes,
                           int64_t ldc, const int32_t* tstate, int col_delta, int min_new, int stop, float penalty,
                           float temperature, int top_k, float top_p, const float* emb, const float* pos_emb,
                           int pos_delta, int D, const float* ln_g, const float* ln_b, float* x, void* h,
                           int h_dtype, int B, const int32_t* forced, void* stream);
/* Beam search / beam sample step, part 1 (rows R = utterances x num_beams, 2 <= num_beams <= 16):
 * per row log_softmax -> repetition penalty on the log-probs (Q4) -> min_new_tokens -> [do_sample:
 * Temperature -> TopK -> TopP, min_keep 2] -> + running beam score; writes the row's 2*num_beams best
 * (key, score, token) candidates (key = score, or score + Gumbel noise when sampling: a without-
 * replacement multinomial draw).  HF 4.36 beam_search / beam_sample (generation/utils.py), called by
 * inference_speech's generate (gpt/model.py:698-703) with infer.py:535-543's defaults. */
int itts_beam_candidates(const float* logits, int64_t ldl, int V, const uint8_t* seen, float* beam_score,
                         const int32_t* tstate, int col_delta, int min_new, int stop, float penalty, int do_sample,
                         float temperature, int top_k, float top_p, int num_beams, float* cand_key,
                         float* cand_score, int32_t* cand_tok, int R, void* stream);
/* Part 2, per utterance: top 2K of its K x 2K candidates (sampling: sorted by score), then
 * BeamSearchScorer.process (HF generation/beam_search.py: eos ranked < K closes a hypothesis scored
 * sum_logprobs / generated_len**length_penalty; the first K non-eos candidates continue; done once K
 * hypotheses exist and the worst >= the best candidate), beam reorder of the running codes, the
 * repetition-penalty flags and the KV lineage table, next input embedding + ln_1 (as
 * itts_sample_embed).  Hypotheses live in hyp_* ([B][K] scores/lengths/list order, [B][K][ldc] codes);
 * the caller finalizes (adds the open beams of unfinished utterances, picks the best). */
int itts_beam_select(const float* cand_key, const float* cand_score, const int32_t* cand_tok, int num_beams, int V,
                     int stop, int do_sample, float length_penalty, const int32_t* tstate, int col_delta,
                     uint8_t* done, float* beam_score, int32_t* codes, int64_t ldc, uint8_t* seen, int64_t lds,
                     const int32_t* base_ids, int n_base, int32_t* kv_rows, int64_t ld_rows, int kv_base,
                     float* hyp_score, int32_t* hyp_len, int32_t* hyp_codes, int32_t* hyp_n, int32_t* hyp_order,
                     float* hyp_worst, const float* emb, const float* pos_emb, int pos_delta, int D,
                     const float* ln_g, const float* ln_b, float* x, void* h, int h_dtype, int B, int max_col,
                     void* stream);
/* tstate[0] += delta on the device (advances the decode column between graph replays). */
int itts_step_advance(int32_t* tstate, int delta, void* stream);

/* ---- the whole decode step (bf16 product mode) ----------------------------------------------- */

/* Weights of one GPT-2 block in the decode packings (engine.fold_ln_weights / pack_skinny[16]). */
typedef struct ItTsGptLayerW {
  const void* qkv_w16;  /* diag(ln_1.g) W_c_attn, 16-column fragment order */
  const float* qkv_u;   /* column sums of qkv_w16 */
  const float* qkv_c;   /* ln_1.b^T W_c_attn + c_attn.bias */
  const void* o_w16;    /* attn.c_proj, 16-column fragment order */
  const float* o_c;     /* attn.c_proj.bias */
  const void* fc_w16;   /* diag(ln_2.g) W_c_fc, 16-column fragment order */
  const float* fc_u;
  const float* fc_c;
  const void* proj_w;   /* mlp.c_proj, 32-column fragment order */
  const float* proj_b;
  const void* o_w;      /* attn.c_proj, 32-column fragment order (split-K 8 over head pairs; ABI 3) */
} ItTsGptLayerW;

/* The UnifiedVoice GPT for decoding (gpt/model.py:255-281,85-192): layers, ln_f + final_norm (Q5),
 * mel_head, the mel embeddings fed back (Q1 positions). */
typedef struct ItTsGptWeights {
  int n_layer, d_model, n_head;
  int n_mel_codes, logits_pitch;  /* V = 8194; row pitch of logits / seen (>= V, multiple of 4) */
  int start_mel, stop_mel;
  const ItTsGptLayerW* layers;    /* HOST array [n_layer] */
  const float *ln_f_g, *ln_f_b, *final_g, *final_b;
  const void* head_w;             /* mel_head, 32-column fragment order */
  const float* head_b;
  const float* mel_emb;           /* [V][D] f32 */
  const float* mel_pos;           /* [max positions][D] f32 */
} ItTsGptWeights;

/* Device-resident decode state of `rows` sequences (the caller allocates everything). */
typedef struct ItTsGptDecodeState {
  int rows, max_kv, kv_base, max_new;  /* kv_base = prompt length s + 1; step j writes key kv_base + j */
  float* x;          /* residual stream [rows][D] f32 */
  void* xh;          /* its bf16 copy, [32-row padded][D] */
  float* qkv;        /* [rows][3D] f32 */
  void* o;           /* attention output [32-row padded][D] bf16 */
  void* f;           /* gelu(c_fc) [32-row padded][4D] bf16 */
  float* part;       /* split-K partials [8][rows][D] f32 */
  float* logits;     /* [rows][logits_pitch] f32 */
  void* k_cache;     /* [n_layer][rows][n_head][max_kv][64] bf16 */
  void* v_cache;
  const int32_t* pad;      /* [rows] left padding (Q2) */
  int32_t* tstate;         /* [4]: step, row base, RNG seed lo / hi */
  const int32_t* kv_rows;  /* beams: [rows][ld_rows] KV lineage table, else NULL */
  int64_t ld_rows;
  uint8_t* seen;           /* [rows][logits_pitch] repetition-penalty flags */
  uint8_t* done;           /* [rows] */
  int32_t* codes;          /* [rows][max_new] */
  const int32_t* forced;   /* teacher forcing (tests) or NULL */
  int num_beams;           /* beams per utterance of a kv_rows state (rows b * num_beams + k), else 0 (ABI 5) */
} ItTsGptDecodeState;

/* Token selection of the step: mode 0 greedy (itts_sample_embed), 1 top-k / top-p sampling
 * (itts_sample_topk_embed), 2 logits only (beam search: the caller runs itts_beam_candidates /
 * itts_beam_select and itts_step_advance). */
typedef struct ItTsSampling {
  int mode, min_new;
  float rep_penalty, temperature;
  int top_k;
  float top_p;
} ItTsSampling;

/* Sizes in bytes of the state buffers for `rows` sequences, in field order: x, xh, qkv, o, f, part,
 * logits, k_cache, v_cache, pad, tstate, seen, done, codes (ITTS_GPT_STATE_NBUF entries; kv_rows,
 * forced: caller's choice).  A host without Python allocates these and fills ItTsGptDecodeState. */
#define ITTS_GPT_STATE_NBUF 14
int itts_gpt_decode_state_bytes(const ItTsGptWeights* w, int rows, int max_kv, int max_new, int64_t* bytes);
/* ---- weight packers (HOST memory in and out, CPU only: callable without a GPU) -------------------
 * What ItTsGptLayerW / ItTsGptPlLayerW point at, built from the checkpoint tensors (HF Conv1D weights
 * [in = K][out = N], gpt/model.py:255-281 -> modeling_gpt2.py:246-306; mel_head [V][D], gpt/model.py:48);
 * copy the outputs to the device.  HipGPT packs through these same functions. */
/* LayerNorm folded into the following linear layer: wt [N][K] bf16 = W'^T with W' = diag(ln_g) W (computed
 * in double, rounded to f32, then to bf16), u [N] = column sums of the rounded W' (exact, in double),
 * c [N] = ln_b^T W + bias (double).  ln_g = ln_b = NULL: wt = bf16(W^T), c = bias, u untouched.
 * -> qkv_u / qkv_c (ln_1 -> c_attn), fc_u / fc_c (ln_2 -> c_fc), o_c (attn.c_proj, no LN). */
int itts_gpt_fold_ln(const float* w_io, const float* bias, const float* ln_g, const float* ln_b, int K, int N,
                     uint16_t* wt, float* u, float* c);
/* MFMA fragment order of W^T [N][K] (f32 rounded to bf16, or bf16), N zero-padded to a multiple of cols:
 * cols 16 -> [N/16][K/32][64][8], lane 16q + c holds W^T[16nt + c][32s + 8q : +8] (qkv_w16, o_w16, fc_w16);
 * cols 32 -> [N/32][K/16][64][8], lane 32h + r holds W^T[32nt + r][16s + 8h : +8] (proj_w, o_w, head_w).
 * out: ceil(N / cols) * cols * K bf16. */
int itts_gpt_pack_frag(const void* wt, int wt_dtype, int N, int K, int cols, uint16_t* out);
/* ItTsGptPlLayerW of one layer from c_attn's folded wt [3D][D] bf16 and its u / c (itts_gpt_fold_ln):
 * workgroup b = 8j + c computes columns 12(j % 16) .. +11 of head h = 2c + j / 16's [q | k | v] 192;
 * w12 [256][D/32][4][12][8] bf16, uc [256][2][12] f32.  D = 1024, H = 16 only. */
int itts_gpt_pack_qkv12(const uint16_t* wt, const float* u, const float* c, int D, int H, uint16_t* w12, float* uc);
/* ---- full-sequence passes (prefill, teacher-forced latent pass) ---------------------------------- */
/* One GPT-2 block's weights for the sequence GEMMs: bf16 mode = the implicit-GEMM packing of W^T [N][K]
 * (itts_igemm_pack_dims, 1 tap), f32 mode = f32 W^T [N][K] (HF Conv1D [in][out] transposed). */
typedef struct ItTsGptSeqLayerW {
  const void *qkv_w, *o_w, *fc_w, *proj_w;
  const float *qkv_b, *o_b, *fc_b, *proj_b;
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
} ItTsGptSeqLayerW;
typedef struct ItTsGptSeqWeights {
  int n_layer, d_model, n_head, dtype; /* dtype ITTS_BF16 (MFMA product mode) or ITTS_F32 (exact f32) */
  const ItTsGptSeqLayerW* layers;
  const float *ln_f_g, *ln_f_b, *final_g, *final_b;
  const float* head_w_f32;             /* f32 mode: mel_head W [n_mel_codes][d_model] (prefill) */
} ItTsGptSeqWeights;
/* Workspace bytes of itts_gpt_forward_rows / itts_gpt_prefill for M packed rows. */
int64_t itts_gpt_forward_rows_workspace_bytes(const ItTsGptSeqWeights* w, int64_t M);
/* Every GPT-2 block over nseq packed sequences (rows seq_start[i] .. + seq_len[i] of x [M][D] f32, in
 * place; keys before seq_pad[i] masked, Q2; causal), writing K/V into the decode cache when cache_k is
 * non-NULL (layer l at cache + l * cache_layer_stride elements, [seq][head][pos][64]); then
 * out[i] = final_norm(ln_f(x[out_idx[i]])) for n_out rows (Q5).  The teacher-forced latent pass of
 * UnifiedVoice.forward(return_latent=True) (gpt/model.py:521-578, get_logits :462-477) and the prefill
 * forward of generate; HF modeling_gpt2.py:246-306 per block. */
int itts_gpt_forward_rows(const ItTsGptSeqWeights* w, float* x, int64_t M, const int32_t* seq_start,
                          const int32_t* seq_len, const int32_t* seq_pad, int nseq, int max_len, void* cache_k,
                          void* cache_v, int64_t cache_bs, int64_t cache_hs, int64_t cache_layer_stride,
                          int cache_dtype, const int32_t* out_idx, int n_out, void* out, int out_dtype,
                          void* workspace, void* stream);
/* The first iteration of generate for every row of a decode state: emb [rows][s+1][D] f32 (the
 * prepare_gpt_inputs block + the start-mel embedding; consumed) through the layers into the state's
 * KV cache (seq_start[b] = b*(s+1), seq_len[b] = s+1, padding st->pad), final_norm(ln_f(.)) of each
 * row's last position (last_idx[b]) -> mel_head -> the first token (ItTsSampling modes 0 / 1, code
 * column 0) and the next embedding; mode 2 stops at the logits (beam search).  Then
 * itts_gpt_decode_step(s) continue.  gpt/model.py:85-192 (prefill branch), :655-708. */
int itts_gpt_prefill(const ItTsGptSeqWeights* ws, const ItTsGptWeights* w, const ItTsGptDecodeState* st, float* emb,
                     int s, const int32_t* seq_start, const int32_t* seq_len, const int32_t* last_idx,
                     const ItTsSampling* sampling, void* workspace, void* stream);

/* One whole KV-cached decode step (one HF generate iteration of inference_speech, gpt/model.py:655-708),
 * per layer: c_attn with ln_1 folded (itts_decode_gemm16x) -> itts_attn_decode[_rows] -> attn.c_proj
 * split-K 8 over head pairs (itts_decode_gemm) -> itts_residual_reduce_ln -> c_fc with ln_2 folded +
 * gelu -> mlp.c_proj split-K 8 (itts_decode_gemm) -> itts_residual_reduce_ln (the last layer's with
 * ln_f + final_norm, Q5); then
 * mel_head, token selection + next embedding (ItTsSampling modes 0/1) and the step advance.  The
 * caller's prefill (itts_attn_prefill + the GEMMs above) fills the cache and the first token; rows
 * padded to whole 32-row tiles in xh / o / f.  Graph-capturable: the step counter lives on the device. */
int itts_gpt_decode_step(const ItTsGptWeights* w, const ItTsGptDecodeState* state, const ItTsSampling* sampling,
                         void* stream);
/* `nsteps` consecutive decode steps (sampling modes 0 / 1; mode 2 = one step) with ONE step-counter
 * advance at the end: step k reads key kv_base + t + k and writes code column t + 1 + k (t = the
 * device counter), so a captured graph of n steps launches n * (launches per step - 1) + 1 kernels.
 * Same results as nsteps calls of itts_gpt_decode_step. */
int itts_gpt_decode_steps(const ItTsGptWeights* w, const ItTsGptDecodeState* state, const ItTsSampling* sampling,
                          int nsteps, void* stream);

/* ---- persistent decode layer (gpt_layer.hip) ----------------------------------------------------
 * One GPT-2 block of the decode step (HF modeling_gpt2.py:246-306 via gpt/model.py:115-192) as ONE
 * launch of 256 workgroups (one per CU) joined by in-launch hand-offs, each workgroup's weights
 * requested at the start of the launch.  IndexTTS-1.5 shapes (d_model 1024, 16 heads), 1..128 rows,
 * with or without the beam lineage table (state.kv_rows); bit-identical to the launch chain
 * (itts_gpt_decode_step[s]).  Extra weights per layer besides ItTsGptLayerW: */
typedef struct ItTsGptPlLayerW {
  const void* qkv_w12;  /* c_attn (ln_1 folded), 12 columns per workgroup: [256][32][4][12][8] bf16 */
  const float* qkv_uc;  /* [256][2][12]: u and c of those columns (itts_decode_gemm16x fold terms) */
} ItTsGptPlLayerW;
/* Bytes of the device scratch the persistent layers share (hand-off buffers, counters, the launch epoch
 * and a sticky error word); zero it once after allocation (or call itts_gpt_pl_reset).  Nothing is reset
 * between steps: every hand-off is tagged with the launch's epoch (ABI 4). */
int64_t itts_gpt_pl_scratch_bytes(void);
/* 1 if the persistent path runs this shape on the current device (256 CUs, one workgroup of each kernel
 * instantiation resident per CU), else 0.  The grid needs every CU at once: run it with no other kernel
 * on the device (a workgroup that cannot be placed makes the others time out, itts_gpt_pl_error). */
int itts_gpt_pl_supported(const ItTsGptWeights* w, int rows);
/* Re-arm the scratch (counters, granules, epoch, error word := 0) with a kernel on `stream`: after an
 * error reported by itts_gpt_pl_error, before the next persistent launch. */
int itts_gpt_pl_reset(void* scratch, void* stream);
/* Layer `layer` of decode step `kstep` of a multi-step call (key kv_base + t + kstep); `last`: leave
 * the mlp.c_proj reduce (+ ln_f + final_norm) to itts_residual_reduce_ln over the scratch partials. */
int itts_gpt_layer_pl(const ItTsGptLayerW* layer_w, const ItTsGptPlLayerW* pl, const ItTsGptDecodeState* state,
                      int layer, int kstep, int last, void* scratch, void* stream);
/* A hand-off timeout recorded in the scratch (0 = none; else every later layer launch runs only its c_attn
 * phase and returns at its q/k/v sweep, without polling -- a few microseconds, so the rest of a graph replay
 * drains quickly -- and the results are invalid until itts_gpt_pl_reset; the launch chain,
 * itts_gpt_decode_steps, gives the same results bit for bit and needs no scratch).  Synchronises `stream`. */
int itts_gpt_pl_error(const void* scratch, void* stream, int* code);
/* itts_gpt_decode_steps with every layer on the persistent path (pl: [n_layer]); sampling mode 2 (beams:
 * logits only, nsteps = 1, the caller runs the beam kernels and the step advance) as itts_gpt_decode_step. */
int itts_gpt_decode_steps_pl(const ItTsGptWeights* w, const ItTsGptPlLayerW* pl, void* scratch,
                             const ItTsGptDecodeState* state, const ItTsSampling* sampling, int nsteps, void* stream);

/* ---- diagnostics ------------------------------------------------------------------------------ */
/* n_wg workgroups that each hold 120 KiB of LDS (one per CU) for `usec` microseconds, then exit (sink: NULL
 * or [n_wg] ints written at exit).  Test instrumentation: keeps CUs away from a persistent grid launched
 * beside it, to exercise the hand-off timeout (itts_gpt_pl_error) and the launch-chain fallback. */
int itts_diag_occupy(int n_wg, int usec, int* sink, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ITTS_HIP_H_ */
