// The whole BigVGAN2 generator behind one C-ABI call (itts_bigvgan_forward): the launch sequence of
// HipBigVGAN.forward (indextts/vocoder/bigvgan.py) in C++, so a host without Python can run the
// vocoder through the ABI alone.  Reference: BigVGAN.forward (BigVGAN/models.py:201-250) with weight
// norm folded (models.py:252-260), AMPBlock1 (:65-74) and the block mean (:237-243); the int16
// conversion of infer.py:627-631 (quirk Q8) in the conv_post kernel.
//
// Per stage i (up-sampling rate u_i):  u_i polyphase ConvTranspose convs (+ conds[i](spk) as a
// per-utterance bias)  ->  n_blocks AMPBlock1 x n_layers dilations, each [act -> conv(dil) -> act ->
// conv + residual]; the last layer of each block accumulates the block sum (r2) and the last block
// applies 1/n_blocks.  Tail: activation_post -> conv_post + tanh (+ int16).  Channel-last bf16
// activations [B][T_stage][C] in six workspace buffers; per-stage lengths and the speaker biases at
// the workspace start.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int kMaxStages = 16;
struct Rates {
  int32_t r[kMaxStages];
};

__global__ void scale_lengths_kernel(const int32_t* __restrict__ lens, int32_t* __restrict__ out, int B, int nst,
                                     Rates rates) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int v = lens[b];
  out[b] = v;
  for (int i = 0; i < nst; ++i) {
    v *= rates.r[i];
    out[(int64_t)(i + 1) * B + b] = v;
  }
}

int64_t align256(int64_t v) { return (v + 255) / 256 * 256; }

// A stage's up-sampler is either up_rate phase convs (phase rho writes rows q*u + rho) or ONE conv
// whose cout = up_rate * C holds the phases as output column blocks (row q of the [T][u*C] output is
// rows q*u .. q*u+u-1 of the [T*u][C] stage input): fused when phases[0].cout == u * C, C the AMP
// layers' channel count.
// ITTS_VOC_TAIL_FUSED=0: activation_post and conv_post as two launches (the fused launch is bit-identical)
bool tail_fused() {
  static const bool on = [] {
    const char* e = getenv("ITTS_VOC_TAIL_FUSED");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool fused_up(const ItTsBigvganStage& st) {
  return st.up_rate > 1 && st.n_blocks > 0 && st.n_layers > 0 && st.layers &&
         st.phases[0].cout == st.up_rate * st.layers[0].c1.cout;
}
int stage_channels(const ItTsBigvganStage& st) {
  return fused_up(st) ? st.phases[0].cout / st.up_rate : st.phases[0].cout;
}

struct Layout {
  int64_t lens, pre_b, stage_b[kMaxStages], bufs[6], total, buf_elems;
};

bool layout(const ItTsBigvganWeights* w, int B, int T, Layout& L) {
  if (!w || B <= 0 || T <= 0 || w->n_stages <= 0 || w->n_stages > kMaxStages || !w->stages) return false;
  int64_t off = 0;
  L.lens = off;
  off = align256(off + (int64_t)(w->n_stages + 1) * B * 4);
  L.pre_b = off;
  off = align256(off + (int64_t)B * w->conv_pre.cout * 4);
  int64_t maxe = (int64_t)B * T * w->conv_pre.cout, t = T;
  for (int i = 0; i < w->n_stages; ++i) {
    const ItTsBigvganStage& st = w->stages[i];
    if (st.up_rate <= 0 || !st.phases) return false;
    L.stage_b[i] = off;
    off = align256(off + (int64_t)B * st.phases[0].cout * 4);
    t *= st.up_rate;
    const int64_t e = (int64_t)B * t * stage_channels(st);
    maxe = e > maxe ? e : maxe;
  }
  L.buf_elems = maxe;
  for (int k = 0; k < 6; ++k) {
    L.bufs[k] = off;
    off = align256(off + maxe * 2);
  }
  L.total = off;
  return true;
}

}  // namespace

extern "C" int64_t itts_bigvgan_workspace_bytes(const ItTsBigvganWeights* w, int B, int T) {
  Layout L;
  return layout(w, B, T, L) ? L.total : -1;
}

extern "C" int itts_bigvgan_forward(const ItTsBigvganWeights* w, const void* latent, const int32_t* lengths,
                                    const float* spk, int B, int T, void* workspace, float* wav, int16_t* pcm,
                                    void* stream) {
  const char* fn = "itts_bigvgan_forward";
  Layout L;
  ITTS_REQUIRE(layout(w, B, T, L), fn, "bad weights or sizes (B, T > 0; 1 <= n_stages <= 16)");
  ITTS_REQUIRE(latent && lengths && spk && workspace && wav, fn, "null pointer");
  ITTS_REQUIRE(w->conv_pre.cin == w->gpt_dim, fn, "conv_pre input channels must equal gpt_dim");
  hipStream_t s = itts::as_stream(stream);
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  int32_t* lens = reinterpret_cast<int32_t*>(ws + L.lens);
  uint16_t* buf[6];
  for (int k = 0; k < 6; ++k) buf[k] = reinterpret_cast<uint16_t*>(ws + L.bufs[k]);
  uint16_t *xs_a = buf[0], *xs_b = buf[1], *xst = buf[2], *t1 = buf[3], *t2 = buf[4], *cur = buf[5];
  const int ns = w->n_stages;
  // per-stage lengths: lens[i][b] = lengths[b] * prod(rates[0 .. i-1])
  Rates rates{};
  for (int i = 0; i < ns; ++i) rates.r[i] = w->stages[i].up_rate;
  hipLaunchKernelGGL(scale_lengths_kernel, dim3((B + 255) / 256), dim3(256), 0, s, lengths, lens, B, ns, rates);
  int rc = itts::check_launch(fn);
  if (rc) return rc;
  // speaker biases (exact-f32 GEMM: per utterance independent of the batch)
  const int C0 = w->conv_pre.cout;
  float* pre_b = reinterpret_cast<float*>(ws + L.pre_b);
  rc = itts_gemm_f32(spk, w->spk_dim, w->cond_pre_w, w->spk_dim, B, C0, w->spk_dim, w->cond_pre_b, 0, nullptr, pre_b,
                     C0, stream);
  for (int i = 0; i < ns && rc == 0; ++i) {
    const int Ci = w->stages[i].phases[0].cout;
    rc = itts_gemm_f32(spk, w->spk_dim, w->stages[i].cond_w, w->spk_dim, B, Ci, w->spk_dim, w->stages[i].cond_b, 0,
                       nullptr, reinterpret_cast<float*>(ws + L.stage_b[i]), Ci, stream);
  }
  if (rc) return rc;

  // launch helpers (argument meaning as in HipBigVGAN._conv / _amp / _act)
  auto conv = [&](const ItTsConv& c, const uint16_t* x, int Tx, uint16_t* y, int Ty, const int32_t* ln,
                  const void* r1, const void* r2, float alpha, const float* bias_b, int ymul, int yoff) {
    return itts_igemm_fwd(x, (int64_t)Tx * c.cin, c.cin, c.w, c.bias, bias_b, r1, r2, y, (int64_t)Ty * c.cout, c.cout, ln,
                          B, Tx, c.cin, c.cout, c.ntaps, c.tap_off, ymul, yoff, alpha, 0, ITTS_BF16, stream);
  };
  auto amp = [&](const ItTsConv& c, const uint16_t* x, int Tx, uint16_t* y, const int32_t* ln, const ItTsAct* a,
                 const void* r1, const void* r2, float alpha) {
    return itts_amp_conv_fwd(x, (int64_t)Tx * c.cin, c.cin, a ? a->up12 : nullptr, a ? a->down12 : nullptr,
                             a ? a->log_alpha : nullptr, a ? a->log_beta : nullptr, c.w, c.bias, r1, r2, y,
                             (int64_t)Tx * c.cout, c.cout, ln, B, Tx, c.cin, c.cout, c.ntaps, c.tap_off, alpha, stream);
  };
  auto act = [&](const ItTsAct& a, const uint16_t* x, uint16_t* y, int C, int Tx, const int32_t* ln) {
    return itts_aa_snakebeta_fwd(x, y, a.up12, a.down12, a.log_alpha, a.log_beta, ln, B, C, Tx, (int64_t)Tx * C, C, 1,
                                 (int64_t)Tx * C, C, 1, ITTS_BF16, ITTS_BF16, stream);
  };

  rc = conv(w->conv_pre, static_cast<const uint16_t*>(latent), T, xs_a, T, lens, nullptr, nullptr, 1.0f, pre_b, 1, 0);
  uint16_t* cur_in = xs_a;
  int Tcur = T;
  for (int i = 0; i < ns && rc == 0; ++i) {
    const ItTsBigvganStage& st = w->stages[i];
    const int u = st.up_rate, C = stage_channels(st), Tn = Tcur * u;
    const int32_t* ln_in = lens + (int64_t)i * B;
    const int32_t* ln = lens + (int64_t)(i + 1) * B;
    const float* sb = reinterpret_cast<const float*>(ws + L.stage_b[i]);
    if (fused_up(st))  // [B][Tcur][u*C] output rows are the [B][Tn][C] rows, speaker bias per phase block
      rc = conv(st.phases[0], cur_in, Tcur, xst, Tcur, ln_in, nullptr, nullptr, 1.0f, sb, 1, 0);
    else
      for (int rho = 0; rho < u && rc == 0; ++rho)
        rc = conv(st.phases[rho], cur_in, Tcur, xst, Tn, ln_in, nullptr, nullptr, 1.0f, sb, u, rho);
    uint16_t* xs = (i % 2 == 0) ? xs_b : xs_a;
    for (int j = 0; j < st.n_blocks && rc == 0; ++j) {
      const uint16_t* src = xst;
      for (int n = 0; n < st.n_layers && rc == 0; ++n) {
        const ItTsAmpLayer& ly = st.layers[j * st.n_layers + n];
        const bool last = n == st.n_layers - 1;
        const float alpha = (last && j == st.n_blocks - 1) ? 1.0f / st.n_blocks : 1.0f;
        uint16_t* dst = last ? xs : cur;
        const uint16_t* r2 = (last && j > 0) ? xs : nullptr;
        if (st.amp_mode == 1) {  // activation fused into the conv's input staging
          rc = amp(ly.c1, src, Tn, t2, ln, &ly.a1, nullptr, nullptr, 1.0f);
          if (!rc) rc = amp(ly.c2, t2, Tn, dst, ln, &ly.a2, src, r2, alpha);
        } else if (st.amp_mode == 2) {  // activation kernel + the conv kernel without activation
          rc = act(ly.a1, src, t1, C, Tn, ln);
          if (!rc) rc = amp(ly.c1, t1, Tn, t2, ln, nullptr, nullptr, nullptr, 1.0f);
          if (!rc) rc = act(ly.a2, t2, t1, C, Tn, ln);
          if (!rc) rc = amp(ly.c2, t1, Tn, dst, ln, nullptr, src, r2, alpha);
        } else {  // activation kernel + implicit-GEMM conv
          rc = act(ly.a1, src, t1, C, Tn, ln);
          if (!rc) rc = conv(ly.c1, t1, Tn, t2, Tn, ln, nullptr, nullptr, 1.0f, nullptr, 1, 0);
          if (!rc) rc = act(ly.a2, t2, t1, C, Tn, ln);
          if (!rc) rc = conv(ly.c2, t1, Tn, dst, Tn, ln, src, r2, alpha, nullptr, 1, 0);
        }
        src = dst;
      }
    }
    cur_in = xs;
    Tcur = Tn;
  }
  if (rc) return rc;
  const int Cl = stage_channels(w->stages[ns - 1]);
  const int32_t* ln = lens + (int64_t)ns * B;
  // activation_post + conv_post + tanh (+ int16): one launch where the last stage is one MFMA channel block
  // (IndexTTS-1.5: 24 channels; bit-identical to the two launches below)
  if (Cl % 8 == 0 && Cl <= 32 && (w->post_k & 1) && w->post_k <= 15 && tail_fused())
    return itts_act_conv_post_tanh(cur_in, (int64_t)Tcur * Cl, Cl, w->act_post.up12, w->act_post.down12,
                                   w->act_post.log_alpha, w->act_post.log_beta, w->post_w, w->post_b, Cl, w->post_k, ln,
                                   B, Tcur, wav, pcm, Tcur, stream);
  rc = act(w->act_post, cur_in, t1, Cl, Tcur, ln);
  if (rc) return rc;
  return itts_conv_post_tanh(t1, (int64_t)Tcur * Cl, Cl, w->post_w, w->post_b, Cl, w->post_k, ln, B, Tcur, wav, pcm,
                             Tcur, ITTS_BF16, stream);
}
