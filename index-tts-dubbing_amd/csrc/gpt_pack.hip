// Host-side weight packers of the decode step (CPU code, host memory in and out; no HIP call): the
// layouts the decode kernels and the persistent layer read, so that a host without Python (cgo / JNI /
// plain C) builds ItTsGptLayerW / ItTsGptPlLayerW from the checkpoint tensors alone.
// HipGPT (indextts/gpt/engine.py) packs through these same entry points; tests/test_pack.py checks them
// against a torch restatement of the layouts.
//
// Reference tensors: HF Conv1D weights [in][out] of GPT2Block (modeling_gpt2.py:246-306; the
// UnifiedVoice keys gpt.h.{i}.attn.c_attn / attn.c_proj / mlp.c_fc / mlp.c_proj, gpt/model.py:255-281)
// and mel_head [V][D] (gpt/model.py:48).
#include <cstring>

#include "common.h"

namespace {

// f32 -> bf16, round to nearest even (finite values; what torch's .to(torch.bfloat16) does)
inline uint16_t host_f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline double host_bf2d(uint16_t v) {
  const uint32_t u = (uint32_t)v << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return (double)f;
}

}  // namespace

extern "C" int itts_gpt_fold_ln(const float* w_io, const float* bias, const float* ln_g, const float* ln_b, int K,
                                int N, uint16_t* wt, float* u, float* c) {
  const char* fn = "itts_gpt_fold_ln";
  ITTS_REQUIRE(w_io && bias && wt && c && K > 0 && N > 0, fn, "null pointer or bad sizes");
  ITTS_REQUIRE((ln_g == nullptr) == (ln_b == nullptr), fn, "ln_g and ln_b: both or neither");
  ITTS_REQUIRE(!ln_g || u, fn, "u is required with a LayerNorm");
  for (int n = 0; n < N; ++n) {
    double us = 0.0, cs = 0.0;
    for (int k = 0; k < K; ++k) {
      const double w = (double)w_io[(int64_t)k * N + n];
      if (ln_g) {
        // W' = diag(g) W in double, rounded to f32, then to bf16 (engine.fold_ln_weights' sequence)
        const uint16_t r = host_f2bf((float)(w * (double)ln_g[k]));
        wt[(int64_t)n * K + k] = r;
        us += host_bf2d(r);  // column sums of the ROUNDED W' (sums of bf16 values: exact in double)
        cs += (double)ln_b[k] * w;
      } else {
        wt[(int64_t)n * K + k] = host_f2bf((float)w);
      }
    }
    if (ln_g) u[n] = (float)us;
    c[n] = (float)(cs + (double)bias[n]);
  }
  return 0;
}

extern "C" int itts_gpt_pack_frag(const void* wt, int wt_dtype, int N, int K, int cols, uint16_t* out) {
  const char* fn = "itts_gpt_pack_frag";
  ITTS_REQUIRE(wt && out && N > 0 && K > 0, fn, "null pointer or bad sizes");
  ITTS_REQUIRE(cols == 16 || cols == 32, fn, "cols must be 16 or 32");
  ITTS_REQUIRE(wt_dtype == ITTS_F32 || wt_dtype == ITTS_BF16, fn, "wt_dtype must be f32 or bf16");
  const int ks = cols == 32 ? 16 : 32;  // K per fragment step
  ITTS_REQUIRE(K % ks == 0, fn, "K must be a multiple of 16 (cols 32) / 32 (cols 16)");
  const int64_t Np = (int64_t)(N + cols - 1) / cols * cols;
  auto src = [&](int64_t n, int64_t k) -> uint16_t {
    if (n >= N) return 0;
    return wt_dtype == ITTS_BF16 ? static_cast<const uint16_t*>(wt)[n * K + k]
                                 : host_f2bf(static_cast<const float*>(wt)[n * K + k]);
  };
  for (int64_t nt = 0; nt < Np / cols; ++nt)
    for (int64_t s = 0; s < K / ks; ++s)
      for (int lane = 0; lane < 64; ++lane) {
        const int r = lane % cols, q = lane / cols;  // lane = cols q + r: K-halves (32) / quarters (16)
        uint16_t* o = out + ((nt * (K / ks) + s) * 64 + lane) * 8;
        for (int e = 0; e < 8; ++e) o[e] = src(nt * cols + r, s * ks + 8 * q + e);
      }
  return 0;
}

extern "C" int itts_gpt_pack_qkv12(const uint16_t* wt, const float* u, const float* c, int D, int H, uint16_t* w12,
                                   float* uc) {
  const char* fn = "itts_gpt_pack_qkv12";
  ITTS_REQUIRE(wt && u && c && w12 && uc, fn, "null pointer");
  ITTS_REQUIRE(D == 1024 && H == 16, fn, "the persistent layer's shape: d_model 1024, 16 heads");
  const int K = D, S = K / 32;
  for (int b = 0; b < 256; ++b) {
    const int cl = b % 8, j = b / 8, h = 2 * cl + j / 16;
    for (int t = 0; t < 12; ++t) {
      const int i = 12 * (j % 16) + t;                        // index in head h's [q | k | v] 192 columns
      const int64_t col = (int64_t)(i / 64) * D + h * 64 + i % 64;  // c_attn output column
      uc[(b * 2 + 0) * 12 + t] = u[col];
      uc[(b * 2 + 1) * 12 + t] = c[col];
      for (int s = 0; s < S; ++s)
        for (int q = 0; q < 4; ++q)
          for (int e = 0; e < 8; ++e)
            w12[((((int64_t)b * S + s) * 4 + q) * 12 + t) * 8 + e] = wt[col * K + 32 * s + 8 * q + e];
    }
  }
  return 0;
}
