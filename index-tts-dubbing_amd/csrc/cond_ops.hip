// Fused kernels of the prompt conditioning encoder's bf16 product path (HipGPT.conditioning(fast=True),
// indextts/gpt/conditioning.py).  The reference computes the encoder under fp16 autocast in its product
// mode (infer.py:572-586); these two kernels replace the permute/cast/unfold chains that dominated the
// per-prompt phase (profiles/prof_prompt_r03.txt: ~8 ms of copies for 32 prompts of 511 frames).
//
//  * itts_cond_subsample: Conv2dSubsampling2 (gpt/conformer/subsampling.py:164-190) = conv2d(1 -> C,
//    3x3, stride 2) + ReLU over the mel image x[time][bin] = mel[bin][time], written channel-last as
//    bf16 y[b][t][f][c] -- the A operand of the following Linear(C * F -> D) once its weight columns are
//    permuted from (c, f) to (f, c) order (utils/hiplinear.py), so no transpose is ever materialised.
//  * itts_cond_glu_dwconv: the middle of ConvolutionModule (gpt/conformer_encoder.py:108-167):
//    GLU over channels, depthwise conv1d (k odd, zero padding k/2 at the sequence ends), LayerNorm over
//    channels, SiLU -> bf16 rows (the A operand of pointwise_conv2).  One workgroup per (row, time step).
#include "common.h"

namespace {

// one workgroup per (t, b); thread tid owns channel group cg = tid % (C / 8) for every f it visits
__global__ __launch_bounds__(256) void subsample_kernel(const float* __restrict__ mel, int64_t mel_sb, int64_t mel_ld,
                                                        int n_bins, const float* __restrict__ w,
                                                        const float* __restrict__ bias, int C, int To, int Fo,
                                                        uint16_t* __restrict__ y) {
  extern __shared__ float rows[];  // [3][n_bins]: mel time rows 2t .. 2t + 2
  const int t = blockIdx.x, b = blockIdx.y;
  const float* src = mel + (int64_t)b * mel_sb + 2 * t;
  for (int i = threadIdx.x; i < 3 * n_bins; i += 256) {
    const int r = i / n_bins, f = i - r * n_bins;
    rows[i] = src[(int64_t)f * mel_ld + r];
  }
  const int ngrp = C / 8, cg = threadIdx.x % ngrp;
  float wr[8][9], br[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    br[c] = bias[cg * 8 + c];
#pragma unroll
    for (int k = 0; k < 9; ++k) wr[c][k] = w[(cg * 8 + c) * 9 + k];
  }
  __syncthreads();
  uint16_t* yr = y + ((int64_t)b * To + t) * Fo * C + cg * 8;
  for (int f = threadIdx.x / ngrp; f < Fo; f += 256 / ngrp) {
    float v[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) v[i * 3 + j] = rows[i * n_bins + 2 * f + j];
    uint32_t o[4];
#pragma unroll
    for (int c = 0; c < 8; c += 2) {
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        a0 = fmaf(v[k], wr[c][k], a0);
        a1 = fmaf(v[k], wr[c + 1][k], a1);
      }
      o[c / 2] = pack2bf(fmaxf(a0 + br[c], 0.f), fmaxf(a1 + br[c + 1], 0.f));
    }
    *reinterpret_cast<uint4*>(yr + (int64_t)f * C) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// one workgroup per (t, b), 4 channels per thread (C / 4 threads, padded to whole waves)
__global__ __launch_bounds__(1024) void glu_dwconv_kernel(const float* __restrict__ a, int64_t lda, int T, int C,
                                                          const float* __restrict__ w, const float* __restrict__ wb,
                                                          int K, const float* __restrict__ g,
                                                          const float* __restrict__ be, float eps,
                                                          uint16_t* __restrict__ y, int64_t ldy) {
  __shared__ float red[16];
  const int t = blockIdx.x, b = blockIdx.y;
  const int c = threadIdx.x * 4;
  const bool on = c < C;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (on) {
    const float* ab = a + (int64_t)b * T * lda;
    const int h = K / 2;
    for (int j = 0; j < K; ++j) {
      const int tt = t + j - h;
      if (tt < 0 || tt >= T) continue;
      const float4 x = *reinterpret_cast<const float4*>(ab + (int64_t)tt * lda + c);
      const float4 gt = *reinterpret_cast<const float4*>(ab + (int64_t)tt * lda + C + c);
      acc[0] = fmaf(x.x * sigm(gt.x), w[(c + 0) * K + j], acc[0]);
      acc[1] = fmaf(x.y * sigm(gt.y), w[(c + 1) * K + j], acc[1]);
      acc[2] = fmaf(x.z * sigm(gt.z), w[(c + 2) * K + j], acc[2]);
      acc[3] = fmaf(x.w * sigm(gt.w), w[(c + 3) * K + j], acc[3]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += wb[c + i];
  }
  const float mean = block_sum(on ? acc[0] + acc[1] + acc[2] + acc[3] : 0.f, red) / C;
  float d2 = 0.f;
  if (on)
#pragma unroll
    for (int i = 0; i < 4; ++i) d2 += (acc[i] - mean) * (acc[i] - mean);
  const float var = block_sum(d2, red) / C;
  if (!on) return;
  const float rs = rsqrtf(var + eps);
  float o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float z = (acc[i] - mean) * rs * g[c + i] + be[c + i];
    o[i] = z * sigm(z);
  }
  *reinterpret_cast<uint2*>(y + ((int64_t)b * T + t) * ldy + c) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
}

// tiled form (C = 256, 512 or 1024): a workgroup takes TT time steps of one row.  GLU of the TT + K - 1
// input steps once into LDS (f32), then per round every wave owns one (step, 256-channel) slice:
// depthwise taps from LDS with the transposed weights wt[K][C] (16-B loads), LayerNorm statistics as
// wave sums combined in wave order (fixed: run-to-run identical), SiLU, 8-B bf16 stores.
__global__ __launch_bounds__(256) void glu_dwconv_tiled_kernel(const float* __restrict__ a, int64_t lda, int T, int C,
                                                               const float* __restrict__ wt,
                                                               const float* __restrict__ wb, int K, int TT,
                                                               const float* __restrict__ g,
                                                               const float* __restrict__ be, float eps,
                                                               uint16_t* __restrict__ y, int64_t ldy) {
  extern __shared__ float glu[];  // [TT + K - 1][C]
  __shared__ float wsum[4];
  const int t0 = blockIdx.x * TT, b = blockIdx.y, h = K / 2, nr = TT + K - 1, C4 = C / 4;
  const float* ab = a + (int64_t)b * T * lda;
  for (int i = threadIdx.x; i < nr * C4; i += 256) {
    const int r = i / C4, c = (i - r * C4) * 4, tt = t0 - h + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tt >= 0 && tt < T) {
      const float4 x = *reinterpret_cast<const float4*>(ab + (int64_t)tt * lda + c);
      const float4 gt = *reinterpret_cast<const float4*>(ab + (int64_t)tt * lda + C + c);
      v = make_float4(x.x * sigm(gt.x), x.y * sigm(gt.y), x.z * sigm(gt.z), x.w * sigm(gt.w));
    }
    *reinterpret_cast<float4*>(glu + (int64_t)r * C + c) = v;
  }
  __syncthreads();
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, wpr = C4 / 64;  // waves per step
  const int nround = (TT * wpr + 3) / 4;
  for (int k = 0; k < nround; ++k) {
    const int item = k * 4 + wid;  // (step, slice) in step-major order
    const int tl = item / wpr, sl = item - tl * wpr, t = t0 + tl;
    const bool on = tl < TT && t < T;
    const int c = (sl * 64 + lane) * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (on) {
      const float4 bb = *reinterpret_cast<const float4*>(wb + c);
      acc[0] = bb.x, acc[1] = bb.y, acc[2] = bb.z, acc[3] = bb.w;
      for (int j = 0; j < K; ++j) {
        const float4 gv = *reinterpret_cast<const float4*>(glu + (int64_t)(tl + j) * C + c);
        const float4 wv = *reinterpret_cast<const float4*>(wt + (int64_t)j * C + c);
        acc[0] = fmaf(gv.x, wv.x, acc[0]);
        acc[1] = fmaf(gv.y, wv.y, acc[1]);
        acc[2] = fmaf(gv.z, wv.z, acc[2]);
        acc[3] = fmaf(gv.w, wv.w, acc[3]);
      }
    }
    // the wpr waves of one step are consecutive wave ids: combine their sums in wave order
    const int first = wid - sl;
    float sm = wave_sum(acc[0] + acc[1] + acc[2] + acc[3]);
    __syncthreads();
    if (lane == 0) wsum[wid] = sm;
    __syncthreads();
    float tot = 0.f;
    for (int i = 0; i < wpr; ++i) tot += wsum[first + i];
    const float mean = tot / C;
    float d2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) d2 += (acc[i] - mean) * (acc[i] - mean);
    d2 = wave_sum(d2);
    __syncthreads();
    if (lane == 0) wsum[wid] = d2;
    __syncthreads();
    float var = 0.f;
    for (int i = 0; i < wpr; ++i) var += wsum[first + i];
    var /= C;
    if (on) {
      const float rs = rsqrtf(var + eps);
      const float4 gg = *reinterpret_cast<const float4*>(g + c);
      const float4 bt = *reinterpret_cast<const float4*>(be + c);
      const float z0 = (acc[0] - mean) * rs * gg.x + bt.x, z1 = (acc[1] - mean) * rs * gg.y + bt.y;
      const float z2 = (acc[2] - mean) * rs * gg.z + bt.z, z3 = (acc[3] - mean) * rs * gg.w + bt.w;
      *reinterpret_cast<uint2*>(y + ((int64_t)b * T + t) * ldy + c) =
          make_uint2(pack2bf(z0 * sigm(z0), z1 * sigm(z1)), pack2bf(z2 * sigm(z2), z3 * sigm(z3)));
    }
  }
}

}  // namespace

extern "C" int itts_cond_subsample(const float* mel, int64_t mel_sb, int64_t mel_ld, int B, int n_bins, int T,
                                   const float* w, const float* bias, int C, void* y, void* stream) {
  const char* fn = "itts_cond_subsample";
  ITTS_REQUIRE(B >= 0 && n_bins >= 3 && T >= 0 && C > 0, fn, "bad sizes");
  ITTS_REQUIRE(C % 8 == 0 && 256 % (C / 8) == 0, fn, "C must be 8 x a power of two <= 2048");
  const int To = T >= 3 ? (T - 3) / 2 + 1 : 0, Fo = (n_bins - 3) / 2 + 1;
  if (B == 0 || To == 0) return 0;
  ITTS_REQUIRE(mel && w && bias && y, fn, "null pointer");
  ITTS_REQUIRE((reinterpret_cast<uintptr_t>(y) & 15) == 0, fn, "y must be 16-byte aligned");
  hipLaunchKernelGGL(subsample_kernel, dim3(To, B), dim3(256), 3 * n_bins * sizeof(float), itts::as_stream(stream),
                     mel, mel_sb, mel_ld, n_bins, w, bias, C, To, Fo, static_cast<uint16_t*>(y));
  return itts::check_launch(fn);
}

extern "C" int itts_cond_glu_dwconv(const float* a, int64_t lda, int B, int T, int C, const float* w,
                                    const float* w_bias, int K, const float* ln_g, const float* ln_b, float eps,
                                    void* y, int64_t ldy, const float* w_t, void* stream) {
  const char* fn = "itts_cond_glu_dwconv";
  ITTS_REQUIRE(B >= 0 && T >= 0 && C > 0 && K >= 1 && K % 2 == 1, fn, "bad sizes (K odd)");
  ITTS_REQUIRE(C % 4 == 0 && C <= 4096 && lda % 4 == 0 && lda >= 2 * C && ldy % 4 == 0 && ldy >= C, fn,
               "C, lda, ldy must be multiples of 4 (C <= 4096)");
  if (B == 0 || T == 0) return 0;
  ITTS_REQUIRE(a && w && w_bias && ln_g && ln_b && y, fn, "null pointer");
  ITTS_REQUIRE((reinterpret_cast<uintptr_t>(a) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 7) == 0, fn,
               "a must be 16-byte, y 8-byte aligned");
  // tiled form: C = 256 / 512 / 1024 (a round of 4 waves holds whole steps), w_t = w transposed [K][C],
  // TT steps per workgroup with the GLU window in at most 64 KB of LDS
  const int TT = 65536 / (4 * C) - (K - 1);
  if (w_t && (C == 256 || C == 512 || C == 1024) && TT >= 4 && ((reinterpret_cast<uintptr_t>(w_t) |
                                                       reinterpret_cast<uintptr_t>(w_bias) |
                                                       reinterpret_cast<uintptr_t>(ln_g) |
                                                       reinterpret_cast<uintptr_t>(ln_b)) & 15) == 0) {
    const int tt = TT < 16 ? TT : 16;
    hipLaunchKernelGGL(glu_dwconv_tiled_kernel, dim3((T + tt - 1) / tt, B), dim3(256),
                       (size_t)(tt + K - 1) * C * sizeof(float), itts::as_stream(stream), a, lda, T, C, w_t, w_bias,
                       K, tt, ln_g, ln_b, eps, static_cast<uint16_t*>(y), ldy);
    return itts::check_launch(fn);
  }
  const int threads = ((C / 4 + 63) / 64) * 64;
  hipLaunchKernelGGL(glu_dwconv_kernel, dim3(T, B), dim3(threads), 0, itts::as_stream(stream), a, lda, T, C, w,
                     w_bias, K, ln_g, ln_b, eps, static_cast<uint16_t*>(y), ldy);
  return itts::check_launch(fn);
}
