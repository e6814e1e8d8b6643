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

// RelPositionMultiHeadedAttention (gpt/conformer/attention.py:235-312, no rel_shift) for head dim 64:
// score(i, j) = ((q_i + u) . k_j + (q_i + v) . p_j) * scale over keys j < len (others excluded, an
// all-masked row gives 0 -- the reference's masked_fill(-inf) / softmax / masked_fill(0)), softmax,
// @ v.  A workgroup takes 32 query steps of one (row, head): the 128-wide concatenations (q+u | q+v)
// and (k | p) make the two products one dot product; keys in tiles of 64 through LDS with an online
// softmax.  f32 FMA throughout, fixed order: a row's result does not depend on the batch.
template <typename OutT>
__global__ __launch_bounds__(256) void rel_attn_kernel(const float* __restrict__ qkv, int64_t ldq,
                                                       const float* __restrict__ pos, int64_t ldp,
                                                       const float* __restrict__ bu, const float* __restrict__ bv,
                                                       const int32_t* __restrict__ lens, int T, int H, float scale,
                                                       OutT* __restrict__ out, int64_t ldo) {
  // row pitches padded to 4 mod 32 words: the 8 keys / rows a wave reads with 16-B loads hit distinct banks
  constexpr int DK = 64, QR = 32, KT = 64, QP = 2 * DK + 4, VP = DK + 4, PP = KT + 4;
  __shared__ __attribute__((aligned(16))) float qs[QR * QP];
  __shared__ __attribute__((aligned(16))) float ks[KT * QP];
  __shared__ __attribute__((aligned(16))) float vs[KT * VP];
  __shared__ __attribute__((aligned(16))) float ps[QR * PP];
  const int i0 = blockIdx.x * QR, h = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
  const int C = H * DK, len = lens ? min(lens[b], T) : T;
  const float* base = qkv + (int64_t)b * T * ldq;
  for (int e = tid; e < QR * DK / 4; e += 256) {
    const int r = e / (DK / 4), d = (e - r * (DK / 4)) * 4, t = i0 + r;
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < T) q = *reinterpret_cast<const float4*>(base + (int64_t)t * ldq + h * DK + d);
    const float4 u = *reinterpret_cast<const float4*>(bu + h * DK + d);
    const float4 v = *reinterpret_cast<const float4*>(bv + h * DK + d);
    *reinterpret_cast<float4*>(qs + r * QP + d) = make_float4(q.x + u.x, q.y + u.y, q.z + u.z, q.w + u.w);
    *reinterpret_cast<float4*>(qs + r * QP + DK + d) = make_float4(q.x + v.x, q.y + v.y, q.z + v.z, q.w + v.w);
  }
  const int r = tid >> 3, g = tid & 7;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mrun = -INFINITY, lrun = 0.f;
  for (int k0 = 0; k0 < len; k0 += KT) {
    __syncthreads();  // previous tile fully consumed (and qs written)
    for (int e = tid; e < KT * DK / 4; e += 256) {
      const int j = e / (DK / 4), d = (e - j * (DK / 4)) * 4, t = k0 + j;
      float4 kk = make_float4(0.f, 0.f, 0.f, 0.f), pp = kk, vv = kk;
      if (t < len) {
        const float* row = base + (int64_t)t * ldq;
        kk = *reinterpret_cast<const float4*>(row + C + h * DK + d);
        vv = *reinterpret_cast<const float4*>(row + 2 * C + h * DK + d);
        pp = *reinterpret_cast<const float4*>(pos + (int64_t)t * ldp + h * DK + d);
      }
      *reinterpret_cast<float4*>(ks + j * QP + d) = kk;
      *reinterpret_cast<float4*>(ks + j * QP + DK + d) = pp;
      *reinterpret_cast<float4*>(vs + j * VP + d) = vv;
    }
    __syncthreads();
    float sc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int d = 0; d < 2 * DK; d += 4) {  // 8 independent dot products, 16-B LDS reads
      const float4 q = *reinterpret_cast<const float4*>(qs + r * QP + d);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const float4 kv = *reinterpret_cast<const float4*>(ks + (g + 8 * m) * QP + d);
        sc[m] = fmaf(q.x, kv.x, sc[m]);
        sc[m] = fmaf(q.y, kv.y, sc[m]);
        sc[m] = fmaf(q.z, kv.z, sc[m]);
        sc[m] = fmaf(q.w, kv.w, sc[m]);
      }
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      sc[m] = (k0 + g + 8 * m < len) ? sc[m] * scale : -INFINITY;
      tmax = fmaxf(tmax, sc[m]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 1, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 2, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 4, 64));
    const float mnew = fmaxf(mrun, tmax);  // finite: key k0 < len is valid
    const float corr = __expf(mrun - mnew);
    float psum = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float pe = sc[m] == -INFINITY ? 0.f : __expf(sc[m] - mnew);
      ps[r * PP + g + 8 * m] = pe;
      psum += pe;
    }
    psum += __shfl_xor(psum, 1, 64);
    psum += __shfl_xor(psum, 2, 64);
    psum += __shfl_xor(psum, 4, 64);
    lrun = lrun * corr + psum;
    mrun = mnew;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= corr;
    __syncthreads();
    for (int j = 0; j < KT; j += 4) {
      const float4 pe = *reinterpret_cast<const float4*>(ps + r * PP + j);
      const float pj[4] = {pe.x, pe.y, pe.z, pe.w};
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float4 v0 = *reinterpret_cast<const float4*>(vs + (j + jj) * VP + g * 8);
        const float4 v1 = *reinterpret_cast<const float4*>(vs + (j + jj) * VP + g * 8 + 4);
        acc[0] = fmaf(pj[jj], v0.x, acc[0]);
        acc[1] = fmaf(pj[jj], v0.y, acc[1]);
        acc[2] = fmaf(pj[jj], v0.z, acc[2]);
        acc[3] = fmaf(pj[jj], v0.w, acc[3]);
        acc[4] = fmaf(pj[jj], v1.x, acc[4]);
        acc[5] = fmaf(pj[jj], v1.y, acc[5]);
        acc[6] = fmaf(pj[jj], v1.z, acc[6]);
        acc[7] = fmaf(pj[jj], v1.w, acc[7]);
      }
    }
  }
  const int t = i0 + r;
  if (t >= T) return;
  const float inv = lrun > 0.f ? 1.f / lrun : 0.f;
  OutT* o = out + ((int64_t)b * T + t) * ldo + h * DK + g * 8;
#pragma unroll
  for (int i = 0; i < 8; ++i) St<OutT>::st(o + i, acc[i] * inv);
}

// ECAPA (channel-last product path): y[b][tp][c] = bf16(x[b][src(tp)][c] (+ x2[b][src(tp)][c])) for
// tp < T + 2 pad, src reflecting at the ends (speechbrain "same" reflect padding) or zero padding;
// channels [C, Cp) zero (pads Cin to a multiple of 8 for the 16-B igemm loads).  4 channels per thread.
__global__ __launch_bounds__(256) void pad_rows_kernel(const float* __restrict__ x, int64_t x_sb, int64_t ldx,
                                                       const float* __restrict__ x2, int64_t x2_sb, int64_t ldx2,
                                                       int T, int C, int pad, int reflect, int Cp,
                                                       uint16_t* __restrict__ y) {
  const int Tp = T + 2 * pad, b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (tp, c4)
  const int cq = Cp / 4;
  if (i >= (int64_t)Tp * cq) return;
  const int tp = (int)(i / cq), c = (int)(i - (int64_t)tp * cq) * 4;
  int t = tp - pad;
  bool ok = true;
  if (t < 0 || t >= T) {
    if (reflect) t = t < 0 ? -t : 2 * (T - 1) - t;
    else ok = false;
  }
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + k < C) {
        v[k] = x[(int64_t)b * x_sb + (int64_t)t * ldx + c + k];
        if (x2) v[k] += x2[(int64_t)b * x2_sb + (int64_t)t * ldx2 + c + k];
      }
  }
  *reinterpret_cast<uint2*>(y + ((int64_t)b * Tp + tp) * Cp + c) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
}

// y = relu(x) * scale[c] + shift[c] (TDNNBlock: BatchNorm1d(eval) after ReLU, folded to an affine map)
__global__ __launch_bounds__(256) void relu_affine_kernel(const float* __restrict__ x, int64_t x_sb, int64_t ldx, int T,
                                                          int C, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, float* __restrict__ y,
                                                          int64_t y_sb, int64_t ldy) {
  const int b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)T * C) return;
  const int t = (int)(i / C), c = (int)(i - (int64_t)t * C);
  const float v = x[(int64_t)b * x_sb + (int64_t)t * ldx + c];
  y[(int64_t)b * y_sb + (int64_t)t * ldy + c] = fmaf(fmaxf(v, 0.f), scale[c], shift[c]);
}

// ECAPA pooling statistics over time (BigVGAN/ECAPA_TDNN.py _compute_statistics): weights w =
// softmax over t of logits[b][t][c] (AttentiveStatisticsPooling's attention) or 1/T when logits is
// null (the global context / SE mean); mean = sum w x, std = sqrt(max(sum w (x - mean)^2, eps)).
// A workgroup = 64 channels x 16 time slices of one utterance; each pass combines the 16 slice
// partials in slice order through LDS (fixed rounding, independent of the batch).
__device__ __forceinline__ float slice_combine(float v, float* red, bool is_max) {
  const int ci = threadIdx.x & 63, sl = threadIdx.x >> 6;
  __syncthreads();  // previous readers of red are done
  red[sl * 64 + ci] = v;
  __syncthreads();
  float acc = red[ci];
  for (int k = 1; k < 16; ++k) acc = is_max ? fmaxf(acc, red[k * 64 + ci]) : acc + red[k * 64 + ci];
  return acc;
}

__global__ __launch_bounds__(1024) void time_stats_kernel(const float* __restrict__ x, int64_t x_sb, int64_t ldx,
                                                          const float* __restrict__ lg, int64_t l_sb, int64_t ldl,
                                                          int T, int C, float eps, float* __restrict__ mean,
                                                          float* __restrict__ stdv) {
  __shared__ float red[16 * 64];
  const int ci = threadIdx.x & 63, sl = threadIdx.x >> 6, c = blockIdx.x * 64 + ci, b = blockIdx.y;
  const bool on = c < C;
  const int per = (T + 15) / 16, t0 = sl * per, t1 = min(T, t0 + per);
  const float* xr = x + (int64_t)b * x_sb + (on ? c : 0);
  const float* lr = lg ? lg + (int64_t)b * l_sb + (on ? c : 0) : nullptr;
  float mx = 0.f, inv = 1.f / (float)T;
  if (lr) {
    float m = -INFINITY;
    if (on)
      for (int t = t0; t < t1; ++t) m = fmaxf(m, lr[(int64_t)t * ldl]);
    mx = slice_combine(m, red, true);
    float d = 0.f;
    if (on)
      for (int t = t0; t < t1; ++t) d += expf(lr[(int64_t)t * ldl] - mx);
    inv = 1.f / slice_combine(d, red, false);
  }
  float m = 0.f;
  if (on)
    for (int t = t0; t < t1; ++t) {
      const float w = lr ? expf(lr[(int64_t)t * ldl] - mx) * inv : inv;
      m = fmaf(w, xr[(int64_t)t * ldx], m);
    }
  m = slice_combine(m, red, false);
  if (on && sl == 0) mean[(int64_t)b * C + c] = m;
  if (!stdv) return;  // uniform per launch
  float v = 0.f;
  if (on)
    for (int t = t0; t < t1; ++t) {
      const float w = lr ? expf(lr[(int64_t)t * ldl] - mx) * inv : inv;
      const float dd = xr[(int64_t)t * ldx] - m;
      v = fmaf(w, dd * dd, v);
    }
  v = slice_combine(v, red, false);
  if (on && sl == 0) stdv[(int64_t)b * C + c] = sqrtf(fmaxf(v, eps));
}


// ---- perceiver cross-attention (PerceiverResampler Attention, gpt/perceiver.py:111-150, 296-317) ----
// out[b][i][h*64 + d] = softmax_j(q_i . k_j * scale, keys with key_mask[b][j] == 0 excluded) . v_j, f32,
// one workgroup per (head, prompt): 256 threads = the 32 latent queries x 8 lanes (8 dims each, DPP
// sums), keys streamed through LDS in 64-key tiles with an online softmax in a fixed order -- a
// prompt's result does not depend on the other prompts in the batch (the torch batched-GEMM form did,
// by up to 5e-3 rel-RMS).  The reference fills masked scores with -finfo.max; the 32 latent keys are
// never masked, so dropping masked keys is the same softmax.
constexpr int kXq = 32, kXt = 64;
__global__ __launch_bounds__(256) void cross_attn_kernel(const float* __restrict__ q, int64_t q_sb, int64_t ldq,
                                                         const float* __restrict__ k, const float* __restrict__ v,
                                                         int64_t kv_sb, int64_t ldkv, const uint8_t* __restrict__ kmask,
                                                         int nk, float scale, float* __restrict__ out, int64_t o_sb,
                                                         int64_t ldo) {
  __shared__ float Ks[kXt][65], Vs[kXt][65];
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, qi = tid >> 3, d8 = tid & 7;
  float qv[8], o[8];
  const float* qr = q + (int64_t)b * q_sb + (int64_t)qi * ldq + h * 64 + 8 * d8;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    qv[e] = qr[e] * scale;
    o[e] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  const float* kb = k + (int64_t)b * kv_sb + h * 64;
  const float* vb = v + (int64_t)b * kv_sb + h * 64;
  const uint8_t* mk = kmask ? kmask + (int64_t)b * nk : nullptr;
  for (int j0 = 0; j0 < nk; j0 += kXt) {
    __syncthreads();
    for (int e = tid; e < kXt * 64; e += 256) {
      const int r = e >> 6, d = e & 63, jj = j0 + r;
      Ks[r][d] = jj < nk ? kb[(int64_t)jj * ldkv + d] : 0.f;
      Vs[r][d] = jj < nk ? vb[(int64_t)jj * ldkv + d] : 0.f;
    }
    __syncthreads();
    const int n = min(kXt, nk - j0);
    for (int r = 0; r < n; ++r) {
      if (mk && !mk[j0 + r]) continue;  // uniform over the workgroup
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s = fmaf(qv[e], Ks[r][8 * d8 + e], s);
      s = sum8_dpp(s);
      const float mn = fmaxf(m, s);
      const float corr = __expf(m - mn), pr = __expf(s - mn);
      l = l * corr + pr;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(pr, Vs[r][8 * d8 + e], o[e] * corr);
      m = mn;
    }
  }
  float* orow = out + (int64_t)b * o_sb + (int64_t)qi * ldo + h * 64 + 8 * d8;
  const float inv = 1.0f / l;
#pragma unroll
  for (int e = 0; e < 8; ++e) orow[e] = o[e] * inv;
}

}  // namespace

extern "C" int itts_time_stats(const float* x, int64_t x_sb, int64_t ldx, const float* logits, int64_t l_sb,
                               int64_t ldl, int B, int T, int C, float eps, float* mean, float* stdv, void* stream) {
  const char* fn = "itts_time_stats";
  ITTS_REQUIRE(B >= 0 && T > 0 && C > 0, fn, "bad sizes (T > 0)");
  if (B == 0) return 0;
  ITTS_REQUIRE(x && mean, fn, "null pointer");
  hipLaunchKernelGGL(time_stats_kernel, dim3((C + 63) / 64, B), dim3(1024), 0, itts::as_stream(stream), x, x_sb, ldx,
                     logits, l_sb, ldl, T, C, eps, mean, stdv);
  return itts::check_launch(fn);
}

extern "C" int itts_pad_rows_bf16(const float* x, int64_t x_sb, int64_t ldx, const float* x2, int64_t x2_sb,
                                  int64_t ldx2, int B, int T, int C, int pad, int reflect, int Cp, void* y,
                                  void* stream) {
  const char* fn = "itts_pad_rows_bf16";
  ITTS_REQUIRE(B >= 0 && T >= 0 && C > 0 && pad >= 0 && Cp >= C && Cp % 4 == 0, fn, "bad sizes (Cp >= C, Cp % 4 == 0)");
  ITTS_REQUIRE(!reflect || pad < T, fn, "reflect padding needs pad < T");
  if (B == 0 || T == 0) return 0;
  ITTS_REQUIRE(x && y && (reinterpret_cast<uintptr_t>(y) & 7) == 0, fn, "null pointer or y not 8-byte aligned");
  const int64_t n = (int64_t)(T + 2 * pad) * (Cp / 4);
  hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, itts::as_stream(stream), x,
                     x_sb, ldx, x2, x2_sb, ldx2, T, C, pad, reflect, Cp, static_cast<uint16_t*>(y));
  return itts::check_launch(fn);
}

extern "C" int itts_relu_affine_rows(const float* x, int64_t x_sb, int64_t ldx, int B, int T, int C, const float* scale,
                                     const float* shift, float* y, int64_t y_sb, int64_t ldy, void* stream) {
  const char* fn = "itts_relu_affine_rows";
  ITTS_REQUIRE(B >= 0 && T >= 0 && C > 0, fn, "bad sizes");
  if (B == 0 || T == 0) return 0;
  ITTS_REQUIRE(x && scale && shift && y, fn, "null pointer");
  const int64_t n = (int64_t)T * C;
  hipLaunchKernelGGL(relu_affine_kernel, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, itts::as_stream(stream),
                     x, x_sb, ldx, T, C, scale, shift, y, y_sb, ldy);
  return itts::check_launch(fn);
}

extern "C" int itts_cond_rel_attn(const float* qkv, int64_t ld_qkv, const float* pos, int64_t ld_pos,
                                  const float* bias_u, const float* bias_v, const int32_t* lens, int B, int T, int H,
                                  float scale, void* out, int64_t ld_out, int out_dtype, void* stream) {
  const char* fn = "itts_cond_rel_attn";
  ITTS_REQUIRE(B >= 0 && T >= 0 && H > 0, fn, "bad sizes");
  ITTS_REQUIRE(ld_qkv >= 3 * 64 * H && ld_pos >= 64 * H && ld_out >= 64 * H, fn, "head dim 64: ld_qkv >= 3C, ld_out >= C");
  ITTS_REQUIRE(out_dtype == ITTS_F32 || out_dtype == ITTS_BF16, fn, "out dtype f32 (0) or bf16 (1)");
  if (B == 0 || T == 0) return 0;
  ITTS_REQUIRE(qkv && pos && bias_u && bias_v && out, fn, "null pointer");
  ITTS_REQUIRE(ld_qkv % 4 == 0 && ld_pos % 4 == 0 && ((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(pos) |
                reinterpret_cast<uintptr_t>(bias_u) | reinterpret_cast<uintptr_t>(bias_v)) & 15) == 0,
               fn, "qkv, pos, biases 16-byte aligned with row pitches a multiple of 4");
  dim3 grid((T + 31) / 32, H, B);
  if (out_dtype == ITTS_BF16)
    hipLaunchKernelGGL(rel_attn_kernel<uint16_t>, grid, dim3(256), 0, itts::as_stream(stream), qkv, ld_qkv, pos, ld_pos,
                       bias_u, bias_v, lens, T, H, scale, static_cast<uint16_t*>(out), ld_out);
  else
    hipLaunchKernelGGL(rel_attn_kernel<float>, grid, dim3(256), 0, itts::as_stream(stream), qkv, ld_qkv, pos, ld_pos,
                       bias_u, bias_v, lens, T, H, scale, static_cast<float*>(out), ld_out);
  return itts::check_launch(fn);
}

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

extern "C" int itts_cross_attn(const float* q, int64_t q_sb, int64_t ldq, const float* k, const float* v, int64_t kv_sb,
                               int64_t ldkv, const uint8_t* key_mask, int B, int nq, int nk, int heads, float scale,
                               float* out, int64_t o_sb, int64_t ldo, void* stream) {
  const char* fn = "itts_cross_attn";
  ITTS_REQUIRE(B >= 0 && heads > 0 && nk >= 1, fn, "bad sizes");
  if (B == 0) return 0;
  ITTS_REQUIRE(q && k && v && out, fn, "null pointer");
  ITTS_REQUIRE(nq == kXq, fn, "32 latent queries (PerceiverResampler num_latents)");
  hipLaunchKernelGGL(cross_attn_kernel, dim3(heads, B), dim3(256), 0, itts::as_stream(stream), q, q_sb, ldq, k, v,
                     kv_sb, ldkv, key_mask, nk, scale, out, o_sb, ldo);
  return itts::check_launch(fn);
}
