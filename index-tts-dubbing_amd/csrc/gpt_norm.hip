// LayerNorm family for the GPT-2 core (HF GPT2Block ln_1/ln_2, ln_f, then UnifiedVoice.final_norm;
// eps 1e-5, HF:modeling_gpt2.py:246-306,620; gpt/model.py:48 -- quirk Q5 double LN before mel_head).
//
//  * itts_layernorm_rows: y[m] = LN2?(LN1(x[m])) for M rows of width D (x f32, y f32|bf16),
//    optional row gather (y row m <- x row idx[m]) so the prefill can normalise only each
//    sequence's last position.
//  * itts_residual_reduce_ln: decode-step split-K epilogue
//       x[b] += bias + sum_s part[s][b]          (deterministic fixed-order sum, no atomics)
//       h[b]  = LN2?(LN1(x[b]))                 (input of the next projection GEMM)
// One 256-thread workgroup per row; two-pass (mean, then centred variance) in f32 like torch.
#include <cstdlib>

#include "common.h"

namespace {
constexpr int kT = 256;
constexpr int kMaxPer = 16;  // D <= 4096

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kT / 64; ++i) s += red[i];
  return s;
}

// normalise the per-thread slice v[0..n) (element index = threadIdx.x + kT*i) in place
__device__ __forceinline__ void ln_inplace(float (&v)[kMaxPer], int n, int D, const float* g, const float* b,
                                           float* red) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i)
    if (i < n) s += v[i];
  const float mean = block_sum(s, red) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i)
    if (i < n) {
      float d = v[i] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(block_sum(q, red) / D + 1e-5f);
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i)
    if (i < n) {
      int e = threadIdx.x + kT * i;
      v[i] = (v[i] - mean) * rstd * g[e] + b[e];
    }
}

template <typename TO>
__global__ __launch_bounds__(kT) void ln_rows_kernel(const float* __restrict__ x, int64_t ldx, const int32_t* __restrict__ idx,
                                                     TO* __restrict__ y, int64_t ldy, int D, const float* g1,
                                                     const float* b1, const float* g2, const float* b2) {
  __shared__ float red[kT / 64];
  const int m = blockIdx.x;
  const float* xr = x + (int64_t)(idx ? idx[m] : m) * ldx;
  float v[kMaxPer];
  const int n = (D - threadIdx.x + kT - 1) / kT;
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i)
    if (i < n) v[i] = xr[threadIdx.x + kT * i];
  ln_inplace(v, n, D, g1, b1, red);
  if (g2) ln_inplace(v, n, D, g2, b2, red);
  TO* yr = y + (int64_t)m * ldy;
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i)
    if (i < n) St<TO>::st(yr + threadIdx.x + kT * i, v[i]);
}

// Decode-step variant: blockDim = D/4 threads, 4 consecutive elements (one float4) per thread, and
// every load of the row (x, bias, all split partials) issued before the first use, so the kernel
// pays one memory round trip instead of one per element group.
constexpr int kMaxSplit = 16;  // 16: one partial per head from itts_attn_decode_proj

__device__ __forceinline__ float block_sum_n(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// g4 / b4: this thread's LayerNorm weights, loaded by the caller together with the row (they do not
// depend on it, so their latency hides under the partial-sum loads instead of following the two
// block reductions: a global load cannot move across the barriers)
__device__ __forceinline__ void ln4(float (&v)[4], int D, const f32x4_t& g4, const f32x4_t& b4, float* red) {
  const float mean = block_sum_n(v[0] + v[1] + v[2] + v[3], red) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) q += (v[i] - mean) * (v[i] - mean);
  const float rstd = rsqrtf(block_sum_n(q, red) / D + 1e-5f);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (v[i] - mean) * rstd * g4[i] + b4[i];
}

template <typename TO>
__global__ __launch_bounds__(1024) void residual_reduce_ln_v4_kernel(
    float* __restrict__ x, int64_t ldx, const float* __restrict__ part, int nsplit, int64_t split_stride, int64_t ldp,
    const float* __restrict__ bias, TO* __restrict__ h, int64_t ldh, int D, const float* g1, const float* b1,
    const float* g2, const float* b2) {
  __shared__ float red[16];
  // without LayerNorm a row is cut into gridDim.y column blocks (more workgroups per launch)
  const int m = blockIdx.x, e = 4 * (blockIdx.y * blockDim.x + threadIdx.x);
  float* xr = x + (int64_t)m * ldx + e;
  f32x4_t acc = *reinterpret_cast<const f32x4_t*>(xr);
  f32x4_t pv[kMaxSplit];
  f32x4_t bv = bias ? *reinterpret_cast<const f32x4_t*>(bias + e) : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < kMaxSplit; ++s)
    if (s < nsplit) pv[s] = ld_stream(reinterpret_cast<const f32x4_t*>(part + s * split_stride + (int64_t)m * ldp + e));
  f32x4_t g1v = {0.f, 0.f, 0.f, 0.f}, b1v = g1v, g2v = g1v, b2v = g1v;
  if (g1) {
    g1v = *reinterpret_cast<const f32x4_t*>(g1 + e);
    b1v = *reinterpret_cast<const f32x4_t*>(b1 + e);
  }
  if (g2) {
    g2v = *reinterpret_cast<const f32x4_t*>(g2 + e);
    b2v = *reinterpret_cast<const f32x4_t*>(b2 + e);
  }
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float p = bv[i];
#pragma unroll
    for (int s = 0; s < kMaxSplit; ++s)
      if (s < nsplit) p += pv[s][i];
    v[i] = acc[i] + p;
  }
  st_out(reinterpret_cast<f32x4_t*>(xr), f32x4_t{v[0], v[1], v[2], v[3]});
  if (!g1) {  // no LayerNorm (folded into the consumer GEMM): h = x, rounded
    if (h) {
      TO* hr = h + (int64_t)m * ldh + e;
#pragma unroll
      for (int i = 0; i < 4; ++i) St<TO>::st(hr + i, v[i]);
    }
    return;
  }
  ln4(v, D, g1v, b1v, red);
  if (g2) ln4(v, D, g2v, b2v, red);
  TO* hr = h + (int64_t)m * ldh + e;
#pragma unroll
  for (int i = 0; i < 4; ++i) St<TO>::st(hr + i, v[i]);
}

template <typename TO>
__global__ __launch_bounds__(kT) void residual_reduce_ln_kernel(float* __restrict__ x, int64_t ldx,
                                                                const float* __restrict__ part, int nsplit,
                                                                int64_t split_stride, int64_t ldp,
                                                                const float* __restrict__ bias, TO* __restrict__ h,
                                                                int64_t ldh, int D, const float* g1, const float* b1,
                                                                const float* g2, const float* b2) {
  __shared__ float red[kT / 64];
  const int m = blockIdx.x;
  float* xr = x + (int64_t)m * ldx;
  float v[kMaxPer];
  const int n = (D - threadIdx.x + kT - 1) / kT;
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i) {
    if (i < n) {
      const int e = threadIdx.x + kT * i;
      float acc = bias ? bias[e] : 0.f;
      for (int s = 0; s < nsplit; ++s) acc += part[s * split_stride + (int64_t)m * ldp + e];
      v[i] = xr[e] + acc;
      xr[e] = v[i];
    }
  }
  if (g1 || h) {
    if (g1) ln_inplace(v, n, D, g1, b1, red);
    if (g1 && g2) ln_inplace(v, n, D, g2, b2, red);
    TO* hr = h + (int64_t)m * ldh;
#pragma unroll
    for (int i = 0; i < kMaxPer; ++i)
      if (i < n) St<TO>::st(hr + threadIdx.x + kT * i, v[i]);
  }
}
}  // namespace

extern "C" int itts_layernorm_rows(const float* x, int64_t ldx, const int32_t* row_idx, void* y, int64_t ldy, int M,
                                   int D, const float* g1, const float* b1, const float* g2, const float* b2,
                                   int out_dtype, void* stream) {
  const char* fn = "itts_layernorm_rows";
  ITTS_REQUIRE(M >= 0 && D > 0 && D <= kT * kMaxPer, fn, "D must be in [1, 4096]");
  if (M == 0) return 0;
  ITTS_REQUIRE(x && y && g1 && b1 && (!g2 || b2), fn, "null pointer");
  hipStream_t s = itts::as_stream(stream);
  if (out_dtype == ITTS_BF16)
    hipLaunchKernelGGL(ln_rows_kernel<uint16_t>, dim3(M), dim3(kT), 0, s, x, ldx, row_idx, (uint16_t*)y, ldy, D, g1,
                       b1, g2, b2);
  else
    hipLaunchKernelGGL(ln_rows_kernel<float>, dim3(M), dim3(kT), 0, s, x, ldx, row_idx, (float*)y, ldy, D, g1, b1, g2,
                       b2);
  return itts::check_launch(fn);
}

extern "C" int itts_residual_reduce_ln(float* x, int64_t ldx, const float* part, int nsplit, int64_t split_stride,
                                       int64_t ldp, const float* bias, void* h, int64_t ldh, int M, int D,
                                       const float* g1, const float* b1, const float* g2, const float* b2,
                                       int out_dtype, void* stream) {
  const char* fn = "itts_residual_reduce_ln";
  ITTS_REQUIRE(M >= 0 && D > 0 && D <= kT * kMaxPer && nsplit >= 0, fn, "bad sizes");
  if (M == 0) return 0;
  ITTS_REQUIRE(x && (nsplit == 0 || part) && (!g1 || (b1 && h)), fn, "null pointer");
  hipStream_t s = itts::as_stream(stream);
  const bool v4 = D % 256 == 0 && D <= 4096 && nsplit <= kMaxSplit && ldx % 4 == 0 && ldp % 4 == 0 &&
                  split_stride % 4 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(part)) & 15) == 0;
  if (v4) {
    // no LayerNorm: 64-thread column blocks of 256 elements, M x D/256 workgroups (32 rows: 128 instead of
    // 32 workgroups of one row each -- the partial rows stream from 4x the CUs); ITTS_REDUCE_COLS=0: one
    // workgroup per row (A/B)
    static const bool cols = [] {
      const char* e = getenv("ITTS_REDUCE_COLS");
      return !(e && e[0] == '0');
    }();
    const bool split = !g1 && cols;
    const dim3 grid(M, split ? D / 256 : 1), block(split ? 64 : D / 4);
    if (out_dtype == ITTS_BF16)
      hipLaunchKernelGGL(residual_reduce_ln_v4_kernel<uint16_t>, grid, block, 0, s, x, ldx, part, nsplit,
                         split_stride, ldp, bias, (uint16_t*)h, ldh, D, g1, b1, g2, b2);
    else
      hipLaunchKernelGGL(residual_reduce_ln_v4_kernel<float>, grid, block, 0, s, x, ldx, part, nsplit,
                         split_stride, ldp, bias, (float*)h, ldh, D, g1, b1, g2, b2);
    return itts::check_launch(fn);
  }
  if (out_dtype == ITTS_BF16)
    hipLaunchKernelGGL(residual_reduce_ln_kernel<uint16_t>, dim3(M), dim3(kT), 0, s, x, ldx, part, nsplit,
                       split_stride, ldp, bias, (uint16_t*)h, ldh, D, g1, b1, g2, b2);
  else
    hipLaunchKernelGGL(residual_reduce_ln_kernel<float>, dim3(M), dim3(kT), 0, s, x, ldx, part, nsplit, split_stride,
                       ldp, bias, (float*)h, ldh, D, g1, b1, g2, b2);
  return itts::check_launch(fn);
}
