// GPT-2 projection GEMMs for the decode step and the f32 verification mode.
//
// HF GPT-2 Conv1D is y = x @ W + b with W [in, out] (HF:pytorch_utils.py:119); the mel head is
// nn.Linear (gpt/model.py:379).  Two kernels:
//
// 1. itts_skinny_gemm_bf16 -- decode step, M = batch (<= 128 rows, MT 32-row tiles), weight-streaming:
//    Wsk is prepacked in MFMA-fragment order [N/32][K/16][64 lanes][8] bf16, so each wave load of
//    one k-step is ONE contiguous 1 KiB dwordx4 read (perfect coalescing, every weight byte read
//    once per step).  A workgroup (8 waves) owns a 32-column tile; its waves take interleaved
//    k-steps (v_mfma_f32_32x32x16_bf16), reduce through LDS in a fixed order (deterministic,
//    batch-invariant per row), then either apply the epilogue (bias, gelu_tanh, f32|bf16 store) or
//    write an f32 split-K partial (grid.y = K splits) for itts_residual_reduce_ln.
// 2. itts_gemm_f32 -- exact-f32 VALU GEMM (fmaf chain in k order) used by the f32 verification
//    mode for prefill, decode and the latent pass.  Same epilogue plus an f32 residual (may alias Y).
#include "common.h"

namespace {

__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
}

constexpr int kSkWaves = 8;

template <int MT, typename OutT>
__global__ __launch_bounds__(64 * kSkWaves) void skinny_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                               const u32x4_t* __restrict__ Wsk, int K, int N, int M,
                                                               const float* __restrict__ bias, int gelu,
                                                               OutT* __restrict__ Y, int64_t ldy,
                                                               float* __restrict__ part, int64_t ldp) {
  __shared__ float red[kSkWaves][MT][16][64];
  const int nt = blockIdx.x, ks = blockIdx.y, nsplit = gridDim.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ksteps = K / 16, kper = ksteps / nsplit, kbeg = ks * kper;
  const u32x4_t* Wt = Wsk + ((int64_t)nt * ksteps) * 64 + lane;
  const int r32 = lane & 31, h = lane >> 5;
  f32x16_t acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
#pragma unroll 4
  for (int s = kbeg + w; s < kbeg + kper; s += kSkWaves) {
    const u32x4_t bw = Wt[(int64_t)s * 64];
    bf16x8_t bfrag = *reinterpret_cast<const bf16x8_t*>(&bw);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(A + (int64_t)(32 * m + r32) * lda + 16 * s + 8 * h);
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bfrag, acc[m], 0, 0, 0);
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w][m][r][lane] = acc[m][r];
  __syncthreads();
  for (int o = threadIdx.x; o < MT * 16 * 64; o += 64 * kSkWaves) {
    const int m = o / 1024, r = (o / 64) % 16, l = o % 64;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < kSkWaves; ++ww) v += red[ww][m][r][l];
    const int row = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    const int n = nt * 32 + (l & 31);
    if (row >= M || n >= N) continue;
    if (part) {
      part[(int64_t)ks * M * ldp + (int64_t)row * ldp + n] = v;
    } else {
      if (bias) v += bias[n];
      if (gelu) v = gelu_tanh_f(v);
      St<OutT>::st(Y + (int64_t)row * ldy + n, v);
    }
  }
}

// ---- exact f32 GEMM: C[m][n] = sum_k A[m][k] * W[n][k] ----
constexpr int kFT = 64, kFK = 16;
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, int64_t lda,
                                                       const float* __restrict__ W, int64_t ldw, int M, int N, int K,
                                                       const float* __restrict__ bias, int gelu,
                                                       const float* r1, float* Y, int64_t ldy) {
  __shared__ float As[kFK][kFT + 1], Ws[kFK][kFT + 1];
  const int m0 = blockIdx.y * kFT, n0 = blockIdx.x * kFT;
  const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += kFK) {
    for (int i = threadIdx.x; i < kFT * kFK; i += 256) {
      const int r = i / kFK, c = i % kFK;
      const int m = m0 + r, n = n0 + r, k = k0 + c;
      As[c][r] = (m < M && k < K) ? A[(int64_t)m * lda + k] : 0.f;
      Ws[c][r] = (n < N && k < K) ? W[(int64_t)n * ldw + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kFK; ++c) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = As[c][ty * 4 + i];
        b[i] = Ws[c][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= N) continue;
      float v = acc[i][j] + (bias ? bias[n] : 0.f);
      if (gelu) v = gelu_tanh_f(v);
      const int64_t off = (int64_t)m * ldy + n;
      if (r1) v += r1[off];
      Y[off] = v;
    }
  }
}

}  // namespace

extern "C" int itts_skinny_gemm_bf16(const void* A, int64_t lda, const void* Wsk, int K, int N, int M,
                                     const float* bias, int gelu, void* Y, int64_t ldy, int out_dtype, float* part,
                                     int64_t ldp, int ksplit, void* stream) {
  const char* fn = "itts_skinny_gemm_bf16";
  ITTS_REQUIRE(M > 0 && M <= 128 && K % 16 == 0 && N > 0, fn, "need 0 < M <= 128 and K % 16 == 0");
  ITTS_REQUIRE(ksplit >= 1 && (K / 16) % ksplit == 0, fn, "K/16 must divide by ksplit");
  ITTS_REQUIRE(A && Wsk && (part || Y), fn, "null pointer");
  ITTS_REQUIRE(part || ksplit == 1, fn, "ksplit > 1 needs a partial buffer");
  dim3 grid((N + 31) / 32, ksplit);
  dim3 block(64 * kSkWaves);
  hipStream_t s = itts::as_stream(stream);
  const int MT = (M + 31) / 32;
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const u32x4_t* w = static_cast<const u32x4_t*>(Wsk);
#define ITTS_SK(MTV, OT)                                                                                     \
  hipLaunchKernelGGL((skinny_kernel<MTV, OT>), grid, block, 0, s, a, lda, w, K, N, M, bias, gelu,           \
                     static_cast<OT*>(Y), ldy, part, ldp)
  if (out_dtype == ITTS_BF16) {
    if (MT == 1) ITTS_SK(1, uint16_t); else if (MT == 2) ITTS_SK(2, uint16_t); else ITTS_SK(4, uint16_t);
  } else {
    if (MT == 1) ITTS_SK(1, float); else if (MT == 2) ITTS_SK(2, float); else ITTS_SK(4, float);
  }
#undef ITTS_SK
  return itts::check_launch(fn);
}

extern "C" int itts_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw, int M, int N, int K,
                             const float* bias, int gelu, const float* r1, float* Y, int64_t ldy, void* stream) {
  const char* fn = "itts_gemm_f32";
  ITTS_REQUIRE(M >= 0 && N > 0 && K > 0, fn, "bad sizes");
  if (M == 0) return 0;
  ITTS_REQUIRE(A && W && Y, fn, "null pointer");
  dim3 grid((N + kFT - 1) / kFT, (M + kFT - 1) / kFT);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, itts::as_stream(stream), A, lda, W, ldw, M, N, K, bias, gelu,
                     r1, Y, ldy);
  return itts::check_launch(fn);
}
