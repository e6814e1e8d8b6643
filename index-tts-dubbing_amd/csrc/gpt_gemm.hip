// Exact-f32 GEMM for the GPT verification mode (f32 weights / activations):
//   Y[m][n] = act(sum_k A[m][k] * W[n][k] + bias[n]) (+ r1[m][n])
// HF GPT-2 Conv1D is y = x @ W + b with W [in, out] (HF:pytorch_utils.py:119); W is passed here
// transposed ([out, in]).  Each output is one fmaf chain in k order (LDS-tiled 64x64, 4x4 per thread),
// so the f32 mode reproduces the fp32 reference to rounding and gives bit-exact greedy ids.
// The bf16 product path uses igemm.hip (sequences) and gpt_decode.hip (decode step) instead.
#include "common.h"

namespace {

__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
}

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
