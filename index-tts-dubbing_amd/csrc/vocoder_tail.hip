// BigVGAN tail: conv_post (Conv1d(C -> 1, k7, zero pad 3)) + tanh, fused with the host-side int16
// conversion of infer() (clamp(32767*wav, +-32767) then a truncating cast, quirk Q8).
//   BigVGAN/models.py:192,246-248 ; infer.py:627-631,658
// Channel-last input [B][Tmax][C] (bf16 or f32). One thread per output sample; the [256+6][C] input
// window of a workgroup is staged once through LDS as f32.
#include "common.h"

namespace {
template <typename TI>
__global__ __launch_bounds__(256) void conv_post_tanh_kernel(const TI* __restrict__ x, int64_t sxb, int64_t ldx,
                                                             const float* __restrict__ w, float bias, int C, int K,
                                                             const int32_t* __restrict__ lens, int Tmax,
                                                             float* __restrict__ wav, int16_t* __restrict__ pcm,
                                                             int64_t syb) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int b = blockIdx.y;
  const int len = lens ? lens[b] : Tmax;
  const int t0 = blockIdx.x * 256;
  if (t0 >= len) return;
  const int half = K / 2, rows = 256 + K - 1;
  const TI* X = x + (int64_t)b * sxb;
  for (int idx = threadIdx.x; idx < rows * C; idx += 256) {
    int r = idx / C, c = idx - r * C;
    int t = t0 - half + r;
    xs[idx] = (t >= 0 && t < len) ? St<TI>::ld(X + (int64_t)t * ldx + c) : 0.f;
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= len) return;
  float acc = bias;
  for (int j = 0; j < K; ++j) {
    const float* row = xs + (threadIdx.x + j) * C;
    for (int c = 0; c < C; ++c) acc = fmaf(w[c * K + j], row[c], acc);
  }
  const float v = tanhf(acc);
  if (wav) wav[(int64_t)b * syb + t] = v;
  if (pcm) {
    float s = fminf(fmaxf(32767.0f * v, -32767.0f), 32767.0f);
    pcm[(int64_t)b * syb + t] = (int16_t)s;  // C cast truncates toward zero, like torch .type(int16)
  }
}
}  // namespace

// w: f32 [C][K] (conv_post weight [1, C, K] squeezed), bias: scalar.
extern "C" int itts_conv_post_tanh(const void* x, int64_t x_sb, int64_t ldx, const float* w, float bias, int C, int K,
                                   const int32_t* lengths, int B, int Tmax, float* wav, int16_t* pcm, int64_t y_sb,
                                   int dtype_in, void* stream) {
  const char* fn = "itts_conv_post_tanh";
  ITTS_REQUIRE(B >= 0 && Tmax >= 0 && C > 0 && K > 0 && (K & 1), fn, "bad sizes (K must be odd)");
  if (B == 0 || Tmax == 0) return 0;
  ITTS_REQUIRE(x && w && (wav || pcm), fn, "null pointer");
  ITTS_REQUIRE((256 + K - 1) * C * 4 <= 64 * 1024, fn, "C too large for the LDS window");
  dim3 grid((Tmax + 255) / 256, B);
  size_t lds = sizeof(float) * (256 + K - 1) * C;
  hipStream_t s = itts::as_stream(stream);
  if (dtype_in == ITTS_BF16)
    hipLaunchKernelGGL(conv_post_tanh_kernel<uint16_t>, grid, dim3(256), lds, s, static_cast<const uint16_t*>(x), x_sb,
                       ldx, w, bias, C, K, lengths, Tmax, wav, pcm, y_sb);
  else if (dtype_in == ITTS_F32)
    hipLaunchKernelGGL(conv_post_tanh_kernel<float>, grid, dim3(256), lds, s, static_cast<const float*>(x), x_sb, ldx,
                       w, bias, C, K, lengths, Tmax, wav, pcm, y_sb);
  else
    return itts::fail(fn, "unsupported dtype");
  return itts::check_launch(fn);
}
