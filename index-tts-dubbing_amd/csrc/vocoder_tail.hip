// BigVGAN tail: conv_post (Conv1d(C -> 1, k7, zero pad 3)) + tanh, fused with the host-side int16
// conversion of infer() (clamp(32767*wav, +-32767) then a truncating cast, quirk Q8).
//   BigVGAN/models.py:192,246-248 ; infer.py:627-631,658
// Channel-last input [B][Tmax][C] (bf16 or f32). One thread per output sample; the [256+6][C] input
// window of a workgroup is staged once through LDS as f32.
//
// itts_act_conv_post_tanh (round 6): activation_post (Activation1d, models.py:245) fused in front -- the
// vocoder's last AMP stage output is read once and the 24-channel activation output (629 MB per C3 batch)
// never goes to HBM.  Bit-identical to itts_aa_snakebeta_fwd (bf16, MFMA path) + itts_conv_post_tanh: the
// activation strips start at multiples of 32 samples as the activation kernel's do (the MFMA sums depend on
// the strip alignment), edge outputs use the same exact formula, the rounded bf16 activation values feed the
// same conv loop in the same order.
#include "act_mfma.h"
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

// ---- activation_post + conv_post + tanh (+ int16) ----
constexpr int kApTiles = 16;               // activation output tiles per job: 4 waves x 4
constexpr int kApTO = 32 * kApTiles - 64;  // conv outputs per job: 448; activation rows [t0 - 32, t0 + 480)
constexpr int kApWin = 32 * kApTiles + 32; // window rows: times t0 - 39 .. t0 + 504 (replicate-clamped)
constexpr int kApPX = 64;                  // window row bytes: one 32-channel block (C <= 32)
constexpr int kApKMax = 15;                // conv taps (odd, halo K / 2 <= 7 < 32)
constexpr int kApLds = kApWin * kApPX + 128 + 32 * kApKMax * 4 + 32 * kApTiles * 32 * 2 + 32 * kApKMax * 4;

struct ApArgs {
  const uint16_t* x;
  int64_t sxb, ldx;
  const float *up, *down, *log_alpha, *log_beta;
  const float* w;  // conv_post [C][K]
  float bias;
  int C, K;
  const int32_t* lens;
  int T;
  float* wav;
  int16_t* pcm;
  int64_t syb;
};

// CK = (C << 8) | K for a compile-time conv_post shape, 0 for the generic loop
template <int CK>
__global__ __launch_bounds__(256, 2) void act_post_conv_kernel(ApArgs p) {
  constexpr int PX = kApPX;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* win = smem;                                            // [kApWin][64] bf16 window
  float* tl = reinterpret_cast<float*>(smem + kApWin * PX);             // 12 up, 12 down taps
  float* wl = tl + 32;                                                  // conv_post [C][K]
  uint16_t* at = reinterpret_cast<uint16_t*>(wl + 32 * kApKMax);        // activation rows [512][C] bf16
  float* wt = reinterpret_cast<float*>(at + 32 * kApTiles * 32);        // conv_post tap-major [K][C] (CK > 0)
  const int b = blockIdx.y;
  const int len = p.lens ? p.lens[b] : p.T;
  const int t0 = blockIdx.x * kApTO;
  if (t0 >= len) return;
  const int ta0 = t0 - 32;  // time of activation row 0 (a multiple of 32, like the activation kernel's strips)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = p.C, K = p.K;
  if (tid < 24) tl[tid] = tid < 12 ? p.up[tid] : p.down[tid - 12];
  for (int i = tid; i < C * K; i += 256) wl[i] = p.w[i];
  if constexpr (CK > 0)
    for (int i = tid; i < C * K; i += 256) wt[(i % K) * C + i / K] = p.w[i];
  // window row r = time ta0 - 7 + r (clamped to [0, len)), channels >= C zero: the activation kernel's window
  const uint16_t* X = p.x + (int64_t)b * p.sxb;
  constexpr int NV = (kApWin * 4 + 255) / 256;
  u32x4_t buf[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = tid + 256 * i;
    const int r = v >> 2, c = (v & 3) * 8;
    const int t = min(max(ta0 - 7 + r, 0), len - 1);
    buf[i] = (v < kApWin * 4 && c < C) ? ld_stream(reinterpret_cast<const u32x4_t*>(X + (int64_t)t * p.ldx + c))
                                       : u32x4_t{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = tid + 256 * i;
    if (v < kApWin * 4) *reinterpret_cast<u32x4_t*>(win + itts_actm::woff<PX>(v >> 2, (v & 3) * 8)) = buf[i];
  }
  __syncthreads();
  // activation strips (act.hip aa_snake_mfma_kernel, NB = 1): wave w -> rows [128 w, 128 w + 128)
  {
    itts_actm::Taps T;
    itts_actm::make_taps(tl, T);
    const int ch = lane & 31, h = lane >> 5;
    const float a_rev = ch < C ? expf(p.log_alpha[ch]) * 0.15915494309189535f : 0.f;
    const float inv_b = ch < C ? 1.0f / (expf(p.log_beta[ch]) + 1e-9f) : 0.f;
    const int ts = ta0 + wave * 128;
    const int ntile = min(4, max(0, (len - ts + 31) / 32));
    itts_actm::strip<PX>(win, wave * 128, 0, ntile, T, a_rev, inv_b, [&](int i, const f32x16_t& acc) {
      const int t = ts + 32 * i + (lane & 31);
      if (t < 3 || t >= len - 3) return;  // edges (and rows outside [0, len)): below
      uint16_t* ar = at + (t - ta0) * C + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (8 * g + 4 * h < C) {
          const u32x2_t o{pack2bf(acc[4 * g], acc[4 * g + 1]), pack2bf(acc[4 * g + 2], acc[4 * g + 3])};
          *reinterpret_cast<u32x2_t*>(ar + 8 * g) = o;
        }
      }
    });
  }
  // rows within 3 samples of an utterance edge: the exact formula; rows outside [0, len): the conv's zeros
  if (ta0 < 3 || ta0 + 32 * kApTiles > len - 3) {
    for (int it = tid; it < 32 * kApTiles * C; it += 256) {
      const int r = it / C, cc = it - r * C;
      const int t = ta0 + r;
      if (t >= 3 && t < len - 3) continue;
      float v = 0.f;
      if (t >= 0 && t < len) {
        const float a = expf(p.log_alpha[cc]) * 0.15915494309189535f;
        const float ib = 1.0f / (expf(p.log_beta[cc]) + 1e-9f);
        v = itts_actm::exact_at<PX>(win, ta0 - 7, t, len, cc, tl, a, ib);
      }
      at[r * C + cc] = f2bf(v);
    }
  }
  __syncthreads();
  // conv_post + tanh (+ int16): conv_post_tanh_kernel's loop order over the bf16 activation rows
  const int half = K / 2;
  if constexpr (CK > 0) {
    // compile-time C x K (BigVGAN2's conv_post: 24 x 7): tap j's C weights read once as 16-B vectors from a
    // tap-major copy (wt) for both of the thread's outputs -- each output's fma chain (bias, then tap-major,
    // channel inner) is the generic loop's below, which reads every weight with its own LDS load inside the
    // chain: latency-bound, ~600 us of the 980 us launch at the C3 shape (bench_r06s_c3.json roofline_vocoder_tail).
    constexpr int CC = CK >> 8, KK = CK & 255, HALF = KK / 2;
    static_assert(CC % 8 == 0 && CC <= 32 && KK <= kApKMax, "conv_post shape");
    float acc[2] = {p.bias, p.bias};
    int ro[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = tid + 256 * q;
      ro[q] = (o < kApTO ? o : 0) + 32 - HALF;  // activation row of tap 0 (t - half - ta0); clamped when idle
    }
#pragma unroll 1  // one tap's weights and rows live at a time (unrolled, the loads of every tap were hoisted: spills)
    for (int j = 0; j < KK; ++j) {
      float wj[CC];
#pragma unroll
      for (int c4 = 0; c4 < CC; c4 += 4) {
        const f32x4_t w4 = *reinterpret_cast<const f32x4_t*>(wt + j * CC + c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) wj[c4 + e] = w4[e];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint16_t* row = at + (ro[q] + j) * CC;
#pragma unroll
        for (int c8 = 0; c8 < CC; c8 += 8) {
          const u32x4_t v = *reinterpret_cast<const u32x4_t*>(row + c8);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t wv = v[e >> 1];
            acc[q] = fmaf(wj[c8 + e], __uint_as_float((e & 1) ? (wv & 0xFFFF0000u) : (wv << 16)), acc[q]);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = tid + 256 * q, t = t0 + o;
      if (o >= kApTO || t >= len) continue;
      const float v = tanhf(acc[q]);
      if (p.wav) p.wav[(int64_t)b * p.syb + t] = v;
      if (p.pcm) {
        const float s = fminf(fmaxf(32767.0f * v, -32767.0f), 32767.0f);
        p.pcm[(int64_t)b * p.syb + t] = (int16_t)s;
      }
    }
    return;
  }
  for (int o = tid; o < kApTO; o += 256) {
    const int t = t0 + o;
    if (t >= len) break;
    float acc = p.bias;
    for (int j = 0; j < K; ++j) {
      const uint16_t* row = at + (t - half + j - ta0) * C;
      for (int c8 = 0; c8 < C; c8 += 8) {
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(row + c8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t wv = v[e >> 1];
          const float xv = __uint_as_float((e & 1) ? (wv & 0xFFFF0000u) : (wv << 16));
          acc = fmaf(wl[(c8 + e) * K + j], xv, acc);
        }
      }
    }
    const float v = tanhf(acc);
    if (p.wav) p.wav[(int64_t)b * p.syb + t] = v;
    if (p.pcm) {
      const float s = fminf(fmaxf(32767.0f * v, -32767.0f), 32767.0f);
      p.pcm[(int64_t)b * p.syb + t] = (int16_t)s;
    }
  }
}
}  // namespace

extern "C" int itts_act_conv_post_tanh(const void* x, int64_t x_sb, int64_t ldx, const float* up12, const float* down12,
                                       const float* log_alpha, const float* log_beta, const float* w, float bias, int C,
                                       int K, const int32_t* lengths, int B, int Tmax, float* wav, int16_t* pcm,
                                       int64_t y_sb, void* stream) {
  const char* fn = "itts_act_conv_post_tanh";
  ITTS_REQUIRE(B >= 0 && Tmax >= 0 && C > 0 && K > 0, fn, "bad sizes");
  if (B == 0 || Tmax == 0) return 0;
  ITTS_REQUIRE(x && up12 && down12 && log_alpha && log_beta && w && (wav || pcm), fn, "null pointer");
  ITTS_REQUIRE(C % 8 == 0 && C <= 32, fn, "C must be a multiple of 8, at most 32 (one MFMA channel block)");
  ITTS_REQUIRE((K & 1) && K <= kApKMax, fn, "K must be odd and at most 15");
  ITTS_REQUIRE(ldx % 8 == 0 && x_sb % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0, fn,
               "channel-last bf16 rows must be 16-B aligned");
  ApArgs a{static_cast<const uint16_t*>(x), x_sb, ldx, up12, down12, log_alpha, log_beta, w, bias, C, K, lengths, Tmax,
           wav, pcm, y_sb};
  dim3 grid((Tmax + kApTO - 1) / kApTO, B);
  if (C == 24 && K == 7)
    hipLaunchKernelGGL(act_post_conv_kernel<(24 << 8) | 7>, grid, dim3(256), kApLds, itts::as_stream(stream), a);
  else
    hipLaunchKernelGGL(act_post_conv_kernel<0>, grid, dim3(256), kApLds, itts::as_stream(stream), a);
  return itts::check_launch(fn);
}


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
