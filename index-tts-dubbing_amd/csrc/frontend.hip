// Prompt front-end on the GPU: log-mel spectrogram of the prompt audio, fused per frame.
// Replaces torchaudio.transforms.MelSpectrogram + safe_log as the reference builds them
// (indextts/utils/feature_extractors.py:24-50 MelSpectrogramFeatures, indextts/infer.py:509-514):
//   frames: center padding by n_fft/2 with reflect, hop `hop`, periodic Hann window (caller's);
//   |STFT| (power 1, onesided) -> @ mel filterbank [n_freqs][n_mels] (HTK, no norm, caller's)
//   -> log(clamp(., 1e-7)).
// One workgroup per (frame, utterance): the windowed frame and a cos/sin table of the n_fft roots
// of unity (sincospi, accurate f32) sit in LDS; each thread computes whole DFT bins by direct
// summation (n_fft = 1024: 1 M MACs per frame -- microseconds for a prompt), then the mel
// projection and the log.  Per-prompt and cached by the caller: not on the throughput path.
#include "common.h"

namespace {
constexpr int kT = 256;
constexpr int kMaxFft = 2048;

__global__ __launch_bounds__(kT) void log_mel_kernel(const float* __restrict__ audio, int64_t lda, int L,
                                                     const float* __restrict__ window, const float* __restrict__ fb,
                                                     int n_fft, int hop, int n_mels, int n_frames,
                                                     float* __restrict__ out) {
  extern __shared__ float sm[];
  float* xs = sm;                 // [n_fft] windowed frame
  float* cs = xs + n_fft;         // [n_fft] cos(2 pi j / n_fft)
  float* sn = cs + n_fft;         // [n_fft] sin(2 pi j / n_fft)
  float* mag = sn + n_fft;        // [n_fft / 2 + 1]
  const int f = blockIdx.x, b = blockIdx.y;
  const float* x = audio + (int64_t)b * lda;
  const int half = n_fft / 2, nfreq = half + 1;
  const int start = f * hop - half;
  for (int n = threadIdx.x; n < n_fft; n += kT) {
    int t = start + n;  // reflect padding (no edge repeat), as torch.stft(center=True, pad_mode="reflect")
    if (t < 0) t = -t;
    if (t >= L) t = 2 * (L - 1) - t;
    xs[n] = x[t] * window[n];
    float s, c;
    sincospif(2.0f * (float)n / (float)n_fft, &s, &c);
    cs[n] = c;
    sn[n] = s;
  }
  __syncthreads();
  const int mask = n_fft - 1;  // n_fft is a power of two
  for (int k = threadIdx.x; k < nfreq; k += kT) {
    float re = 0.f, im = 0.f;
    int idx = 0;
    for (int n = 0; n < n_fft; ++n) {
      const float v = xs[n];
      re = fmaf(v, cs[idx], re);
      im = fmaf(v, sn[idx], im);
      idx = (idx + k) & mask;
    }
    mag[k] = sqrtf(re * re + im * im);
  }
  __syncthreads();
  for (int m = threadIdx.x; m < n_mels; m += kT) {
    float acc = 0.f;
    for (int k = 0; k < nfreq; ++k) acc = fmaf(mag[k], fb[(int64_t)k * n_mels + m], acc);
    out[((int64_t)b * n_mels + m) * n_frames + f] = logf(fmaxf(acc, 1e-7f));
  }
}
}  // namespace

extern "C" int itts_log_mel(const float* audio, int64_t ld_audio, int B, int L, const float* window,
                            const float* mel_fb, int n_fft, int hop, int n_mels, float* out, void* stream) {
  const char* fn = "itts_log_mel";
  ITTS_REQUIRE(B >= 0 && L > 0 && hop > 0 && n_mels > 0, fn, "bad sizes");
  ITTS_REQUIRE(n_fft >= 16 && n_fft <= kMaxFft && (n_fft & (n_fft - 1)) == 0, fn, "n_fft must be a power of two <= 2048");
  ITTS_REQUIRE(L > n_fft / 2, fn, "reflect padding needs more than n_fft/2 samples");
  if (B == 0) return 0;
  ITTS_REQUIRE(audio && window && mel_fb && out, fn, "null pointer");
  const int n_frames = L / hop + 1;  // center=True
  const size_t lds = sizeof(float) * (3 * (size_t)n_fft + n_fft / 2 + 1);
  hipLaunchKernelGGL(log_mel_kernel, dim3(n_frames, B), dim3(kT), lds, itts::as_stream(stream), audio, ld_audio, L,
                     window, mel_fb, n_fft, hop, n_mels, n_frames, out);
  return itts::check_launch(fn);
}

// ---- band-limited resampling (torchaudio.functional.resample, sinc_interp_hann) -------------------
// Reference: infer.py:509-514 (torchaudio.transforms.Resample(sr, 24000) of the prompt).  With the
// rates reduced by their gcd to orig : new, output i = new * f + p (frame f, phase p) is
//   y[i] = sum_{k < K} xpad[orig * f + k] * kern[p][k],   xpad[j] = x[j - width] (zero outside [0, L)),
// K = 2 * width + orig; kern is the windowed-sinc table built on the host (utils/audio.py
// sinc_resample_kernel, float64 -> f32).  One thread per output sample, taps in k order (fixed
// rounding); the table rows are L1/L2-resident (a few KB to ~100 KB).
namespace {
__global__ __launch_bounds__(256) void resample_kernel(const float* __restrict__ x, int64_t ldx, int L,
                                                       const float* __restrict__ kern, int orig, int nw, int width,
                                                       float* __restrict__ y, int64_t ldy, int Lout) {
  const int i = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (i >= Lout) return;
  const int K = 2 * width + orig;
  const int f = i / nw, ph = i - f * nw;
  const float* xr = x + (int64_t)b * ldx;
  const float* kr = kern + (int64_t)ph * K;
  const int j0 = orig * f - width;  // x index of tap 0
  float acc = 0.f;
  if (j0 >= 0 && j0 + K <= L) {
    for (int k = 0; k < K; ++k) acc = fmaf(xr[j0 + k], kr[k], acc);
  } else {
    for (int k = 0; k < K; ++k) {
      const int j = j0 + k;
      if (j >= 0 && j < L) acc = fmaf(xr[j], kr[k], acc);
    }
  }
  y[(int64_t)b * ldy + i] = acc;
}
}  // namespace

extern "C" int itts_resample_sinc(const float* x, int64_t ldx, int B, int L, const float* kern, int orig, int new_rate,
                                  int width, float* y, int64_t ldy, int Lout, void* stream) {
  const char* fn = "itts_resample_sinc";
  ITTS_REQUIRE(B >= 0 && L >= 0 && Lout >= 0 && orig > 0 && new_rate > 0 && width >= 0, fn, "bad sizes");
  if (B == 0 || Lout == 0) return 0;
  ITTS_REQUIRE(x && kern && y, fn, "null pointer");
  ITTS_REQUIRE((int64_t)(Lout - 1) / new_rate * orig + 2 * width + orig < (int64_t)1 << 31, fn, "too long");
  hipLaunchKernelGGL(resample_kernel, dim3((Lout + 255) / 256, B), dim3(256), 0, itts::as_stream(stream), x, ldx, L,
                     kern, orig, new_rate, width, y, ldy, Lout);
  return itts::check_launch(fn);
}
