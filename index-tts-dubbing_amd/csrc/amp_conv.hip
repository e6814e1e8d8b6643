// Fused anti-aliased SnakeBeta + dilated Conv1d (+ residual) for the narrow BigVGAN stages, gfx950.
//
// One AMPBlock1 layer (BigVGAN/models.py:65-74) is  x' = conv2(act2(conv1(act1(x)))) + x  and the
// block outputs are averaged (models.py:237-243).  At C <= 96 (stages 3-5: 96 / 48 / 24 channels at
// 256 / 512 / 1024 samples per latent frame) these layers move most of the vocoder's bytes and do
// little arithmetic (24*24*k MACs per sample), so they are HBM-bound: this kernel reads the
// pre-activation input once, applies Activation1d (up2 -> SnakeBeta -> down2, torch-path edge
// semantics, see act.hip) while staging the time window in LDS, runs every tap of the conv on MFMA
// out of LDS, and writes the output tile (+ bias, + r1 + r2, * alpha) with 16-B coalesced stores:
//   y[b, t, :] = alpha * ( sum_j W_j . act(x)[b, t + off_j, :] + bias + r1[b, t, :] + r2[b, t, :] )
// with act(x) rows outside [0, len_b) reading as zero (the conv's zero padding) and act's own
// replicate padding at len_b (ragged batches exact).  Without `act` the raw input is convolved.
//
// Tile: TT (256 at C=24, 128 otherwise) output rows x all Cout columns per 256-thread workgroup
// (4 waves, each 32-row MFMA tiles x every N tile).  LDS: raw input window (bf16, TT + taps span +
// 12 rows), activated window (bf16, padded pitch for conflict-free ds_read_b128 MFMA fragments);
// a 2-slot tap-weight ring overlays the raw window, and the f32 output tile overlays everything
// after the MFMAs.  Activation work item = 16 rows of one channel with the up-sampled values in
// registers (42 snake evaluations per 16 outputs).  Weights: the igemm packing [tap][co_pad][ci_pad]
// (ci_pad, co_pad multiples of 32), staged tap by tap through the LDS ring by the whole workgroup.
#include "act_mfma.h"
#include "common.h"

namespace {

constexpr int kMaxTapsAc = 16;
// output rows per workgroup by padded channel count (tuning: -DITTS_AMP_TT32=... etc.)
#ifndef ITTS_AMP_TT32
#define ITTS_AMP_TT32 256
#endif
#ifndef ITTS_AMP_TT64
#define ITTS_AMP_TT64 256
#endif
#ifndef ITTS_AMP_TT96
#define ITTS_AMP_TT96 128
#endif
#ifndef ITTS_AMP_K48  // K extent of the C = 48 instantiation (48: no all-zero K chunk)
#define ITTS_AMP_K48 48
#endif
#ifndef ITTS_AMP_TTC32  // conv-only (activation in its own kernel)
#define ITTS_AMP_TTC32 ITTS_AMP_TT32
#endif
#ifndef ITTS_AMP_TTC64
#define ITTS_AMP_TTC64 ITTS_AMP_TT64
#endif
#ifndef ITTS_AMP_TTC96
#define ITTS_AMP_TTC96 ITTS_AMP_TT96
#endif
constexpr int kSpan = 64;  // max (max_off - min_off) of the taps

struct AcArgs {
  const uint16_t* x;
  int64_t sxb, ldx;
  const float *up, *down, *log_alpha, *log_beta;  // log_alpha == nullptr: no activation
  const uint16_t* w;
  const float* bias;
  const uint16_t* r1;
  const uint16_t* r2;
  uint16_t* y;
  int64_t syb, ldy;
  const int32_t* lens;
  int B, Tmax, Cin, Cout, ntaps, hl, hr;
  float alpha;
  int tap_off[kMaxTapsAc];
};

// a_rev = exp(alpha) / (2 pi): v_sin_f32 takes revolutions (see act.hip)
__device__ __forceinline__ float snake_f(float u, float a_rev, float inv_b) {
  const float s = __builtin_amdgcn_sinf(u * a_rev);
  return fmaf(inv_b, s * s, u);
}

__device__ __forceinline__ float ld_bf(const uint16_t* p) { return __uint_as_float(((uint32_t)*p) << 16); }

// CK: the channel count (Cin == Cout) as a compile-time constant for the BigVGAN stages, 0 = runtime
// CIN_PAD: the K extent staged and multiplied (a multiple of 16 >= Cin); the packed weights' rows
// are WS = CIN_PAD rounded up to 32 wide (the igemm packing)
template <int CIN_PAD, int COUT_PAD, int TT, bool ACT, int CK>
__device__ __forceinline__ void amp_conv_body(const AcArgs& p) {
  constexpr int WS = (CIN_PAD + 31) / 32 * 32;
  constexpr int PA = CIN_PAD * 2 + 16;  // activated-window row pitch (bytes)
  constexpr int FN = COUT_PAD / 32, KS = CIN_PAD / 16, FM = TT / 128;
  constexpr int SR = 16;                // activation rows per work item
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.z;
  const int len = p.lens ? p.lens[b] : p.Tmax;
  const int q0 = blockIdx.x * TT;  // first output (= conv) row of the tile
  if (q0 >= len) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Cin = CK ? CK : p.Cin, Cout = CK ? CK : p.Cout;
  const int WR = TT + p.hl + p.hr;  // activated window rows: t = q0 - hl + r
  constexpr bool act = ACT;  // compile-time: the no-activation variant keeps its registers for the conv
  const uint16_t* X = p.x + (int64_t)b * p.sxb;
  unsigned char* Aw = smem;                         // [WR][PA]
  unsigned char* Xr = smem + (TT + kSpan) * PA;     // raw window, then the tap-weight ring

  // ---- 1. raw window -> LDS (16-B vectors); padding channels of the window zeroed ----
  const int cv8 = Cin / 8;
  if (CIN_PAD > Cin) {
    const int pv = (CIN_PAD - Cin) / 8;
    for (int v = tid; v < WR * pv; v += 256) {
      const int r = v / pv, c = Cin + (v - r * pv) * 8;
      *reinterpret_cast<u32x4_t*>(Aw + r * PA + c * 2) = u32x4_t{0u, 0u, 0u, 0u};
    }
  }
  // every 16-B load of the window is issued before the first LDS write (one memory latency per
  // block, not one per loop trip): at most kLV vectors per thread
  constexpr int kLV = ((TT + kSpan + 12) * (CIN_PAD / 8) + 255) / 256;
  u32x4_t lv[kLV];
  if constexpr (ACT) {  // rows replicate-clamped: the activation's own padding at the utterance edges
    const int XR = WR + 12;  // t = q0 - hl - 6 + r
    uint16_t* xr = reinterpret_cast<uint16_t*>(Xr);
#pragma unroll
    for (int i = 0; i < kLV; ++i) {  // unconditional loads (clamped rows): no per-element branches,
      const int v = min(tid + 256 * i, XR * cv8 - 1);  // which make the compiler copy all of lv[]
      const int r = v / cv8, c = (v - r * cv8) * 8;
      const int t = min(max(q0 - p.hl - 6 + r, 0), len - 1);
      lv[i] = ld_stream(reinterpret_cast<const u32x4_t*>(X + (int64_t)t * p.ldx + c));
    }
#pragma unroll
    for (int i = 0; i < kLV; ++i) {
      const int v = tid + 256 * i;
      if (v < XR * cv8) {
        const int r = v / cv8, c = (v - r * cv8) * 8;
        *reinterpret_cast<u32x4_t*>(xr + r * Cin + c) = lv[i];
      }
    }
  } else {  // rows outside [0, len) are the conv's zero padding
#pragma unroll
    for (int i = 0; i < kLV; ++i) {  // clamped loads + select (see above)
      const int v = min(tid + 256 * i, WR * cv8 - 1);
      const int r = v / cv8, c = (v - r * cv8) * 8;
      const int t = q0 - p.hl + r;
      const bool ok = t >= 0 && t < len;
      const u32x4_t x = ld_stream(reinterpret_cast<const u32x4_t*>(X + (int64_t)min(max(t, 0), len - 1) * p.ldx + c));
#pragma unroll
      for (int k = 0; k < 4; ++k) lv[i][k] = ok ? x[k] : 0u;
    }
#pragma unroll
    for (int i = 0; i < kLV; ++i) {
      const int v = tid + 256 * i;
      if (v < WR * cv8) {
        const int r = v / cv8, c = (v - r * cv8) * 8;
        *reinterpret_cast<u32x4_t*>(Aw + r * PA + c * 2) = lv[i];
      }
    }
  }
  __syncthreads();

  // ---- 2. activation: work item = 16 consecutive rows of one channel (register window) ----
  if constexpr (ACT) {
    const uint16_t* xr = reinterpret_cast<const uint16_t*>(Xr);
    const int nstrip = (WR + SR - 1) / SR;
    float f[12], g[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) { f[k] = 2.0f * p.up[k]; g[k] = p.down[k]; }  // x2: up-sampler gain (exact)
    for (int item = tid; item < nstrip * Cin; item += 256) {
      const int s = item / Cin, c = item - s * Cin;
      const int r0 = s * SR;
      uint16_t* dst = reinterpret_cast<uint16_t*>(Aw) + c;  // row pitch PA/2 elements
      const float a = expf(p.log_alpha[c]) * 0.15915494309189535f;
      const float inv_b = 1.0f / (expf(p.log_beta[c]) + 1e-9f);
      const int t0 = q0 - p.hl + r0;  // time of row r0; raw rows r0 .. r0+SR+11 hold x[t0-6 ..]
      const uint16_t* col = xr + r0 * Cin + c;
      if (t0 >= 3 && t0 + SR + 3 <= len && r0 + SR <= WR) {
        float xv[SR + 12];
#pragma unroll
        for (int i = 0; i < SR + 12; ++i) xv[i] = ld_bf(col + i * Cin);
        float v[2 * SR + 10];
#pragma unroll
        for (int j = 0; j < 2 * SR + 10; ++j) {
          float acc = 0.f;
          if (j & 1) {
#pragma unroll
            for (int q = -3; q <= 2; ++q) acc = fmaf(xv[4 + (j - 1) / 2 + q], f[5 - 2 * q], acc);
          } else {
#pragma unroll
            for (int q = -2; q <= 3; ++q) acc = fmaf(xv[3 + j / 2 + q], f[6 - 2 * q], acc);
          }
          v[j] = snake_f(acc, a, inv_b);
        }
#pragma unroll
        for (int i = 0; i < SR; ++i) {
          float o = 0.f;
#pragma unroll
          for (int k = 0; k < 12; ++k) o = fmaf(g[k], v[2 * i + k], o);
          dst[(r0 + i) * (PA / 2)] = f2bf(o);
        }
      } else {
        for (int i = 0; i < SR && r0 + i < WR; ++i) {
          const int t = t0 + i;
          float o = 0.f;
          if (t >= 0 && t < len) {
#pragma unroll
            for (int k = 0; k < 12; ++k) {
              const int m = min(max(2 * t + k - 5, 0), 2 * len - 1);
              const int pp = m >> 1;
              // raw row of time tt: tt - (q0 - hl - 6); x rows are already replicate-clamped
              const uint16_t* xp = xr + (pp - (q0 - p.hl - 6)) * Cin + c;
              float ae = 0.f, ao = 0.f;
#pragma unroll
              for (int q = -3; q <= 2; ++q) ae = fmaf(ld_bf(xp + q * Cin), f[5 - 2 * q], ae);
#pragma unroll
              for (int q = -2; q <= 3; ++q) ao = fmaf(ld_bf(xp + q * Cin), f[6 - 2 * q], ao);
              o = fmaf(g[k], snake_f((m & 1) ? ao : ae, a, inv_b), o);
            }
          }
          dst[(r0 + i) * (PA / 2)] = f2bf(o);  // rows outside [0, len): the conv's zero padding
        }
      }
    }
    __syncthreads();
  }

  // residual rows of this tile: loads issued now, consumed in the epilogue (latency hidden by the MFMAs)
  constexpr int kEV = (TT * (CK ? CK : COUT_PAD) / 8 + 255) / 256;
  const int rows = min(TT, len - q0);
  const int nvec = rows * Cout / 8;
  uint16_t* Y = p.y + (int64_t)b * p.syb + (int64_t)q0 * p.ldy;
  const uint16_t* R1 = p.r1 ? p.r1 + (int64_t)b * p.syb + (int64_t)q0 * p.ldy : nullptr;
  const uint16_t* R2 = p.r2 ? p.r2 + (int64_t)b * p.syb + (int64_t)q0 * p.ldy : nullptr;
  u32x4_t rv1[kEV], rv2[kEV];
  // clamped unconditional loads (see the window loads); lanes past nvec do not store
  if (R1) {
#pragma unroll
    for (int i = 0; i < kEV; ++i) {
      const int e = min(tid + 256 * i, nvec - 1) * 8, r = e / Cout, c = e - r * Cout;
      rv1[i] = ld_stream(reinterpret_cast<const u32x4_t*>(R1 + (int64_t)r * p.ldy + c));
    }
  }
  if (R2) {
#pragma unroll
    for (int i = 0; i < kEV; ++i) {
      const int e = min(tid + 256 * i, nvec - 1) * 8, r = e / Cout, c = e - r * Cout;
      rv2[i] = ld_stream(reinterpret_cast<const u32x4_t*>(R2 + (int64_t)r * p.ldy + c));
    }
  }

  // ---- 3. MFMA over taps x K chunks; wave w owns output rows [32(w + 4i), +32), i < FM ----
  // The tap weights go through a 2-slot LDS ring filled cooperatively by the whole workgroup (each
  // weight byte crosses L2 -> CU once per block, not once per wave), next tap's loads in flight
  // while this tap's MFMAs run; B fragments are then conflict-free ds_read_b128.
  constexpr int PW = CIN_PAD * 2 + 16;                   // ring row pitch (bytes)
  constexpr int WV = COUT_PAD * CIN_PAD / 8;             // 16-B vectors per tap
  constexpr int kWV = (WV + 255) / 256;                  // per thread
  unsigned char* Wr = Xr;                                // ring overlays the (consumed) raw window
  const int r32 = lane & 31, h = lane >> 5;
  f32x16_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int n = 0; n < FN; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][n][r] = 0.f;
  u32x4_t wv[kWV];
  auto wload = [&](int j) {
    const uint16_t* Wj = p.w + (int64_t)j * COUT_PAD * WS;
#pragma unroll
    for (int i = 0; i < kWV; ++i) {
      const int v = min(tid + 256 * i, WV - 1);
      const int n = v / (CIN_PAD / 8), c = (v - n * (CIN_PAD / 8)) * 8;
      wv[i] = *reinterpret_cast<const u32x4_t*>(Wj + n * WS + c);
    }
  };
  auto wstore = [&](int slot) {
    unsigned char* dst = Wr + slot * COUT_PAD * PW;
#pragma unroll
    for (int i = 0; i < kWV; ++i) {
      const int v = tid + 256 * i;
      if (v < WV) {
        const int n = v / (CIN_PAD / 8), c = (v - n * (CIN_PAD / 8)) * 8;
        *reinterpret_cast<u32x4_t*>(dst + n * PW + c * 2) = wv[i];
      }
    }
  };
  wload(0);
  wstore(0);  // the raw window is consumed: the activation phase ended with a barrier
  __syncthreads();
  for (int j = 0; j < p.ntaps; ++j) {
    if (j + 1 < p.ntaps) wload(j + 1);
    const unsigned char* wsl = Wr + (j & 1) * COUT_PAD * PW;
    const int roff = r32 + p.tap_off[j] + p.hl;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8_t bf[FN];
#pragma unroll
      for (int n = 0; n < FN; ++n) bf[n] = *reinterpret_cast<const bf16x8_t*>(wsl + (32 * n + r32) * PW + ks * 32 + h * 16);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(Aw + (32 * (wave + 4 * i) + roff) * PA + h * 16 + ks * 32);
#pragma unroll
        for (int n = 0; n < FN; ++n)
          acc[i][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf[n], acc[i][n], 0, 0, 0);
      }
    }
    if (j + 1 < p.ntaps) wstore((j + 1) & 1);  // slot last read in tap j-1, fenced by its barrier
    __syncthreads();
  }

  // ---- 4. epilogue: acc -> LDS f32 tile [TT][Cout] (overlays the window + ring) -> bias /
  //         residuals / alpha -> 16-B stores ----
  float* Ys = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int n = 0; n < FN; ++n) {
      const int col = 32 * n + r32;
      if (col >= Cout) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        Ys[(32 * (wave + 4 * i) + (r & 3) + 8 * (r >> 2) + 4 * h) * Cout + col] = acc[i][n][r];
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kEV; ++i) {
    const int v = tid + 256 * i;
    if (v >= nvec) continue;
    const int e = v * 8, r = e / Cout, c = e - r * Cout;
    const int64_t off = (int64_t)r * p.ldy + c;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = Ys[e + k] + p.bias[c + k];
    if (R1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[2 * k] += __uint_as_float(rv1[i][k] << 16);
        o[2 * k + 1] += __uint_as_float(rv1[i][k] & 0xFFFF0000u);
      }
    }
    if (R2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[2 * k] += __uint_as_float(rv2[i][k] << 16);
        o[2 * k + 1] += __uint_as_float(rv2[i][k] & 0xFFFF0000u);
      }
    }
    u32x4_t out;
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = pack2bf(p.alpha * o[2 * k], p.alpha * o[2 * k + 1]);
    *reinterpret_cast<u32x4_t*>(Y + off) = out;
  }
}

template <int CIN_PAD, int COUT_PAD, int TT, bool ACT, int CK>
__global__ __launch_bounds__(256) void amp_conv_kernel(AcArgs p) {
  amp_conv_body<CIN_PAD, COUT_PAD, TT, ACT, CK>(p);
}

// the same with the register budget of 3 waves per SIMD, for instantiations whose LDS allows 3
// workgroups per CU
template <int CIN_PAD, int COUT_PAD, int TT, bool ACT, int CK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void amp_conv_kernel_w3(AcArgs p) {
  amp_conv_body<CIN_PAD, COUT_PAD, TT, ACT, CK>(p);
}

template <int CI, int CO, int TT, bool ACT, int CK>
void launch_one(const AcArgs& a, hipStream_t s) {
  constexpr int PA = CI * 2 + 16;
  const int WR = TT + a.hl + a.hr;
  const size_t raw = ACT ? (size_t)(WR + 12) * a.Cin * 2 : 0;
  const size_t ring = (size_t)2 * CO * (CI * 2 + 16);
  const size_t win = (size_t)(TT + kSpan) * PA;
  const size_t out = (size_t)TT * a.Cout * 4;  // overlays window + ring after the MFMAs
  size_t lds = win + (raw > ring ? raw : ring);
  if (lds < out) lds = out;
  dim3 grid((a.Tmax + TT - 1) / TT, 1, a.B);
  if constexpr (!ACT && CK == 48 && CI == 48)
    hipLaunchKernelGGL((amp_conv_kernel_w3<CI, CO, TT, ACT, CK>), grid, dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL((amp_conv_kernel<CI, CO, TT, ACT, CK>), grid, dim3(256), lds, s, a);
}

// TTA / TTC: output rows per workgroup with / without the fused activation; CKN: the stage's channel
// count that gets the compile-time-channel instantiation, with K extent CIK (a multiple of 16)
template <int CI, int CO, int TTA, int TTC, int CKN, int CIK>
void launch_ac(const AcArgs& a, hipStream_t s) {
  const bool ck = a.Cin == CKN && a.Cout == CKN;
  if (a.log_alpha) {
    if (ck) launch_one<CIK, CO, TTA, true, CKN>(a, s);
    else launch_one<CI, CO, TTA, true, 0>(a, s);
  } else {
    if (ck) launch_one<CIK, CO, TTC, false, CKN>(a, s);
    else launch_one<CI, CO, TTC, false, 0>(a, s);
  }
}

}  // namespace

extern "C" int itts_amp_conv_fwd(const void* x, int64_t x_sb, int64_t ldx, const float* up12, const float* down12,
                                 const float* log_alpha, const float* log_beta, const void* w_packed,
                                 const float* bias, const void* r1, const void* r2, void* y, int64_t y_sb,
                                 int64_t ldy, const int32_t* lengths, int B, int Tmax, int Cin, int Cout, int ntaps,
                                 const int32_t* tap_off, float alpha, void* stream) {
  const char* fn = "itts_amp_conv_fwd";
  ITTS_REQUIRE(B >= 0 && Tmax >= 0 && Cin > 0 && Cout > 0, fn, "bad sizes");
  if (B == 0 || Tmax == 0) return 0;
  ITTS_REQUIRE(x && w_packed && bias && y && tap_off, fn, "null pointer");
  ITTS_REQUIRE(!log_alpha || (up12 && down12 && log_beta), fn, "activation needs filters and alpha/beta");
  ITTS_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && x_sb % 8 == 0 && y_sb % 8 == 0,
               fn, "channels / strides must be multiples of 8 (16-B vectors)");
  ITTS_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                 reinterpret_cast<uintptr_t>(r1) | reinterpret_cast<uintptr_t>(r2)) & 15) == 0,
               fn, "tensors must be 16-B aligned");
  ITTS_REQUIRE(ntaps >= 1 && ntaps <= kMaxTapsAc, fn, "ntaps must be in [1, 16]");
  AcArgs a{};
  a.x = static_cast<const uint16_t*>(x);
  a.sxb = x_sb;
  a.ldx = ldx;
  a.up = up12;
  a.down = down12;
  a.log_alpha = log_alpha;
  a.log_beta = log_beta;
  a.w = static_cast<const uint16_t*>(w_packed);
  a.bias = bias;
  a.r1 = static_cast<const uint16_t*>(r1);
  a.r2 = static_cast<const uint16_t*>(r2);
  a.y = static_cast<uint16_t*>(y);
  a.syb = y_sb;
  a.ldy = ldy;
  a.lens = lengths;
  a.B = B;
  a.Tmax = Tmax;
  a.Cin = Cin;
  a.Cout = Cout;
  a.ntaps = ntaps;
  a.alpha = alpha;
  int lo = 0, hi = 0;
  for (int j = 0; j < ntaps; ++j) {
    a.tap_off[j] = tap_off[j];
    lo = tap_off[j] < lo ? tap_off[j] : lo;
    hi = tap_off[j] > hi ? tap_off[j] : hi;
  }
  a.hl = -lo;
  a.hr = hi;
  ITTS_REQUIRE(hi - lo <= kSpan, fn, "tap span exceeds 64 rows");
  hipStream_t s = itts::as_stream(stream);
  const int ci = (Cin + 31) / 32 * 32, co = (Cout + 31) / 32 * 32;
  if (ci == 32 && co == 32) launch_ac<32, 32, ITTS_AMP_TT32, ITTS_AMP_TTC32, 24, 32>(a, s);
  else if (ci == 64 && co == 64) launch_ac<64, 64, ITTS_AMP_TT64, ITTS_AMP_TTC64, 48, ITTS_AMP_K48>(a, s);
  else if (ci == 96 && co == 96) launch_ac<96, 96, ITTS_AMP_TT96, ITTS_AMP_TTC96, 96, 96>(a, s);
  else return itts::fail(fn, "supported (Cin, Cout) padded pairs: (32,32), (64,64), (96,96)");
  return itts::check_launch(fn);
}
