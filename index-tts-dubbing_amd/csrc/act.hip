// Fused anti-aliased SnakeBeta activation (BigVGAN Activation1d) for gfx950.
//
// Replaces the reference's native op anti_alias_activation_cuda.forward
// (indextts/BigVGAN/alias_free_activation/cuda/anti_alias_activation.cpp:19-23) but follows the
// semantics of the *torch* path (alias_free_torch/act.py:24-29, resample.py:25-49, quirk Q7):
//   u[2p]   = 2 * sum_{q=-3..2} x[clamp(p+q)] * f[5-2q]        (replicate pad 5, 2x conv_transpose, crop 15)
//   u[2p+1] = 2 * sum_{q=-2..3} x[clamp(p+q)] * f[6-2q]
//   v[m]    = u[m] + 1/(exp(b)+1e-9) * sin(u[m]*exp(a))^2       (SnakeBeta, log-scale a/b)
//   y[t]    = sum_{k=0..11} g[k] * v[clamp(2t+k-5, 0, 2L-1)]    (replicate pad 5/6, stride-2 low-pass)
// where clamp() is per utterance length L (ragged batches are exact: every utterance sees its own edges).
//
// Layout: any strides (the vocoder uses channel-last [B, T, C]; the reference op is [B, C, T]).
// One workgroup = 256 threads = a [TT x CT] (time x channel) output tile; the raw input window
// [TT+12 x CT] is staged once through LDS as f32 (replicate-clamped rows), then each thread runs a
// 16-output register window along time for one channel (HBM-bound: 1 read + 1 write per element).
#include <cstdlib>
#include <type_traits>

#include "act_mfma.h"
#include "common.h"

namespace {

constexpr int kThreads = 256;
#ifndef ITTS_ACT_TO
#define ITTS_ACT_TO 16
#endif
constexpr int kTO = ITTS_ACT_TO;  // outputs per thread along time
constexpr int kHalo = 6;  // input samples each side that one output depends on

struct ActArgs {
  const void* x;
  void* y;
  const float* up;
  const float* down;
  const float* log_alpha;
  const float* log_beta;
  const int32_t* lens;
  int B, C, T, CT, nsub;
  int64_t sxb, sxt, sxc, syb, syt, syc;
};

// a_rev = exp(alpha) / (2 pi): v_sin_f32 takes revolutions, so sin(u * a) is one multiply + v_sin
// (__sinf would add a second multiply by 1/(2 pi)); accurate sinf was ~2x the kernel time
__device__ __forceinline__ float snake(float u, float a_rev, float inv_b) {
  const float s = __builtin_amdgcn_sinf(u * a_rev);
  return fmaf(inv_b, s * s, u);
}

// VOUT (bf16 channel-last output, C % 8 == 0): outputs go to an LDS tile [TT][CT] bf16 as they are
// computed and leave as 16-B row vectors after one barrier (2 wide stores per thread instead of 16
// 2-byte stores, one per output)
template <typename TI, typename TO, bool VEC, bool VOUT>
__global__ __launch_bounds__(kThreads) void aa_snakebeta_kernel(ActArgs p) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int b = blockIdx.z;
  const int CT = p.CT, nsub = p.nsub, TT = nsub * kTO;
  const int t0 = blockIdx.x * TT;
  const int c0 = blockIdx.y * CT;
  const int len = p.lens ? p.lens[b] : p.T;
  if (t0 >= len) return;  // uniform per block
  const TI* x = reinterpret_cast<const TI*>(p.x) + (int64_t)b * p.sxb;
  TO* y = reinterpret_cast<TO*>(p.y) + (int64_t)b * p.syb;

  const int rows = TT + 2 * kHalo;
  if constexpr (VEC) {
    // channel-last bf16 with C % 8 == 0: 16-B loads, every load of the tile issued before the
    // first LDS write (one memory latency per block instead of one per loop trip)
    constexpr int kMaxV = kTO <= 16 ? 3 : 5;  // vectors per thread: rows*CT/8 = (256/CT*kTO + 12)*CT/8
    const int cv = CT / 8, nv = rows * cv;
    u32x4_t buf[kMaxV];
#pragma unroll
    for (int i = 0; i < kMaxV; ++i) {
      const int v = threadIdx.x + kThreads * i;
      buf[i] = u32x4_t{0u, 0u, 0u, 0u};
      if (v < nv) {
        const int r = v / cv, c = (v - r * cv) * 8;
        const int t = min(max(t0 - kHalo + r, 0), len - 1);
        if (c0 + c < p.C)
          buf[i] = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(x) + (int64_t)t * p.sxt + c0 + c);
      }
    }
#pragma unroll
    for (int i = 0; i < kMaxV; ++i) {
      const int v = threadIdx.x + kThreads * i;
      if (v < nv) {
        const int r = v / cv, c = (v - r * cv) * 8;
        // two 16-B LDS writes per vector (eight 4-B writes 32 B apart were 8-way bank conflicts)
        f32x4_t* d = reinterpret_cast<f32x4_t*>(xs + r * CT + c);
        d[0] = f32x4_t{__uint_as_float(buf[i][0] << 16), __uint_as_float(buf[i][0] & 0xFFFF0000u),
                       __uint_as_float(buf[i][1] << 16), __uint_as_float(buf[i][1] & 0xFFFF0000u)};
        d[1] = f32x4_t{__uint_as_float(buf[i][2] << 16), __uint_as_float(buf[i][2] & 0xFFFF0000u),
                       __uint_as_float(buf[i][3] << 16), __uint_as_float(buf[i][3] & 0xFFFF0000u)};
      }
    }
  } else {
    for (int idx = threadIdx.x; idx < rows * CT; idx += kThreads) {
      int r = idx / CT, c = idx - r * CT;
      int t = min(max(t0 - kHalo + r, 0), len - 1);
      int ch = c0 + c;
      xs[idx] = ch < p.C ? St<TI>::ld(x + (int64_t)t * p.sxt + (int64_t)ch * p.sxc) : 0.f;
    }
  }
  __syncthreads();

  uint16_t* ys = reinterpret_cast<uint16_t*>(xs + rows * CT);  // VOUT: [TT][CT] bf16 output tile
  const int c = threadIdx.x % CT, sub = threadIdx.x / CT;
  const int ch = c0 + c;
  const int ts = t0 + sub * kTO;
  auto emit = [&](int t, float o) {
    if constexpr (VOUT) ys[(t - t0) * CT + c] = f2bf(o);
    else St<TO>::st(y + (int64_t)t * p.syt + (int64_t)ch * p.syc, o);
  };
  if (sub < nsub && ch < p.C && ts < len) {
  float f[12], g[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) { f[k] = 2.0f * p.up[k]; g[k] = p.down[k]; }  // x2: the up-sampler gain (exact)
  const float a = expf(p.log_alpha[ch]) * 0.15915494309189535f;
  const float inv_b = 1.0f / (expf(p.log_beta[ch]) + 1e-9f);
  const float* col = xs + (sub * kTO) * CT + c;  // row r <-> t = ts - 6 + r

  if (ts >= 3 && ts + kTO + 3 <= len) {
    float xr[kTO + 2 * kHalo];
#pragma unroll
    for (int i = 0; i < kTO + 2 * kHalo; ++i) xr[i] = col[i * CT];
    float v[2 * kTO + 10];
#pragma unroll
    for (int j = 0; j < 2 * kTO + 10; ++j) {
      float acc = 0.f;
      if (j & 1) {  // even upsampled index
#pragma unroll
        for (int q = -3; q <= 2; ++q) acc = fmaf(xr[4 + (j - 1) / 2 + q], f[5 - 2 * q], acc);
      } else {
#pragma unroll
        for (int q = -2; q <= 3; ++q) acc = fmaf(xr[3 + j / 2 + q], f[6 - 2 * q], acc);
      }
      v[j] = snake(acc, a, inv_b);
    }
#pragma unroll
    for (int i = 0; i < kTO; ++i) {
      float o = 0.f;
#pragma unroll
      for (int k = 0; k < 12; ++k) o = fmaf(g[k], v[2 * i + k], o);
      emit(ts + i, o);
    }
  } else {
    // edge chunk: explicit two-level replicate clamping (x level and activated-signal level)
    const int base = ts - kHalo;  // t of LDS row `sub*kTO`
    const int te = min(ts + kTO, len);
    for (int t = ts; t < te; ++t) {
      float o = 0.f;
      for (int k = 0; k < 12; ++k) {
        int m = min(max(2 * t + k - 5, 0), 2 * len - 1);
        int pp = m >> 1;
        float acc = 0.f;
        if ((m & 1) == 0) {
          for (int q = -3; q <= 2; ++q) acc = fmaf(col[(min(max(pp + q, 0), len - 1) - base) * CT], f[5 - 2 * q], acc);
        } else {
          for (int q = -2; q <= 3; ++q) acc = fmaf(col[(min(max(pp + q, 0), len - 1) - base) * CT], f[6 - 2 * q], acc);
        }
        o = fmaf(g[k], snake(acc, a, inv_b), o);
      }
      emit(t, o);
    }
  }
  }  // active thread
  if constexpr (VOUT) {
    __syncthreads();
    const int nrow = min(TT, len - t0), cv = CT / 8;
    for (int v = threadIdx.x; v < nrow * cv; v += kThreads) {
      const int r = v / cv, cc = (v - r * cv) * 8;
      if (c0 + cc < p.C)
        *reinterpret_cast<u32x4_t*>(y + (int64_t)(t0 + r) * p.syt + c0 + cc) =
            *reinterpret_cast<const u32x4_t*>(ys + r * CT + cc);
    }
  }
}

// ---- bf16 channel-last path with both FIRs on MFMA (act_mfma.h) ----
// Job = TT = (4 / NB) * 32 * S output rows x NB * 32 channels of one utterance; a workgroup (4 waves
// = NB 32-channel blocks x (4 / NB) strips of S 32-row tiles) keeps one channel group and walks jobs
// blockIdx.y, + gridDim.y, ... (persistent): the taps and channel constants are built once, and the
// next job's window loads are in flight while this job's strips compute.  The window [TT + 32
// rows][NB * 64 B] holds x rows t0 - 7 .. t0 + TT + 24 (rows the FIRs weight by zero are zero, not
// loaded), replicate-clamped per utterance.  Interior outputs leave straight from the down product's
// accumulators (8-B stores of 4 channels); outputs within 3 samples of an utterance edge, where the
// down-sampler's own replicate pad applies, are recomputed by the VALU formula from the same window.
#ifndef ITTS_ACT_TAPS_LDS  // the FIR operands in LDS instead of 56 VGPRs per lane
#define ITTS_ACT_TAPS_LDS 0  // measured neutral (profiles/ubench_act_r03.txt): the taps are not what holds the registers
#endif
// (16-B interior stores, lane pairs swapping channel halves, were bit-identical and measured neutral -- vocoder
// 87.6 / 88.0 / 87.4 ms vs 87.7 / 87.2 / 87.0, profiles/r05xa_ab.txt -- and removed in round 6)
template <int NB, int S>
#ifndef ITTS_ACT_WPS  // waves per SIMD the register allocation targets
#define ITTS_ACT_WPS 2  // 3 spills 32-37 VGPRs: 30-40 % slower (profiles/ubench_act_r03.txt)
#endif
__global__ __launch_bounds__(256, ITTS_ACT_WPS) void aa_snake_mfma_kernel(ActArgs p, int ntt, int njobs) {
  constexpr int PX = NB * 64, NS = 4 / NB, TT = NS * 32 * S, WROWS = TT + 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char win[];
  const int c0 = blockIdx.x * NB * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int CV = NB * 4;  // 16-B vectors per row
  constexpr int NV = (WROWS * CV + 255) / 256;
  float* tl = reinterpret_cast<float*>(win + WROWS * PX);  // 12 up taps, 12 down taps
  bf16x8_t* tap_lds = reinterpret_cast<bf16x8_t*>(win + WROWS * PX + 128);  // 16-B aligned (PX % 64 == 0)
  if (tid < 24) tl[tid] = tid < 12 ? p.up[tid] : p.down[tid - 12];

  // window rows 1 .. TT + 12 (t0 - 6 .. t0 + TT + 5) of job j into registers
  u32x4_t buf[NV];
  auto wload = [&](int j) {
    const int b = j / ntt, t0 = (j - b * ntt) * TT;
    const int len = p.lens ? p.lens[b] : p.T;
    const uint16_t* x = reinterpret_cast<const uint16_t*>(p.x) + (int64_t)b * p.sxb;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + 256 * i;
      buf[i] = u32x4_t{0u, 0u, 0u, 0u};
      const int r = v / CV, c = (v - r * CV) * 8;
      if (t0 < len && v < WROWS * CV && r >= 1 && r <= TT + 12 && c0 + c < p.C) {
        const int t = min(max(t0 - 7 + r, 0), len - 1);
        buf[i] = ld_stream(reinterpret_cast<const u32x4_t*>(x + (int64_t)t * p.sxt + c0 + c));
      }
    }
  };
  int job = blockIdx.y;
  if (job < njobs) wload(job);
  __syncthreads();  // taps staged

  const int blk = wave % NB, sidx = wave / NB;
  const int cb = 32 * blk;  // window column of the block
#if ITTS_ACT_TAPS_LDS
  itts_actm::store_taps(tl, tap_lds);  // visible after the barrier at the first job's window store
  const itts_actm::TapsL T{tap_lds};
#else
  itts_actm::Taps T;
  itts_actm::make_taps(tl, T);
#endif
  const int ch = c0 + cb + (lane & 31);
  const float a_rev = ch < p.C ? expf(p.log_alpha[ch]) * 0.15915494309189535f : 0.f;
  const float inv_b = ch < p.C ? 1.0f / (expf(p.log_beta[ch]) + 1e-9f) : 0.f;
  const int h = lane >> 5;

  for (; job < njobs; job += gridDim.y) {
    const int b = job / ntt, t0 = (job - b * ntt) * TT;
    const int len = p.lens ? p.lens[b] : p.T;
    __syncthreads();  // the previous job's readers of the window are done
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + 256 * i;
      const int r = v / CV, c = (v - r * CV) * 8;
      if (v < WROWS * CV) *reinterpret_cast<u32x4_t*>(win + itts_actm::woff<PX>(r, c)) = buf[i];
    }
    __syncthreads();
    if (job + gridDim.y < njobs) wload(job + gridDim.y);  // in flight during this job's strips
    if (t0 >= len) continue;  // uniform per workgroup
    uint16_t* y = reinterpret_cast<uint16_t*>(p.y) + (int64_t)b * p.syb;

    // ---- strips ----
    const int ts = t0 + sidx * 32 * S;  // first output of the strip
    // NB = 3 (C = 96: whole 192-B rows per job): one strip per block, the fourth wave has none
    const int ntile = sidx < NS ? min(S, max(0, (len - ts + 31) / 32)) : 0;
    itts_actm::strip<PX>(win, sidx * 32 * S, cb, ntile, T, a_rev, inv_b, [&](int i, const f32x16_t& acc) {
      const int t = ts + 32 * i + (lane & 31);
      if (t < 3 || t >= len - 3) return;  // edges: VALU fix-up below
      uint16_t* yr = y + (int64_t)t * p.syt + c0 + cb + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (c0 + cb + 8 * g + 4 * h < p.C) {
          const u32x2_t o{pack2bf(acc[4 * g], acc[4 * g + 1]), pack2bf(acc[4 * g + 2], acc[4 * g + 3])};
          *reinterpret_cast<u32x2_t*>(yr + 8 * g) = o;
        }
      }
    });

    // ---- outputs within 3 samples of an utterance edge (uniform per block) ----
    if (t0 < 3 || t0 + TT > len - 3) {
      const int te = min(t0 + TT, len);
      for (int it = tid; it < 6 * NB * 32; it += 256) {
        const int e = it / (NB * 32), cc = it - e * (NB * 32);
        const int t = e < 3 ? e : len - 6 + e;
        if (t < t0 || t >= te || t < 0 || (e >= 3 && t < 3) || c0 + cc >= p.C) continue;
        const float a = expf(p.log_alpha[c0 + cc]) * 0.15915494309189535f;
        const float ib = 1.0f / (expf(p.log_beta[c0 + cc]) + 1e-9f);
        y[(int64_t)t * p.syt + c0 + cc] = f2bf(itts_actm::exact_at<PX>(win, t0 - 7, t, len, cc, tl, a, ib));
      }
    }
  }
}

#ifndef ITTS_ACT_S  // 32-row output tiles per wave strip (job = (4 / NB) * 32 * S rows)
#define ITTS_ACT_S 4
#endif
#ifndef ITTS_ACT_WGS  // resident workgroups targeted by the persistent activation grid
#define ITTS_ACT_WGS 512
#endif
template <int NB, int S>
void launch_mfma(const ActArgs& a, hipStream_t s) {
  constexpr int TT = (4 / NB) * 32 * S;
  const int nblk = (a.C + 31) / 32, ngrp = (nblk + NB - 1) / NB;
  const int ntt = (a.T + TT - 1) / TT, njobs = ntt * a.B;
  int per = ITTS_ACT_WGS / ngrp;
  per = per < 1 ? 1 : (per > njobs ? njobs : per);
  const size_t lds = (size_t)(TT + 32) * NB * 64 + 128 + (ITTS_ACT_TAPS_LDS ? itts_actm::kTapsLdsBytes : 0);
  hipLaunchKernelGGL((aa_snake_mfma_kernel<NB, S>), dim3(ngrp, per, 1), dim3(256), lds, s, a, ntt, njobs);
}

template <typename TI, typename TO>
void launch(const ActArgs& a, bool vec, bool vout, hipStream_t s) {
  dim3 grid((a.T + a.nsub * kTO - 1) / (a.nsub * kTO), (a.C + a.CT - 1) / a.CT, a.B);
  const int TT = a.nsub * kTO;
  size_t lds = sizeof(float) * (size_t)(TT + 2 * kHalo) * a.CT;
  if constexpr (std::is_same<TO, uint16_t>::value) {
    if (vout) {
      lds += sizeof(uint16_t) * (size_t)TT * a.CT;
      if (vec)
        hipLaunchKernelGGL((aa_snakebeta_kernel<TI, TO, true, true>), grid, dim3(kThreads), lds, s, a);
      else
        hipLaunchKernelGGL((aa_snakebeta_kernel<TI, TO, false, true>), grid, dim3(kThreads), lds, s, a);
      return;
    }
  }
  if (vec)
    hipLaunchKernelGGL((aa_snakebeta_kernel<TI, TO, true, false>), grid, dim3(kThreads), lds, s, a);
  else
    hipLaunchKernelGGL((aa_snakebeta_kernel<TI, TO, false, false>), grid, dim3(kThreads), lds, s, a);
}

}  // namespace

// C = 96 as ONE 3-block channel group per job (whole 192-B rows: every window row one contiguous read)
// instead of three 1-block groups each reading 64 B of every row; ITTS_ACT_NB3=0: the 1-block form (A/B)
bool act_nb3_enabled() {  // read per launch (tests toggle it in one process)
  const char* e = getenv("ITTS_ACT_NB3");
  return !(e && e[0] == '0');
}

// ITTS_ACT_MFMA=0 selects the VALU kernel for the bf16 channel-last layout too (A/B measurements)
bool act_mfma_enabled() {
  static const bool on = [] {
    const char* e = getenv("ITTS_ACT_MFMA");
    return !(e && e[0] == '0');
  }();
  return on;
}

extern "C" int itts_aa_snakebeta_fwd(const void* x, void* y, const float* up12, const float* down12,
                                     const float* log_alpha, const float* log_beta, const int32_t* lengths,
                                     int B, int C, int T, int64_t x_sb, int64_t x_st, int64_t x_sc, int64_t y_sb,
                                     int64_t y_st, int64_t y_sc, int dtype_in, int dtype_out, void* stream) {
  const char* fn = "itts_aa_snakebeta_fwd";
  ITTS_REQUIRE(B >= 0 && C >= 0 && T >= 0, fn, "negative size");
  if (B == 0 || C == 0 || T == 0) return 0;
  ITTS_REQUIRE(x && y && up12 && down12 && log_alpha && log_beta, fn, "null pointer");
  ITTS_REQUIRE((dtype_in == ITTS_F32 || dtype_in == ITTS_BF16 || dtype_in == ITTS_F16) &&
                   (dtype_out == ITTS_F32 || dtype_out == ITTS_BF16 || dtype_out == ITTS_F16),
               fn, "unsupported dtype (f32=0, bf16=1, f16=2)");
  ITTS_REQUIRE((dtype_in == ITTS_F16) == (dtype_out == ITTS_F16), fn, "f16 input needs f16 output (and vice versa)");
  ActArgs a{x, y, up12, down12, log_alpha, log_beta, lengths, B, C, T, 0, 0, x_sb, x_st, x_sc, y_sb, y_st, y_sc};
  // channel tile: all channels when C <= 64, else 64 -- or 32 when 32 divides C and 64 does not
  // (C = 96: two 64-channel tiles would leave half the second tile's threads idle)
  a.CT = C <= 64 ? C : (C % 64 != 0 && C % 32 == 0 ? 32 : 64);
  a.nsub = kThreads / a.CT;
  hipStream_t s = itts::as_stream(stream);
  // vectorised staging: channel-last bf16 input, 16-B aligned rows
  const bool vec = dtype_in == ITTS_BF16 && x_sc == 1 && C % 8 == 0 && x_st % 8 == 0 && x_sb % 8 == 0 &&
                   (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  // vectorised output through LDS: channel-last bf16 output, 16-B aligned rows
  const bool vout = dtype_out == ITTS_BF16 && y_sc == 1 && C % 8 == 0 && y_st % 8 == 0 && y_sb % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(y) & 15) == 0;
  if (dtype_in == ITTS_F16) launch<_Float16, _Float16>(a, false, false, s);  // f32 math, RNE half stores
  else if (dtype_in == ITTS_BF16 && dtype_out == ITTS_BF16 && vec && vout && act_mfma_enabled()) {
    // the vocoder's layout: both FIRs on MFMA
    const int nblk = (C + 31) / 32;
    if (nblk % 4 == 0) launch_mfma<4, ITTS_ACT_S>(a, s);
    else if (nblk % 2 == 0) launch_mfma<2, ITTS_ACT_S>(a, s);
    else if (nblk == 3 && act_nb3_enabled()) launch_mfma<3, 2 * ITTS_ACT_S>(a, s);
    else launch_mfma<1, ITTS_ACT_S>(a, s);
  } else if (dtype_in == ITTS_BF16 && dtype_out == ITTS_BF16) launch<uint16_t, uint16_t>(a, vec, vout, s);
  else if (dtype_in == ITTS_F32 && dtype_out == ITTS_F32) launch<float, float>(a, false, false, s);
  else if (dtype_in == ITTS_F32) launch<float, uint16_t>(a, false, vout, s);
  else launch<uint16_t, float>(a, vec, false, s);
  return itts::check_launch(fn);
}

// Drop-in for the reference's contiguous [B, C, T] op (anti_alias_activation_cuda.forward),
// with caller-owned output (torch-path edge semantics, see header).
extern "C" int itts_aa_snakebeta_bct(const void* x, void* y, const float* up12, const float* down12,
                                     const float* log_alpha, const float* log_beta, int B, int C, int T, int dtype,
                                     void* stream) {
  return itts_aa_snakebeta_fwd(x, y, up12, down12, log_alpha, log_beta, nullptr, B, C, T, (int64_t)C * T, 1, T,
                               (int64_t)C * T, 1, T, dtype, dtype, stream);
}
