// Activation1d (2x up-sample -> SnakeBeta -> 2x down-sample, BigVGAN alias_free_torch/act.py:24-29,
// resample.py:25-49) with both 12-tap FIRs on MFMA, for bf16 channel-last tiles staged in LDS.
//
// Why: the VALU form (act.hip) spends ~24 FMAs + a sine per output and runs VALU-issue-bound at
// 0.2-0.3 of HBM (profiles/pmc_sq_vocoder_r02b.txt).  Here each FIR is a banded Toeplitz product
// on v_mfma_f32_32x32x16_bf16 and only the SnakeBeta nonlinearity stays on the VALU:
//   up:   U[pos][ch]  = F[pos][row] . X[row][ch]     32 up-sampled positions x 32 channels per tile,
//                                                   K = 32 input rows (22 used)
//   down: Y^T[ch][t]  = V^T[ch][pos] . G^T[pos][t]   32 outputs x 32 channels, K = 80 positions
// The up product's accumulator (lane = channel, 16 positions) is, after SnakeBeta and a bf16 pack,
// exactly the A operand of the down product (lane = channel, 8 consecutive K per half-wave), so V
// never leaves the registers; F and G are lane-dependent constants built once per wave, the
// position order inside a K-block being the accumulator's row order (rows (e&3) + 8(e>>2) + 4h).
// X fragments come from the [time][channel] LDS window with ds_read_b64_tr_b16 (one 4-row x
// 16-column block per 16 lanes, delivered column-major).
//
// Precision: taps are split into bf16 hi + lo (two MFMAs each, MFMA is not the bound), x is bf16
// already, so U is f32-accurate; V is rounded to bf16 (2^-9 relative) before the down product --
// outputs agree with the f32 VALU path to about one bf16 ulp (tests/test_gpu_vocoder.py).
//
// Strip: a wave produces 32*ntile consecutive outputs of one 32-channel block.  Outputs [t0, t0+32i)
// need positions [2 t0 - 5, ...); positions are grouped in 16-blocks from P0 = 2 t0 - 8, up tile j
// covers blocks 2j, 2j+1 and reads input rows t0 - 7 + 16 j + [0, 32).  Output tile i uses blocks
// 4i .. 4i+4, so each tile computes two new up tiles and carries one (2 positions per output in
// steady state).  The window must hold rows t0 - 7 .. t0 + 32 ntile + 24 (replicate-clamped at the
// utterance edges by the caller).  Outputs whose FIR reaches past an utterance edge (t < 3 or
// t >= len - 3: the signal-level replicate pad of the down-sampler) are the caller's to recompute.
//
// Used by the standalone activation (act.hip, bf16 channel-last: 2.4-2.5 TB/s vs 1.2-2.0 for the
// VALU form, profiles/ubench_act_r02.txt).  Fused into the C <= 48 AMP convs (amp_conv.hip) it was
// measured slower (+20-50 %, profiles/ubench_vocoder_r02_ampmfma.txt): the 266-row windows split
// into 2-3 tile strips per wave pay a prologue tile each, and the extra registers halve occupancy.
#pragma once
#include "common.h"

namespace itts_actm {

typedef __attribute__((ext_vector_type(4))) short v4s;
typedef __attribute__((ext_vector_type(8))) short v8s;
typedef __attribute__((address_space(3))) v4s lds_v4s;

struct Taps {
  bf16x8_t fu_[2][2];  // up F (A operand):    [K-block][hi, lo]
  bf16x8_t gd_[5][2];  // down G^T (B operand): [K-block][hi, lo]
  __device__ __forceinline__ bf16x8_t fu(int kb, int hl) const { return fu_[kb][hl]; }
  __device__ __forceinline__ bf16x8_t gd(int kk, int hl) const { return gd_[kk][hl]; }
};
// The same 14 lane-dependent operands kept in LDS ([14][64 lanes] x 16 B, written once per workgroup by
// store_taps) and read at their MFMA: 56 VGPRs fewer per wave than Taps in registers.
struct TapsL {
  const bf16x8_t* p;  // LDS
  __device__ __forceinline__ bf16x8_t fu(int kb, int hl) const { return p[(2 * kb + hl) * 64 + (threadIdx.x & 63)]; }
  __device__ __forceinline__ bf16x8_t gd(int kk, int hl) const {
    return p[(4 + 2 * kk + hl) * 64 + (threadIdx.x & 63)];
  }
};
constexpr int kTapsLdsBytes = 14 * 64 * 16;

__device__ __forceinline__ __bf16 hi_part(float v) { return (__bf16)v; }
__device__ __forceinline__ __bf16 lo_part(float v) { return (__bf16)(v - (float)(__bf16)v); }

// up: F[r][k] for position row r, input row k (tile-relative): even r = 2a -> x rows a+3+q, q in
// [-3, 2], tap 2 f[5 - 2q]; odd r = 2a+1 -> rows a+3+q, q in [-2, 3], tap 2 f[6 - 2q] (the x2 gain
// of the zero-stuffing up-sampler folded in, exact).  down: G^T[pos][n] = g[16 kk + rho - 2 n - 3].
// `tl` = the 12 up taps then the 12 down taps, staged in LDS by the caller (lane-dependent reads
// from LDS: no serialized global loads in the prologue).
__device__ inline void make_taps(const float* tl, Taps& T) {
  const int lane = threadIdx.x & 63, m = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 16 * kb + 8 * h + e;
      const int q = k - 3 - (m >> 1);
      const bool odd = (m & 1) != 0;
      const bool ok = odd ? (q >= -2 && q <= 3) : (q >= -3 && q <= 2);
      const int idx = ok ? (odd ? 6 - 2 * q : 5 - 2 * q) : 0;
      const float t = tl[idx];
      const float v = ok ? 2.0f * t : 0.f;
      T.fu_[kb][0][e] = hi_part(v);
      T.fu_[kb][1][e] = lo_part(v);
    }
#pragma unroll
  for (int kk = 0; kk < 5; ++kk)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int rho = (e & 3) + 8 * (e >> 2) + 4 * h;
      const int idx = 16 * kk + rho - 2 * m - 3;
      const bool ok = idx >= 0 && idx < 12;
      const float t = tl[12 + (ok ? idx : 0)];
      const float v = ok ? t : 0.f;
      T.gd_[kk][0][e] = hi_part(v);
      T.gd_[kk][1][e] = lo_part(v);
    }
}

// wave 0 of the workgroup builds the taps and stores them for TapsL (caller: barrier before use)
__device__ inline void store_taps(const float* tl, bf16x8_t* lds) {
  if ((threadIdx.x >> 6) != 0) return;
  Taps T;
  make_taps(tl, T);
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) lds[(2 * kb + hl) * 64 + lane] = T.fu_[kb][hl];
#pragma unroll
  for (int kk = 0; kk < 5; ++kk)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) lds[(4 + 2 * kk + hl) * 64 + lane] = T.gd_[kk][hl];
}

__device__ __forceinline__ float snake_rev(float u, float a_rev, float inv_b) {
  const float s = __builtin_amdgcn_sinf(u * a_rev);  // v_sin_f32 takes revolutions
  return fmaf(inv_b, s * s, u);
}

// Window addressing: byte offset of (row, channel) in a [rows][PX bytes] bf16 tile, with the 16-B
// slot XOR that keeps the transposed reads (4 rows x 64 B per half-wave) conflict-free:
// PX = 64 / 192: none; 128: rows 2,3 mod 4 swap their 64-B halves; 256 (and multiples): row r's
// 64-B quarter q moves to q ^ (r & 3).
template <int PX>
__device__ __forceinline__ int woff(int row, int ch) {
  int b = ch * 2;
  if constexpr (PX == 128) b ^= ((row >> 1) & 1) << 6;
  else if constexpr (PX % 256 == 0) b ^= (row & 3) << 6;
  return row * PX + b;
}

// U tile: 32 up-sampled positions x 32 channels from input rows row0 .. row0+31, channels cb ..
// cb+31 of the window (EXEC must be full: the transposed read gathers across lanes)
template <int PX, class TT>
__device__ __forceinline__ f32x16_t up_tile(const unsigned char* win, int row0, int cb, const TT& T) {
  const int lane = threadIdx.x & 63, li = lane & 15, h = lane >> 5;
  const int q = li >> 2, p = li & 3;
  const int col = cb + 16 * ((lane >> 4) & 1) + 4 * p;
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int r = row0 + 16 * kb + 8 * h + q;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(win + woff<PX>(r, col)));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(win + woff<PX>(r + 4, col)));
    const v8s b8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    const bf16x8_t b = __builtin_bit_cast(bf16x8_t, b8);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(T.fu(kb, 0), b, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(T.fu(kb, 1), b, acc, 0, 0, 0);
  }
  return acc;
}

// SnakeBeta on a U tile (lane's channel constants) -> two bf16 K-blocks of the down product
__device__ __forceinline__ void snake_pack(const f32x16_t& u, float a_rev, float inv_b, bf16x8_t& b0,
                                           bf16x8_t& b1) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    b0[i] = (__bf16)snake_rev(u[i], a_rev, inv_b);
    b1[i] = (__bf16)snake_rev(u[8 + i], a_rev, inv_b);
  }
}

// One strip: outputs t0 + [0, 32 ntile) for channels cb .. cb+31.  `row0` = window row of time
// t0 - 7.  emit(i, acc): acc = Y^T of output tile i, lane (h, n) holding output time t0 + 32 i + n
// and channels cb + 8 g + 4 h + (0..3) in acc[4 g .. 4 g + 3].
template <int PX, class TT, class Emit>
__device__ __forceinline__ void strip(const unsigned char* win, int row0, int cb, int ntile, const TT& T,
                                      float a_rev, float inv_b, Emit&& emit) {
  bf16x8_t c0, c1;
  snake_pack(up_tile<PX>(win, row0, cb, T), a_rev, inv_b, c0, c1);  // T: Taps or TapsL
  for (int i = 0; i < ntile; ++i) {
    bf16x8_t b2, b3, b4, b5;
    snake_pack(up_tile<PX>(win, row0 + 32 * i + 16, cb, T), a_rev, inv_b, b2, b3);
    snake_pack(up_tile<PX>(win, row0 + 32 * i + 32, cb, T), a_rev, inv_b, b4, b5);
    f32x16_t acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const bf16x8_t blk[5] = {c0, c1, b2, b3, b4};
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(blk[kk], T.gd(kk, 0), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(blk[kk], T.gd(kk, 1), acc, 0, 0, 0);
    }
    emit(i, acc);
    c0 = b4;
    c1 = b5;
  }
}

// Exact Activation1d output at time t (0 <= t < len) for window column ch by the VALU formula (the
// torch path, both replicate pads: x at the up-sampler, the up-sampled signal at the down-sampler);
// window row (tau - tbase) holds x at time tau (replicate-clamped rows).  tl: 12 up, 12 down taps.
template <int PX>
__device__ inline float exact_at(const unsigned char* win, int tbase, int t, int len, int ch, const float* tl,
                                 float a_rev, float inv_b) {
  float o = 0.f;
  for (int k = 0; k < 12; ++k) {
    const int m = min(max(2 * t + k - 5, 0), 2 * len - 1);
    const int pp = m >> 1;
    float acc = 0.f;
    if ((m & 1) == 0) {
      for (int q = -3; q <= 2; ++q)
        acc = fmaf(bf2f(*reinterpret_cast<const uint16_t*>(win + woff<PX>(pp + q - tbase, ch))), 2.0f * tl[5 - 2 * q],
                   acc);
    } else {
      for (int q = -2; q <= 3; ++q)
        acc = fmaf(bf2f(*reinterpret_cast<const uint16_t*>(win + woff<PX>(pp + q - tbase, ch))), 2.0f * tl[6 - 2 * q],
                   acc);
    }
    o = fmaf(tl[12 + k], snake_rev(acc, a_rev, inv_b), o);
  }
  return o;
}

}  // namespace itts_actm
