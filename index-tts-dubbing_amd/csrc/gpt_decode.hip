// Fused decode-step projection GEMM for gfx950 (batch rows M <= 32 per launch tile).
//
//   Y = epi( prologue(X) @ W^T )
//     prologue: A = X (bf16 [M][K], global)                      -- LNMODE 0
//               A = LN_1(X) (X f32 residual stream [M][K])         -- LNMODE 1  (HF ln_1 / ln_2)
//               A = LN_2(LN_1(X))                                  -- LNMODE 2  (ln_f then final_norm, Q5)
//     epilogue: EPI 0: Y = act(acc + bias) stored as OutT (act = gelu_tanh optional)
//               EPI 1: Y(f32) += acc + bias                        (residual add, in place)
//               EPI 2: Y[ks] = acc  (f32 partial of K split ks; reduced + LayerNormed by
//                      itts_residual_reduce_ln in gpt_norm.hip -- deterministic, no atomics)
//
// Product decode step (engine.HipGPT._decode_step) uses LNMODE 0 everywhere: the residual add and
// the following LayerNorm are fused into one reduce kernel per sub-layer, and the O / MLP-proj
// GEMMs (K = D or 4D, N = D: only D/32 column tiles) are split along K so that >= 256 workgroups
// stream the weights.  LNMODE 1/2 (LayerNorm recomputed per workgroup from the L2-resident
// residual stream, staged in LDS as bf16) measured slower at batch 32 and is kept for small-D
// models and the unit tests.
//
// Weights are prepacked in MFMA-fragment order [N/32][K/16][64][8] bf16 (see pack_skinny): one
// wave load = one contiguous 1 KiB line pair.  Workgroup = NW waves over interleaved k-steps,
// 2-stage register pipeline (next 8 k-steps' loads issued before this batch's MFMAs), fixed-order
// cross-wave reduction through LDS (bitwise batch-invariant per row).
#include "common.h"

namespace {

constexpr int kU = 8;
constexpr int kNI = 4;  // decode_gemm16x: k-steps per wave of the straight-line form (K = 1024 at 8 waves)

__device__ __forceinline__ float gelu_tanh_d(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
}

template <int NW>
__device__ __forceinline__ float wg_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += red[i];
  return s;
}

// weight-stream loads of the decode GEMMs (A/B builds: ITTS_W_NT=0 uses plain loads)
#ifndef ITTS_W_NT
#define ITTS_W_NT 1
#endif
#if ITTS_W_NT
#define ITTS_WLOAD(p) __builtin_nontemporal_load(p)
#else
#define ITTS_WLOAD(p) (*(p))
#endif

struct DgArgs {
  const void* a;      // LNMODE 0: bf16 A [.][lda]; else f32 X [.][lda]
  int64_t lda;
  const u32x4_t* w;   // packed weights
  int K, N, M;
  const float* bias;
  const float *g1, *b1, *g2, *b2;
  int gelu;
  void* y;
  int64_t ldy;
  int64_t split_stride;  // EPI 2: floats between the partial products of consecutive K splits
};

// normalise RPW rows held in registers (one wave, 64 lanes x KPL elements per row)
template <int KPL>
__device__ __forceinline__ void ln_vec(float (&v)[KPL], const float* g, const float* b, int K) {
  const int lane = threadIdx.x & 63;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < KPL; ++i) s += v[i];
  const float mean = wave_sum(s) / K;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < KPL; ++i) q += (v[i] - mean) * (v[i] - mean);
  const float rstd = rsqrtf(wave_sum(q) / K + 1e-5f);
#pragma unroll
  for (int i = 0; i < KPL / 4; ++i) {
    const int e = 4 * (lane + 64 * i);
    const f32x4_t g4 = *reinterpret_cast<const f32x4_t*>(g + e);
    const f32x4_t b4 = *reinterpret_cast<const f32x4_t*>(b + e);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * i + j] = (v[4 * i + j] - mean) * rstd * g4[j] + b4[j];
  }
}

// EPI: 0 store act(acc + bias) as OutT; 1 f32 Y += acc + bias; 2 split-K over gridDim.y, each split
// stores its f32 partial product (an in-kernel last-arriver reduction was measured slower: the two
// agent-scope fences it needs cost more than the separate reduce launch).
// MT (LNMODE 0 only): 32-row tiles per workgroup sharing every weight fragment (beam decoding).
template <int NW, int LNMODE, int EPI, int KLN, typename OutT, int MT = 1>
__global__ __launch_bounds__(64 * NW) void decode_gemm_kernel(DgArgs p) {
  static_assert(MT == 1 || LNMODE == 0, "row-tile batching needs a bf16 A operand");
  constexpr int APITCH = KLN * 2 + 16;  // LDS row pitch (bytes) of the normalised A tile
  constexpr int RED_BYTES = NW * 16 * 64 * sizeof(float);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem);                 // [NW][16][64] f32
  unsigned char* As = smem + RED_BYTES;                         // [32][APITCH] bf16 (LN modes)
  const int nt = blockIdx.x, ks = blockIdx.y, nsplit = gridDim.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int K = LNMODE ? KLN : p.K;
  const int ksteps = K / 16, kper = ksteps / nsplit, kbeg = ks * kper;
  const int niter = (kper - w + NW - 1) / NW;  // this wave's k-steps: kbeg + w + NW*i
  const u32x4_t* Wt = p.w + ((int64_t)nt * ksteps + kbeg) * 64 + lane;
  const int r32 = lane & 31, h = lane >> 5;

  // zero-initialised: guarded (i < niter) MFMAs on never-loaded slots were speculated by hipcc and
  // produced NaN columns for short K (measured: K=256/512) -- keep every slot defined
  u32x4_t wa[kU] = {}, wb[kU] = {};
  auto wload = [&](u32x4_t (&dst)[kU], int i0) {
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + u < niter) dst[u] = ITTS_WLOAD(Wt + (int64_t)(w + NW * (i0 + u)) * 64);
  };
  wload(wa, 0);  // weight stream starts before the prologue

  if (LNMODE) {
    // wave w normalises rows w + NW*j (j < 32/NW); all row loads issued before the first reduction
    constexpr int KPL = KLN / 64, RPW = 32 / NW;
    const float* X = reinterpret_cast<const float*>(p.a);
    float v[RPW][KPL];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int r = w + NW * j;
#pragma unroll
      for (int i = 0; i < KPL / 4; ++i) {
        f32x4_t x4 = {0.f, 0.f, 0.f, 0.f};
        if (r < p.M) x4 = *reinterpret_cast<const f32x4_t*>(X + (int64_t)r * p.lda + 4 * (lane + 64 * i));
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][4 * i + e] = x4[e];
      }
    }
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int r = w + NW * j;
      if (r < p.M) {  // wave-uniform
        ln_vec<KPL>(v[j], p.g1, p.b1, KLN);
        if (LNMODE == 2) ln_vec<KPL>(v[j], p.g2, p.b2, KLN);
      }
#pragma unroll
      for (int i = 0; i < KPL / 4; ++i) {
        const u32x2_t pk = {pack2bf(v[j][4 * i], v[j][4 * i + 1]), pack2bf(v[j][4 * i + 2], v[j][4 * i + 3])};
        *reinterpret_cast<u32x2_t*>(As + r * APITCH + 8 * (lane + 64 * i)) = pk;
      }
    }
    __syncthreads();
  }

  f32x16_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  auto afrag = [&](int s, int t) -> bf16x8_t {
    if (LNMODE) return *reinterpret_cast<const bf16x8_t*>(As + r32 * APITCH + 32 * s + 16 * h);
    const uint16_t* A = reinterpret_cast<const uint16_t*>(p.a);
    return *reinterpret_cast<const bf16x8_t*>(A + (int64_t)(32 * t + r32) * p.lda + 16 * s + 8 * h);
  };
  auto compute = [&](const u32x4_t (&src)[kU], int i0) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      bf16x8_t af[kU] = {};
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (i0 + u < niter) af[u] = afrag(kbeg + w + NW * (i0 + u), t);
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (i0 + u < niter)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[u], *reinterpret_cast<const bf16x8_t*>(&src[u]), acc[t],
                                                           0, 0, 0);
    }
  };
  for (int i0 = 0; i0 < niter; i0 += 2 * kU) {
    if (i0 + kU < niter) wload(wb, i0 + kU);
    compute(wa, i0);
    if (i0 + 2 * kU < niter) wload(wa, i0 + 2 * kU);
    if (i0 + kU < niter) compute(wb, i0 + kU);
  }

  // epilogue tile by tile through one [NW][16][64] LDS buffer (32 KiB at NW = 8, any MT)
  float* myred = red + w * 16 * 64;
  constexpr int PER = 1024 / (64 * NW);  // tile outputs per thread
#pragma unroll
  for (int tile = 0; tile < MT; ++tile) {
    if (tile > 0) __syncthreads();  // previous tile's reads done
#pragma unroll
    for (int r = 0; r < 16; ++r) myred[r * 64 + lane] = acc[tile][r];
    __syncthreads();
    float tv[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int o = threadIdx.x + 64 * NW * k;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) v += red[ww * 1024 + o];
      tv[k] = v;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int o = threadIdx.x + 64 * NW * k;
      const int r = o / 64, l = o % 64;
      const int row = 32 * tile + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      const int n = nt * 32 + (l & 31);
      if (row >= p.M || n >= p.N) continue;
      if (EPI == 2) {  // split-K partial (no bias); reduced in fixed order by itts_residual_reduce_ln
        st_out(reinterpret_cast<float*>(p.y) + ks * p.split_stride + (int64_t)row * p.ldy + n, tv[k]);
        continue;
      }
      float v = tv[k];
      if (p.bias) v += p.bias[n];
      if (EPI >= 1) {
        float* Y = reinterpret_cast<float*>(p.y) + (int64_t)row * p.ldy + n;
        *Y = *Y + v;
      } else {
        if (p.gelu) v = gelu_tanh_d(v);
        St<OutT>::st(reinterpret_cast<OutT*>(p.y) + (int64_t)row * p.ldy + n, v);
      }
    }
  }
}

template <int NW, int LNMODE, int EPI, int KLN, typename OutT>
void launch_dg(const DgArgs& a, int row_tiles, int ksplit, hipStream_t s) {
  if constexpr (LNMODE == 0) {
    if (row_tiles > 1) {  // up to 4 row tiles per launch share the weight stream
      for (int t = 0; t < row_tiles; t += 4) {
        DgArgs b = a;
        const int64_t ra = (int64_t)t * 32;
        const int rows = a.M - 32 * t < 128 ? a.M - 32 * t : 128, mt = (rows + 31) / 32;
        b.M = rows;
        b.a = reinterpret_cast<const uint16_t*>(a.a) + ra * a.lda;
        if (EPI >= 1) b.y = reinterpret_cast<float*>(a.y) + ra * a.ldy;
        else b.y = reinterpret_cast<OutT*>(a.y) + ra * a.ldy;
        const dim3 grid((a.N + 31) / 32, ksplit), block(64 * NW);
        const size_t lds = NW * 16 * 64 * sizeof(float);
        switch (mt) {
          case 1: hipLaunchKernelGGL((decode_gemm_kernel<NW, 0, EPI, KLN, OutT, 1>), grid, block, lds, s, b); break;
          case 2: hipLaunchKernelGGL((decode_gemm_kernel<NW, 0, EPI, KLN, OutT, 2>), grid, block, lds, s, b); break;
          case 3: hipLaunchKernelGGL((decode_gemm_kernel<NW, 0, EPI, KLN, OutT, 3>), grid, block, lds, s, b); break;
          default: hipLaunchKernelGGL((decode_gemm_kernel<NW, 0, EPI, KLN, OutT, 4>), grid, block, lds, s, b); break;
        }
      }
      return;
    }
  }
  size_t lds = NW * 16 * 64 * sizeof(float) + (LNMODE ? 32 * (KLN * 2 + 16) : 0);
  for (int t = 0; t < row_tiles; ++t) {
    DgArgs b = a;
    const int64_t ra = (int64_t)t * 32;
    b.M = a.M - 32 * t < 32 ? a.M - 32 * t : 32;
    if (LNMODE) b.a = reinterpret_cast<const float*>(a.a) + ra * a.lda;
    else b.a = reinterpret_cast<const uint16_t*>(a.a) + ra * a.lda;
    if (EPI >= 1) b.y = reinterpret_cast<float*>(a.y) + ra * a.ldy;
    else b.y = reinterpret_cast<OutT*>(a.y) + ra * a.ldy;
    hipLaunchKernelGGL((decode_gemm_kernel<NW, LNMODE, EPI, KLN, OutT>), dim3((a.N + 31) / 32, ksplit), dim3(64 * NW),
                       lds, s, b);
  }
}

// ---- 16-column tiles (v_mfma_f32_16x16x32_bf16) for the wide store-epilogue projections ----------
// On 32-column tiles c_fc (N = 4096) and mel_head (N = 8194) launch 128 / 257 workgroups that stream
// 64 KiB of weights each, and these latency-bound launches take about as long as one workgroup's
// stream; on 16-column tiles they launch 256 / 513 workgroups of 32 KiB (every CU busy, half the
// bytes per workgroup).  Weights [N/16][K/32][64 lanes][8] bf16: lane l = 16q + c holds
// W^T[16nt + c][32s + 8q : +8] (pack_skinny16); one wave load = one contiguous 1 KiB.  A = bf16
// [32-row tile][lda]; the two 16-row halves of the tile share every weight fragment.  Same wave /
// k-step interleave, register pipeline and fixed-order cross-wave LDS reduction as decode_gemm_kernel
// (bitwise batch-invariant per row).  Store epilogue only: y = act(acc + bias).
template <int NW, typename OutT>
__global__ __launch_bounds__(64 * NW) void decode_gemm16_kernel(DgArgs p) {
  __shared__ float red[NW][8][64];
  const int nt = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ksteps = p.K / 32;
  const int niter = (ksteps - w + NW - 1) / NW;  // this wave's k-steps: w + NW*i
  const u32x4_t* Wt = p.w + (int64_t)nt * ksteps * 64 + lane;
  const int c16 = lane & 15, q = lane >> 4;
  const uint16_t* A = reinterpret_cast<const uint16_t*>(p.a);

  u32x4_t wa[kU] = {}, wb[kU] = {};  // zero-initialised: see decode_gemm_kernel
  auto wload = [&](u32x4_t (&dst)[kU], int i0) {
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + u < niter) dst[u] = ITTS_WLOAD(Wt + (int64_t)(w + NW * (i0 + u)) * 64);
  };
  wload(wa, 0);
  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const u32x4_t (&src)[kU], int i0) {
    bf16x8_t a0[kU] = {}, a1[kU] = {};
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + u < niter) {
        const int64_t col = 32 * (w + NW * (i0 + u)) + 8 * q;
        a0[u] = *reinterpret_cast<const bf16x8_t*>(A + (int64_t)c16 * p.lda + col);
        a1[u] = *reinterpret_cast<const bf16x8_t*>(A + (int64_t)(16 + c16) * p.lda + col);
      }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + u < niter) {
        const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(&src[u]);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], bfr, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], bfr, acc1, 0, 0, 0);
      }
  };
  for (int i0 = 0; i0 < niter; i0 += 2 * kU) {
    if (i0 + kU < niter) wload(wb, i0 + kU);
    compute(wa, i0);
    if (i0 + 2 * kU < niter) wload(wa, i0 + 2 * kU);
    if (i0 + kU < niter) compute(wb, i0 + kU);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[w][r][lane] = acc0[r];
    red[w][4 + r][lane] = acc1[r];
  }
  __syncthreads();
  // 512 outputs (32 rows x 16 columns); C/D layout of 16x16x32: row = 4*(lane>>4) + reg, col = lane&15
  for (int o = threadIdx.x; o < 512; o += 64 * NW) {
    const int e = o >> 6, l = o & 63;  // e = 4 * (row half) + reg
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[ww][e][l];
    const int row = 16 * (e >> 2) + 4 * (l >> 4) + (e & 3);
    const int n = nt * 16 + (l & 15);
    if (row >= p.M || n >= p.N) continue;
    if (p.bias) v += p.bias[n];
    if (p.gelu) v = gelu_tanh_d(v);
    St<OutT>::st(reinterpret_cast<OutT*>(p.y) + (int64_t)row * p.ldy + n, v);
  }
}

template <int NW, typename OutT>
void launch_dg16(const DgArgs& a, int row_tiles, hipStream_t s) {
  for (int t = 0; t < row_tiles; ++t) {
    DgArgs b = a;
    b.M = a.M - 32 * t < 32 ? a.M - 32 * t : 32;
    b.a = reinterpret_cast<const uint16_t*>(a.a) + (int64_t)t * 32 * a.lda;
    b.y = reinterpret_cast<OutT*>(a.y) + (int64_t)t * 32 * a.ldy;
    hipLaunchKernelGGL((decode_gemm16_kernel<NW, OutT>), dim3((a.N + 15) / 16), dim3(64 * NW), 0, s, b);
  }
}

// ---- 16-column tiles with the LayerNorm folded in, and the residual epilogue -------------------
// Product decode step (bf16): five launches per layer instead of seven.  The residual stream is kept
// as x (f32) plus its bf16 copy x^ (the GEMM A operand), and LayerNorm is never materialised:
//   LN(x) W + bias = rstd * (x W' - mean * u) + c,   W' = diag(g) W,  u = 1^T W',  c = b^T W + bias
// (W' rounded to bf16 and u summed from those rounded values, so the mean term cancels exactly what
// the MFMA accumulates).  Every workgroup streams its whole K range of A = x^ for the MFMAs anyway,
// so it takes the row statistics (sum and sum of squares of x^) from the same fragments: per lane,
// then over the 4 lanes sharing a row (xor shuffles), then over the waves in a fixed order through
// LDS -- bitwise batch-invariant per row.  (Measured |mean| / std of the residual rows <= 0.09 with
// the IndexTTS-1.5 shapes, so the mean subtraction after the product loses nothing measurable; see
// DESIGN.md.)  Epilogues: EPI 0 y = act(...) stored as OutT (c_attn -> q/k/v f32, c_fc + gelu ->
// bf16); EPI 1 residual: x += acc + c in place and x^ = bf16(x) (attn.c_proj / mlp.c_proj without
// split-K, so no partial slabs and no reduce launch).
struct Dg16xArgs {
  const uint16_t* a;
  int64_t lda;
  const u32x4_t* w;
  int K, N, M;
  const float* c;   // additive per-column term (bias, + b^T W when folded); may be null
  const float* u;   // FOLD: column sums of W'
  float eps;
  int gelu;
  void* y;
  int64_t ldy;
  uint16_t* xh;     // EPI 1: bf16 copy of the updated residual
  int64_t ldxh;
};

// MT = 32-row tiles per workgroup (beam decoding: 3 x 32 rows): every weight fragment is loaded once
// and multiplied into all MT tiles, so the weights cross HBM once per step, not once per tile.
template <int NW, bool FOLD, int EPI, typename OutT, int MT>
__global__ __launch_bounds__(64 * NW) void decode_gemm16x_kernel(Dg16xArgs p) {
  constexpr int R = 32 * MT;
  __shared__ float red[NW][8][64];  // one 32-row tile at a time
  __shared__ float rsum[FOLD ? NW : 1][FOLD ? R : 1], rsq[FOLD ? NW : 1][FOLD ? R : 1];
  __shared__ float mu[FOLD ? R : 1], rs[FOLD ? R : 1];
  const int nt = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ksteps = p.K / 32;
  const int niter = (ksteps - w + NW - 1) / NW;  // this wave's k-steps: w + NW*i
  const u32x4_t* Wt = p.w + (int64_t)nt * ksteps * 64 + lane;
  const int c16 = lane & 15, q = lane >> 4;
  const uint16_t* A = p.a;

  u32x4_t wa[kU] = {}, wb[kU] = {};  // zero-initialised: see decode_gemm_kernel
  auto wload = [&](u32x4_t (&dst)[kU], int i0) {
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + u < niter) dst[u] = ITTS_WLOAD(Wt + (int64_t)(w + NW * (i0 + u)) * 64);
  };
  const bool straight = niter == kNI && kU >= kNI;  // wave-uniform
  f32x4_t acc[2 * MT];
  float ssum[2 * MT], ssq[2 * MT];  // FOLD: sums of the rows this lane holds (16-row half h: c16 + 16h)
#pragma unroll
  for (int t = 0; t < 2 * MT; ++t) {
    acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    ssum[t] = ssq[t] = 0.f;
  }
  auto aload = [&](bf16x8_t (&dst)[2 * MT], int kstep) __attribute__((always_inline)) {
    const int64_t col = 32 * (w + NW * kstep) + 8 * q;
#pragma unroll
    for (int t = 0; t < 2 * MT; ++t) dst[t] = *reinterpret_cast<const bf16x8_t*>(A + (int64_t)(16 * t + c16) * p.lda + col);
  };
  auto step = [&](const bf16x8_t (&av)[2 * MT], const u32x4_t& wsrc) __attribute__((always_inline)) {
    const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(&wsrc);
#pragma unroll
    for (int t = 0; t < 2 * MT; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[t], bfr, acc[t], 0, 0, 0);
      if constexpr (FOLD) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = (float)av[t][e];
          ssum[t] += v;
          ssq[t] = fmaf(v, v, ssq[t]);
        }
      }
    }
  };
  auto compute = [&](const u32x4_t (&src)[kU], int i0) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (i0 + u >= niter) continue;
      bf16x8_t av[2 * MT];
      aload(av, i0 + u);
      step(av, src[u]);
    }
  };
  if (straight) {
    // K = 32 kNI NW (1024 at NW = 8): straight-line k-steps, k-step u + 1's A fragments requested before k-step
    // u's MFMAs (requested right before them, every k-step paid a full L2 round trip: 12.5 us per 128-row launch
    // in the C5 chain, profiles/kernel_stats_c5_r06r.txt); the same values in the same order: bit-identical
    u32x4_t wf[kNI];  // the wave's kNI weight fragments, loaded unconditionally
#pragma unroll
    for (int u = 0; u < kNI; ++u) wf[u] = ITTS_WLOAD(Wt + (int64_t)(w + NW * u) * 64);
    bf16x8_t a0[2 * MT], a1[2 * MT];
    aload(a0, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kNI; ++u) {
      if (u + 1 < kNI) aload((u & 1) ? a0 : a1, u + 1);
      step((u & 1) ? a1 : a0, wf[u]);
    }
  } else {
  wload(wa, 0);
  for (int i0 = 0; i0 < niter; i0 += 2 * kU) {
    if (i0 + kU < niter) wload(wb, i0 + kU);
    compute(wa, i0);
    if (i0 + 2 * kU < niter) wload(wa, i0 + 2 * kU);
    if (i0 + kU < niter) compute(wb, i0 + kU);
  }
  }
  if constexpr (FOLD) {
#pragma unroll
    for (int t = 0; t < 2 * MT; ++t) {
      float a = ssum[t], b = ssq[t];
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b += __shfl_xor(b, 16, 64);
      b += __shfl_xor(b, 32, 64);
      if (q == 0) {
        rsum[w][16 * t + c16] = a;
        rsq[w][16 * t + c16] = b;
      }
    }
  }
  if constexpr (FOLD) {
    __syncthreads();
    for (int r = threadIdx.x; r < R; r += 64 * NW) {
      float S = 0.f, Q = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) {
        S += rsum[ww][r];
        Q += rsq[ww][r];
      }
      fold_mu_rs(S, Q, 1.0f / p.K, p.eps, mu[r], rs[r]);
    }
    __syncthreads();
  }
  // R rows x 16 columns, one 32-row tile at a time through red; C/D layout of 16x16x32:
  // row = 4*(lane>>4) + reg, col = lane&15
#pragma unroll
  for (int tile = 0; tile < MT; ++tile) {
    if (tile > 0) __syncthreads();  // previous tile's reads done
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][4 * hf + r][lane] = acc[2 * tile + hf][r];
    __syncthreads();
    for (int o = threadIdx.x; o < 512; o += 64 * NW) {
      const int e = o >> 6, l = o & 63;  // e = 4 * (16-row half) + reg
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) v += red[ww][e][l];
      const int row = 32 * tile + 16 * (e >> 2) + 4 * (l >> 4) + (e & 3);
      const int n = nt * 16 + (l & 15);
      if (row >= p.M || n >= p.N) continue;
      if constexpr (FOLD) v = fold_apply(v, rs[row], mu[row], p.u[n], p.c ? p.c[n] : 0.f);
      else if (p.c) v += p.c[n];
      if constexpr (EPI == 1) {
        float* X = reinterpret_cast<float*>(p.y) + (int64_t)row * p.ldy + n;
        const float xv = *X + v;
        st_out(X, xv);
        st_out(p.xh + (int64_t)row * p.ldxh + n, f2bf(xv));
      } else {
        if (p.gelu) v = gelu_tanh_nc(v);
        St<OutT>::st(reinterpret_cast<OutT*>(p.y) + (int64_t)row * p.ldy + n, v);
      }
    }
  }
}

template <int NW, bool FOLD, int EPI, typename OutT>
void launch_dg16x(const Dg16xArgs& a, hipStream_t s) {
  // up to 4 row tiles (128 rows) per launch share the weight stream; more rows: further launches
  for (int t = 0; t * 32 < a.M; t += 4) {
    Dg16xArgs b = a;
    const int rows = a.M - 32 * t < 128 ? a.M - 32 * t : 128;
    b.M = rows;
    b.a = a.a + (int64_t)t * 32 * a.lda;
    if (EPI == 1) {
      b.y = reinterpret_cast<float*>(a.y) + (int64_t)t * 32 * a.ldy;
      b.xh = a.xh + (int64_t)t * 32 * a.ldxh;
    } else {
      b.y = reinterpret_cast<OutT*>(a.y) + (int64_t)t * 32 * a.ldy;
    }
    const dim3 grid((a.N + 15) / 16), block(64 * NW);
    switch ((rows + 31) / 32) {
      case 1: hipLaunchKernelGGL((decode_gemm16x_kernel<NW, FOLD, EPI, OutT, 1>), grid, block, 0, s, b); break;
      case 2: hipLaunchKernelGGL((decode_gemm16x_kernel<NW, FOLD, EPI, OutT, 2>), grid, block, 0, s, b); break;
      case 3: hipLaunchKernelGGL((decode_gemm16x_kernel<NW, FOLD, EPI, OutT, 3>), grid, block, 0, s, b); break;
      default: hipLaunchKernelGGL((decode_gemm16x_kernel<NW, FOLD, EPI, OutT, 4>), grid, block, 0, s, b); break;
    }
  }
}

}  // namespace

// lnmode: 0 = A is bf16; 1 = A = LN(X f32) with (g1,b1); 2 = A = LN(LN(X)) with (g1,b1) then (g2,b2).
// epi: 0 = store act(acc+bias) as out_dtype; 1 = f32 Y += acc + bias; 2 = split-K partial products
// (f32, no bias) for split s at Y + s*split_stride + row*ldy + n, K split over ksplit workgroups per
// column tile -- reduced (with bias + residual + the next LayerNorm) by itts_residual_reduce_ln.
// M > 32 runs ceil(M/32) row tiles.
extern "C" int itts_decode_gemm(const void* a, int64_t lda, const void* w_packed, int K, int N, int M,
                                const float* bias, const float* g1, const float* b1, const float* g2, const float* b2,
                                int lnmode, int gelu, int epi, void* y, int64_t ldy, int out_dtype,
                                int64_t split_stride, int ksplit, void* stream) {
  const char* fn = "itts_decode_gemm";
  ITTS_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 16 == 0, fn, "bad sizes");
  if (M == 0) return 0;
  ITTS_REQUIRE(a && w_packed && y, fn, "null pointer");
  ITTS_REQUIRE(lnmode == 0 || (g1 && b1 && (lnmode == 1 || (g2 && b2))), fn, "LayerNorm params missing");
  ITTS_REQUIRE(lnmode == 0 || K == 1024 || K == 256 || K == 512, fn, "LN prologue supports K in {256, 512, 1024}");
  ITTS_REQUIRE(epi >= 0 && epi <= 2, fn, "epi must be 0, 1 or 2");
  ITTS_REQUIRE(epi == 0 || out_dtype == ITTS_F32, fn, "residual / partial epilogues are f32");
  ITTS_REQUIRE(lnmode != 2 || epi == 0, fn, "double-LN prologue only with the store epilogue");
  ITTS_REQUIRE(ksplit >= 1 && (K / 16) % ksplit == 0, fn, "K/16 must be a multiple of ksplit");
  ITTS_REQUIRE(ksplit == 1 || epi == 2, fn, "ksplit > 1 requires epi 2");
  ITTS_REQUIRE(epi != 2 || (lnmode == 0 && split_stride >= (int64_t)M * ldy), fn, "bad split-K partial layout");
  DgArgs d{a, lda, static_cast<const u32x4_t*>(w_packed), K, N, M, bias, g1, b1, g2, b2, gelu, y, ldy, split_stride};
  const int tiles = (M + 31) / 32;
  hipStream_t s = itts::as_stream(stream);
#define DG_LN(NWV, LNM, EPIV, OT)                                            \
  do {                                                                       \
    if (K == 1024) launch_dg<NWV, LNM, EPIV, 1024, OT>(d, tiles, 1, s);      \
    else if (K == 512) launch_dg<NWV, LNM, EPIV, 512, OT>(d, tiles, 1, s);   \
    else launch_dg<NWV, LNM, EPIV, 256, OT>(d, tiles, 1, s);                 \
  } while (0)
  if (lnmode == 0) {
    if (epi == 2) {
      launch_dg<8, 0, 2, 256, float>(d, tiles, ksplit, s);
    } else if (epi == 1) {
      launch_dg<8, 0, 1, 256, float>(d, tiles, 1, s);
    } else if (out_dtype == ITTS_BF16) {
      launch_dg<8, 0, 0, 256, uint16_t>(d, tiles, 1, s);
    } else {
      launch_dg<8, 0, 0, 256, float>(d, tiles, 1, s);
    }
  } else if (lnmode == 1) {
    if (epi == 1) DG_LN(8, 1, 1, float);
    else if (out_dtype == ITTS_BF16) DG_LN(8, 1, 0, uint16_t);
    else DG_LN(8, 1, 0, float);
  } else {
    if (out_dtype == ITTS_BF16) DG_LN(8, 2, 0, uint16_t);
    else DG_LN(8, 2, 0, float);
  }
#undef DG_LN
  return itts::check_launch(fn);
}

// 16-column tiles, store epilogue: y = act(a @ W^T + bias) as out_dtype (act = gelu_tanh if gelu);
// weights from pack_skinny16; a: bf16 rows padded to whole 32-row tiles.
extern "C" int itts_decode_gemm16(const void* a, int64_t lda, const void* w_packed16, int K, int N, int M,
                                  const float* bias, int gelu, void* y, int64_t ldy, int out_dtype, void* stream) {
  const char* fn = "itts_decode_gemm16";
  ITTS_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 32 == 0, fn, "bad sizes (K must be a multiple of 32)");
  if (M == 0) return 0;
  ITTS_REQUIRE(a && w_packed16 && y, fn, "null pointer");
  ITTS_REQUIRE(lda % 8 == 0 && (reinterpret_cast<uintptr_t>(a) & 15) == 0, fn, "A rows must be 16-B aligned");
  DgArgs d{a, lda, static_cast<const u32x4_t*>(w_packed16), K, N, M, bias, nullptr, nullptr, nullptr, nullptr,
           gelu, y, ldy, 0};
  const int tiles = (M + 31) / 32;
  hipStream_t s = itts::as_stream(stream);
  if (out_dtype == ITTS_BF16) launch_dg16<8, uint16_t>(d, tiles, s);
  else launch_dg16<8, float>(d, tiles, s);
  return itts::check_launch(fn);
}

// 16-column tiles (pack_skinny16 weights), A = bf16 rows padded to whole 32-row tiles:
//   fold (u != null): y = rstd * (a @ W'^T - mean * u) + c   (LayerNorm of a folded in, eps)
//   else:             y = a @ W^T + c
//   epi 0: store act(y) as out_dtype (act = gelu_tanh if gelu)
//   epi 1: residual, y is the f32 stream x [M][ldy]: x += y in place, xh[M][ldxh] = bf16(x)
// nwaves: 8 or 16 waves per workgroup.  A holds whole 32-row tiles (rows >= M are read, never stored);
// up to 128 rows share one weight stream.
extern "C" int itts_decode_gemm16x(const void* a, int64_t lda, const void* w_packed16, int K, int N, int M,
                                   const float* c, const float* u, float eps, int gelu, int epi, void* y, int64_t ldy,
                                   int out_dtype, void* xh, int64_t ldxh, int nwaves, void* stream) {
  const char* fn = "itts_decode_gemm16x";
  ITTS_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 32 == 0, fn, "bad sizes (K must be a multiple of 32)");
  if (M == 0) return 0;
  ITTS_REQUIRE(a && w_packed16 && y, fn, "null pointer");
  ITTS_REQUIRE(lda % 8 == 0 && (reinterpret_cast<uintptr_t>(a) & 15) == 0, fn, "A rows must be 16-B aligned");
  ITTS_REQUIRE(epi == 0 || epi == 1, fn, "epi must be 0 or 1");
  ITTS_REQUIRE(epi == 0 || (xh && out_dtype == ITTS_F32 && !gelu && !u), fn,
               "residual epilogue: f32 stream, bf16 copy, no activation, no fold");
  ITTS_REQUIRE(nwaves == 8 || nwaves == 16, fn, "nwaves must be 8 or 16");
  ITTS_REQUIRE(out_dtype == ITTS_F32 || out_dtype == ITTS_BF16, fn, "unsupported dtype");
  Dg16xArgs d{static_cast<const uint16_t*>(a), lda, static_cast<const u32x4_t*>(w_packed16), K, N, M, c, u, eps, gelu,
              y, ldy, static_cast<uint16_t*>(xh), ldxh};
  hipStream_t s = itts::as_stream(stream);
#define DGX(NWV)                                                                            \
  do {                                                                                      \
    if (epi == 1) launch_dg16x<NWV, false, 1, float>(d, s);                                 \
    else if (u && out_dtype == ITTS_BF16) launch_dg16x<NWV, true, 0, uint16_t>(d, s);       \
    else if (u) launch_dg16x<NWV, true, 0, float>(d, s);                                    \
    else if (out_dtype == ITTS_BF16) launch_dg16x<NWV, false, 0, uint16_t>(d, s);           \
    else launch_dg16x<NWV, false, 0, float>(d, s);                                          \
  } while (0)
  if (nwaves == 16) DGX(16);
  else DGX(8);
#undef DGX
  return itts::check_launch(fn);
}
