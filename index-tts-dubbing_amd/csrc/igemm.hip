// Implicit-GEMM on MFMA for gfx950 (igemm256: v_mfma_f32_16x16x32_bf16; the register-staged igemm_kernel: 32x32x16): one kernel serves
//   * BigVGAN Conv1d (dilated, zero "same" padding)      BigVGAN/models.py:24-42, utils.py:59-60
//   * BigVGAN ConvTranspose1d as u polyphase convs        BigVGAN/models.py:155-161 (torch ConvTranspose1d)
//   * conv_pre                                             BigVGAN/models.py:149,224
//   * GPT-2 projection GEMMs for prefill + latent pass     HF:modeling_gpt2.py Conv1D = addmm(b, x, W)
//
//   Y[b, q*ymul + yoff, n] = epi( sum_j sum_c  X[b, q + tap_off[j], c] * Wp[j][n][c] )
// with X rows outside [0, len_b) reading as zero (per-utterance zero padding, so ragged batches are
// exact).  Layout is channel-last: X [B][Tmax][ldx] bf16, Y [B][Tout][ldy] (bf16 or f32).
// Wp is prepacked on the host: [ntaps][co_pad][ci_pad] bf16, zero padded.
//
// Epilogue: v = acc + bias[n] + bias_b[b][n]; gelu 1: v = gelu_tanh(v), 2: v = silu(v); v = alpha*(v + r1 + r2)
// (r1/r2 residual tensors with Y's layout and dtype; r1 may alias Y).
//
// Tiling: one wave per WM x WN sub-tile of the TM x TN block tile, K step KC (channels of one tap) staged
// through double-buffered LDS (row pitch padded by 16 B -> conflict-free ds_read_b128 fragments),
// with a 3-deep register ring (K-step it+2's global loads in flight while step it computes).
// Tiles are remapped XCD-aware (output-channel tiles of one row tile run together on one XCD).
// WIN (convs of >= 3 taps, tap span <= 64 rows): K steps run channel chunk outer, tap inner, and the A
// operand of a chunk is ONE input window of TM + span rows staged once for all its taps (tap j reads
// it at row offset off_j - min_off), instead of TM rows per tap: an 11-tap conv moves 178 input rows
// per chunk through L2 -> LDS instead of 1408.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

constexpr int kMaxTaps = 16;
#ifndef ITTS_IG_MFMA16  // igemm256: 16x16x32 MFMA blocks (-DITTS_IG_MFMA16=0: 32x32x16, A/B build)
#define ITTS_IG_MFMA16 1  // latent GEMMs +3-8 %, vocoder convs within noise (profiles/mfma16_ab_r03.txt)
#endif
constexpr int kWinSpan = 64;  // WIN: max tap span (rows)
#ifndef ITTS_IG_WIN_MINTAPS  // fewest taps that take the window form
#define ITTS_IG_WIN_MINTAPS 3
#endif

struct IgArgs {
  const uint16_t* x;
  const uint16_t* w;
  const float* bias;
  const float* bias_b;
  const void* r1;
  const void* r2;
  void* y;
  const int32_t* lens;
  int B, Tmax, Cin, Cout, ci_pad, co_pad, ntaps;
  int64_t sxb, ldx, syb, ldy;
  int64_t wsb;  // weight stride between batches (0: shared; split-K chunks: one packed chunk each)
  int ymul, yoff;
  float alpha;
  int gelu;
  int min_off, span;  // WIN: smallest tap offset, window rows beyond TM
  int tap_off[kMaxTaps];
};

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
}

template <int TM, int TN, int WM, int WN, int KC, bool VEC, typename OutT, bool WIN = false>
__global__ __launch_bounds__(64 * (TM / WM) * (TN / WN)) void igemm_kernel(IgArgs p) {
  constexpr int NT = 64 * (TM / WM) * (TN / WN);  // threads (one wave per WM x WN sub-tile)
  constexpr int PITCH = KC * 2 + 16;            // bytes per LDS row
  constexpr int AR = WIN ? TM + kWinSpan : TM;  // A rows staged per buffer
  constexpr int A_BYTES = AR * PITCH, B_BYTES = TN * PITCH;
  constexpr int VPR = KC / 8;                   // 16-B vectors per row
  constexpr int A_TOT = AR * VPR, B_TOT = TN * VPR;  // 16-B vectors per tile (A: upper bound)
  constexpr int A_VEC = (A_TOT + NT - 1) / NT, B_VEC = (B_TOT + NT - 1) / NT;
  constexpr int FM = WM / 32, FN = WN / 32;     // MFMA tiles per wave
  constexpr int WAVES_N = TN / WN;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  // XCD-aware tile order (guide T1): dispatch places block p on XCD p % 8, so a bijective remap
  // gives every XCD a contiguous run of logical tiles, ordered N-tile fastest -- the blocks that share
  // an input window (same rows, different output channels) run together on one XCD and hit its L2.
  const int ntn = (p.Cout + TN - 1) / TN, ntm = (p.Tmax + TM - 1) / TM;
  const int nblk = ntn * ntm * p.B;
  const int pid = blockIdx.x, xcd = pid % 8, qn = nblk / 8, rn = nblk % 8;
  const int lid = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + pid / 8;
  const int b = lid / (ntn * ntm);
  const int len = p.lens ? p.lens[b] : p.Tmax;
  const int q0 = ((lid / ntn) % ntm) * TM;
  if (q0 >= len) return;
  const int n0 = (lid % ntn) * TN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const uint16_t* X = p.x + (int64_t)b * p.sxb;
  const int nchunks = p.ci_pad / KC;
  const int kiters = p.ntaps * nchunks;

  // 3-deep register ring: the global loads of K-step it+2 are issued while step it computes, so
  // every load has two steps of MFMAs (plus the other block's) to arrive before its LDS write.
  // WIN: the ring carries B only; a chunk's window goes through one register set (loaded at the
  // step two before the chunk's first, written at the step before) into ONE LDS window buffer.
  struct Stage {
    u32x4_t a[WIN ? 1 : A_VEC], b[B_VEC];
  };
  Stage S0, S1, S2;
  u32x4_t wa[WIN ? A_VEC : 1];
  // K step it -> (tap j, channel chunk c0): tap outer (per-tap A tiles) or, WIN, chunk outer
  auto kstep = [&](int it, int& j, int& c0) {
    if (WIN) {
      const int c = it / p.ntaps;
      j = it - c * p.ntaps;
      c0 = c * KC;
    } else {
      j = it / nchunks;
      c0 = (it - j * nchunks) * KC;
    }
  };
  const int a_rows = WIN ? TM + p.span : TM;
  auto aload = [&](u32x4_t* dst, int toff, int c0) {
#pragma unroll
    for (int i = 0; i < A_VEC; ++i) {
      const int v = tid + NT * i, row = v / VPR, cv = (v % VPR) * 8;
      const int t = q0 + row + toff, c = c0 + cv;
      u32x4_t val = {0u, 0u, 0u, 0u};
      if (row < a_rows && v < A_TOT && t >= 0 && t < len) {
        const uint16_t* src = X + (int64_t)t * p.ldx + c;
        if (VEC) {
          if (c < p.Cin) val = *reinterpret_cast<const u32x4_t*>(src);
        } else {
          uint32_t e[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) e[u] = (c + u < p.Cin) ? src[u] : 0u;
          val = u32x4_t{e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16)};
        }
      }
      dst[i] = val;
    }
  };
  auto gload = [&](int it, Stage& r) {
    int j, c0;
    kstep(it, j, c0);
    if (WIN) {
      if (j == 0) aload(wa, p.min_off, c0);
    } else {
      aload(r.a, p.tap_off[j], c0);
    }
    const uint16_t* Wj = p.w + b * p.wsb + ((int64_t)j * p.co_pad + n0) * p.ci_pad + c0;
#pragma unroll
    for (int i = 0; i < B_VEC; ++i) {
      const int v = tid + NT * i, row = v / VPR, cv = (v % VPR) * 8;
      if (v < B_TOT) r.b[i] = *reinterpret_cast<const u32x4_t*>(Wj + (int64_t)row * p.ci_pad + cv);
    }
  };
  // LDS: per-tap mode [A 0][B 0][A 1][B 1]; WIN [window][B 0][B 1]
  auto abase = [&](int it) -> unsigned char* {
    return WIN ? smem : smem + (it & 1) * (A_BYTES + B_BYTES);
  };
  auto bbase = [&](int it) -> unsigned char* {
    return WIN ? smem + A_BYTES + (it & 1) * B_BYTES : smem + (it & 1) * (A_BYTES + B_BYTES) + A_BYTES;
  };
  auto swrite = [&](int it, const Stage& r) {
    unsigned char* As = abase(it);
    unsigned char* Bs = bbase(it);
    if (!WIN || it % p.ntaps == 0) {
      const u32x4_t* src = WIN ? wa : r.a;
#pragma unroll
      for (int i = 0; i < A_VEC; ++i) {
        const int v = tid + NT * i, row = v / VPR, cv = v % VPR;
        if (v < A_TOT && row < a_rows) *reinterpret_cast<u32x4_t*>(As + row * PITCH + cv * 16) = src[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_VEC; ++i) {
      const int v = tid + NT * i, row = v / VPR, cv = v % VPR;
      if (v < B_TOT) *reinterpret_cast<u32x4_t*>(Bs + row * PITCH + cv * 16) = r.b[i];
    }
  };

  f32x16_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  auto compute = [&](int it) {
    const unsigned char* As = abase(it);
    const unsigned char* Bs = bbase(it);
    int arow = 0;  // WIN: this tap's first window row
    if (WIN) {
      int j, c0;
      kstep(it, j, c0);
      arow = p.tap_off[j] - p.min_off;
    }
#pragma unroll
    for (int ks = 0; ks < KC / 16; ++ks) {
      bf16x8_t af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(As + (arow + wm + 32 * i + r32) * PITCH + ks * 32 + h * 16);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + (wn + 32 * j + r32) * PITCH + ks * 32 + h * 16);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // step it: issue loads for it+2 into `ld`, compute LDS buffer it&1, write stage it+1 (`wr`) into
  // the other buffer (last read in step it-1, fenced by that step's barrier), barrier
  auto step = [&](int it, Stage& ld, const Stage& wr) {
    if (it + 2 < kiters) gload(it + 2, ld);
    compute(it);
    if (it + 1 < kiters) {
      if (WIN && (it + 1) % p.ntaps == 0) __syncthreads();  // every wave is done with the window
      swrite(it + 1, wr);
      __syncthreads();
    }
  };
  gload(0, S0);
  if (kiters > 1) gload(1, S1);
  swrite(0, S0);
  __syncthreads();
  for (int it = 0; it < kiters; it += 3) {
    step(it, S2, S1);
    if (it + 1 < kiters) step(it + 1, S0, S2);
    if (it + 2 < kiters) step(it + 2, S1, S0);
  }

  // epilogue: lane holds column n = wn + 32j + (lane&31); rows (r&3) + 8(r>>2) + 4h
  OutT* Y = reinterpret_cast<OutT*>(p.y) + (int64_t)b * p.syb;
  const OutT* R1 = reinterpret_cast<const OutT*>(p.r1);
  const OutT* R2 = reinterpret_cast<const OutT*>(p.r2);
  if (R1) R1 += (int64_t)b * p.syb;
  if (R2) R2 += (int64_t)b * p.syb;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn + 32 * j + r32;
    if (n >= p.Cout) continue;
    float bn = p.bias ? p.bias[n] : 0.f;
    if (p.bias_b) bn += p.bias_b[(int64_t)b * p.Cout + n];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = q0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (q >= len) continue;
        const int64_t off = (int64_t)(q * p.ymul + p.yoff) * p.ldy + n;
        float v = acc[i][j][r] + bn;
        if (p.gelu) v = p.gelu == 2 ? v / (1.f + __expf(-v)) : gelu_tanh(v);
        if (R1) v += St<OutT>::ld(R1 + off);
        if (R2) v += St<OutT>::ld(R2 + off);
        St<OutT>::st(Y + off, p.alpha * v);
      }
    }
  }
}

// ---- 256-row tiles staged by LDS-DMA (global_load_lds_dwordx4) ----------------------------------
// For the wide layers (Cin >= 128 channels, Cout a multiple of 128, >= 256): the GPT latent-pass /
// prefill GEMMs (M = thousands of rows, K 1024 / 4096, N 1024 .. 4096), conv_pre and the C = 768 /
// 384 generator stages.  One 512-thread workgroup per 256 x TN output tile, 8 waves (WAVES_M x
// WAVES_N) of 32x32x16 MFMAs, K steps of 32 channels of one tap.  Each step's A (256 rows) and B (TN
// rows of the packed W^T) images land in LDS straight from global memory -- no register stage, no
// ds_write pass -- in a ring of 4 step images with 3 steps in flight: step it+3 is issued before step
// it's MFMAs, and a counted s_waitcnt vmcnt (2 steps may stay outstanding) + raw s_barrier retire step
// it+1 (a __syncthreads() would drain every DMA with vmcnt(0); MI355X guide §5 "Pipelining across
// barriers").  One 1 KiB DMA wave-instruction fills 16 rows of 64 B.
// LDS image: 64-B rows (32 bf16 channels), 16-B slot s of row r stored at slot s ^ ((r >> 2) & 3): the
// 16 rows of one ds_read_b128 lane group fall on 16 distinct bank quads; the DMA writes lane-linearly,
// so each lane loads the SOURCE slot that lands at its destination (the permutation is an involution).
// Rows outside [0, len) (zero "same" padding, ragged lengths), channels >= Cin and W rows >= co_pad
// load from a zero line.  Epilogue: per 32-row band the wave's accumulators go through LDS as f32
// rows, then 16-B row-contiguous reads / residual loads / stores (the scattered 2-B stores of the
// fragment layout were the kernel's tail).
__device__ __attribute__((aligned(256))) uint32_t g_zero_line[64];  // 256 zero bytes (module-initialised)

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <int TN, int WAVES_M, int WAVES_N, int BK, int NSLOT, typename OutT, bool WIN = false>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void igemm256_kernel(IgArgs p) {
  constexpr int NW = WAVES_M * WAVES_N;  // 8 waves of 128 x 64 (or 64 x 96 ...), or 4 of 128 x 128
  constexpr int TM = 256, ROWB = BK * 2, SPR = BK / 8, RPI = 1024 / ROWB;  // 16-B slots per row, rows per DMA
  constexpr int D = NSLOT - 1;  // K steps in flight ahead of the one computed
  constexpr int WM = TM / WAVES_M, WN = TN / WAVES_N, FM = WM / 32, FN = WN / 32;
  constexpr int A_BYTES = TM * ROWB, B_BYTES = TN * ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int A_INS = TM / RPI / NW, B_INS = TN / RPI / NW;  // DMA instructions per wave per K step
  constexpr int P = A_INS + B_INS;
  constexpr int EP = WN + 4;  // epilogue staging pitch (floats): rows r and r + 4 on other banks
  // WIN (convs of >= 3 taps): K steps run channel chunk outer, tap inner; a chunk's A operand is ONE
  // window of TM + kWinSpan input rows, in its own double buffer, and a K step moves only B.  The next
  // chunk's window is issued at the first step of a chunk, after that step's B, so it may stay in flight
  // across one barrier (counted vmcnt) and lands during the chunk's taps.
  constexpr int WROWS = TM + kWinSpan, W_BYTES = WROWS * ROWB, W_INS = WROWS / RPI / NW;
  static_assert((NW == 8 || NW == 4) && B_INS >= 1 && (BK == 32 || BK == 64) && D >= 1, "geometry");
  static_assert(A_INS * RPI * NW == TM && B_INS * RPI * NW == TN, "whole DMA instructions per wave");
  static_assert(!WIN || (NSLOT == 2 && WROWS % (RPI * NW) == 0), "window form: double-buffered B");
  static_assert(NW * 32 * EP * 4 <= (WIN ? 2 * (W_BYTES + B_BYTES) : NSLOT * STAGE), "epilogue staging fits");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // slot permutation of a row (an involution on the row's SPR slots): 16 consecutive rows of a fragment
  // read fall on 16 distinct bank quads
  auto swz = [](int row) { return SPR == 4 ? (row >> 2) & 3 : (row >> 1) & 7; };

  const int ntn = (p.Cout + TN - 1) / TN, ntm = (p.Tmax + TM - 1) / TM;
  const int nblk = ntn * ntm * p.B;
  const int pid = blockIdx.x, xcd = pid % 8, qn = nblk / 8, rn = nblk % 8;
  const int lid = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + pid / 8;
  const int b = lid / (ntn * ntm);
  const int len = p.lens ? p.lens[b] : p.Tmax;
  const int q0 = ((lid / ntn) % ntm) * TM;
  if (q0 >= len) return;
  const int n0 = (lid % ntn) * TN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const uint16_t* X = p.x + (int64_t)b * p.sxb;
  const int nchunks = p.ci_pad / BK;
  const int kiters = p.ntaps * nchunks;
  typedef __attribute__((address_space(3))) void lds_void;

  // DMA of K step it into ring slot it % NSLOT: lane l of an instruction covers row R + l / SPR,
  // physical slot l % SPR = logical slot (l % SPR) ^ swz(row)
  const int lr = lane / SPR, ls = lane % SPR;
  // WIN: [window 0][window 1][B 0][B 1]
  auto issue_win = [&](int c) {
    const int c0 = c * BK;
    unsigned char* Ws = smem + (c & 1) * W_BYTES;
#pragma unroll
    for (int i = 0; i < W_INS; ++i) {
      const int R = (wave * W_INS + i) * RPI, row = R + lr;
      const int s = ls ^ swz(row);
      const int t = q0 + row + p.min_off, cc = c0 + 8 * s;
      const void* src = (t >= 0 && t < len && cc < p.Cin) ? static_cast<const void*>(X + (int64_t)t * p.ldx + cc)
                                                          : static_cast<const void*>(g_zero_line);
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(Ws + R * ROWB), 16, 0, 0);
    }
  };
  auto issue_b = [&](int it) {
    const int c = it / p.ntaps, j = it - c * p.ntaps;
    unsigned char* Bs = smem + 2 * W_BYTES + (it & 1) * B_BYTES;
    const uint16_t* Wj = p.w + b * p.wsb + (int64_t)j * p.co_pad * p.ci_pad + c * BK;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int R = (wave * B_INS + i) * RPI, row = R + lr;
      const int s = ls ^ swz(row);
      const int n = n0 + row;
      const void* src = n < p.co_pad ? static_cast<const void*>(Wj + (int64_t)n * p.ci_pad + 8 * s)
                                     : static_cast<const void*>(g_zero_line);
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(Bs + R * ROWB), 16, 0, 0);
    }
  };
  auto issue = [&](int it) {
    const int j = it / nchunks, c0 = (it - j * nchunks) * BK;
    const int toff = p.tap_off[j];
    unsigned char* As = smem + (it % NSLOT) * STAGE;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      const int R = (wave * A_INS + i) * RPI, row = R + lr;
      const int s = ls ^ swz(row);
      const int t = q0 + row + toff, c = c0 + 8 * s;
      const void* src = (t >= 0 && t < len && c < p.Cin) ? static_cast<const void*>(X + (int64_t)t * p.ldx + c)
                                                         : static_cast<const void*>(g_zero_line);
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(As + R * ROWB), 16, 0, 0);
    }
    unsigned char* Bs = As + A_BYTES;
    const uint16_t* Wj = p.w + b * p.wsb + (int64_t)j * p.co_pad * p.ci_pad + c0;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int R = (wave * B_INS + i) * RPI, row = R + lr;
      const int s = ls ^ swz(row);
      const int n = n0 + row;
      const void* src = n < p.co_pad ? static_cast<const void*>(Wj + (int64_t)n * p.ci_pad + 8 * s)
                                     : static_cast<const void*>(g_zero_line);
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(Bs + R * ROWB), 16, 0, 0);
    }
  };
  // retire step it+1: later steps (up to D - 1 of them) may stay in flight
  auto retire_next = [&](int it) {
    const int later = min(it + D, kiters - 1) - (it + 1);
    if (later >= 2) wait_vm<2 * P>();
    else if (later == 1) wait_vm<P>();
    else wait_vm<0>();
  };

  // MFMA16 (ITTS_IG_MFMA16, BK = 64): v_mfma_f32_16x16x32_bf16 on 16 x 16 blocks instead of 32 x 32 x 16
  // (the same LDS fragment bytes per K step; MI355X_MICROARCH.md measures the 16x16x32 form at
  // 1.12-1.15x the 32x32x16 FLOP rate with LDS operands)
  constexpr bool M16 = ITTS_IG_MFMA16 && BK == 64;
  constexpr int AM = M16 ? 2 * FM : FM, AN = M16 ? 2 * FN : FN;
  typedef typename std::conditional<M16, f32x4_t, f32x16_t>::type acc_t;
  constexpr int AR = M16 ? 4 : 16;
  acc_t acc[AM][AN];
#pragma unroll
  for (int i = 0; i < AM; ++i)
#pragma unroll
    for (int j = 0; j < AN; ++j)
#pragma unroll
      for (int r = 0; r < AR; ++r) acc[i][j][r] = 0.f;
  const int r32 = lane & 31, h = lane >> 5;
  const int r16 = lane & 15, qg = lane >> 4;
  auto compute = [&](int it) {
    const unsigned char* As = smem + (it % NSLOT) * STAGE;
    const unsigned char* Bs = As + A_BYTES;
    int arow = 0;  // WIN: this tap's first window row
    if constexpr (WIN) {
      const int c = it / p.ntaps, j = it - c * p.ntaps;
      As = smem + (c & 1) * W_BYTES;
      Bs = smem + 2 * W_BYTES + (it & 1) * B_BYTES;
      arow = p.tap_off[j] - p.min_off;
    }
    if constexpr (M16) {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8_t af[AM], bfr[AN];
#pragma unroll
        for (int i = 0; i < AM; ++i) {
          const int row = arow + wm + 16 * i + r16;
          af[i] = *reinterpret_cast<const bf16x8_t*>(As + row * ROWB + (((4 * ks + qg) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int j = 0; j < AN; ++j) {
          const int row = wn + 16 * j + r16;
          bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + row * ROWB + (((4 * ks + qg) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
          for (int j = 0; j < AN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8_t af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = arow + wm + 32 * i + r32;
          af[i] = *reinterpret_cast<const bf16x8_t*>(As + row * ROWB + (((2 * ks + h) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn + 32 * j + r32;
          bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + row * ROWB + (((2 * ks + h) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  if constexpr (WIN) {
    issue_win(0);
    issue_b(0);
    wait_vm<0>();
    lds_barrier();
    for (int it = 0; it < kiters; ++it) {
      const int c = it / p.ntaps, j = it - c * p.ntaps;
      const bool nextwin = j == 0 && (c + 1) * BK < p.ci_pad;
      if (it + 1 < kiters) issue_b(it + 1);  // B slot (it + 1) & 1 was last read in step it - 1
      if (nextwin) issue_win(c + 1);          // window slot (c + 1) & 1 was last read in chunk c - 1
      compute(it);
      if (nextwin) wait_vm<W_INS>();  // B(it + 1) retired; the window stays in flight one more step
      else wait_vm<0>();
      lds_barrier();
    }
  } else {
    // prologue: steps 0 .. D-1 in flight, step 0 retired
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k < kiters) issue(k);
    retire_next(-1);
    lds_barrier();
    for (int it = 0; it < kiters; ++it) {
      // slot (it + D) % NSLOT was last read in step it - 1, which every wave finished before the last barrier
      if (it + D < kiters) issue(it + D);
      compute(it);
      retire_next(it);
      lds_barrier();
    }
  }

  // ---- epilogue: per 32-row band, f32 rows through this wave's LDS staging, 16-B row accesses
  float* stg = reinterpret_cast<float*>(smem) + wave * 32 * EP;
  OutT* Y = reinterpret_cast<OutT*>(p.y) + (int64_t)b * p.syb;
  const OutT* R1 = reinterpret_cast<const OutT*>(p.r1);
  const OutT* R2 = reinterpret_cast<const OutT*>(p.r2);
  if (R1) R1 += (int64_t)b * p.syb;
  if (R2) R2 += (int64_t)b * p.syb;
  float bn[AN];
#pragma unroll
  for (int j = 0; j < AN; ++j) {
    const int n = n0 + wn + (M16 ? 16 * j + r16 : 32 * j + r32);
    bn[j] = 0.f;
    if (n < p.Cout) {
      if (p.bias) bn[j] = p.bias[n];
      if (p.bias_b) bn[j] += p.bias_b[(int64_t)b * p.Cout + n];
    }
  }
  constexpr int V = 16 / sizeof(OutT);  // outputs per 16-B store
  constexpr int CPR = WN / V;            // chunks per staged row
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    if constexpr (M16) {  // 32-row band i = 16-row blocks 2i, 2i+1; C/D: row 4*(lane>>4) + reg, col lane&15
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[2 * i + i2][j][r] + bn[j];
            if (p.gelu) v = p.gelu == 2 ? v / (1.f + __expf(-v)) : gelu_tanh(v);
            stg[(16 * i2 + 4 * qg + r) * EP + 16 * j + r16] = v;
          }
    } else {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[i][j][r] + bn[j];
          if (p.gelu) v = p.gelu == 2 ? v / (1.f + __expf(-v)) : gelu_tanh(v);
          stg[((r & 3) + 8 * (r >> 2) + 4 * h) * EP + 32 * j + r32] = v;
        }
    }
#pragma unroll
    for (int k = 0; k < 32 * CPR / 64; ++k) {
      const int c = lane + 64 * k, row = c / CPR, col = (c - row * CPR) * V;
      const int q = q0 + wm + 32 * i + row, n = n0 + wn + col;
      float v[V];
#pragma unroll
      for (int e = 0; e < V; e += 4) {
        const f32x4_t f = *reinterpret_cast<const f32x4_t*>(stg + row * EP + col + e);
        v[e] = f[0];
        v[e + 1] = f[1];
        v[e + 2] = f[2];
        v[e + 3] = f[3];
      }
      if (q < len && n < p.Cout) {
        const int64_t off = (int64_t)(q * p.ymul + p.yoff) * p.ldy + n;
        if constexpr (sizeof(OutT) == 4) {
          if (R1) {
            const f32x4_t a = *reinterpret_cast<const f32x4_t*>(R1 + off);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += a[e];
          }
          if (R2) {
            const f32x4_t a = *reinterpret_cast<const f32x4_t*>(R2 + off);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += a[e];
          }
          *reinterpret_cast<f32x4_t*>(Y + off) =
              f32x4_t{p.alpha * v[0], p.alpha * v[1], p.alpha * v[2], p.alpha * v[3]};
        } else {
          if (R1) {
            const u32x4_t a = *reinterpret_cast<const u32x4_t*>(R1 + off);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] += __uint_as_float(a[e] << 16);
              v[2 * e + 1] += __uint_as_float(a[e] & 0xFFFF0000u);
            }
          }
          if (R2) {
            const u32x4_t a = *reinterpret_cast<const u32x4_t*>(R2 + off);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] += __uint_as_float(a[e] << 16);
              v[2 * e + 1] += __uint_as_float(a[e] & 0xFFFF0000u);
            }
          }
          u32x4_t o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = pack2bf(p.alpha * v[2 * e], p.alpha * v[2 * e + 1]);
          *reinterpret_cast<u32x4_t*>(Y + off) = o;
        }
      }
    }
  }
}

// ITTS_IGEMM_256=0 keeps the register-staged 128-row tiles for every layer (A/B measurements)
bool igemm256_enabled() {
  static const bool on = [] {
    const char* e = getenv("ITTS_IGEMM_256");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool igemm_win_enabled();

template <int TN, int WAVES_M, int WAVES_N, int BK, int NSLOT, typename OutT>
void launch256(const IgArgs& a, hipStream_t s) {
  dim3 grid(((a.Tmax + 255) / 256) * ((a.Cout + TN - 1) / TN) * a.B);
  if constexpr (NSLOT == 2 && BK == 64) {
    if (a.ntaps >= ITTS_IG_WIN_MINTAPS && a.span <= kWinSpan && igemm_win_enabled()) {
      const size_t lds = 2 * (size_t)(256 + kWinSpan + TN) * 2 * BK;
      hipLaunchKernelGGL((igemm256_kernel<TN, WAVES_M, WAVES_N, BK, 2, OutT, true>), grid, dim3(64 * WAVES_M * WAVES_N),
                         lds, s, a);
      return;
    }
  }
  const size_t lds = (size_t)NSLOT * (256 + TN) * 2 * BK;
  hipLaunchKernelGGL((igemm256_kernel<TN, WAVES_M, WAVES_N, BK, NSLOT, OutT>), grid, dim3(64 * WAVES_M * WAVES_N), lds,
                     s, a);
}
// tile variant (ITTS_IG256_VARIANT, A/B; profiles/ubench_igemm256_r03.txt): 0 = K steps of 32 (64-B rows),
// 4-slot ring, 3 steps in flight; 1 = 256 x 128, K steps of 64, 3 slots; 2 = 256 x 256 K steps of 64
// (whole 128-B lines), double-buffered, 256 x 128 of 32 for Cout % 256 != 0; 3 (default) = K steps of 64
// double-buffered for both tile widths.  Whole lines beat depth: latent GEMMs 600 / 872 / 771 / 487
// TF/s (v2) vs 573 / 787 / 721 / 461 (v0) vs 529 / 634 / 579 / 337 for the 128-row register-staged tile.
int ig256_variant() {
  static const int v = [] {
    const char* e = getenv("ITTS_IG256_VARIANT");
    return e ? atoi(e) : 3;
  }();
  return v;
}

// Cout = 192 on whole-width 256 x 192 tiles (read per launch: A/B in one process)
bool ig192_enabled() {
  const char* e = getenv("ITTS_IG192");
  return e ? atoi(e) != 0 : true;
}

// ITTS_IGEMM_WIN=0 keeps the per-tap A tiles (A/B measurements)
bool igemm_win_enabled() {
  static const bool on = [] {
    const char* e = getenv("ITTS_IGEMM_WIN");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int TM, int TN, int WM, int WN, int KC, typename OutT>
void launch_cfg(const IgArgs& a, bool vec, hipStream_t s) {
  dim3 grid(((a.Tmax + TM - 1) / TM) * ((a.Cout + TN - 1) / TN) * a.B);
  constexpr int NT = 64 * (TM / WM) * (TN / WN);
  // the window form for convs of >= 3 taps on the vectorised path (span within the staged rows);
  // with 128 x 128 / 128 x 64 tiles 3 taps were a wash (profiles/ubench_vocoder_r02_win.txt), with the
  // 256 x 64 Cout = 192 tile the window form wins there too (572 -> 532 us, profiles/igemm_ab_r02.txt)
  if (vec && a.ntaps >= ITTS_IG_WIN_MINTAPS && a.span <= kWinSpan && igemm_win_enabled()) {
    const size_t lds = (size_t)(TM + kWinSpan + 2 * TN) * (KC * 2 + 16);
    hipLaunchKernelGGL((igemm_kernel<TM, TN, WM, WN, KC, true, OutT, true>), grid, dim3(NT), lds, s, a);
    return;
  }
  const size_t lds = 2 * (size_t)(TM + TN) * (KC * 2 + 16);
  if (vec)
    hipLaunchKernelGGL((igemm_kernel<TM, TN, WM, WN, KC, true, OutT>), grid, dim3(NT), lds, s, a);
  else
    hipLaunchKernelGGL((igemm_kernel<TM, TN, WM, WN, KC, false, OutT>), grid, dim3(NT), lds, s, a);
}

// tile configs (TM, TN, WM, WN, KC) of the two vocoder-dominant shapes, overridable for A/B builds
#ifndef ITTS_IG_WIDE
#define ITTS_IG_WIDE 128, 128, 64, 32, 64
#endif
#ifndef ITTS_IG_C192
#define ITTS_IG_C192 128, 64, 32, 32, 64
#endif
#ifndef ITTS_IG_C192W  // Cout = 192 in the window form: 256 rows, 8 waves of 64 x 32
#define ITTS_IG_C192W 256, 64, 64, 32, 64
#endif
#ifndef ITTS_IG_WIDEW
#define ITTS_IG_WIDEW ITTS_IG_WIDE
#endif
template <typename OutT>
void dispatch_old(const IgArgs& a, bool vec, hipStream_t s);

template <typename OutT>
void dispatch(const IgArgs& a, bool vec, hipStream_t s) {
  const bool wide_n = a.Cout >= 128, wide_k = a.Cin >= 128;
  // wide layers: 8 waves per 128 x 128 tile (64 x 32 each) -- more waves per CU to hide the staging
  // latency than 4 waves of 64 x 64 (+25-30 % on the latent-pass GEMMs, profiles/ubench_igemm.py);
  // Cout = 192 (stage 2): 64-column tiles instead of a half-empty second 128-column tile; in the
  // window form 256 x 64 tiles of 8 x (64 x 32) (conv k = 11: 1247 -> 912 us, profiles/igemm_ab_r02.txt)
  const bool win = vec && a.ntaps >= ITTS_IG_WIN_MINTAPS && a.span <= kWinSpan && igemm_win_enabled();
  // 256-row LDS-DMA tiles: 16-B aligned rows, 64-channel chunks, Cout a multiple of 128 (>= 256)
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool g256 = vec && a.ci_pad % 32 == 0 && a.Cout >= 192 && a.Cout % 64 == 0 && a.ldx % 8 == 0 &&
                    a.sxb % 8 == 0 && al16(a.x) && a.ldy % 8 == 0 && a.syb % 8 == 0 && al16(a.y) &&
                    (!a.r1 || al16(a.r1)) && (!a.r2 || al16(a.r2)) && igemm256_enabled();
  if (g256) {
    const int v = ig256_variant();
    const bool k64 = a.ci_pad % 64 == 0;
    if (a.Cout % 128 != 0) {  // Cout = 192 (generator stage 2)
      // 256 x 192 tiles, 4 x 2 waves of 64 x 96 (ITTS_IG192=1) or 256 x 64 tiles of 64 x 32
      if (k64 && a.Cout == 192 && ig192_enabled()) launch256<192, 4, 2, 64, 2, OutT>(a, s);
      else if (k64) launch256<64, 4, 2, 64, 2, OutT>(a, s);
      else dispatch_old<OutT>(a, vec, s);
      return;
    }
    // 4 (A/B): 4 waves of 128 x 128 (half the LDS fragment reads per flop, one wave per SIMD, 256 VGPRs + 256
    // AGPRs): measured 30-40 % SLOWER on every latent GEMM (c_attn 227 vs 158 us, c_fc 364 vs 237, profiles/r05_ig.sh)
    if (v == 4 && k64 && a.Cout % 256 == 0) {
      launch256<256, 2, 2, 64, 2, OutT>(a, s);
      return;
    }
    if (v == 1 && k64) launch256<128, 4, 2, 64, 3, OutT>(a, s);
    else if (v == 3 && k64) {
      if (a.Cout % 256 == 0) launch256<256, 2, 4, 64, 2, OutT>(a, s);
      else launch256<128, 4, 2, 64, 2, OutT>(a, s);
    } else if (v == 0 || !k64) {
      if (a.Cout % 256 == 0) launch256<256, 2, 4, 32, 4, OutT>(a, s);
      else launch256<128, 4, 2, 32, 4, OutT>(a, s);
    } else {  // default (2): whole 128-B rows, double-buffered
      if (a.Cout % 256 == 0) launch256<256, 2, 4, 64, 2, OutT>(a, s);
      else launch256<128, 4, 2, 32, 4, OutT>(a, s);
    }
    return;
  }
  dispatch_old<OutT>(a, vec, s);
}

// the register-staged 128 / 256-row tiles (layers the LDS-DMA tile does not take)
template <typename OutT>
void dispatch_old(const IgArgs& a, bool vec, hipStream_t s) {
  const bool wide_n = a.Cout >= 128, wide_k = a.Cin >= 128;
  const bool win = vec && a.ntaps >= ITTS_IG_WIN_MINTAPS && a.span <= kWinSpan && igemm_win_enabled();
  if (wide_n && wide_k && a.Cout % 128 == 0) {
    if (win) launch_cfg<ITTS_IG_WIDEW, OutT>(a, vec, s);
    else launch_cfg<ITTS_IG_WIDE, OutT>(a, vec, s);
  } else if (wide_n && wide_k && a.Cout % 64 == 0) {
    if (win) launch_cfg<ITTS_IG_C192W, OutT>(a, vec, s);
    else launch_cfg<ITTS_IG_C192, OutT>(a, vec, s);
  }
  else if (wide_n && wide_k) launch_cfg<128, 128, 64, 64, 64, OutT>(a, vec, s);
  else if (wide_n) launch_cfg<128, 128, 64, 64, 32, OutT>(a, vec, s);
  else if (wide_k) launch_cfg<128, 32, 32, 32, 64, OutT>(a, vec, s);
  else launch_cfg<128, 32, 32, 32, 32, OutT>(a, vec, s);
}

}  // namespace

// Packing contract for Wp: ci_pad = round_up(Cin, Cin >= 128 ? 64 : 32),
// co_pad = round_up(Cout, Cout >= 128 ? 128 : 32).
extern "C" int itts_igemm_pack_dims(int Cin, int Cout, int* ci_pad, int* co_pad) {
  if (!ci_pad || !co_pad || Cin <= 0 || Cout <= 0) return itts::fail("itts_igemm_pack_dims", "bad args");
  const int kc = Cin >= 128 ? 64 : 32, tn = Cout >= 128 ? 128 : 32;
  *ci_pad = (Cin + kc - 1) / kc * kc;
  *co_pad = (Cout + tn - 1) / tn * tn;
  return 0;
}

namespace {
int igemm_fwd_impl(const char* fn, const void* x, int64_t x_sb, int64_t ldx, const void* w_packed, int64_t w_sb,
                   const float* bias, const float* bias_b, const void* r1, const void* r2, void* y, int64_t y_sb,
                   int64_t ldy, const int32_t* lengths, int B, int Tmax, int Cin, int Cout, int ntaps,
                   const int32_t* tap_off, int y_row_mul, int y_row_off, float alpha, int gelu, int out_dtype,
                   void* stream) {
  ITTS_REQUIRE(B >= 0 && Tmax >= 0 && Cin > 0 && Cout > 0, fn, "bad sizes");
  if (B == 0 || Tmax == 0) return 0;
  ITTS_REQUIRE(ntaps >= 1 && ntaps <= kMaxTaps, fn, "ntaps must be in [1, 16]");
  ITTS_REQUIRE(x && w_packed && y && tap_off, fn, "null pointer");
  ITTS_REQUIRE(out_dtype == ITTS_F32 || out_dtype == ITTS_BF16, fn, "out dtype must be f32 (0) or bf16 (1)");
  ITTS_REQUIRE(y_row_mul >= 1 && y_row_off >= 0, fn, "bad output row mapping");
  IgArgs a{};
  a.x = static_cast<const uint16_t*>(x);
  a.w = static_cast<const uint16_t*>(w_packed);
  a.wsb = w_sb;
  a.bias = bias;
  a.bias_b = bias_b;
  a.r1 = r1;
  a.r2 = r2;
  a.y = y;
  a.lens = lengths;
  a.B = B;
  a.Tmax = Tmax;
  a.Cin = Cin;
  a.Cout = Cout;
  itts_igemm_pack_dims(Cin, Cout, &a.ci_pad, &a.co_pad);
  a.ntaps = ntaps;
  a.sxb = x_sb;
  a.ldx = ldx;
  a.syb = y_sb;
  a.ldy = ldy;
  a.ymul = y_row_mul;
  a.yoff = y_row_off;
  a.alpha = alpha;
  a.gelu = gelu;
  int lo = tap_off[0], hi = tap_off[0];
  for (int j = 0; j < ntaps; ++j) {
    a.tap_off[j] = tap_off[j];
    lo = tap_off[j] < lo ? tap_off[j] : lo;
    hi = tap_off[j] > hi ? tap_off[j] : hi;
  }
  a.min_off = lo;
  a.span = hi - lo;
  const bool vec = (Cin % 8 == 0) && (ldx % 8 == 0) && (x_sb % 8 == 0) &&
                   ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  hipStream_t s = itts::as_stream(stream);
  if (out_dtype == ITTS_BF16) dispatch<uint16_t>(a, vec, s);
  else dispatch<float>(a, vec, s);
  return itts::check_launch(fn);
}

// y[m][n] = bias[n] + sum_s part[s][m][n], s ascending (fixed order: row-independent, run-to-run exact)
__global__ __launch_bounds__(256) void splitk_sum_kernel(const float4* __restrict__ part, int nsplit, int64_t n4,
                                                         int N4, const float4* __restrict__ bias,
                                                         float4* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 acc = bias ? bias[i % N4] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < nsplit; ++s) {
    const float4 v = part[(int64_t)s * n4 + i];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  y[i] = acc;
}
}  // namespace

extern "C" int itts_igemm_fwd(const void* x, int64_t x_sb, int64_t ldx, const void* w_packed, const float* bias,
                              const float* bias_b, const void* r1, const void* r2, void* y, int64_t y_sb, int64_t ldy,
                              const int32_t* lengths, int B, int Tmax, int Cin, int Cout, int ntaps,
                              const int32_t* tap_off, int y_row_mul, int y_row_off, float alpha, int gelu,
                              int out_dtype, void* stream) {
  return igemm_fwd_impl("itts_igemm_fwd", x, x_sb, ldx, w_packed, 0, bias, bias_b, r1, r2, y, y_sb, ldy, lengths, B,
                        Tmax, Cin, Cout, ntaps, tap_off, y_row_mul, y_row_off, alpha, gelu, out_dtype, stream);
}

extern "C" int itts_igemm_splitk(const void* x, int64_t ldx, int M, int K, const void* w_chunks, int nsplit, int N,
                                 const float* bias, float* partials, float* y, void* stream) {
  const char* fn = "itts_igemm_splitk";
  ITTS_REQUIRE(M >= 0 && K > 0 && N > 0 && nsplit >= 1 && K % nsplit == 0, fn, "bad sizes (K % nsplit == 0)");
  ITTS_REQUIRE((K / nsplit) % 8 == 0 && N % 4 == 0 && ldx >= K, fn, "K / nsplit must be a multiple of 8, N of 4");
  if (M == 0) return 0;
  ITTS_REQUIRE(x && w_chunks && partials && y, fn, "null pointer");
  ITTS_REQUIRE((reinterpret_cast<uintptr_t>(partials) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
                   (!bias || (reinterpret_cast<uintptr_t>(bias) & 15) == 0), fn, "partials, y, bias 16-byte aligned");
  const int Kc = K / nsplit;
  int ci_pad = 0, co_pad = 0;
  itts_igemm_pack_dims(Kc, N, &ci_pad, &co_pad);
  static const int32_t tap0 = 0;
  const int rc = igemm_fwd_impl(fn, x, Kc, ldx, w_chunks, (int64_t)ci_pad * co_pad, nullptr, nullptr, nullptr, nullptr,
                                partials, (int64_t)M * N, N, nullptr, nsplit, M, Kc, N, 1, &tap0, 1, 0, 1.0f, 0, ITTS_F32,
                                stream);
  if (rc) return rc;
  const int64_t n4 = (int64_t)M * N / 4;
  hipLaunchKernelGGL(splitk_sum_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, itts::as_stream(stream),
                     reinterpret_cast<const float4*>(partials), nsplit, n4, N / 4,
                     reinterpret_cast<const float4*>(bias), reinterpret_cast<float4*>(y));
  return itts::check_launch(fn);
}
