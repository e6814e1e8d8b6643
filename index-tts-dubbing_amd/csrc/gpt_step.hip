// Whole GPT decode step on gfx950: two multi-role launches per layer that keep weight streams off
// the dependency chain, and the C-ABI step driver (itts_gpt_decode_step).
//
// Reference: one KV-cached step of UnifiedVoice.inference_speech's generate (gpt/model.py:85-192 ->
// HF GPT2Block, modeling_gpt2.py:246-306: ln_1 -> c_attn -> attention (:54-72, :185-225) -> c_proj
// -> ln_2 -> c_fc -> gelu -> mlp.c_proj), then ln_f + final_norm -> mel_head (Q5) and the token
// selection (HF generation/utils.py), exactly as the per-kernel path in engine.HipGPT._decode_step.
//
// Per layer (bf16 product mode, R <= 128 rows):
//   1. itts_decode_qkv_attn: ONE launch, two roles.
//        blocks [0, 3D/16): c_attn producers -- the 16-column LayerNorm-folded GEMM of
//          decode_gemm16x_kernel (gpt_decode.hip; same fragments, same k order, same fixed-order
//          cross-wave sums: bit-identical q/k/v), epilogue stored write-through (sc1), then one
//          counter add per head (12 column tiles = q, k and v of one head).
//        blocks after: attention, one (row, head) pair per 256-thread block.  Each pair first
//          requests its cached K/V rows (they do not depend on this step), THEN waits for its head's
//          counter, reads q/k/v with sc1 loads and runs attn_decode_kernel's math (gpt_attn.hip).
//      The c_attn weight stream and the K/V stream overlap instead of following each other.
//   2. attn.c_proj: itts_decode_gemm16x residual epilogue (x += ., x^ = bf16 x).
//   3. itts_decode_mlp: ONE launch, three roles.
//        blocks [0, 4D/16): c_fc producers (ln_2 folded, gelu, bf16 pairs stored sc1), one counter
//          add per K-split group (the 4D/KS columns one split of mlp.c_proj consumes).
//        blocks after: mlp.c_proj split-K blocks (decode_gemm_kernel's 32-column MFMA tiles): the
//          weight slice is requested first, then the block waits for its group, reads its A slice
//          with sc1 loads, stores its f32 partial sc1 and adds to its column tile's ticket; the
//          block that draws the last ticket sums the KS partials in split order with the bias into
//          x and writes x^ -- the arithmetic of itts_residual_reduce_ln (no LayerNorm: folded).
//   The last layer keeps the separate launches (its reduce applies ln_f + final_norm for mel_head).
//
// Hand-offs (MI355X_MICROARCH.md "Valid forms", row 1; cdna_hip_programming.md Guideline 16):
// payload stored sc1 by every producing wave, each wave drains (s_waitcnt vmcnt(0)), block barrier,
// ONE lane adds to an agent-scope counter; the consumer polls that counter with relaxed sc1 loads
// (s_sleep between polls, bounded: a timeout sets a word the host checks), block barrier, and EVERY
// load of handed-off bytes is an sc1 load.  Counters are zeroed by one memset node per step.
// Producers have lower block indices than their consumers and never wait themselves, so progress
// does not depend on co-residency.
#include "common.h"

namespace {

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) float gf32;
#define ITTS_RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

constexpr int kU = 8;
constexpr int kNW = 8;                  // waves per block, every role
constexpr int kHD = 64;                 // head size
constexpr unsigned kSpinLimit = 1u << 20;  // polls before giving up (>= ~1 s): sets the timeout word
constexpr int kAttnKB = 10;             // keys per 8-lane group per round (as gpt_attn.hip)
// timing-only builds (profiles/ubench_fused.py; results invalid): 1 = consumers do not wait,
// 2 = producer roles return at once and consumers do not wait, 3 = consumer roles return at once
#ifndef ITTS_STEP_DIAG
#define ITTS_STEP_DIAG 0
#endif

__device__ __forceinline__ float gelu_tanh_d(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
}

// one lane: wait until *cnt >= need (relaxed agent-scope polls).  false: timed out (or an earlier
// wait of this step did) -- the timeout word is set and the caller goes on with whatever it reads.
__device__ __forceinline__ bool wait_geq(const uint32_t* cnt, unsigned need, uint32_t* tmo) {
  if (ITTS_STEP_DIAG == 1 || ITTS_STEP_DIAG == 2) return true;
  if (__hip_atomic_load((gu32*)tmo, ITTS_RLX_AGENT) != 0u) return false;
  unsigned spins = 0;
  while (__hip_atomic_load((gu32*)cnt, ITTS_RLX_AGENT) < need) {
    if (++spins > kSpinLimit) {
      __hip_atomic_store((gu32*)tmo, 1u, ITTS_RLX_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

__device__ __forceinline__ void st_sc1(float* p, float v) { __hip_atomic_store((gf32*)p, v, ITTS_RLX_AGENT); }
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) { __hip_atomic_store((gu32*)p, v, ITTS_RLX_AGENT); }
__device__ __forceinline__ float ld_sc1(const float* p) { return __hip_atomic_load((gf32*)p, ITTS_RLX_AGENT); }

// every storing wave drains its sc1 stores, the block meets, one lane adds `inc` to the counter
__device__ __forceinline__ unsigned publish_add(uint32_t* cnt, unsigned inc) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned old = 0;
  if (threadIdx.x == 0) old = __hip_atomic_fetch_add((gu32*)cnt, inc, ITTS_RLX_AGENT);
  return old;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
// 16-B load through the buffer path with sc1 (aux 16): bypasses this CU's L1
__device__ __forceinline__ u32x4_t ld16_sc1(__amdgpu_buffer_rsrc_t r, int64_t byte_off) {
  return __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 16));
}

// ---------------------------------------------------------------------------------------------
// 16-column producer body: decode_gemm16x_kernel<8, FOLD, ., ., MT>'s main loop and statistics.
// acc[2t + hf] = 16-row half hf of row tile t; with FOLD the row mean / rstd of A land in mu / rs.
template <int MT, int NW>
struct G16Lds {
  float red[NW][8][64];
  float rsum[NW][32 * MT], rsq[NW][32 * MT];
  float mu[32 * MT], rs[32 * MT];
};

template <int MT, bool FOLD, int NW>
__device__ __forceinline__ void g16_body(const uint16_t* __restrict__ A, int64_t lda, const u32x4_t* __restrict__ W,
                                         int K, int nt, float eps, G16Lds<MT, NW>& sm, f32x4_t (&acc)[2 * MT]) {
  constexpr int R = 32 * MT, kNW = NW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ksteps = K / 32;
  const int niter = (ksteps - w + kNW - 1) / kNW;  // this wave's k-steps: w + kNW*i
  const u32x4_t* Wt = W + (int64_t)nt * ksteps * 64 + lane;
  const int c16 = lane & 15, q = lane >> 4;

  u32x4_t wa[kU] = {}, wb[kU] = {};
  auto wload = [&](u32x4_t (&dst)[kU], int i0) {
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + u < niter) dst[u] = __builtin_nontemporal_load(Wt + (int64_t)(w + kNW * (i0 + u)) * 64);
  };
  wload(wa, 0);
  float ssum[2 * MT], ssq[2 * MT];
#pragma unroll
  for (int t = 0; t < 2 * MT; ++t) {
    acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    ssum[t] = ssq[t] = 0.f;
  }
  auto compute = [&](const u32x4_t (&src)[kU], int i0) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (i0 + u >= niter) continue;
      const int64_t col = 32 * (w + kNW * (i0 + u)) + 8 * q;
      bf16x8_t av[2 * MT];
#pragma unroll
      for (int t = 0; t < 2 * MT; ++t) av[t] = *reinterpret_cast<const bf16x8_t*>(A + (int64_t)(16 * t + c16) * lda + col);
      const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(&src[u]);
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
    }
  };
  for (int i0 = 0; i0 < niter; i0 += 2 * kU) {
    if (i0 + kU < niter) wload(wb, i0 + kU);
    compute(wa, i0);
    if (i0 + 2 * kU < niter) wload(wa, i0 + 2 * kU);
    if (i0 + kU < niter) compute(wb, i0 + kU);
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
        sm.rsum[w][16 * t + c16] = a;
        sm.rsq[w][16 * t + c16] = b;
      }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < R; r += 64 * kNW) {
      float S = 0.f, Q = 0.f;
#pragma unroll
      for (int ww = 0; ww < kNW; ++ww) {
        S += sm.rsum[ww][r];
        Q += sm.rsq[ww][r];
      }
      const float inv = 1.0f / K, m = S * inv;
      sm.mu[r] = m;
      sm.rs[r] = rsqrtf(fmaxf(Q * inv - m * m, 0.f) + eps);
    }
    __syncthreads();
  }
}

// row tile `tile` of the accumulators -> sm.red (one 32-row tile at a time)
template <int MT, int NW>
__device__ __forceinline__ void g16_stage_tile(G16Lds<MT, NW>& sm, const f32x4_t (&acc)[2 * MT], int tile) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (tile > 0) __syncthreads();  // previous tile's reads done
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int r = 0; r < 4; ++r) sm.red[w][4 * hf + r][lane] = acc[2 * tile + hf][r];
  __syncthreads();
}

// finished value of output (row-in-tile rr, column c16) of the staged tile, the fixed-order wave sum
// and the fold / additive terms exactly as decode_gemm16x_kernel's epilogue
template <int MT, bool FOLD, int NW>
__device__ __forceinline__ float g16_value(const G16Lds<MT, NW>& sm, int tile, int rr, int c16, int n, const float* u,
                                           const float* c) {
  const int hf = rr >> 4, r16 = rr & 15;
  const int e = 4 * hf + (r16 & 3), l = 16 * (r16 >> 2) + c16;
  float v = 0.f;
#pragma unroll
  for (int ww = 0; ww < NW; ++ww) v += sm.red[ww][e][l];
  const int row = 32 * tile + rr;
  if constexpr (FOLD) v = sm.rs[row] * (v - sm.mu[row] * u[n]);
  if (c) v += c[n];
  return v;
}

// ---------------------------------------------------------------------------------------------
// attention of one (row b, head h) pair on a 256-thread block: the math of
// attn_decode_kernel<bf16, bf16, 256, ROWS, false> (gpt_attn.hip), with q/k/v read by sc1 loads
// after the head's producers signalled.
struct AttnLds {
  float qs[kHD], kn[kHD], vn[kHD];
  float gm[32], gl[32];
  float pv[32][kHD + 1];
};

template <int ROWS_T>
__device__ __forceinline__ void attn_pair(int b, int h, const float* __restrict__ qkv,
                                          int64_t ldqkv, uint16_t* __restrict__ cache_k, uint16_t* __restrict__ cache_v,
                                          int64_t cache_bs, int64_t cache_hs, const int32_t* pad, int kv_base,
                                          const int32_t* __restrict__ tstate, uint16_t* __restrict__ out, int64_t ldo,
                                          int H, const int32_t* __restrict__ kv_rows, int64_t ld_rows,
                                          const uint32_t* head_cnt, unsigned need, uint32_t* tmo, AttnLds& sm) {
  constexpr bool ROWS = ROWS_T != 0;
  constexpr int NG = 32, KB = kAttnKB;
  const int tid = threadIdx.x;
  const int D = H * kHD;
  const int kidx = kv_base + tstate[0];
  const int p0 = pad ? pad[b] : 0;
  const int nk = kidx + 1 - p0;
  uint16_t* Kc = cache_k + (int64_t)b * cache_bs + (int64_t)h * cache_hs;
  uint16_t* Vc = cache_v + (int64_t)b * cache_bs + (int64_t)h * cache_hs;
  const int32_t* rows = ROWS ? kv_rows + (int64_t)b * ld_rows : nullptr;
  auto koff = [&](int p) -> int64_t {
    if constexpr (ROWS) return (int64_t)(rows[p] - b) * cache_bs + (int64_t)p * kHD;
    else return (int64_t)p * kHD;
  };
  const int g = tid >> 3, d8 = tid & 7;
  // (1) this round's cached K/V rows: independent of this step's q/k/v, requested first
  u32x4_t kr[KB], vr[KB];
#pragma unroll
  for (int u = 0; u < KB; ++u) {
    const int j = NG * u + g;
    if (j < nk - 1) {
      kr[u] = *reinterpret_cast<const u32x4_t*>(Kc + koff(p0 + j) + 8 * d8);
      vr[u] = *reinterpret_cast<const u32x4_t*>(Vc + koff(p0 + j) + 8 * d8);
    }
  }
  // (2) wait for the head's 12 producer tiles (one lane per pair), then the block meets
  if (tid == 0) wait_geq(head_cnt, need, tmo);
  __syncthreads();
  if (tid < 3 * kHD) {
    const int part = tid / kHD, d = tid - part * kHD;  // 0: q, 1: k, 2: v
    const int col = part * D + h * kHD + d;
    float v = 0.f;
    v += ld_sc1(qkv + (int64_t)b * ldqkv + col);
    if (part == 0) {
      sm.qs[d] = v * 0.125f;  // 1/sqrt(64), exact
    } else if (part == 1) {
      sm.kn[d] = v;
      Kc[(int64_t)kidx * kHD + d] = f2bf(v);
    } else {
      sm.vn[d] = v;
      Vc[(int64_t)kidx * kHD + d] = f2bf(v);
    }
  }
  __syncthreads();
  float q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) q[e] = sm.qs[8 * d8 + e];
  auto unpack = [&](const u32x4_t& r, float (&x)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[2 * i] = __uint_as_float(r[i] << 16);
      x[2 * i + 1] = __uint_as_float(r[i] & 0xFFFF0000u);
    }
  };
  float m = -INFINITY, l = 0.f;
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nk; j0 += NG * KB) {
    if (j0 > 0) {
#pragma unroll
      for (int u = 0; u < KB; ++u) {
        const int j = j0 + NG * u + g;
        if (j < nk - 1) {
          kr[u] = *reinterpret_cast<const u32x4_t*>(Kc + koff(p0 + j) + 8 * d8);
          vr[u] = *reinterpret_cast<const u32x4_t*>(Vc + koff(p0 + j) + 8 * d8);
        }
      }
    }
    float s[KB];
    float bm = -INFINITY;
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int j = j0 + NG * u + g;
      float kx[8];
      if (j < nk - 1) {
        unpack(kr[u], kx);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) kx[e] = sm.kn[8 * d8 + e];
      }
      float part = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) part = fmaf(q[e], kx[e], part);
      part = sum8_dpp(part);
      s[u] = j < nk ? part : -INFINITY;
      bm = fmaxf(bm, s[u]);
    }
    if (bm == -INFINITY) continue;
    const float mn = fmaxf(m, bm);
    const float corr = __expf(m - mn);
    l *= corr;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] *= corr;
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int j = j0 + NG * u + g;
      const float pr = __expf(s[u] - mn);
      l += pr;
      float vx[8];
      if (j < nk - 1) {
        unpack(vr[u], vx);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) vx[e] = sm.vn[8 * d8 + e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(pr, vx[e], o[e]);
    }
    m = mn;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) sm.pv[g][8 * d8 + e] = o[e];
  if (d8 == 0) {
    sm.gm[g] = m;
    sm.gl[g] = l;
  }
  __syncthreads();
  if (tid < kHD) {
    float M = -INFINITY;
#pragma unroll 8
    for (int i = 0; i < NG; ++i) M = fmaxf(M, sm.gm[i]);
    float L = 0.f, acc = 0.f;
#pragma unroll 8
    for (int i = 0; i < NG; ++i) {
      const float w = __expf(sm.gm[i] - M);
      L = fmaf(sm.gl[i], w, L);
      acc = fmaf(sm.pv[i][tid], w, acc);
    }
    out[(int64_t)b * ldo + h * kHD + tid] = f2bf(acc / L);
  }
}

struct QkvAttnArgs {
  const uint16_t* xh;
  int64_t ldxh;
  const u32x4_t* w16;
  const float *u, *c;
  float eps;
  float* qkv;
  int64_t ldqkv;
  uint16_t *cache_k, *cache_v;
  int64_t cache_bs, cache_hs;
  const int32_t* pad;
  int kv_base;
  const int32_t* tstate;
  uint16_t* out;
  int64_t ldo;
  int R, H, nprod;
  const int32_t* kv_rows;
  int64_t ld_rows;
  uint32_t* cnt;  // [H]
  uint32_t* tmo;
};

// 256-thread blocks for both roles: the attention body needs ~200 VGPRs (2 blocks per CU), and
// 512-thread blocks would then fit one per CU.  Producers therefore run 4 waves (the unfused path's
// c_attn uses the same 4-wave itts_decode_gemm16x, so the two paths agree bit for bit).
constexpr int kQkvNW = 4;

template <int MT, int ROWS>
__global__ __launch_bounds__(256) void qkv_attn_kernel(QkvAttnArgs p) {
  const int D = p.H * kHD;
  if ((int)blockIdx.x < p.nprod) {
    if (ITTS_STEP_DIAG == 2) return;
    // ---- c_attn producer: 16 columns of q|k|v for all R rows ----
    __shared__ G16Lds<MT, kQkvNW> sm;
    const int nt = blockIdx.x;
    f32x4_t acc[2 * MT];
    g16_body<MT, true, kQkvNW>(p.xh, p.ldxh, p.w16, D, nt, p.eps, sm, acc);
    for (int tile = 0; tile < MT; ++tile) {
      g16_stage_tile<MT, kQkvNW>(sm, acc, tile);
#pragma unroll
      for (int k = 0; k < 2; ++k) {  // 32 rows x 16 columns, two per thread
        const int o = threadIdx.x + 256 * k;
        const int rr = o >> 4, c16 = o & 15;
        const int row = 32 * tile + rr, n = nt * 16 + c16;
        if (row < p.R)
          st_sc1(p.qkv + (int64_t)row * p.ldqkv + n, g16_value<MT, true, kQkvNW>(sm, tile, rr, c16, n, p.u, p.c));
      }
    }
    const int head = ((nt * 16) % D) / kHD;
    publish_add(p.cnt + head, 1u);
    return;
  }
  // ---- attention: pair = b * H + h ----
  if (ITTS_STEP_DIAG == 3) return;
  __shared__ AttnLds sa;
  const int pair = blockIdx.x - p.nprod;
  const int b = pair / p.H, h = pair % p.H;
  attn_pair<ROWS>(b, h, p.qkv, p.ldqkv, p.cache_k, p.cache_v, p.cache_bs, p.cache_hs, p.pad, p.kv_base, p.tstate,
                  p.out, p.ldo, p.H, p.kv_rows, p.ld_rows, p.cnt + h, 3u * (kHD / 16), p.tmo, sa);
}

// ---------------------------------------------------------------------------------------------
struct MlpArgs {
  const uint16_t* xh;  // bf16 residual copy [Rpad][ldxh] (c_fc's A; rewritten by the reducers)
  int64_t ldxh;
  const u32x4_t* fc_w16;
  const float *fc_u, *fc_c;
  float eps;
  uint16_t* f;         // gelu(c_fc) bf16 [Rpad][ldf]
  int64_t ldf, f_bytes;
  const u32x4_t* proj_w;  // mlp.c_proj in 32-column fragment order (pack_skinny)
  const float* proj_b;
  float* part;         // [KS][R][D] f32
  float* x;            // f32 residual [R][ldx]
  int64_t ldx;
  int R, D, nfc;
  uint32_t* cnt;       // [KS] group counters, then [D/32] column-tile tickets
  uint32_t* tmo;
};

template <int MT>
struct ProjLds {
  float red[kNW * 16 * 64];
  int last;
};

template <int MT, int KS>
__global__ __launch_bounds__(512) void mlp_kernel(MlpArgs p) {
  const int D = p.D, F = 4 * D;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if ((int)blockIdx.x < p.nfc) {
    if (ITTS_STEP_DIAG == 2) return;
    // ---- c_fc producer: 16 columns of gelu(LN_2(x) W_fc + b) for all R rows ----
    __shared__ G16Lds<MT, kNW> sm;
    const int nt = blockIdx.x;
    f32x4_t acc[2 * MT];
    g16_body<MT, true, kNW>(p.xh, p.ldxh, p.fc_w16, D, nt, p.eps, sm, acc);
    for (int tile = 0; tile < MT; ++tile) {
      g16_stage_tile<MT, kNW>(sm, acc, tile);
      if (threadIdx.x < 256) {  // 32 rows x 8 column pairs, one 4-B (2 x bf16) store each
        const int rr = threadIdx.x >> 3, c2 = 2 * (threadIdx.x & 7);
        const int row = 32 * tile + rr, n = nt * 16 + c2;
        if (row < p.R) {
          const float v0 = gelu_tanh_d(g16_value<MT, true, kNW>(sm, tile, rr, c2, n, p.fc_u, p.fc_c));
          const float v1 = gelu_tanh_d(g16_value<MT, true, kNW>(sm, tile, rr, c2 + 1, n + 1, p.fc_u, p.fc_c));
          st_sc1(reinterpret_cast<uint32_t*>(p.f + (int64_t)row * p.ldf + n), pack2bf(v0, v1));
        }
      }
    }
    const int group = (nt * 16) / (F / KS);
    publish_add(p.cnt + group, 1u);
    return;
  }
  // ---- mlp.c_proj split-K block (ks, nt): decode_gemm_kernel<8, 0, 2, ., float, MT> ----
  if (ITTS_STEP_DIAG == 3) return;
  __shared__ ProjLds<MT> sp;
  const int pb = blockIdx.x - p.nfc, ntiles = D / 32;
  const int ks = pb / ntiles, nt = pb % ntiles;
  const int ksteps = F / 16, kper = ksteps / KS, kbeg = ks * kper;
  const int niter = (kper - w + kNW - 1) / kNW;
  const u32x4_t* Wt = p.proj_w + ((int64_t)nt * ksteps + kbeg) * 64 + lane;
  const int r32 = lane & 31, hh = lane >> 5;
  u32x4_t wa[kU] = {}, wb[kU] = {};
  auto wload = [&](u32x4_t (&dst)[kU], int i0) {
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + u < niter) dst[u] = __builtin_nontemporal_load(Wt + (int64_t)(w + kNW * (i0 + u)) * 64);
  };
  wload(wa, 0);  // the weight slice does not depend on c_fc: requested before the wait
  if (threadIdx.x == 0) wait_geq(p.cnt + ks, (unsigned)((F / KS) / 16), p.tmo);
  __syncthreads();
  const __amdgpu_buffer_rsrc_t fr = rsrc_of(p.f, p.f_bytes);
  f32x16_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  auto compute = [&](const u32x4_t (&src)[kU], int i0) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      bf16x8_t af[kU] = {};
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (i0 + u < niter) {
          const int s = kbeg + w + kNW * (i0 + u);
          af[u] = __builtin_bit_cast(bf16x8_t, ld16_sc1(fr, ((int64_t)(32 * t + r32) * p.ldf + 16 * s + 8 * hh) * 2));
        }
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
  // partial tile(s) -> part[ks] (sc1), through the fixed-order cross-wave sum
  float* myred = sp.red + w * 16 * 64;
  constexpr int PER = 1024 / (64 * kNW);
  const int64_t split_stride = (int64_t)p.R * D;
#pragma unroll
  for (int tile = 0; tile < MT; ++tile) {
    if (tile > 0) __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) myred[r * 64 + lane] = acc[tile][r];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int o = threadIdx.x + 64 * kNW * k;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < kNW; ++ww) v += sp.red[ww * 1024 + o];
      const int r = o / 64, l = o % 64;
      const int row = 32 * tile + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      const int n = nt * 32 + (l & 31);
      if (row < p.R) st_sc1(p.part + ks * split_stride + (int64_t)row * D + n, v);
    }
  }
  // ticket: the block drawing the last one of this column tile reduces it
  const unsigned old = publish_add(p.cnt + KS + nt, 1u);
  if (threadIdx.x == 0) sp.last = old == (unsigned)(KS - 1);
  __syncthreads();
  if (!sp.last) return;
  const __amdgpu_buffer_rsrc_t pr = rsrc_of(p.part, (int64_t)KS * split_stride * 4);
  for (int i = threadIdx.x; i < 32 * MT * 8; i += 64 * kNW) {
    const int row = i >> 3, n = nt * 32 + 4 * (i & 7);
    if (row >= p.R) continue;
    float* xr = p.x + (int64_t)row * p.ldx + n;
    const f32x4_t acc4 = *reinterpret_cast<const f32x4_t*>(xr);
    const f32x4_t bv = *reinterpret_cast<const f32x4_t*>(p.proj_b + n);
    f32x4_t pv[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      pv[s] = __builtin_bit_cast(f32x4_t, ld16_sc1(pr, (s * split_stride + (int64_t)row * D + n) * 4));
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s4 = bv[e];
#pragma unroll
      for (int s = 0; s < KS; ++s) s4 += pv[s][e];
      v[e] = acc4[e] + s4;
    }
    *reinterpret_cast<f32x4_t*>(xr) = f32x4_t{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<u32x2_t*>(const_cast<uint16_t*>(p.xh) + (int64_t)row * p.ldxh + n) =
        u32x2_t{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
  }
}

// ---------------------------------------------------------------------------------------------
// KV prefetch (launch_mode 2): read one layer's valid cached keys / values once on a side stream
// while the latency-bound GEMM chain runs, so that the attention's own reads find the lines in the
// die-level Infinity Cache (MALL) instead of HBM.  Nothing is stored (the XOR of the bytes goes to
// `sink` only if it equals an arbitrary constant, which keeps the loads alive).
constexpr int kPfU = 8;  // 16-B loads of K and of V in flight per thread

__global__ __launch_bounds__(256) void kv_prefetch_kernel(const u32x4_t* __restrict__ kc, const u32x4_t* __restrict__ vc,
                                                          int64_t bs16, int64_t hs16, int R, int H,
                                                          const int32_t* __restrict__ pad, int kv_base,
                                                          const int32_t* __restrict__ tstate, uint32_t* sink) {
  const int kidx = kv_base + tstate[0];  // keys [pad, kidx) exist before this step's append
  uint32_t acc = 0;
  for (int pair = blockIdx.x; pair < R * H; pair += gridDim.x) {
    const int b = pair / H, h = pair - b * H;
    const int p0 = pad ? pad[b] : 0;
    const int64_t base = b * bs16 + h * hs16 + (int64_t)p0 * (kHD * 2 / 16);
    const int n16 = (kidx - p0) * (kHD * 2 / 16);
    for (int i0 = threadIdx.x; i0 < n16; i0 += 256 * kPfU) {
      u32x4_t a[kPfU], v[kPfU];
#pragma unroll
      for (int u = 0; u < kPfU; ++u) {
        const int i = i0 + 256 * u;
        if (i < n16) {
          a[u] = kc[base + i];  // default policy: the lines must stay in the caches
          v[u] = vc[base + i];
        } else {
          a[u] = v[u] = u32x4_t{0u, 0u, 0u, 0u};
        }
      }
#pragma unroll
      for (int u = 0; u < kPfU; ++u) acc ^= a[u][0] ^ v[u][3];
    }
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// C ABI

extern "C" int itts_decode_qkv_attn(const void* xh, int64_t ldxh, const void* w_packed16, const float* u, const float* c,
                                    float eps, float* qkv, int64_t ldqkv, void* cache_k, void* cache_v,
                                    int64_t cache_bs, int64_t cache_hs, int smax, const int32_t* pad, int kv_base,
                                    const int32_t* tstate, void* out, int64_t ldo, int R, int H,
                                    const int32_t* kv_rows, int64_t ld_rows, uint32_t* counters, uint32_t* timeout,
                                    void* stream) {
  const char* fn = "itts_decode_qkv_attn";
  ITTS_REQUIRE(R >= 0 && R <= 128 && H > 0 && H <= 64, fn, "rows must be in [0, 128], heads in [1, 64]");
  if (R == 0) return 0;
  ITTS_REQUIRE(xh && w_packed16 && u && c && qkv && cache_k && cache_v && tstate && out && counters && timeout, fn,
               "null pointer");
  ITTS_REQUIRE(ldxh % 8 == 0 && (reinterpret_cast<uintptr_t>(xh) & 15) == 0, fn, "x^ rows must be 16-B aligned");
  ITTS_REQUIRE(ldqkv >= 3 * H * kHD && cache_hs >= (int64_t)smax * kHD, fn, "bad strides");
  ITTS_REQUIRE(!kv_rows || ld_rows >= smax, fn, "kv_rows [R][ld_rows >= smax] required");
  const int D = H * kHD, nprod = 3 * D / 16, npairs = R * H;
  QkvAttnArgs a{static_cast<const uint16_t*>(xh), ldxh, static_cast<const u32x4_t*>(w_packed16), u, c, eps, qkv, ldqkv,
                static_cast<uint16_t*>(cache_k), static_cast<uint16_t*>(cache_v), cache_bs, cache_hs, pad, kv_base,
                tstate, static_cast<uint16_t*>(out), ldo, R, H, nprod, kv_rows, ld_rows, counters, timeout};
  const dim3 grid(nprod + npairs), block(256);
  hipStream_t s = itts::as_stream(stream);
  const int mt = (R + 31) / 32;
#define QA(MTV)                                                                         \
  do {                                                                                  \
    if (kv_rows) hipLaunchKernelGGL((qkv_attn_kernel<MTV, 1>), grid, block, 0, s, a);   \
    else hipLaunchKernelGGL((qkv_attn_kernel<MTV, 0>), grid, block, 0, s, a);           \
  } while (0)
  switch (mt) {
    case 1: QA(1); break;
    case 2: QA(2); break;
    case 3: QA(3); break;
    default: QA(4); break;
  }
#undef QA
  return itts::check_launch(fn);
}

extern "C" int itts_decode_mlp(const void* xh, int64_t ldxh, const void* fc_w16, const float* fc_u, const float* fc_c,
                               float eps, void* f, int64_t ldf, const void* proj_w, const float* proj_b, float* part,
                               float* x, int64_t ldx, int R, int D, int ksplit, uint32_t* counters, uint32_t* timeout,
                               void* stream) {
  const char* fn = "itts_decode_mlp";
  ITTS_REQUIRE(R >= 0 && R <= 128 && D > 0 && D % 256 == 0, fn, "rows must be in [0, 128], D a multiple of 256");
  if (R == 0) return 0;
  ITTS_REQUIRE(ksplit == 8, fn, "ksplit must be 8");
  ITTS_REQUIRE(xh && fc_w16 && fc_u && fc_c && f && proj_w && proj_b && part && x && counters && timeout, fn,
               "null pointer");
  ITTS_REQUIRE(ldxh % 8 == 0 && ldf % 8 == 0 && ldx % 4 == 0, fn, "rows must be 16-B aligned");
  ITTS_REQUIRE(((reinterpret_cast<uintptr_t>(xh) | reinterpret_cast<uintptr_t>(f) | reinterpret_cast<uintptr_t>(x) |
                 reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(proj_b)) & 15) == 0,
               fn, "buffers must be 16-B aligned");
  const int mt = (R + 31) / 32;
  const int64_t f_bytes = (int64_t)32 * mt * ldf * 2;
  ITTS_REQUIRE(f_bytes < (1ll << 31) && (int64_t)ksplit * R * D * 4 < (1ll << 31), fn, "buffers too large");
  const int nfc = 4 * D / 16, nproj = (D / 32) * ksplit;
  MlpArgs a{static_cast<const uint16_t*>(xh), ldxh, static_cast<const u32x4_t*>(fc_w16), fc_u, fc_c, eps,
            static_cast<uint16_t*>(f), ldf, f_bytes, static_cast<const u32x4_t*>(proj_w), proj_b, part, x, ldx, R, D,
            nfc, counters, timeout};
  const dim3 grid(nfc + nproj), block(512);
  hipStream_t s = itts::as_stream(stream);
  switch (mt) {
    case 1: hipLaunchKernelGGL((mlp_kernel<1, 8>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((mlp_kernel<2, 8>), grid, block, 0, s, a); break;
    case 3: hipLaunchKernelGGL((mlp_kernel<3, 8>), grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL((mlp_kernel<4, 8>), grid, block, 0, s, a); break;
  }
  return itts::check_launch(fn);
}

// ---- the whole step ---------------------------------------------------------------------------
namespace {
constexpr int kMlpSplit = 8;
int sync_words_per_layer(int D, int H) { return (H + kMlpSplit + D / 32 + 3) / 4 * 4; }
int64_t sync_bytes(const ItTsGptWeights* w) {
  return ((int64_t)w->n_layer * sync_words_per_layer(w->d_model, w->n_head) * 4 + 15) / 16 * 16;
}
}  // namespace

constexpr int kPfBlocks = 64;  // KV prefetch grid (a quarter of the CUs)

extern "C" int64_t itts_gpt_decode_workspace_bytes(const ItTsGptWeights* w) {
  if (!w || w->n_layer <= 0 || w->d_model <= 0 || w->n_head <= 0) return -1;
  return sync_bytes(w) + kPfBlocks * 4 + 16;  // counters, the prefetch sink, the timeout word (+ padding)
}

namespace {
// side stream + fork/join events of launch_mode 2, per device (created once, kept for the process)
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork[64], join[64];
};
SideStream* side_stream() {
  static SideStream per_dev[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  SideStream& ss = per_dev[dev];
  if (!ss.s) {
    if (hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    for (int i = 0; i < 64; ++i)
      if (hipEventCreateWithFlags(&ss.fork[i], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&ss.join[i], hipEventDisableTiming) != hipSuccess)
        return nullptr;
  }
  return &ss;
}
}  // namespace

extern "C" int itts_gpt_decode_step(const ItTsGptWeights* w, const ItTsGptDecodeState* st, const ItTsSampling* smp,
                                    void* stream) {
  const char* fn = "itts_gpt_decode_step";
  ITTS_REQUIRE(w && st && smp && w->layers, fn, "null pointer");
  const int L = w->n_layer, D = w->d_model, H = w->n_head, R = st->rows;
  ITTS_REQUIRE(L > 0 && D == H * kHD && D % 256 == 0, fn, "d_model must be 64 * n_head and a multiple of 256");
  ITTS_REQUIRE(R > 0 && (R <= 128 || st->launch_mode == 0), fn, "multi-role launches need rows <= 128");
  ITTS_REQUIRE(smp->mode >= 0 && smp->mode <= 2, fn, "sampling mode must be 0 (greedy), 1 (sample) or 2 (logits)");
  ITTS_REQUIRE(st->x && st->xh && st->qkv && st->o && st->f && st->part && st->logits && st->k_cache && st->v_cache &&
                   st->tstate && st->workspace,
               fn, "null state buffer");
  ITTS_REQUIRE(smp->mode == 2 || (st->seen && st->done && st->codes), fn, "sampler state missing");
  ITTS_REQUIRE(st->launch_mode >= 0 && st->launch_mode <= 2, fn, "launch_mode must be 0, 1 or 2");
  ITTS_REQUIRE(L <= 64, fn, "at most 64 layers");
  hipStream_t s = itts::as_stream(stream);
  const float eps = 1e-5f;
  const bool multirole = st->launch_mode == 1;
  const bool prefetch = st->launch_mode == 2 && !st->kv_rows;
  const int wpl = sync_words_per_layer(D, H);
  uint32_t* sync = static_cast<uint32_t*>(st->workspace);
  uint32_t* sink = reinterpret_cast<uint32_t*>(static_cast<unsigned char*>(st->workspace) + sync_bytes(w));
  uint32_t* tmo = sink + kPfBlocks;
  if (multirole && hipMemsetAsync(sync, 0, sync_bytes(w), s) != hipSuccess) return itts::check_launch(fn);
  const int64_t cache_hs = (int64_t)st->max_kv * kHD, cache_bs = (int64_t)H * cache_hs;
  const int64_t layer_cache = (int64_t)R * cache_bs;
  SideStream* ss = prefetch ? side_stream() : nullptr;
  ITTS_REQUIRE(!prefetch || ss, fn, "side stream / events could not be created");
  // side stream: wait for `after` on the main stream, prefetch layer l's K/V, record join[l]
  auto fork_prefetch = [&](int l) -> int {
    if (hipEventRecord(ss->fork[l], s) != hipSuccess || hipStreamWaitEvent(ss->s, ss->fork[l], 0) != hipSuccess)
      return itts::check_launch(fn);
    const uint16_t* kcl = static_cast<const uint16_t*>(st->k_cache) + l * layer_cache;
    const uint16_t* vcl = static_cast<const uint16_t*>(st->v_cache) + l * layer_cache;
    hipLaunchKernelGGL(kv_prefetch_kernel, dim3(kPfBlocks), dim3(256), 0, ss->s,
                       reinterpret_cast<const u32x4_t*>(kcl), reinterpret_cast<const u32x4_t*>(vcl), cache_bs / 8,
                       cache_hs / 8, R, H, st->pad, st->kv_base, st->tstate, sink);
    if (hipEventRecord(ss->join[l], ss->s) != hipSuccess) return itts::check_launch(fn);
    return itts::check_launch(fn);
  };
  int rc = 0;
  if (prefetch) rc = fork_prefetch(0);
  for (int l = 0; l < L && rc == 0; ++l) {
    const ItTsGptLayerW& ly = w->layers[l];
    uint16_t* kc = static_cast<uint16_t*>(st->k_cache) + l * layer_cache;
    uint16_t* vc = static_cast<uint16_t*>(st->v_cache) + l * layer_cache;
    uint32_t* cnt = sync + (int64_t)l * wpl;
    if (multirole) {
      rc = itts_decode_qkv_attn(st->xh, D, ly.qkv_w16, ly.qkv_u, ly.qkv_c, eps, st->qkv, 3 * D, kc, vc, cache_bs,
                                cache_hs, st->max_kv, st->pad, st->kv_base, st->tstate, st->o, D, R, H, st->kv_rows,
                                st->ld_rows, cnt, tmo, stream);
    } else {
      rc = itts_decode_gemm16x(st->xh, D, ly.qkv_w16, D, 3 * D, R, ly.qkv_c, ly.qkv_u, eps, 0, 0, st->qkv, 3 * D,
                               ITTS_F32, nullptr, 0, 8, stream);
      if (!rc && prefetch && hipStreamWaitEvent(s, ss->join[l], 0) != hipSuccess) rc = itts::check_launch(fn);
      if (!rc && st->kv_rows)
        rc = itts_attn_decode_rows(st->qkv, 3 * D, 1, (int64_t)R * 3 * D, nullptr, kc, vc, cache_bs, cache_hs,
                                   st->max_kv, st->pad, st->kv_base, st->tstate, st->o, D, R, H, ITTS_BF16, ITTS_BF16,
                                   st->kv_rows, st->ld_rows, stream);
      else if (!rc)
        rc = itts_attn_decode(st->qkv, 3 * D, 1, (int64_t)R * 3 * D, nullptr, kc, vc, cache_bs, cache_hs, st->max_kv,
                              st->pad, st->kv_base, st->tstate, st->o, D, R, H, ITTS_BF16, ITTS_BF16, stream);
    }
    if (rc) break;
    if (prefetch && l + 1 < L && (rc = fork_prefetch(l + 1)) != 0) break;  // next layer's K/V beside the GEMMs
    rc = itts_decode_gemm16x(st->o, D, ly.o_w16, D, D, R, ly.o_c, nullptr, eps, 0, 1, st->x, D, ITTS_F32, st->xh, D, 8,
                             stream);
    if (rc) break;
    if (l + 1 < L && multirole) {
      rc = itts_decode_mlp(st->xh, D, ly.fc_w16, ly.fc_u, ly.fc_c, eps, st->f, 4 * D, ly.proj_w, ly.proj_b, st->part,
                           st->x, D, R, D, kMlpSplit, cnt + H, tmo, stream);
    } else {  // (the last layer's reduce applies ln_f + final_norm for mel_head, Q5)
      const bool last = l + 1 == L;
      rc = itts_decode_gemm16x(st->xh, D, ly.fc_w16, D, 4 * D, R, ly.fc_c, ly.fc_u, eps, 1, 0, st->f, 4 * D, ITTS_BF16,
                               nullptr, 0, 8, stream);
      if (!rc)
        rc = itts_decode_gemm(st->f, 4 * D, ly.proj_w, 4 * D, D, R, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0,
                              2, st->part, D, ITTS_F32, (int64_t)R * D, kMlpSplit, stream);
      if (!rc)
        rc = itts_residual_reduce_ln(st->x, D, st->part, kMlpSplit, (int64_t)R * D, D, ly.proj_b, st->xh, D, R, D,
                                     last ? w->ln_f_g : nullptr, last ? w->ln_f_b : nullptr,
                                     last ? w->final_g : nullptr, last ? w->final_b : nullptr, ITTS_BF16, stream);
    }
  }
  if (rc) return rc;
  rc = itts_decode_gemm(st->xh, D, w->head_w, D, w->n_mel_codes, R, w->head_b, nullptr, nullptr, nullptr, nullptr, 0, 0,
                        0, st->logits, w->logits_pitch, ITTS_F32, (int64_t)R * w->n_mel_codes, 1, stream);
  if (rc) return rc;
  if (smp->mode == 0) {
    rc = itts_sample_embed(st->logits, w->logits_pitch, w->n_mel_codes, st->seen, st->done, st->codes, st->max_new,
                           st->tstate, 1, smp->min_new, w->stop_mel, smp->rep_penalty, w->mel_emb, w->mel_pos, 2, D,
                           nullptr, nullptr, st->x, st->xh, ITTS_BF16, R, st->forced, stream);
  } else if (smp->mode == 1) {
    rc = itts_sample_topk_embed(st->logits, w->logits_pitch, w->n_mel_codes, st->seen, st->done, st->codes,
                                st->max_new, st->tstate, 1, smp->min_new, w->stop_mel, smp->rep_penalty,
                                smp->temperature, smp->top_k, smp->top_p, w->mel_emb, w->mel_pos, 2, D, nullptr,
                                nullptr, st->x, st->xh, ITTS_BF16, R, st->forced, stream);
  }
  if (rc == 0 && smp->mode != 2) rc = itts_step_advance(st->tstate, 1, stream);
  return rc;
}
