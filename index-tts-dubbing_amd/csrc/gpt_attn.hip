// GPT-2 self-attention (16 heads x 64, scale 1/8, causal + left-padding key mask) for gfx950.
// Math: HF:modeling_gpt2.py:54-72 (softmax(q k^T * 1/sqrt(64) + mask) v, f32); padding semantics
// of prepare_gpt_inputs (gpt/model.py:628-635: keys of left-pad positions masked, quirk Q2).
//
// 1. itts_attn_decode: one new token per sequence.  Appends its k/v (from the QKV projection, f32)
//    into the KV cache at index kv_base + *t (device counter -> hipGraph-replayable), then attends
//    over keys [pad_b, kv_base + *t].  One 256-thread workgroup per (head, sequence), ONE pass over
//    the cache: 8 lanes per key row (one 1 KiB coalesced wave load = 8 rows of K, one of V), online
//    softmax per 8-lane group, log-sum-exp merge of the 32 groups through LDS.  HBM-bound: it
//    streams 2 * S * 64 * sizeof(cache) bytes per (sequence, head).  The c_attn output may arrive
//    as split-K partial slabs (summed here with the bias, so the GEMM needs no reduce pass).
// 2. itts_attn_prefill: variable-length causal attention over packed sequences (prefill of the
//    prompt block, and the teacher-forced latent pass).  One thread per query, K/V staged through
//    LDS in 32-key blocks, block-wise online softmax; optionally writes K/V into the decode cache.
#include "common.h"

namespace {

constexpr int kHD = 64;

template <typename TC>
__device__ __forceinline__ void load8(const TC* p, float (&v)[8]);
template <>
__device__ __forceinline__ void load8<float>(const float* p, float (&v)[8]) {
  const f32x4_t a = *reinterpret_cast<const f32x4_t*>(p), b = *reinterpret_cast<const f32x4_t*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
template <>
__device__ __forceinline__ void load8<uint16_t>(const uint16_t* p, float (&v)[8]) {
  const u32x4_t a = *reinterpret_cast<const u32x4_t*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(a[i] << 16);
    v[2 * i + 1] = __uint_as_float(a[i] & 0xFFFF0000u);
  }
}

constexpr int kMaxKeys = 1 << 20;  // positions are int32; the cache capacity is the caller's

// One workgroup of NT threads per (head, sequence): NT/8 groups of 8 lanes, group g owns keys
// g, g + NT/8, ...; lane d8 holds dims 8*d8 .. 8*d8+7.  The first round's cached K and V rows (KB = 8
// keys per group, kept packed: 256 keys at NT = 256) are requested before anything else -- they do
// not depend on this step's q/k/v -- so their HBM latency overlaps the c_attn slab summation; later
// rounds (S > 256) load in turn.  Scores via 8-lane shuffles, an online softmax per group (running
// max m, sum l, partial output o); the groups merge through LDS.  (Measured alternatives, slower at
// B=32, S~283: 512-thread workgroups; 16 packed keys per group -- 308 VGPRs, 1 wave/SIMD.)
// q/k/v = bias + sum of `nsplit` split-K partial slabs of the c_attn GEMM (stride split_stride).
template <typename TC, typename TO, int NT>
__global__ __launch_bounds__(NT) void attn_decode_kernel(const float* __restrict__ qkv, int64_t ldqkv, int nsplit,
                                                         int64_t split_stride, const float* __restrict__ qkv_bias,
                                                         TC* __restrict__ cache_k, TC* __restrict__ cache_v,
                                                         int64_t cache_bs, int64_t cache_hs, const int32_t* pad,
                                                         int kv_base, const int32_t* __restrict__ tstate,
                                                         TO* __restrict__ out, int64_t ldo, int H) {
  constexpr int NG = NT / 8;
  constexpr int KB = 8;                          // keys per group per round (packed rows in registers)
  constexpr int RW = sizeof(TC) * 8 / 16;       // 16-B vectors per lane per row (bf16: 1, f32: 2)
  __shared__ float qs[kHD], kn[kHD], vn[kHD];
  __shared__ float gm[NG], gl[NG];
  __shared__ float pv[NG][kHD + 1];
  const int h = blockIdx.x, b = blockIdx.y;
  const int D = H * kHD;
  const int kidx = kv_base + tstate[0];
  const int p0 = pad ? pad[b] : 0;
  const int nk = kidx + 1 - p0;  // keys p0 .. kidx; the last one is this step's (from LDS)
  TC* Kc = cache_k + (int64_t)b * cache_bs + (int64_t)h * cache_hs;
  TC* Vc = cache_v + (int64_t)b * cache_bs + (int64_t)h * cache_hs;
  const int g = threadIdx.x >> 3, d8 = threadIdx.x & 7;
  // (1) the first round's cached K/V rows do not depend on this step's q/k/v: issue them first
  u32x4_t kr[KB][RW], vr[KB][RW];
#pragma unroll
  for (int u = 0; u < KB; ++u) {
    const int j = NG * u + g;
    if (j < nk - 1) {
#pragma unroll
      for (int w = 0; w < RW; ++w) {
        kr[u][w] = reinterpret_cast<const u32x4_t*>(Kc + (int64_t)(p0 + j) * kHD + 8 * d8)[w];
        vr[u][w] = reinterpret_cast<const u32x4_t*>(Vc + (int64_t)(p0 + j) * kHD + 8 * d8)[w];
      }
    }
  }
  // (2) q/k/v of this step = bias + sum of the c_attn split-K slabs; new k/v appended to the cache
  if (threadIdx.x < 3 * kHD) {
    const int part = threadIdx.x / kHD, d = threadIdx.x - part * kHD;  // 0: q, 1: k, 2: v
    const int col = part * D + h * kHD + d;
    const float* src = qkv + (int64_t)b * ldqkv + col;
    float v = qkv_bias ? qkv_bias[col] : 0.f;
    // up to 4 slabs loaded together (independent loads in flight), summed in slab order
    float sl[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) sl[s] = s < nsplit ? src[s * split_stride] : 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (s < nsplit) v += sl[s];
    for (int s = 4; s < nsplit; ++s) v += src[s * split_stride];
    if (part == 0) {
      qs[d] = v * 0.125f;  // 1/sqrt(64), exact
    } else if (part == 1) {
      kn[d] = v;
      St<TC>::st(Kc + (int64_t)kidx * kHD + d, v);
    } else {
      vn[d] = v;
      St<TC>::st(Vc + (int64_t)kidx * kHD + d, v);
    }
  }
  __syncthreads();
  float q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) q[e] = qs[8 * d8 + e];
  auto unpack = [&](const u32x4_t (&r)[RW], float (&x)[8]) {
    if constexpr (sizeof(TC) == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[2 * i] = __uint_as_float(r[0][i] << 16);
        x[2 * i + 1] = __uint_as_float(r[0][i] & 0xFFFF0000u);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = __uint_as_float(r[i / 4][i % 4]);
    }
  };
  // (3) online softmax per 8-lane group over rounds of NG*KB keys (one round for S <= 512 at bf16)
  float m = -INFINITY, l = 0.f;
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nk; j0 += NG * KB) {
    if (j0 > 0) {  // later rounds (S > 512): load now
#pragma unroll
      for (int u = 0; u < KB; ++u) {
        const int j = j0 + NG * u + g;
        if (j < nk - 1) {
#pragma unroll
          for (int w = 0; w < RW; ++w) {
            kr[u][w] = reinterpret_cast<const u32x4_t*>(Kc + (int64_t)(p0 + j) * kHD + 8 * d8)[w];
            vr[u][w] = reinterpret_cast<const u32x4_t*>(Vc + (int64_t)(p0 + j) * kHD + 8 * d8)[w];
          }
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
        for (int e = 0; e < 8; ++e) kx[e] = kn[8 * d8 + e];  // this step's key (or padding)
      }
      float part = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) part = fmaf(q[e], kx[e], part);
      part += __shfl_xor(part, 1, 64);
      part += __shfl_xor(part, 2, 64);
      part += __shfl_xor(part, 4, 64);
      s[u] = j < nk ? part : -INFINITY;
      bm = fmaxf(bm, s[u]);
    }
    if (bm == -INFINITY) continue;  // this group has no valid key in the round
    const float mn = fmaxf(m, bm);
    const float corr = __expf(m - mn);  // m = -inf -> 0
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
        for (int e = 0; e < 8; ++e) vx[e] = vn[8 * d8 + e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(pr, vx[e], o[e]);
    }
    m = mn;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) pv[g][8 * d8 + e] = o[e];
  if (d8 == 0) {
    gm[g] = m;
    gl[g] = l;
  }
  __syncthreads();
  if (threadIdx.x < kHD) {
    float M = -INFINITY;
#pragma unroll 8
    for (int i = 0; i < NG; ++i) M = fmaxf(M, gm[i]);
    float L = 0.f, acc = 0.f;
#pragma unroll 8
    for (int i = 0; i < NG; ++i) {
      const float w = __expf(gm[i] - M);  // empty group: exp(-inf) = 0
      L = fmaf(gl[i], w, L);
      acc = fmaf(pv[i][threadIdx.x], w, acc);
    }
    St<TO>::st(out + (int64_t)b * ldo + h * kHD + threadIdx.x, acc / L);
  }
}

constexpr int kQB = 128;  // queries per workgroup (one per thread)
constexpr int kKB = 32;   // keys per LDS block

template <typename TC, typename TO>
__global__ __launch_bounds__(kQB) void attn_prefill_kernel(const float* __restrict__ qkv, int64_t ldqkv,
                                                           const int32_t* __restrict__ seq_start,
                                                           const int32_t* __restrict__ seq_len,
                                                           const int32_t* __restrict__ seq_pad, TC* cache_k,
                                                           TC* cache_v, int64_t cache_bs, int64_t cache_hs,
                                                           TO* __restrict__ out, int64_t ldo, int H) {
  __shared__ float Ks[kKB][kHD], Vs[kKB][kHD];
  const int qb = blockIdx.x, h = blockIdx.y, sq = blockIdx.z;
  const int len = seq_len[sq], p0 = seq_pad ? seq_pad[sq] : 0;
  const int q_lo = qb * kQB;
  if (q_lo >= len) return;
  const int q_hi = min(q_lo + kQB, len);
  const int D = H * kHD;
  const float* base = qkv + (int64_t)seq_start[sq] * ldqkv;
  const int i = q_lo + threadIdx.x;
  const bool active = i < len && i >= p0;
  float q[kHD], o[kHD];
#pragma unroll
  for (int d = 0; d < kHD; ++d) {
    q[d] = active ? base[(int64_t)i * ldqkv + h * kHD + d] * 0.125f : 0.f;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int kb = p0; kb < q_hi; kb += kKB) {
    __syncthreads();
    for (int e = threadIdx.x; e < kKB * kHD; e += kQB) {
      const int r = e / kHD, d = e % kHD, j = kb + r;
      float kv = 0.f, vv = 0.f;
      if (j < len) {
        kv = base[(int64_t)j * ldqkv + D + h * kHD + d];
        vv = base[(int64_t)j * ldqkv + 2 * D + h * kHD + d];
        if (cache_k && j >= q_lo && j < q_hi) {
          St<TC>::st(cache_k + (int64_t)sq * cache_bs + (int64_t)h * cache_hs + (int64_t)j * kHD + d, kv);
          St<TC>::st(cache_v + (int64_t)sq * cache_bs + (int64_t)h * cache_hs + (int64_t)j * kHD + d, vv);
        }
      }
      Ks[r][d] = kv;
      Vs[r][d] = vv;
    }
    __syncthreads();
    if (!active || kb > i) continue;
    const int nvalid = min(kKB, i - kb + 1);
    float s[kKB];
    float bm = -INFINITY;
#pragma unroll
    for (int r = 0; r < kKB; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < kHD; ++d) acc = fmaf(q[d], Ks[r][d], acc);
      s[r] = r < nvalid ? acc : -INFINITY;
      bm = fmaxf(bm, s[r]);
    }
    const float mn = fmaxf(m, bm);
    const float corr = __expf(m - mn);
    l *= corr;
#pragma unroll
    for (int d = 0; d < kHD; ++d) o[d] *= corr;
#pragma unroll
    for (int r = 0; r < kKB; ++r) {
      const float p = __expf(s[r] - mn);
      l += p;
#pragma unroll
      for (int d = 0; d < kHD; ++d) o[d] = fmaf(p, Vs[r][d], o[d]);
    }
    m = mn;
  }
  if (i < len) {
    TO* orow = out + (int64_t)(seq_start[sq] + i) * ldo + h * kHD;
    const float inv = active ? 1.0f / l : 0.f;
#pragma unroll
    for (int d = 0; d < kHD; ++d) St<TO>::st(orow + d, o[d] * inv);
  }
}

}  // namespace

extern "C" int itts_attn_decode(const float* qkv, int64_t ldqkv, int nsplit, int64_t split_stride,
                                const float* qkv_bias, void* cache_k, void* cache_v, int64_t cache_bs,
                                int64_t cache_hs, int smax, const int32_t* pad, int kv_base, const int32_t* tstate,
                                void* out, int64_t ldo, int B, int H, int cache_dtype, int out_dtype, void* stream) {
  const char* fn = "itts_attn_decode";
  ITTS_REQUIRE(B >= 0 && H > 0 && nsplit >= 1, fn, "bad sizes");
  if (B == 0) return 0;
  ITTS_REQUIRE(qkv && cache_k && cache_v && tstate && out, fn, "null pointer");
  ITTS_REQUIRE(smax <= kMaxKeys && cache_hs >= (int64_t)smax * kHD, fn, "bad cache capacity");
  dim3 grid(H, B);
  hipStream_t s = itts::as_stream(stream);
#define ITTS_AD(TC, TO)                                                                                             \
  hipLaunchKernelGGL((attn_decode_kernel<TC, TO, 256>), grid, dim3(256), 0, s, qkv, ldqkv, nsplit, split_stride,    \
                     qkv_bias, (TC*)cache_k, (TC*)cache_v, cache_bs, cache_hs, pad, kv_base, tstate, (TO*)out, ldo, H)
  if (cache_dtype == ITTS_BF16 && out_dtype == ITTS_BF16) ITTS_AD(uint16_t, uint16_t);
  else if (cache_dtype == ITTS_F32 && out_dtype == ITTS_F32) ITTS_AD(float, float);
  else if (cache_dtype == ITTS_BF16) ITTS_AD(uint16_t, float);
  else ITTS_AD(float, uint16_t);
#undef ITTS_AD
  return itts::check_launch(fn);
}

extern "C" int itts_attn_prefill(const float* qkv, int64_t ldqkv, const int32_t* seq_start, const int32_t* seq_len,
                                 const int32_t* seq_pad, int nseq, int max_len, void* cache_k, void* cache_v,
                                 int64_t cache_bs, int64_t cache_hs, void* out, int64_t ldo, int H, int cache_dtype,
                                 int out_dtype, void* stream) {
  const char* fn = "itts_attn_prefill";
  ITTS_REQUIRE(nseq >= 0 && H > 0 && max_len >= 0, fn, "bad sizes");
  if (nseq == 0 || max_len == 0) return 0;
  ITTS_REQUIRE(qkv && seq_start && seq_len && out, fn, "null pointer");
  dim3 grid((max_len + kQB - 1) / kQB, H, nseq);
  hipStream_t s = itts::as_stream(stream);
#define ITTS_AP(TC, TO)                                                                                           \
  hipLaunchKernelGGL((attn_prefill_kernel<TC, TO>), grid, dim3(kQB), 0, s, qkv, ldqkv, seq_start, seq_len, seq_pad, \
                     (TC*)cache_k, (TC*)cache_v, cache_bs, cache_hs, (TO*)out, ldo, H)
  if (cache_dtype == ITTS_BF16 && out_dtype == ITTS_BF16) ITTS_AP(uint16_t, uint16_t);
  else if (cache_dtype == ITTS_F32 && out_dtype == ITTS_F32) ITTS_AP(float, float);
  else if (cache_dtype == ITTS_BF16) ITTS_AP(uint16_t, float);
  else ITTS_AP(float, uint16_t);
#undef ITTS_AP
  return itts::check_launch(fn);
}
