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
//    prompt block, and the teacher-forced latent pass); optionally writes K/V into the decode cache.
//    bf16 mode: MFMA flash attention (attn_prefill_mfma_kernel); f32 verification mode: one thread
//    per query, K/V staged through LDS in 32-key blocks, exact-f32 block-wise online softmax.
#include <cstdlib>

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
// g, g + NT/8, ...; lane d8 holds dims 8*d8 .. 8*d8+7.  Issue order: this step's q/k/v, then the
// round's cached K rows, then its V rows (KB keys per group kept packed in registers: 384 keys per
// round at NT = 256, KB = 12), so the scores start as soon as K has landed while V still streams;
// later rounds are requested while the current one computes.  Scores via 8-lane DPP sums, an online
// softmax per group (running max m, sum l, partial output o); the groups merge through LDS with all
// NT threads.  (Measured alternatives, slower at B=32, S~283: 512-thread workgroups; 16 packed keys
// per group -- 308 VGPRs, 1 wave/SIMD; q/k/v requested after the K/V rows: the first score then
// waited for every K/V byte, 12.7 us at S = 283.)
// q/k/v = bias + sum of `nsplit` split-K partial slabs of the c_attn GEMM (stride split_stride).
// ROWS (beam search): key position p of sequence b lives in cache row kv_rows[b * ld_rows + p] (beams
// share their common prefix, HF's per-step cache reorder becomes this lineage table); this step's
// key/value go to the sequence's own row b.
#ifndef ITTS_ATTN_KB
#define ITTS_ATTN_KB 12
#endif
constexpr int kSub = 4;  // keys per group per online-softmax update (every KB is a multiple of it)
#ifndef ITTS_ATTN_WPS
#define ITTS_ATTN_WPS 1
#endif
#ifndef ITTS_ATTN_GUARD
#define ITTS_ATTN_GUARD 0  // measured slower for every KB at every shape (profiles/ubench_attn_kb_r03.txt)
#endif
#ifndef ITTS_ATTN_PROJ_WPS  // fused c_proj: 256 VGPRs without spills at 1; 2 spills 96 VGPRs
#define ITTS_ATTN_PROJ_WPS 1
#endif
// PROJ (attn.c_proj fused, bf16 product decode): the head's output o_h [64] (f32, never rounded)
// times its 64 rows of the c_proj weight W [H*64][N] (HF Conv1D [in, out] order, bf16) is written as
// the split-K partial part[h][b][0..N) (split = head); itts_residual_reduce_ln sums the H partials
// with the bias and the residual.  W's rows do not depend on this step either: they are requested
// right after the q/k/v slab loads (thread (kh, j) holds rows 64h + 32kh .. +31, columns 8j .. 8j+7)
// and arrive while the keys stream.  The 32 workgroups of one head land on one XCD (dispatch is
// round-robin over XCDs and the grid is head-fastest), so each XCD's L2 holds only 2 heads' rows.
// One kernel boundary and the separate c_proj launch less per layer.
// K/V cache rows are read once per step: non-temporal loads (decode step 816 -> 792 us at C3 vs
// plain loads; the weight stream stays non-temporal too, plain weight loads were slower:
// profiles/nt_ab_r02.txt).  ITTS_KV_NT=0 builds the plain-load variant.
#ifndef ITTS_KV_NT
#define ITTS_KV_NT 1
#endif
// beams (ROWS): the beams of an utterance read the same lineage rows at about the same time (neighbouring
// workgroups of one XCD), so their K/V loads keep the default cache policy -- a non-temporal line is not kept in
// L2 for the next beam's read (round 6, profiles/r06_b3nt.txt); ITTS_BEAM_KV_NT=1: non-temporal as greedy (A/B)
#ifndef ITTS_BEAM_KV_NT
#define ITTS_BEAM_KV_NT 0
#endif
constexpr int kAttnKviMax = 3584;  // beams: keys per row whose lineage indices the kernel stages in LDS
template <typename TC, typename TO, int NT, bool ROWS, bool PROJ, int KB = ITTS_ATTN_KB>
__global__ __launch_bounds__(NT, PROJ ? ITTS_ATTN_PROJ_WPS : ITTS_ATTN_WPS) void attn_decode_kernel(const float* __restrict__ qkv, int64_t ldqkv, int nsplit,
                                                         int64_t split_stride, const float* __restrict__ qkv_bias,
                                                         TC* __restrict__ cache_k, TC* __restrict__ cache_v,
                                                         int64_t cache_bs, int64_t cache_hs, const int32_t* pad,
                                                         int kv_base, const int32_t* __restrict__ tstate,
                                                         TO* __restrict__ out, int64_t ldo, int H,
                                                         const int32_t* __restrict__ kv_rows, int64_t ld_rows,
                                                         const uint16_t* __restrict__ wproj, int N,
                                                         float* __restrict__ part, int64_t part_stride, int64_t ldp) {
  static_assert(!PROJ || NT == 256, "the c_proj epilogue maps 256 threads onto 2 x 128 column slots");
  constexpr int NG = NT / 8;
  // KB: keys per group per round (packed rows in registers)
  constexpr int RW = sizeof(TC) * 8 / 16;       // 16-B vectors per lane per row (bf16: 1, f32: 2)
  __shared__ float qs[kHD], kn[kHD], vn[kHD];
  __shared__ float gm[NG], gl[NG];
  __shared__ float pv[NG + NT / kHD + 1][kHD + 1];  // group partials, then the quarter sums and L
  __shared__ float ofin[PROJ ? kHD : 1];  // PROJ: the merged head output
  const int h = blockIdx.x, b = blockIdx.y;
  const int D = H * kHD;
  const int kidx = kv_base + tstate[0];
  const int p0 = pad ? pad[b] : 0;
  const int nk = kidx + 1 - p0;  // keys p0 .. kidx; the last one is this step's (from LDS)
  TC* Kc = cache_k + (int64_t)b * cache_bs + (int64_t)h * cache_hs;
  TC* Vc = cache_v + (int64_t)b * cache_bs + (int64_t)h * cache_hs;
  const int32_t* rows = ROWS ? kv_rows + (int64_t)b * ld_rows : nullptr;
  // ROWS: the row's lineage indices of keys p0 .. kidx staged in LDS first, so a round's K/V addresses need an
  // LDS read instead of a global load (whose in-order vmcnt wait also waited for the previous round's V rows)
  __shared__ int32_t rws[ROWS ? kAttnKviMax : 1];
  if constexpr (ROWS) {
    for (int i = threadIdx.x; i < nk; i += NT) rws[i] = rows[p0 + i];
    __syncthreads();
  }
  // element offset of key position p (relative to Kc / Vc)
  auto koff = [&](int p) -> int64_t {
    if constexpr (ROWS) return (int64_t)(rws[p - p0] - b) * cache_bs + (int64_t)p * kHD;
    else return (int64_t)p * kHD;
  };
  const int g = threadIdx.x >> 3, d8 = threadIdx.x & 7;
  // (1) q/k/v of this step (bias + sum of the c_attn split-K slabs) are requested FIRST: loads complete
  // in issue order, and everything below waits for them, not for the K/V stream behind them
  const bool qkv_lane = threadIdx.x < 3 * kHD;
  const int which = threadIdx.x / kHD, dq = threadIdx.x - which * kHD;  // 0: q, 1: k, 2: v
  const int col = which * D + h * kHD + dq;
  float sl[4] = {0.f, 0.f, 0.f, 0.f}, qb = 0.f;
  if (qkv_lane) {
    const float* src = qkv + (int64_t)b * ldqkv + col;
    qb = qkv_bias ? qkv_bias[col] : 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) sl[s] = s < nsplit ? src[s * split_stride] : 0.f;
  }
  // (2) this round's cached K rows, then its V rows (the scores need only K).  Every lane loads a valid
  // row (key index clamped into the cache), so the loads are unconditional and retire in order; rows
  // past the round's keys are never used.
  u32x4_t kr[KB][RW] = {}, vr[KB][RW] = {};
  auto kv_load = [&](u32x4_t (&dst)[KB][RW], const TC* base, int j0) {
#pragma unroll
    for (int u = 0; u < KB; ++u) {
#if ITTS_ATTN_GUARD
      // slots whose whole 8-row block lies past the keys are not loaded (workgroup-uniform test): a
      // short sequence (long-form chunks, early steps) does not pay KB rows per lane; such slots are
      // never read (keys j >= nk - 1 take this step's k / v from LDS)
      if (j0 + NG * u >= nk - 1) continue;
#endif
      const int j = min(j0 + NG * u + g, max(nk - 2, 0));
#pragma unroll
      for (int w = 0; w < RW; ++w) {
        const u32x4_t* src = reinterpret_cast<const u32x4_t*>(base + koff(p0 + j) + 8 * d8) + w;
        if constexpr (ITTS_KV_NT && (!ROWS || ITTS_BEAM_KV_NT))
          dst[u][w] = __builtin_nontemporal_load(src);
        else
          dst[u][w] = *src;
      }
    }
  };
  kv_load(kr, Kc, 0);
  kv_load(vr, Vc, 0);
  // (2b) PROJ: this head's 64 rows of W (needed last: requested last)
  constexpr int PK = PROJ ? kHD / 2 : 1;
  const int kh = threadIdx.x >> 7, pj = threadIdx.x & 127, n0 = 8 * pj;
  u32x4_t wr[PK];
  if constexpr (PROJ) {
    if (n0 < N) {
      const uint16_t* wsrc = wproj + (int64_t)(h * kHD + kh * PK) * N + n0;
#pragma unroll
      for (int k = 0; k < PK; ++k) wr[k] = *reinterpret_cast<const u32x4_t*>(wsrc + (int64_t)k * N);
    }
  }
  // (3) finish q/k/v; this step's k/v appended to the cache
  if (qkv_lane) {
    float v = qb;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (s < nsplit) v += sl[s];
    for (int s = 4; s < nsplit; ++s) v += qkv[(int64_t)b * ldqkv + col + s * split_stride];
    if (which == 0) {
      qs[dq] = v * 0.125f;  // 1/sqrt(64), exact
    } else if (which == 1) {
      kn[dq] = v;
      St<TC>::st(Kc + (int64_t)kidx * kHD + dq, v);
    } else {
      vn[dq] = v;
      St<TC>::st(Vc + (int64_t)kidx * kHD + dq, v);
    }
  }
  __syncthreads();
  float q[8], kme[8], vme[8];  // q, and this step's own key / value (the last key, from LDS)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    q[e] = qs[8 * d8 + e];
    kme[e] = kn[8 * d8 + e];
    vme[e] = vn[8 * d8 + e];
  }
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
  // (4) online softmax per 8-lane group over rounds of NG*KB keys.  Software-pipelined: the next
  // round's K rows are requested as soon as this round's scores no longer need kr, its V rows once
  // this round's P.V is done.  The softmax itself advances in fixed chunks of kSub keys per group
  // whatever KB is (KB only sets how far the loads run ahead), so the rounding of a row's result does
  // not depend on the KB the launcher picked for its batch size: a row decodes bit-identically alone
  // and inside a 128-row long-form chunk.
  static_assert(KB % kSub == 0, "keys per round must be a multiple of the softmax chunk");
  float m = -INFINITY, l = 0.f;
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nk; j0 += NG * KB) {
    const bool more = j0 + NG * KB < nk;
    float s[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int j = j0 + NG * u + g;
      float kx[8];
      unpack(kr[u], kx);
      if (j >= nk - 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) kx[e] = kme[e];  // this step's key (or padding)
      }
      float pt = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) pt = fmaf(q[e], kx[e], pt);
      pt = sum8_dpp(pt);
      s[u] = j < nk ? pt : -INFINITY;
    }
    if (more) kv_load(kr, Kc, j0 + NG * KB);
#pragma unroll
    for (int c0 = 0; c0 < KB; c0 += kSub) {
      float bm = -INFINITY;
#pragma unroll
      for (int u = c0; u < c0 + kSub; ++u) bm = fmaxf(bm, s[u]);
      if (bm == -INFINITY) continue;  // this group has no valid key in the chunk
      const float mn = fmaxf(m, bm);
      const float corr = __expf(m - mn);  // m = -inf -> 0
      l *= corr;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= corr;
#pragma unroll
      for (int u = c0; u < c0 + kSub; ++u) {
        const int j = j0 + NG * u + g;
        const float pr = __expf(s[u] - mn);
        l += pr;
        float vx[8];
        unpack(vr[u], vx);
        if (j >= nk - 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) vx[e] = vme[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = fmaf(pr, vx[e], o[e]);
      }
      m = mn;
    }
    if (more) kv_load(vr, Vc, j0 + NG * KB);
  }
  // (5) merge the NG groups: every thread takes the max M, then quarter qd of the block sums groups
  // 8qd .. 8qd+7 for its dim, the quarters combine in order (fixed-order sums: batch-invariant)
#pragma unroll
  for (int e = 0; e < 8; ++e) pv[g][8 * d8 + e] = o[e];
  if (d8 == 0) {
    gm[g] = m;
    gl[g] = l;
  }
  __syncthreads();
  constexpr int NQ = NT / kHD, GPQ = NG / NQ;  // quarters, groups per quarter
  float* qsum = &pv[0][0] + NG * (kHD + 1);     // [NQ][kHD + 1] after pv
  float* lsum = qsum + NQ * (kHD + 1);          // [NQ]
  {
    const int dd = threadIdx.x & (kHD - 1), qd = threadIdx.x / kHD;
    float M = -INFINITY;
#pragma unroll 8
    for (int i = 0; i < NG; ++i) M = fmaxf(M, gm[i]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int i = qd * GPQ; i < qd * GPQ + GPQ; ++i) {
      const float w = __expf(gm[i] - M);  // empty group: exp(-inf) = 0
      L = fmaf(gl[i], w, L);
      acc = fmaf(pv[i][dd], w, acc);
    }
    qsum[qd * (kHD + 1) + dd] = acc;
    if (dd == 0) lsum[qd] = L;
  }
  __syncthreads();
  if (threadIdx.x < kHD) {
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      L += lsum[i];
      acc += qsum[i * (kHD + 1) + threadIdx.x];
    }
    if constexpr (PROJ) ofin[threadIdx.x] = acc / L;
    else St<TO>::st(out + (int64_t)b * ldo + h * kHD + threadIdx.x, acc / L);
  }
  if constexpr (PROJ) {
    // (4) part[h][b][n] = sum_d o_h[d] * W[64h + d][n]: each half of the workgroup sums 32 rows of W,
    // the halves combine through LDS in a fixed order (rows 0..31, then 32..63)
    __syncthreads();
    float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (n0 < N) {
#pragma unroll
      for (int k = 0; k < PK; ++k) {
        const float ov = ofin[kh * PK + k];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a8[2 * i] = fmaf(ov, __uint_as_float(wr[k][i] << 16), a8[2 * i]);
          a8[2 * i + 1] = fmaf(ov, __uint_as_float(wr[k][i] & 0xFFFF0000u), a8[2 * i + 1]);
        }
      }
    }
    float* xch = &pv[0][0];  // [8][128]: pv's last readers (the merge) are past the barrier above
    if (kh == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) xch[e * 128 + pj] = a8[e];
    }
    __syncthreads();
    if (kh == 0 && n0 < N) {
#pragma unroll
      for (int e = 0; e < 8; ++e) a8[e] += xch[e * 128 + pj];
      f32x4_t* dst = reinterpret_cast<f32x4_t*>(part + (int64_t)h * part_stride + (int64_t)b * ldp + n0);
      dst[0] = f32x4_t{a8[0], a8[1], a8[2], a8[3]};
      dst[1] = f32x4_t{a8[4], a8[5], a8[6], a8[7]};
    }
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

// ---- MFMA flash-attention prefill (bf16 operands, f32 softmax / accumulation) -----------------
// Used in bf16 mode (cache dtype bf16): one 256-thread workgroup = 128 queries (4 waves x 32) of one
// head of one packed sequence.  Per 32-key tile: S^T = K . Q^T on v_mfma_f32_32x32x16_bf16 (keys
// are the MFMA rows, the wave's 32 queries its columns, so every lane owns one query and a row
// softmax is 16 in-lane values + one xor-32 shuffle), online softmax, then O^T += V^T . P^T with P
// re-packed to the B-fragment layout by one xor-32 exchange per 16 keys.  K is staged in LDS as
// [key][dim] and V transposed as [dim][key] (bf16, padded rows), so every MFMA fragment is one
// ds_read_b128.  Masks: causal, left padding (keys < pad) and the sequence length.  Keys of this
// workgroup's query range are written to the decode KV cache while staging.
constexpr int kFQ = 128;  // queries per workgroup
constexpr int kFK = 32;   // keys per tile
constexpr int kKP = 64 * 2 + 16;   // K tile row pitch (bytes)
constexpr int kVP = kFK * 2 + 16;  // V^T tile row pitch (bytes)

template <typename TO>
__global__ __launch_bounds__(256) void attn_prefill_mfma_kernel(const float* __restrict__ qkv, int64_t ldqkv,
                                                                const int32_t* __restrict__ seq_start,
                                                                const int32_t* __restrict__ seq_len,
                                                                const int32_t* __restrict__ seq_pad,
                                                                uint16_t* cache_k, uint16_t* cache_v, int64_t cache_bs,
                                                                int64_t cache_hs, TO* __restrict__ out, int64_t ldo,
                                                                int H) {
  __shared__ __attribute__((aligned(16))) unsigned char Ks[kFK * kKP];
  __shared__ __attribute__((aligned(16))) unsigned char Vt[64 * kVP];
  const int qb = blockIdx.x, h = blockIdx.y, sq = blockIdx.z;
  const int len = seq_len[sq], p0 = seq_pad ? seq_pad[sq] : 0;
  const int q_lo = qb * kFQ;
  if (q_lo >= len) return;
  const int q_hi = min(q_lo + kFQ, len);
  const int D = H * kHD;
  const float* base = qkv + (int64_t)seq_start[sq] * ldqkv + h * kHD;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int q = q_lo + 32 * wave + r32;  // this lane's query
  const bool qv = q < len && q >= p0;
  // Q^T B-fragments: lane (q, hh) holds Q[q][16ks + 8hh .. +7] * 1/8 (exact), bf16
  bf16x8_t qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    float t[8];
    if (q < len) {
      const f32x4_t a = *reinterpret_cast<const f32x4_t*>(base + (int64_t)q * ldqkv + 16 * ks + 8 * hh);
      const f32x4_t b = *reinterpret_cast<const f32x4_t*>(base + (int64_t)q * ldqkv + 16 * ks + 8 * hh + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) { t[i] = a[i] * 0.125f; t[4 + i] = b[i] * 0.125f; }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) qf[ks][i] = (__bf16)t[i];
  }
  f32x16_t o[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int kmax = min(q_hi, len);  // keys [p0, kmax) can be attended by this block
  // key tiles start at the first valid key p0 (not at a multiple of 32): the partition of a
  // sequence's keys into tiles -- and so its f32 rounding -- does not depend on its left padding
  // (batch invariance: a row decodes the same ids in a padded batch as alone, padding_test.py)
  for (int k0 = p0; k0 < kmax; k0 += kFK) {
    __syncthreads();  // previous tile fully consumed
    {  // stage K [key][dim] and V^T [dim][key] (bf16); write the cache for keys of this block's range
      const int kk = tid >> 3, d0 = (tid & 7) * 8, key = k0 + kk;
      float kv[8], vv[8];
      if (key < len) {
        const float* kr = base + (int64_t)key * ldqkv + D + d0;
        const float* vr = base + (int64_t)key * ldqkv + 2 * D + d0;
        const f32x4_t k0v = *reinterpret_cast<const f32x4_t*>(kr), k1v = *reinterpret_cast<const f32x4_t*>(kr + 4);
        const f32x4_t v0v = *reinterpret_cast<const f32x4_t*>(vr), v1v = *reinterpret_cast<const f32x4_t*>(vr + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) { kv[i] = k0v[i]; kv[4 + i] = k1v[i]; vv[i] = v0v[i]; vv[4 + i] = v1v[i]; }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) kv[i] = vv[i] = 0.f;
      }
      u32x4_t kp;
#pragma unroll
      for (int i = 0; i < 4; ++i) kp[i] = pack2bf(kv[2 * i], kv[2 * i + 1]);
      *reinterpret_cast<u32x4_t*>(Ks + kk * kKP + d0 * 2) = kp;
#pragma unroll
      for (int i = 0; i < 8; ++i) *reinterpret_cast<uint16_t*>(Vt + (d0 + i) * kVP + kk * 2) = f2bf(vv[i]);
      if (cache_k && key >= q_lo && key < q_hi) {
        uint16_t* ck = cache_k + (int64_t)sq * cache_bs + (int64_t)h * cache_hs + (int64_t)key * kHD + d0;
        uint16_t* cv = cache_v + (int64_t)sq * cache_bs + (int64_t)h * cache_hs + (int64_t)key * kHD + d0;
        *reinterpret_cast<u32x4_t*>(ck) = kp;
        u32x4_t vp;
#pragma unroll
        for (int i = 0; i < 4; ++i) vp[i] = pack2bf(vv[2 * i], vv[2 * i + 1]);
        *reinterpret_cast<u32x4_t*>(cv) = vp;
      }
    }
    __syncthreads();
    if (k0 > q_lo + 32 * wave + 31) continue;  // the whole tile is in this wave's causal future
    // S^T[key][q] for keys k0 + (r&3) + 8(r>>2) + 4hh
    f32x16_t s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(Ks + r32 * kKP + ks * 32 + hh * 16);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s, 0, 0, 0);
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (!qv || key > q || key < p0 || key >= len) s[r] = -INFINITY;
      tmax = fmaxf(tmax, s[r]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    float psum = 0.f;
    float pr[16];
    if (mn == -INFINITY) {  // nothing valid yet for this query
#pragma unroll
      for (int r = 0; r < 16; ++r) pr[r] = 0.f;
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        pr[r] = __expf(s[r] - mn);
        psum += pr[r];
      }
      const float corr = __expf(m - mn);
      l = l * corr + psum + __shfl_xor(psum, 32, 64);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= corr;
      m = mn;
    }
    // P^T B-fragments: lane (q, hh) needs P[q][keys 16ks + 8hh .. +7]; it holds keys
    // {8j + 4hh + 0..3}: exchange one half with the xor-32 partner
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ra = 8 * ks, rb = 8 * ks + 4;  // regs of keys 16ks + 4hh + 0..3 and 16ks + 8 + 4hh + 0..3
      const uint32_t own_lo = pack2bf(pr[ra], pr[ra + 1]), own_hi = pack2bf(pr[ra + 2], pr[ra + 3]);
      const uint32_t own2_lo = pack2bf(pr[rb], pr[rb + 1]), own2_hi = pack2bf(pr[rb + 2], pr[rb + 3]);
      // hh = 0 sends keys 8..11 (rb regs), hh = 1 sends keys 4..7 of the pair (ra regs)
      const uint32_t send_lo = hh ? own_lo : own2_lo, send_hi = hh ? own_hi : own2_hi;
      const uint32_t recv_lo = __shfl_xor(send_lo, 32, 64), recv_hi = __shfl_xor(send_hi, 32, 64);
      u32x4_t pf;
      if (hh == 0) {  // keys 16ks + 0..3 (own ra) then 4..7 (partner's ra)
        pf = u32x4_t{own_lo, own_hi, recv_lo, recv_hi};
      } else {        // keys 16ks + 8..11 (partner's rb) then 12..15 (own rb)
        pf = u32x4_t{recv_lo, recv_hi, own2_lo, own2_hi};
      }
      const bf16x8_t pb = *reinterpret_cast<const bf16x8_t*>(&pf);
#pragma unroll
      for (int i = 0; i < 2; ++i) {  // O^T rows d = 32i + .. : A = V^T[d][keys 16ks + 8hh ..]
        const bf16x8_t vf = *reinterpret_cast<const bf16x8_t*>(Vt + (32 * i + r32) * kVP + ks * 32 + hh * 16);
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb, o[i], 0, 0, 0);
      }
    }
  }
  if (q >= len) return;
  const float inv = (qv && l > 0.f) ? 1.0f / l : 0.f;
  TO* orow = out + (int64_t)(seq_start[sq] + q) * ldo + h * kHD;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) St<TO>::st(orow + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh, o[i][r] * inv);
}

}  // namespace

namespace {
int attn_decode_launch(const char* fn, const float* qkv, int64_t ldqkv, int nsplit, int64_t split_stride,
                       const float* qkv_bias, void* cache_k, void* cache_v, int64_t cache_bs, int64_t cache_hs,
                       int smax, const int32_t* pad, int kv_base, const int32_t* tstate, void* out, int64_t ldo,
                       int B, int H, int cache_dtype, int out_dtype, const int32_t* kv_rows, int64_t ld_rows,
                       const void* wproj, int N, float* part, int64_t part_stride, int64_t ldp, void* stream) {
  ITTS_REQUIRE(B >= 0 && H > 0 && nsplit >= 1, fn, "bad sizes");
  if (B == 0) return 0;
  ITTS_REQUIRE(qkv && cache_k && cache_v && tstate && (out || wproj), fn, "null pointer");
  ITTS_REQUIRE(smax <= kMaxKeys && cache_hs >= (int64_t)smax * kHD, fn, "bad cache capacity");
  ITTS_REQUIRE(!kv_rows || smax <= kAttnKviMax, fn, "beam decoding: at most 3584 keys per row (LDS lineage)");
  ITTS_REQUIRE(!wproj || (part && N > 0 && N <= 1024 && N % 8 == 0 && ldp >= N && ldp % 4 == 0 &&
                          part_stride % 4 == 0 &&
                          ((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(wproj)) & 15) == 0),
               fn, "c_proj partials need N % 8 == 0, N <= 1024 and 16-B aligned rows");
  dim3 grid(H, B);
  hipStream_t s = itts::as_stream(stream);
  const uint16_t* wp = static_cast<const uint16_t*>(wproj);
  // keys per group per round (the load depth only: the softmax runs in kSub-key chunks whatever KB is,
  // so the choice below never changes a result bit): 12 (384 keys per workgroup round) for the 32-row
  // steps (round 3 measured 10; KB must now be a multiple of kSub), 4 for steps of
  // >= 128 rows (long-form chunks), whose 2048+ workgroups are occupancy-bound at 10 -- B = 128: S = 71
  // 23.8 -> 15.5 us, S = 300 31.1 vs 31.7 (profiles/ubench_attn_kb_r03.txt) -- and for the beam
  // lineage form at any row count: its beams re-read a shared prefix out of L2, so 4 workgroups per CU
  // (120 VGPRs) beat 2 (224): beam3 C3 757 -> 787 audio-s/s.  A per-utterance form (the beams of one
  // utterance in one workgroup, each shared row loaded once) was slower still: 744
  // (profiles/beam_attn_ab_r03.txt).
  static const bool small_ok = [] {  // ITTS_ATTN_SMALLKB=0: always 10 (A/B)
    const char* e = getenv("ITTS_ATTN_SMALLKB");
    return !(e && e[0] == '0');
  }();
  const bool small_kb = small_ok && (B >= 128 || kv_rows) && !wproj;
#define ITTS_AD1(TC, TO, PR, KBV)                                                                                     \
  do {                                                                                                            \
    if (kv_rows)                                                                                                  \
      hipLaunchKernelGGL((attn_decode_kernel<TC, TO, 256, true, PR, KBV>), grid, dim3(256), 0, s, qkv, ldqkv,      \
                         nsplit, split_stride, qkv_bias, (TC*)cache_k, (TC*)cache_v, cache_bs, cache_hs, pad,       \
                         kv_base, tstate, (TO*)out, ldo, H, kv_rows, ld_rows, wp, N, part, part_stride, ldp);       \
    else                                                                                                          \
      hipLaunchKernelGGL((attn_decode_kernel<TC, TO, 256, false, PR, KBV>), grid, dim3(256), 0, s, qkv, ldqkv,     \
                         nsplit, split_stride, qkv_bias, (TC*)cache_k, (TC*)cache_v, cache_bs, cache_hs, pad,       \
                         kv_base, tstate, (TO*)out, ldo, H, nullptr, 0, wp, N, part, part_stride, ldp);             \
  } while (0)
#define ITTS_AD(TC, TO, PR)                  \
  do {                                       \
    if (!PR && small_kb) ITTS_AD1(TC, TO, false, 4); \
    else ITTS_AD1(TC, TO, PR, ITTS_ATTN_KB); \
  } while (0)
  if (wproj) {
    if (cache_dtype == ITTS_BF16) ITTS_AD(uint16_t, float, true);
    else ITTS_AD(float, float, true);
  } else if (cache_dtype == ITTS_BF16 && out_dtype == ITTS_BF16) {
    ITTS_AD(uint16_t, uint16_t, false);
  } else if (cache_dtype == ITTS_F32 && out_dtype == ITTS_F32) {
    ITTS_AD(float, float, false);
  } else if (cache_dtype == ITTS_BF16) {
    ITTS_AD(uint16_t, float, false);
  } else {
    ITTS_AD(float, uint16_t, false);
  }
#undef ITTS_AD
#undef ITTS_AD1
  return itts::check_launch(fn);
}
}  // namespace

extern "C" int itts_attn_decode(const float* qkv, int64_t ldqkv, int nsplit, int64_t split_stride,
                                const float* qkv_bias, void* cache_k, void* cache_v, int64_t cache_bs,
                                int64_t cache_hs, int smax, const int32_t* pad, int kv_base, const int32_t* tstate,
                                void* out, int64_t ldo, int B, int H, int cache_dtype, int out_dtype, void* stream) {
  return attn_decode_launch("itts_attn_decode", qkv, ldqkv, nsplit, split_stride, qkv_bias, cache_k, cache_v,
                            cache_bs, cache_hs, smax, pad, kv_base, tstate, out, ldo, B, H, cache_dtype, out_dtype,
                            nullptr, 0, nullptr, 0, nullptr, 0, 0, stream);
}

extern "C" int itts_attn_decode_proj(const float* qkv, int64_t ldqkv, int nsplit, int64_t split_stride,
                                     const float* qkv_bias, void* cache_k, void* cache_v, int64_t cache_bs,
                                     int64_t cache_hs, int smax, const int32_t* pad, int kv_base,
                                     const int32_t* tstate, const void* w_proj, int N, float* part,
                                     int64_t part_stride, int64_t ldp, int B, int H, int cache_dtype,
                                     const int32_t* kv_rows, int64_t ld_rows, void* stream) {
  const char* fn = "itts_attn_decode_proj";
  ITTS_REQUIRE(w_proj, fn, "w_proj required");
  ITTS_REQUIRE(!kv_rows || ld_rows >= smax, fn, "kv_rows [B][ld_rows >= smax] required");
  ITTS_REQUIRE(!kv_rows || smax <= kAttnKviMax, fn, "beam decoding: at most 3584 keys per row");
  return attn_decode_launch(fn, qkv, ldqkv, nsplit, split_stride, qkv_bias, cache_k, cache_v, cache_bs, cache_hs,
                            smax, pad, kv_base, tstate, nullptr, 0, B, H, cache_dtype, ITTS_F32, kv_rows, ld_rows,
                            w_proj, N, part, part_stride, ldp, stream);
}

extern "C" int itts_attn_decode_rows(const float* qkv, int64_t ldqkv, int nsplit, int64_t split_stride,
                                     const float* qkv_bias, void* cache_k, void* cache_v, int64_t cache_bs,
                                     int64_t cache_hs, int smax, const int32_t* pad, int kv_base,
                                     const int32_t* tstate, void* out, int64_t ldo, int B, int H, int cache_dtype,
                                     int out_dtype, const int32_t* kv_rows, int64_t ld_rows, void* stream) {
  const char* fn = "itts_attn_decode_rows";
  ITTS_REQUIRE(kv_rows && ld_rows >= smax, fn, "kv_rows [B][ld_rows >= smax] required");
  ITTS_REQUIRE(smax <= kAttnKviMax, fn, "beam decoding: at most 3584 keys per row");
  return attn_decode_launch(fn, qkv, ldqkv, nsplit, split_stride, qkv_bias, cache_k, cache_v, cache_bs, cache_hs,
                            smax, pad, kv_base, tstate, out, ldo, B, H, cache_dtype, out_dtype, kv_rows, ld_rows,
                            nullptr, 0, nullptr, 0, 0, stream);
}

extern "C" int itts_attn_prefill(const float* qkv, int64_t ldqkv, const int32_t* seq_start, const int32_t* seq_len,
                                 const int32_t* seq_pad, int nseq, int max_len, void* cache_k, void* cache_v,
                                 int64_t cache_bs, int64_t cache_hs, void* out, int64_t ldo, int H, int cache_dtype,
                                 int out_dtype, void* stream) {
  const char* fn = "itts_attn_prefill";
  ITTS_REQUIRE(nseq >= 0 && H > 0 && max_len >= 0, fn, "bad sizes");
  if (nseq == 0 || max_len == 0) return 0;
  ITTS_REQUIRE(qkv && seq_start && seq_len && out, fn, "null pointer");
  hipStream_t s = itts::as_stream(stream);
  if (cache_dtype == ITTS_BF16 && (ldqkv % 4) == 0 && ((reinterpret_cast<uintptr_t>(qkv) & 15) == 0)) {
    dim3 gridf((max_len + kFQ - 1) / kFQ, H, nseq);  // product (bf16) mode: MFMA flash attention
    if (out_dtype == ITTS_BF16)
      hipLaunchKernelGGL((attn_prefill_mfma_kernel<uint16_t>), gridf, dim3(256), 0, s, qkv, ldqkv, seq_start, seq_len,
                         seq_pad, (uint16_t*)cache_k, (uint16_t*)cache_v, cache_bs, cache_hs, (uint16_t*)out, ldo, H);
    else
      hipLaunchKernelGGL((attn_prefill_mfma_kernel<float>), gridf, dim3(256), 0, s, qkv, ldqkv, seq_start, seq_len,
                         seq_pad, (uint16_t*)cache_k, (uint16_t*)cache_v, cache_bs, cache_hs, (float*)out, ldo, H);
    return itts::check_launch(fn);
  }
  dim3 grid((max_len + kQB - 1) / kQB, H, nseq);  // verification (f32) mode: exact f32 VALU kernel
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
