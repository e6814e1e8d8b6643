// Block-wide warper thresholds for token selection over a whole vocabulary row staged in LDS, for any
// top_k and top-p-only sampling (the register / repeated-argmax fast paths cover 0 < top_k <= 64).
//
//   TopKLogitsWarper (HF generation/logits_process.py): keep every score >= the k-th largest score
//     (ties kept; k = max(top_k, min_tokens_to_keep)).  Exact k-th largest by a 4-pass 8-bit radix
//     select over order-preserving 32-bit keys, integer histogram counts (deterministic).
//   TopPLogitsWarper: sort ascending, cumulative softmax, drop tokens while the cumulative probability
//     <= 1 - top_p, keep the last min_tokens_to_keep.  With distinct scores token j survives iff the
//     probability mass of the tokens scoring strictly above it is < top_p, so the survivors are the
//     keys >= T* = min{T : mass(key > T) < top_p}; T* by bitwise descent over the key space with
//     fixed-order block sums (deterministic; 32 passes).
// One 256-thread block per row; `sc` = the row's processed scores [V] in LDS (-inf = removed).
#pragma once
#include "common.h"

namespace itts_select {

constexpr int kT = 256;
constexpr int kRegRow = 36;  // register-resident row in the top-p descent: V <= 256 x 36 (IndexTTS: 8194)

// order-preserving float -> uint32 (larger float, larger key; -inf maps below every finite score)
__device__ __forceinline__ uint32_t okey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// fixed-order block sum (wave butterfly, then the 4 waves in order); every thread gets the result
__device__ __forceinline__ float block_sum_fixed(float v, float* red4) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red4[w] = v;
  __syncthreads();
  return (red4[0] + red4[1]) + (red4[2] + red4[3]);
}

__device__ __forceinline__ float block_max(float v, float* red4) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red4[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3]));
}

// Top-k extraction loops: 1 = a winner's owner takes its cached second best as its next candidate
// (rescans only when it wins twice), 0 = the owner rescans its registers after every win.
#ifndef ITTS_TOPK_CACHE2
#define ITTS_TOPK_CACHE2 1
#endif

// (score desc, index asc) order of the top-k extraction loops
__device__ __forceinline__ bool before(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

// Best two of a thread's register-resident scores s[i] (token idx(i)) among those that come after
// (lv, li) in the extraction order (every score before it has already left).  The top-k loops keep
// the second as the owner's next candidate, so a winner's owner rescans only when it wins twice.
struct Top2 {
  float b1;
  int i1;
  float b2;
  int i2;
};
template <int N, typename IdxF>
__device__ __forceinline__ Top2 top2_after(const float (&s)[N], IdxF idx, float lv, int li) {
  Top2 r{-INFINITY, 0x7fffffff, -INFINITY, 0x7fffffff};
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int t = idx(i);
    const float x = s[i];
    const bool ok = before(lv, li, x, t);
    const bool f1 = ok && before(x, t, r.b1, r.i1);
    const bool f2 = ok && !f1 && before(x, t, r.b2, r.i2);
    // branch-free: every lane runs the same selects (the owner is a single lane)
    r.b2 = f1 ? r.b1 : (f2 ? x : r.b2);
    r.i2 = f1 ? r.i1 : (f2 ? t : r.i2);
    r.b1 = f1 ? x : r.b1;
    r.i1 = f1 ? t : r.i1;
  }
  return r;
}

// (score, token) as one 64-bit key whose unsigned order is the extraction order: hi = okey(score)
// (zeros canonicalised: -0 and +0 compare equal as floats, the token then decides), lo = ~token.
// NaN maps to 0 (below every score, decodes to NaN, which ends a top-k loop as before()'s never-winning
// NaN does).
struct Key64 {
  uint32_t hi, lo;
};
__device__ __forceinline__ Key64 key64(float v, int t) {
  if (!(v == v)) return {0u, 0u};
  return {okey(v + 0.0f), ~(uint32_t)t};
}
__device__ __forceinline__ float key64_score(const Key64& k) {
  return __uint_as_float((k.hi & 0x80000000u) ? (k.hi & 0x7fffffffu) : ~k.hi);
}
__device__ __forceinline__ bool key64_gt(const Key64& a, const Key64& b) {
  return (a.hi > b.hi) | ((a.hi == b.hi) & (a.lo > b.lo));
}
template <int CTRL>
__device__ __forceinline__ void key64_max_dpp(Key64& k) {
  const Key64 o{(uint32_t)__builtin_amdgcn_mov_dpp((int)k.hi, CTRL, 0xF, 0xF, false),
                (uint32_t)__builtin_amdgcn_mov_dpp((int)k.lo, CTRL, 0xF, 0xF, false)};
  const bool t = key64_gt(o, k);
  k.hi = t ? o.hi : k.hi;
  k.lo = t ? o.lo : k.lo;
}
// wave-wide max key, uniform in every lane: DPP within each 16-lane row (quad_perm xor 1, xor 2,
// row_half_mirror, row_mirror -- VALU operands, no LDS round trip), then the 4 row maxima by readlane
__device__ __forceinline__ Key64 wave_max_key64(Key64 k) {
  key64_max_dpp<0xB1>(k);   // quad_perm [1,0,3,2]
  key64_max_dpp<0x4E>(k);   // quad_perm [2,3,0,1]
  key64_max_dpp<0x141>(k);  // row_half_mirror
  key64_max_dpp<0x140>(k);  // row_mirror
  Key64 w{(uint32_t)__builtin_amdgcn_readlane((int)k.hi, 0), (uint32_t)__builtin_amdgcn_readlane((int)k.lo, 0)};
#pragma unroll
  for (int r = 1; r < 4; ++r) {
    const Key64 o{(uint32_t)__builtin_amdgcn_readlane((int)k.hi, 16 * r),
                  (uint32_t)__builtin_amdgcn_readlane((int)k.lo, 16 * r)};
    if (key64_gt(o, w)) w = o;
  }
  return w;
}

// key of the k-th largest score (1 <= k <= V); hist: 256 ints of LDS, bc: 2 ints of LDS (kT == 256:
// one thread per histogram bin)
__device__ inline uint32_t kth_largest_key(const float* sc, int V, int k, int* hist, int* bc) {
  uint32_t prefix = 0, mask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += kT) hist[i] = 0;
    __syncthreads();
    for (int v = threadIdx.x; v < V; v += kT) {
      const uint32_t kv = okey(sc[v]);
      if ((kv & mask) == prefix) atomicAdd(&hist[(kv >> shift) & 255u], 1);
    }
    __syncthreads();
    // the digit: the largest d with count(bins > d) < k <= count(bins >= d) (d = 0 if none), by a
    // suffix scan over the 256 bins -- thread i owns bin 255 - i (wave scan, then the waves in order)
    {
      __shared__ int wtot[kT / 64];
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, d = 255 - (int)threadIdx.x;
      const int c = hist[d];
      int incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int up = __shfl_up(incl, o, 64);
        if (lane >= o) incl += up;
      }
      if (lane == 63) wtot[w] = incl;
      __syncthreads();
      for (int ww = 0; ww < w; ++ww) incl += wtot[ww];
      const int excl = incl - c;
      if (excl < k && (incl >= k || d == 0)) {
        bc[0] = d;
        bc[1] = k - excl;
      }
    }
    __syncthreads();
    prefix |= (uint32_t)bc[0] << shift;
    mask |= 0xFFu << shift;
    k = bc[1];
    __syncthreads();  // bc / hist reused by the next pass
  }
  return prefix;
}

// HF TopK (k > 0; 0 = off) then TopP (top_p < 1; renormalised over the TopK survivors) with
// min_keep survivors: returns T, the survivors being the scores whose okey() >= T.
__device__ inline uint32_t warper_threshold(const float* sc, int V, int top_k, float top_p, int min_keep, int* hist,
                                            int* bc, float* red4) {
  uint32_t tk = 0;  // TopK threshold key (0: keep all)
  if (top_k > 0) {
    const int k = top_k < min_keep ? min_keep : top_k;
    if (k < V) tk = kth_largest_key(sc, V, k, hist, bc);
  }
  if (!(top_p < 1.f)) return tk;
  if (!(top_p > 0.f)) {  // nothing survives the cumulative test: only the min_keep best remain
    const uint32_t kmin = kth_largest_key(sc, V, min_keep < V ? min_keep : V, hist, bc);
    return kmin > tk ? kmin : tk;
  }
  // softmax over the TopK survivors: m = max, Z = sum exp(s - m)
  float mx = -INFINITY;
  for (int v = threadIdx.x; v < V; v += kT)
    if (okey(sc[v]) >= tk) mx = fmaxf(mx, sc[v]);
  mx = block_max(mx, red4);
  if (mx == -INFINITY) return tk;
  float z = 0.f;
  for (int v = threadIdx.x; v < V; v += kT)
    if (okey(sc[v]) >= tk) z += __expf(sc[v] - mx);
  z = block_sum_fixed(z, red4);
  const float target = top_p * z;
  // mass(T) = sum over survivors with key > T; non-increasing in T.  cur = the largest T with
  // mass(T) >= target (mass(0) = z >= target), built bit by bit; T* = cur + 1.
  uint32_t cur = 0;
  if (V <= kT * kRegRow) {
    // the row's keys and exps held in registers once (same terms, same order as below; excluded
    // entries add +0, which leaves a sum bitwise unchanged): 32 passes of compares and adds
    uint32_t kr[kRegRow];
    float er[kRegRow];
#pragma unroll
    for (int j = 0; j < kRegRow; ++j) {
      const int v = threadIdx.x + kT * j;
      kr[j] = v < V ? okey(sc[v]) : 0u;
      er[j] = (v < V && kr[j] >= tk) ? __expf(sc[v] - mx) : 0.f;
    }
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = cur | (1u << bit);
      float m = 0.f;
#pragma unroll
      for (int j = 0; j < kRegRow; ++j) m += kr[j] > cand ? er[j] : 0.f;
      if (block_sum_fixed(m, red4) >= target) cur = cand;
    }
  } else {
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = cur | (1u << bit);
      float m = 0.f;
      for (int v = threadIdx.x; v < V; v += kT) {
        const uint32_t kv = okey(sc[v]);
        if (kv >= tk && kv > cand) m += __expf(sc[v] - mx);
      }
      if (block_sum_fixed(m, red4) >= target) cur = cand;
    }
  }
  uint32_t tp = cur + 1u;
  if (min_keep > 1) {  // the min_keep best always survive
    const uint32_t kmin = kth_largest_key(sc, V, min_keep < V ? min_keep : V, hist, bc);
    tp = tp < kmin ? tp : kmin;
  }
  return tp > tk ? tp : tk;
}

}  // namespace itts_select
