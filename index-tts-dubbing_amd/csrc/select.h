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

// key of the k-th largest score (1 <= k <= V); hist: 256 ints of LDS, bc: 2 ints of LDS
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
    if (threadIdx.x == 0) {
      int cum = 0, d = 255;
      for (; d > 0; --d) {
        if (cum + hist[d] >= k) break;
        cum += hist[d];
      }
      bc[0] = d;
      bc[1] = k - cum;
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
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t cand = cur | (1u << bit);
    float m = 0.f;
    for (int v = threadIdx.x; v < V; v += kT) {
      const uint32_t kv = okey(sc[v]);
      if (kv >= tk && kv > cand) m += __expf(sc[v] - mx);
    }
    if (block_sum_fixed(m, red4) >= target) cur = cand;
  }
  uint32_t tp = cur + 1u;
  if (min_keep > 1) {  // the min_keep best always survive
    const uint32_t kmin = kth_largest_key(sc, V, min_keep < V ? min_keep : V, hist, bc);
    tp = tp < kmin ? tp : kmin;
  }
  return tp > tk ? tp : tk;
}

}  // namespace itts_select
