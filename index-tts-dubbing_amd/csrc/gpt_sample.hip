// Token selection + next-token embedding for the KV-cached decode loop (greedy path).
//   * RepetitionPenaltyLogitsProcessor over every id already in the sequence, including the fake
//     prefix ids 1 and 8192 (quirk Q4): x<0 ? x*p : x/p        HF:generation/logits_process.py:409-412
//   * MinNewTokensLengthLogitsProcessor: stop token -> -inf while fewer than min_new tokens exist
//   * first-index argmax on f32 logits                          HF:generation/utils.py:2894-2925
//   * finished rows emit the pad token (= stop 8193)
//   * next input embedding mel_emb(tok) + mel_pos[col + 2]     gpt/model.py:151-155 (quirk Q1)
//     followed by ln_1 of layer 0 (the next GEMM's input), fused.
// The column index comes from a device counter (tstate[0] + col_delta) so a captured hipGraph
// replays the identical launch every step; itts_step_advance bumps the counter.
#include "common.h"

namespace {
constexpr int kT = 256;
constexpr int kMaxPer = 16;

template <typename TH>
__global__ __launch_bounds__(kT) void sample_embed_kernel(const float* __restrict__ logits, int64_t ldl, int V,
                                                          uint8_t* __restrict__ seen, uint8_t* __restrict__ done,
                                                          int32_t* __restrict__ codes, int64_t ldc,
                                                          const int32_t* __restrict__ tstate, int col_delta,
                                                          int min_new, int stop, float penalty,
                                                          const float* __restrict__ emb, const float* __restrict__ pos_emb,
                                                          int pos_delta, int D, const float* g, const float* bta,
                                                          float* __restrict__ x, TH* __restrict__ h,
                                                          const int32_t* __restrict__ forced) {
  __shared__ float rv[kT / 64];
  __shared__ int ri[kT / 64];
  __shared__ int tok_s;
  const int b = blockIdx.x;
  const int col = tstate[0] + col_delta;
  const float* lr = logits + (int64_t)b * ldl;
  uint8_t* sr = seen + (int64_t)b * V;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = threadIdx.x; v < V; v += kT) {
    float s = lr[v];
    if (sr[v]) s = s < 0.f ? s * penalty : s / penalty;
    if (v == stop && col < min_new) s = -INFINITY;
    if (s > best || (s == best && v < bi)) {
      best = s;
      bi = v;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) {
      best = ov;
      bi = oi;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    rv[w] = best;
    ri[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float bb = rv[0];
    int ii = ri[0];
    for (int i = 1; i < kT / 64; ++i)
      if (rv[i] > bb || (rv[i] == bb && ri[i] < ii)) {
        bb = rv[i];
        ii = ri[i];
      }
    if (ii < 0 || ii >= V) ii = stop;  // all -inf / NaN row: behave like a finished row
    int tok = done[b] ? stop : ii;
    codes[(int64_t)b * ldc + col] = tok;
    if (forced) tok = forced[(int64_t)b * ldc + col];  // teacher forcing: record argmax, feed given id
    sr[tok] = 1;
    if (tok == stop) done[b] = 1;
    tok_s = tok;
  }
  __syncthreads();
  if (!x) return;
  const int tok = tok_s;
  const float* er = emb + (int64_t)tok * D;
  const float* pr = pos_emb + (int64_t)(col + pos_delta) * D;
  float v[kMaxPer];
  const int n = (D - threadIdx.x + kT - 1) / kT;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i)
    if (i < n) {
      const int e = threadIdx.x + kT * i;
      v[i] = er[e] + pr[e];
      x[(int64_t)b * D + e] = v[i];
      s += v[i];
    }
  if (!h) return;  // bf16 decode path: the next GEMM normalises x in its own prologue
  // layer-0 ln_1
  s = wave_sum(s);
  __syncthreads();
  if (lane == 0) rv[w] = s;
  __syncthreads();
  const float mean = (rv[0] + rv[1] + rv[2] + rv[3]) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i)
    if (i < n) q += (v[i] - mean) * (v[i] - mean);
  q = wave_sum(q);
  __syncthreads();
  if (lane == 0) rv[w] = q;
  __syncthreads();
  const float rstd = rsqrtf((rv[0] + rv[1] + rv[2] + rv[3]) / D + 1e-5f);
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i)
    if (i < n) {
      const int e = threadIdx.x + kT * i;
      St<TH>::st(h + (int64_t)b * D + e, (v[i] - mean) * rstd * g[e] + bta[e]);
    }
}

__global__ void advance_kernel(int32_t* t, int delta) {
  if (threadIdx.x == 0 && blockIdx.x == 0) t[0] += delta;
}
}  // namespace

extern "C" int itts_sample_embed(const float* logits, int64_t ldl, int V, uint8_t* seen, uint8_t* done, int32_t* codes,
                                 int64_t ldc, const int32_t* tstate, int col_delta, int min_new, int stop,
                                 float penalty, const float* emb, const float* pos_emb, int pos_delta, int D,
                                 const float* ln_g, const float* ln_b, float* x, void* h, int h_dtype, int B,
                                 const int32_t* forced, void* stream) {
  const char* fn = "itts_sample_embed";
  ITTS_REQUIRE(B >= 0 && V > 0 && D > 0 && D <= kT * kMaxPer && (D % 64 == 0 || D < 64), fn, "bad sizes");
  if (B == 0) return 0;
  ITTS_REQUIRE(logits && seen && done && codes && tstate, fn, "null pointer");
  ITTS_REQUIRE(!x || (emb && pos_emb), fn, "embedding output needs the embedding tables");
  ITTS_REQUIRE(!h || (x && ln_g && ln_b), fn, "h output needs x and ln_1 params");
  hipStream_t s = itts::as_stream(stream);
  if (h_dtype == ITTS_BF16)
    hipLaunchKernelGGL(sample_embed_kernel<uint16_t>, dim3(B), dim3(kT), 0, s, logits, ldl, V, seen, done, codes, ldc,
                       tstate, col_delta, min_new, stop, penalty, emb, pos_emb, pos_delta, D, ln_g, ln_b, x,
                       (uint16_t*)h, forced);
  else
    hipLaunchKernelGGL(sample_embed_kernel<float>, dim3(B), dim3(kT), 0, s, logits, ldl, V, seen, done, codes, ldc,
                       tstate, col_delta, min_new, stop, penalty, emb, pos_emb, pos_delta, D, ln_g, ln_b, x,
                       (float*)h, forced);
  return itts::check_launch(fn);
}

extern "C" int itts_step_advance(int32_t* tstate, int delta, void* stream) {
  if (!tstate) return itts::fail("itts_step_advance", "null pointer");
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, itts::as_stream(stream), tstate, delta);
  return itts::check_launch("itts_step_advance");
}
