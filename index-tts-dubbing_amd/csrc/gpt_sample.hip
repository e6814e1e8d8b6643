// Token selection + next-token embedding for the KV-cached decode loop.
//   * RepetitionPenaltyLogitsProcessor over every id already in the sequence, including the fake
//     prefix ids 1 and 8192 (quirk Q4): x<0 ? x*p : x/p        HF:generation/logits_process.py:409-412
//   * MinNewTokensLengthLogitsProcessor: stop token -> -inf while fewer than min_new tokens exist
//   * greedy: first-index argmax on f32 logits                 HF:generation/utils.py:2894-2925
//   * sampling (do_sample=True, num_beams=1; HF 4.36 `sample`): Temperature -> TopK -> TopP warpers
//     (HF:generation/logits_process.py TemperatureLogitsWarper / TopKLogitsWarper / TopPLogitsWarper),
//     softmax, one multinomial draw per row.  The draw uses a counter-based hash RNG keyed by
//     (seed, global row = tstate[1] + row, column) with the seed in device memory (tstate[2..3]) so a captured hipGraph
//     replays it; the distribution equals torch's, the individual draws do not (torch's CPU/GPU
//     Philox streams differ anyway), so sampling parity is statistical (tests/test_gpu_gpt.py).
//   * finished rows emit the pad token (= stop 8193)
//   * next input embedding mel_emb(tok) + mel_pos[col + 2]     gpt/model.py:151-155 (quirk Q1)
//     followed by ln_1 of layer 0 (the next GEMM's input), fused.
// The column index comes from a device counter (tstate[0] + col_delta) so a captured hipGraph
// replays the identical launch every step; itts_step_advance bumps the counter.
#include "common.h"
#include "select.h"

namespace {
constexpr int kT = 256;
constexpr int kMaxPer = 16;
constexpr int kMaxK = 64;  // top-k candidates kept (ties at the k-th value included, up to this cap)

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

// block-wide (value, index) argmax with first-index tie break; result broadcast to every thread
__device__ __forceinline__ void block_argmax(float& best, int& bi, float* rv, int* ri) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (better(ov, oi, best, bi)) {
      best = ov;
      bi = oi;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    rv[w] = best;
    ri[w] = bi;
  }
  __syncthreads();
  best = rv[0];
  bi = ri[0];
#pragma unroll
  for (int i = 1; i < kT / 64; ++i)
    if (better(rv[i], ri[i], best, bi)) {
      best = rv[i];
      bi = ri[i];
    }
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// uniform in (0, 1), 24 random bits
__device__ __forceinline__ float uniform01(uint64_t key) { return ((float)(mix64(key) >> 40) + 0.5f) * 5.9604645e-8f; }

// record the chosen token, then write x = mel_emb[tok] + mel_pos[col + pos_delta] and h = ln_1(x)
// (h = x when g is null: ln_1 is folded into the c_attn GEMM)
template <typename TH>
// was_done: done[b] as loaded at the kernel's start (only this row's workgroup writes it, at the end),
// so the commit does not wait on a global load after the argmax
__device__ __forceinline__ void commit_and_embed(int b, int ii, int col, int V, int stop, uint8_t* sr, uint8_t* done,
                                                 bool was_done, int32_t* codes, int64_t ldc, const int32_t* forced,
                                                 const float* emb, const float* pos_emb, int pos_delta, int D,
                                                 const float* g, const float* bta, float* x, TH* h, int* tok_s,
                                                 float* rv) {
  if (threadIdx.x == 0) {
    if (ii < 0 || ii >= V) ii = stop;  // all -inf / NaN row: behave like a finished row
    int tok = was_done ? stop : ii;
    codes[(int64_t)b * ldc + col] = tok;
    if (forced) tok = forced[(int64_t)b * ldc + col];  // teacher forcing: record choice, feed given id
    sr[tok] = 1;
    if (tok == stop) done[b] = 1;
    *tok_s = tok;
  }
  __syncthreads();
  if (!x) return;
  const int tok = *tok_s;
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
  if (!h) return;
  if (!g) {  // LayerNorm folded into the consumer GEMM (itts_decode_gemm16x): h = x, rounded
#pragma unroll
    for (int i = 0; i < kMaxPer; ++i)
      if (i < n) St<TH>::st(h + (int64_t)b * D + threadIdx.x + kT * i, v[i]);
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
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

struct SampleArgs {
  const float* logits;
  int64_t ldl;
  int V;
  uint8_t* seen;
  uint8_t* done;
  int32_t* codes;
  int64_t ldc;
  const int32_t* tstate;
  int col_delta, min_new, stop;
  float penalty;
  // sampling warpers (do_sample only)
  float inv_temp;
  int top_k;
  float top_p;
  const float* emb;
  const float* pos_emb;
  int pos_delta, D;
  const float *g, *bta;
  float* x;
  void* h;
  const int32_t* forced;
};

__device__ __forceinline__ float processed_score(const SampleArgs& p, const float* lr, const uint8_t* sr, int v,
                                                 int col) {
  float s = lr[v];
  if (sr[v]) s = s < 0.f ? s * p.penalty : s / p.penalty;
  if (v == p.stop && col < p.min_new) s = -INFINITY;
  return s;
}

template <typename TH, bool VEC4>
__global__ __launch_bounds__(kT) void sample_embed_kernel(SampleArgs p) {
  __shared__ float rv[kT / 64];
  __shared__ int ri[kT / 64];
  __shared__ int tok_s;
  const int b = blockIdx.x;
  const bool was_done = p.done[b] != 0;
  const int col = p.tstate[0] + p.col_delta;
  const float* lr = p.logits + (int64_t)b * p.ldl;
  uint8_t* sr = p.seen + (int64_t)b * p.ldl;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  if constexpr (VEC4) {
    // 16-B logits + 4-B seen-flag loads, a whole row's loads in flight per thread (kI per trip)
    constexpr int kI = 9;  // ceil(ceil(8194 / 4) / 256): the IndexTTS mel vocabulary in one trip
    const int nv4 = (p.V + 3) >> 2;
    const f32x4_t* l4 = reinterpret_cast<const f32x4_t*>(lr);
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(sr);
    for (int base = 0; base < nv4; base += kT * kI) {
      f32x4_t lv[kI];
      uint32_t sv[kI];
#pragma unroll
      for (int i = 0; i < kI; ++i) {
        const int idx = base + threadIdx.x + kT * i;
        if (idx < nv4) {
          lv[i] = l4[idx];
          sv[i] = s4[idx];
        }
      }
#pragma unroll
      for (int i = 0; i < kI; ++i) {
        const int idx = base + threadIdx.x + kT * i;
        if (idx >= nv4) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int v = 4 * idx + e;
          if (v >= p.V) continue;
          float s = lv[i][e];
          if ((sv[i] >> (8 * e)) & 0xFFu) s = s < 0.f ? s * p.penalty : s / p.penalty;
          if (v == p.stop && col < p.min_new) s = -INFINITY;
          if (better(s, v, best, bi)) {
            best = s;
            bi = v;
          }
        }
      }
    }
  } else {
    for (int v = threadIdx.x; v < p.V; v += kT) {
      const float s = processed_score(p, lr, sr, v, col);
      if (better(s, v, best, bi)) {
        best = s;
        bi = v;
      }
    }
  }
  block_argmax(best, bi, rv, ri);
  commit_and_embed<TH>(b, bi, col, p.V, p.stop, sr, p.done, was_done, p.codes, p.ldc, p.forced, p.emb, p.pos_emb,
                       p.pos_delta, p.D, p.g, p.bta, p.x, reinterpret_cast<TH*>(p.h), &tok_s, rv);
}

// do_sample: scores (after processors, / temperature) staged in LDS.  0 < top_k <= 64: the top-k
// candidates are extracted in descending order by repeated block argmax (each thread caches the max
// of its own strided slice, only the winner rescans); top-p + the multinomial draw run on the
// candidates.  top_k > 64 or top-p alone: warper thresholds (select.h) + a Gumbel-max draw among the
// survivors.  top_k == 0 and top_p == 1: Gumbel-max draw over the whole vocabulary.
constexpr int kRegS = 33;  // register-resident row: ceil(8194 / 256) scores per thread

// thread 0: TopP over the nc top-k candidates (descending), then the multinomial draw -> ri[0]
__device__ __forceinline__ void topk_top_p_pick(const SampleArgs& p, const float* cv, const int* ci, int nc,
                                                uint64_t key, float* rv, int* ri) {
  int pick = nc > 0 ? ci[0] : p.stop;
  if (nc > 1) {
    // softmax over the candidates (all other scores are -inf after top-k)
    float e[kMaxK];
    float z = 0.f;
    for (int i = 0; i < nc; ++i) {
      e[i] = __expf(cv[i] - cv[0]);
      z += e[i];
    }
    // TopP: ascending cumulative probability; drop while cum <= 1 - top_p; keep the largest
    int keep = nc;
    if (p.top_p < 1.f) {
      float cum = 0.f;
      for (int i = nc - 1; i > 0; --i) {
        cum += e[i] / z;
        if (cum <= 1.f - p.top_p) keep = i;
        else break;
      }
    }
    float zk = 0.f;
    for (int i = 0; i < keep; ++i) zk += e[i];
    const float u = uniform01(key) * zk;
    float acc = 0.f;
    pick = ci[keep - 1];
    for (int i = 0; i < keep; ++i) {
      acc += e[i];
      if (u < acc) {
        pick = ci[i];
        break;
      }
    }
  }
  rv[0] = 0.f;
  ri[0] = pick;
}

template <typename TH>
__global__ __launch_bounds__(kT) void sample_topk_embed_kernel(SampleArgs p) {
  extern __shared__ float sc[];  // [V]
  __shared__ float rv[kT / 64];
  __shared__ int ri[kT / 64];
  __shared__ float cv[kMaxK];
  __shared__ int ci[kMaxK];
  __shared__ int hist[256], bc[2];  // general warper thresholds (select.h)
  __shared__ int tok_s;
  const int b = blockIdx.x;
  const bool was_done = p.done[b] != 0;
  const int col = p.tstate[0] + p.col_delta;
  const uint64_t seed = (uint64_t)(uint32_t)p.tstate[2] | ((uint64_t)(uint32_t)p.tstate[3] << 32);
  const uint64_t row = (uint64_t)(uint32_t)(b + p.tstate[1]);  // tstate[1]: global index of row 0
  const uint64_t key = mix64(seed ^ mix64((row << 32) | (uint32_t)col));
  const float* lr = p.logits + (int64_t)b * p.ldl;
  uint8_t* sr = p.seen + (int64_t)b * p.ldl;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  if (p.top_k > kMaxK || (p.top_k <= 0 && p.top_p < 1.f)) {
    // any top_k, or top-p only: warper thresholds over the staged row (select.h), then a Gumbel-max
    // draw among the survivors == a multinomial draw from their renormalised softmax
    for (int v = threadIdx.x; v < p.V; v += kT) sc[v] = processed_score(p, lr, sr, v, col) * p.inv_temp;
    __syncthreads();
    const uint32_t T = itts_select::warper_threshold(sc, p.V, p.top_k, p.top_p, 1, hist, bc, rv);
    for (int v = threadIdx.x; v < p.V; v += kT) {
      const float s = sc[v];
      if (s == -INFINITY || itts_select::okey(s) < T) continue;
      const float gmb = s - __logf(-__logf(uniform01(key + (uint64_t)v + 1)));
      if (better(gmb, v, best, bi)) {
        best = gmb;
        bi = v;
      }
    }
    block_argmax(best, bi, rv, ri);
  } else if (p.top_k <= 0) {  // plain multinomial == argmax(score + Gumbel noise)
    for (int v = threadIdx.x; v < p.V; v += kT) {
      const float s = processed_score(p, lr, sr, v, col) * p.inv_temp;
      const float gmb = s - __logf(-__logf(uniform01(key + (uint64_t)v + 1)));
      if (s != -INFINITY && better(gmb, v, best, bi)) {
        best = gmb;
        bi = v;
      }
    }
    block_argmax(best, bi, rv, ri);
  } else if (p.V <= kT * kRegS) {
    // 0 < top_k <= 64, row in registers (element j*kT + tid): repeated block argmax with one barrier
    // per round (wave winners alternate between two LDS slots); the winner's owner clears it and
    // rescans its registers.  Same candidates, same order as the LDS-staged form below (the IndexTTS
    // vocabulary always takes this path).
    float s[kRegS];
#pragma unroll
    for (int j = 0; j < kRegS; ++j) {
      const int v = threadIdx.x + kT * j;
      s[j] = v < p.V ? processed_score(p, lr, sr, v, col) * p.inv_temp : -INFINITY;
    }
    auto tok = [](int j) { return (int)threadIdx.x + kT * j; };
    __shared__ uint32_t wk2[2][2][kT / 64];  // [slot][hi, lo][wave]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float mine, nxt;
    int mine_i, nxt_i;
    {
      const itts_select::Top2 t2 = itts_select::top2_after(s, tok, INFINITY, -1);
      mine = t2.b1;
      mine_i = t2.i1;
      nxt = t2.b2;
      nxt_i = t2.i2;
    }
    bool has_nxt = ITTS_TOPK_CACHE2 != 0;
    int nc = 0;
    float tau = -INFINITY;
    while (nc < kMaxK) {
      // the round's winner: one max over (score, token) keys -- DPP within the wave, the 4 wave maxima
      // through LDS (two slots: a slot is rewritten two rounds later, after the next round's barrier)
      const itts_select::Key64 wk = itts_select::wave_max_key64(itts_select::key64(mine, mine_i));
      const int slot = nc & 1;
      if (lane == 0) {
        wk2[slot][0][wid] = wk.hi;
        wk2[slot][1][wid] = wk.lo;
      }
      __syncthreads();
      itts_select::Key64 bk{wk2[slot][0][0], wk2[slot][1][0]};
#pragma unroll
      for (int w = 1; w < kT / 64; ++w) {
        const itts_select::Key64 o{wk2[slot][0][w], wk2[slot][1][w]};
        if (itts_select::key64_gt(o, bk)) bk = o;
      }
      const float bv = itts_select::key64_score(bk);
      const int bidx = (int)~bk.lo;
      if (bv == -INFINITY || !(bv == bv)) break;
      if (nc >= p.top_k && bv < tau) break;  // HF keeps every score >= the k-th largest
      if (threadIdx.x == 0) {
        cv[nc] = bv;
        ci[nc] = bidx;
      }
      if (nc == p.top_k - 1) tau = bv;
      ++nc;
      if (mine_i == bidx) {  // the owner (tokens are unique): next candidate = its cached second
        if (has_nxt) {
          mine = nxt;
          mine_i = nxt_i;
          has_nxt = false;
        } else {
          const itts_select::Top2 t2 = itts_select::top2_after(s, tok, bv, bidx);
          mine = t2.b1;
          mine_i = t2.i1;
          nxt = t2.b2;
          nxt_i = t2.i2;
          has_nxt = ITTS_TOPK_CACHE2 != 0;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) topk_top_p_pick(p, cv, ci, nc, key, rv, ri);
    __syncthreads();
    bi = ri[0];
  } else {
    for (int v = threadIdx.x; v < p.V; v += kT) {
      const float s = processed_score(p, lr, sr, v, col) * p.inv_temp;
      sc[v] = s;
      if (better(s, v, best, bi)) {
        best = s;
        bi = v;
      }
    }
    float mine = best;
    int mine_i = bi;
    int nc = 0;
    float tau = -INFINITY;
    while (nc < kMaxK) {
      float bv = mine;
      int bidx = mine_i;
      block_argmax(bv, bidx, rv, ri);  // uniform across the block
      if (bv == -INFINITY || !(bv == bv)) break;
      if (nc >= p.top_k && bv < tau) break;  // HF keeps every score >= the k-th largest
      if (threadIdx.x == 0) {
        cv[nc] = bv;
        ci[nc] = bidx;
      }
      if (nc == p.top_k - 1) tau = bv;
      ++nc;
      if ((bidx % kT) == (int)threadIdx.x) {  // owner: drop it and rescan its slice
        sc[bidx] = -INFINITY;
        mine = -INFINITY;
        mine_i = 0x7fffffff;
        for (int v = threadIdx.x; v < p.V; v += kT)
          if (better(sc[v], v, mine, mine_i)) {
            mine = sc[v];
            mine_i = v;
          }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) topk_top_p_pick(p, cv, ci, nc, key, rv, ri);
    __syncthreads();
    bi = ri[0];
  }
  commit_and_embed<TH>(b, bi, col, p.V, p.stop, sr, p.done, was_done, p.codes, p.ldc, p.forced, p.emb, p.pos_emb,
                       p.pos_delta, p.D, p.g, p.bta, p.x, reinterpret_cast<TH*>(p.h), &tok_s, rv);
}

__global__ void advance_kernel(int32_t* t, int delta) {
  if (threadIdx.x == 0 && blockIdx.x == 0) t[0] += delta;
}

int launch_sample(const char* fn, SampleArgs& p, int h_dtype, int B, bool do_sample, void* stream) {
  ITTS_REQUIRE(B >= 0 && p.V > 0 && p.D > 0 && p.D <= kT * kMaxPer && (p.D % 64 == 0 || p.D < 64), fn, "bad sizes");
  if (B == 0) return 0;
  ITTS_REQUIRE(p.logits && p.seen && p.done && p.codes && p.tstate, fn, "null pointer");
  ITTS_REQUIRE(!p.x || (p.emb && p.pos_emb), fn, "embedding output needs the embedding tables");
  ITTS_REQUIRE(!p.h || (p.x && (!p.g || p.bta)), fn, "h output needs x (and ln_1 bias with ln_1 weight; no ln_1: h = x)");
  hipStream_t s = itts::as_stream(stream);
  ITTS_REQUIRE(p.ldl >= p.V, fn, "row pitch ldl < V");
  if (!do_sample) {
    const bool vec = p.ldl % 4 == 0 && ((reinterpret_cast<uintptr_t>(p.logits) | reinterpret_cast<uintptr_t>(p.seen)) & 15) == 0;
    if (h_dtype == ITTS_BF16 && vec)
      hipLaunchKernelGGL((sample_embed_kernel<uint16_t, true>), dim3(B), dim3(kT), 0, s, p);
    else if (h_dtype == ITTS_BF16)
      hipLaunchKernelGGL((sample_embed_kernel<uint16_t, false>), dim3(B), dim3(kT), 0, s, p);
    else if (vec)
      hipLaunchKernelGGL((sample_embed_kernel<float, true>), dim3(B), dim3(kT), 0, s, p);
    else
      hipLaunchKernelGGL((sample_embed_kernel<float, false>), dim3(B), dim3(kT), 0, s, p);
  } else {
    ITTS_REQUIRE(p.top_k >= 0, fn, "top_k must be >= 0");
    ITTS_REQUIRE(p.inv_temp > 0.f, fn, "temperature must be > 0");
    const size_t lds = (p.top_k > 0 || p.top_p < 1.f) ? (size_t)p.V * sizeof(float) : 0;
    ITTS_REQUIRE(lds <= 64 * 1024 - 1024, fn, "vocabulary too large for the LDS score buffer");
    if (h_dtype == ITTS_BF16)
      hipLaunchKernelGGL(sample_topk_embed_kernel<uint16_t>, dim3(B), dim3(kT), lds, s, p);
    else
      hipLaunchKernelGGL(sample_topk_embed_kernel<float>, dim3(B), dim3(kT), lds, s, p);
  }
  return itts::check_launch(fn);
}
}  // namespace

extern "C" int itts_sample_embed(const float* logits, int64_t ldl, int V, uint8_t* seen, uint8_t* done, int32_t* codes,
                                 int64_t ldc, const int32_t* tstate, int col_delta, int min_new, int stop,
                                 float penalty, const float* emb, const float* pos_emb, int pos_delta, int D,
                                 const float* ln_g, const float* ln_b, float* x, void* h, int h_dtype, int B,
                                 const int32_t* forced, void* stream) {
  SampleArgs p{logits, ldl, V, seen, done, codes, ldc, tstate, col_delta, min_new, stop, penalty, 1.f, 0, 1.f,
               emb, pos_emb, pos_delta, D, ln_g, ln_b, x, h, forced};
  return launch_sample("itts_sample_embed", p, h_dtype, B, false, stream);
}

extern "C" int itts_sample_topk_embed(const float* logits, int64_t ldl, int V, uint8_t* seen, uint8_t* done,
                                      int32_t* codes, int64_t ldc, const int32_t* tstate, int col_delta, int min_new,
                                      int stop, float penalty, float temperature, int top_k, float top_p,
                                      const float* emb, const float* pos_emb, int pos_delta, int D, const float* ln_g,
                                      const float* ln_b, float* x, void* h, int h_dtype, int B,
                                      const int32_t* forced, void* stream) {
  SampleArgs p{logits, ldl, V, seen, done, codes, ldc, tstate, col_delta, min_new, stop, penalty,
               temperature > 0.f ? 1.f / temperature : 0.f, top_k, top_p, emb, pos_emb, pos_delta, D, ln_g, ln_b, x,
               h, forced};
  return launch_sample("itts_sample_topk_embed", p, h_dtype, B, true, stream);
}

extern "C" int itts_step_advance(int32_t* tstate, int delta, void* stream) {
  if (!tstate) return itts::fail("itts_step_advance", "null pointer");
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, itts::as_stream(stream), tstate, delta);
  return itts::check_launch("itts_step_advance");
}
