// Beam search / beam sample for the KV-cached decode loop (num_beams = K > 1), the reference's
// default decoding (infer.py:535-543: do_sample=True, num_beams=3, top_k 30, top_p 0.8), with
// transformers 4.36 semantics (the version the reference pins, setup.py:50):
//   HF:generation/utils.py beam_search / beam_sample, HF:generation/beam_search.py
//   BeamSearchScorer.process / BeamHypotheses.add / is_done (early_stopping=False); finalize runs on
//   the host (HipGPT.generate, once per call).
//
// Rows r = b*K + k (utterance b, beam k).  Two kernels per step, both graph-replayable (step column
// from the device counter tstate[0] + col_delta):
//   1. beam_cand_kernel (one workgroup per row): log_softmax of the row -> repetition penalty on the
//      log-probs over the row's whole sequence (fake prefix incl., Q4) -> min_new_tokens mask ->
//      [sample: Temperature -> TopK -> TopP warpers, min_keep 2] -> + running beam score -> the row's
//      2K best candidates by key (search: key = score; sample: key = score + Gumbel noise, so the
//      global top-2K keys are a draw of 2K without replacement from softmax(scores over K x V),
//      i.e. torch.multinomial(probs, 2K) in distribution).
//   2. beam_select_kernel (one workgroup per utterance): merges its K x 2K candidates into the
//      utterance's top 2K (sample: then sorted by score, as HF sorts the multinomial draws), runs
//      the scorer (eos among the top K closes a hypothesis, the first K non-eos continue), updates the
//      hypotheses and the done flag, reorders the K beams -- running codes, repetition-penalty flags
//      and the KV lineage table (kv_rows: cache row holding each key position; HF's per-step
//      _reorder_cache copy of every layer's K/V becomes a copy of 4 B per generated position) --
//      and writes the next input embedding + ln_1 of each row.
#include <atomic>

#include "common.h"
#include "select.h"

namespace {
constexpr int kT = 256;
constexpr int kMaxBeams = 16;  // num_beams <= 16 (candidate tables in LDS, 8 per lane in the merge)
constexpr int kMaxC = 2 * kMaxBeams;  // candidates per row / per utterance
constexpr int kMaxK = 64;             // top-k cap of the sampling warper

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float uniform01(uint64_t key) { return ((float)(mix64(key) >> 40) + 0.5f) * 5.9604645e-8f; }
__device__ __forceinline__ float gumbel(uint64_t key) { return -__logf(-__logf(uniform01(key))); }

template <int NT>
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
  for (int i = 1; i < NT / 64; ++i)
    if (better(rv[i], ri[i], best, bi)) {
      best = rv[i];
      bi = ri[i];
    }
}

template <int NT>
__device__ __forceinline__ float block_reduce(float v, float* rv, bool is_max) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    v = is_max ? fmaxf(v, ov) : v + ov;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) rv[w] = v;
  __syncthreads();
  float r = rv[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) r = is_max ? fmaxf(r, rv[i]) : r + rv[i];
  return r;
}

struct BeamArgs {
  const float* logits;
  int64_t ldl;
  int V;
  uint8_t* seen;
  float* beam_score;       // [R]
  const int32_t* tstate;   // [0] step counter, [1] global row of row 0, [2..3] seed
  int col_delta, min_new, stop;
  float penalty;
  int do_sample;
  float inv_temp;
  int top_k;
  float top_p;
  int K;                   // beams
  float* cand_key;         // [R][2K]
  float* cand_score;       // [R][2K]
  int32_t* cand_tok;       // [R][2K]
};

constexpr int kPer = 36;  // logits per thread held in registers: ceil(8194 / 256) rounded to 4

// ---------------------------------------------------------------- 1. per-row candidates
__global__ __launch_bounds__(kT) void beam_cand_kernel(BeamArgs p) {
  extern __shared__ float sc[];  // [V] (sampling with top-k only)
  __shared__ float rv[kT / 64];
  __shared__ int ri[kT / 64];
  __shared__ float tk_v[kMaxK];
  __shared__ int tk_i[kMaxK];
  __shared__ int ntk;
  __shared__ int hist[256], bc[2];  // general warper thresholds (select.h)
  const int r = blockIdx.x;
  const int C = 2 * p.K;
  const int col = p.tstate[0] + p.col_delta;
  const float* lr = p.logits + (int64_t)r * p.ldl;
  const uint8_t* sr = p.seen + (int64_t)r * p.ldl;
  const float bs = p.beam_score[r];
  // registers: element v = 4 * (threadIdx.x + kT * i) + e
  float v[kPer];
  uint32_t s4r[kPer / 4];  // seen flags, requested with the logits (one memory round trip, not two)
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < kPer / 4; ++i) {
    const int v4 = threadIdx.x + kT * i;
    s4r[i] = 4 * v4 < p.V ? reinterpret_cast<const uint32_t*>(sr)[v4] : 0u;
  }
#pragma unroll
  for (int i = 0; i < kPer / 4; ++i) {
    const int v4 = threadIdx.x + kT * i;
    f32x4_t l4 = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    if (4 * v4 < p.V) l4 = reinterpret_cast<const f32x4_t*>(lr)[v4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = (4 * v4 + e < p.V) ? l4[e] : -INFINITY;
      v[4 * i + e] = x;
      m = fmaxf(m, x);
    }
  }
  m = block_reduce<kT>(m, rv, true);
  float z = 0.f;
#pragma unroll
  for (int i = 0; i < kPer; ++i) z += __expf(v[i] - m);  // -inf -> 0
  z = block_reduce<kT>(z, rv, false);
  const float lse = m + __logf(z);
  // processed step scores (log_softmax -> repetition penalty -> min_new_tokens)
#pragma unroll
  for (int i = 0; i < kPer / 4; ++i) {
    const int v4 = threadIdx.x + kT * i;
    const uint32_t s4 = s4r[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int t = 4 * v4 + e;
      float x = v[4 * i + e] - lse;
      if ((s4 >> (8 * e)) & 0xFFu) x = x < 0.f ? x * p.penalty : x / p.penalty;
      if (t == p.stop && col < p.min_new) x = -INFINITY;
      if (t >= p.V) x = -INFINITY;
      v[4 * i + e] = x;
    }
  }
  float* ck = p.cand_key + (int64_t)r * C;
  float* cs = p.cand_score + (int64_t)r * C;
  int32_t* ct = p.cand_tok + (int64_t)r * C;
  const uint64_t seed = (uint64_t)(uint32_t)p.tstate[2] | ((uint64_t)(uint32_t)p.tstate[3] << 32);
  const uint64_t grow = (uint64_t)(uint32_t)(r + p.tstate[1]);
  const uint64_t rkey = mix64(seed ^ mix64((grow << 32) | (uint32_t)col));

  if (!p.do_sample || (p.top_k <= 0 && !(p.top_p < 1.f))) {
    // keys in registers: search -> score; sample without top-k/top-p -> score / T + Gumbel
    if (p.do_sample) {
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int t = 4 * (threadIdx.x + kT * (i / 4)) + (i & 3);
        const float x = v[i] * p.inv_temp;
        v[i] = x == -INFINITY ? x : x + gumbel(rkey + (uint64_t)t + 1);
      }
    }
    // C rounds of block argmax over the register-resident keys (owner clears its winner)
    for (int c = 0; c < C; ++c) {
      float best = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int t = 4 * (threadIdx.x + kT * (i / 4)) + (i & 3);
        if (better(v[i], t, best, bi)) {
          best = v[i];
          bi = t;
        }
      }
      block_argmax<kT>(best, bi, rv, ri);
      if (threadIdx.x == 0) {
        if (best == -INFINITY || bi >= p.V) {
          ck[c] = -INFINITY;
          cs[c] = -INFINITY;
          ct[c] = p.stop;
        } else {
          float score;
          if (p.do_sample) {  // recover the unperturbed score of the winner
            const float g = gumbel(rkey + (uint64_t)bi + 1);
            score = best - g + bs;
            ck[c] = best + bs;
          } else {
            score = best + bs;
            ck[c] = score;
          }
          cs[c] = score;
          ct[c] = bi;
        }
      }
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int t = 4 * (threadIdx.x + kT * (i / 4)) + (i & 3);
        if (t == bi) v[i] = -INFINITY;
      }
    }
    return;
  }
  // ---- sampling with warpers: Temperature -> TopK (k' = max(top_k, 2), ties kept) -> TopP (min 2)
  if (p.top_k > kMaxK || p.top_k <= 0) {
    for (int i = 0; i < kPer; ++i) {
      const int t = 4 * (threadIdx.x + kT * (i / 4)) + (i & 3);
      if (t < p.V) sc[t] = v[i] * p.inv_temp;
    }
    __syncthreads();
    // any top_k, or top-p only: survivors = keys >= the warper threshold (select.h); Gumbel keys of
    // the survivors in place, then the row's C best keys by C rounds of block argmax
    const uint32_t T = itts_select::warper_threshold(sc, p.V, p.top_k, p.top_p, 2, hist, bc, rv);
    for (int t = threadIdx.x; t < p.V; t += kT) {
      const float x = sc[t];
      sc[t] = (x == -INFINITY || itts_select::okey(x) < T) ? -INFINITY : x + bs + gumbel(rkey + (uint64_t)t + 1);
    }
    __syncthreads();
    for (int c = 0; c < C; ++c) {
      float best = -INFINITY;
      int bi = 0x7fffffff;
      for (int t = threadIdx.x; t < p.V; t += kT)
        if (better(sc[t], t, best, bi)) {
          best = sc[t];
          bi = t;
        }
      block_argmax<kT>(best, bi, rv, ri);
      if (threadIdx.x == 0) {
        if (best == -INFINITY) {
          ck[c] = -INFINITY;
          cs[c] = -INFINITY;
          ct[c] = p.stop;
        } else {
          ck[c] = best;
          cs[c] = best - gumbel(rkey + (uint64_t)bi + 1);  // the unperturbed score (incl. the beam's)
          ct[c] = bi;
        }
      }
      if (best != -INFINITY && (bi % kT) == (int)threadIdx.x) sc[bi] = -INFINITY;
      __syncthreads();
    }
    return;
  }
  // 0 < top_k <= 64: the survivors leave in descending (score, lowest index first) order by repeated
  // block argmax over the register-resident scores; the winner's owner clears it and rescans its own
  // registers.  One barrier per round (the wave winners alternate between two LDS slots).  The LDS-
  // staged form (one thread rescanning its 32-entry LDS slice per round, two barriers) took 128 us
  // of a 96-row beam3 step (profiles/kernel_stats_r02f_beam3.txt).
  const int kk = p.top_k < 2 ? 2 : p.top_k;
#pragma unroll
  for (int i = 0; i < kPer; ++i) v[i] *= p.inv_temp;  // -inf stays -inf (inv_temp > 0)
  auto tok = [](int i) { return 4 * ((int)threadIdx.x + kT * (i / 4)) + (i & 3); };
  float mine, nxt;
  int mine_i, nxt_i;
  {
    const itts_select::Top2 t2 = itts_select::top2_after(v, tok, INFINITY, -1);
    mine = t2.b1;
    mine_i = t2.i1;
    nxt = t2.b2;
    nxt_i = t2.i2;
  }
  bool has_nxt = ITTS_TOPK_CACHE2 != 0;
  __shared__ uint32_t wk2[2][2][kT / 64];  // [slot][hi, lo][wave]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
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
    if (nc >= kk && bv < tau) break;  // HF keeps every score >= the k-th largest
    if (threadIdx.x == 0) {
      tk_v[nc] = bv;
      tk_i[nc] = bidx;
    }
    if (nc == kk - 1) tau = bv;
    ++nc;
    if (mine_i == bidx) {  // the owner (tokens are unique): next candidate = its cached second
      if (has_nxt) {
        mine = nxt;
        mine_i = nxt_i;
        has_nxt = false;
      } else {
        const itts_select::Top2 t2 = itts_select::top2_after(v, tok, bv, bidx);
        mine = t2.b1;
        mine_i = t2.i1;
        nxt = t2.b2;
        nxt_i = t2.i2;
        has_nxt = ITTS_TOPK_CACHE2 != 0;
      }
    }
  }
  if (threadIdx.x == 0) {
    // TopP over the (descending) top-k survivors: drop the ascending tail while its cumulative
    // probability <= 1 - top_p, keeping at least 2
    int keep = nc;
    if (p.top_p < 1.f && nc > 2) {
      float zz = 0.f;
      for (int i = 0; i < nc; ++i) zz += __expf(tk_v[i] - tk_v[0]);
      float cum = 0.f;
      for (int i = nc - 1; i >= 2; --i) {
        cum += __expf(tk_v[i] - tk_v[0]) / zz;
        if (cum <= 1.f - p.top_p) keep = i;
        else break;
      }
    }
    ntk = keep;
  }
  __syncthreads();
  // Gumbel keys of the survivors; the row's C best keys (one wave; <= 64 survivors)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int n = ntk;
    float key = -INFINITY;
    int tok = 0x7fffffff;
    float score = -INFINITY;
    if (lane < n) {
      tok = tk_i[lane];
      score = tk_v[lane] + bs;
      key = score + gumbel(rkey + (uint64_t)tok + 1);
    }
    for (int c = 0; c < C; ++c) {
      float bk = key;
      int bt = tok;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ok = __shfl_xor(bk, o, 64);
        const int ot = __shfl_xor(bt, o, 64);
        if (better(ok, ot, bk, bt)) {
          bk = ok;
          bt = ot;
        }
      }
      const bool mine_w = (tok == bt) && key != -INFINITY;
      if (lane == 0 && bk == -INFINITY) {
        ck[c] = -INFINITY;
        cs[c] = -INFINITY;
        ct[c] = p.stop;
      }
      if (mine_w) {
        ck[c] = key;
        cs[c] = score;
        ct[c] = tok;
        key = -INFINITY;
      }
    }
  }
}

// ---------------------------------------------------------------- 2. per-utterance selection
struct SelArgs {
  const float* cand_key;
  const float* cand_score;
  const int32_t* cand_tok;
  int K, V, stop, do_sample;
  float length_penalty;
  const int32_t* tstate;
  int col_delta;
  uint8_t* done;           // [B]
  float* beam_score;       // [R]
  int32_t* codes;          // [R][ldc] running (generated) tokens
  int64_t ldc;
  uint8_t* seen;           // [R][lds]
  int64_t lds;
  const int32_t* base_ids; // ids flagged in every row from the start (fake prefix: 1, 8192)
  int n_base;
  int32_t* kv_rows;        // [R][ld_rows]
  int64_t ld_rows;
  int kv_base;             // cache position of generated token 0
  float* hyp_score;        // [B][K]
  int32_t* hyp_len;        // [B][K]
  int32_t* hyp_codes;      // [B][K][ldc]
  int32_t* hyp_n;          // [B]
  int32_t* hyp_order;      // [B][K] list order of hypothesis slots
  float* hyp_worst;        // [B]
  const float* emb;
  const float* pos_emb;
  int pos_delta, D;
  const float *g, *bta;
  float* x;
  void* h;
};

template <typename TH>
__global__ __launch_bounds__(kT) void beam_select_kernel(SelArgs p) {
  extern __shared__ int32_t lds_i[];  // [K][col] parent codes, then [K][col] parent table entries
  __shared__ float s_key[kMaxBeams * kMaxC], s_score[kMaxBeams * kMaxC];
  __shared__ int s_tok[kMaxBeams * kMaxC], s_par[kMaxBeams * kMaxC];
  __shared__ float top_key[kMaxC], top_score[kMaxC];
  __shared__ int top_tok[kMaxC], top_par[kMaxC], ntop;
  __shared__ int new_tok[kMaxBeams], new_par[kMaxBeams];
  __shared__ float new_score[kMaxBeams];
  __shared__ int slot_src[kMaxBeams];  // per hypothesis slot: parent row whose codes it takes (-1: unchanged)
  __shared__ int s_done, s_was_done;
  __shared__ float rv[kT / 64];
  const int b = blockIdx.x;
  const int K = p.K, C = 2 * K;
  const int col = p.tstate[0] + p.col_delta;  // index of the token chosen now
  const int r0 = b * K;
  if (threadIdx.x == 0) {
    s_was_done = p.done[b];
    s_done = s_was_done;
  }
  if (threadIdx.x < kMaxBeams) slot_src[threadIdx.x] = -1;
  __syncthreads();
  const bool was_done = s_was_done;
  if (!was_done) {
    // gather the K x C row candidates
    for (int i = threadIdx.x; i < K * C; i += kT) {
      s_key[i] = p.cand_key[(int64_t)r0 * C + i];
      s_score[i] = p.cand_score[(int64_t)r0 * C + i];
      s_tok[i] = p.cand_tok[(int64_t)r0 * C + i];
      s_par[i] = i / C;
    }
    __syncthreads();
    // the utterance's C best keys (one wave, up to 8 candidates per lane; ties -> lower flat index
    // beam * V + token)
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      constexpr int NPL = kMaxBeams * kMaxC / 64;
      float kk[NPL];
      int ff[NPL];
#pragma unroll
      for (int j = 0; j < NPL; ++j) {
        const int i = lane + 64 * j;
        kk[j] = i < K * C ? s_key[i] : -INFINITY;
        ff[j] = i < K * C ? s_par[i] * p.V + s_tok[i] : 0x7fffffff;
      }
      int n = 0;
      for (int c = 0; c < C; ++c) {
        float bk = kk[0];
        int bf = ff[0], bs = lane;
#pragma unroll
        for (int j = 1; j < NPL; ++j) {
          const bool u = kk[j] > bk || (kk[j] == bk && ff[j] < bf);
          bk = u ? kk[j] : bk;
          bf = u ? ff[j] : bf;
          bs = u ? lane + 64 * j : bs;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const float ok = __shfl_xor(bk, o, 64);
          const int of = __shfl_xor(bf, o, 64);
          const int os = __shfl_xor(bs, o, 64);
          if (ok > bk || (ok == bk && of < bf)) {
            bk = ok;
            bf = of;
            bs = os;
          }
        }
        if (bk == -INFINITY) break;
        if (lane == 0) {
          top_key[c] = bk;
          top_score[c] = s_score[bs];
          top_tok[c] = s_tok[bs];
          top_par[c] = s_par[bs];
        }
#pragma unroll
        for (int j = 0; j < NPL; ++j)
          if (bs == lane + 64 * j) kk[j] = -INFINITY;
        ++n;
      }
      if (lane == 0) ntop = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const int n = ntop;
      if (p.do_sample) {  // HF: torch.sort(sampled scores, descending) -- insertion sort, key order on ties
        for (int i = 1; i < n; ++i) {
          const float vs = top_score[i], vk = top_key[i];
          const int vt = top_tok[i], vp = top_par[i];
          int j = i - 1;
          while (j >= 0 && top_score[j] < vs) {
            top_score[j + 1] = top_score[j];
            top_key[j + 1] = top_key[j];
            top_tok[j + 1] = top_tok[j];
            top_par[j + 1] = top_par[j];
            --j;
          }
          top_score[j + 1] = vs;
          top_key[j + 1] = vk;
          top_tok[j + 1] = vt;
          top_par[j + 1] = vp;
        }
      }
      // BeamSearchScorer.process
      const float glen_pow = powf((float)(col + 1), p.length_penalty);
      float* hs = p.hyp_score + (int64_t)b * K;
      int32_t* hl = p.hyp_len + (int64_t)b * K;
      int32_t* ho = p.hyp_order + (int64_t)b * K;
      int hn = p.hyp_n[b];
      float worst = p.hyp_worst[b];
      int j = 0;
      for (int rank = 0; rank < n && j < K; ++rank) {
        const int t = top_tok[rank];
        const float v = top_score[rank];
        if (t == p.stop) {
          if (rank >= K) continue;
          // BeamHypotheses.add(parent sequence, v, generated_len = col + 1)
          const float s = v / glen_pow;
          if (hn < K || s > worst) {
            if (hn < K) {
              const int slot = hn;
              ho[hn] = slot;
              hs[slot] = s;
              hl[slot] = col;
              slot_src[slot] = r0 + top_par[rank];
              ++hn;
              worst = fminf(s, worst);
            } else {
              // append, then delete the (score, list index)-smallest entry; the new one takes its slot
              int mi = 0;
              for (int i = 1; i < hn; ++i)
                if (hs[ho[i]] < hs[ho[mi]]) mi = i;
              const int slot = ho[mi];
              // second smallest over the remaining list + the new entry (list index order for ties)
              float w2 = INFINITY;
              for (int i = 0; i < hn; ++i)
                if (i != mi) w2 = fminf(w2, hs[ho[i]]);
              w2 = fminf(w2, s);
              if (!(s < hs[slot])) {
                for (int i = mi; i < hn - 1; ++i) ho[i] = ho[i + 1];
                ho[hn - 1] = slot;
                hs[slot] = s;
                hl[slot] = col;
                slot_src[slot] = r0 + top_par[rank];
              }
              worst = w2;
            }
          }
        } else {
          new_score[j] = v;
          new_tok[j] = t;
          new_par[j] = top_par[rank];
          ++j;
        }
      }
      for (; j < K; ++j) {  // cannot happen with 2K candidates and one eos id; keep rows valid
        new_score[j] = -INFINITY;
        new_tok[j] = p.stop;
        new_par[j] = j;
      }
      p.hyp_n[b] = hn;
      p.hyp_worst[b] = worst;
      const float best = n > 0 ? top_score[0] : -INFINITY;
      if (hn >= K && worst >= best / glen_pow) s_done = 1;
      p.done[b] = (uint8_t)s_done;
    }
    __syncthreads();
  } else if (threadIdx.x < K) {  // finished utterance: beams frozen, fed the pad token
    new_tok[threadIdx.x] = p.stop;
    new_par[threadIdx.x] = threadIdx.x;
    new_score[threadIdx.x] = p.beam_score[r0 + threadIdx.x];
  }
  __syncthreads();
  // hypothesis codes: slot <- parent's running codes [0, col)
  for (int slot = 0; slot < K; ++slot) {
    const int src = slot_src[slot];
    if (src < 0) continue;
    int32_t* dst = p.hyp_codes + ((int64_t)b * K + slot) * p.ldc;
    const int32_t* sp = p.codes + (int64_t)src * p.ldc;
    for (int i = threadIdx.x; i < col; i += kT) dst[i] = sp[i];
  }
  // reorder the K beams: stage parents' codes and table entries of the generated positions in LDS,
  // clear each row's old repetition flags (from its own old codes), then write the new state
  int32_t* pc = lds_i;
  int32_t* pt = lds_i + K * col;
  bool ident = true;
  for (int k = 0; k < K; ++k) ident = ident && new_par[k] == k;
  if (!ident) {
    for (int i = threadIdx.x; i < K * col; i += kT) {
      const int k = i / col, j = i - k * col;
      const int src = r0 + new_par[k];
      pc[i] = p.codes[(int64_t)src * p.ldc + j];
      pt[i] = p.kv_rows[(int64_t)src * p.ld_rows + p.kv_base + j];
    }
    for (int i = threadIdx.x; i < K * col; i += kT) {
      const int k = i / col, j = i - k * col;
      if (new_par[k] == k) continue;
      const int r = r0 + k;
      p.seen[(int64_t)r * p.lds + p.codes[(int64_t)r * p.ldc + j]] = 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < K * col; i += kT) {
      const int k = i / col, j = i - k * col;
      if (new_par[k] == k) continue;
      const int r = r0 + k;
      p.codes[(int64_t)r * p.ldc + j] = pc[i];
      p.kv_rows[(int64_t)r * p.ld_rows + p.kv_base + j] = pt[i];
      p.seen[(int64_t)r * p.lds + pc[i]] = 1;
    }
    __syncthreads();
    if (threadIdx.x < K * p.n_base) {  // the fake prefix ids stay flagged
      const int k = threadIdx.x / p.n_base;
      p.seen[(int64_t)(r0 + k) * p.lds + p.base_ids[threadIdx.x - k * p.n_base]] = 1;
    }
  }
  __syncthreads();
  if (threadIdx.x < K) {
    const int r = r0 + threadIdx.x;
    const int t = new_tok[threadIdx.x];
    p.codes[(int64_t)r * p.ldc + col] = t;
    p.seen[(int64_t)r * p.lds + t] = 1;
    p.kv_rows[(int64_t)r * p.ld_rows + p.kv_base + col] = r;
    p.beam_score[r] = new_score[threadIdx.x];
  }
  // next input: x = mel_emb[tok] + mel_pos[col + pos_delta] (Q1), h = ln_1(x)
  for (int k = 0; k < K; ++k) {
    const int r = r0 + k;
    const int t = new_tok[k];
    const float* er = p.emb + (int64_t)t * p.D;
    const float* pr = p.pos_emb + (int64_t)(col + p.pos_delta) * p.D;
    float vals[16];
    float s = 0.f;
    const int n = (p.D - threadIdx.x + kT - 1) / kT;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < n) {
        const int e = threadIdx.x + kT * i;
        vals[i] = er[e] + pr[e];
        p.x[(int64_t)r * p.D + e] = vals[i];
        s += vals[i];
      }
    if (!p.g) {  // ln_1 folded into the c_attn GEMM: h = x, rounded
      TH* hr = reinterpret_cast<TH*>(p.h) + (int64_t)r * p.D;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (i < n) St<TH>::st(hr + threadIdx.x + kT * i, vals[i]);
      continue;
    }
    const float mean = block_reduce<kT>(s, rv, false) / p.D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < n) q += (vals[i] - mean) * (vals[i] - mean);
    const float rstd = rsqrtf(block_reduce<kT>(q, rv, false) / p.D + 1e-5f);
    TH* hr = reinterpret_cast<TH*>(p.h) + (int64_t)r * p.D;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < n) {
        const int e = threadIdx.x + kT * i;
        St<TH>::st(hr + e, (vals[i] - mean) * rstd * p.g[e] + p.bta[e]);
      }
  }
}

}  // namespace

extern "C" int itts_beam_candidates(const float* logits, int64_t ldl, int V, const uint8_t* seen, float* beam_score,
                                    const int32_t* tstate, int col_delta, int min_new, int stop, float penalty,
                                    int do_sample, float temperature, int top_k, float top_p, int num_beams,
                                    float* cand_key, float* cand_score, int32_t* cand_tok, int R, void* stream) {
  const char* fn = "itts_beam_candidates";
  ITTS_REQUIRE(R >= 0 && V > 0 && num_beams >= 2 && num_beams <= kMaxBeams, fn, "bad sizes (2 <= num_beams <= 16)");
  if (R == 0) return 0;
  ITTS_REQUIRE(R % num_beams == 0, fn, "rows must be utterances x num_beams");
  ITTS_REQUIRE(logits && seen && beam_score && tstate && cand_key && cand_score && cand_tok, fn, "null pointer");
  ITTS_REQUIRE(V <= kT * kPer, fn, "vocabulary too large (<= 9216)");
  ITTS_REQUIRE(ldl % 4 == 0 && ldl >= V && ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(seen)) & 15) == 0,
               fn, "logits / seen rows must be 16-B aligned with ldl % 4 == 0");
  ITTS_REQUIRE(!do_sample || temperature > 0.f, fn, "temperature must be > 0");
  ITTS_REQUIRE(!do_sample || top_k >= 0, fn, "top_k must be >= 0");
  BeamArgs a{logits, ldl, V, const_cast<uint8_t*>(seen), beam_score, tstate, col_delta, min_new, stop, penalty,
             do_sample, do_sample ? 1.f / temperature : 1.f, top_k, top_p, num_beams, cand_key, cand_score, cand_tok};
  // the LDS-staged row is only for the general warper path (top_k > 64, or top-p alone)
  const size_t lds = (do_sample && (top_k > kMaxK || (top_k <= 0 && top_p < 1.f))) ? (size_t)V * sizeof(float) : 0;
  ITTS_REQUIRE(lds <= 64 * 1024 - 2048, fn, "vocabulary too large for the LDS score buffer");
  hipLaunchKernelGGL(beam_cand_kernel, dim3(R), dim3(kT), lds, itts::as_stream(stream), a);
  return itts::check_launch(fn);
}

extern "C" int itts_beam_select(const float* cand_key, const float* cand_score, const int32_t* cand_tok,
                                int num_beams, int V, int stop, int do_sample, float length_penalty,
                                const int32_t* tstate, int col_delta, uint8_t* done, float* beam_score, int32_t* codes,
                                int64_t ldc, uint8_t* seen, int64_t lds, const int32_t* base_ids, int n_base,
                                int32_t* kv_rows, int64_t ld_rows, int kv_base, float* hyp_score, int32_t* hyp_len,
                                int32_t* hyp_codes, int32_t* hyp_n, int32_t* hyp_order, float* hyp_worst,
                                const float* emb, const float* pos_emb, int pos_delta, int D, const float* ln_g,
                                const float* ln_b, float* x, void* h, int h_dtype, int B, int max_col,
                                void* stream) {
  const char* fn = "itts_beam_select";
  ITTS_REQUIRE(B >= 0 && num_beams >= 2 && num_beams <= kMaxBeams && D > 0 && D <= kT * 16, fn, "bad sizes");
  if (B == 0) return 0;
  ITTS_REQUIRE(cand_key && cand_score && cand_tok && tstate && done && beam_score && codes && seen && kv_rows &&
                   hyp_score && hyp_len && hyp_codes && hyp_n && hyp_order && hyp_worst && emb && pos_emb && (!ln_g || ln_b) &&
                   x && h && (n_base == 0 || base_ids),
               fn, "null pointer");
  ITTS_REQUIRE(n_base >= 0 && num_beams * n_base <= kT, fn, "too many base ids");
  ITTS_REQUIRE(max_col >= 1 && max_col <= ldc && kv_base + max_col <= ld_rows, fn, "bad step capacity");
  const size_t lds_bytes = (size_t)2 * num_beams * max_col * sizeof(int32_t);
  ITTS_REQUIRE(lds_bytes <= 144 * 1024, fn, "num_beams x max_new_tokens too large for the reorder buffer");
  SelArgs a{cand_key, cand_score, cand_tok, num_beams, V, stop, do_sample, length_penalty, tstate, col_delta, done,
            beam_score, codes, ldc, seen, lds, base_ids, n_base, kv_rows, ld_rows, kv_base, hyp_score, hyp_len,
            hyp_codes, hyp_n, hyp_order, hyp_worst, emb, pos_emb, pos_delta, D, ln_g, ln_b, x, h};
  hipStream_t s = itts::as_stream(stream);
  if (lds_bytes > 64 * 1024) {  // beyond the default dynamic LDS cap (160 KiB per workgroup on gfx950)
    // per device (the attribute binds to the current device's module), retried until it succeeds
    static std::atomic<unsigned> raised_mask{0};
    int dev = 0;
    ITTS_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 32, fn, "no current HIP device");
    bool once = (raised_mask.load() >> dev) & 1u;
    if (!once) {
      const int cap = 144 * 1024;
      once = hipFuncSetAttribute(reinterpret_cast<const void*>(beam_select_kernel<uint16_t>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, cap) == hipSuccess &&
             hipFuncSetAttribute(reinterpret_cast<const void*>(beam_select_kernel<float>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, cap) == hipSuccess;
      if (once) raised_mask.fetch_or(1u << dev);
    }
    ITTS_REQUIRE(once, fn, "could not raise the dynamic LDS limit for the reorder buffer");
  }
  if (h_dtype == ITTS_BF16)
    hipLaunchKernelGGL(beam_select_kernel<uint16_t>, dim3(B), dim3(kT), lds_bytes, s, a);
  else
    hipLaunchKernelGGL(beam_select_kernel<float>, dim3(B), dim3(kT), lds_bytes, s, a);
  return itts::check_launch(fn);
}
