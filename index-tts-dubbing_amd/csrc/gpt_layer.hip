// One GPT-2 decode layer as ONE persistent launch (gfx950): the five dependent kernels of the launch
// chain (gpt_step.hip: c_attn, attention, attn.c_proj + reduce, c_fc, mlp.c_proj + reduce) become the
// phases of one grid of 256 workgroups (one per CU), joined by in-launch hand-offs, with every weight
// byte of the layer requested at the START of the launch -- before the dependency edges it would
// otherwise wait behind (MI355X_MICROARCH.md rows prefetch-credit / engine-vs-launches).
//
// Reference op: HF GPT2Block (modeling_gpt2.py:246-306) inside GPT2InferenceModel.forward
// (gpt/model.py:115-192) for one KV-cached decode step of inference_speech (gpt/model.py:655-708).
//
// Geometry (IndexTTS-1.5: D = 1024, 16 heads x 64, F = 4096; rows R <= 32, one 32-row MFMA tile):
//   workgroup b = 8 j + c: cluster c = b % 8 (round-robin dispatch puts a cluster on one XCD: a speed
//   assumption only, never a correctness one), index j in the cluster.  Cluster c owns heads 2c, 2c+1,
//   c_fc columns [512c, 512c+512) and K range [512c, 512c+512) of mlp.c_proj (= split s of the chain's
//   split-K 8), and k-steps [128c, 128c+128) of attn.c_proj (its split c).  8 waves; after the q/k/v
//   sweep each wave requests 1/8 of this workgroup's attn.c_proj slice (8 KiB) into LDS by LDS-DMA, and
//   after the E2 add 1/8 of its c_fc / mlp.c_proj slices (64 KiB, round 6: issued with the attention,
//   the first key round waited for them), so the weights of the later phases stream while the hand-offs
//   run.  (A dedicated 9th loader wave cost 3 waves per SIMD = 168 VGPRs and spilled.)
//   A  c_attn (ln_1 folded): 12 columns of head h = 2c + j/16 (3072 / 256), A = x^ (previous launch).
//      The attention waves request their first round of K/V rows BEFORE this phase's MFMAs.
//   E1 q/k/v -> attention: 8-byte {tag, value} granules (the data is the flag: no drain, so the K/V
//      loads stay in flight), 16 producers -> the same 16 workgroups.
//   B  attention of rows 2(j%16), 2(j%16)+1 of head h (4 waves each; the attn_decode_kernel algorithm).
//   E2 o -> attn.c_proj: write-through stores, drain, one counter per cluster (32 adders).
//   C  attn.c_proj split c: 32 output columns (tile j), 8 k-steps of 16 (one per wave) -> partial.
//   E3 partials -> reduce: one counter per column tile j (8 adders, one per cluster).
//   D  tile j's owner (cluster j % 8, round 6): x1 = x + (b_o + sum_c partial_c), x1^ -> every cluster's copy (E4:
//      32 adders, the tile owners) and f32 x1 for phase G; the other workgroups go straight to E4.
//   E  c_fc (ln_2 folded) + gelu: 16 columns (tile 32c + j), A = the cluster's x1^.
//   E5 f -> mlp.c_proj: cluster counter (32 adders).
//   F  mlp.c_proj split c: 32 columns (tile j), 32 k-steps of 16 (4 per wave) -> partial.
//   E6 partials -> reduce (8 adders per tile); G  x2 = x1 + (b_proj + sum_c partial_c), x, x^ stored.
// Every phase is the chain kernel's arithmetic in the chain kernel's order (same MFMA shapes, same
// k-step-to-wave interleave, same fixed-order cross-wave and cross-split sums), so the layer is
// bit-identical to the launch chain with attn.c_proj as split-K 8 + reduce (gpt_step.hip).
// Hand-offs (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md visibility table row 1):
// payload stored sc1 (write-through), every storing wave s_waitcnt vmcnt(0), workgroup barrier, ONE
// lane adds to the counter (relaxed, agent scope); the consumer polls relaxed with s_sleep, every load
// of handed-off bytes is an sc1 load.  Every spin is bounded: a timeout sets an error word and the
// whole grid drains (results then garbage, the host reports the error and re-arms the scratch with
// itts_gpt_pl_reset).
// Epochs (round 5): nothing is reset between steps.  Launch number E (a u32 in the scratch, E = seq + 1,
// advanced by workgroup 0 once every workgroup of the launch has read it) tags every q/k/v granule, and
// every hand-off counter only grows: after launch E a counter with n adders per launch holds n * E, so
// the poll target is n * E (wrap-safe signed compare).  A value left by an earlier launch (a granule's
// tag, a counter line some cache kept) is below / unequal to this launch's and can never satisfy a
// poll, whatever happened between the launches (round 4 zeroed them per step: as a memset node that let
// 30 of 64 reused-lane cues decode wrong data).
#include <cstdlib>

#include "common.h"

namespace {

constexpr int kD = 1024, kH = 16, kHD = 64, kF = 4096;
constexpr int kNC = 8, kCPC = 32, kWG = kNC * kCPC;  // clusters, workgroups per cluster, grid
constexpr int kNW = 8;                                // compute waves
constexpr int kThreads = kNW * 64;
constexpr int kQC = 12;                               // c_attn columns per workgroup
#ifndef ITTS_PL_KB
#define ITTS_PL_KB 4  // 8: 666.5 us per C3 step, 4: 661.3, 12: 684 (profiles/lib_ab2.sh)
#endif
constexpr int kKB = ITTS_PL_KB;  // attention keys per group per round (load depth; results do not depend on it)
// steps of at most kSmallRows rows (C2 = one row, the long-form tail chunks): the c_attn / c_fc phases skip the
// second 16-row half of their A operands (H16) and the attention keeps kKBSmall keys per group per round in
// flight.  C2 decode step (profiles/r05e_batch1.txt): 567-580 us with neither, 527-529 with H16 and 12 keys,
// 521-523 with H16 and 8 (4: 524-525, 16: 545, which spills)
#ifndef ITTS_PL_KB_SMALL
#define ITTS_PL_KB_SMALL 8
#endif
#ifndef ITTS_PL_SMALL_ROWS
#define ITTS_PL_SMALL_ROWS 16
#endif
constexpr int kKBSmall = ITTS_PL_KB_SMALL, kSmallRows = ITTS_PL_SMALL_ROWS;
#ifndef ITTS_PL_KV_UNCOND
#define ITTS_PL_KV_UNCOND 1
#endif
#ifndef ITTS_PL_DMA_SPLIT  // small steps: an idle unit's waves issue the weight DMA of a half-active workgroup
#define ITTS_PL_DMA_SPLIT 1
#endif
// full steps: only attn.c_proj's slice (8 KiB) goes out with the attention; the c_fc / mlp.c_proj slices (64 KiB)
// after the E2 add, in the hand-off's idle window (the first key round waits for every DMA the wave issued before
// it: the compiler's vmcnt(0) after an LDS-DMA)
#ifndef ITTS_PL_DMA_TAIL
#define ITTS_PL_DMA_TAIL 1
#endif
#ifndef ITTS_PL_SMALL_H16  // small steps also skip the second 16-row half of the c_attn / c_fc A operands
#define ITTS_PL_SMALL_H16 1
#endif
constexpr bool kSmallH16 = ITTS_PL_SMALL_H16 != 0;
#ifndef ITTS_BEAM_KV_NT
#define ITTS_BEAM_KV_NT 0
#endif
static_assert(kSmallRows <= 16, "small steps fit one 16-row half");
static_assert(kKB % 4 == 0 && kKBSmall % 4 == 0, "keys per round: whole kSub chunks");
constexpr int kSub = 4;                               // keys per online-softmax chunk (gpt_attn.hip)
constexpr uint32_t kSpinMax = 1u << 19;               // bounded spins (~0.3 s), then the grid drains
// ITTS_PL_TRACE=1 (timing builds): wave 0 of every workgroup stamps the 100-MHz real-time counter at
// the phase boundaries of layer ITTS_PL_TRACE_LAYER into the scratch trace block (profiles/pl_trace.py)
#ifndef ITTS_PL_TRACE
#define ITTS_PL_TRACE 0
#endif
#ifndef ITTS_PL_TRACE_LAYER
#define ITTS_PL_TRACE_LAYER 10
#endif
// hand-off accesses: agent scope (the grid is one device); write-through stores / loads carry sc1 (aux 16)
#define PL_SCOPE __HIP_MEMORY_SCOPE_AGENT
constexpr int PL_AUX = 16;
// Variants built, measured slower or neutral and removed in round 6 (their numbers stay in DESIGN.md §4c):
// several layers per launch (C3 714 vs 647 us), split softmax groups for one-row steps (C2 604 vs 500 us),
// beam-major attention rows (beam3 1422 vs 1330 us), 16-B x1^ / partial stores (neutral), pass-0 K/V after
// c_attn (687 vs 665 us), the weight DMA at launch start (685 vs 665 us) or after the first key round (653 vs
// 648 us), every layer's weights with the default cache policy (neutral), the debug / protocol A/B switches.

// scratch layout (bytes) for up to kMaxR rows; counters, granules, the epoch and the error word are zero after
// itts_gpt_pl_reset (and after the caller's zero fill at allocation), never between steps
constexpr int kMaxR = 128;
// hand-off counters, one per 4-KiB block: 256 workgroups polling counters that share one line saturated
// it (hand-offs observed 2.5-6 us after the last arrival, profiles/pl_trace_r04b.txt); ITTS_PL_CNT_STRIDE=1
// packs them (A/B)
#ifndef ITTS_PL_CNT_STRIDE
#define ITTS_PL_CNT_STRIDE 1024
#endif
constexpr int kCntStride = ITTS_PL_CNT_STRIDE;  // u32 units
constexpr int kNumCnt = 88;
constexpr int64_t kOffCnt = 0;
constexpr int64_t kOffGq = ((int64_t)kNumCnt * kCntStride * 4 + 511) / 512 * 512;                                       // [128 rows][16 heads][192] u64
constexpr int64_t kOffOb = kOffGq + (int64_t)kMaxR * kH * 192 * 8;    // [8][128][128] bf16
constexpr int64_t kOffP1 = kOffOb + (int64_t)kNC * kMaxR * 128 * 2;   // [8][128][1024] f32
constexpr int64_t kOffXc = kOffP1 + (int64_t)kNC * kMaxR * kD * 4;    // [8][128][1024] bf16
constexpr int64_t kOffFc = kOffXc + (int64_t)kNC * kMaxR * kD * 2;    // [8][128][512] bf16
constexpr int64_t kOffP2 = kOffFc + (int64_t)kNC * kMaxR * 512 * 2;   // [8][128][1024] f32
constexpr int64_t kOffX1 = kOffP2 + (int64_t)kNC * kMaxR * kD * 4;    // [128][1024] f32: x1 (phase D -> phase G)
constexpr int64_t kOffTrace = kOffX1 + (int64_t)kMaxR * kD * 4;       // [256 WG][32] u64 (ITTS_PL_TRACE builds)
constexpr int64_t kOffSeq = kOffTrace + (int64_t)kWG * 32 * 8;        // u32 epoch: launches since the reset
constexpr int64_t kOffErr = kOffSeq + 4;  // sticky error word, beside the epoch: one 8-B load reads both
constexpr int64_t kScratchBytes = kOffSeq + 256;
constexpr int64_t kZeroBytes = kOffGq + (int64_t)kMaxR * kH * 192 * 8;  // counters + every granule (x16)
enum { CNT2 = 0, CNT3 = 8, CNT4 = 40, CNT5 = 48, CNT6 = 56 };

// LDS layout (bytes)
constexpr int L_WO = 0, L_WFC = L_WO + 8 * 1024, L_WPJ = L_WFC + 32 * 1024, L_RED = L_WPJ + 32 * 1024;
constexpr int L_STAT = L_RED + 32 * 1024;                      // rsum[8][32], rsq[8][32], mu[32], rs[32]
constexpr int kPvRows = 32 + 4 + 1, kPvPitch = kHD + 1;
constexpr int kUnitBytes = (3 * kHD + 2 * 32 + kPvRows * kPvPitch + kHD) * 4;  // qs kn vn gm gl pv ofin
constexpr int L_ATT = L_STAT + (2 * 8 * 32 + 2 * 32) * 4;
constexpr int L_OBF = L_ATT + 2 * ((kUnitBytes + 15) / 16 * 16);  // [2][64] bf16 o, then [32][16] bf16 f
constexpr int L_FLAG = L_OBF + 32 * 16 * 2;
constexpr int kLdsBytes = L_FLAG + 16;
constexpr int kRestBytes = kLdsBytes - L_RED;  // everything after the weight slices
// LDS as four static objects: the three weight-slice destinations of the LDS-DMA and the rest.  With one
// dynamic array the compiler cannot tell the in-flight DMA's destination from the attention / merge
// scratch and put `s_waitcnt vmcnt(0)` (the whole 72 KiB DMA) in front of every LDS access after the
// DMA issue; distinct objects get distinct alias scopes, so only the reads of the weights wait.

// one layer's weights
struct PlLayerPtrs {
  const u32x4_t* qkv_w12;  // [256][32 ks][4 q][12 c] x 16 B
  const float* qkv_uc;     // [256][2][12]
  const u32x4_t* o_w;      // attn.c_proj, pack_skinny [32 tiles][64 ks][64][8]
  const float* o_b;
  const u32x4_t* fc_w16;   // c_fc (ln_2 folded), pack_skinny16 [256 tiles][32 ks][64][8]
  const float *fc_u, *fc_c;
  const u32x4_t* proj_w;   // mlp.c_proj, pack_skinny [32 tiles][256 ks][64][8]
  const float* proj_b;
};
// beams (kv_rows): each attention unit stages its row's lineage indices (keys 0 .. nk-1) in LDS, so a key
// round's K/V addresses need an LDS read, not a global load whose vmcnt wait (in order) also waited for the
// round's V rows still in flight; max_kv of a beam state must not exceed this
constexpr int kKviMax = 3584;
struct PlArgs {
  float* x;                // [R][1024] f32
  uint16_t* xh;            // [32][1024] bf16 (rows >= R: read, never written)
  uint16_t *kc, *vc;       // this layer's cache [R][16][max_kv][64]
  int64_t cache_bs, cache_hs;
  const int32_t* pad;
  const int32_t* tstate;
  const int32_t* kv_rows;  // beams: [R][ld_rows] cache row of each prefix position, else null
  int64_t ld_rows;
  int kv_base, kstep, R, layer, last;  // last: the model's last layer (its x2 reduce runs outside, with ln_f)
  float eps;
  unsigned char* scratch;
  PlLayerPtrs ly;
};

// workgroup barrier that waits for this wave's LDS traffic only: a __syncthreads() would also drain
// every vector-memory load in flight (the K/V rows requested ahead of the c_attn phase)
__device__ __forceinline__ void bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// Cancelled buffer stores (row tiles > 1): a lane with nothing to store hands its buffer store the offset kDrop,
// past the range kDropLimit of every descriptor such a store uses, and the hardware drops it.  kDrop must lie past
// the range under either bounds rule (offset >= range, or offset + size > range), and ONLY buffer stores whose
// descriptor carries the kDropLimit range may ever see it: with the full 0x7fffffff range a 2- or 8-byte store at
// 0x7ffffff0 is in range and lands 2 GiB past the base (the r05t illegal address).  The host checks
// that every real offset such a descriptor addresses lies below kDropLimit (check_state: the K/V cache extent).
constexpr int kDropLimit = 0x7fff0000, kDrop = 0x7ffffff0;
static_assert(kDrop >= kDropLimit && (int64_t)kDrop + 2 > kDropLimit, "cancelled stores must be out of range");
// s_waitcnt immediate (gfx9 encoding) waiting for vmcnt <= n only (expcnt / lgkmcnt at their maxima)
constexpr int vm_wait_enc(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
// every storing wave's write-through stores have left (Guideline 16 R1: before the counter add)
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t ld_relaxed(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, PL_SCOPE);
}
__device__ __forceinline__ void add_relaxed(uint32_t* p) {
  __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, PL_SCOPE);
}
__device__ __forceinline__ void st_sc1_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, PL_SCOPE);
}
__device__ __forceinline__ uint64_t ld_sc1_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, PL_SCOPE);
}

// one lane polls `ctr` until it reaches target (bounded; counters only grow, so the compare is the wrap-safe
// signed difference); returns false on timeout / a failed grid
__device__ bool poll_ge(const uint32_t* ctr, uint32_t target, uint32_t* err, uint32_t code) {
  for (uint32_t n = 0;; ++n) {
    if ((int32_t)(ld_relaxed(ctr) - target) >= 0) return true;
    if ((n & 255) == 255 && ld_relaxed(err) != 0) return false;
    if (n > kSpinMax) {
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, PL_SCOPE);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// H16 (steps of at most 16 rows, MT = 1): the c_attn / c_fc phases load and multiply only the first 16-row
// half of their A operands (rows 16-31 are padding: their outputs, never read, come out as the fold terms)
// NBM (beam states of NBM beams, R <= 32 NBM): the attention runs ONE pass, unit (jj, u) taking utterance 2 jj + u
// with all its beams (rows NBM ui + k): a key's lineage rows of the NBM beams are requested together (default cache
// policy: where the beams share a row, one request fetches it and the others hit in L1 / L2), instead of MT passes
// of one row per unit one after the other.  Per row the same arithmetic in the same order: bit-identical.
template <int MT, bool ROWS, int KB = kKB, bool H16 = false, int NBM = 0>
__global__ __launch_bounds__(kThreads) void gpt_layer_pl_kernel(PlArgs p) {
  static_assert(!H16 || MT == 1, "16-row halves: one row tile");
  static_assert(NBM == 0 || (ROWS && !H16 && NBM >= 2 && NBM <= 4 && MT <= NBM), "beam-major: beam states");
  constexpr int NLD = NBM > 0 ? NBM : 1;
  constexpr int WAUX = 2;              // LDS-DMA cache policy of the weight stream: non-temporal
  constexpr int NHF = H16 ? 1 : 2;     // 16-row halves of the A operands loaded / multiplied
  __shared__ __attribute__((aligned(16))) unsigned char lds_wo[8 * 1024];
  __shared__ __attribute__((aligned(16))) unsigned char lds_wfc[32 * 1024];
  __shared__ __attribute__((aligned(16))) unsigned char lds_wpj[32 * 1024];
  __shared__ __attribute__((aligned(16))) unsigned char lds_rest[kRestBytes];
  __shared__ int32_t lds_kvi[ROWS ? 2 * kKviMax : 1];  // [unit][key] lineage cache rows (beams)
  unsigned char* const smem = lds_rest - L_RED;  // offsets >= L_RED address lds_rest
  typedef __attribute__((address_space(3))) void lds_void;
  const PlLayerPtrs& Ly = p.ly;
  const int b = blockIdx.x;
  const int c = b % kNC, j = b / kNC;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = j >> 4, jj = j & 15, h = 2 * c + hh;
  uint32_t* const cnt = reinterpret_cast<uint32_t*>(p.scratch + kOffCnt);
  auto cnt_ = [&](int i) { return cnt + (int64_t)i * kCntStride; };
  uint32_t* const err = reinterpret_cast<uint32_t*>(p.scratch + kOffErr);
  uint32_t* const seq = reinterpret_cast<uint32_t*>(p.scratch + kOffSeq);
  uint64_t* const gq = reinterpret_cast<uint64_t*>(p.scratch + kOffGq);
  float* const p1 = reinterpret_cast<float*>(p.scratch + kOffP1);
  float* const p2 = reinterpret_cast<float*>(p.scratch + kOffP2);
  unsigned char* const xc = p.scratch + kOffXc;
  auto rsrc_of = [&](int64_t off) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(p.scratch + off, 0, 0x7fffffff, 0x00020000);
  };
  // descriptors whose stores a lane can cancel: range kDropLimit, and a cancelled lane's offset kDrop lies past it
  auto rsrc_lim = [&](void* base) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, kDropLimit, 0x00020000);
  };
  float* red = reinterpret_cast<float*>(smem + L_RED);
  float* rsum = reinterpret_cast<float*>(smem + L_STAT);
  float* rsq = rsum + 8 * 32;
  float* mu = rsq + 8 * 32;
  float* rsd = mu + 32;
  int* abort_flag = reinterpret_cast<int*>(smem + L_FLAG);
  uint16_t* obf = reinterpret_cast<uint16_t*>(smem + L_OBF);  // o staging [2][64], then f tiles [32][16]
  const int R = p.R;
  if (tid == 0) *abort_flag = 0;
  uint64_t* trace = reinterpret_cast<uint64_t*>(p.scratch + kOffTrace) + 32 * b;
  auto mark = [&](int i) {
    if (ITTS_PL_TRACE && p.layer == ITTS_PL_TRACE_LAYER && tid == 0) trace[i] = __builtin_amdgcn_s_memrealtime();
  };
  mark(0);

  const int c16 = lane & 15, q4 = lane >> 4, r32 = lane & 31, hb = lane >> 5;
  const int kidx = p.kv_base + p.tstate[0] + p.kstep;
  // this launch's epoch and the sticky error word: plain loads (written by earlier launches) beside the step
  // counter's, so all are waited for together before the K/V addresses (an sc1 load at launch start was waited
  // for on its own: +12 us per step, r05a).  After a hand-off timeout every later launch returns here at once, so
  // the rest of a graph replay drains in microseconds and the host's launch-chain re-run starts right away.
  const uint64_t seq_err = *reinterpret_cast<const uint64_t*>(seq);
  const uint32_t L1 = (uint32_t)seq_err + 1u;
  // a hand-off of an earlier launch timed out: this launch only runs to its q/k/v sweep and returns (no poll, no
  // spin), so the rest of a graph replay drains in microseconds.  (Not an early return at entry: the branch would
  // serialise this load in front of the step counter's and cost a scalar round trip on every launch.)
  const bool dead = (uint32_t)(seq_err >> 32) != 0u;
  // attention: this workgroup's rows of head h are 32 pt + 2 jj + u (pass pt, unit u = waves 4u .. 4u+3)
  const int u = w >> 2;
  const int tu = tid - 256 * u, g = tu >> 3, d8 = tu & 7;
  constexpr int NG = 32;
  u32x4_t kr[KB], vr[KB];
  u32x4_t kb[NLD][KB], vb[NLD][KB];  // NBM: every beam's rows of a round
  // K/V rows of key index jk (0-based from the row's first valid key) of row `row`: the row's own cache
  // row, or (beams) the row of kv_rows[row][position] that holds that prefix position
  auto kv_ptr = [&](const uint16_t* cache, int row, int pos, int jk) -> const uint16_t* {
    int crow = row;
    if constexpr (ROWS) crow = lds_kvi[u * kKviMax + jk];
    return cache + (int64_t)crow * p.cache_bs + (int64_t)h * p.cache_hs + (int64_t)pos * kHD + 8 * d8;
  };
  auto kv_load = [&](u32x4_t (&dst)[KB], const uint16_t* cache, int row, int p0, int nk, int j0) {
#pragma unroll
    for (int uu = 0; uu < KB; ++uu) {
      const int jk = min(j0 + NG * uu + g, max(nk - 2, 0));
      const u32x4_t* src = reinterpret_cast<const u32x4_t*>(kv_ptr(cache, row, p0 + jk, jk));
      // beams: default cache policy, so the other beams of the utterance (units of this cluster, one XCD) find
      // the shared lineage rows in L2 (gpt_attn.hip ITTS_BEAM_KV_NT)
      if constexpr (ROWS && !ITTS_BEAM_KV_NT)
        dst[uu] = *src;
      else
        dst[uu] = __builtin_nontemporal_load(src);
    }
  };
  auto unit_row = [&](int pt) { return 32 * pt + 2 * jj + u; };
  // NBM: this unit's utterance (NBM rows) and whether it exists
  const int ui = 2 * jj + u;
  const bool act_bm = NBM > 0 && NBM * ui < R;
  const int uib = act_bm ? ui : 0;
  // NBM: the lineage cache rows of the unit's beams (keys 0 .. nk-1) packed one byte a beam (rows < 128) into
  // LDS; every thread of the workgroup calls it (it ends with the barrier the readers need)
  auto stage_kvi_bm = [&](int p0, int nk) __attribute__((always_inline)) {
    if constexpr (NBM > 0) {
      const int32_t* src = p.kv_rows + (int64_t)(NBM * uib) * p.ld_rows + p0;
      for (int i = tu; i < nk; i += 256) {
        uint32_t pk = 0;
#pragma unroll
        for (int k = 0; k < NBM; ++k) pk |= (uint32_t)src[(int64_t)k * p.ld_rows + i] << (8 * k);
        lds_kvi[u * kKviMax + i] = (int32_t)pk;
      }
      bar();
    }
  };
  auto kv_load_bm = [&](u32x4_t (&dst)[NLD][KB], const uint16_t* cache, int p0, int nk, int j0) {
#pragma unroll
    for (int uu = 0; uu < KB; ++uu) {
      const int jk = min(j0 + NG * uu + g, max(nk - 2, 0));
      const uint32_t pk = (uint32_t)lds_kvi[u * kKviMax + jk];
#pragma unroll
      for (int k = 0; k < NLD; ++k) {
        const int crow = (pk >> (8 * k)) & 255;
        dst[k][uu] = *reinterpret_cast<const u32x4_t*>(cache + (int64_t)crow * p.cache_bs + (int64_t)h * p.cache_hs +
                                                       (int64_t)(p0 + jk) * kHD + 8 * d8);
      }
    }
  };
  // beams: this unit's lineage indices of row `row` (keys 0 .. nk-1) into LDS; every thread of the workgroup
  // calls it (it ends with the barrier the readers need)
  auto stage_kvi = [&](int row, int p0, int nk) __attribute__((always_inline)) {
    if constexpr (ROWS) {
      const int32_t* src = p.kv_rows + (int64_t)row * p.ld_rows + p0;
      for (int i = tu; i < nk; i += 256) lds_kvi[u * kKviMax + i] = src[i];
      bar();
    }
  };
  const int xrow = tid >> 4, xcol = 32 * j + 2 * (tid & 15);  // phases D / G: this thread's 2 columns per tile
  // (phase G: wave w holds rows 4w .. 4w+3 of every row tile, xrow >> 2 == w)

  // ---- (A0) c_attn operands first (12 of 16 fragment columns real, default cache policy: 126 MB over the
  // layers that can stay in the Infinity Cache; A = x^ tile 0), then the attention's first round of K/V rows
  // (pass 0), then the residual slices; the weight DMA goes out after the q/k/v sweep
  u32x4_t bw[4], av[4][2];
  float uc0, uc1;  // the lane's c_attn fold terms (column lane % 16 of this workgroup's 12)
  // the residual slices (rows xrow of every tile, this thread's 2 columns), selected at phase D: no early wait
  float2 x_raw[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int row = 32 * t + xrow, xr = row < R ? row : R - 1;
    x_raw[t] = *reinterpret_cast<const float2*>(p.x + (int64_t)xr * kD + xcol);
  }
  // this workgroup's attn.c_proj (8 KiB), c_fc (32 KiB), mlp.c_proj (32 KiB) weight slices, global ->
  // LDS by DMA (1 KiB per wave instruction, lane-linear = fragment order, nt), instruction t by wave t % 8
  // small steps (H16) in a workgroup whose unit 0 has a row and unit 1 none (odd R; C2: R = 1): unit 1's idle
  // waves issue the whole burst, so unit 0's later K/V rounds do not retire behind it (in-order vmcnt) -- at
  // one row per head those few units are the critical path
  const bool dma_split = ITTS_PL_DMA_SPLIT && H16 && 2 * jj < R && 2 * jj + 1 >= R;  // workgroup-uniform
  auto dma_one = [&](int t) {
    // t is wave-uniform: each branch is one uniform DMA into its own LDS object
    if (t < 8)
      __builtin_amdgcn_global_load_lds(Ly.o_w + (((int64_t)j * 64 + 8 * c + t) * 64 + lane),
                                       (lds_void*)(lds_wo + t * 1024), 16, 0, WAUX);
    else if (t < 40)
      __builtin_amdgcn_global_load_lds(Ly.fc_w16 + (((int64_t)(32 * c + j) * 32 + (t - 8)) * 64 + lane),
                                       (lds_void*)(lds_wfc + (t - 8) * 1024), 16, 0, WAUX);
    else
      __builtin_amdgcn_global_load_lds(Ly.proj_w + (((int64_t)j * 256 + 32 * c + (t - 40)) * 64 + lane),
                                       (lds_void*)(lds_wpj + (t - 40) * 1024), 16, 0, WAUX);
  };
  // straight-line issue (a data-dependent trip count leaves the compiler's vmcnt tracking a join it resolves
  // with vmcnt(0): the first key round then waited for the whole burst)
  auto issue_dma = [&]() {
    if (dma_split) {
      if (w >= 4) {
#pragma unroll
        for (int m = 0; m < 18; ++m) dma_one(w - 4 + 4 * m);
      }
    } else if (ITTS_PL_DMA_TAIL) {
      dma_one(w);  // attn.c_proj's slice; the rest in issue_dma_tail
    } else {
#pragma unroll
      for (int m = 0; m < 9; ++m) dma_one(w + 8 * m);
    }
  };
  // the c_fc / mlp.c_proj slices (instructions 8 .. 71), every wave, after the E2 add (ITTS_PL_DMA_TAIL).
  // Measured and not kept (profiles/dmatail_r06fg.txt, dmatail_r06hk.txt): the burst by waves 1-7 only (the E2
  // poller none), the mlp.c_proj half after the E3 add, and the burst by the six waves that store no o row as their
  // key loop ends or once the merge is past their last LDS read -- issuing 64 KiB of DMA holds a CU's memory pipe
  // for ~2.5 us wherever it goes, and only the E2 wait has that much idle time
  auto issue_dma_tail = [&]() __attribute__((always_inline)) {
    if (ITTS_PL_DMA_TAIL && !dma_split) {
#pragma unroll
      for (int m = 1; m < 9; ++m) dma_one(w + 8 * m);
    }
  };
  // pass 0's first valid key (its row's left padding), loaded once here: re-read at the pass (after the asm memory
  // clobbers of the barriers, a fresh load) it was a vector load whose vmcnt(0) waited for phase A's granule and
  // cache stores
  // (one row tile only: at 96 beam rows beam3 measured 1172 -> 1183 us with it, r06q)
  const int rr0 = NBM > 0 ? NBM * uib : (unit_row(0) < R ? unit_row(0) : 0);
  const int p0_first = MT == 1 && p.pad ? p.pad[rr0] : 0;
  // the attention's first round of K/V rows (pass 0)
  auto kv_round0 = [&]() {
    if constexpr (NBM > 0) {
      const int p0 = p.pad ? p.pad[NBM * uib] : 0, nk = kidx + 1 - p0;
      stage_kvi_bm(p0, nk);
      kv_load_bm(kb, p.kc, p0, nk, 0);
      kv_load_bm(vb, p.vc, p0, nk, 0);
    } else {
      const int rr = rr0;
      const int p0 = MT == 1 ? p0_first : (p.pad ? p.pad[rr] : 0), nk = kidx + 1 - p0;
      stage_kvi(rr, p0, nk);
      kv_load(kr, p.kc, rr, p0, nk, 0);
      kv_load(vr, p.vc, rr, p0, nk, 0);
    }
  };
  // x^ rows of the NEXT row tiles were written by the previous launch: plain buffer loads (sc1, as any hand-off)
  const auto rsrc_xh = __builtin_amdgcn_make_buffer_rsrc(p.xh, 0, 0x7fffffff, 0x00020000);
  {
    const u32x4_t* wq = Ly.qkv_w12 + (int64_t)b * 32 * 4 * kQC;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = w + 8 * i;
      bw[i] = wq[(s * 4 + q4) * kQC + (c16 < kQC ? c16 : 0)];
#pragma unroll
      for (int t = 0; t < NHF; ++t)
        av[i][t] = *reinterpret_cast<const u32x4_t*>(p.xh + (int64_t)(16 * t + c16) * kD + 32 * s + 8 * q4);
    }
    // the lane's fold terms: one row tile (MT = 1) beside the operands (loaded in the epilogue, behind the K/V rows,
    // it waited for the whole first K/V round, in-order vmcnt: C2 479 -> 473 us, C3 unchanged, r06p); row tiles
    // > 1 behind the K/V rows (beside them beam3 measured 1174 -> 1185 us)
    const int cq = (lane & 15) < kQC ? (lane & 15) : 0;
    if constexpr (MT == 1) {
      uc0 = Ly.qkv_uc[(int64_t)b * 2 * kQC + cq];
      uc1 = Ly.qkv_uc[(int64_t)b * 2 * kQC + kQC + cq];
    }
    __builtin_amdgcn_sched_barrier(0);
    kv_round0();
    if constexpr (MT > 1) {
      uc0 = Ly.qkv_uc[(int64_t)b * 2 * kQC + cq];
      uc1 = Ly.qkv_uc[(int64_t)b * 2 * kQC + kQC + cq];
    }
  }

  // fold statistics of one 32-row tile (the A fragments a wave accumulated): sums -> mu / rstd in LDS
  auto fold_stats = [&](const float (&ss)[2], const float (&sq)[2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float a = ss[t], s2 = sq[t];
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (q4 == 0) {
        rsum[w * 32 + 16 * t + c16] = a;
        rsq[w * 32 + 16 * t + c16] = s2;
      }
    }
  };
  auto mu_rs = [&]() {
    if (tid < 32) {
      float S = 0.f, Q = 0.f;
#pragma unroll
      for (int ww = 0; ww < kNW; ++ww) {
        S += rsum[ww * 32 + tid];
        Q += rsq[ww * 32 + tid];
      }
      fold_mu_rs(S, Q, 1.0f / kD, p.eps, mu[tid], rsd[tid]);
    }
  };
  mark(1);

  // ---- (A) c_attn per 32-row tile: decode_gemm16x FOLD arithmetic (k-steps w + 8i, statistics from the
  // A fragments); q / k / v of row r, head h -> granules gq[r][h][192]; this step's k / v into the cache
  // row tiles > 0 (beams, long-form chunks): the next tile's A fragments are requested before this tile's
  // MFMAs (double-buffered; loaded inside the loop they were one serial round trip per tile: c_attn 8.8 us
  // at 3 tiles, profiles/pl_trace_r05q_96.txt)
  u32x4_t avn[4][2];
#pragma unroll  // (MT > 1: straight-line tiles, so the compiler's vmcnt counts stay exact across them)
  for (int t = 0; t < MT; ++t) {
    if (MT > 1 && t + 1 < MT) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
          avn[i][hf] = __builtin_amdgcn_raw_buffer_load_b128(
              rsrc_xh, ((32 * (t + 1) + 16 * hf + c16) * kD + 32 * (w + 8 * i) + 8 * q4) * 2, 0, PL_AUX);
    }
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
    float ssum[2] = {0.f, 0.f}, ssq[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(&bw[i]);
      const bf16x8_t bz = c16 < kQC ? bfr : bf16x8_t{};
#pragma unroll
      for (int hf = 0; hf < NHF; ++hf) {
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&av[i][hf]);
        acc[hf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bz, acc[hf], 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = (float)a[e];
          ssum[hf] += v;
          ssq[hf] = fmaf(v, v, ssq[hf]);
        }
      }
    }
    fold_stats(ssum, ssq);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(w * 8 + 4 * hf + r) * 64 + lane] = acc[hf][r];
    bar();
    mu_rs();
    bar();
    if constexpr (MT > 1) {
      // several row tiles: the same outputs, but every store instruction issued by every wave (lanes with no
      // output get the offset kDrop past the descriptor's range: the hardware drops them), so the compiler counts
      // the stores exactly and waits for the next tile's A fragments without waiting for these write-through
      // stores (with lane-conditional stores its wait at the tile loop's head was vmcnt(0))
      const int e = tid >> 6, l = lane, col = l & 15;
      const bool ok = col < kQC;
      const int cq = ok ? col : 0;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < kNW; ++ww) v += red[(ww * 8 + e) * 64 + l];
      const int rt = 16 * (e >> 2) + 4 * (l >> 4) + (e & 3), row = 32 * t + rt;
      v = fold_apply(v, rsd[rt], mu[rt], uc0, uc1);
      const int i = kQC * jj + cq;
      const uint64_t gr = ((uint64_t)L1 << 32) | __float_as_uint(v);
      const int goff = ok ? (((row * kH + h) * 192 + i) * 8) : kDrop;
      __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{(uint32_t)gr, (uint32_t)(gr >> 32)}, rsrc_lim(gq), goff, 0,
                                            PL_AUX);
      const int coff = (row * (int)p.cache_bs + h * (int)p.cache_hs + kidx * kHD + (i & (kHD - 1))) * 2;
      const bool kv_ok = ok && row < R;
      const uint16_t hv = f2bf(0.f + v);
      __builtin_amdgcn_raw_buffer_store_b16(hv, rsrc_lim(p.kc), kv_ok && i >= kHD && i < 2 * kHD ? coff : kDrop, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b16(hv, rsrc_lim(p.vc), kv_ok && i >= 2 * kHD ? coff : kDrop, 0, 0);
    } else {  // one output per thread: 32 rows x 16 fragment columns (12 real)
      const int e = tid >> 6, l = lane, col = l & 15;
      if (col < kQC) {
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < kNW; ++ww) v += red[(ww * 8 + e) * 64 + l];
        const int rt = 16 * (e >> 2) + 4 * (l >> 4) + (e & 3), row = 32 * t + rt;
        v = fold_apply(v, rsd[rt], mu[rt], uc0, uc1);
        const int i = kQC * jj + col;  // index in head h's [q | k | v] 192 columns
        const uint64_t gr = ((uint64_t)L1 << 32) | __float_as_uint(v);
        __hip_atomic_store(gq + ((int64_t)row * kH + h) * 192 + i, gr, __ATOMIC_RELAXED, PL_SCOPE);
        if (i >= kHD && row < R) {  // this step's key / value into the row's own cache row (0 + v, rounded)
          uint16_t* dst = (i < 2 * kHD ? p.kc : p.vc) + (int64_t)row * p.cache_bs + (int64_t)h * p.cache_hs +
                          (int64_t)kidx * kHD + (i & (kHD - 1));
          *dst = f2bf(0.f + v);
        }
      }
    }
    if (MT > 1) {
      bar();  // red / statistics are reused by the next tile
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) av[i][hf] = avn[i][hf];
    }
  }
  mark(2);

  // ---- (E1 + B) attention passes: unit u of pass pt = row 32 pt + 2 jj + u of head h (attn_decode_kernel
  // algorithm: 32 groups x 8 lanes, keys g + 32 n, fixed kSub-key softmax chunks, fixed-order merge)
  unsigned char* ub = smem + L_ATT + u * ((kUnitBytes + 15) / 16 * 16);
  float* qs = reinterpret_cast<float*>(ub);
  float* kn = qs + kHD;
  float* vn = kn + kHD;
  float* gm = vn + kHD;
  float* gl = gm + 32;
  float* pv = gl + 32;
  constexpr int NQ = 4, GPQ = 8;
  float* qsum = pv + 32 * kPvPitch;
  float* lsum = qsum + NQ * kPvPitch;
  // the unit's 32 group partials (pv, gm, gl: written by the caller) -> o row r_store (fixed-order merge); every
  // thread of the workgroup calls it
  auto merge_store = [&](bool act, int r_store) __attribute__((always_inline)) {
    bar();
    if (act) {
      const int dd = tu & (kHD - 1), qd = tu / kHD;
      float M = -INFINITY;
#pragma unroll
      for (int i = 0; i < NG; ++i) M = fmaxf(M, gm[i]);
      float Ls = 0.f, a = 0.f;
#pragma unroll
      for (int i = qd * GPQ; i < qd * GPQ + GPQ; ++i) {
        const float wgt = __expf(gm[i] - M);
        Ls = fmaf(gl[i], wgt, Ls);
        a = fmaf(pv[i * kPvPitch + dd], wgt, a);
      }
      qsum[qd * kPvPitch + dd] = a;
      if (dd == 0) lsum[qd] = Ls;
    }
    bar();
    if (tu < kHD) {
      float v = 0.f;
      if (act) {
        float Ls = 0.f, a = 0.f;
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
          Ls += lsum[i];
          a += qsum[i * kPvPitch + tu];
        }
        v = a / Ls;
      }
      obf[u * kHD + tu] = f2bf(v);
    }
    bar();
    if (tu < 8) {  // o rows -> the cluster's [rows][128] tile, write-through 16-B stores
      const int d0 = 8 * tu;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(obf + u * kHD + d0);
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc_of(kOffOb), ((c * kMaxR + r_store) * 128 + hh * kHD + d0) * 2, 0,
                                             PL_AUX);
    }
  };
  if constexpr (NBM == 0) {
#pragma unroll 1
  for (int pt = 0; pt < MT; ++pt) {
    const int r_u = unit_row(pt);
    const bool act_u = r_u < R;
    const int rr = act_u ? r_u : 0;
    const int p0 = MT == 1 ? p0_first : (p.pad ? p.pad[rr] : 0), nk = kidx + 1 - p0;
    if (pt > 0) {  // later passes: this pass's first round now
      stage_kvi(rr, p0, nk);
      kv_load(kr, p.kc, rr, p0, nk, 0);
      kv_load(vr, p.vc, rr, p0, nk, 0);
    }
    if ((w & 3) == 0 && act_u) {  // the unit's first wave sweeps its 192 granules
      const uint64_t* src = gq + ((int64_t)r_u * kH + h) * 192;
      uint64_t g0, g1, g2;
      bool ok = false;
      for (uint32_t n = 0; !dead; ++n) {
        g0 = ld_sc1_u64(src + lane);
        g1 = ld_sc1_u64(src + 64 + lane);
        g2 = ld_sc1_u64(src + 128 + lane);
        const bool mine = (uint32_t)(g0 >> 32) == L1 && (uint32_t)(g1 >> 32) == L1 && (uint32_t)(g2 >> 32) == L1;
        if (__all(mine)) {
          ok = true;
          break;
        }
        if (n > kSpinMax || ((n & 255) == 255 && ld_relaxed(err) != 0)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (!ok) {
        if (lane == 0) {
          if (!dead) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, PL_SCOPE);
          *abort_flag = 1;
        }
      } else {
        qs[lane] = (0.f + __uint_as_float((uint32_t)g0)) * 0.125f;  // 1/sqrt(64), exact
        kn[lane] = 0.f + __uint_as_float((uint32_t)g1);
        vn[lane] = 0.f + __uint_as_float((uint32_t)g2);
      }
    }
    bar();
    if (pt == 0) mark(3);
    if (*abort_flag || dead) return;
    // the later phases' weights: behind the c_attn operands and this pass's K/V rows, after the q/k/v
    // granule sweep (a burst issued earlier queued in front of those loads: profiles/pl_trace_r04b.txt)
    if (pt == 0) issue_dma();
    if (act_u) {
      float o8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      float m_run = -INFINITY, l_run = 0.f;
      float q[8], kme[8], vme[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        q[e] = qs[8 * d8 + e];
        kme[e] = kn[8 * d8 + e];
        vme[e] = vn[8 * d8 + e];
      }
      auto unpack = [&](const u32x4_t& r, float (&xv)[8]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          xv[2 * i] = __uint_as_float(r[i] << 16);
          xv[2 * i + 1] = __uint_as_float(r[i] & 0xFFFF0000u);
        }
      };
      // one round of KB keys per group; round 0 is peeled out of the loop: in straight-line code the
      // compiler waits only for this round's K/V rows (issued at launch start), whereas a loop header
      // waits for every load in flight -- here also the weight DMA issued after the q/k/v sweep
      auto key_round = [&](int j0) __attribute__((always_inline)) {
        // ITTS_PL_KV_UNCOND (full steps): the next round's rows are requested whether or not it exists (past
        // the last key every lane's index clamps to the row's key nk - 2), so the issue count is the same on
        // every path and the compiler's waits stay counted -- a conditional issue merges into vmcnt(0), and
        // this round's V rows were then waited for together with the next round's K rows: C3 step 648.8 /
        // 649.5 -> 640.8 / 640.6 us.  Small steps keep the conditional issue: there the one active unit's
        // useless last round sits on the critical path (C2 504.8 / 504.3 -> 516.7 / 517.3 us unconditional)
        const bool more = (ITTS_PL_KV_UNCOND && !H16) || j0 + NG * KB < nk;
        float sc[KB];
#pragma unroll
        for (int uu = 0; uu < KB; ++uu) {
          const int jk = j0 + NG * uu + g;
          float kx[8];
          unpack(kr[uu], kx);
          if (jk >= nk - 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) kx[e] = kme[e];
          }
          float pt_ = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) pt_ = fmaf(q[e], kx[e], pt_);
          pt_ = sum8_dpp(pt_);
          sc[uu] = jk < nk ? pt_ : -INFINITY;
        }
        if (more) kv_load(kr, p.kc, rr, p0, nk, j0 + NG * KB);
#pragma unroll
        for (int c0 = 0; c0 < KB; c0 += kSub) {
          float bm = -INFINITY;
#pragma unroll
          for (int uu = c0; uu < c0 + kSub; ++uu) bm = fmaxf(bm, sc[uu]);
          if (bm == -INFINITY) continue;
          const float mn = fmaxf(m_run, bm);
          const float corr = __expf(m_run - mn);
          l_run *= corr;
#pragma unroll
          for (int e = 0; e < 8; ++e) o8[e] *= corr;
#pragma unroll
          for (int uu = c0; uu < c0 + kSub; ++uu) {
            const int jk = j0 + NG * uu + g;
            const float pr = __expf(sc[uu] - mn);
            l_run += pr;
            float vx[8];
            unpack(vr[uu], vx);
            if (jk >= nk - 1) {
#pragma unroll
              for (int e = 0; e < 8; ++e) vx[e] = vme[e];
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) o8[e] = fmaf(pr, vx[e], o8[e]);
          }
          m_run = mn;
        }
        if (more) kv_load(vr, p.vc, rr, p0, nk, j0 + NG * KB);
      };
      key_round(0);  // nk >= 1: round 0 always runs
      if (pt == 0) mark(21);
      for (int j0 = NG * KB; j0 < nk; j0 += NG * KB) key_round(j0);
      if (pt == 0) mark(20);
#pragma unroll
      for (int e = 0; e < 8; ++e) pv[g * kPvPitch + 8 * d8 + e] = o8[e];
      if (d8 == 0) {
        gm[g] = m_run;
        gl[g] = l_run;
      }
    }
    merge_store(act_u, r_u);
    if (MT > 1) bar();  // the unit scratch and obf are reused by the next pass
  }
  } else {
  // ---- NBM: ONE pass over the unit's utterance, all its beams per key round ----
  float* bq = pv;  // [NBM][q | k | v][64] of this step (the merge scratch is free until the key loop ends)
  {
    const int p0 = p.pad ? p.pad[NBM * uib] : 0, nk = kidx + 1 - p0;
    if ((w & 3) < NBM && act_bm) {  // wave k of the unit sweeps beam k's 192 granules
      const int kk = w & 3, r_k = NBM * ui + kk;
      const uint64_t* src = gq + ((int64_t)r_k * kH + h) * 192;
      uint64_t g0, g1, g2;
      bool ok = false;
      for (uint32_t n = 0; !dead; ++n) {
        g0 = ld_sc1_u64(src + lane);
        g1 = ld_sc1_u64(src + 64 + lane);
        g2 = ld_sc1_u64(src + 128 + lane);
        const bool mine = (uint32_t)(g0 >> 32) == L1 && (uint32_t)(g1 >> 32) == L1 && (uint32_t)(g2 >> 32) == L1;
        if (__all(mine)) {
          ok = true;
          break;
        }
        if (n > kSpinMax || ((n & 255) == 255 && ld_relaxed(err) != 0)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (!ok) {
        if (lane == 0) {
          if (!dead) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, PL_SCOPE);
          *abort_flag = 1;
        }
      } else {
        bq[kk * 192 + lane] = (0.f + __uint_as_float((uint32_t)g0)) * 0.125f;  // 1/sqrt(64), exact
        bq[kk * 192 + 64 + lane] = 0.f + __uint_as_float((uint32_t)g1);
        bq[kk * 192 + 128 + lane] = 0.f + __uint_as_float((uint32_t)g2);
      }
    }
    bar();
    mark(3);
    if (*abort_flag || dead) return;
    issue_dma();
    float o8[NLD][8], m_run[NLD], l_run[NLD], q[NLD][8];
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      m_run[k] = -INFINITY;
      l_run[k] = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o8[k][e] = 0.f;
        q[k][e] = bq[k * 192 + 8 * d8 + e];
      }
    }
    if (act_bm) {
      auto unpack = [&](const u32x4_t& r, float (&xv)[8]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          xv[2 * i] = __uint_as_float(r[i] << 16);
          xv[2 * i + 1] = __uint_as_float(r[i] & 0xFFFF0000u);
        }
      };
      // one round of KB keys per group for every beam: the per-row arithmetic of key_round (same chunks, same
      // order); this step's own key / value (keys >= nk - 1) from the granules in LDS
      auto key_round_bm = [&](int j0) __attribute__((always_inline)) {
        float sc[NLD][KB];
#pragma unroll
        for (int k = 0; k < NLD; ++k)
#pragma unroll
          for (int uu = 0; uu < KB; ++uu) {
            const int jk = j0 + NG * uu + g;
            float kx[8];
            unpack(kb[k][uu], kx);
            if (jk >= nk - 1) {
#pragma unroll
              for (int e = 0; e < 8; ++e) kx[e] = bq[k * 192 + 64 + 8 * d8 + e];
            }
            float pt_ = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) pt_ = fmaf(q[k][e], kx[e], pt_);
            pt_ = sum8_dpp(pt_);
            sc[k][uu] = jk < nk ? pt_ : -INFINITY;
          }
        kv_load_bm(kb, p.kc, p0, nk, j0 + NG * KB);
#pragma unroll
        for (int k = 0; k < NLD; ++k)
#pragma unroll
          for (int c0 = 0; c0 < KB; c0 += kSub) {
            float bm = -INFINITY;
#pragma unroll
            for (int uu = c0; uu < c0 + kSub; ++uu) bm = fmaxf(bm, sc[k][uu]);
            if (bm == -INFINITY) continue;
            const float mn = fmaxf(m_run[k], bm);
            const float corr = __expf(m_run[k] - mn);
            l_run[k] *= corr;
#pragma unroll
            for (int e = 0; e < 8; ++e) o8[k][e] *= corr;
#pragma unroll
            for (int uu = c0; uu < c0 + kSub; ++uu) {
              const int jk = j0 + NG * uu + g;
              const float pr = __expf(sc[k][uu] - mn);
              l_run[k] += pr;
              float vx[8];
              unpack(vb[k][uu], vx);
              if (jk >= nk - 1) {
#pragma unroll
                for (int e = 0; e < 8; ++e) vx[e] = bq[k * 192 + 128 + 8 * d8 + e];
              }
#pragma unroll
              for (int e = 0; e < 8; ++e) o8[k][e] = fmaf(pr, vx[e], o8[k][e]);
            }
            m_run[k] = mn;
          }
        kv_load_bm(vb, p.vc, p0, nk, j0 + NG * KB);
      };
      key_round_bm(0);
      mark(21);
      for (int j0 = NG * KB; j0 < nk; j0 += NG * KB) key_round_bm(j0);
      mark(20);
    }
    // every beam's partials -> merge -> o row, the beams side by side (three barriers for all of them, not three
    // per beam): beam 0 in the unit scratch, beams 1.. in areas of `red` and of the lineage table (both free now);
    // the merge arithmetic and order are merge_store's
    constexpr int kArea = kPvRows * kPvPitch + 2 * 32;  // floats: pv (+ the qsum / lsum rows), gm, gl
    static_assert(NBM == 0 || 2 * (NBM - 1) * kArea <= 8192 + (ROWS ? 2 * kKviMax : 0), "merge areas fit");
    auto area = [&](int k) -> float* {  // beam k >= 1 of this unit: red first, then the lineage table
      const int a = 2 * (k - 1) + u;
      return a * kArea + kArea <= 8192 ? red + a * kArea
                                       : reinterpret_cast<float*>(lds_kvi) + (a * kArea - (8192 / kArea) * kArea);
    };
    bar();  // every wave is past its reads of bq and of the lineage table
    if (act_bm) {
#pragma unroll
      for (int k = 0; k < NLD; ++k) {
        float* pk = k == 0 ? pv : area(k);
        float* gk = k == 0 ? gm : pk + kPvRows * kPvPitch;
#pragma unroll
        for (int e = 0; e < 8; ++e) pk[g * kPvPitch + 8 * d8 + e] = o8[k][e];
        if (d8 == 0) {
          gk[g] = m_run[k];
          gk[32 + g] = l_run[k];
        }
      }
    }
    bar();
    if (act_bm) {
      const int dd = tu & (kHD - 1), qd = tu / kHD;
#pragma unroll
      for (int k = 0; k < NLD; ++k) {
        float* pk = k == 0 ? pv : area(k);
        const float* gk = k == 0 ? gm : pk + kPvRows * kPvPitch;
        const float* lk = k == 0 ? gl : gk + 32;
        float M = -INFINITY;
#pragma unroll
        for (int i = 0; i < NG; ++i) M = fmaxf(M, gk[i]);
        float Ls = 0.f, a = 0.f;
#pragma unroll
        for (int i = qd * GPQ; i < qd * GPQ + GPQ; ++i) {
          const float wgt = __expf(gk[i] - M);
          Ls = fmaf(lk[i], wgt, Ls);
          a = fmaf(pk[i * kPvPitch + dd], wgt, a);
        }
        pk[(32 + qd) * kPvPitch + dd] = a;  // qsum rows
        if (dd == 0) pk[36 * kPvPitch + qd] = Ls;  // lsum row
      }
    }
    bar();
    uint16_t* obm = reinterpret_cast<uint16_t*>(smem + L_OBF);  // [2 units][NLD][64] bf16 (fits the 1-KB o / f stage)
    if (tu < NLD * kHD) {
      const int k = tu / kHD, d = tu & (kHD - 1);
      float v = 0.f;
      if (act_bm) {
        const float* pk = k == 0 ? pv : area(k);
        float Ls = 0.f, a = 0.f;
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
          Ls += pk[36 * kPvPitch + i];
          a += pk[(32 + i) * kPvPitch + d];
        }
        v = a / Ls;
      }
      obm[(u * NLD + k) * kHD + d] = f2bf(v);
    }
    bar();
    if (tu < 8 * NLD) {  // o rows NBM ui + k -> the cluster's [rows][128] tile (a unit past the utterances: zeros)
      const int k = tu >> 3, d0 = 8 * (tu & 7);
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(obm + (u * NLD + k) * kHD + d0);
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc_of(kOffOb), ((c * kMaxR + NBM * ui + k) * 128 + hh * kHD + d0) * 2,
                                             0, PL_AUX);
    }
  }
  }  // NBM
  mark(4);
  drain();  // the o stores, and this wave's weight DMA (read from LDS from phase C on)
  bar();
  mark(15);
  if (tid == 0) add_relaxed(cnt_(CNT2 + c));
  issue_dma_tail();  // c_fc / mlp.c_proj slices (read from phase E on: drained at phase C's end)

  // ---- (C) attn.c_proj split c, tile j, per 32-row tile: decode_gemm_kernel EPI 2 (one k-step per wave)
  if (tid == 0 && !poll_ge(cnt_(CNT2 + c), kCPC * L1, err, 2)) *abort_flag = 1;
  mark(5);
  bar();
  if (*abort_flag) return;
  // 1024 outputs of row tile t, fixed-order sum over the waves, 4-B write-through stores (16-B stores gathered
  // over 4 lanes measured neutral)
  auto store_partial = [&](float* dst, int t) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int o = tid + 512 * k;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < kNW; ++ww) v += red[ww * 1024 + o];
      const int r = o >> 6, l = o & 63;
      const int row = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      st_sc1_u32(reinterpret_cast<uint32_t*>(dst + ((int64_t)c * kMaxR + row) * kD + 32 * j + (l & 31)),
                 __float_as_uint(v));
    }
  };
  {
    const u32x4_t bb = *reinterpret_cast<const u32x4_t*>(lds_wo + w * 1024 + lane * 16);
    u32x4_t ao[MT];  // every row tile's o fragment requested up front (4 VGPRs a tile)
#pragma unroll
    for (int t = 0; t < MT; ++t)
      ao[t] = __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(kOffOb),
                                                    ((c * kMaxR + 32 * t + r32) * 128 + 16 * w + 8 * hb) * 2, 0, PL_AUX);
#pragma unroll  // (MT > 1: straight-line tiles, so the compiler's vmcnt counts stay exact across them)
    for (int t = 0; t < MT; ++t) {
      const u32x4_t a = ao[t];
      f32x16_t acc32;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc32[r] = 0.f;
      acc32 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8_t*>(&a),
                                                      *reinterpret_cast<const bf16x8_t*>(&bb), acc32, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(w * 16 + r) * 64 + lane] = acc32[r];
      bar();
      store_partial(p1, t);
      bar();
    }
  }
  mark(6);
  drain();
  bar();
  mark(16);
  if (tid == 0) add_relaxed(cnt_(CNT3 + j));

  // ---- (D) x1 = x + (b_o + sum_c partial_c) on tile j (residual_reduce_ln_v4 order), by the tile's owner only
  // (cluster j % 8): one reduce per tile instead of eight (the 8 partial slabs of a tile were read by all eight
  // clusters: 8 MB per layer at 32 rows), x1^ stored into every cluster's copy (16-B write-through stores, 8 columns
  // gathered over 4 lanes), f32 x1 into the x1 slab for the other clusters' phase G
  const bool owner = c == (j & (kNC - 1));
  float2 x1[MT];
  if (owner) {
    if (tid == 0 && !poll_ge(cnt_(CNT3 + j), kNC * L1, err, 3)) *abort_flag = 1;
    mark(7);
    bar();
    if (*abort_flag) return;
    const float2 ob2 = *reinterpret_cast<const float2*>(Ly.o_b + xcol);
    const auto rxc = rsrc_of(kOffXc), rx1 = rsrc_of(kOffX1);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int row = 32 * t + xrow;
      float2 pp = ob2;
#pragma unroll
      for (int cc = 0; cc < kNC; ++cc) {
        const uint64_t v = ld_sc1_u64(reinterpret_cast<const uint64_t*>(p1 + ((int64_t)cc * kMaxR + row) * kD + xcol));
        pp.x += __uint_as_float((uint32_t)v);
        pp.y += __uint_as_float((uint32_t)(v >> 32));
      }
      const float2 xo = row < R ? x_raw[t] : float2{0.f, 0.f};
      x1[t] = float2{xo.x + pp.x, xo.y + pp.y};
      const uint32_t pk = pack2bf(x1[t].x, x1[t].y);
      const uint32_t n1 = __shfl_down(pk, 1, 64), n2 = __shfl_down(pk, 2, 64), n3 = __shfl_down(pk, 3, 64);
      if ((lane & 3) == 0) {
#pragma unroll
        for (int cc = 0; cc < kNC; ++cc)
          __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{pk, n1, n2, n3}, rxc, ((cc * kMaxR + row) * kD + xcol) * 2, 0,
                                                 PL_AUX);
      }
      __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{__float_as_uint(x1[t].x), __float_as_uint(x1[t].y)}, rx1,
                                            (row * kD + xcol) * 4, 0, PL_AUX);
    }
    mark(8);
    drain();
    bar();
    mark(17);
    if (tid < kNC) add_relaxed(cnt_(CNT4 + tid));  // one wave instruction, one lane per cluster's counter
  }

  // ---- (E) c_fc (ln_2 folded) + gelu on column tile 32c + j, per row tile, A = the cluster's x1^
  if (tid == 0 && !poll_ge(cnt_(CNT4 + c), kCPC * L1, err, 4)) *abort_flag = 1;
  // past this poll every workgroup of the grid has added at E3 (the 32 tile owners, whose adds this counter holds,
  // each waited for the 8 clusters of its tile), so all have read the epoch: workgroup 0 advances it
  if (b == 0 && tid == 0 && !*abort_flag) st_sc1_u32(seq, L1);
  mark(9);
  bar();
  if (*abort_flag) return;
  // phase G's x1 rows (wave c: rows 4c .. 4c+3 of every tile) of a tile this workgroup does not own: requested now,
  // beside the c_fc operands (visible: every owner drained before its E4 add)
  if (!owner && w == c) {
    const auto rx1 = rsrc_of(kOffX1);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rx1, ((32 * t + xrow) * kD + xcol) * 4, 0, PL_AUX);
      x1[t] = float2{__uint_as_float(v[0]), __uint_as_float(v[1])};
    }
  }
  {
    auto rsrc = rsrc_of(kOffXc);
    auto rsrc_f = rsrc_of(kOffFc);
    u32x4_t ax[4][2], axn[4][2];  // this / the next row tile's A fragments (double-buffered, as phase A)
    auto load_ax = [&](u32x4_t (&dst)[4][2], int t) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int hf = 0; hf < NHF; ++hf)
          dst[i][hf] = __builtin_amdgcn_raw_buffer_load_b128(
              rsrc, ((c * kMaxR + 32 * t + 16 * hf + c16) * kD + 32 * (w + 8 * i) + 8 * q4) * 2, 0, PL_AUX);
    };
    load_ax(ax, 0);
    const int nfc = (32 * c + j) * 16 + (lane & 15);  // this lane's c_fc column (every row tile's)
    const float fcu = Ly.fc_u[nfc], fcc = Ly.fc_c[nfc];
#pragma unroll  // (MT > 1: straight-line tiles, so the compiler's vmcnt counts stay exact across them)
    for (int t = 0; t < MT; ++t) {
      if (MT > 1 && t + 1 < MT) load_ax(axn, t + 1);
      f32x4_t af[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
      float fs[2] = {0.f, 0.f}, fq[2] = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(lds_wfc + (w + 8 * i) * 1024 + lane * 16);
#pragma unroll
        for (int hf = 0; hf < NHF; ++hf) {
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&ax[i][hf]);
          af[hf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr, af[hf], 0, 0, 0);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = (float)a[e];
            fs[hf] += v;
            fq[hf] = fmaf(v, v, fq[hf]);
          }
        }
      }
      fold_stats(fs, fq);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(w * 8 + 4 * hf + r) * 64 + lane] = af[hf][r];
      bar();
      mu_rs();
      bar();
      {
        const int e = tid >> 6, l = lane;
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < kNW; ++ww) v += red[(ww * 8 + e) * 64 + l];
        const int rt = 16 * (e >> 2) + 4 * (l >> 4) + (e & 3);
        v = gelu_tanh_nc(fold_apply(v, rsd[rt], mu[rt], fcu, fcc));
        obf[rt * 16 + (l & 15)] = f2bf(v);
      }
      bar();
      if (MT > 1) {  // as phase A: the store issued by every wave, dropped (offset out of range) but in wave 0
        const int rt = lane >> 1, half = lane & 1;
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(obf + rt * 16 + 8 * half);
        __builtin_amdgcn_raw_buffer_store_b128(
            v, rsrc_lim(p.scratch + kOffFc), w == 0 ? ((c * kMaxR + 32 * t + rt) * 512 + 16 * j + 8 * half) * 2 : kDrop,
            0, PL_AUX);
      } else if (tid < 64) {  // [32 rows][16 columns] bf16 -> the cluster's f tile, write-through 16-B stores
        const int rt = tid >> 1, half = tid & 1;
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(obf + rt * 16 + 8 * half);
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc_f, ((c * kMaxR + 32 * t + rt) * 512 + 16 * j + 8 * half) * 2,
                                               0, PL_AUX);
      }
      if (MT > 1) {
        bar();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) ax[i][hf] = axn[i][hf];
      }
    }
  }
  mark(10);
  drain();
  bar();
  mark(18);
  if (tid == 0) add_relaxed(cnt_(CNT5 + c));

  // ---- (F) mlp.c_proj split c, tile j, per row tile: decode_gemm_kernel EPI 2 (k-steps w + 8i of the split)
  if (tid == 0 && !poll_ge(cnt_(CNT5 + c), kCPC * L1, err, 5)) *abort_flag = 1;
  mark(11);
  bar();
  if (*abort_flag) return;
  {
    auto rsrc = rsrc_of(kOffFc);
    u32x4_t a4[4], a4n[4];  // double-buffered over row tiles, as phase A
    auto load_a4 = [&](u32x4_t (&dst)[4], int t) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dst[i] = __builtin_amdgcn_raw_buffer_load_b128(
            rsrc, ((c * kMaxR + 32 * t + r32) * 512 + 16 * (w + 8 * i) + 8 * hb) * 2, 0, PL_AUX);
    };
    load_a4(a4, 0);
#pragma unroll  // (MT > 1: straight-line tiles, so the compiler's vmcnt counts stay exact across them)
    for (int t = 0; t < MT; ++t) {
      if (MT > 1 && t + 1 < MT) load_a4(a4n, t + 1);
      f32x16_t acc32;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc32[r] = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc32 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            *reinterpret_cast<const bf16x8_t*>(&a4[i]),
            *reinterpret_cast<const bf16x8_t*>(lds_wpj + (w + 8 * i) * 1024 + lane * 16), acc32, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(w * 16 + r) * 64 + lane] = acc32[r];
      bar();
      store_partial(p2, t);
      bar();
      if (MT > 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a4[i] = a4n[i];
      }
    }
  }
  mark(12);
  drain();
  bar();
  mark(19);
  if (tid == 0) add_relaxed(cnt_(CNT6 + j));

  // ---- (G) x2 = x1 + (b_proj + sum_c partial_c) on tile j: wave c (rows 4c .. 4c+3 of every tile) stores x and
  // x^ for the next launch.  The model's last layer stores x1 and leaves this reduce (with ln_f + final_norm, Q5)
  // to itts_residual_reduce_ln over the partials.
  if (p.last) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int row = 32 * t + xrow;
      if ((xrow >> 2) == c && row < R) *reinterpret_cast<float2*>(p.x + (int64_t)row * kD + xcol) = x1[t];
    }
    return;
  }
  if (tid == 0 && !poll_ge(cnt_(CNT6 + j), kNC * L1, err, 6)) *abort_flag = 1;
  mark(13);
  bar();
  if (*abort_flag) return;
  if (w == c) {
    const float2 pb2 = *reinterpret_cast<const float2*>(Ly.proj_b + xcol);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int row = 32 * t + xrow;
      if (row >= R) continue;
      float2 pp = pb2;
#pragma unroll
      for (int cc = 0; cc < kNC; ++cc) {
        const uint64_t v = ld_sc1_u64(reinterpret_cast<const uint64_t*>(p2 + ((int64_t)cc * kMaxR + row) * kD + xcol));
        pp.x += __uint_as_float((uint32_t)v);
        pp.y += __uint_as_float((uint32_t)(v >> 32));
      }
      const float2 x2 = float2{x1[t].x + pp.x, x1[t].y + pp.y};
      *reinterpret_cast<float2*>(p.x + (int64_t)row * kD + xcol) = x2;
      *reinterpret_cast<uint32_t*>(p.xh + (int64_t)row * kD + xcol) = pack2bf(x2.x, x2.y);
    }
  }
  mark(14);
}

// occupancy of the instantiations the default path launches, per row-tile count MT (both the plain and the
// lineage form: a caller of itts_gpt_pl_supported need not say whether the state has beams) and the small-step
// form: each must fit one workgroup per CU (LDS, registers), the grid being one workgroup per CU.  -1: not
// queried yet.
int g_cu_count = -1;
int g_occ[5] = {-1, -1, -1, -1, -1};  // [0]: the small-step form; [MT]: MT row tiles

template <typename K>
int fits(K k) {
  int nb = 0;
  const bool ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(k), kThreads, 0) ==
                  hipSuccess && nb >= 1;
  (void)hipGetLastError();
  return ok ? 1 : 0;
}

int occ_ok(int slot) {
  if (g_occ[slot] < 0) {
    switch (slot) {
      case 0: g_occ[0] = fits(gpt_layer_pl_kernel<1, false, kKBSmall, kSmallH16>); break;
      case 1:
        g_occ[1] = fits(gpt_layer_pl_kernel<1, false>) & fits(gpt_layer_pl_kernel<1, true>) &
                   fits(gpt_layer_pl_kernel<1, true, kKB, false, 3>);
        break;
      case 2:
        g_occ[2] = fits(gpt_layer_pl_kernel<2, false>) & fits(gpt_layer_pl_kernel<2, true>) &
                   fits(gpt_layer_pl_kernel<2, true, kKB, false, 3>);
        break;
      case 3:
        g_occ[3] = fits(gpt_layer_pl_kernel<3, false>) & fits(gpt_layer_pl_kernel<3, true>) &
                   fits(gpt_layer_pl_kernel<3, true, kKB, false, 3>);
        break;
      default: g_occ[4] = fits(gpt_layer_pl_kernel<4, false>) & fits(gpt_layer_pl_kernel<4, true>); break;
    }
  }
  return g_occ[slot];
}

}  // namespace

extern "C" int64_t itts_gpt_pl_scratch_bytes(void) { return kScratchBytes; }

extern "C" int itts_gpt_pl_supported(const ItTsGptWeights* w, int rows) {
  if (!w || w->d_model != kD || w->n_head != kH || rows < 1 || rows > kMaxR) return 0;
  if (g_cu_count < 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 0;
    (void)hipGetLastError();
    g_cu_count = n;
  }
  // every workgroup must be resident at once (one per CU); the caller must also keep other work off the
  // device's CUs while a layer runs: a workgroup that cannot be placed makes the
  // resident ones time out (itts_gpt_pl_error), never hang
  if (g_cu_count < kWG) return 0;
  const int mt = (rows + 31) / 32;
  return occ_ok(mt) && (rows > kSmallRows || occ_ok(0)) ? 1 : 0;
}

extern "C" int itts_gpt_pl_error(const void* scratch, void* stream, int* code) {
  const char* fn = "itts_gpt_pl_error";
  ITTS_REQUIRE(scratch && code, fn, "null pointer");
  hipStream_t s = itts::as_stream(stream);
  uint32_t v = 0;
  if (hipMemcpyAsync(&v, static_cast<const unsigned char*>(scratch) + kOffErr, 4, hipMemcpyDeviceToHost,
                     s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return itts::check_launch(fn);
  *code = (int)v;
  return 0;
}

namespace {
PlLayerPtrs layer_ptrs(const ItTsGptLayerW* ly, const ItTsGptPlLayerW* pl) {
  PlLayerPtrs q;
  q.qkv_w12 = static_cast<const u32x4_t*>(pl->qkv_w12);
  q.qkv_uc = pl->qkv_uc;
  q.o_w = static_cast<const u32x4_t*>(ly->o_w);
  q.o_b = ly->o_c;
  q.fc_w16 = static_cast<const u32x4_t*>(ly->fc_w16);
  q.fc_u = ly->fc_u;
  q.fc_c = ly->fc_c;
  q.proj_w = static_cast<const u32x4_t*>(ly->proj_w);
  q.proj_b = ly->proj_b;
  return q;
}

bool layer_ok(const ItTsGptLayerW* ly, const ItTsGptPlLayerW* pl) {
  return ly && pl && pl->qkv_w12 && pl->qkv_uc && ly->o_w && ly->fc_w16 && ly->fc_u && ly->fc_c && ly->proj_w &&
         ly->proj_b && ly->o_c;
}

// beam states of num_beams = 3 and at most 96 rows run the beam-major attention (ITTS_PL_BEAM_SHARED=0: the
// row passes, bit-identical; A/B)
bool beam_major(const ItTsGptDecodeState* st) {
  static const bool on = [] {
    const char* e = getenv("ITTS_PL_BEAM_SHARED");
    return !(e && e[0] == '0');
  }();
  return on && st->kv_rows && st->num_beams == 3 && st->rows % 3 == 0 && st->rows <= 96;
}

// layer `layer` of decode step kstep as ONE launch
int launch_layer(const ItTsGptLayerW* lyw, const ItTsGptPlLayerW* plw, const ItTsGptDecodeState* st, int layer,
                 int kstep, int last, void* scratch, hipStream_t s, const char* fn) {
  const int64_t cache_hs = (int64_t)st->max_kv * kHD, cache_bs = (int64_t)kH * cache_hs;
  const int64_t layer_cache = (int64_t)st->rows * cache_bs;
  PlArgs a;
  a.ly = layer_ptrs(lyw, plw);
  a.x = st->x;
  a.xh = static_cast<uint16_t*>(st->xh);
  a.kc = static_cast<uint16_t*>(st->k_cache) + layer * layer_cache;
  a.vc = static_cast<uint16_t*>(st->v_cache) + layer * layer_cache;
  a.cache_bs = cache_bs;
  a.cache_hs = cache_hs;
  a.pad = st->pad;
  a.tstate = st->tstate;
  a.kv_rows = st->kv_rows;
  a.ld_rows = st->ld_rows;
  a.kv_base = st->kv_base;
  a.kstep = kstep;
  a.R = st->rows;
  a.layer = layer;
  a.last = last;
  a.eps = 1e-5f;
  a.scratch = static_cast<unsigned char*>(scratch);
  const int mt = (st->rows + 31) / 32;
  const int ki = 2 * (mt - 1) + (st->kv_rows ? 1 : 0);
  if (beam_major(st)) {  // beam3 states of <= 96 rows: one attention pass over each utterance's beams
    switch (mt) {
      case 1: hipLaunchKernelGGL((gpt_layer_pl_kernel<1, true, kKB, false, 3>), dim3(kWG), dim3(kThreads), 0, s, a); break;
      case 2: hipLaunchKernelGGL((gpt_layer_pl_kernel<2, true, kKB, false, 3>), dim3(kWG), dim3(kThreads), 0, s, a); break;
      default: hipLaunchKernelGGL((gpt_layer_pl_kernel<3, true, kKB, false, 3>), dim3(kWG), dim3(kThreads), 0, s, a); break;
    }
    return itts::check_launch(fn);
  }
  if (ki == 0 && st->rows <= kSmallRows) {  // kSmallRows <= 16: one 16-row half
    hipLaunchKernelGGL((gpt_layer_pl_kernel<1, false, kKBSmall, kSmallH16>), dim3(kWG), dim3(kThreads), 0, s, a);
    return itts::check_launch(fn);
  }
  switch (ki) {
    case 0: hipLaunchKernelGGL((gpt_layer_pl_kernel<1, false>), dim3(kWG), dim3(kThreads), 0, s, a); break;
    case 1: hipLaunchKernelGGL((gpt_layer_pl_kernel<1, true>), dim3(kWG), dim3(kThreads), 0, s, a); break;
    case 2: hipLaunchKernelGGL((gpt_layer_pl_kernel<2, false>), dim3(kWG), dim3(kThreads), 0, s, a); break;
    case 3: hipLaunchKernelGGL((gpt_layer_pl_kernel<2, true>), dim3(kWG), dim3(kThreads), 0, s, a); break;
    case 4: hipLaunchKernelGGL((gpt_layer_pl_kernel<3, false>), dim3(kWG), dim3(kThreads), 0, s, a); break;
    case 5: hipLaunchKernelGGL((gpt_layer_pl_kernel<3, true>), dim3(kWG), dim3(kThreads), 0, s, a); break;
    case 6: hipLaunchKernelGGL((gpt_layer_pl_kernel<4, false>), dim3(kWG), dim3(kThreads), 0, s, a); break;
    default: hipLaunchKernelGGL((gpt_layer_pl_kernel<4, true>), dim3(kWG), dim3(kThreads), 0, s, a); break;
  }
  return itts::check_launch(fn);
}

int check_state(const ItTsGptDecodeState* st, void* scratch, const char* fn) {
  ITTS_REQUIRE(st->rows >= 1 && st->rows <= kMaxR, fn, "1..128 rows");
  ITTS_REQUIRE(st->max_kv >= 1, fn, "max_kv >= 1");
  ITTS_REQUIRE(!st->kv_rows || st->ld_rows >= st->max_kv, fn, "kv_rows [rows][ld_rows >= max_kv]");
  ITTS_REQUIRE(!st->kv_rows || st->max_kv <= kKviMax, fn, "beam states: max_kv <= 3584 on the persistent path");
  // the K/V stores of row tiles > 1 are cancellable buffer stores (range kDropLimit, int32 byte offsets): every
  // real offset into one layer's cache, R x 16 heads x max_kv x 64 x 2 B, must lie below kDropLimit (beyond it a
  // real store would be dropped silently)
  ITTS_REQUIRE((int64_t)st->rows * kH * st->max_kv * kHD * 2 < (int64_t)kDropLimit, fn,
               "K/V cache of one layer must be < 2 GiB - 64 KiB (rows x max_kv <= 1,048,543)");
  ITTS_REQUIRE(st->x && st->xh && st->k_cache && st->v_cache && st->tstate, fn, "null state buffer");
  ITTS_REQUIRE((reinterpret_cast<uintptr_t>(scratch) & 255) == 0, fn, "scratch must be 256-B aligned");
  return 0;
}
}  // namespace

extern "C" int itts_gpt_layer_pl(const ItTsGptLayerW* ly, const ItTsGptPlLayerW* pl, const ItTsGptDecodeState* st,
                                 int layer, int kstep, int last, void* scratch, void* stream) {
  const char* fn = "itts_gpt_layer_pl";
  ITTS_REQUIRE(ly && pl && st && scratch, fn, "null pointer");
  ITTS_REQUIRE(layer_ok(ly, pl), fn, "incomplete layer weights");
  if (int rc = check_state(st, scratch, fn)) return rc;
  return launch_layer(ly, pl, st, layer, kstep, last, scratch, itts::as_stream(stream), fn);
}

// Re-arm the scratch: counters, every granule, the epoch and the error word to zero.  An ordinary kernel
// (the stores go through the caches like any kernel's), needed only after an error: a timeout leaves the
// counters short of their epoch.  Never per step (the epochs make stale values harmless).
namespace {
__global__ __launch_bounds__(256) void pl_zero_kernel(u32x4_t* p, int64_t n16, u32x4_t* tail, int64_t t16) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16 + t16; i += (int64_t)gridDim.x * 256) {
    if (i < n16)
      p[i] = u32x4_t{0u, 0u, 0u, 0u};
    else
      tail[i - n16] = u32x4_t{0u, 0u, 0u, 0u};
  }
}
}  // namespace

extern "C" int itts_gpt_pl_reset(void* scratch, void* stream) {
  const char* fn = "itts_gpt_pl_reset";
  ITTS_REQUIRE(scratch, fn, "null scratch");
  ITTS_REQUIRE((reinterpret_cast<uintptr_t>(scratch) & 255) == 0, fn, "scratch must be 256-B aligned");
  unsigned char* s = static_cast<unsigned char*>(scratch);
  const int64_t n16 = kZeroBytes / 16, t16 = (kScratchBytes - kOffSeq) / 16;
  hipLaunchKernelGGL(pl_zero_kernel, dim3(1024), dim3(256), 0, itts::as_stream(stream), reinterpret_cast<u32x4_t*>(s),
                     n16, reinterpret_cast<u32x4_t*>(s + kOffSeq), t16);
  return itts::check_launch(fn);
}

extern "C" int itts_gpt_decode_steps_pl(const ItTsGptWeights* w, const ItTsGptPlLayerW* pl, void* scratch,
                                        const ItTsGptDecodeState* st, const ItTsSampling* smp, int nsteps,
                                        void* stream) {
  const char* fn = "itts_gpt_decode_steps_pl";
  ITTS_REQUIRE(w && pl && scratch && st && smp && w->layers, fn, "null pointer");
  ITTS_REQUIRE(nsteps >= 1 && nsteps <= 64, fn, "nsteps must be in [1, 64]");
  ITTS_REQUIRE(smp->mode >= 0 && smp->mode <= 2, fn, "sampling mode must be 0, 1 or 2");
  ITTS_REQUIRE(nsteps == 1 || smp->mode != 2, fn, "beam decoding (mode 2) runs one step per call");
  ITTS_REQUIRE(itts_gpt_pl_supported(w, st->rows), fn, "shape or device not supported (see itts_gpt_pl_supported)");
  ITTS_REQUIRE(st->logits && w->head_w && (smp->mode == 2 || (st->seen && st->done && st->codes)), fn,
               "sampler state missing");
  const int L = w->n_layer, D = w->d_model, R = st->rows;
  if (int rc = check_state(st, scratch, fn)) return rc;
  for (int l = 0; l < L; ++l) ITTS_REQUIRE(layer_ok(&w->layers[l], &pl[l]), fn, "incomplete layer weights");
  hipStream_t s = itts::as_stream(stream);
  int rc = 0;
  for (int k = 0; k < nsteps && rc == 0; ++k) {
    for (int l = 0; l < L && rc == 0; ++l) rc = launch_layer(&w->layers[l], &pl[l], st, l, k, l + 1 == L, scratch, s, fn);
    // the last layer's mlp.c_proj reduce with ln_f + final_norm (Q5) over the persistent partials
    if (rc == 0)
      rc = itts_residual_reduce_ln(st->x, D, reinterpret_cast<float*>(static_cast<unsigned char*>(scratch) + kOffP2),
                                   kNC, (int64_t)kMaxR * kD, kD, w->layers[L - 1].proj_b, st->xh, D, R, D,
                                   w->ln_f_g, w->ln_f_b, w->final_g, w->final_b, ITTS_BF16, stream);
    if (rc == 0) rc = itts::gpt_head_sample(w, st, smp, k, stream);
  }
  if (rc == 0 && smp->mode != 2) rc = itts_step_advance(st->tstate, nsteps, stream);
  return rc;
}
