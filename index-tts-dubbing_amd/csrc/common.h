// Shared device/host helpers for libitts_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "itts_hip.h"  // the public C ABI: definitions below must match these declarations

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2_t;

enum ItTsDtype { ITTS_F32 = 0, ITTS_BF16 = 1, ITTS_F16 = 2 };

// ---- bf16 <-> f32 (bf16 carried as raw uint16_t) ----
__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  // hardware round-to-nearest-even (v_cvt_pk_bf16_f32 on gfx950: one instruction instead of four
  // integer ops; bit-identical to the integer RNE for every finite value)
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
__device__ __forceinline__ uint32_t pack2bf(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

// Storage-type traits: every kernel computes in f32 and loads/stores T.  ITTS_NT_STORE=1 (A/B build):
// non-temporal stores everywhere St<> is used and at the decode kernels' explicit stores.
#ifndef ITTS_NT_STORE
#define ITTS_NT_STORE 0
#endif
template <typename T>
__device__ __forceinline__ void st_out(T* p, T v) {
#if ITTS_NT_STORE
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
template <typename T> struct St;
template <> struct St<float> {
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static void st(float* p, float v) { st_out(p, v); }
};
template <> struct St<uint16_t> {
  __device__ __forceinline__ static float ld(const uint16_t* p) { return bf2f(*p); }
  __device__ __forceinline__ static void st(uint16_t* p, float v) { st_out(p, f2bf(v)); }
};
// IEEE half (the reference activation op also dispatches Half: type_shim.h:20-43); round to nearest even
template <> struct St<_Float16> {
  __device__ __forceinline__ static float ld(const _Float16* p) { return (float)*p; }
  __device__ __forceinline__ static void st(_Float16* p, float v) { *p = (_Float16)v; }
};

// Loads of data a kernel reads once (activation windows, residual rows, split-K partials): non-temporal
// when ITTS_STREAM_NT (A/B builds; the K/V cache loads are non-temporal unconditionally, gpt_attn.hip)
#ifndef ITTS_STREAM_NT
#define ITTS_STREAM_NT 0
#endif
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
#if ITTS_STREAM_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over each aligned group of 8 lanes, every lane of the group receiving the same value: DPP
// quad_perm xor-1 and xor-2 (within 4 lanes) then row_half_mirror (lane i <-> 7 - i of each 8),
// all VALU data-path operands -- no LDS round trip as ds_swizzle / ds_bpermute would take
// (attention at S = 283: 13.6 -> 12.7 us).  Each step adds the same two values in every lane
// (a + b == b + a), so the 8 lanes agree bitwise.
template <int CTRL>
__device__ __forceinline__ float mov_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum8_dpp(float v) {
  v += mov_dpp<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
  v += mov_dpp<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
  v += mov_dpp<0x141>(v);  // row_half_mirror: lanes 0-3 <-> 7-4
  return v;
}

// ---- the folded-LayerNorm GEMM epilogue (itts_decode_gemm16x and the persistent layer, gpt_layer.hip):
// one fixed rounding sequence with FMA contraction off, so the two kernels agree bit for bit whatever
// the compiler would fuse in each context (round 4: a contracted rs * t + c in one of them and not in
// the other left q/k/v 1 ulp apart) ----
__device__ __forceinline__ void fold_mu_rs(float S, float Q, float inv, float eps, float& mu, float& rs) {
#pragma clang fp contract(off)
  const float m = S * inv;
  mu = m;
  rs = rsqrtf(fmaxf(Q * inv - m * m, 0.f) + eps);
}
__device__ __forceinline__ float fold_apply(float acc, float rs, float mu, float u, float c) {
#pragma clang fp contract(off)
  return rs * (acc - mu * u) + c;
}
__device__ __forceinline__ float gelu_tanh_nc(float x) {
#pragma clang fp contract(off)
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
}

// ---- host-side error plumbing (no C++ exception crosses the C ABI) ----
namespace itts {
void set_error(const std::string& msg);
int fail(const char* fn, const char* what);
int check_launch(const char* fn);
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
// mel_head + token selection + next embedding of decode step k (gpt_step.hip)
int gpt_head_sample(const ItTsGptWeights* w, const ItTsGptDecodeState* st, const ItTsSampling* smp, int k,
                    void* stream);
}  // namespace itts

#define ITTS_REQUIRE(cond, fn, what) \
  do {                               \
    if (!(cond)) return itts::fail(fn, what); \
  } while (0)
