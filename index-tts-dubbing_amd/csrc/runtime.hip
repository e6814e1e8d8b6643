// C-ABI runtime plumbing for libitts_hip: thread-local error strings, launch checks, version.
#include <cstdio>

#include "common.h"

namespace itts {
static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(const char* fn, const char* what) {
  set_error(std::string(fn) + ": " + what);
  return -1;
}

int check_launch(const char* fn) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(fn) + ": " + hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}
}  // namespace itts

extern "C" const char* itts_last_error(void) { return itts::g_last_error.c_str(); }

extern "C" int itts_abi_version(void) { return 5; }  // 3: persistent decode layer, attn.c_proj split-K;
                                                     // 4: epoch-tagged hand-offs (itts_gpt_pl_reset), host packers;
                                                     // 5: ItTsGptDecodeState.num_beams, itts_act_conv_post_tanh

// Which gfx target this code object was built for (sanity check from the host).
extern "C" const char* itts_build_target(void) { return "gfx950"; }

// sizeof of the ABI structs (include/itts_hip.h), so bindings can check their layouts:
// 0 ItTsGptLayerW, 1 ItTsGptWeights, 2 ItTsGptDecodeState, 3 ItTsSampling, 4-8 the vocoder structs
extern "C" int64_t itts_struct_size(int which) {
  switch (which) {
    case 0: return sizeof(ItTsGptLayerW);
    case 1: return sizeof(ItTsGptWeights);
    case 2: return sizeof(ItTsGptDecodeState);
    case 3: return sizeof(ItTsSampling);
    case 4: return sizeof(ItTsConv);
    case 5: return sizeof(ItTsAct);
    case 6: return sizeof(ItTsAmpLayer);
    case 7: return sizeof(ItTsBigvganStage);
    case 8: return sizeof(ItTsBigvganWeights);
    case 9: return sizeof(ItTsGptSeqLayerW);
    case 10: return sizeof(ItTsGptSeqWeights);
    case 11: return sizeof(ItTsGptPlLayerW);
    default: return -1;
  }
}

// Diagnostics (tests): n_wg workgroups of 64 threads, each holding 120 KiB of LDS (so no other workgroup
// needing more than 40 KiB shares its CU), that sleep for `usec` microseconds of the 100-MHz real-time
// counter and exit.  Holds CUs away from a persistent grid launched beside it on another stream
// (tests/test_gpu_pl.py: the hand-off timeout and the launch-chain fallback).  Bounded: every wave exits.
namespace {
__global__ __launch_bounds__(64) void diag_occupy_kernel(uint64_t ticks, int* sink) {
  __shared__ int hold[120 * 1024 / 4];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  hold[threadIdx.x] = (int)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
  __syncthreads();
  if (sink && threadIdx.x == 0) sink[blockIdx.x] = hold[63];
}
}  // namespace

extern "C" int itts_diag_occupy(int n_wg, int usec, int* sink, void* stream) {
  const char* fn = "itts_diag_occupy";
  ITTS_REQUIRE(n_wg >= 1 && n_wg <= 4096 && usec >= 0 && usec <= 10000000, fn, "n_wg 1..4096, usec 0..1e7");
  hipLaunchKernelGGL(diag_occupy_kernel, dim3(n_wg), dim3(64), 0, itts::as_stream(stream), (uint64_t)usec * 100u,
                     sink);
  return itts::check_launch(fn);
}
