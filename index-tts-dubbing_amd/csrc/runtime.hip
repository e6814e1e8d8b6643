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

extern "C" int itts_abi_version(void) { return 3; }  // 3: persistent decode layer, attn.c_proj split-K

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
