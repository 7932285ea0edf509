// abi.hip — error plumbing shared by every C-ABI entry point.
#include <string>

#include "rlmd_common.h"
#include "rlmd_internal.h"

namespace {
thread_local std::string g_last_error;
}

namespace rlmd {
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace rlmd

extern "C" {

const char* rlmd_last_error(void) { return g_last_error.c_str(); }

int rlmd_device_sync(void) {
  RLMD_HIP(hipDeviceSynchronize());
  return 0;
}

}  // extern "C"
