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

// Streams created by the HIP runtime this library launches on (SeedGroup wraps
// them as torch external streams): non-blocking, each placed on the process's
// hardware queues by HIP at creation.
int rlmd_stream_create(void** out) {
  RLMD_CHECK(out, "null argument");
  hipStream_t s = nullptr;
  RLMD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *out = s;
  return 0;
}

int rlmd_stream_create_cu(const uint32_t* cu_mask, int32_t n_words, void** out) {
  RLMD_CHECK(out && cu_mask && n_words > 0, "null argument or empty CU mask");
  hipStream_t s = nullptr;
  RLMD_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, cu_mask));
  *out = s;
  return 0;
}

int rlmd_stream_destroy(void* stream) {
  RLMD_CHECK(stream, "null stream");
  RLMD_HIP(hipStreamDestroy((hipStream_t)stream));
  return 0;
}

}  // extern "C"
