// C-ABI core: error reporting and library metadata.  See include/autovc_hip.h.
#include "common.h"
#include "../../include/autovc_hip.h"

#include <cstring>

#include <hip/hip_ext.h>

namespace avc {
static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace avc

extern "C" {

const char* autovc_last_error(void) { return avc::g_err; }

int autovc_abi_version(void) { return AUTOVC_HIP_ABI_VERSION; }

int autovc_device_sync(void) {
  AVC_HIP(hipDeviceSynchronize(), "autovc_device_sync");
  return avc::kOk;
}

int autovc_stream_create_cu_mask(int n_words, const uint32_t* mask, hipStream_t* out) {
  AVC_CHECK_ARG(n_words > 0 && mask && out, "autovc_stream_create_cu_mask: bad arguments");
  AVC_HIP(hipExtStreamCreateWithCUMask(out, (uint32_t)n_words, mask), "hipExtStreamCreateWithCUMask");
  return avc::kOk;
}

int autovc_stream_destroy(hipStream_t stream) {
  AVC_HIP(hipStreamDestroy(stream), "hipStreamDestroy");
  return avc::kOk;
}

}  // extern "C"
