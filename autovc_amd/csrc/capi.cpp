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

// ---- gradient-ready marks (autovc_amd.functional / ddp): events that eager work outside a
// captured step graph (the data-parallel collectives) can wait on
int autovc_event_create(hipEvent_t* out) {
  AVC_CHECK_ARG(out != nullptr, "autovc_event_create: null out");
  AVC_HIP(hipEventCreateWithFlags(out, hipEventDisableTiming), "hipEventCreateWithFlags");
  return avc::kOk;
}

int autovc_event_destroy(hipEvent_t ev) {
  AVC_HIP(hipEventDestroy(ev), "hipEventDestroy");
  return avc::kOk;
}

// Record `ev` on `stream`.  While the stream is being captured into a graph, an event-record
// node is added after the stream's current capture dependencies and becomes the stream's only
// dependency (hipEventRecord itself is refused inside a capture for an event meant to be
// waited on outside the graph): every replay of the graph records `ev` at that point.
int autovc_event_record_any(hipEvent_t ev, hipStream_t stream) {
  AVC_CHECK_ARG(ev != nullptr, "autovc_event_record_any: null event");
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  unsigned long long id = 0;
  AVC_HIP(hipStreamGetCaptureInfo_v2(stream, &st, &id, &graph, &deps, &ndeps), "hipStreamGetCaptureInfo_v2");
  if (st == hipStreamCaptureStatusNone) {
    AVC_HIP(hipEventRecord(ev, stream), "hipEventRecord");
    return avc::kOk;
  }
  AVC_CHECK_ARG(st == hipStreamCaptureStatusActive && graph != nullptr,
                "autovc_event_record_any: stream capture is invalidated");
  hipGraphNode_t node = nullptr;
  AVC_HIP(hipGraphAddEventRecordNode(&node, graph, deps, ndeps, ev), "hipGraphAddEventRecordNode");
  AVC_HIP(hipStreamUpdateCaptureDependencies(stream, &node, 1, hipStreamSetCaptureDependencies),
          "hipStreamUpdateCaptureDependencies");
  return avc::kOk;
}

int autovc_stream_wait_event(hipStream_t stream, hipEvent_t ev) {
  AVC_CHECK_ARG(ev != nullptr, "autovc_stream_wait_event: null event");
  AVC_HIP(hipStreamWaitEvent(stream, ev, 0), "hipStreamWaitEvent");
  return avc::kOk;
}

}  // extern "C"

// ---- measurement: a one-thread kernel that stores the chip's 100 MHz clock when the stream
// reaches it.  Unlike an event it is an ordinary kernel node inside a captured graph, so an
// unprofiled replay can be time-stamped on several streams at once (tools/side_timeline.py).
namespace {
__global__ void stamp_kernel(unsigned long long* dst) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) dst[0] = t;
}
}  // namespace

extern "C" int autovc_stamp(uint64_t* dst, hipStream_t stream) {
  AVC_CHECK_ARG(dst != nullptr, "autovc_stamp: null destination");
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, stream, reinterpret_cast<unsigned long long*>(dst));
  AVC_CHECK_LAUNCH("autovc_stamp");
  return avc::kOk;
}
