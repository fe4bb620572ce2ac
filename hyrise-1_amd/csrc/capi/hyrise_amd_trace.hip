// Timing events for the operators' OperatorPerformanceData (include/hyrise_amd_trace.h).
#include <hip/hip_runtime.h>

#include "hyrise_amd_trace.h"
#include "capi_common.hpp"

using namespace hyc;

extern "C" {

hy_status hy_event_create(hy_event_t* event) {
  if (!event) return fail(HY_ERR_INVALID_ARGUMENT, "event is NULL");
  hipEvent_t e = nullptr;
  HY_HIP(hipEventCreate(&e));
  *event = reinterpret_cast<hy_event_t>(e);
  return HY_OK;
}

hy_status hy_event_record(hy_event_t event, hy_stream_t stream) {
  if (!event) return fail(HY_ERR_INVALID_ARGUMENT, "event is NULL");
  HY_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(event), S(stream)));
  return HY_OK;
}

hy_status hy_event_elapsed_ns(hy_event_t start, hy_event_t stop, uint64_t* ns) {
  if (!start || !stop || !ns) return fail(HY_ERR_INVALID_ARGUMENT, "NULL argument");
  HY_HIP(hipEventSynchronize(reinterpret_cast<hipEvent_t>(stop)));
  float ms = 0;
  HY_HIP(hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)));
  *ns = ms > 0 ? static_cast<uint64_t>(static_cast<double>(ms) * 1e6) : 0;
  return HY_OK;
}

hy_status hy_event_destroy(hy_event_t event) {
  if (event) HY_HIP(hipEventDestroy(reinterpret_cast<hipEvent_t>(event)));
  return HY_OK;
}

}  // extern "C"
