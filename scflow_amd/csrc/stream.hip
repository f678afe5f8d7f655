// Cross-stream ordering for the decoder's two HIP streams (a12's side branches).
//
// hipEventRecord's default release is system-scope: every fork/join writes back and invalidates
// the GPU caches (≈ 6 µs of queue time per event on MI355X, visible as gaps between the
// decoder's kernels).  The two streams are on one device in one process, so a device-scope
// release suffices: these events are created with hipEventDisableSystemFence (and without
// timing).
#include "common.h"

SCFLOW_API int scflow_sync_event_create(void** event) {
  if (!event) return SCFLOW_EINVAL;
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence);
  if (r != hipSuccess) return (int)r;
  *event = (void*)e;
  return SCFLOW_OK;
}

SCFLOW_API int scflow_sync_event_destroy(void* event) {
  if (!event) return SCFLOW_EINVAL;
  return (int)hipEventDestroy((hipEvent_t)event);
}

SCFLOW_API int scflow_sync_event_record(void* event, void* stream) {
  if (!event) return SCFLOW_EINVAL;
  return (int)hipEventRecord((hipEvent_t)event, (hipStream_t)stream);
}

SCFLOW_API int scflow_stream_wait_event(void* stream, void* event) {
  if (!event) return SCFLOW_EINVAL;
  return (int)hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0);
}

// Timing events for the bench's live kernel timing: timing enabled, device-scope release, so
// an event pair brackets the kernel without a system-scope cache writeback inside the bracket.
SCFLOW_API int scflow_timing_event_create(void** event) {
  if (!event) return SCFLOW_EINVAL;
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  if (r != hipSuccess) return (int)r;
  *event = (void*)e;
  return SCFLOW_OK;
}

SCFLOW_API int scflow_event_elapsed_ms(void* start, void* end, float* ms) {
  if (!start || !end || !ms) return SCFLOW_EINVAL;
  const hipError_t r = hipEventSynchronize((hipEvent_t)end);
  if (r != hipSuccess) return (int)r;
  return (int)hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end);
}


// ABI markers (scflow_hip.h): the version of the exported interface and sizeof(scflow_conv_args),
// so a binding built against another header revision can refuse to run instead of passing a
// struct of the wrong size
SCFLOW_API int scflow_abi_version(void) { return SCFLOW_ABI_VERSION; }
SCFLOW_API long long scflow_conv_args_size(void) { return (long long)sizeof(scflow_conv_args); }

// launch-time A/B switches (EnvSwitch, common.h): re-read the environment at their next use
std::atomic<int> g_switch_gen{0};
SCFLOW_API int scflow_debug_reload_switches(void) {
  g_switch_gen.fetch_add(1, std::memory_order_relaxed);
  return SCFLOW_OK;
}
