// roctx annotations: rocprofv3 --marker-trace shows these ranges next to the kernel
// trace, so a batch's enqueue -> host-verify latency, the node collectives and share submission
// line up with the gfx950 kernels they surround. Without a profiler attached each call is a
// branch on an unset callback table (librocprofiler-sdk-roctx).
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace otedama {

using TraceId = roctx_range_id_t;

inline void trace_push(const char* name) { roctxRangePushA(name); }
inline void trace_pop() { roctxRangePop(); }
inline void trace_mark(const char* name) { roctxMarkA(name); }
inline TraceId trace_start(const char* name) { return roctxRangeStartA(name); }
inline void trace_stop(TraceId id) { roctxRangeStop(id); }
inline void trace_name_thread(const char* name) { roctxNameOsThread(name); }

// RAII push/pop for host-side scopes.
struct TraceScope {
  explicit TraceScope(const char* name) { trace_push(name); }
  ~TraceScope() { trace_pop(); }
  TraceScope(const TraceScope&) = delete;
  TraceScope& operator=(const TraceScope&) = delete;
};

}  // namespace otedama
