// roctx ranges around the job's phases and the engine's pipeline stages — the reference
// has no tracing at all (no NVTX, no timers, main.c / cudaFunctions.cu). The ranges cost one call into
// librocprofiler-sdk-roctx (a no-op unless a profiler is attached) and show up in
//   rocprofv3 --marker-trace --kernel-trace -- ./final ...
// next to the kernels. The roctx library is loaded on first use when a rocprofiler tool is present
// (MOC_TRACE=1 forces it, MOC_TRACE=0 turns the ranges off entirely).
#pragma once

namespace moc {

bool trace_enabled();
void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);
void trace_name_thread(const char* name);

// RAII range.
class TraceRange {
 public:
  explicit TraceRange(const char* name) { trace_push(name); }
  ~TraceRange() { trace_pop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace moc
