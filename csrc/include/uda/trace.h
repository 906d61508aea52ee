// Timeline annotations: roctx ranges visible in `rocprofv3 --marker-trace` next to the kernel and
// copy traces (reference: TRACE-level logs only, SURVEY.md §5 "Tracing / profiling").
//
// The roctx library is loaded on demand (UDA_ROCTX=1), not linked: a process that links it and
// runs under rocprofv3 crashes in its exit-time destructors, so annotations are opt-in.
#pragma once

#include <cstdint>

namespace uda {
namespace trace {

void push(const char* name);
void pop();
void mark(const char* what);

// Thread-scoped range (push/pop); a no-op unless UDA_ROCTX=1 loaded roctx.
class Range {
 public:
  explicit Range(const char* name) { push(name); }
  ~Range() { pop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

// Host event recorder (UDA_HOST_TRACE=<path>): timed intervals from any thread, kept in memory and
// written as CSV (kind,tid,a,b,t0_ns,t1_ns; steady clock) by dump() or at process exit. Off: one
// relaxed load per call. Used to take apart host-side pipelines (fetch / staging / delivery).
bool host_enabled();
int64_t now_ns();
void host_event(const char* kind, int64_t a, int64_t b, int64_t t0_ns, int64_t t1_ns);
void host_dump();

}  // namespace trace
}  // namespace uda
