// Timeline annotations: roctx ranges visible in `rocprofv3 --marker-trace` next to the kernel and
// copy traces (reference: TRACE-level logs only, SURVEY.md §5 "Tracing / profiling").
//
// The roctx library is loaded on demand (UDA_ROCTX=1), not linked: a process that links it and
// runs under rocprofv3 crashes in its exit-time destructors, so annotations are opt-in.
#pragma once

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

}  // namespace trace
}  // namespace uda
