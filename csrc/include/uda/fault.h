// Fault injection (tests and chaos runs). UDA_FAULT_<SITE>=<n> makes the n-th event at that site
// fail; the count restarts whenever the variable's value changes. Sites:
//   FETCH         a fetch request (transport round) fails          -> consumer failure callback
//   AIO           an AsyncIO read/write completes with -EIO         -> provider/consumer failure
//   DEVICE_ALLOC  a device (HBM) allocation fails                   -> failure callback / error
//   HOST_ALLOC    the consumer's fetch-buffer pool allocation fails -> INIT error (UdaRuntimeException)
// Reference analogue: none (the reference only has the fallback path itself); SURVEY.md §7.4.
#pragma once

namespace uda {
bool fault_hit(const char* site);
}  // namespace uda
