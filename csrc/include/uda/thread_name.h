// Names the calling thread (shown in /proc/<pid>/task/<tid>/comm, by top -H, gdb and the stall probe).
#pragma once
#include <pthread.h>

namespace uda {

inline void name_thread(const char* name) { (void)pthread_setname_np(pthread_self(), name); }  // <= 15 chars

}  // namespace uda
