// Name the calling thread (visible in /proc/<pid>/task/*/comm, top -H, rocprofv3 traces): the
// per-thread CPU attribution of the serving path (tools/host_profile.py) groups threads by it.
#pragma once
#include <pthread.h>

#include <string>

namespace igp {

inline void name_thread(const std::string& name) {
  // the kernel keeps 15 characters
  pthread_setname_np(pthread_self(), name.substr(0, 15).c_str());
}

}  // namespace igp
