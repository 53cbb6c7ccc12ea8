// roctx ranges (batch phases visible to `rocprofv3 --marker-trace`), resolved
// lazily with dlopen so the extension has no link-time dependency on the profiler SDK.
#pragma once
#include <dlfcn.h>

#include <cstdlib>

namespace igp {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    const char* env = std::getenv("IGP_ROCTX");  // IGP_ROCTX=0: no ranges, no profiler library load
    if (env && env[0] == '0') return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_LOCAL);
    if (h) {
      push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      if (!push || !pop) push = nullptr;
    }
  }
};
inline const Roctx& roctx() {
  static Roctx r;
  return r;
}
struct Range {
  explicit Range(const char* name) : on(roctx().push != nullptr) {
    if (on) roctx().push(name);
  }
  ~Range() {
    if (on) roctx().pop();
  }
  bool on;
};

}  // namespace igp
