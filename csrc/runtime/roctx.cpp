// roctx ranges emitted from the native library: the trainer's
// phases (forward / backward / comm wait / optimizer) and the engine's
// prefill / decode steps appear as named ranges in `rocprofv3 --marker-trace`.
//
// rocprofiler-sdk's roctx is loaded lazily with dlopen, so the extension
// imports (and the ops are no-ops) on a machine without it.
#include <torch/library.h>

#include <dlfcn.h>

#include <mutex>
#include <string>

namespace {

using push_fn = int (*)(const char*);
using pop_fn = int (*)();
using mark_fn = void (*)(const char*);

struct Roctx {
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  mark_fn mark = nullptr;
};

const Roctx& roctx() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                           "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"};
    for (const char* n : names) {
      void* h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      r.push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
      r.pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
      r.mark = reinterpret_cast<mark_fn>(dlsym(h, "roctxMarkA"));
      if (r.push && r.pop) break;
      r = Roctx{};
    }
  });
  return r;
}

int64_t range_push(std::string name) {
  const Roctx& r = roctx();
  return r.push ? r.push(name.c_str()) : -1;
}

int64_t range_pop() {
  const Roctx& r = roctx();
  return r.pop ? r.pop() : -1;
}

void mark(std::string name) {
  const Roctx& r = roctx();
  if (r.mark) r.mark(name.c_str());
}

bool roctx_available() { return roctx().push != nullptr; }

}  // namespace

TORCH_LIBRARY_FRAGMENT(mxllm, m) {
  m.def("roctx_push(str name) -> int", &range_push);
  m.def("roctx_pop() -> int", &range_pop);
  m.def("roctx_mark(str name) -> ()", &mark);
  m.def("roctx_available() -> bool", &roctx_available);
}
