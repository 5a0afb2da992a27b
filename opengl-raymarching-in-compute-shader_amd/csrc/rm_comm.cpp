// rm_comm.cpp — run-time binding of RCCL (see rm_comm.hpp).
#include "rm_comm.hpp"

#include <dlfcn.h>

#include <mutex>
#include <type_traits>

namespace rm {

namespace {

Rccl g_rccl;
const Rccl* g_ok = nullptr;
std::string g_err;
std::once_flag g_once;

void load() {
  // librccl.so.1 first: the soname torch's bundled copy and /opt/rocm's share, so
  // an already-loaded RCCL is reused; then /opt/rocm's by path.
  void* h = nullptr;
  for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
    h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
    if (h) break;
  }
  if (!h) {
    const char* e = dlerror();
    g_err = std::string("RCCL not found (librccl.so.1): ") + (e ? e : "");
    return;
  }
  bool ok = true;
  auto sym = [&](const char* name, auto& fn) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
    if (!fn) {
      ok = false;
      g_err += std::string(g_err.empty() ? "RCCL lacks " : ", ") + name;
    }
  };
  sym("ncclGetUniqueId", g_rccl.GetUniqueId);
  sym("ncclCommInitRank", g_rccl.CommInitRank);
  sym("ncclCommInitAll", g_rccl.CommInitAll);
  sym("ncclCommDestroy", g_rccl.CommDestroy);
  sym("ncclGroupStart", g_rccl.GroupStart);
  sym("ncclGroupEnd", g_rccl.GroupEnd);
  sym("ncclGather", g_rccl.Gather);
  sym("ncclGetErrorString", g_rccl.GetErrorString);
  sym("ncclGetVersion", g_rccl.GetVersion);
  if (ok) g_ok = &g_rccl;
}

}  // namespace

const Rccl* rccl(std::string* err) {
  std::call_once(g_once, load);
  if (!g_ok && err) *err = g_err;
  return g_ok;
}

}  // namespace rm
