// rm_comm.cpp — run-time binding of RCCL (see rm_comm.hpp).
#include "rm_comm.hpp"

#include <dlfcn.h>

#include <chrono>
#include <mutex>
#include <thread>
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
  sym("ncclCommInitRankConfig", g_rccl.CommInitRankConfig);
  sym("ncclCommFinalize", g_rccl.CommFinalize);
  sym("ncclCommDestroy", g_rccl.CommDestroy);
  sym("ncclCommAbort", g_rccl.CommAbort);
  sym("ncclCommGetAsyncError", g_rccl.CommGetAsyncError);
  sym("ncclGroupStart", g_rccl.GroupStart);
  sym("ncclGroupEnd", g_rccl.GroupEnd);
  sym("ncclGather", g_rccl.Gather);
  sym("ncclAllGather", g_rccl.AllGather);
  sym("ncclGetErrorString", g_rccl.GetErrorString);
  sym("ncclGetVersion", g_rccl.GetVersion);
  sym("ncclCommCount", g_rccl.CommCount);
  sym("ncclCommUserRank", g_rccl.CommUserRank);
  sym("ncclCommCuDevice", g_rccl.CommCuDevice);
  if (ok) g_ok = &g_rccl;
}

}  // namespace

const Rccl* rccl(std::string* err) {
  std::call_once(g_once, load);
  if (!g_ok && err) *err = g_err;
  return g_ok;
}

ncclConfig_t nonblocking_config() {
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  return cfg;
}

void poll_pause(int spins) {
  // Yield (a few us per poll) for the first ~10-40 ms: a frame or a bench's timed
  // steps at N = 8 end within that, and a sleeping poll would add up to its
  // period to the measured time.  Then back off: 100 us, and 1 ms past ~1 s.
  if (spins < 20000) std::this_thread::yield();
  else std::this_thread::sleep_for(std::chrono::microseconds(spins < 30000 ? 100 : 1000));
}

ncclResult_t wait_ready(const Rccl* r, const ncclComm_t* comms, int n, long timeout_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int spins = 0;; ++spins) {
    bool pending = false;
    for (int i = 0; i < n; ++i) {
      if (!comms[i]) continue;
      ncclResult_t st = ncclSuccess;
      const ncclResult_t e = r->CommGetAsyncError(comms[i], &st);
      if (e != ncclSuccess) return e;
      if (st == ncclInProgress) pending = true;
      else if (st != ncclSuccess) return st;
    }
    if (!pending) return ncclSuccess;
    if (timeout_ms > 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
      return ncclInProgress;
    poll_pause(spins);
  }
}

void teardown(const Rccl* r, ncclComm_t* comms, int n, long timeout_ms) {
  bool ok = true;
  for (int i = 0; i < n; ++i) {
    if (!comms[i]) continue;
    const ncclResult_t e = r->CommFinalize(comms[i]);
    ok = ok && (e == ncclSuccess || e == ncclInProgress);
  }
  if (ok) ok = wait_ready(r, comms, n, timeout_ms) == ncclSuccess;
  for (int i = 0; i < n; ++i) {
    if (!comms[i]) continue;
    if (ok) (void)r->CommDestroy(comms[i]);
    else (void)r->CommAbort(comms[i]);
    comms[i] = nullptr;
  }
}

}  // namespace rm
