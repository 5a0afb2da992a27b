// rm_comm.hpp — RCCL entry points librm uses for multi-GPU frames.
//
// librm does not link RCCL: the first multi-GPU call dlopen()s librccl.so.1.  In
// a process that already holds an RCCL of that soname (PyTorch-ROCm bundles one)
// the loader returns that same copy, so librm and torch share one RCCL; a plain
// C++ host (rm_frameloop --gpus N) gets /opt/rocm's.  Single-GPU users never
// load it.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>

namespace rm {

struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId;
  decltype(&ncclCommInitRank) CommInitRank;
  decltype(&ncclCommInitRankConfig) CommInitRankConfig;
  decltype(&ncclCommFinalize) CommFinalize;
  decltype(&ncclCommDestroy) CommDestroy;
  decltype(&ncclCommAbort) CommAbort;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError;
  decltype(&ncclGroupStart) GroupStart;
  decltype(&ncclGroupEnd) GroupEnd;
  decltype(&ncclGather) Gather;
  decltype(&ncclAllGather) AllGather;  // rm_comm_init's check that every rank cuts the frame alike
  decltype(&ncclGetErrorString) GetErrorString;
  decltype(&ncclGetVersion) GetVersion;
  // what the communicator itself reports (rm_comm_rccl_info): the rank count and
  // this member's rank as RCCL formed them, and the device it is bound to
  decltype(&ncclCommCount) CommCount;
  decltype(&ncclCommUserRank) CommUserRank;
  decltype(&ncclCommCuDevice) CommCuDevice;
};

// The loaded entry points, or nullptr with *err set (no RCCL on this host, or one
// without ncclGather).  Thread-safe; loads once per process.
const Rccl* rccl(std::string* err);

// Every communicator librm creates is non-blocking (ncclConfig_t.blocking = 0):
// init and enqueue calls may return ncclInProgress, and their progress is polled
// with ncclCommGetAsyncError against a deadline, so a peer that never joins or a
// collective that never completes becomes an error (RM_ERR_COMM) instead of a
// host thread blocked forever.  SURVEY 5 "Failure detection".
ncclConfig_t nonblocking_config();

// Polls ncclCommGetAsyncError on comms[0..n) until none is ncclInProgress.
// Returns ncclSuccess, the first error, or ncclInProgress when timeout_ms (> 0)
// passed first (timeout_ms <= 0: no deadline).
ncclResult_t wait_ready(const Rccl* r, const ncclComm_t* comms, int n, long timeout_ms);

// Back-off for host polling loops: yields for the first ~10-40 ms (no added
// latency at the end of a short wait), then sleeps 100 us, then 1 ms.
void poll_pause(int spins);

// Tears down comms[0..n) of one process (the devices of a multi-GPU context, or
// one rank): ncclCommFinalize on all of them first (a single-process
// communicator is quiescent only once every device has finalized), then waits
// for them within timeout_ms and destroys them, or aborts them all when the
// wait fails (a dead peer cannot hang the teardown).
void teardown(const Rccl* r, ncclComm_t* comms, int n, long timeout_ms);

}  // namespace rm
