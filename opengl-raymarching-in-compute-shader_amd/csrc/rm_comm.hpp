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
  decltype(&ncclCommInitAll) CommInitAll;
  decltype(&ncclCommDestroy) CommDestroy;
  decltype(&ncclGroupStart) GroupStart;
  decltype(&ncclGroupEnd) GroupEnd;
  decltype(&ncclGather) Gather;
  decltype(&ncclGetErrorString) GetErrorString;
  decltype(&ncclGetVersion) GetVersion;
};

// The loaded entry points, or nullptr with *err set (no RCCL on this host, or one
// without ncclGather).  Thread-safe; loads once per process.
const Rccl* rccl(std::string* err);

}  // namespace rm
