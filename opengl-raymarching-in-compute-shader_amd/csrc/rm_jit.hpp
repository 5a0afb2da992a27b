// rm_jit.hpp — hiprtc specialisation of the scene-table kernels (rm_jit.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "rm_internal.hpp"

namespace rmd {
struct Frame;
struct FrameBatch;
}

namespace rm {

// The table kernels compiled for one table: the counting builds
// k_table_{pixel,sample}<true> (fnc[aa]) and the production batch kernels
// k_table_{pixel,sample}_frames (fnb[aa]), which also render single frames (a
// batch of one, rm_jit.hip kNames).  waves == 0 (mod null): the table fits no
// spill-free register bound and renders with the generic table kernel.
struct JitTable {
  hipModule_t mod = nullptr;
  hipFunction_t fnc[2] = {nullptr, nullptr};
  hipFunction_t fnb[2] = {nullptr, nullptr};
  int waves = 0;  // the register bound compiled for (waves per SIMD, rm_jit.hip)
};

// Compiles (or finds in the process-wide cache) the table kernels for the
// compiled table words[0..scene_words(n)) on the current device.  RM_OK, or an
// RM_ERR_* code with err set (the hiprtc log on a compile error).
int jit_table(const uint32_t* words, int32_t n, const JitTable** out, std::string& err);
// The same grid and block as launch_table (rm_table.hip); no dynamic LDS.  A
// production frame launches the batch kernel with one frame (its argument is a
// FrameBatch: a graph that captures it takes a FrameBatch node argument).
hipError_t launch_table_jit(const JitTable* j, const rmd::Frame& F, bool counters, hipStream_t s);
// n frames of one batch (rm_dispatch_frames): grid.z = the frame.
hipError_t launch_table_jit_frames(const JitTable* j, const rmd::FrameBatch& B, int n, hipStream_t s);

}  // namespace rm
