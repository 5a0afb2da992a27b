// rm_internal.hpp — declarations shared by librm's translation units.
#pragma once

#ifndef __HIPCC_RTC__
#include <cstddef>
#include <cstdint>
#else  // hiprtc (rm_jit.hip): the fixed-width types live in __hip_internal
typedef __hip_internal::int8_t int8_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
#endif

#include "../../include/rm_api.h"

namespace rm {

// By-name uniform lookup (shader.hpp:19-69 + glGetUniformLocation semantics).
// Returns nullptr for names that are not in the uniform block.
float* uniform_floats(rm_uniforms* u, const char* name, int* n);
int32_t* uniform_ints(rm_uniforms* u, const char* name);

// Runtime scene table, device layout (rm_table.hip): TABLE_WORDS 32-bit words
// per primitive.  Words 0-3 are ints (type, swizzle, id, paint), the rest
// floats: material, colour[3], centre[3], then the per-type parameters with
// the uniform-only subexpressions folded in on the host (capsule ba = b - a,
// dot(ba, ba): the same float operations the GLSL performs per call).
constexpr int TABLE_WORDS = 24;
enum TableWord : int {
  TW_TYPE = 0, TW_SWIZZLE = 1, TW_ID = 2, TW_PAINT = 3, TW_MATERIAL = 4, TW_COLOR = 5,
  TW_CENTER = 8, TW_P = 11,  // 9 parameter words
  TW_BALL = 20,              // culling ball: world centre (3), radius (+inf: never culled)
};
// After the n entries: EXIT_WORDS words of per-table bounds for the provable
// early exits of the table kernels (rm_table.hip): every non-plane entry lies in
// the ball (EX_C, EX_R); planes are linear along a ray; EX_SIGMA, EX_S scale the
// float-error slack; every non-plane entry also lies in the box EX_BOX (round
// 5: the slab exits of table_exit_T).  EX_VALID = 0 disables the exits
// (unbounded or degenerate entries, more than EX_MAX_PLANES planes).
// The same header lists the entries the march tracks lazily (EX_SLOTS, at most
// EX_MAX_SLOTS bounded entries, in table order), the bitmask of the entries
// evaluated at every step (EX_EVAL_MASK, bit k = entry k: planes and untracked
// entries), and EX_LIP >= 1, a Lipschitz constant of the scene minimum (the
// largest plane |n|; every other entry is 1-Lipschitz).
constexpr int EX_MAX_PLANES = 4;
constexpr int EX_MAX_SLOTS = 8;
// The generic table kernel also comes in an instance holding this many slots,
// taken for tables that track no more (rm_table.hip launch_table).
constexpr int TABLE_FEW_SLOTS = 5;
enum ExitWord : int {
  EX_VALID = 0, EX_CX = 1, EX_CY = 2, EX_CZ = 3, EX_R = 4, EX_SIGMA = 5, EX_S = 6,
  EX_NPLANES = 7, EX_PLANES = 8,  // per plane: world normal n' (3), offset: value ~ dot(p, n') + off
  EX_LIP = EX_PLANES + 4 * EX_MAX_PLANES, EX_NSLOTS, EX_EVAL_MASK, EX_PLANE_MASK, EX_SLOTS,
  EX_BOX = EX_SLOTS + EX_MAX_SLOTS,  // the bounded entries' box: lo (3), hi (3), rounded outward
  EX_END = EX_BOX + 6,
};
constexpr int EXIT_WORDS = EX_END;
// Step 0 of a table's primary rays, formed on the host per frame (rm_api.hip
// table_prep_host) and passed in Frame::prepv when a table renders: every
// primary ray starts at the camera, so step 0 is one uniform evaluation.
enum TablePrep : int {
  TP_VALID = 0,  // 1 when 0 < d0 <= 400
  TP_D0 = 1,     // sdf(camera) (opU over the table, the device's float operations)
  TP_G = 2,      // per lazy slot j (EX_SLOTS): the step-0 re-test's gap (lb - U) - sl
};
// Words for n entries plus the exit header.
constexpr size_t scene_words(int n) { return (size_t)n * TABLE_WORDS + EXIT_WORDS; }
// Validates prims[0..n) and writes scene_words(n) words to out; returns
// RM_OK or RM_ERR_INVALID with *why set.
int compile_scene(const rm_primitive* prims, int32_t n, uint32_t* out, const char** why);

}  // namespace rm
