// rm_internal.hpp — declarations shared by librm's translation units.
#pragma once

#include <cstddef>
#include <cstdint>

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
constexpr int TABLE_WORDS = 20;
enum TableWord : int {
  TW_TYPE = 0, TW_SWIZZLE = 1, TW_ID = 2, TW_PAINT = 3, TW_MATERIAL = 4, TW_COLOR = 5,
  TW_CENTER = 8, TW_P = 11,  // 9 parameter words
};
// Validates prims[0..n) and writes n * TABLE_WORDS words to out; returns
// RM_OK or RM_ERR_INVALID with *why set.
int compile_scene(const rm_primitive* prims, int32_t n, uint32_t* out, const char** why);

}  // namespace rm
