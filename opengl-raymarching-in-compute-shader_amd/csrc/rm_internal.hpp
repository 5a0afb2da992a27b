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

}  // namespace rm
