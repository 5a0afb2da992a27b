// rm_fastmath.hpp — cheap f32 sequences that are bit-identical to the
// correctly-rounded IEEE operations they replace, over the stated domains.
// Each one is proven exhaustively (every input of its domain) on gfx950 by
// tools/exhaustive_fp.hip; the proof log is committed in profiles/.
#pragma once

#include <hip/hip_runtime.h>

namespace rmd {

// Capsule constants (computeShader.glsl:120): ba = b - a, dot(ba, ba), in float.
constexpr float CAP_AX = -0.1f, CAP_AY = 0.1f, CAP_AZ = -0.1f;
constexpr float CAP_BAX = 2.0f - CAP_AX, CAP_BAY = 4.0f - CAP_AY, CAP_BAZ = 2.0f - CAP_AZ;
constexpr float CAP_BB_HOST = (CAP_BAX * CAP_BAX + CAP_BAY * CAP_BAY) + CAP_BAZ * CAP_BAZ;
constexpr float CAP_BB_RCP = 1.0f / CAP_BB_HOST;  // correctly rounded reciprocal

// Core of the correctly-rounded sqrt without the denormal pre-scale:
// v_sqrt_f32 (within one ulp) and the one-ulp neighbour correction.
// Exhaustively equal to __builtin_sqrtf for x == 0 and x in [2^-96, FLT_MAX];
// callers route x in (0, 2^-96) to sqrt_cr_nonneg.
__device__ __forceinline__ float sqrt_core(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  const int si = __float_as_int(s);
  const float sm = __int_as_float(si - 1);
  const float sp = __int_as_float(si + 1);
  const float rm = __builtin_fmaf(-sm, s, x);
  const float rp = __builtin_fmaf(-sp, s, x);
  s = (rm <= 0.0f) ? sm : s;
  s = (rp > 0.0f) ? sp : s;
  return s;
}

// Smallest input sqrt_core handles exactly (besides 0).
constexpr float SQRT_CORE_MIN = 0x1p-96f;
// Smallest |x| for which div_capbb is exact.
constexpr float DIV_CAPBB_MIN = 0x1p-100f;

// sqrt(x) for x >= 0 (finite), correctly rounded.  v_sqrt_f32 plus the
// one-ulp neighbour correction of the compiler's own lowering, with the
// denormal pre-scale kept (x < 2^-96) but without the inf/nan class fixup
// (not in the domain).  Exhaustively equal to __builtin_sqrtf on [0, FLT_MAX].
__device__ __forceinline__ float sqrt_cr_nonneg(float x) {
  const bool small = x < 0x1p-96f;
  const float xs = small ? x * 0x1p32f : x;
  float s = __builtin_amdgcn_sqrtf(xs);
  const int si = __float_as_int(s);
  const float sm = __int_as_float(si - 1);
  const float sp = __int_as_float(si + 1);
  const float rm = __builtin_fmaf(-sm, s, xs);
  const float rp = __builtin_fmaf(-sp, s, xs);
  s = (rm <= 0.0f) ? sm : s;
  s = (rp > 0.0f) ? sp : s;
  return small ? s * 0x1p-16f : s;
}

// x / CAP_BB correctly rounded, as a multiply by the correctly-rounded
// reciprocal and one fma remainder correction (Markstein).  Domain: all
// finite x; exhaustively equal to the IEEE division on gfx950.
__device__ __forceinline__ float div_capbb(float x) {
  const float q = x * CAP_BB_RCP;
  const float r = __builtin_fmaf(-q, CAP_BB_HOST, x);
  return __builtin_fmaf(r, CAP_BB_RCP, q);
}

}  // namespace rmd
