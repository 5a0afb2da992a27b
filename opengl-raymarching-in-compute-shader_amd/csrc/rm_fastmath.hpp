// rm_fastmath.hpp — cheap f32 sequences that are bit-identical to the
// correctly-rounded IEEE operations they replace, over the stated domains.
// Each one is proven exhaustively (every input of its domain) on gfx950 by
// tools/exhaustive_fp.hip; the proof log is committed in profiles/.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

namespace rmd {

// Capsule constants (computeShader.glsl:120): ba = b - a, dot(ba, ba), in float.
constexpr float CAP_AX = -0.1f, CAP_AY = 0.1f, CAP_AZ = -0.1f;
constexpr float CAP_BAX = 2.0f - CAP_AX, CAP_BAY = 4.0f - CAP_AY, CAP_BAZ = 2.0f - CAP_AZ;
constexpr float CAP_BB_HOST = (CAP_BAX * CAP_BAX + CAP_BAY * CAP_BAY) + CAP_BAZ * CAP_BAZ;
constexpr float CAP_BB_RCP = 1.0f / CAP_BB_HOST;  // correctly rounded reciprocal

// Correctly-rounded sqrt on {0} U [2^-96, FLT_MAX] in six instructions:
// v_rsq_f32 and one Newton step (s = x y, r = x - s^2, s + (y/2) r), the way
// the reciprocal-sqrt-based lowerings do it, proven bit-exact on every input of
// that domain by tools/exhaustive_fp.hip.  The 2^-126 added before the rsq
// vanishes in RN for x >= 2^-96 (ulp(x) >= 2^-119) and keeps x = 0 finite:
// y = 2^63, s = 0, result exactly 0.  On (0, 2^-96) the result stays in
// [0, 2^-47) (also checked exhaustively), so RN(sqrt_core(x) - R) = -R for the
// radii R in {3, 2.5, 1, 0.5} it is always used with.  NaN stays NaN.
__device__ __forceinline__ float sqrt_core(float x) {
  const float y = __builtin_amdgcn_rsqf(x + 0x1p-126f);
  const float s = x * y;
  const float h = 0.5f * y;
  const float r = __builtin_fmaf(-s, s, x);
  return __builtin_fmaf(h, r, s);
}

// 1/x and x / i (the bounce weights, i = 1..5, glsl:186-187) are IEEE
// divisions: a v_rcp_f32 + Newton form (exact for 2^-125 <= |x| <= 2^125) and a
// Markstein x/3, x/5 (exact over all finite x) were proven by
// tools/exhaustive_fp.hip (profiles/r01_exhaustive_fp.log) but measured no
// faster here than the division.
__device__ __forceinline__ float rcp_exact(float x) { return 1.0f / x; }
__device__ __forceinline__ float div_small(float x, int i) { return x / (float)i; }

// 1/s for s = sqrt_cr_nonneg(d) of a finite d >= 0, i.e. s = 0 or
// 2^-74.5 <= s <= 2^64, inside the v_rcp + Newton form's proven range
// (tools/exhaustive_fp.hip): no guard needed.  For
// s = 0 (and NaN) it gives NaN where the IEEE 1/s gives inf; normalize()
// multiplies that by the zero vector, and 0 * inf is NaN too.
__device__ __forceinline__ float rcp_of_sqrt(float s) {
  const float y = __builtin_amdgcn_rcpf(s);
  const float e = __builtin_fmaf(-s, y, 1.0f);
  return __builtin_fmaf(e, y, y);
}

// Smallest input sqrt_core handles exactly (besides 0).
constexpr float SQRT_CORE_MIN = 0x1p-96f;
// Smallest |x| for which div_capbb is exact.
constexpr float DIV_CAPBB_MIN = 0x1p-100f;

// sqrt(x) for x >= 0 (finite), correctly rounded on all of [0, FLT_MAX]:
// inputs below 2^-96 are scaled by 2^64 into sqrt_core's exact domain (the
// smallest denormal becomes 2^-85) and the result by 2^-32 (both exact).  Exhaustively equal to __builtin_sqrtf on
// [0, FLT_MAX] (tools/exhaustive_fp.hip).
__device__ __forceinline__ float sqrt_cr_nonneg(float x) {
  const bool small = x < 0x1p-96f;
  const float s = sqrt_core(small ? x * 0x1p64f : x);
  return small ? s * 0x1p-32f : s;
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
