// rm_scene.hpp — device-side scene + shading for gfx950 (HIP).
//
// The per-sample math of shaders/computeShader.glsl, written for the GPU under
// the built-in semantics contract of DESIGN.md §2.  Compiled with
// -ffp-contract=off and HIP's default correctly-rounded f32 sqrt/div, so every
// + - * / sqrt below is one IEEE binary32 operation in GLSL source order, and
// the geometry (march, normals, shadows, reflections) is bit-identical to the
// CPU oracle.  Two deliberate, value-preserving deviations from a literal
// transcription, each proven equal in DESIGN.md §3:
//   * the sdf returns the minimum distance with v_min_f32 and tracks the opU id
//     (glsl:105, ties go to the later primitive) with a compare + select;
//   * sdPlane(p, (0,1,0,5.5)) = dot(p,(0,1,0)) + 5.5 is computed as p.y + 5.5
//     (the x*0 and z*0 terms are signed zeros that cannot change the sum).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rm_fastmath.hpp"

namespace rmd {

struct f3 {
  float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 muls(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 subs(f3 a, float s) { return mk(a.x - s, a.y - s, a.z - s); }
__device__ __forceinline__ f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ float len(f3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return muls(a, 1.0f / __builtin_sqrtf(dot(a, a))); }
// v_min_f32 / v_min3_f32 without the NaN-quieting canonicalisations LLVM adds
// when it cannot prove an operand canonical (values merged from branches).
// All operands here are finite sdf values or +inf, never NaN.
__device__ __forceinline__ float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// GLSL min/max (y < x ? y : x) — used where a signed zero or NaN could differ.
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return x < y ? y : x; }
__device__ __forceinline__ f3 reflect(f3 i, f3 n) { return sub(i, muls(n, 2.0f * dot(n, i))); }

// Frame constants, passed by value as kernel arguments (lands in SGPRs).
struct Frame {
  float cam_pos[4], cam_dir[4], cam_y[4], cam_x[4];
  float lpos[3], lamb[3], ldif[3], lspec[3];
  float lconst, llin, lquad;
  float blend;     // sin(iTime)/2 + 0.5, host sinf (glsl:117)
  float omblend;   // 1 - blend (uniform-only subexpression of mix)
  float k;         // softshadow k: 2.0 (glsl:185,236) or +inf (hard-shadow extension)
  float persp;     // radians(45) = 45 * 0.017453292519943295f (glsl:70)
  int32_t bounces; // bounceVar, 0..5
  int32_t aa;      // AA
  int32_t width, height;
  int32_t row_block, shard, nshards;
  int32_t rows;          // rows this launch renders (height, or the shard's rows_cap)
  uint8_t* rgba8;        // [rows][width][4] or null
  float* rgba32f;        // [rows][width][4] or null
  uint32_t* sdf_counts;  // [rows][width] or null (counter builds)
  unsigned long long* counters;  // 6 x u64 (counter builds)
  uint32_t* queue;       // work-queue head (wave-queue kernel), zeroed per dispatch
};

// ---- scene: computeShader.glsl:83-123 ----------------------------------------
// Minimum scene distance and the opU id (glsl:107-123).  `id` follows opU's
// rule exactly: a later primitive replaces the running one unless the running
// distance is strictly smaller.  blend/omblend carry mix()'s a and 1-a.
//
// SAFE = false uses the cheap exact sequences of rm_fastmath.hpp (sqrt_core,
// div_capbb), each exact on its proven domain; any lane whose operands leave
// that domain (a sqrt argument in (0, 2^-96), |capsule numerator| < 2^-100)
// sets `tiny`, and scene() recomputes those lanes with SAFE = true (the full
// correctly-rounded forms).  Either way the result is the IEEE value.
template <bool WANT_ID, bool SAFE>
__device__ __forceinline__ float scene_impl(f3 p, float blend, float omblend, int& id, bool& tiny) {
  auto SQ = [](float x) { return SAFE ? sqrt_cr_nonneg(x) : sqrt_core(x); };
  // sphere (15,0,-10) r3, id 0   glsl:111
  const float ax = p.x - 15.0f, ay = p.y, az = p.z + 10.0f;
  const float ay2 = ay * ay, az2 = az * az;
  const float x0 = (ax * ax + ay2) + az2;
  float d = SQ(x0) - 3.0f;
  if (WANT_ID) id = 0;
  // sphere (-25,0,-10) r3, id 1  glsl:112
  const float bx = p.x + 25.0f;
  const float x1 = (bx * bx + ay2) + az2;
  const float d1 = SQ(x1) - 3.0f;
  if (WANT_ID) id = (d < d1) ? id : 1;
  d = fminf(d, d1);
  // mix(box, sphere, blend) at (-5,0,-10), id 4   glsl:87-91,115-117
  const float cx = p.x + 5.0f;
  const float cx2 = cx * cx;
  const float qx = fabsf(cx) - 3.0f, qy = fabsf(ay) - 2.5f, qz = fabsf(az) - 2.5f;
  const float mx = fmaxf(qx, 0.0f), my = fmaxf(qy, 0.0f), mz = fmaxf(qz, 0.0f);
  const float xb = (mx * mx + my * my) + mz * mz;
  const float box = fminf(fmaxf(qx, fmaxf(qy, qz)), 0.0f) + SQ(xb);
  const float xs = (cx2 + ay2) + az2;
  const float sph = SQ(xs) - 3.0f;
  const float d4 = box * omblend + sph * blend;
  if (WANT_ID) id = (d < d4) ? id : 4;
  d = fminf(d, d4);
  // torus at (-5,0,10), (pos - c).xzy, t = (2.5, 0.5), id 5   glsl:93-96,119
  const float tz = p.z - 10.0f;
  const float xt1 = cx2 + ay2;
  const float l = SQ(xt1) - 2.5f;
  const float xt2 = l * l + tz * tz;
  const float d5 = SQ(xt2) - 0.5f;
  if (WANT_ID) id = (d < d5) ? id : 5;
  d = fminf(d, d5);
  // capsule at (-5,-2,-30), a(-.1,.1,-.1) b(2,4,2) r1, id 6   glsl:98-103,120
  const float px_ = cx - CAP_AX, py_ = (p.y + 2.0f) - CAP_AY, pz_ = (p.z + 30.0f) - CAP_AZ;
  const float hn = (px_ * CAP_BAX + py_ * CAP_BAY) + pz_ * CAP_BAZ;
  float h = SAFE ? hn / CAP_BB_HOST : div_capbb(hn);
  h = fminf(fmaxf(h, 0.0f), 1.0f);
  const float ex = px_ - CAP_BAX * h, ey = py_ - CAP_BAY * h, ez = pz_ - CAP_BAZ * h;
  const float xc = (ex * ex + ey * ey) + ez * ez;
  const float d6 = SQ(xc) - 1.0f;
  if (WANT_ID) id = (d < d6) ? id : 6;
  d = fminf(d, d6);
  // plane y = -5.5, id 7 (MATTE)   glsl:85,121
  const float d7 = p.y + 5.5f;
  if (WANT_ID) id = (d < d7) ? id : 7;
  d = fminf(d, d7);
  if (!SAFE) {
    // operands outside the fast sequences' proven domains (see above)
    const float m = fminf(fminf(fminf(x0, x1), fminf(xs, xt1)), fminf(xt2, xc));
    tiny = (m < SQRT_CORE_MIN) | ((xb > 0.0f) & (xb < SQRT_CORE_MIN)) |
           (fabsf(hn) < DIV_CAPBB_MIN);
  }
  return d;
}

// ---- scene with exact bounding-sphere culling --------------------------------
// Same value and id as scene_impl.  Each expensive primitive k gets a lower
// bound LB_k <= its float sdf and the plane/spheres/blend give an upper bound
// U >= the float minimum, from raw v_sqrt_f32 (within 1.5 ulp, see
// rm_fastmath.hpp) widened by a relative 2^-12 and an absolute 2^-18 margin.
// If LB_k > U the primitive is strictly farther than the minimum: it can
// neither be the minimum nor tie it (opU ties go to the later primitive), so
// skipping it changes nothing.  A primitive is evaluated exactly when any lane
// of the wave needs it (the branch is skipped only when no lane does).
//   bounding spheres (centre, radius):   sdf >= |p - c| - R   and, for U,
//   sphere  (15,0,-10) / (-25,0,-10): R = 3 (exact: sdf = |p - c| - 3)
//   box/sphere blend (-5,0,-10): R = |(3,2.5,2.5)| = 4.6368 (box circumradius);
//                                upper bound |p - c| - 2.5 (box inradius)
//   torus (-5,0,10): R = 2.5 + 0.5
//   capsule: centre = midpoint of a..b = (-4.05,0.05,-29.05), R = |b-a|/2 + 1
constexpr float CULL_REL_LO = 1.0f - 0x1p-12f;
constexpr float CULL_REL_HI = 1.0f + 0x1p-12f;
constexpr float CULL_ABS = 0x1p-18f;
constexpr float R_BLEND_LO = 4.63682f;   // >= sqrt(3^2 + 2.5^2 + 2.5^2) = 4.636809
constexpr float R_TORUS = 3.0f;
constexpr float R_CAPSULE = 3.45115f;    // >= sqrt(24.03)/2 + 1 = 3.451050
constexpr float CAP_MX = -4.05f, CAP_MY = 0.05f, CAP_MZ = -29.05f;

#ifdef RM_STATS
// Diagnostic build only: wave-level counts of exact primitive evaluations.
__device__ unsigned long long g_stats[16];
#define RM_STAT(k)                                                   \
  do {                                                               \
    if (__lane_id() == __builtin_ffsll(__ballot(1)) - 1) atomicAdd(&g_stats[k], 1ull); \
  } while (0)
#else
#define RM_STAT(k) \
  do {             \
  } while (0)
#endif

template <bool WANT_ID>
__device__ __forceinline__ float scene_cull(f3 p, float blend, float omblend, int& id, bool& tiny) {
  // centre offsets and squared centre distances (shared sub-terms)
  const float ax = p.x - 15.0f, ay = p.y, az = p.z + 10.0f;
  const float bx = p.x + 25.0f, cx = p.x + 5.0f, tz = p.z - 10.0f;
  const float ay2 = ay * ay, az2 = az * az, cx2 = cx * cx;
  const float x0 = (ax * ax + ay2) + az2;     // sphere 0 (exact sdf argument)
  const float x1 = (bx * bx + ay2) + az2;     // sphere 1 (exact sdf argument)
  const float xs = (cx2 + ay2) + az2;         // blend centre (= its sphere's argument)
  const float xt1 = cx2 + ay2;                // torus inner argument
  const float kx = p.x - CAP_MX, ky = p.y - CAP_MY, kz = p.z - CAP_MZ;
  const float xtc = xt1 + tz * tz;            // torus centre (bound only)
  const float xk = (kx * kx + ky * ky) + kz * kz;  // capsule centre (bound only)
  const float r0 = __builtin_amdgcn_sqrtf(x0), r1 = __builtin_amdgcn_sqrtf(x1);
  const float rs = __builtin_amdgcn_sqrtf(xs), rt = __builtin_amdgcn_sqrtf(xtc);
  const float rk = __builtin_amdgcn_sqrtf(xk);
  const float d7 = p.y + 5.5f;  // plane, exact (glsl:85,121)
  // upper bound of the minimum
  float U = fminf(d7, __builtin_fmaf(r0, CULL_REL_HI, CULL_ABS - 3.0f));
  U = fminf(U, __builtin_fmaf(r1, CULL_REL_HI, CULL_ABS - 3.0f));
  U = fminf(U, __builtin_fmaf(rs, CULL_REL_HI, CULL_ABS - 2.5f));
  RM_STAT(0);
  const float INF = __builtin_huge_valf();
  float d0 = INF, d1 = INF, d4 = INF, d5 = INF, d6 = INF;
  bool tn = false;
  if (__builtin_fmaf(r0, CULL_REL_LO, -(CULL_ABS + 3.0f)) <= U) {
    RM_STAT(1);
    d0 = sqrt_core(x0) - 3.0f;  // glsl:111
    tn |= x0 < SQRT_CORE_MIN;
  }
  if (__builtin_fmaf(r1, CULL_REL_LO, -(CULL_ABS + 3.0f)) <= U) {
    RM_STAT(2);
    d1 = sqrt_core(x1) - 3.0f;  // glsl:112
    tn |= x1 < SQRT_CORE_MIN;
  }
  if (__builtin_fmaf(rs, CULL_REL_LO, -(CULL_ABS + R_BLEND_LO)) <= U) {  // glsl:87-91,115-117
    RM_STAT(3);
    const float qx = fabsf(cx) - 3.0f, qy = fabsf(ay) - 2.5f, qz = fabsf(az) - 2.5f;
    const float mx = fmaxf(qx, 0.0f), my = fmaxf(qy, 0.0f), mz = fmaxf(qz, 0.0f);
    const float xb = (mx * mx + my * my) + mz * mz;
    const float box = fminf(fmaxf(qx, fmaxf(qy, qz)), 0.0f) + sqrt_core(xb);
    const float sph = sqrt_core(xs) - 3.0f;
    d4 = box * omblend + sph * blend;
    tn |= (xs < SQRT_CORE_MIN) | ((xb > 0.0f) & (xb < SQRT_CORE_MIN));
  }
  if (__builtin_fmaf(rt, CULL_REL_LO, -(CULL_ABS + R_TORUS)) <= U) {  // glsl:93-96,119
    RM_STAT(4);
    const float l = sqrt_core(xt1) - 2.5f;
    const float xt2 = l * l + tz * tz;
    d5 = sqrt_core(xt2) - 0.5f;
    tn |= (xt1 < SQRT_CORE_MIN) | (xt2 < SQRT_CORE_MIN);
  }
  if (__builtin_fmaf(rk, CULL_REL_LO, -(CULL_ABS + R_CAPSULE)) <= U) {  // glsl:98-103,120
    RM_STAT(5);
    const float px_ = cx - CAP_AX, py_ = (p.y + 2.0f) - CAP_AY, pz_ = (p.z + 30.0f) - CAP_AZ;
    const float hn = (px_ * CAP_BAX + py_ * CAP_BAY) + pz_ * CAP_BAZ;
    const float h = fminf(fmaxf(div_capbb(hn), 0.0f), 1.0f);
    const float ex = px_ - CAP_BAX * h, ey = py_ - CAP_BAY * h, ez = pz_ - CAP_BAZ * h;
    const float xc = (ex * ex + ey * ey) + ez * ez;
    d6 = sqrt_core(xc) - 1.0f;
    tn |= (xc < SQRT_CORE_MIN) | (fabsf(hn) < DIV_CAPBB_MIN);
  }
  tiny = tn;
  // opU chain in the reference order (glsl:111-121); culled entries are +inf
  float d = d0;
  if (WANT_ID) {
    id = 0;
    id = (d < d1) ? id : 1;
    d = vmin(d, d1);
    id = (d < d4) ? id : 4;
    d = vmin(d, d4);
    id = (d < d5) ? id : 5;
    d = vmin(d, d5);
    id = (d < d6) ? id : 6;
    d = vmin(d, d6);
    id = (d < d7) ? id : 7;
    d = vmin(d, d7);
  } else {
    d = vmin3(vmin3(d, d1, d4), vmin(d5, d6), d7);
  }
  return d;
}

// ---- scene with LAZY culling along a ray ----------------------------------------
// For a march p(t) = ro + rd*t.  Primitive k is skipped while t < te[k].  When a
// primitive is re-tested at p_i (t_i) with upper bound U_i >= min(p_i) and
// lower bound LB_k(p_i) <= sdf_k(p_i), and LB_k > U_i, then for any later
// point p_j on the ray, by the 1-Lipschitz property of the distances,
//   sdf_k(p_j) - min(p_j) >= (LB_k - U_i) - 2 |p_j - p_i|,  |p_j - p_i| ~ |rd| (t_j - t_i),
// so k stays strictly above the minimum (cannot be it, cannot tie it) while
//   t_j < te_k = t_i + (LB_k - U_i - slack) / (2 |rd| (1 + 2^-10)).
// `slack` covers the float error of the evaluated sdfs and of p(t) itself
// (relative 2^-14 of |ro|_1 + |rd| t + 64 — generous against ~2^-21 actual).
// A primitive whose bound does not cull it is evaluated exactly and re-tested
// at the next step.  U_i = min(plane, exact values evaluated so far this
// step).  The minimum and the opU id are merged in the reference order, so the
// result equals scene_impl's.
struct LazyCull {
  float te[5];   // expiry t of spheres 0/1, blend, torus, capsule
  float temin;   // min over te[]
  float rdlen;   // |rd| (upper-rounded)
  float ro1;     // |ro|_1
};

__device__ __forceinline__ void lazy_init(LazyCull& c, f3 ro, f3 rd) {
  const float NEG = -__builtin_huge_valf();
#pragma unroll
  for (int k = 0; k < 5; ++k) c.te[k] = NEG;
  c.temin = NEG;
  c.rdlen = __builtin_amdgcn_sqrtf(dot(rd, rd)) * (1.0f + 0x1p-16f);
  c.ro1 = fabsf(ro.x) + fabsf(ro.y) + fabsf(ro.z);
}

template <bool WANT_ID>
__device__ __forceinline__ float scene_lazy(f3 p, float t, LazyCull& lc, float blend, float omblend,
                                            int& id, bool& tiny) {
  const float INF = __builtin_huge_valf();
  const float d7 = p.y + 5.5f;  // plane, exact (glsl:85,121)
  float d0 = INF, d1 = INF, d4 = INF, d5 = INF, d6 = INF;
  bool tn = false;
  if (t >= lc.temin) {
    float U = d7;
    const float slack = 0x1p-14f * (lc.ro1 + lc.rdlen * t + 64.0f);
    const float inv2v = 0.5f * (1.0f - 0x1p-10f) / lc.rdlen;
    // expiry update: k stays culled while the ray travels (lb - U - slack)/2
    auto retest = [&](float x, float R, float& te) -> bool {  // true: evaluate exactly
      const float lb = __builtin_fmaf(__builtin_amdgcn_sqrtf(x), CULL_REL_LO, -(CULL_ABS + R));
      const float m = lb - U - slack;
      if (m > 0.0f) {
        te = __builtin_fmaf(m, inv2v, t);
        return false;
      }
      te = t;
      return true;
    };
    const float ax = p.x - 15.0f, ay = p.y, az = p.z + 10.0f;
    const float ay2 = ay * ay, az2 = az * az;
    const float cx = p.x + 5.0f, cx2 = cx * cx;
    if (t >= lc.te[0]) {  // sphere (15,0,-10) r3, glsl:111
      const float x0 = (ax * ax + ay2) + az2;
      if (retest(x0, 3.0f, lc.te[0])) {
        d0 = sqrt_core(x0) - 3.0f;
        U = vmin(U, d0);
        tn |= x0 < SQRT_CORE_MIN;
      }
    }
    if (t >= lc.te[1]) {  // sphere (-25,0,-10) r3, glsl:112
      const float bx = p.x + 25.0f;
      const float x1 = (bx * bx + ay2) + az2;
      if (retest(x1, 3.0f, lc.te[1])) {
        d1 = sqrt_core(x1) - 3.0f;
        U = vmin(U, d1);
        tn |= x1 < SQRT_CORE_MIN;
      }
    }
    if (t >= lc.te[2]) {  // box/sphere blend, glsl:87-91,115-117
      const float xs = (cx2 + ay2) + az2;
      if (retest(xs, R_BLEND_LO, lc.te[2])) {
        const float qx = fabsf(cx) - 3.0f, qy = fabsf(ay) - 2.5f, qz = fabsf(az) - 2.5f;
        const float mx = fmaxf(qx, 0.0f), my = fmaxf(qy, 0.0f), mz = fmaxf(qz, 0.0f);
        const float xb = (mx * mx + my * my) + mz * mz;
        const float box = fminf(fmaxf(qx, fmaxf(qy, qz)), 0.0f) + sqrt_core(xb);
        const float sph = sqrt_core(xs) - 3.0f;
        d4 = box * omblend + sph * blend;
        U = vmin(U, d4);
        tn |= (xs < SQRT_CORE_MIN) | ((xb > 0.0f) & (xb < SQRT_CORE_MIN));
      }
    }
    if (t >= lc.te[3]) {  // torus, glsl:93-96,119
      const float tz = p.z - 10.0f;
      const float xt1 = cx2 + ay2;
      if (retest(xt1 + tz * tz, R_TORUS, lc.te[3])) {
        const float l = sqrt_core(xt1) - 2.5f;
        const float xt2 = l * l + tz * tz;
        d5 = sqrt_core(xt2) - 0.5f;
        U = vmin(U, d5);
        tn |= (xt1 < SQRT_CORE_MIN) | (xt2 < SQRT_CORE_MIN);
      }
    }
    if (t >= lc.te[4]) {  // capsule, glsl:98-103,120
      const float kx = p.x - CAP_MX, ky = p.y - CAP_MY, kz = p.z - CAP_MZ;
      if (retest((kx * kx + ky * ky) + kz * kz, R_CAPSULE, lc.te[4])) {
        const float px_ = cx - CAP_AX, py_ = (p.y + 2.0f) - CAP_AY, pz_ = (p.z + 30.0f) - CAP_AZ;
        const float hn = (px_ * CAP_BAX + py_ * CAP_BAY) + pz_ * CAP_BAZ;
        const float h = fminf(fmaxf(div_capbb(hn), 0.0f), 1.0f);
        const float ex = px_ - CAP_BAX * h, ey = py_ - CAP_BAY * h, ez = pz_ - CAP_BAZ * h;
        const float xc = (ex * ex + ey * ey) + ez * ez;
        d6 = sqrt_core(xc) - 1.0f;
        U = vmin(U, d6);
        tn |= (xc < SQRT_CORE_MIN) | (fabsf(hn) < DIV_CAPBB_MIN);
      }
    }
    lc.temin = vmin3(vmin3(lc.te[0], lc.te[1], lc.te[2]), lc.te[3], lc.te[4]);
  }
  tiny = tn;
  float d = d0;
  if (WANT_ID) {
    id = 0;
    id = (d < d1) ? id : 1;
    d = vmin(d, d1);
    id = (d < d4) ? id : 4;
    d = vmin(d, d4);
    id = (d < d5) ? id : 5;
    d = vmin(d, d5);
    id = (d < d6) ? id : 6;
    d = vmin(d, d6);
    id = (d < d7) ? id : 7;
    d = vmin(d, d7);
  } else {
    d = vmin3(vmin3(d, d1, d4), vmin(d5, d6), d7);
  }
  return d;
}

#ifndef RM_SCENE_CULL
#define RM_SCENE_CULL 1
#endif

template <bool WANT_ID>
__device__ __forceinline__ float scene(f3 p, float blend, float omblend, int& id) {
  bool tiny = false;
  float d = RM_SCENE_CULL ? scene_cull<WANT_ID>(p, blend, omblend, id, tiny)
                          : scene_impl<WANT_ID, false>(p, blend, omblend, id, tiny);
  if (__builtin_expect(tiny, 0)) d = scene_impl<WANT_ID, true>(p, blend, omblend, id, tiny);
  return d;
}

// softshadow's  res = min(res, k * h / t)  (glsl:211), exactly.  The quotient
// only matters when it is below res, so it is first bounded with v_rcp_f32
// (within 1 ulp): if (k*h)*rcp(t) exceeds res by a 2^-16 relative margin the
// exact quotient does too and res is unchanged; otherwise the correctly
// rounded division decides.  k = +inf (hard shadows) gives +inf: unchanged.
__device__ __forceinline__ float shadow_min(float res, float k, float h, float t) {
  const float kh = k * h;
  const float qa = kh * __builtin_amdgcn_rcpf(t);
  if (qa > res * (1.0f + 0x1p-16f)) return res;
  return gmin(res, kh / t);
}

// checkers(p) glsl:77-80
__device__ __forceinline__ float checkers(f3 p) {
  int a = (int)(1000.0f + p.x) % 2;
  int b = (int)(1000.0f + p.z) % 2;
  return (a != b) ? 1.0f : 0.2f;
}

// Colour of primitive `id` (glsl:111-121); `chk` is checkers() at the hit
// point, used for the floor (id 7).
__device__ __forceinline__ f3 id_color(int id, float chk) {
  switch (id) {
    case 0: return mk(0.1804f, 0.6f, 0.2157f);
    case 1: return mk(0.0f, 0.851f, 1.0f);
    case 4: return mk(0.4863f, 0.3529f, 0.702f);
    case 5: return mk(0.9137f, 0.549f, 0.0f);
    case 6: return mk(0.8f, 0.0902f, 0.4824f);
    default: return mk(chk, chk, chk);
  }
}

__device__ __forceinline__ f3 hit_color(int id, f3 p) {
  return id_color(id, id == 7 ? checkers(p) : 0.0f);
}

// getPointLight glsl:253-276
__device__ __forceinline__ f3 point_light(const Frame& F, f3 color, f3 normal, f3 pos) {
  f3 lpos = mk(F.lpos[0], F.lpos[1], F.lpos[2]);
  f3 ambient = mk(F.lamb[0], F.lamb[1], F.lamb[2]);
  f3 viewDir = normalize(sub(pos, mk(F.cam_pos[0], F.cam_pos[1], F.cam_pos[2])));
  f3 lightDir = normalize(sub(lpos, pos));
  float NtoL = gmax(dot(normal, lightDir), 0.0f);
  f3 diffuse = muls(mk(F.ldif[0], F.ldif[1], F.ldif[2]), NtoL);
  f3 reflectDir = reflect(lightDir, normal);
  float spec = powf(gmax(dot(viewDir, reflectDir), 0.0f), 32.0f);
  f3 specular = muls(mk(F.lspec[0], F.lspec[1], F.lspec[2]), spec);
  float distance = len(sub(lpos, pos));
  float attenuation = 1.0f / ((F.lconst + F.llin * distance) + F.lquad * (distance * distance));
  diffuse = muls(diffuse, attenuation);
  ambient = muls(ambient, attenuation);
  specular = muls(specular, attenuation);
  return mul(color, add(add(diffuse, ambient), specular));
}

__device__ __forceinline__ f3 gamma(f3 c) {
  return mk(powf(c.x, 0.4545f), powf(c.y, 0.4545f), powf(c.z, 0.4545f));
}

// castRay glsl:68-74 over vec4 (w included, as the GLSL does).
__device__ __forceinline__ void cast_ray(const Frame& F, float uvx, float uvy, f3& ro, f3& rd) {
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = (uvx * F.cam_x[k] + uvy * F.cam_y[k]) + F.cam_dir[k] * F.persp;
  float dd = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
  float inv = 1.0f / __builtin_sqrtf(dd);
  ro = mk(F.cam_pos[0], F.cam_pos[1], F.cam_pos[2]);
  rd = mk(v[0] * inv, v[1] * inv, v[2] * inv);
}

// RGBA8 quantization round(clamp(c,0,1)*255), NaN -> 0.
__device__ __forceinline__ uint32_t quantize(float c) {
  float v = (c > 0.0f) ? ((c < 1.0f) ? c : 1.0f) : 0.0f;
  return (uint32_t)(v * 255.0f + 0.5f);
}

// Global row of a launch-local row (row sharding).
__device__ __forceinline__ int global_row(const Frame& F, int local_row) {
  if (F.nshards <= 1) return local_row;
  int lb = local_row / F.row_block;
  int g = (lb * F.nshards + F.shard) * F.row_block + local_row % F.row_block;
  return g < F.height ? g : -1;
}

__device__ __forceinline__ void store_pixel(const Frame& F, size_t idx, float r, float g, float b,
                                            float a) {
  if (F.rgba8) {
    uint32_t w = quantize(r) | (quantize(g) << 8) | (quantize(b) << 16) | (quantize(a) << 24);
    reinterpret_cast<uint32_t*>(F.rgba8)[idx] = w;
  }
  if (F.rgba32f) reinterpret_cast<float4*>(F.rgba32f)[idx] = make_float4(r, g, b, a);
}

}  // namespace rmd
