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

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "rm_fastmath.hpp"
#include "rm_shard.hpp"

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
// a / i for the bounce weights (rm_fastmath.hpp div_small), exact
__device__ __forceinline__ f3 divi(f3 a, int i) { return mk(div_small(a.x, i), div_small(a.y, i), div_small(a.z, i)); }
// sqrt_cr_nonneg == the correctly rounded sqrt on [0, FLT_MAX] (rm_fastmath.hpp),
// with NaN and +inf passing through unchanged
__device__ __forceinline__ float len(f3 a) { return sqrt_cr_nonneg(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return muls(a, rcp_of_sqrt(sqrt_cr_nonneg(dot(a, a)))); }
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
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
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
  float shc;       // the soft-shadow exit's ratio bound c = (1 + 2^-9) / k (1 + 2^-12), 0 for
                   // k = +inf (shadow_exit_init): uniform, formed once per frame on the host
  float persp;     // radians(45) = 45 * 0.017453292519943295f (glsl:70)
  // uv of every pixel column / row, host IEEE in the shader's order (glsl:301-332):
  // [k = 0] (2 p - dims) / dims, [k = 1 + s] after the cumulative sub-sample
  // offsets offset[0..s] / dims; 5 floats per column (uvx) and per row (uvy)
  const float* uvx;
  const float* uvy;
  // The same uv from arithmetic (lane_uv), when the host has checked that it is
  // exact for every column and row of this frame size (uv_exact): the division
  // (2p - dims) / dims as a multiply by RN(1 / dims) plus one fma remainder
  // correction, and the cumulative offsets RN(offset_k / dims) added in order.
  float uv_rcp[2];       // RN(1 / W), RN(1 / H)
  float uv_dims[2];      // W, H as floats
  float uv_off[2][4];    // RN(ox_k / W), RN(oy_k / H)
  int32_t uv_exact;
  int32_t unit_rd; // every primary rd of this frame has |rd| within 2^-20 of 1 (host check, march)
  int32_t bounces; // bounceVar, 0..5
  int32_t aa;      // AA
  int32_t width, height;
  int32_t row_block, shard, nshards;
  int32_t row_block0;    // shard 0's rows per round (rm_shard.hpp; = row_block unsharded)
  int32_t rows;          // rows this launch renders (height, or the shard's rows_cap)
  uint8_t* rgba8;        // [rows][width][4] or null
  float* rgba32f;        // [rows][width][4] or null
  uint32_t* sdf_counts;  // [rows][width] or null (counter builds)
  unsigned long long* counters;  // 6 x u64 (counter builds)
  float prepv[16];       // step 0 of the primary rays (PrepSlot), from the host per frame
  const float* scene;    // runtime scene table (rm_set_scene), TABLE_WORDS per primitive, or null
  int32_t nprims;        // entries in `scene`
  int32_t grid_x, grid_y;  // k_pixel / k_sample grid (rm::pixel_grid): ordinary kernel
                           // arguments, loaded with the rest of the prologue's
  int32_t rgb3;  // rgba8 holds a packed RGB shard, [rows][width][3] (rm_config.shard_format):
                 // the alpha the reference stores is the constant 1.0 (glsl:314-341), so a
                 // gathered shard carries 3 B per pixel and the un-shard writes alpha 255
};

// A batch of frames of one context (rm_dispatch_frames): one grid over n frames
// of the same size and AA setting, frame z = blockIdx.z, each with its own
// constants and output pointers.  Kernel arguments, like a single Frame: the
// frame's fields are scalar loads from the kernarg segment at a wave-uniform
// offset.
constexpr int kMaxBatch = 32;  // == RM_MAX_BATCH (rm_api.h; static_assert in rm_api.hip)
struct FrameBatch {
  Frame f[kMaxBatch];
};

// ---- scene: computeShader.glsl:83-123 ----------------------------------------
// Three exact evaluations of the same sdf (value and opU id equal to a literal
// transcription):
//   scene_exact  — every primitive;
//   scene_cull   — bounding-sphere culling (shadow march, normal probes);
//   scene_lazy   — lazy culling along a march ray (RayMarch / reflectedRay loops).
// opU (glsl:105): a later primitive replaces the running one unless the
// running distance is strictly smaller, so ties go to the later primitive.
//
// Square roots use sqrt_core (rm_fastmath.hpp): correctly rounded on {0} U
// [2^-96, FLT_MAX] and < 2^-47 on (0, 2^-96) (both proven exhaustively).  Every
// use but one subtracts R in {3, 2.5, 1, 0.5} right away, and RN(s - R) = -R for
// every s < 2^-26, so the result is exact on the whole domain; the box's outer
// length (used unshifted) takes the full-range sqrt_cr_nonneg.  The capsule
// divide div_capbb is exact for |x| >= 2^-100; below that, h <= 2^-104 and
// every BA*h term underflows out of (BA*h)^2 or is absorbed by a |pa| >= 2^-27,
// so xc (hence the sdf) is identical.
//
// Culled primitives are strictly farther than the minimum, so the distance-only
// variants return the running minimum over the plane and the evaluated
// primitives directly (no merge needed).

// Capsule and bounding-sphere constants.
constexpr float CULL_REL_LO = 1.0f - 0x1p-12f;
constexpr float CULL_REL_HI = 1.0f + 0x1p-12f;
constexpr float CULL_ABS = 0x1p-18f;
constexpr float R_BLEND_LO = 4.63682f;   // >= |(3,2.5,2.5)| = 4.636809, box circumradius
constexpr float R_TORUS = 3.0f;          // 2.5 + 0.5
constexpr float R_CAPSULE = 3.45115f;    // >= |b-a|/2 + 1 = sqrt(24.03)/2 + 1 = 3.451050
constexpr float CAP_MX = -4.05f, CAP_MY = 0.05f, CAP_MZ = -29.05f;  // segment midpoint

// The cull test LB_k <= U of the torus and the capsule without the square root
// (round 3: a v_sqrt takes two VALU issue slots): evaluate iff
//   RN(x (1 - 2^-11)) <= RN(a^2),  a = RN(U + CULL_ABS + R),  x = |p - c|^2.
// For a >= 0 this is sqrt(x) (1 - 2^-11)^(1/2) <= a up to the roundings, and
// (1 - 2^-11)^(1/2) < CULL_REL_LO: a cull keeps the 2^-12 relative margin of the
// v_sqrt form less at most 0.5 ulp of a (the v_sqrt form: up to 1.5 ulp;
// tests/test_cull_bounds.py checks this on samples at the boundary).  For a < 0 the
// v_sqrt form culls (LB >= -CULL_ABS - R > U); this one culls or evaluates, and
// an extra exact evaluation is never wrong.  A NaN U culls in both.
constexpr float CULL_SQ_LO = 1.0f - 0x1p-11f;
__device__ __forceinline__ bool ball_needs(float x, float U, float R) {
  const float a = U + (CULL_ABS + R);
  return x * CULL_SQ_LO <= a * a;
}

#ifdef RM_STATS
// Diagnostic build only: g_stats[k] counts waves reaching point k, g_stats[32+k]
// the active lanes there (k < 32).
__device__ unsigned long long g_stats[64];
#define RM_STAT(k)                                                   \
  do {                                                               \
    const unsigned long long m_ = __ballot(1);                       \
    if (__lane_id() == __builtin_ffsll(m_) - 1) {                    \
      atomicAdd(&g_stats[k], 1ull);                                  \
      atomicAdd(&g_stats[32 + (k)], (unsigned long long)__popcll(m_)); \
    }                                                                \
  } while (0)
#elif defined(RM_WAVE_STATS)
// Diagnostic build only (tools/wave_timeline.hip): per-wave counts of the same
// points, g_wave_stats[32 w + k] for the wave of tile w (k_sample's tile order).
__device__ unsigned long long* g_wave_stats;
__device__ __forceinline__ int tile_row(int b, int n);
__device__ __forceinline__ int tile_col(int b, int gx, int G);
#define RM_STAT(k)                                                                             \
  do {                                                                                         \
    const unsigned long long m_ = __ballot(1);                                                 \
    if (__lane_id() == __builtin_ffsll(m_) - 1) {                                              \
      const size_t w_ = (size_t)tile_row(blockIdx.y, gridDim.y) * gridDim.x + tile_col(blockIdx.x, gridDim.x, 8); \
      atomicAdd(&g_wave_stats[32 * w_ + (k)], 1ull);                                           \
    }                                                                                          \
  } while (0)
#else
#define RM_STAT(k) \
  do {             \
  } while (0)
#endif

// Exact per-primitive distances from shared centre offsets.
struct Offs {
  float ax, ay, az, bx, cx, ay2, az2, cx2;
};
__device__ __forceinline__ Offs offsets(f3 p) {
  Offs o;
  o.ax = p.x - 15.0f;  // sphere 0 centre (15,0,-10)
  o.ay = p.y;
  o.az = p.z + 10.0f;
  o.bx = p.x + 25.0f;  // sphere 1 centre (-25,0,-10)
  o.cx = p.x + 5.0f;   // blend (-5,0,-10), torus (-5,0,10), capsule (-5,-2,-30)
  o.ay2 = o.ay * o.ay;
  o.az2 = o.az * o.az;
  o.cx2 = o.cx * o.cx;
  return o;
}
__device__ __forceinline__ float sd_sphere0(const Offs& o, float x0) { return sqrt_core(x0) - 3.0f; }
__device__ __forceinline__ float sd_blend(const Offs& o, float xs, float blend, float omblend) {
  // mix(sdBox(q, (3,2.5,2.5)), sdSphere(q, 3), blend)   glsl:87-91,115-117
  const float qx = fabsf(o.cx) - 3.0f, qy = fabsf(o.ay) - 2.5f, qz = fabsf(o.az) - 2.5f;
  const float mx = fmaxf(qx, 0.0f), my = fmaxf(qy, 0.0f), mz = fmaxf(qz, 0.0f);
  const float xb = (mx * mx + my * my) + mz * mz;
  const float box = fminf(fmaxf(qx, fmaxf(qy, qz)), 0.0f) + sqrt_cr_nonneg(xb);
  const float sph = sqrt_core(xs) - 3.0f;
  return box * omblend + sph * blend;
}
__device__ __forceinline__ float sd_torus(const Offs& o, float tz) {
  // sdTorus((p - c).xzy, (2.5, 0.5))   glsl:93-96,119
  const float l = sqrt_core(o.cx2 + o.ay2) - 2.5f;
  return sqrt_core(l * l + tz * tz) - 0.5f;
}
__device__ __forceinline__ float sd_capsule(const Offs& o, f3 p) {
  // sdCapsule(p - c, a, b, 1)   glsl:98-103,120
  const float px_ = o.cx - CAP_AX, py_ = (p.y + 2.0f) - CAP_AY, pz_ = (p.z + 30.0f) - CAP_AZ;
  const float hn = (px_ * CAP_BAX + py_ * CAP_BAY) + pz_ * CAP_BAZ;
  const float h = fminf(fmaxf(div_capbb(hn), 0.0f), 1.0f);
  const float ex = px_ - CAP_BAX * h, ey = py_ - CAP_BAY * h, ez = pz_ - CAP_BAZ * h;
  return sqrt_core((ex * ex + ey * ey) + ez * ez) - 1.0f;
}

template <bool WANT_ID>
__device__ __forceinline__ float scene_exact(f3 p, float blend, float omblend, int& id) {
  const Offs o = offsets(p);
  const float x0 = (o.ax * o.ax + o.ay2) + o.az2;
  const float x1 = (o.bx * o.bx + o.ay2) + o.az2;
  const float xs = (o.cx2 + o.ay2) + o.az2;
  float d = sqrt_core(x0) - 3.0f;                           // glsl:111
  const float d1 = sqrt_core(x1) - 3.0f;                    // glsl:112
  const float d4 = sd_blend(o, xs, blend, omblend);          // glsl:115-117
  const float d5 = sd_torus(o, p.z - 10.0f);                 // glsl:119
  const float d6 = sd_capsule(o, p);                         // glsl:120
  const float d7 = p.y + 5.5f;                               // glsl:85,121
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
    return d;
  }
  return vmin3(vmin3(d, d1, d4), vmin(d5, d6), d7);
}

// Bounding-sphere culling.  Each expensive primitive k has a lower bound
// LB_k <= its float sdf and the plane/spheres/blend give an upper bound
// U >= the float minimum, from raw v_sqrt_f32 (within 1.5 ulp) widened by a
// relative 2^-12 and an absolute 2^-18 margin:
//   sdf >= |p - c| - R:  spheres R = 3 (exact), blend R = box circumradius,
//   torus R = 3, capsule R = |b-a|/2 + 1 about the segment midpoint;
//   U candidates: plane (exact), spheres |p-c| - 3, blend |p-c| - 2.5 (box inradius).
// LB_k > U  =>  primitive k is strictly farther than the minimum: skip it.  The
// branch for k runs when any lane of the wave needs it.
template <bool WANT_ID, bool PLANE_U = false>
__device__ __forceinline__ float scene_cull(f3 p, float blend, float omblend, int& id) {
  const Offs o = offsets(p);
  const float tz = p.z - 10.0f;
  const float x0 = (o.ax * o.ax + o.ay2) + o.az2;
  const float x1 = (o.bx * o.bx + o.ay2) + o.az2;
  const float xs = (o.cx2 + o.ay2) + o.az2;
  const float kx = p.x - CAP_MX, ky = p.y - CAP_MY, kz = p.z - CAP_MZ;
  const float xtc = (o.cx2 + o.ay2) + tz * tz;
  const float xk = (kx * kx + ky * ky) + kz * kz;
  const float r0 = __builtin_amdgcn_sqrtf(x0), r1 = __builtin_amdgcn_sqrtf(x1);
  const float rs = __builtin_amdgcn_sqrtf(xs);
  const float d7 = p.y + 5.5f;
  float U = vmin(d7, __builtin_fmaf(r0, CULL_REL_HI, CULL_ABS - 3.0f));
  U = vmin3(U, __builtin_fmaf(r1, CULL_REL_HI, CULL_ABS - 3.0f),
            __builtin_fmaf(rs, CULL_REL_HI, CULL_ABS - 2.5f));
  RM_STAT(0);
  if (WANT_ID) {
    const float INF = __builtin_huge_valf();
    float d0 = INF, d1 = INF, d4 = INF, d5 = INF, d6 = INF;
    if (__builtin_fmaf(r0, CULL_REL_LO, -(CULL_ABS + 3.0f)) <= U) d0 = sqrt_core(x0) - 3.0f;
    if (__builtin_fmaf(r1, CULL_REL_LO, -(CULL_ABS + 3.0f)) <= U) d1 = sqrt_core(x1) - 3.0f;
    if (__builtin_fmaf(rs, CULL_REL_LO, -(CULL_ABS + R_BLEND_LO)) <= U)
      d4 = sd_blend(o, xs, blend, omblend);
    if (ball_needs(xtc, U, R_TORUS)) d5 = sd_torus(o, tz);
    if (ball_needs(xk, U, R_CAPSULE)) d6 = sd_capsule(o, p);
    float d = d0;
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
    return d;
  }
  float m = d7;  // running minimum over the plane and the evaluated primitives
  if (PLANE_U) {
    // U = the plane alone and every cull test squared (ball_needs): no v_sqrt at
    // all.  The shadow march starts 0.02 above the floor, where the plane is the
    // tightest bound anyway; the spheres' bounds in U cost three transcendentals
    // per step for the few steps they tighten (round 3: -1.3 % per cfg3 frame,
    // DESIGN.md §4.4 item 13 f).
    if (ball_needs(x0, d7, 3.0f)) m = vmin(m, sqrt_core(x0) - 3.0f);
    if (ball_needs(x1, d7, 3.0f)) m = vmin(m, sqrt_core(x1) - 3.0f);
    if (ball_needs(xs, d7, R_BLEND_LO)) m = vmin(m, sd_blend(o, xs, blend, omblend));
    if (ball_needs(xtc, d7, R_TORUS)) m = vmin(m, sd_torus(o, tz));
    if (ball_needs(xk, d7, R_CAPSULE)) m = vmin(m, sd_capsule(o, p));
    return m;
  }
  if (__builtin_fmaf(r0, CULL_REL_LO, -(CULL_ABS + 3.0f)) <= U) {
    m = vmin(m, sqrt_core(x0) - 3.0f);
  }
  if (__builtin_fmaf(r1, CULL_REL_LO, -(CULL_ABS + 3.0f)) <= U) {
    m = vmin(m, sqrt_core(x1) - 3.0f);
  }
  if (__builtin_fmaf(rs, CULL_REL_LO, -(CULL_ABS + R_BLEND_LO)) <= U) {
    m = vmin(m, sd_blend(o, xs, blend, omblend));
  }
  if (ball_needs(xtc, U, R_TORUS)) {
    m = vmin(m, sd_torus(o, tz));
  }
  if (ball_needs(xk, U, R_CAPSULE)) {
    m = vmin(m, sd_capsule(o, p));
  }
  return m;
}

// ---- GetNormal's samples with shared culling (glsl:278-288) --------------------------
// sdf at pos and at pos + 0.001 e_x/e_y/e_z.  The four points lie within
// e = 0.001 + 2^-22 (|pos|_1 + 1) of pos (the float adds round), so by the
// 1-Lipschitz property one set of bounds at pos culls primitive k at all four:
//   LB_k(p') >= LB_k(pos) - e,   U(p') <= U(pos) + e   =>   cull if LB_k(pos) - 2e > U(pos).
// The survivors are evaluated exactly at each point (the same float ops as
// scene_exact), so every value is the exact float minimum.  With HAVE_C0 the
// centre value is the march's last distance at this very point (render's
// pos == the march's final q, glsl:226 vs :129): only three points remain.
__device__ __forceinline__ float ev_sph0(f3 p) {
  const Offs o = offsets(p);
  return sqrt_core((o.ax * o.ax + o.ay2) + o.az2) - 3.0f;
}
__device__ __forceinline__ float ev_sph1(f3 p) {
  const Offs o = offsets(p);
  return sqrt_core((o.bx * o.bx + o.ay2) + o.az2) - 3.0f;
}
__device__ __forceinline__ float ev_blend(f3 p, float blend, float omblend) {
  const Offs o = offsets(p);
  return sd_blend(o, (o.cx2 + o.ay2) + o.az2, blend, omblend);
}
__device__ __forceinline__ float ev_torus(f3 p) { return sd_torus(offsets(p), p.z - 10.0f); }
__device__ __forceinline__ float ev_capsule(f3 p) { return sd_capsule(offsets(p), p); }

template <bool HAVE_C0>
__device__ __forceinline__ void normal_samples(f3 pos, float blend, float omblend, float& c0,
                                               float& vx, float& vy, float& vz) {
  const f3 px = add(pos, mk(0.001f, 0.0f, 0.0f));
  const f3 py = add(pos, mk(0.0f, 0.001f, 0.0f));
  const f3 pz = add(pos, mk(0.0f, 0.0f, 0.001f));
  const Offs o = offsets(pos);
  const float tz = pos.z - 10.0f;
  const float kx = pos.x - CAP_MX, ky = pos.y - CAP_MY, kz = pos.z - CAP_MZ;
  const float r0 = __builtin_amdgcn_sqrtf((o.ax * o.ax + o.ay2) + o.az2);
  const float r1 = __builtin_amdgcn_sqrtf((o.bx * o.bx + o.ay2) + o.az2);
  const float rs = __builtin_amdgcn_sqrtf((o.cx2 + o.ay2) + o.az2);
  const float xt = (o.cx2 + o.ay2) + tz * tz;
  const float xk = (kx * kx + ky * ky) + kz * kz;
  const float e2 = 2.0f * (0.001f + 0x1p-22f * (((fabsf(pos.x) + fabsf(pos.y)) + fabsf(pos.z)) + 1.0f));
  float U = vmin(pos.y + 5.5f, __builtin_fmaf(r0, CULL_REL_HI, CULL_ABS - 3.0f));
  U = vmin3(U, __builtin_fmaf(r1, CULL_REL_HI, CULL_ABS - 3.0f),
            __builtin_fmaf(rs, CULL_REL_HI, CULL_ABS - 2.5f));
  U = U + e2;  // U(pos) + e, compared with LB(pos) - e; 2e absorbs the add's rounding
  float mc = pos.y + 5.5f, mx = px.y + 5.5f, my = py.y + 5.5f, mz = pz.y + 5.5f;
  if (__builtin_fmaf(r0, CULL_REL_LO, -(CULL_ABS + 3.0f)) <= U) {
    if (!HAVE_C0) mc = vmin(mc, ev_sph0(pos));
    mx = vmin(mx, ev_sph0(px));
    my = vmin(my, ev_sph0(py));
    mz = vmin(mz, ev_sph0(pz));
  }
  if (__builtin_fmaf(r1, CULL_REL_LO, -(CULL_ABS + 3.0f)) <= U) {
    if (!HAVE_C0) mc = vmin(mc, ev_sph1(pos));
    mx = vmin(mx, ev_sph1(px));
    my = vmin(my, ev_sph1(py));
    mz = vmin(mz, ev_sph1(pz));
  }
  if (__builtin_fmaf(rs, CULL_REL_LO, -(CULL_ABS + R_BLEND_LO)) <= U) {
    if (!HAVE_C0) mc = vmin(mc, ev_blend(pos, blend, omblend));
    mx = vmin(mx, ev_blend(px, blend, omblend));
    my = vmin(my, ev_blend(py, blend, omblend));
    mz = vmin(mz, ev_blend(pz, blend, omblend));
  }
  if (ball_needs(xt, U, R_TORUS)) {
    if (!HAVE_C0) mc = vmin(mc, ev_torus(pos));
    mx = vmin(mx, ev_torus(px));
    my = vmin(my, ev_torus(py));
    mz = vmin(mz, ev_torus(pz));
  }
  if (ball_needs(xk, U, R_CAPSULE)) {
    if (!HAVE_C0) mc = vmin(mc, ev_capsule(pos));
    mx = vmin(mx, ev_capsule(px));
    my = vmin(my, ev_capsule(py));
    mz = vmin(mz, ev_capsule(pz));
  }
  if (!HAVE_C0) c0 = mc;
  vx = mx;
  vy = my;
  vz = mz;
}

// ---- lazy culling along a ray ------------------------------------------------------
// For a march p(t) = ro + rd*t.  Primitive k is skipped while t < te[k].  When k
// is re-tested at p_i (t_i) with U_i >= min(p_i) and LB_k(p_i) > U_i, then for
// any later point p_j of the ray, by the 1-Lipschitz property of distances,
//   sdf_k(p_j) - min(p_j) >= (LB_k - U_i) - 2 |p_j - p_i|,   |p_j - p_i| ~ |rd| (t_j - t_i),
// so k stays strictly above the minimum while
//   t_j < te_k = t_i + (LB_k - U_i - slack) / (2 |rd|) * (1 - 2^-10).
// `slack` covers the float error of the evaluated sdfs and of p(t) itself:
// relative 2^-14 of |ro|_1 + |rd| t + 64 (the actual errors are ~2^-21).
// U_i = min(plane, exact values of this step's evaluated primitives).  A
// primitive whose bound does not cull it is evaluated exactly and re-tested at
// the next step.  The distance returned is the running minimum.
// Second, often longer budget: the plane distance is linear along the ray,
// plane(p_j) = plane(p_i) + rd.y (t_j - t_i), and min(p_j) <= plane(p_j), so k
// also stays above the minimum while
//   t_j < t_i + (LB_k - plane(p_i) - slack) / (|rd| + rd.y) * (1 - 2^-10)
// (|rd| + rd.y >= 0; level and downward rays get 2x and more).  Any valid
// expiry will do, and the later of several is valid too.  Step 0 of a primary
// ray (host gaps, PREP_G / PREP_H) takes the later of both; the block's
// re-tests take the plane budget alone (round 4): where U_i is the plane, the
// plane budget is the longer one (1 / (|rd| + rd.y) >= 1 / (2 |rd|)), and
// forming the first costs two subtractions and an fma per re-test, more than
// the re-tests it saves where a primitive is nearer than the plane (cfg3
// -1.1 %, cfg2 -2.8 % per frame, tools/patches/plane_budget_only.diff A/B).
struct LazyCull {
  float te[5];   // expiry t of spheres 0/1, blend, torus, capsule
  float temin;   // min over te[]
  float tegrp;   // min over te[] but the torus's: one compare for four primitives
  float s0, s1;  // slack(t) = s0 + s1 t >= 2^-14 (|ro|_1 + |rd| t + 64)  (rounded up)
  float inv2v;   // (1 - 2^-10) / (2 |rd|)  (rounded down)
  float invp;    // (1 - 2^-10) / (|rd| + rd.y)  (rounded down)
  int idb;       // the opU id among the primitives the last block evaluated (7: none taken)
};

// Step 0 of every primary ray is the same computation: castRay starts all of
// them at the camera (glsl:68-74) and p(0) = ro + rd*0 = ro exactly.  The host
// forms it once per frame (rm_api.hip prep_host, the same IEEE operations; the
// bounds only need to be valid, and the IEEE sqrt is within the 2^-12 margins
// made for v_sqrt) and passes these values by value in Frame::prepv, so the
// render kernel's prologue has no dependent load:
enum PrepSlot : int {
  PREP_VALID = 0,   // 1 when 0 < d0 <= 400 (no hit or escape at step 0)
  PREP_D0 = 1,      // sdf(camera), the step-0 distance (exact, same ops as scene_lazy)
  PREP_SLACK = 2,   // ray_s0(camera): slack(0) of scene_lazy at the camera
  PREP_G = 3,       // 5 gaps g_k = (LB_k - d0) - slack of the step-0 re-test (LB_k as
                    // scene_lazy's re-test forms it), or -inf when g_k <= 0 (no budget)
  PREP_H = 8,       // 5 plane gaps LB_k - (plane(camera) + slack), or -inf when g_k <= 0
  PREP_B1 = 13,     // lin_exit_b(camera, slack, 0): the miss exit's ro-dependent terms
  PREP_B2 = 14,
  PREP_B3 = 15,     // lin_exit_b3(camera, slack, 0): the object slab's intercept
  PREP_COUNT = 16
};
// Per-ray constants shared by the lazy culler and the linear exits: |rd| from
// one v_sqrt (within 1.5 ulp) and the slack line s0 + s1 t, rounded up with
// 2^-12 margins: s0 >= 2^-14 (|ro|_1 + 64), s1 >= 2^-14 |rd|.
__device__ __forceinline__ float ray_rdl(f3 rd) { return __builtin_amdgcn_sqrtf(dot(rd, rd)); }
__device__ __forceinline__ float ray_s0(f3 ro) {
  const float HI = 1.0f + 0x1p-12f;
  return 0x1p-14f * (((fabsf(ro.x) + fabsf(ro.y)) + fabsf(ro.z)) * HI + 64.0f) * HI;
}
__device__ __forceinline__ float ray_s1(float rdl) {
  const float HI = 1.0f + 0x1p-12f;
  return 0x1p-14f * rdl * (HI * HI);
}

__device__ __forceinline__ void lazy_init(LazyCull& c, f3 rd, float rdl, float s0, float s1) {
  const float NEG = -__builtin_huge_valf();
#pragma unroll
  for (int k = 0; k < 5; ++k) c.te[k] = NEG;
  c.temin = NEG;
  c.tegrp = NEG;
  const float rdlen = rdl * (1.0f + 0x1p-16f);  // >= |rd|
  c.inv2v = (0.5f * (1.0f - 0x1p-10f)) * __builtin_amdgcn_rcpf(rdlen) * (1.0f - 0x1p-16f);
  // rdlen over-estimates |rd| by >= 2^-17 |rd|, so the rounded sum is above
  // the true |rd| + rd.y even under cancellation; its reciprocal may be large.
  c.invp = (1.0f - 0x1p-10f) * __builtin_amdgcn_rcpf(rdlen + rd.y) * (1.0f - 0x1p-16f);
  c.s0 = s0;
  c.s1 = s1;
  c.idb = 7;
}

// lazy_init for |rd| within 2^-20 of 1 (Frame::unit_rd): rdlen = 1 + 2^-16 >= |rd|
// (over by >= 2^-17 |rd|), so inv2v is the constant (1/2)(1 - 2^-10)/(1 + 2^-16)
// rounded down (the rcp form's (1 - 2^-16) factor covered its 1 ulp).
__device__ __forceinline__ void lazy_init_unit(LazyCull& c, f3 rd, float s0, float s1) {
  const float NEG = -__builtin_huge_valf();
#pragma unroll
  for (int k = 0; k < 5; ++k) c.te[k] = NEG;
  c.temin = NEG;
  c.tegrp = NEG;
  constexpr float RDLEN = 1.0f + 0x1p-16f;
  c.inv2v = 0x1.ff7ep-2f;  // 0.5 (1 - 2^-10) / (1 + 2^-16) = 0.499504097 rounded down
  c.invp = (1.0f - 0x1p-10f) * __builtin_amdgcn_rcpf(RDLEN + rd.y) * (1.0f - 0x1p-16f);
  c.s0 = s0;
  c.s1 = s1;
  c.idb = 7;
}

// The block and each re-test are entered per wave (any lane expired) and every
// active lane re-tests: lanes whose te has not expired keep max(te, new te) --
// both expiries are valid -- so the idle lanes of a divergent re-test extend
// their budgets for free.
// The opU id of the minimum (glsl:105,110-121), as scene_exact<true> gives it,
// is lazy_id(): the primitives are taken in the reference's order with ties
// going to the later one, the plane last; culled primitives are strictly above
// the minimum and can neither win nor tie.  A step that skips the block has
// only the plane left: id 7.  The block records its primitives' winner (idb);
// the plane, last in the chain, wins a tie with it.  So at the hit step, whose
// distance d is not NaN (d < 1e-6 t), the id is 7 exactly when d equals the
// step's plane value: a step that skipped the block returns the plane value
// itself, and a step that entered it returns the plane value only when no
// primitive is strictly below it.  Otherwise the block ran at this very step
// and idb is its winner.  lazy_id re-forms the plane value with the same
// operations once per hit, where the block used to record the step's t and
// compare and select at every entry (round 4: ~2.5 issue slots per entry, 13
// entries per wave).
// The point is p = ro + rd t (the march's q); only p.y is needed outside the
// re-test block, so p.x / p.z are formed inside it.
__device__ __forceinline__ float scene_lazy(f3 ro, f3 rd, float t, LazyCull& lc, float blend,
                                            float omblend) {
  const float py = ro.y + rd.y * t;
  float m = py + 5.5f;  // plane, exact (glsl:85,121); running minimum
  RM_STAT(8);
  if (__any(t >= lc.temin)) {
    int idp = 7;

    RM_STAT(9);
    const float slack = __builtin_fmaf(lc.s1, t, lc.s0);
    const float invp = lc.invp;
    const float pl = m + slack;  // plane(p_i) + slack
    // The opU id among the evaluated primitives, later wins ties, compared with
    // the running minimum m (plane included) rather than a separate minimum over
    // the primitives: a primitive above the plane is never taken, which only
    // matters when the plane wins (m == plane below: id 7); otherwise the winner
    // v* < plane is <= every m before it and every later tie is taken, as with a
    // primitives-only minimum.  One v_min per evaluation fewer (round 3).
    auto take = [&](float v, int k) {
      idp = (v <= m) ? k : idp;
      m = vmin(m, v);
    };
    // re-test k; returns true when k must be evaluated exactly at this step
    auto retest = [&](float x, float R, float& te, int k) -> bool {
      RM_STAT(1);
      RM_STAT(16 + k);
      const float lb = __builtin_fmaf(__builtin_amdgcn_sqrtf(x), CULL_REL_LO, -(CULL_ABS + R));
      // The new expiry is the later of the old one and the plane budget's end;
      // both are valid, so their max is.  A gap lb - pl <= 0 ends the budget at
      // or before t, leaving an expired lane with te <= t: evaluated now and
      // re-tested at its next step, whatever the exact value below t.  An idle
      // lane keeps its te > t.  The fma rounds once instead of twice (t + g b
      // rather than t + RN(g b)), inside the budget's 2^-10 margin.  The float
      // max (a te below t may be negative) without t among its operands: a te
      // below t is as expired as te = t (round 3).
      te = vmax(__builtin_fmaf(lb - pl, invp, t), te);
      // Evaluate exactly when the new expiry does not pass t: an expired lane
      // whose gap is <= 0, and also one whose tiny gap > 0 cannot move t -- an
      // extra exact evaluation, never a wrong skip.  One compare instead of two
      // (`expired & !(g > 0)`, round 3).
      return te <= t;
    };
    const f3 p = mk(ro.x + rd.x * t, py, ro.z + rd.z * t);
    const Offs o = offsets(p);
    // One wave vote for the four primitives other than the torus, which takes
    // half of the re-tests (cfg3 frame 60: 10 of 21 per wave): a block entered
    // for the torus alone then costs one compare instead of four (round 3,
    // VALU issue slots: -1.0 % cfg3, -2.0 % cfg2 per frame).  Evaluation order,
    // hence opU's tie rule, is unchanged.
    const bool GRP = __any(t >= lc.tegrp);
    if (GRP && __any(t >= lc.te[0])) {  // sphere (15,0,-10) r3, glsl:111
      const float x0 = (o.ax * o.ax + o.ay2) + o.az2;
      if (retest(x0, 3.0f, lc.te[0], 0)) {
        RM_STAT(10);
        take(sqrt_core(x0) - 3.0f, 0);
      }
    }
    if (GRP && __any(t >= lc.te[1])) {  // sphere (-25,0,-10) r3, glsl:112
      const float x1 = (o.bx * o.bx + o.ay2) + o.az2;
      if (retest(x1, 3.0f, lc.te[1], 1)) {
        RM_STAT(11);
        take(sqrt_core(x1) - 3.0f, 1);
      }
    }
    if (GRP && __any(t >= lc.te[2])) {  // box/sphere blend, glsl:115-117
      const float xs = (o.cx2 + o.ay2) + o.az2;
      if (retest(xs, R_BLEND_LO, lc.te[2], 2)) {
        RM_STAT(12);
        take(sd_blend(o, xs, blend, omblend), 4);
      }
    }
    if (__any(t >= lc.te[3])) {  // torus, glsl:119
      // Evaluated exactly instead of re-tested against its ball (round 5): most
      // torus re-tests ended in the evaluation anyway (6.55 of 8.0 per wave, cfg3
      // frame 60), so the ball's v_sqrt and compare were extra work.  The exact
      // value serves as the budget's lower bound (its float error is far inside
      // the slack), and taking it for a lane that did not need it is what the
      // reference's opU does (it evaluates everything).  -2.9 % per cfg3 frame
      // (with the tegrp change below; profiles/r05_ab_tegrp_torus.txt).
      RM_STAT(1);
      RM_STAT(16 + 3);
      RM_STAT(13);
      const float tz = p.z - 10.0f;
      const float v = sd_torus(o, tz);
      take(v, 5);
      lc.te[3] = vmax(__builtin_fmaf(v - pl, invp, t), lc.te[3]);
    }
    if (GRP && __any(t >= lc.te[4])) {  // capsule, glsl:120
      const float kx = p.x - CAP_MX, ky = p.y - CAP_MY, kz = p.z - CAP_MZ;
      if (retest((kx * kx + ky * ky) + kz * kz, R_CAPSULE, lc.te[4], 4)) {
        RM_STAT(14);
        take(sd_capsule(o, p), 6);
      }
    }
    // a block entered for the torus alone changed no other expiry: tegrp stands
    // (two v_min fewer, wave-uniform branch)
    if (GRP) lc.tegrp = vmin(vmin3(lc.te[0], lc.te[1], lc.te[2]), lc.te[4]);
    lc.temin = vmin(lc.tegrp, lc.te[3]);
    lc.idb = idp;  // (the plane's tie rule and the step: lazy_id)
  }
  return m;
}
// The hit's id: the block's winner unless the hit step's distance d is its
// plane value (ro.y + rd.y t) + 5.5, formed as scene_lazy forms it (above).
__device__ __forceinline__ int lazy_id(const LazyCull& lc, float t, float d, float roy, float rdy) {
  const float plane = (roy + rdy * t) + 5.5f;
  return d != plane ? lc.idb : 7;
}

// ---- provable early exits (softshadow, misses) ---------------------------------------
// With C, R_ALL a sphere enclosing all five bounded primitives and
// slack(t) = s0 + s1 t the float-error bound of the lazy culler, every float
// scene value at p(t) = ro + rd t obeys
//   h(t) >= min(|rd| t - |ro - C| - R_ALL,  ro.y + 5.5 + rd.y t) - slack(t).
// Both lower bounds are linear in t.  If at t_j both stay above
// max(hmin, c t) for every t >= t_j, every later step of a march along the ray
// sees h > hmin and h / t > c:
//   * softshadow (glsl:201-216; rd = light - pos unnormalised, so t passes the
//     light after 3-4 steps): hmin = 0.001, c = (1 + 2^-9) / k: no later step
//     returns 0.05 and every later k h / t rounds above 1 >= res, so the result
//     is `res` now (16 steps otherwise);
//   * RayMarch / reflectedRay (glsl:125-161): hmin = 0, c = 1e-6 (1 + 2^-9): no
//     later step hits (d < 1e-6 t), so the march ends in a miss whatever the
//     number of steps to d > tmax or the step cap -- and a miss discards t.
// The two linear conditions are
//   a1 t - b1 > 0,  a1 = |rd|lo - s1 - c,       b1 = |ro - C|hi + R_ALL + s0 + hmin
//   a2 t + b2 > 0,  a2 = rd.y - s1 - c (> 0),   b2 = ro.y + 5.5 - s0 - hmin
// (the second covers the plane's ratio both for b2 + hmin >= 0, where a2 > 0 is
// enough, and for b2 < 0, where its inf over t >= t_j is at t_j).  Coefficients
// are rounded toward failure by 2^-12 relative plus 2^-20 absolute.  Both hold
// for t > T = max(b1 / a1, -b2 / a2) (+inf unless a1, a2 > 0); T is rounded up
// (v_rcp_f32 is within 1 ulp; the 2^-20 factor covers it and the two products),
// so the per-step test is one compare, t > T.
constexpr float SH_CX = -5.0f, SH_CY = 0.0f, SH_CZ = -10.0f;
constexpr float SH_RALL = 23.001f;  // >= max_k |C - c_k| + R_k = 20 + 3 (spheres, torus)
// The ro-dependent half (b1, b2): uniform for primary rays, so k_prep forms it
// once per frame (PREP_B1/B2); the rd-dependent half gives T per ray.
__device__ __forceinline__ void lin_exit_b(f3 ro, float s0, float hmin, float& b1, float& b2) {
  const float HI = 1.0f + 0x1p-12f;
  const float ex = ro.x - SH_CX, ey = ro.y - SH_CY, ez = ro.z - SH_CZ;
  const float rc = __builtin_fmaf(__builtin_amdgcn_sqrtf((ex * ex + ey * ey) + ez * ez), HI, 0x1p-18f);
  b1 = (rc + SH_RALL + s0 + hmin) * HI;
  b2 = ((ro.y + 5.5f) - s0 - hmin * HI) - 0x1p-19f * (fabsf(ro.y) + 5.5f + hmin + s0);
}
constexpr float SH_YTOP = 3.001f;  // >= the top of every bounded primitive (below)
// Two more lower bounds of the five objects (round 5), each linear in t like the
// ball's, so either one holding from t_j on proves the objects term as well:
//   * the slab below SH_YTOP, which holds every bounded primitive (each reaches
//     y = 3 and no higher: the spheres, the blend's sphere over its box, the
//     torus ring in its vertical plane, the capsule's end (-3, 2, -28) + 1):
//     objects >= p.y - SH_YTOP - err, so with the plane's slope a2
//       a2 t - b3 > 0,  b3 = SH_YTOP + s0 + hmin - ro.y   (rounded up),
//     T3 = b3 / a2: an upward ray is past every object once above the slab;
//   * the ball seen along the ray: |p(t) - C| >= |rd| t + u with
//     u = rd.(ro - C) / |rd| (|p - C|^2 = (|rd| t + u)^2 + |ro - C|^2 - u^2),
//     so b1 may take -u (rounded down) for |ro - C|: a ray leaving the ball is
//     past it at once, where the triangle inequality waits for |rd| t > |ro - C|
//     + R_ALL.  (The step-cap exit keeps the plain b1.)
// A blend of box and sphere (weights in [0, 1] summing to 1) is above the lower
// of the two, so both bounds cover it as the ball does.
__device__ __forceinline__ float lin_exit_b3(float roy, float s0, float hmin) {
  return ((SH_YTOP - roy) + s0 + hmin * (1.0f + 0x1p-12f)) +
         0x1p-19f * (fabsf(roy) + SH_YTOP + hmin + s0);
}
// b1 from the projection, rounded up: every rounding of e, the dot product and
// the 1 / |rd| scaling is within 2^-17 |ro - C|_1 (|u| <= |ro - C|), and the
// sum's within 2^-17 of its terms.  invl: 1 / |rd| within 2^-20 (1 for unit rays).
__device__ __forceinline__ float lin_exit_b1p(f3 ro, f3 rd, float invl, float s0, float hmin) {
  const float ex = ro.x - SH_CX, ey = ro.y - SH_CY, ez = ro.z - SH_CZ;
  const float u = ((rd.x * ex + rd.y * ey) + rd.z * ez) * invl;
  const float e1 = (fabsf(ex) + fabsf(ey)) + fabsf(ez);
  const float k = (SH_RALL + s0) + hmin;
  return (k - u) + 0x1p-17f * (e1 + k);
}
__device__ __forceinline__ float lin_exit_T(float c, float rdl, float rdy, float s1, float b1, float b2,
                                            float b3 = __builtin_huge_valf()) {
  const float LO = 1.0f - 0x1p-12f;
  // absolute 2^-20 terms: the rounding of a difference is relative to its
  // operands, not to a small (cancelled) result
  const float a1 = (rdl * LO - s1 - c) * LO - 0x1p-20f * (rdl + c);
  const float a2 = (rdy - s1 - c) * LO - 0x1p-20f * (fabsf(rdy) + s1 + c);
  const float UP = 1.0f + 0x1p-20f, DN = 1.0f - 0x1p-20f;
  const float INF = __builtin_huge_valf();
  // b1 may be negative (the projection): T1 rounded up either way
  const float T1 = b1 * __builtin_amdgcn_rcpf(a1) * (b1 >= 0.0f ? UP : DN);
  const float r2 = __builtin_amdgcn_rcpf(a2);
  const float T2 = -(b2 * r2 * (b2 >= 0.0f ? DN : UP));
  const float T3 = b3 * r2 * (b3 >= 0.0f ? UP : DN);  // +inf for b3 = +inf
  const float Tobj = a1 > 0.0f ? __builtin_fminf(T1, T3) : T3;
  return a2 > 0.0f ? __builtin_fmaxf(Tobj, T2) : INF;
}
constexpr float MISS_C = 0.000001f * (1.0f + 0x1p-9f);
__device__ __forceinline__ float lin_exit_init(float c, float hmin, f3 ro, f3 rd, float rdl) {
  const float s0 = ray_s0(ro);
  float b1, b2, b3;
  lin_exit_b(ro, s0, hmin, b1, b2);
  // the slab, not the projection: shadow rays rise from the floor toward the light,
  // and the projection's ~8 VALU per call saved nothing (cfg3 -0.6 % without it,
  // profiles/r05_ab_shadow_noproj.txt)
  b3 = lin_exit_b3(ro.y, s0, hmin);
  return lin_exit_T(c, rdl, rd.y, ray_s1(rdl), b1, b2, b3);
}
// c = Frame::shc, (1 + 2^-9) / k (1 + 2^-12) (0 for k = +inf): the host forms it
// with the same float operations once per frame (rm_api.hip make_frame), where
// the device would have spent a full IEEE division (~14 VALU) per shadow call
// site and wave on a uniform value.
// rdl: |rd| within 1.5 ulp.  A shadow ray's rd is light - pos, whose exact
// length the light term at the same pos has already formed (point_light's
// `distance`, correctly rounded): the caller passes it instead of a v_sqrt
// (round 4).
// lpos_in_ball: the light lies within the objects' ball (|light - C| <= R_ALL; a
// uniform of the frame, so a wave-uniform branch).  Then every shadow ray has
// |rd| = |light - ro| <= |ro - C| + R_ALL, and the ball's bound holds only past
// t = 1, the light: the exit takes the plane and the object slab alone, without
// the ball's v_sqrt and v_rcp (cfg3 -0.8 % per frame, the sweep's light at
// (-5, 5, -10); profiles/r05_ab_shadow_slab.txt).
__device__ __forceinline__ float shadow_exit_init(float c, f3 ro, f3 rd, float rdl, bool lpos_in_ball) {
  if (!lpos_in_ball) return lin_exit_init(c, 0.001f, ro, rd, rdl);
  const float s0 = ray_s0(ro), s1 = ray_s1(rdl), hmin = 0.001f;
  const float b2 = ((ro.y + 5.5f) - s0 - hmin * (1.0f + 0x1p-12f)) - 0x1p-19f * (fabsf(ro.y) + 5.5f + hmin + s0);
  const float b3 = lin_exit_b3(ro.y, s0, hmin);
  const float a2 = (rd.y - s1 - c) * (1.0f - 0x1p-12f) - 0x1p-20f * (fabsf(rd.y) + s1 + c);
  const float UP = 1.0f + 0x1p-20f, DN = 1.0f - 0x1p-20f;
  const float r2 = __builtin_amdgcn_rcpf(a2);
  const float T2 = -(b2 * r2 * (b2 >= 0.0f ? DN : UP));
  const float T3 = b3 * r2 * (b3 >= 0.0f ? UP : DN);
  return a2 > 0.0f ? __builtin_fmaxf(T3, T2) : __builtin_huge_valf();
}
// |light - C| <= R_ALL (rounded toward "outside": a light at the boundary keeps the ball)
__device__ __forceinline__ bool light_in_ball(const Frame& F) {
  const float ex = F.lpos[0] - SH_CX, ey = F.lpos[1] - SH_CY, ez = F.lpos[2] - SH_CZ;
  return (ex * ex + ey * ey) + ez * ez <= SH_RALL * SH_RALL * (1.0f - 0x1p-10f);
}
__device__ __forceinline__ float miss_exit_init(f3 ro, f3 rd) { return lin_exit_init(MISS_C, 0.0f, ro, rd, ray_rdl(rd)); }
__device__ __forceinline__ bool lin_exit(float T, float t) { return t > T; }

// ---- step-cap miss exit (RayMarch / reflectedRay, glsl:125-161) ---------------
// A march that spends its nmax steps without a hit is a miss (glsl:141,160), as
// is an escape; a miss discards t.  Downward rays grazing the floor toward the
// horizon approach the plane geometrically and many reach the cap: with every
// object provably above the hit threshold, the plane distance P(t) = ro.y + 5.5
// + rd.y t (exact real; rd.y < 0, q = 1 + rd.y in (0.5, 1)) shrinks by at most
// the factor q per step.  Let u = 2^-24 and, for a ray above the floor (P0 =
// ro.y + 5.5 > 0), Tb >= P0 / |rd.y| + slack the largest t reached while P > 0.
//   * the computed plane h = RN(RN(RN(rd.y t) + ro.y) + 5.5) is within
//     E1 = 2^-21 (|ro.y| + 5.5) >= 5u (|ro.y| + 5.5)(1 + u) of P(t), t <= Tb;
//   * a step moves t by  RN(t + d) - t <= d + u Tb <= h + u Tb  (d = min(h,
//     objects) <= h), so  P' >= P - |rd.y| (P + E1 + u Tb) = q P - |rd.y| E2,
//     E2 = E1 + 2u Tb, and over k steps (|rd.y| sum q^j <= 1)  P_k >= q^k P - E2;
//   * a hit needs d < RN(1e-6 t) <= thr = 1e-6 Tb (1 + 2^-20); objects are above
//     MISS_C t > thr once t > T1 (lin_exit_T1), so a hit needs h < thr, i.e.
//     P < thr + E1;
//   * P_n >= d_n - E1 at the current step (its hit test failed).
// Hence, at step i with K = nmax - i evaluations left and t > T1, if
//   (d - E1) q^K >= A = (thr + E1 + E2)(1 + 2^-10)
// then P stays above thr + E1 > 0 (so t < Tb, closing the induction) on every
// remaining step: no step hits and the march ends in a miss.  q^K is bounded
// below with v_log / v_exp and relative (2^-12) plus absolute (2^-20 in the
// exponent) margins far above their errors; NaNs fail the compare (no exit).
// Only rays with -0.05 < rd.y < 0 can pass (q^K |rd.y| >= 1e-6 needs it for K
// >= 240), so the check runs behind that wave-uniform test.
__device__ __forceinline__ float lin_exit_T1(float c, float rdl, float s1, float b1) {
  const float LO = 1.0f - 0x1p-12f;
  const float a1 = (rdl * LO - s1 - c) * LO - 0x1p-20f * (rdl + c);
  const float T1 = b1 * __builtin_amdgcn_rcpf(a1) * (1.0f + 0x1p-20f);
  return a1 > 0.0f ? T1 : __builtin_huge_valf();
}
__device__ __forceinline__ bool cap_miss(float t, float d, int K, float roy, float rdy, float T1) {
  const float P0 = (roy + 5.5f) * (1.0f + 0x1p-22f);  // >= ro.y + 5.5 when that is > 0
  const float nr = -rdy;
  const float Tb = __builtin_fmaf(P0 * __builtin_amdgcn_rcpf(nr), 1.0f + 0x1p-20f, 0x1p-10f);
  const float E1 = 0x1p-21f * (fabsf(roy) + 5.5f);
  const float E2 = __builtin_fmaf(0x1p-23f, Tb, E1);
  const float A = ((0.000001f * (1.0f + 0x1p-20f)) * Tb + E1 + E2) * (1.0f + 0x1p-10f);
  const float q = (1.0f + rdy) - 0x1p-23f;  // < 1 + rd.y
  const float L = __builtin_fmaf(__builtin_amdgcn_logf(q), 1.0f + 0x1p-12f, -0x1p-20f);  // < log2 q
  const float qK = __builtin_amdgcn_exp2f((float)K * L) * (1.0f - 0x1p-12f);          // < q^K
  return (rdy < 0.0f) & (rdy > -0.5f) & (P0 > 0.0f) & (t > T1) & ((d - E1) * qK >= A);
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

// GLSL int(float) (glsl:79): truncation; a value outside the int range, which
// GLSL leaves undefined, saturates and NaN gives 0: the
// v_cvt_i32_f32 conversion itself, written out so that no compiler may assume
// the C++ cast's undefined range away.
__device__ __forceinline__ int glsl_int(float x) {
  int r;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// checkers(p) glsl:77-80
__device__ __forceinline__ float checkers(f3 p) {
  int a = glsl_int(1000.0f + p.x) % 2;
  int b = glsl_int(1000.0f + p.z) % 2;
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

// pow(x, y) for x >= 0, y > 0, as GLSL specifies its precision: exp2(y * log2(x))
// (GLSL 4.50 §8.2; the GL drivers the reference runs on evaluate it this way),
// on the hardware transcendentals v_log_f32 / v_exp_f32.  pow(0, y) = 0.  Its
// difference to a correctly rounded pow is a few float ulps (measured in
// tests/test_gpu_parity.py, tools/pow_error.py).
__device__ __forceinline__ float gpow(float x, float y) {
  return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}

// getPointLight glsl:253-276
// dist_out: length(light - pos), the shadow ray's |rd| (shadow_exit_init).
__device__ __forceinline__ f3 point_light(const Frame& F, f3 color, f3 normal, f3 pos, float* dist_out = nullptr) {
  f3 lpos = mk(F.lpos[0], F.lpos[1], F.lpos[2]);
  f3 ambient = mk(F.lamb[0], F.lamb[1], F.lamb[2]);
  f3 viewDir = normalize(sub(pos, mk(F.cam_pos[0], F.cam_pos[1], F.cam_pos[2])));
  f3 lightDir = normalize(sub(lpos, pos));
  float NtoL = gmax(dot(normal, lightDir), 0.0f);
  f3 diffuse = muls(mk(F.ldif[0], F.ldif[1], F.ldif[2]), NtoL);
  f3 reflectDir = reflect(lightDir, normal);
  float spec = gpow(gmax(dot(viewDir, reflectDir), 0.0f), 32.0f);
  f3 specular = muls(mk(F.lspec[0], F.lspec[1], F.lspec[2]), spec);
  float distance = len(sub(lpos, pos));
  if (dist_out) *dist_out = distance;
  float attenuation = rcp_exact((F.lconst + F.llin * distance) + F.lquad * (distance * distance));
  diffuse = muls(diffuse, attenuation);
  ambient = muls(ambient, attenuation);
  specular = muls(specular, attenuation);
  return mul(color, add(add(diffuse, ambient), specular));
}

__device__ __forceinline__ f3 gamma(f3 c) {
  return mk(gpow(c.x, 0.4545f), gpow(c.y, 0.4545f), gpow(c.z, 0.4545f));
}

// uv of pixel column (axis 0) / row (axis 1) p, sample s (-1: no supersampling):
// glsl:301-305 and the cumulative sub-sample offsets of :309-332.  With
// F.uv_exact the host has checked, for every p of this frame size, that the
// fma-corrected product below equals the IEEE division (2p - n) / n
// (rm_api.hip uv_exact_check); otherwise the host-built table is read.
__device__ __forceinline__ float lane_uv(const Frame& F, int axis, int p, int s) {
#ifdef RM_UV_COMPUTE
  if (F.uv_exact) {
    const float a = (float)(2 * p - (axis ? F.height : F.width));
    const float r = F.uv_rcp[axis], n = F.uv_dims[axis];
    const float q0 = a * r;
    float v = __builtin_fmaf(__builtin_fmaf(-q0, n, a), r, q0);
    if (s >= 0) {
      const float v1 = v + F.uv_off[axis][0], v2 = v1 + F.uv_off[axis][1], v3 = v2 + F.uv_off[axis][2];
      const float v4 = v3 + F.uv_off[axis][3];
      v = s == 0 ? v1 : s == 1 ? v2 : s == 2 ? v3 : v4;
    }
    return v;
  }
#endif
  return (axis ? F.uvy : F.uvx)[p * 5 + 1 + s];
}

// castRay glsl:68-74 over vec4 (w included, as the GLSL does).
__device__ __forceinline__ void cast_ray(const Frame& F, float uvx, float uvy, f3& ro, f3& rd) {
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = (uvx * F.cam_x[k] + uvy * F.cam_y[k]) + F.cam_dir[k] * F.persp;
  float dd = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
  float inv = rcp_of_sqrt(sqrt_cr_nonneg(dd));
  ro = mk(F.cam_pos[0], F.cam_pos[1], F.cam_pos[2]);
  rd = mk(v[0] * inv, v[1] * inv, v[2] * inv);
}

// RGBA8 quantization round(clamp(c,0,1)*255), NaN -> 0.
__device__ __forceinline__ uint32_t quantize(float c) {
  float v = (c > 0.0f) ? ((c < 1.0f) ? c : 1.0f) : 0.0f;
  return (uint32_t)(v * 255.0f + 0.5f);
}

// Dispatch order of the tile rows: inside out (the middle row first, then
// alternately below and above).  The slowest waves (rays grazing the floor near
// the horizon, silhouettes) sit in the middle band of an upright view; started
// first they no longer form a tail behind the cheap sky and near-floor rows
// (cfg3 1.24 -> 1.18 ms against the natural order).
__device__ __forceinline__ int tile_row(int b, int n) {
  // mid, mid-1, mid+1, mid-2, ...: b < n covers [mid - n/2, mid + (n-1)/2] = [0, n-1]
  const int mid = n / 2, k = (b + 1) >> 1;
  return (b & 1) ? mid - k : mid + k;
}

// XCD-aware tile column: one-wave workgroups go round-robin to the 8 XCDs
// (block b -> XCD b % 8), so consecutive blocks land in different L2s and the
// 16-32 B row segments that neighbouring tiles store into one 128 B line are
// written back separately (PMC: 2x write amplification).  Within each window of
// 8 G blocks, XCD k takes the G adjacent tiles [k G, (k+1) G): a line's
// segments meet in one L2, while the XCDs still interleave at G-tile grain
// (a coarse split, XCD k = columns [k gx/8, ...), unbalanced the XCDs: 2x slower).
__device__ __forceinline__ int tile_col(int b, int gx, int G) {
  const int win = 8 * G;
  const int w0 = (b / win) * win;
  const int r = b - w0;
  return (w0 + win > gx) ? b : w0 + (r & 7) * G + (r >> 3);  // ragged last window: natural order
}

// Global row of a launch-local row (row sharding; rm_shard.hpp).
__device__ __forceinline__ int global_row(const Frame& F, int local_row) {
  if (F.nshards <= 1) return local_row;
  const int g = rm::shard_row(rm::ShardMap{F.row_block, F.row_block0, F.nshards}, F.shard, local_row);
  return g < F.height ? g : -1;
}

__device__ __forceinline__ void store_pixel(const Frame& F, size_t idx, float r, float g, float b,
                                            float a) {
  if (F.rgba8) {
    if (F.rgb3) {  // uniform: a scalar branch
      uint8_t* p = F.rgba8 + idx * 3;
      p[0] = (uint8_t)quantize(r);
      p[1] = (uint8_t)quantize(g);
      p[2] = (uint8_t)quantize(b);
    } else {
      uint32_t w = quantize(r) | (quantize(g) << 8) | (quantize(b) << 16) | (quantize(a) << 24);
      reinterpret_cast<uint32_t*>(F.rgba8)[idx] = w;
    }
  }
  if (F.rgba32f) reinterpret_cast<float4*>(F.rgba32f)[idx] = make_float4(r, g, b, a);
}

}  // namespace rmd
