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
// Capsule constants (glsl:120): ba = b - a and dot(ba, ba), folded in float.
constexpr float CAP_AX = -0.1f, CAP_AY = 0.1f, CAP_AZ = -0.1f;
constexpr float CAP_BAX = 2.0f - CAP_AX, CAP_BAY = 4.0f - CAP_AY, CAP_BAZ = 2.0f - CAP_AZ;
constexpr float CAP_BB = (CAP_BAX * CAP_BAX + CAP_BAY * CAP_BAY) + CAP_BAZ * CAP_BAZ;

// Minimum scene distance and the opU id (glsl:107-123).  `id` follows opU's
// rule exactly: a later primitive replaces the running one unless the running
// distance is strictly smaller.  blend/omblend carry mix()'s a and 1-a.
template <bool WANT_ID>
__device__ __forceinline__ float scene(f3 p, float blend, float omblend, int& id) {
  // sphere (15,0,-10) r3, id 0   glsl:111
  float ax = p.x - 15.0f, ay = p.y, az = p.z + 10.0f;
  float d = __builtin_sqrtf((ax * ax + ay * ay) + az * az) - 3.0f;
  if (WANT_ID) id = 0;
  // sphere (-25,0,-10) r3, id 1  glsl:112
  float bx = p.x + 25.0f;
  float d1 = __builtin_sqrtf((bx * bx + ay * ay) + az * az) - 3.0f;
  if (WANT_ID) id = (d < d1) ? id : 1;
  d = fminf(d, d1);
  // mix(box, sphere, blend) at (-5,0,-10), id 4   glsl:115-117
  float cx = p.x + 5.0f;
  float qx = fabsf(cx) - 3.0f, qy = fabsf(ay) - 2.5f, qz = fabsf(az) - 2.5f;
  float mx = fmaxf(qx, 0.0f), my = fmaxf(qy, 0.0f), mz = fmaxf(qz, 0.0f);
  float box = fminf(fmaxf(qx, fmaxf(qy, qz)), 0.0f) + __builtin_sqrtf((mx * mx + my * my) + mz * mz);
  float sph = __builtin_sqrtf((cx * cx + ay * ay) + az * az) - 3.0f;
  float d4 = box * omblend + sph * blend;
  if (WANT_ID) id = (d < d4) ? id : 4;
  d = fminf(d, d4);
  // torus at (-5,0,10), (pos - c).xzy, t = (2.5, 0.5), id 5   glsl:93-96,119
  float tz = p.z - 10.0f;
  float l = __builtin_sqrtf(cx * cx + ay * ay) - 2.5f;
  float d5 = __builtin_sqrtf(l * l + tz * tz) - 0.5f;
  if (WANT_ID) id = (d < d5) ? id : 5;
  d = fminf(d, d5);
  // capsule at (-5,-2,-30), a(-.1,.1,-.1) b(2,4,2) r1, id 6   glsl:98-103,120
  float px_ = cx - CAP_AX, py_ = (p.y + 2.0f) - CAP_AY, pz_ = (p.z + 30.0f) - CAP_AZ;
  float h = (px_ * CAP_BAX + py_ * CAP_BAY) + pz_ * CAP_BAZ;
  h = fminf(fmaxf(h / CAP_BB, 0.0f), 1.0f);
  float ex = px_ - CAP_BAX * h, ey = py_ - CAP_BAY * h, ez = pz_ - CAP_BAZ * h;
  float d6 = __builtin_sqrtf((ex * ex + ey * ey) + ez * ez) - 1.0f;
  if (WANT_ID) id = (d < d6) ? id : 6;
  d = fminf(d, d6);
  // plane y = -5.5, id 7 (MATTE)   glsl:85,121
  float d7 = p.y + 5.5f;
  if (WANT_ID) id = (d < d7) ? id : 7;
  d = fminf(d, d7);
  return d;
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
