// rm_table.hip — the runtime-scene-table path.
//
// The reference hard-codes its scene in sdf() (computeShader.glsl:107-123).
// This kernel renders any scene given as a table of primitives (rm_set_scene,
// include/rm_api.h), with the reference's march / normal / shadow / light /
// bounce logic (glsl:125-344) unchanged around a generic sdf:
//
//   * each workgroup stages the table (n x 80 B) from HBM into LDS once; every
//     sdf() step then loops over the LDS entries in table order.  All lanes
//     read the same entry (an LDS broadcast, no bank conflicts) and the
//     primitive type is made wave-uniform (readfirstlane), so the per-type
//     switch is a scalar branch;
//   * opU (glsl:105) as in the GLSL: a later entry wins unless the running
//     distance is strictly smaller; the hit's colour / id / material are read
//     from the winning entry after the march (the colour at the same point);
//   * every float operation is the IEEE one the GLSL specifies:
//     correctly rounded sqrt (sqrt_cr_nonneg, proven equal to the IEEE sqrt on
//     [0, FLT_MAX]) and division, no contraction;
//   * the shortcuts are the generic forms of the specialised kernel's proofs,
//     from per-entry bounding balls and plane bounds computed on the host
//     (rm::exit_bounds): provable miss / shadow exits (table_exit_T), lazy
//     per-entry culling along marches (tmarch) and per-point culling (dist).
//     Each only skips work whose result is proven not to change (d, best).
// For the reference scene (rm_default_scene) the image equals the built-in
// kernel's bit for bit (tests/test_gpu_scene.py); other tables are checked
// against the oracle's table mode (oracle/rm_oracle.c rmo_render_scene).
//
// Diagnostic builds only: RM_TDBL_<MARCH|BMARCH|SHADOW|NORMAL> runs that phase
// twice (its marginal cost per frame, tools/ab_kernel.py --table / --spec; the
// specialised kernels get the define through RM_JIT_EXTRA, rm_jit.hip).
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#include "rm_internal.hpp"
#ifndef __HIPCC_RTC__
#include <cstring>
#include <type_traits>
#endif
#include "rm_scene.hpp"

// RM_TABLE_STATIC: this file compiled at rm_set_scene time by hiprtc
// (rm_jit.cpp) for one table, whose compiled words (rm::compile_scene) come as
// the constant array RM_TS_WORDS[scene_words(RM_TS_N)] of the generated header.
// Every entry loop is then unrolled over a compile-time table: types, masks and
// parameters fold into the instruction stream (no LDS staging, no type switch).
#ifdef RM_TABLE_STATIC
#include "rm_table_static.h"
#define RM_TS_UNROLL _Pragma("unroll")
#define RM_TS_INLINE __forceinline__  // (the unrolled bodies would otherwise become calls)
#else
#define RM_TS_UNROLL
#define RM_TS_INLINE
#endif


namespace rmd {

struct TCnt {
  uint32_t rays, march, reflect, shadow, normals, lights;
};
// compile-time flags of the march-loop variants (no <type_traits> under hiprtc)
struct Yes { static constexpr bool value = true; };
struct No { static constexpr bool value = false; };
template <int V>
struct IntC { static constexpr int value = V; };

using rm::TABLE_WORDS;

// The specialised kernels only render frames whose march and normal points are
// bounded (prim_dist's BOUNDED form; rm_api.hip frame_jit).
#ifdef RM_TABLE_STATIC
constexpr bool kBoundedPoints = true;
#else
constexpr bool kBoundedPoints = false;
#endif

// Wave vote on the ballot builtin itself (hiprtc's __any widens the predicate
// to an int and compares it again: two extra VALU per vote).
__device__ __forceinline__ bool wany(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0; }
// A table word every lane reads alike, in a scalar register.
__device__ __forceinline__ float uword(const float* p) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(*p)));
}

// Correctly rounded sqrt of a sum of squares (x >= 0, +inf or NaN).  The fast
// form is sqrt_cr_nonneg (exact on [0, FLT_MAX], rm_fastmath.hpp) with +inf
// passed through, so it equals the IEEE sqrt on the whole domain.
__device__ __forceinline__ float isqrt_ieee(float x) {
  const float s = sqrt_cr_nonneg(x);
  return x == __builtin_inff() ? x : s;
}
__device__ __forceinline__ float tlen(f3 a) { return isqrt_ieee(dot(a, a)); }
// GLSL normalize over the full float range (v * (1 / sqrt(dot)))
__device__ __forceinline__ f3 tnormalize(f3 a) { return muls(a, 1.0f / isqrt_ieee(dot(a, a))); }

// sqrt(x) - R as the IEEE operations give it.  BOUNDED: a specialised table's
// march and normal points, within 2^53 of every entry's centre (the host renders
// a frame whose camera is farther than 10^15 from the origin with the generic
// kernel, rm_api.hip frame_jit; entries lie within 10^15, rm::exit_bounds; a
// march moves at most nmax tmax along a unit ray, 5 bounces add 5 x 256 x 200),
// so x is a finite sum of squares, and for a compile-time R >= 2^-20 sqrt_core
// alone is exact: on [2^-96, FLT_MAX] it is the correctly rounded sqrt
// (rm_fastmath.hpp); below, both roots are under 2^-47, inside half an ulp of R,
// and both differences round to -R.  Otherwise the full-range form.
template <bool BOUNDED>
__device__ __forceinline__ float sqrt_sub(float x, float R) {
  if (BOUNDED && R >= 0x1p-20f) return sqrt_core(x) - R;
  return isqrt_ieee(x) - R;
}

// One table entry's distance at p (glsl:83-103, 115-121).
template <bool BOUNDED = false>
__device__ __forceinline__ float prim_dist(const float* P, int type, f3 p, float blend,
                                           float omblend) {
  f3 q = sub(p, mk(P[rm::TW_CENTER], P[rm::TW_CENTER + 1], P[rm::TW_CENTER + 2]));
  if (__float_as_int(P[rm::TW_SWIZZLE]) == RM_SWIZZLE_XZY) q = mk(q.x, q.z, q.y);
  const float* a = P + rm::TW_P;
  switch (type) {
    case RM_PRIM_SPHERE:
      return sqrt_sub<BOUNDED>(dot(q, q), a[0]);
    case RM_PRIM_BOX:
    case RM_PRIM_BLEND: {
      const f3 d = mk(fabsf(q.x) - a[0], fabsf(q.y) - a[1], fabsf(q.z) - a[2]);
      const f3 m = mk(gmax(d.x, 0.0f), gmax(d.y, 0.0f), gmax(d.z, 0.0f));
      const float box = gmin(gmax(d.x, gmax(d.y, d.z)), 0.0f) + tlen(m);
      if (type == RM_PRIM_BOX) return box;
      const float sph = sqrt_sub<BOUNDED>(dot(q, q), a[3]);
      return box * omblend + sph * blend;  // mix(box, sphere, blend)
    }
    case RM_PRIM_TORUS: {
      const float l = sqrt_sub<BOUNDED>(q.x * q.x + q.z * q.z, a[0]);
      return sqrt_sub<BOUNDED>(l * l + q.y * q.y, a[1]);
    }
    case RM_PRIM_CAPSULE: {
      const f3 pa = sub(q, mk(a[0], a[1], a[2])), ba = mk(a[3], a[4], a[5]);
      const float h = gmin(gmax(dot(pa, ba) / a[6], 0.0f), 1.0f);
      const f3 r = sub(pa, muls(ba, h));
      return sqrt_sub<BOUNDED>(dot(r, r), a[7]);
    }
    default:  // RM_PRIM_PLANE
#ifdef RM_TABLE_STATIC
      // A specialised table's axis-aligned normal (0, n_y, 0), as the reference's
      // floor (a compile-time test): the x and z terms of the dot are signed
      // zeros for finite q, which leave the sum as it is (the built-in kernel's
      // p.y + 5.5, rm_scene.hpp), so q.x and q.z are not read.  (A runtime test
      // in the generic kernel measured 5 % slower.)
      if (a[0] == 0.0f && a[2] == 0.0f) return q.y * a[1] + a[3];
#endif
      return dot(q, mk(a[0], a[1], a[2])) + a[3];
  }
}

// The slots' balls are staged with their radius negated (Table::sb), so the
// re-test's fma(|p - c|, 1 - 2^-12, -R) takes it as a VGPR addend with its
// literal factor (v_fmamk_f32, dual-issued) instead of the factor in an SGPR.
#define RM_SBR(r) (-(r))
struct Table {
  const float* t;  // LDS (or global) copy of the compiled table
#ifdef RM_TABLE_STATIC
  static constexpr int n = RM_TS_N;
#else
  int n;
  // The fast plane (generic kernel): the table's only plane when it has exactly
  // one (the reference's floor, and most scenes), staged so that the every-step
  // plane evaluation needs no type dispatch and no entry loop (plane_fast:
  // prim_dist's plane arithmetic, the same float operations); the reference's
  // floor (fpunit) is one add of the offset w.  fp = -1: none.
  int fp;
  // The fast plane's offset w in a scalar register; its centre, normal and
  // swizzle are read from its LDS entry where a path needs them (round 6: held in
  // scalar registers they took 7 of the kernel's, which is at its scalar-register
  // limit: 13 -> 2 spilled SGPRs and no scratch in the reference-shaped instance,
  // -0.7 % per cfg3 frame; the tilted-plane shape, whose every step reads them,
  // +5 %; profiles/r06_ab_fplds*.txt)
  float fpw;
  __device__ __forceinline__ float FPC(int j) const { return t[fp * TABLE_WORDS + rm::TW_CENTER + j]; }
  __device__ __forceinline__ float FPN(int j) const { return t[fp * TABLE_WORDS + rm::TW_P + j]; }
  __device__ __forceinline__ int FPSWZ() const { return __float_as_int(t[fp * TABLE_WORDS + rm::TW_SWIZZLE]); }
  const float* sb;  // the lazy slots' balls, 4 words each (centre, -radius: RM_SBR), slot order, in LDS
  bool fpaxis;  // normal (0, n_y, 0): the plane is q.y n_y + w (the specialised kernel's shortcut)
  // ... with centre y 0 and n_y = 1, unswizzled (the reference's floor): q.y = p.y - 0 = p.y and
  // q.y * 1 = q.y exactly for every float, so the plane is the one add p.y + w (round 6: the
  // specialised kernel folds the same at compile time)
  bool fpunit;
#endif
  float blend, omblend;

  __device__ __forceinline__ const float* exits() const { return t + n * TABLE_WORDS; }
#ifndef RM_TABLE_STATIC
  __device__ __forceinline__ float plane_fast(f3 p) const {
    // q.x n_x and q.z n_z are signed zeros for finite q: the sum is q.y n_y + w
    // (prim_dist's RM_TABLE_STATIC shortcut, here on a uniform flag: -1.2 % per
    // cfg3 frame; the per-lane test inside the type switch had measured +5 %)
    if (fpunit) return p.y + fpw;
    if (fpaxis) return ((FPSWZ() == RM_SWIZZLE_XZY ? p.z - FPC(2) : p.y - FPC(1))) * FPN(1) + fpw;
    f3 q = sub(p, mk(FPC(0), FPC(1), FPC(2)));
    if (FPSWZ() == RM_SWIZZLE_XZY) q = mk(q.x, q.z, q.y);
    return dot(q, mk(FPN(0), FPN(1), FPN(2))) + fpw;
  }
#endif

  __device__ __forceinline__ const float* entry(int k) const { return t + k * TABLE_WORDS; }
  __device__ __forceinline__ int type(int k) const {
    return __builtin_amdgcn_readfirstlane(__float_as_int(entry(k)[rm::TW_TYPE]));
  }
  // sdf(p).hitpoint and the index of the opU winner.
  //
  // Culling: an entry whose lower bound at p exceeds an upper
  // bound U of the final minimum is strictly above that minimum, so it can
  // neither be the opU winner nor tie it (ties go to the later entry) and
  // skipping it leaves (d, best) unchanged.  U = min(running minimum, the
  // planes' values at p computed first with the same operations); the bound
  // is |p - c'| - R - slack(p) from the entry's ball (TW_BALL, rm::exit_bounds),
  // slack(p) = sigma (|p|_1 + S) (rounded up) covering the float error of the
  // entry's value and of the bound.  A culled entry's value is finite (its
  // |p - c'| < 2^60, finite parameters), so NaN propagation through opU is
  // unchanged too.  d starts at +inf: opU(+inf, v) takes v for every v, as the
  // GLSL's first assignment does.
  __device__ __forceinline__ float dist(f3 p, int& best) const {
    const float INF = __builtin_huge_valf();
    float U = INF, slack = 0.0f;
    {
      RM_TS_UNROLL
      for (int k = 0; k < n; ++k)
        if (type(k) == RM_PRIM_PLANE) U = gmin(U, prim_dist(entry(k), RM_PRIM_PLANE, p, blend, omblend));
      const float* ex = exits();
      slack = ex[rm::EX_SIGMA] * (((fabsf(p.x) + fabsf(p.y)) + fabsf(p.z)) + ex[rm::EX_S]) *
              ((1.0f + 0x1p-12f) * (1.0f + 0x1p-12f));
    }
    float d = INF;
    best = 0;
    RM_TS_UNROLL
    for (int k = 0; k < n; ++k) {
      const float* P = entry(k);
      // (spheres: the exact value costs no more than the bound)
      if (P[rm::TW_BALL + 3] != INF && type(k) != RM_PRIM_SPHERE) {
        const float bx = p.x - P[rm::TW_BALL], by = p.y - P[rm::TW_BALL + 1], bz = p.z - P[rm::TW_BALL + 2];
        const float x = (bx * bx + by * by) + bz * bz;
        const float lb = __builtin_fmaf(__builtin_amdgcn_sqrtf(x), 1.0f - 0x1p-12f, -(P[rm::TW_BALL + 3] + slack));
        if ((lb > gmin(d, U)) & (x < 0x1p120f)) continue;
      }
      const float dk = prim_dist(P, type(k), p, blend, omblend);
      const bool keep = d < dk;  // opU(t, new) = (t < new) ? t : new
      best = keep ? best : k;
      d = keep ? d : dk;
    }
    return d;
  }
  // GetNormal's four samples, sdf at pos and at pos + 0.001 e_x / e_y / e_z
  // (glsl:278-288), with one culling pass for all four (the generic form of
  // rm_scene.hpp normal_samples).  The samples lie within e = 0.001 + 2^-22
  // (|pos|_1 + 1) of pos (the float adds round).  An entry's ball bound is
  // 1-Lipschitz, so at a sample it is at least its value at pos minus e, and
  // the minimum there is at most U + L e (U: the planes at pos, L = EX_LIP):
  // an entry whose bound at pos exceeds U + (1 + L) e (rounded up), with the
  // slack taken at |pos|_1 + 0.002 >= every sample's |p|_1, is strictly above
  // the minimum at all four.  The others are evaluated at every sample with
  // opU in table order, so each value equals dist()'s at that point.  With
  // have_c0 the centre sample is c0 and is not evaluated.
  __device__ __forceinline__ void normal_samples(f3 pos, bool have_c0, float& c0, float& vx, float& vy,
                                                 float& vz) const {
    const float INF = __builtin_huge_valf();
    const f3 px = add(pos, mk(0.001f, 0.0f, 0.0f));
    const f3 py = add(pos, mk(0.0f, 0.001f, 0.0f));
    const f3 pz = add(pos, mk(0.0f, 0.0f, 0.001f));
    const float* ex = exits();
    const float p1 = (fabsf(pos.x) + fabsf(pos.y)) + fabsf(pos.z);
    float U = INF;
#ifndef RM_TABLE_STATIC
    // the planes' bound from the fast plane, or the plane mask: no pass over every
    // entry's type (round 6: -1 % per cfg3 frame, profiles/r06_ab_gen3.txt)
    if (fp >= 0) {
      U = gmin(U, plane_fast(pos));  // (TLazy::dist's bound the same way)
    } else {
      for (uint32_t pm = __float_as_uint(ex[rm::EX_PLANE_MASK]); pm; pm &= pm - 1u)
        U = gmin(U, prim_dist(entry(__builtin_ctz(pm)), RM_PRIM_PLANE, pos, blend, omblend));
    }
#else
    RM_TS_UNROLL
    for (int k = 0; k < n; ++k)
      if (type(k) == RM_PRIM_PLANE) U = gmin(U, prim_dist(entry(k), RM_PRIM_PLANE, pos, blend, omblend));
#endif
    const float e = 0.001f + 0x1p-22f * (p1 + 1.0f);
    const float Ue = U + ((1.0f + ex[rm::EX_LIP]) * e * (1.0f + 0x1p-10f) + 0x1p-20f * fabsf(U));
    const float slack = ex[rm::EX_SIGMA] * ((p1 + 0.002f) + ex[rm::EX_S]) *
                        ((1.0f + 0x1p-12f) * (1.0f + 0x1p-12f));
    uint32_t keep = 0;  // entries some lane did not cull at its samples (uniform, as dist_mask)
    RM_TS_UNROLL
    for (int k = 0; k < n; ++k) {
      const float* P = entry(k);
      bool cull = false;
      if (P[rm::TW_BALL + 3] != INF && type(k) != RM_PRIM_SPHERE) {
        const float bx = pos.x - P[rm::TW_BALL], by = pos.y - P[rm::TW_BALL + 1], bz = pos.z - P[rm::TW_BALL + 2];
        const float x = (bx * bx + by * by) + bz * bz;
        const float lb = __builtin_fmaf(__builtin_amdgcn_sqrtf(x), 1.0f - 0x1p-12f, -(P[rm::TW_BALL + 3] + slack));
        cull = (lb > Ue) & (x < 0x1p120f);
      }
      if (wany(!cull)) keep |= 1u << k;
    }
#ifndef RM_TABLE_STATIC
    // The generic kernel (round 6): the kept entries in table order, each entry's
    // words read from LDS once and its type switched on once for all four samples
    // (one sample at a time, every sample had re-read the entry and re-run the
    // switch): -8.4 % per cfg3 frame (profiles/r06_ab_gen2.txt; the words moved to
    // scalar registers instead, v_readfirstlane each, gave -4.0 %).  Per sample the
    // same opU over the same entries in the same order: the same four values.
    float d0 = INF, dx = INF, dy = INF, dz = INF;
    for (uint32_t w = keep; w; w &= w - 1u) {
      const int k = __builtin_ctz(w);
      float P[TABLE_WORDS];
#pragma unroll
      for (int i = rm::TW_SWIZZLE; i < rm::TW_BALL; ++i) P[i] = entry(k)[i];
      auto eval4 = [&](auto T) {
        constexpr int ty = decltype(T)::value;
        auto opu = [](float d, float v) { return d < v ? d : v; };
        if (!have_c0) d0 = opu(d0, prim_dist<kBoundedPoints>(P, ty, pos, blend, omblend));
        dx = opu(dx, prim_dist<kBoundedPoints>(P, ty, px, blend, omblend));
        dy = opu(dy, prim_dist<kBoundedPoints>(P, ty, py, blend, omblend));
        dz = opu(dz, prim_dist<kBoundedPoints>(P, ty, pz, blend, omblend));
      };
      switch (type(k)) {
        case RM_PRIM_SPHERE: eval4(IntC<RM_PRIM_SPHERE>()); break;
        case RM_PRIM_BOX: eval4(IntC<RM_PRIM_BOX>()); break;
        case RM_PRIM_BLEND: eval4(IntC<RM_PRIM_BLEND>()); break;
        case RM_PRIM_TORUS: eval4(IntC<RM_PRIM_TORUS>()); break;
        case RM_PRIM_CAPSULE: eval4(IntC<RM_PRIM_CAPSULE>()); break;
        default: eval4(IntC<RM_PRIM_PLANE>()); break;
      }
    }
    if (!have_c0) c0 = d0;
    vx = dx;
    vy = dy;
    vz = dz;
    return;
#endif
    // one sample at a time (fewer live values): opU in table order over `keep`
    // (an entry this lane culled is strictly above its minimum at the sample)
    auto sample = [&](f3 q) {
      float d = INF;
      RM_TS_UNROLL
      for (int k = 0; k < n; ++k) {
        if (!((keep >> k) & 1u)) continue;
        const float v = prim_dist<kBoundedPoints>(entry(k), type(k), q, blend, omblend);
        d = d < v ? d : v;
      }
      return d;
    };
    if (!have_c0) c0 = sample(pos);
    vx = sample(px);
    vy = sample(py);
    vz = sample(pz);
  }
  // sdf(p) over the entries whose bit is set in `wave` (uniform: every entry
  // some lane of the wave could not cull), opU in table order.  An entry a lane
  // did cull is proven strictly above that lane's minimum, so evaluating it
  // there changes neither d nor best: no per-lane mask tests (exec-masked
  // lanes would cost the same cycles).
  __device__ __forceinline__ float dist_mask(f3 p, uint32_t wave, int& best) const {
#ifndef RM_TABLE_STATIC
    if (fp >= 0 && wave == (1u << fp)) {  // opU(+inf, v) = v (dist_mask's first take)
      best = fp;
      return plane_fast(p);
    }
#endif
    float d = __builtin_huge_valf();
    best = 0;
#ifdef RM_TABLE_STATIC
    RM_TS_UNROLL
    for (int k = 0; k < n; ++k) {
      if (!((wave >> k) & 1u)) continue;
#else
    for (; wave; wave &= wave - 1u) {
      const int k = __builtin_ctz(wave);
#endif
      const float dk = prim_dist(entry(k), type(k), p, blend, omblend);
      const bool keep = d < dk;
      best = keep ? best : k;
      d = keep ? d : dk;
    }
    return d;
  }
  __device__ __forceinline__ f3 color(int k, f3 p) const {
    const float* P = entry(k);
    if (__float_as_int(P[rm::TW_PAINT]) == RM_PAINT_CHECKERS) {
      const float c = checkers(p);
      return mk(c, c, c);
    }
    return mk(P[rm::TW_COLOR], P[rm::TW_COLOR + 1], P[rm::TW_COLOR + 2]);
  }
  __device__ __forceinline__ int id(int k) const { return __float_as_int(entry(k)[rm::TW_ID]); }
  // True when no step of a march from ro along rd can see a distance > tmax:
  // some axis-aligned plane (normal (0, n_y, 0), a specialised table's
  // compile-time test, the generic kernel's fast plane) has a value that does not
  // grow along the ray and starts at or below tmax.  Its float value RN(RN(q.y n_y) + off), q.y = RN(p.y - c.y),
  // p.y = RN(ro.y + RN(rd.y t)), is monotone in t (rounding is monotone), non-
  // increasing when n_y rd.y <= 0, and the minimum is at most that value.  NaNs
  // fail every compare (false).
  __device__ __forceinline__ bool no_escape(f3 ro, f3 rd, float tmax) const {
    bool ok = false;
#ifdef RM_TABLE_STATIC
    RM_TS_UNROLL
    for (int k = 0; k < n; ++k) {
      const float* P = entry(k);
      const float* a = P + rm::TW_P;
      if (type(k) != RM_PRIM_PLANE || !(a[0] == 0.0f && a[2] == 0.0f)) continue;
      const bool swz = __float_as_int(P[rm::TW_SWIZZLE]) == RM_SWIZZLE_XZY;
      const float oy = swz ? ro.z : ro.y, ry = swz ? rd.z : rd.y;  // q = (p - c).xzy: q.y = p.z - c.z
      const float cy = swz ? P[rm::TW_CENTER + 2] : P[rm::TW_CENTER + 1];
      const bool mono = (a[1] > 0.0f && ry <= 0.0f) || (a[1] < 0.0f && ry >= 0.0f);
      ok = ok || (mono && (oy - cy) * a[1] + a[3] <= tmax);
    }
#else
    // the generic kernel's fast plane when axis-aligned: the same argument with
    // its staged parameters (round 6: the escape compare leaves the step loop of
    // waves of downward rays, -1.5 % per cfg3 frame, profiles/r06_ab_gen5.txt)
    if (fp >= 0 && fpaxis) {
      const bool swz = FPSWZ() == RM_SWIZZLE_XZY;
      const float oy = swz ? ro.z : ro.y, ry = swz ? rd.z : rd.y, cy = swz ? FPC(2) : FPC(1);
      const bool mono = (FPN(1) > 0.0f && ry <= 0.0f) || (FPN(1) < 0.0f && ry >= 0.0f);
      ok = mono && (oy - cy) * FPN(1) + fpw <= tmax;
    }
#endif
    return ok;
  }
  __device__ __forceinline__ float material(int k) const { return entry(k)[rm::TW_MATERIAL]; }
};

// Provable early exits for any table (the generic form of rm_scene.hpp's
// lin_exit_T; bounds from rm::exit_bounds, rm_host.cpp).  Every entry's float
// value at p(t) = ro + rd t is at least
//   |rd| t - |ro - C| - R - slack(t)            (entries inside the ball C, R)
//   dot(ro, n') + off + dot(rd, n') t - slack(t) (plane entries)
// with slack(t) = s0 + s1 t = sigma (|ro|_1 + S) + sigma |rd|_1 t (rounded up),
// all linear in t.  Once each bound stays above max(hmin, c t) for every later
// t -- past T, returned here (+inf: not provable) -- no later step of a march
// along the ray can see a distance <= hmin or a ratio d / t <= c:
//   * RayMarch / reflectedRay: c = 1e-6 (1 + 2^-9), hmin = 0: no later step
//     hits, the march ends in a miss (t is discarded);
//   * softshadow (rd = light - pos): c = (1 + 2^-9) / k, hmin = 0.001: no
//     later step returns 0.05 and every k h / t rounds above 1 >= res.
// Coefficients are rounded toward failure (2^-12 relative, 2^-20 absolute terms),
// as in lin_exit_T.
__device__ __forceinline__ float table_exit_T(const float* ex, float c, float hmin, f3 ro, f3 rd) {
  const float INF = __builtin_huge_valf();
  if (ex[rm::EX_VALID] == 0.0f) return INF;
  const float HI = 1.0f + 0x1p-12f, LO = 1.0f - 0x1p-12f;
  const float UP = 1.0f + 0x1p-20f, DN = 1.0f - 0x1p-20f;
  const float sig = ex[rm::EX_SIGMA];
  const float ro1 = (fabsf(ro.x) + fabsf(ro.y)) + fabsf(ro.z);
  const float rd1 = (fabsf(rd.x) + fabsf(rd.y)) + fabsf(rd.z);
  const float s0 = sig * (ro1 + ex[rm::EX_S]) * (HI * HI);
  const float s1 = sig * rd1 * (HI * HI);
  float T = -INF;
  if (ex[rm::EX_R] > -1e29f) {  // the ball of the bounded entries
    const float ex0 = ro.x - ex[rm::EX_CX], ey = ro.y - ex[rm::EX_CY], ez = ro.z - ex[rm::EX_CZ];
    const float rc = __builtin_fmaf(__builtin_amdgcn_sqrtf((ex0 * ex0 + ey * ey) + ez * ez), HI, 0x1p-18f);
    const float rdl = __builtin_amdgcn_sqrtf(dot(rd, rd));
    const float a1 = (rdl * LO - s1 - c) * LO - 0x1p-20f * (rdl + c);
    const float b1 = (rc + ex[rm::EX_R] + s0 + hmin) * HI;
    float To = a1 > 0.0f ? b1 * __builtin_amdgcn_rcpf(a1) * UP : INF;
    // ... or the slab of their box along y (round 5, as rm_scene.hpp's slab below
    // the objects): on the side of the box the ray leaves it by, every entry is
    // at least (p.y - hi.y) (or lo.y - p.y) - slack, linear in t; the first of
    // the bounds to hold for good proves the entries' term.  The x and z slabs
    // cost more than they saved (reference-shaped table, cfg3: specialised
    // +4.6 %, generic +1 %, profiles/r05_ab_tableslab.txt), as for the built-in.
    {
      const float r = rd.y, ra = fabsf(r), sc = s1 + c, sh = s0 + hmin;
      const float edge = r > 0.0f ? ex[rm::EX_BOX + 4] : ex[rm::EX_BOX + 1];
      const float as = (ra - sc) - 0x1p-20f * (ra + sc);
      const float bs = ((r > 0.0f ? edge - ro.y : ro.y - edge) + sh) + 0x1p-20f * ((fabsf(edge) + fabsf(ro.y)) + sh);
      if (as > 0.0f) To = __builtin_fminf(To, bs * __builtin_amdgcn_rcpf(as) * (bs >= 0.0f ? UP : DN));
    }
    if (!(To < INF)) return INF;
    T = To;
  }
  const int np = (int)ex[rm::EX_NPLANES];
  for (int j = 0; j < np; ++j) {
    const float* pl = ex + rm::EX_PLANES + 4 * j;
    const f3 nw = mk(pl[0], pl[1], pl[2]);
    const float A = dot(ro, nw) + pl[3], B = dot(rd, nw);
    const float a2 = (B - s1 - c) - 0x1p-20f * (fabsf(B) + s1 + c);
    const float b2 = (A - s0 - hmin) - 0x1p-20f * (fabsf(A) + s0 + hmin);
    if (!(a2 > 0.0f)) return INF;
    T = __builtin_fmaxf(T, -(b2 * __builtin_amdgcn_rcpf(a2) * (b2 >= 0.0f ? DN : UP)));
  }
  return T;
}

// Lazy culling along a march (the generic form of scene_lazy,
// rm_scene.hpp) for p(t) = ro + rd t with t growing by the returned distance
// after every step (tmarch, tshadow).  Slot j tracks entry k_j (rm::exit_bounds)
// with an expiry te[j] before which k_j is proven strictly above the minimum.
// A re-test at p = p(t) bounds k_j below by its ball, lb = |p - c'| - R, and
// the minimum above by U = min(the planes' values at p, d_prev (1 + L |rd|) +
// sl): the previous step moved p by |rd| d_prev (d_prev >= 0: a march that goes
// on past a step has a non-negative distance there) and the minimum is
// L-Lipschitz.  With sl = 2 sigma (|p|_1 + |ro|_1 + S) covering the float error
// of both sides (and of p(t) itself), k_j stays above the minimum while
// t' - t < g / ((1 + L) |rd| + 2 sigma |rd|_1), g = lb - U - sl (the second
// term: the slack's growth along the ray); g <= 0 evaluates k_j now.
// Untracked entries and planes are evaluated at every step (EX_EVAL_MASK).
// Lanes whose te has not expired re-test for free and keep the later expiry.
// The negated compares send NaN rays (degenerate uniforms) through the
// re-test, whose NaN bound evaluates every entry.
// KL: the slots this instance holds (>= the table's EX_NSLOTS; launch_table
// picks the generic kernel's instance from the table, a specialised table's
// unrolled loops fold the unused slots away).
// The first expiry of slot j of a march that starts without the host's step 0
// (reflected and shadow marches): -inf (re-test at the first step) for the
// table's ns slots, +inf (never) for an instance's unused ones.  In a
// specialised kernel ns is a compile-time count and this folds to a constant.
// In the generic kernel ns is the table's, at run time; the select there is
// formed in scalar registers where the march starts (volatile: LLVM had hoisted
// the KL uniform selects out of the bounce loop into VGPRs live across the
// whole kernel, 5 of them spilled in the reference-shaped instance, round 5).
__device__ __forceinline__ float slot_init(int j, int ns) {
#ifdef RM_TABLE_STATIC
  return j < ns ? -__builtin_huge_valf() : __builtin_huge_valf();
#else
  uint32_t b;
  asm volatile(
      "s_mov_b32 %0, 0x7f800000\n\t"
      "s_cmp_gt_i32 %1, %2\n\t"
      "s_cselect_b32 %0, 0xff800000, %0"
      : "=&s"(b)
      : "s"(__builtin_amdgcn_readfirstlane(ns)), "i"(j)
      : "scc");
  return __uint_as_float(b);
#endif
}

template <int KL>
struct TLazy {
  const float* ex;
  int ns;
  uint32_t always;
  float te_[KL];
  __device__ __forceinline__ float& te(int j) { return te_[j]; }
  float temin, sig2, sl0, inv, grow, dprev;

  __device__ __forceinline__ TLazy(const Table& S, f3 ro, f3 rd) {
    const float INF = __builtin_huge_valf();
    ex = S.exits();
    ns = (int)ex[rm::EX_NSLOTS];
    const uint32_t all = S.n >= 32 ? 0xffffffffu : (1u << S.n) - 1u;
    always = ns > 0 ? __float_as_uint(ex[rm::EX_EVAL_MASK]) : all;
#pragma unroll
    for (int j = 0; j < KL; ++j) te(j) = slot_init(j, ns);
    temin = ns > 0 ? -INF : INF;
    const float lip = ex[rm::EX_LIP];
    sig2 = 2.0f * ex[rm::EX_SIGMA];
    const float rdl = __builtin_amdgcn_sqrtf(dot(rd, rd)) * (1.0f + 0x1p-16f);  // >= |rd|
    const float rd1 = ((fabsf(rd.x) + fabsf(rd.y)) + fabsf(rd.z)) * (1.0f + 0x1p-16f);
    sl0 = (((fabsf(ro.x) + fabsf(ro.y)) + fabsf(ro.z)) + ex[rm::EX_S]) * (1.0f + 0x1p-16f);
    // the slack grows by sig2 |rd|_1 per unit of t
    inv = (1.0f - 0x1p-10f) * __builtin_amdgcn_rcpf((1.0f + lip) * rdl + sig2 * rd1) * (1.0f - 0x1p-16f);
    grow = (__builtin_fmaf(lip, rdl, 1.0f) + sig2 * rd1) * (1.0f + 0x1p-10f);
    dprev = INF;
  }
  // True when some lane's re-test is due at its t (uniform).
  __device__ __forceinline__ bool due(float t) const { return ns > 0 && wany(!(t < temin)); }
  // A step when no lane's re-test is due: the `always` entries.
  __device__ __forceinline__ float fast(const Table& S, f3 p, int& best) {
    dprev = S.dist_mask(p, always, best);
    return dprev;
  }
  // sdf(p(t)) and its opU winner; p = ro + rd t as the caller computed it.
  __device__ __forceinline__ float dist(const Table& S, f3 p, float t, int& best) {
    uint32_t wmask = always;
#ifdef RM_TABLE_STATIC
    // A step with no re-test evaluates the `always` entries under their
    // compile-time masks: no per-entry mask tests (-4.4 % per cfg3 frame; the
    // generic kernel's ctz loop measured 5.5 % slower split this way).
    if (!(ns > 0 && wany(!(t < temin)))) {
      dprev = S.dist_mask(p, always, best);
      return dprev;
    }
    {
#else
    if (ns > 0 && wany(!(t < temin))) {
#endif
      const float sl = sig2 * (((fabsf(p.x) + fabsf(p.y)) + fabsf(p.z)) + sl0) * (1.0f + 0x1p-10f);
      float U = __builtin_fmaf(dprev, grow, sl);
#ifdef RM_TABLE_STATIC
      RM_TS_UNROLL
      for (int k = 0; k < S.n; ++k)
        if (S.type(k) == RM_PRIM_PLANE) U = gmin(U, prim_dist(S.entry(k), RM_PRIM_PLANE, p, S.blend, S.omblend));
#else
      if (S.fp >= 0) {
        U = gmin(U, S.plane_fast(p));
      } else {
        for (uint32_t pm = __float_as_uint(ex[rm::EX_PLANE_MASK]); pm; pm &= pm - 1u)
          U = gmin(U, prim_dist(S.entry(__builtin_ctz(pm)), RM_PRIM_PLANE, p, S.blend, S.omblend));
      }
#endif
#pragma unroll
      for (int j = 0; j < KL; ++j) {
        if (j < ns && wany(!(t < te(j)))) {
          const int k = (int)ex[rm::EX_SLOTS + j];
#ifndef RM_TABLE_STATIC
          // the slot's ball gathered at staging: one 16-byte LDS read (-0.9 / -1.9 %
          // per cfg3 / cfg2 frame against its four words read through the entry)
          const float4 B4 = reinterpret_cast<const float4*>(S.sb)[j];
          const float B[4] = {B4.x, B4.y, B4.z, RM_SBR(B4.w)};
#else
          const float* B = S.entry(k) + rm::TW_BALL;
#endif
          const float bx = p.x - B[0], by = p.y - B[1], bz = p.z - B[2];
          const float lb = __builtin_fmaf(__builtin_amdgcn_sqrtf((bx * bx + by * by) + bz * bz),
                                          1.0f - 0x1p-12f, -B[3]);
          const float g = lb - U - sl;
          // the later of the old expiry and the budget's end; an expired lane
          // whose g <= 0 (or too small to move t) keeps te <= t and evaluates
          // now, an idle lane keeps te > t; a NaN bound leaves te as it was and
          // a NaN t evaluates (the negated compare).  One max and one compare
          // fewer than max(te, max(t + g inv, t)) and `expired & !(g > 0)`
          // (round 3, VALU issue slots: DESIGN.md §6).
          te(j) = __builtin_fmaxf(te(j), __builtin_fmaf(g, inv, t));
          if (wany(!(t < te(j)))) wmask |= 1u << k;
        }
      }
      temin = te(0);
#pragma unroll
      for (int j = 1; j < KL; ++j) temin = __builtin_fminf(temin, te(j));
    }
    dprev = S.dist_mask(p, wmask, best);
    return dprev;
  }
};

// An opaque VGPR copy: a uniform value used as a VGPR operand (an f32 op with an
// SGPR operand takes a whole VALU issue slot, with VGPRs two pair in one,
// DESIGN.md §6), and the RM_TDBL_<PHASE> probes' opaque inputs (diagnostic
// builds, tools/ab_kernel.py: a phase run twice, its marginal cost per frame).
__device__ __forceinline__ float topaque(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ f3 topaque(f3 v) { return mk(topaque(v.x), topaque(v.y), topaque(v.z)); }

struct THit {
  float t;  // -1: the dummy RayHit {-1, 0, -1, 1.0} (glsl:128)
  int id;
  float material;
  f3 color;
  float d;  // a hit's last distance: sdf at the hit point itself (GetNormal's centre sample)
};

// ---- the built-in kernel's march shape for reference-shaped tables -------------
// A table whose bounded entries all sit in lazy slots and whose one plane is its
// last entry, axis-aligned (q.y n_y + w, as the reference's floor): the
// production march then runs scene_lazy's block (rm_scene.hpp) over the table
// instead of TLazy -- in the specialised kernels (the table folded in), and in
// the generic kernel's reference-shaped instances (SL, chosen on the host:
// rm::table_slazy; one march per instance keeps its registers as they were).
// Per step only p.y and the plane value; the block is entered when some lane's
// expiry passes t, forms p.x / p.z, the slack from a line in t and re-tests the
// due slots in table order, evaluating an entry exactly where its new expiry
// does not pass t.  Same values, fewer instructions: the culling only skips
// entries proven strictly above the minimum, as TLazy's.
#ifdef RM_TABLE_STATIC
__device__ __forceinline__ bool slazy_table(const Table& S) {
  const float* ex = S.exits();
  const int kp = S.n - 1;
  if (ex[rm::EX_VALID] == 0.0f || ex[rm::EX_NPLANES] != 1.0f || S.type(kp) != RM_PRIM_PLANE) return false;
  const float* P = S.entry(kp);
  if (__float_as_int(P[rm::TW_SWIZZLE]) != RM_SWIZZLE_XYZ) return false;
  if (!(P[rm::TW_P] == 0.0f && P[rm::TW_P + 2] == 0.0f)) return false;
  if ((int)ex[rm::EX_NSLOTS] != S.n - 1) return false;  // every other entry tracked ...
  RM_TS_UNROLL
  for (int j = 0; j < S.n - 1; ++j)
    if ((int)ex[rm::EX_SLOTS + j] != j) return false;  // ... slot j holding entry j
  return true;
}

// gmarch's condition (a specialised table, compile-time): valid exit bounds and
// at least one plane.
__device__ __forceinline__ bool glazy_table(const Table& S) {
  const float* ex = S.exits();
  return ex[rm::EX_VALID] != 0.0f && ex[rm::EX_NPLANES] >= 1.0f;
}
#endif

// Expiries by TLazy's argument (above), in scene_lazy's form:
//   * the slack is the line s0 + s1 t >= TLazy's sl(p(t)): |p|_1 <= (|ro|_1 +
//     |rd|_1 t)(1 + 2^-22) for the float p, so sig2 (|p|_1 + |ro|_1 + S)(1 + 2^-10)
//     <= sig2 (2 |ro|_1 + S)(1 + 2^-9) + sig2 |rd|_1 (1 + 2^-9) t; s0, s1 carry
//     (1 + 2^-8) for their own roundings.  A larger slack gives a smaller gap.
//   * the budget is the plane's: its value P is linear along the ray with slope
//     n_y rd.y exactly and bounds the minimum from above (TLazy's U may be any
//     such bound), so an entry whose gap (lb - P) - sl is positive stays above
//     the minimum while the gap, shrinking at most at |rd| + n_y rd.y + s1 per
//     unit of t, lasts (invp = 0 when that rate is not positive: no budget).
//     TLazy's own budget, at rate inv, serves the host's step-0 gaps.
//   * the exact evaluations of a step run inline in table order against the
//     running minimum m (the plane first: it is the last entry and wins ties).
template <int KL>
struct SLazy {
  float te[KL];
  float temin, s0, s1, inv, invp;
  int idb;  // the entry the last block's values made the winner (the plane: n - 1)
};

// The minimum over the expiries, three at a time (v_min3_f32): the first ns
// (a compile-time count) in a specialised kernel; all KL in the generic one,
// whose unused slots hold +inf (a runtime bound would index the array, which
// then lives in scratch).
template <int KL>
__device__ __forceinline__ float slot_min(const float (&te)[KL], int ns) {
#ifndef RM_TABLE_STATIC
  ns = KL;
#endif
  float m = te[0];
  int j = 1;
  #pragma unroll
  for (; j + 1 < KL && j + 1 < ns; j += 2) m = vmin3(m, te[j], te[j + 1]);
  #pragma unroll
  for (; j < KL && j < ns; ++j) m = vmin(m, te[j]);
  return m;
}

template <int KL>
__device__ __forceinline__ THit smarch(const Table& S, f3 ro, f3 rd, bool reflected, const float* prep) {
  ro = topaque(ro);
  const float* ex = S.exits();
  const int ns = S.n - 1, kp = S.n - 1;
  const float tmax = reflected ? 200.0f : 400.0f;
  const int nmax = reflected ? 256 : 512;
  const float T = table_exit_T(ex, MISS_C, 0.0f, ro, rd);
  // the plane's value at height y, prim_dist's float operations (q.x, q.z unused;
  // the generic kernel's fast plane is the same arithmetic on staged registers)
#ifdef RM_TABLE_STATIC
  const float* PL = S.entry(kp);
  auto plane = [&](float y) { return prim_dist(PL, RM_PRIM_PLANE, mk(0.0f, y, 0.0f), S.blend, S.omblend); };
#else
  // the reference's floor (fpunit) as the common path, p.y + w with w in a VGPR
  // (an SGPR operand takes a whole issue slot), other planes overwrite it (round 6:
  // -0.5 % per cfg3 frame, -1.5 % cfg2; the step's value no longer needs a copy
  // to merge two paths, profiles/r06_ab_tnu*.txt)
  const float pw = topaque(S.fpw);
  auto plane = [&](float y) {
    float m = y + pw;
    if (!S.fpunit) m = S.plane_fast(mk(0.0f, y, 0.0f));
    return m;
  };
#endif
  SLazy<KL> lz;
  {
    const float sig2 = 2.0f * ex[rm::EX_SIGMA];
    const float rdl = __builtin_amdgcn_sqrtf(dot(rd, rd)) * (1.0f + 0x1p-16f);  // >= |rd|
    const float rd1 = ((fabsf(rd.x) + fabsf(rd.y)) + fabsf(rd.z)) * (1.0f + 0x1p-16f);
    const float ro1 = (fabsf(ro.x) + fabsf(ro.y)) + fabsf(ro.z);
    lz.s0 = sig2 * (2.0f * ro1 + ex[rm::EX_S]) * ((1.0f + 0x1p-9f) * (1.0f + 0x1p-8f));
    lz.s1 = sig2 * rd1 * ((1.0f + 0x1p-9f) * (1.0f + 0x1p-8f));
    lz.inv = (1.0f - 0x1p-10f) *
             __builtin_amdgcn_rcpf((1.0f + ex[rm::EX_LIP]) * rdl + sig2 * rd1) * (1.0f - 0x1p-16f);
    // the plane's world normal is (0, n_y, 0): its slope along the ray is n_y rd.y
    // (one rounding, far inside the 2^-8 added to s1)
    const float ratep = (rdl + ex[rm::EX_PLANES + 1] * rd.y) + lz.s1 * (1.0f + 0x1p-8f);
    lz.invp = ratep > 0.0f ? (1.0f - 0x1p-10f) * __builtin_amdgcn_rcpf(ratep) * (1.0f - 0x1p-16f) : 0.0f;
    lz.idb = kp;
  }
  float t = 0.0f, dl = 0.0f;
  int i0 = 1;  // sdf evaluations the first loop step brings the count to
  if (prep && prep[rm::TP_VALID] != 0.0f) {
    // step 0 at the camera, evaluated on the host (tmarch above); the gaps are
    // TLazy's, their expiries at TLazy's rate
    #pragma unroll
    for (int j = 0; j < KL; ++j) lz.te[j] = j < ns ? __builtin_fmaxf(prep[rm::TP_G + j] * lz.inv, 0.0f) : __builtin_huge_valf();
    dl = prep[rm::TP_D0];
    t = dl;
    i0 = 2;
  } else {
    #pragma unroll
    for (int j = 0; j < KL; ++j) lz.te[j] = slot_init(j, ns);
  }
  lz.temin = slot_min(lz.te, ns);
  if (!(t <= T)) return THit{-1.0f, -1, 1.0f, mk(0.0f, 0.0f, 0.0f), 0.0f};

  // sdf(ro + rd t): the plane, and the block when some lane's expiry has passed
  auto step = [&](float tt) {
    const float py = ro.y + rd.y * tt;
    float m = plane(py);
    if (wany(tt >= lz.temin)) {
      const float sl = __builtin_fmaf(lz.s1, tt, lz.s0);
      const float pl = m + sl;
      const f3 p = mk(ro.x + rd.x * tt, py, ro.z + rd.z * tt);
      int idp = kp;
      #pragma unroll
      for (int j = 0; j < KL; ++j) {
        if (j >= ns || !wany(tt >= lz.te[j])) continue;
        // (a compile-time test in the specialised kernels; a uniform branch in the
        // generic one's 5-slot instance since round 6: -1 % per cfg3 frame,
        // profiles/r06_ab_gen2.txt; in the 8-slot instance it makes the batch kernel
        // copy its FrameBatch argument to scratch, 12 KB per lane)
#ifndef RM_TABLE_STATIC
        if (KL <= rm::TABLE_FEW_SLOTS)
#endif
        if (S.type(j) == RM_PRIM_TORUS) {
          // evaluated instead of re-tested, as the built-in march does (rm_scene.hpp
          // scene_lazy): the exact value is the budget's lower bound
          const float v = prim_dist<kBoundedPoints>(S.entry(j), RM_PRIM_TORUS, p, S.blend, S.omblend);
          idp = (v <= m) ? j : idp;
          m = vmin(m, v);
          lz.te[j] = vmax(__builtin_fmaf(v - pl, lz.invp, tt), lz.te[j]);
          continue;
        }
#ifdef RM_TABLE_STATIC
        const float* B = S.entry(j) + rm::TW_BALL;
#else
        const float4 B4 = reinterpret_cast<const float4*>(S.sb)[j];  // the slot's ball, staged
        const float B[4] = {B4.x, B4.y, B4.z, RM_SBR(B4.w)};
#endif
        const float bx = p.x - B[0], by = p.y - B[1], bz = p.z - B[2];
        const float lb = __builtin_fmaf(__builtin_amdgcn_sqrtf((bx * bx + by * by) + bz * bz),
                                        1.0f - 0x1p-12f, -B[3]);
        // (the plane budget alone, as scene_lazy's re-test: rm_scene.hpp)
        lz.te[j] = vmax(__builtin_fmaf(lb - pl, lz.invp, tt), lz.te[j]);
        if (lz.te[j] <= tt) {  // opU in table order, later entries win ties
          const float v = prim_dist<kBoundedPoints>(S.entry(j), S.type(j), p, S.blend, S.omblend);
          idp = (v <= m) ? j : idp;
          m = vmin(m, v);
        }
      }
      lz.temin = slot_min(lz.te, ns);
      lz.idb = idp;
    }
    return m;
  };
  float tp = t;
  auto run = [&](auto esc, auto useT) {
    if (!decltype(esc)::value && !decltype(useT)::value) {
      // downward waves: t advances at the top of the step and the loop carries
      // only the step's (t, d) (the built-in march's form, rm_kernels.hip; round
      // 6: generic -0.5 %, specialised -0.4 % per cfg3 frame,
      // profiles/r06_ab_thadd_*.txt)
      float dp = 0.0f;
      for (int i = i0;; ++i) {
        t = t + dp;
        const float d = step(t);
        dp = d;
        if ((d < 0.000001f * t) | (i >= nmax)) break;
      }
      dl = dp;
      return;
    }
    for (int i = i0;; ++i) {
      const float d = step(t);
      bool e = d < 0.000001f * t;
      dl = d;
      tp = t;
      t = t + d;
      if (decltype(useT)::value) e = e | !(t <= T);
      if (decltype(esc)::value) e = e | (d > tmax);
      if (e | (i >= nmax)) break;
    }
    t = tp;
  };
  const bool useT = wany(!(T == __builtin_huge_valf()));
  // (the generic 8-slot instance keeps its escape compare: the proof's registers
  // spilled it, 12 B of scratch per lane)
  if ((kBoundedPoints || KL <= rm::TABLE_FEW_SLOTS) && __all(S.no_escape(ro, rd, tmax))) {
    if (useT) run(No(), Yes());
    else run(No(), No());
  } else {
    if (useT) run(Yes(), Yes());
    else run(Yes(), No());
  }
  if (dl < 0.000001f * t) {
    // the winner: the plane (last in opU order, it wins a tie) exactly when the
    // hit step's distance is its value; otherwise the block ran at this step and
    // idb is its winner (lazy_id, rm_scene.hpp)
    const f3 p = add(ro, muls(rd, t));
    int k = dl != plane(p.y) ? lz.idb : kp;
    // the winner as a 32-bit index here: LLVM otherwise carried its zero-extended
    // 64-bit table offset through the bounce loop, in scratch (round 5)
    asm volatile("" : "+v"(k));
    return THit{t, S.id(k), S.material(k), S.color(k, p), dl};
  }
  return THit{-1.0f, -1, 1.0f, mk(0.0f, 0.0f, 0.0f), 0.0f};
}

// ---- the block shape for any plane-bounded table (round 5) ----
// smarch needs the reference's shape (one axis-aligned plane, last, every other
// entry in a slot).  gmarch takes any table with valid exit bounds and at least
// one plane: several planes of any orientation anywhere in the table, and more
// bounded entries than the slots (the untracked ones are evaluated at every
// step, as the planes).  Per step: p(t), the always-evaluated entries (EX_EVAL_
// MASK) into the running minimum m, the planes' minimum U among them; the block
// when some lane's expiry passes t re-tests the due slots against U with the
// planes' budget and evaluates an entry where its new expiry does not pass t.
//   * budget: every plane's exact value is linear along the ray, slope
//     dot(rd, n'_j) (EX_PLANES world normals), so U(t') <= U(t) + s_max (t' - t)
//     with s_max the largest slope, and a slot's ball bound falls at most |rd|
//     per unit of t: a positive gap (lb - U) - sl lasts while it shrinks at
//     |rd| + s_max + s1 (the float error of the slopes is far inside the 2^-8
//     added to s1, as in smarch);
//   * the distance is exact: culled entries are strictly above the minimum;
//   * the opU winner is taken once, at the hit: every entry evaluated at the hit
//     point in table order (dist_mask), ties to the later entry -- the winner of
//     the reference's sdf() at that point.
template <int KL>
__device__ __forceinline__ THit gmarch(const Table& S, f3 ro, f3 rd, bool reflected, const float* prep) {
  ro = topaque(ro);
  const float* ex = S.exits();
  const int ns = (int)ex[rm::EX_NSLOTS];
  const int np = (int)ex[rm::EX_NPLANES];
  const uint32_t always = __float_as_uint(uword(ex + rm::EX_EVAL_MASK));
  const float tmax = reflected ? 200.0f : 400.0f;
  const int nmax = reflected ? 256 : 512;
  const float T = table_exit_T(ex, MISS_C, 0.0f, ro, rd);
  SLazy<KL> lz;
  {
    const float sig2 = 2.0f * ex[rm::EX_SIGMA];
    const float rdl = __builtin_amdgcn_sqrtf(dot(rd, rd)) * (1.0f + 0x1p-16f);  // >= |rd|
    const float rd1 = ((fabsf(rd.x) + fabsf(rd.y)) + fabsf(rd.z)) * (1.0f + 0x1p-16f);
    const float ro1 = (fabsf(ro.x) + fabsf(ro.y)) + fabsf(ro.z);
    lz.s0 = sig2 * (2.0f * ro1 + ex[rm::EX_S]) * ((1.0f + 0x1p-9f) * (1.0f + 0x1p-8f));
    lz.s1 = sig2 * rd1 * ((1.0f + 0x1p-9f) * (1.0f + 0x1p-8f));
    lz.inv = (1.0f - 0x1p-10f) *
             __builtin_amdgcn_rcpf((1.0f + ex[rm::EX_LIP]) * rdl + sig2 * rd1) * (1.0f - 0x1p-16f);
    float smax = -__builtin_huge_valf();
    RM_TS_UNROLL
    for (int j = 0; j < rm::EX_MAX_PLANES; ++j)
      if (j < np) smax = fmaxf(smax, dot(rd, mk(ex[rm::EX_PLANES + 4 * j], ex[rm::EX_PLANES + 4 * j + 1],
                                                 ex[rm::EX_PLANES + 4 * j + 2])));
    const float ratep = (rdl + smax) + lz.s1 * (1.0f + 0x1p-8f);
    lz.invp = ratep > 0.0f ? (1.0f - 0x1p-10f) * __builtin_amdgcn_rcpf(ratep) * (1.0f - 0x1p-16f) : 0.0f;
  }
  float t = 0.0f, dl = 0.0f;
  int i0 = 1;
  if (prep && prep[rm::TP_VALID] != 0.0f) {
    // step 0 at the camera, evaluated on the host (table_prep_host: slot j's gap
    // with U = the planes at the camera), at TLazy's rate as in smarch
    #pragma unroll
    for (int j = 0; j < KL; ++j) lz.te[j] = j < ns ? __builtin_fmaxf(prep[rm::TP_G + j] * lz.inv, 0.0f) : __builtin_huge_valf();
    dl = prep[rm::TP_D0];
    t = dl;
    i0 = 2;
  } else {
    #pragma unroll
    for (int j = 0; j < KL; ++j) lz.te[j] = slot_init(j, ns);
  }
  lz.temin = slot_min(lz.te, ns);
  if (!(t <= T)) return THit{-1.0f, -1, 1.0f, mk(0.0f, 0.0f, 0.0f), 0.0f};

  auto step = [&](float tt) {
    const f3 p = mk(ro.x + rd.x * tt, ro.y + rd.y * tt, ro.z + rd.z * tt);
    float m = __builtin_huge_valf(), U = __builtin_huge_valf();
#ifdef RM_TABLE_STATIC
    RM_TS_UNROLL
    for (int k = 0; k < S.n; ++k) {
      if (!((always >> k) & 1u)) continue;
      const float v = prim_dist<kBoundedPoints>(S.entry(k), S.type(k), p, S.blend, S.omblend);
      m = vmin(m, v);
      if (S.type(k) == RM_PRIM_PLANE) U = vmin(U, v);
    }
#else
    if (S.fp >= 0 && always == (1u << S.fp)) {
      m = U = S.plane_fast(p);  // one plane and every bounded entry in a slot
    } else {
      for (uint32_t w = always; w; w &= w - 1u) {
        const int k = __builtin_ctz(w);
        const int ty = S.type(k);
        const float v = prim_dist(S.entry(k), ty, p, S.blend, S.omblend);
        m = vmin(m, v);
        if (ty == RM_PRIM_PLANE) U = vmin(U, v);
      }
    }
#endif
    if (wany(tt >= lz.temin)) {
      const float sl = __builtin_fmaf(lz.s1, tt, lz.s0);
      const float pl = U + sl;
      // the re-tests (unrolled over the slots), then the entries some lane must
      // evaluate (a lane whose expiry passes t takes a value proven above its
      // minimum: m is unchanged), in one loop over their mask
      uint32_t due = 0;
      #pragma unroll
      for (int j = 0; j < KL; ++j) {
        if (j >= ns || !wany(tt >= lz.te[j])) continue;
#ifdef RM_TABLE_STATIC
        const float* B = S.entry((int)ex[rm::EX_SLOTS + j]) + rm::TW_BALL;
#else
        const float4 B4 = reinterpret_cast<const float4*>(S.sb)[j];  // the slot's ball, staged
        const float B[4] = {B4.x, B4.y, B4.z, RM_SBR(B4.w)};
#endif
        const float bx = p.x - B[0], by = p.y - B[1], bz = p.z - B[2];
        const float lb = __builtin_fmaf(__builtin_amdgcn_sqrtf((bx * bx + by * by) + bz * bz),
                                        1.0f - 0x1p-12f, -B[3]);
        lz.te[j] = vmax(__builtin_fmaf(lb - pl, lz.invp, tt), lz.te[j]);
        if (wany(lz.te[j] <= tt)) due |= 1u << j;
      }
      lz.temin = slot_min(lz.te, ns);
#ifdef RM_TABLE_STATIC
      RM_TS_UNROLL
      for (int j = 0; j < KL; ++j) {
        if (j >= ns || !((due >> j) & 1u)) continue;
        const int k = (int)ex[rm::EX_SLOTS + j];
        m = vmin(m, prim_dist<kBoundedPoints>(S.entry(k), S.type(k), p, S.blend, S.omblend));
      }
#else
      for (; due; due &= due - 1u) {
        const int k = (int)ex[rm::EX_SLOTS + __builtin_ctz(due)];
        m = vmin(m, prim_dist(S.entry(k), S.type(k), p, S.blend, S.omblend));
      }
#endif
    }
    return m;
  };
  float tp = t;
  auto run = [&](auto esc, auto useT) {
    if (!decltype(esc)::value && !decltype(useT)::value) {  // (smarch's form)
      float dp = 0.0f;
      for (int i = i0;; ++i) {
        t = t + dp;
        const float d = step(t);
        dp = d;
        if ((d < 0.000001f * t) | (i >= nmax)) break;
      }
      dl = dp;
      return;
    }
    for (int i = i0;; ++i) {
      const float d = step(t);
      bool e = d < 0.000001f * t;
      dl = d;
      tp = t;
      t = t + d;
      if (decltype(useT)::value) e = e | !(t <= T);
      if (decltype(esc)::value) e = e | (d > tmax);
      if (e | (i >= nmax)) break;
    }
    t = tp;
  };
  const bool useT = wany(!(T == __builtin_huge_valf()));
  if (__all(S.no_escape(ro, rd, tmax))) {
    if (useT) run(No(), Yes());
    else run(No(), No());
  } else {
    if (useT) run(Yes(), Yes());
    else run(Yes(), No());
  }
  if (dl < 0.000001f * t) {
    const f3 p = add(ro, muls(rd, t));
    int k;
    (void)S.dist_mask(p, S.n >= 32 ? 0xffffffffu : (1u << S.n) - 1u, k);
    asm volatile("" : "+v"(k));  // (a 32-bit index: smarch's note)
    return THit{t, S.id(k), S.material(k), S.color(k, p), dl};
  }
  return THit{-1.0f, -1, 1.0f, mk(0.0f, 0.0f, 0.0f), 0.0f};
}

// RayMarch glsl:125-142 / reflectedRay glsl:144-161.  SL: the production
// march's shape, 0 TLazy (below), 1 smarch (reference-shaped tables), 2 gmarch
// (any plane-bounded table): the generic kernel's instance, chosen on the host
// (rm::table_shape); a specialised table's shape is a compile-time test.
template <bool COUNT, int KL, int SL = 0>
__device__ RM_TS_INLINE THit tmarch(const Table& S, f3 ro, f3 rd, bool reflected, TCnt& c,
                                   const float* prep = nullptr) {
#ifdef RM_TABLE_STATIC
  if (!COUNT && slazy_table(S)) return smarch<KL>(S, ro, rd, reflected, prep);
  if (!COUNT && glazy_table(S)) return gmarch<KL>(S, ro, rd, reflected, prep);
#else
  if (!COUNT && SL == 1) return smarch<KL>(S, ro, rd, reflected, prep);
  if (!COUNT && SL == 2) return gmarch<KL>(S, ro, rd, reflected, prep);
#endif
  // ro in VGPRs (a primary ray's ro is the camera, uniform): every step's p(t)
  // then pairs for dual issue instead of taking a whole slot per component, and
  // the generic kernel spills less (28 -> 12 B of scratch per lane): -2.9 % per
  // cfg3 frame (round 3).  The fast plane's parameters moved to
  // VGPRs the same way measured +0.5 % against this (more spills).
  ro = topaque(ro);
  const float tmax = reflected ? 200.0f : 400.0f;
  const int nmax = reflected ? 256 : 512;
  float t = 0.0f;
  int i0 = 0;  // steps already taken
  // provable miss (table_exit_T): production stops there; the counting build
  // runs on and poisons the colour with NaN should the ray hit after all
  const float T = table_exit_T(S.exits(), MISS_C, 0.0f, ro, rd);
  bool proven = false;
  TLazy<KL> lz(S, ro, rd);
  if (prep && prep[rm::TP_VALID] != 0.0f) {
    // Primary rays: step 0 is at the camera for every pixel; the host evaluated
    // it (table_prep_host: d0 exact, the slots' gaps as TLazy::dist's step-0
    // re-test forms them with U = the planes at the camera).  Each lane turns
    // the gaps into expiries with its own rate: te = max(fma(g, inv, 0), 0).
    const float d0 = prep[rm::TP_D0];
#pragma unroll
    for (int j = 0; j < KL; ++j)
      if (j < lz.ns) lz.te(j) = __builtin_fmaxf(prep[rm::TP_G + j] * lz.inv, 0.0f);
    lz.temin = lz.te(0);
#pragma unroll
    for (int j = 1; j < KL; ++j) lz.temin = __builtin_fminf(lz.temin, lz.te(j));
    lz.dprev = d0;
    t = d0;
    i0 = 1;
    if (COUNT) c.march++;
  }
  if (!COUNT) {
    // Production: one exit at the latch (as march<false>, rm_kernels.hip).  The
    // step at t runs when t <= T and fewer than nmax steps were taken; after it,
    // the march ends on hit | escape | t + d past T (a NaN t + d fails the
    // compare; the reference would march on with t = NaN to the cap, also a
    // miss) | the step cap.  The last step's t is kept, so its hit test re-forms.
    if (!(t <= T)) return THit{-1.0f, -1, 1.0f, mk(0.0f, 0.0f, 0.0f), 0.0f};
    float tp = 0.0f, d = 0.0f;
    int k = 0;
    // Variants of the loop (as march<false>'s): the T compare is dropped when T
    // is +inf on every lane (a NaN t then marches on to the cap, a miss as
    // before), the escape test when no lane can escape (S.no_escape).
    // A specialised table's march is written as two loops: a step that may
    // re-test, then steps while no lane's re-test is due (the lazy state is
    // loop-invariant there, so the compiler keeps it in place instead of copying
    // it around the back edges: -7 % per cfg3 frame).  A lane that ends leaves
    // both.
    auto run = [&](auto esc, auto useT) {
      int i = 1 + i0;
      bool ex = false;
      auto latch = [&]() {
        tp = t;
        t = t + d;
        ex = (d < 0.000001f * tp) | (i >= nmax);
        if (decltype(useT)::value) ex = ex | !(t <= T);
        if (decltype(esc)::value) ex = ex | (d > tmax);
        ++i;
      };
#ifdef RM_TABLE_STATIC
      do {
        d = lz.dist(S, add(ro, muls(rd, t)), t, k);
        latch();
        while (!ex && !lz.due(t)) {
          d = lz.fast(S, add(ro, muls(rd, t)), k);
          latch();
        }
      } while (!ex);
#else
      // (the generic kernel measured 6 % slower with the two loops)
      do {
        d = lz.dist(S, add(ro, muls(rd, t)), t, k);
        latch();
      } while (!ex);
#endif
    };
    const bool useT = wany(!(T == __builtin_huge_valf()));
    if (__all(S.no_escape(ro, rd, tmax))) {
      if (useT) run(No(), Yes());
      else run(No(), No());
    } else {
      if (useT) run(Yes(), Yes());
      else run(Yes(), No());
    }
    if (d < 0.000001f * tp) {
      const f3 p = add(ro, muls(rd, tp));
      return THit{tp, S.id(k), S.material(k), S.color(k, p), d};
    }
    return THit{-1.0f, -1, 1.0f, mk(0.0f, 0.0f, 0.0f), 0.0f};
  }
  for (int i = i0; i < nmax; ++i) {
    if (t > T) {
      if (!COUNT) break;
      proven = true;
    }
    const f3 p = add(ro, muls(rd, t));
    int k;
    const float d = lz.dist(S, p, t, k);
    if (COUNT) {
      if (reflected) c.reflect++;
      else c.march++;
    }
    if (d < 0.000001f * t)
      return THit{t, S.id(k), S.material(k),
                  (COUNT && proven) ? mk(__builtin_nanf(""), 0.0f, 0.0f) : S.color(k, p), d};
    if (d > tmax) break;
    t += d;
  }
  return THit{-1.0f, -1, 1.0f, mk(0.0f, 0.0f, 0.0f), 0.0f};
}

// GetNormal glsl:278-288
template <bool COUNT>
// With have_c0 the centre sample sdf(pos) is c0, the march's last distance at
// this very point (render's pos == the march's last p, glsl:226 vs :129).
__device__ RM_TS_INLINE f3 tnormal(const Table& S, f3 pos, TCnt& c, bool have_c0 = false,
                                   float c0 = 0.0f) {
  if (COUNT) c.normals++;
  float x, y, z;
  S.normal_samples(pos, have_c0, c0, x, y, z);
  return tnormalize(subs(mk(x, y, z), c0));
}

// softshadow glsl:201-216
template <bool COUNT, int KL>
__device__ RM_TS_INLINE float tshadow(const Frame& F, const Table& S, f3 ro, f3 rd, TCnt& c) {
  float res = 1.0f, t = 0.0f;
  const float c_sh = F.shc;  // (1 + 2^-9) / k (1 + 2^-12), 0 for k = +inf (host, make_frame)
  const float T = table_exit_T(S.exits(), c_sh, 0.001f, ro, rd);
  TLazy<KL> lz(S, ro, rd);
  for (int i = 0; i < 16; ++i) {
    if (t > T) {  // the remaining steps are no-ops (table_exit_T)
      if (COUNT) c.shadow += 16 - i;
      return res;
    }
    int k;
    const float h = lz.dist(S, add(ro, muls(rd, t)), t, k);
    if (COUNT) c.shadow++;
    if (h < 0.001f) return 0.05f;
    res = shadow_min(res, F.k, h, t);  // min(res, k h / t) (rm_scene.hpp: the divide only when it can matter)
    t += h;
  }
  return res;
}

// bounce glsl:163-199.  Once prevObject is MATTE every later iteration leaves
// the colour unchanged (glsl:181, 189-190): the loop stops there.
template <bool COUNT, int KL, int SL = 0>
__device__ RM_TS_INLINE f3 tbounce(const Frame& F, const Table& S, f3 rayDir, f3 pos, f3 normal, f3 color,
                      const THit& primary, TCnt& c) {
  float prevMat = primary.material;
  f3 prevColor = primary.color;
  const f3 lpos = mk(F.lpos[0], F.lpos[1], F.lpos[2]);
  for (int i = 1; i <= F.bounces; ++i) {
    if (prevMat == 0.0f) break;
    rayDir = reflect(rayDir, normal);
    THit h = tmarch<COUNT, KL, SL>(S, add(pos, muls(normal, 0.001f)), rayDir, true, c);
#ifdef RM_TDBL_BMARCH
    if (!COUNT) {
      const THit h2 = tmarch<COUNT, KL, SL>(S, topaque(add(pos, muls(normal, 0.001f))), rayDir, true, c);
      h.t = (h2.t == h.t) ? h.t : __builtin_nanf("");
    }
#endif
    pos = add(pos, muls(rayDir, h.t));
    // the normal of a miss on the last bounce is never read
    if (h.t != -1.0f || i < F.bounces) normal = tnormal<COUNT>(S, pos, c);
#ifdef RM_TDBL_NORMAL
    if (!COUNT && (h.t != -1.0f || i < F.bounces)) {
      const f3 n2 = tnormal<COUNT>(S, topaque(pos), c);
      normal = mk(fminf(normal.x, n2.x), fminf(normal.y, n2.y), fminf(normal.z, n2.z));
    }
#endif
    if (h.t == -1.0f) {
      h.color = subs(mk(0.36f, 0.36f, 0.60f), rayDir.y * 0.2f);
    } else {
      if (COUNT) c.lights++;
      h.color = point_light(F, h.color, normal, pos);
    }
    // (x / i stays a division here: the built-in kernel's power-of-two products,
    // rm_kernels.hip bounce, make the generic kernel spill 45 VGPRs -- 588 B of
    // scratch per lane instead of 28, round 4)
    if (h.id == 7 && i < 3) {  // prevObject.material != MATTE here
      float sh = tshadow<COUNT, KL>(F, S, add(pos, muls(normal, 0.02f)), sub(lpos, pos), c);
#ifdef RM_TDBL_SHADOW
      if (!COUNT) sh = fminf(sh, tshadow<COUNT, KL>(F, S, topaque(add(pos, muls(normal, 0.02f))), sub(lpos, pos), c));
#endif
      color = muls(color, sh / (float)i);
    }
    color = add(color, divs(mul(h.color, prevColor), (float)i));
    prevColor = h.color;
    prevMat = h.material;
  }
  return color;
}

// render glsl:218-251
template <bool COUNT, int KL, int SL = 0>
__device__ RM_TS_INLINE f3 trender(const Frame& F, const Table& S, f3 ro, f3 rd, TCnt& c) {
  f3 color = subs(mk(0.30f, 0.36f, 0.60f), rd.y * 0.2f);
  THit h = tmarch<COUNT, KL, SL>(S, ro, rd, false, c, F.prepv);
#ifdef RM_TDBL_MARCH
  if (!COUNT) {
    const THit h2 = tmarch<COUNT, KL, SL>(S, topaque(ro), rd, false, c, F.prepv);
    h.t = (h2.t == h.t) ? h.t : __builtin_nanf("");
  }
#endif
  if (h.t != -1.0f) {
    const f3 pos = add(ro, muls(rd, h.t));
    f3 normal = tnormal<COUNT>(S, pos, c, true, h.d);
#ifdef RM_TDBL_NORMAL
    if (!COUNT) {
      const f3 n2 = tnormal<COUNT>(S, topaque(pos), c, true, h.d);
      normal = mk(fminf(normal.x, n2.x), fminf(normal.y, n2.y), fminf(normal.z, n2.z));
    }
#endif
    if (COUNT) c.lights++;
    color = point_light(F, h.color, normal, pos);
    if (h.id == 7) {
      const f3 lpos = mk(F.lpos[0], F.lpos[1], F.lpos[2]);
      float sh = tshadow<COUNT, KL>(F, S, add(pos, muls(normal, 0.02f)), sub(lpos, pos), c);
#ifdef RM_TDBL_SHADOW
      if (!COUNT) sh = fminf(sh, tshadow<COUNT, KL>(F, S, topaque(add(pos, muls(normal, 0.02f))), sub(lpos, pos), c));
#endif
      return gamma(muls(color, sh));
    }
    if (F.bounces > 0) color = tbounce<COUNT, KL, SL>(F, S, rd, pos, normal, color, h, c);
  }
  return gamma(color);
}

// Stage the table into LDS (one-wave workgroups: the barrier is cheap).
__device__ __forceinline__ Table stage(const Frame& F, float* lds) {
  Table S;
  S.blend = F.blend;
  S.omblend = F.omblend;
#ifdef RM_TABLE_STATIC
  (void)lds;
  S.t = reinterpret_cast<const float*>(RM_TS_WORDS);
  return S;
#else
  S.n = F.nprims;
  // staged in LDS: every entry read is a broadcast (the scalar cache measured
  // 1-4 % slower)
  for (int i = threadIdx.x; i < (int)rm::scene_words(F.nprims); i += blockDim.x) lds[i] = F.scene[i];
  __syncthreads();
  S.t = lds;
  {
    // the slots' balls gathered after the table (16-byte aligned): lane l copies
    // word l % 4 of slot l / 4's ball
    const int nw = (int)rm::scene_words(F.nprims);
    float* sb = lds + ((nw + 3) & ~3);
    const int l = threadIdx.x, ns = (int)S.exits()[rm::EX_NSLOTS];
    if (l < 4 * ns) {
      const float v = S.entry((int)S.exits()[rm::EX_SLOTS + l / 4])[rm::TW_BALL + l % 4];
      sb[l] = l % 4 == 3 ? RM_SBR(v) : v;
    }
    __syncthreads();
    S.sb = sb;
  }
  const uint32_t pm = __float_as_uint(uword(S.exits() + rm::EX_PLANE_MASK));
  S.fp = (pm != 0 && (pm & (pm - 1u)) == 0) ? __builtin_ctz(pm) : -1;
  if (S.fp >= 0) {
    const float* P = S.entry(S.fp);
    float c[3], nv[3];
    for (int j = 0; j < 3; ++j) {
      c[j] = uword(P + rm::TW_CENTER + j);
      nv[j] = uword(P + rm::TW_P + j);
    }
    const int swz = __float_as_int(uword(P + rm::TW_SWIZZLE));
    S.fpw = uword(P + rm::TW_P + 3);
    S.fpaxis = nv[0] == 0.0f && nv[2] == 0.0f;
    // (+0 exactly: p.y - (+0) = p.y for every p.y, -0 included; a -0 centre would turn
    // p.y = -0 into +0)
    S.fpunit = S.fpaxis && swz != RM_SWIZZLE_XZY && __float_as_uint(c[1]) == 0u && nv[1] == 1.0f;
  }
  return S;
#endif
}

__device__ __forceinline__ void flush_counts(const Frame& F, const TCnt& c) {
  atomicAdd(&F.counters[0], (unsigned long long)c.rays);
  atomicAdd(&F.counters[1], (unsigned long long)c.march);
  atomicAdd(&F.counters[2], (unsigned long long)c.reflect);
  atomicAdd(&F.counters[3], (unsigned long long)c.shadow);
  atomicAdd(&F.counters[4], (unsigned long long)c.normals);
  atomicAdd(&F.counters[5], (unsigned long long)c.lights);
}

// Waves per SIMD the register allocation must allow.  The per-table specialised
// kernels (RM_TABLE_STATIC) get the bound from rm_jit.hip: the most waves at
// which the table's code needs no scratch.  The generic kernel is latency bound
// and fastest at 7 waves (72 VGPRs, 15 spilled to 52 B/lane of scratch): cfg3
// table 3.06 -> 2.87 ms per frame against 6 waves (80 VGPRs, 5 spills); 8 waves
// (36 spills) measured the same as 7.
#ifndef RM_TABLE_MIN_WAVES
#define RM_TABLE_MIN_WAVES 7
#endif
// The reference-shaped instance (SL): 7 waves, 7 spilled VGPRs (32 B per lane),
// -4.5 % per cfg3 frame against 6 waves (80 VGPRs, no scratch), round 4.
#ifndef RM_TABLE_SL_WAVES
#define RM_TABLE_SL_WAVES 7
#endif

// The lane id re-formed after the march (v_mbcnt, one-wave workgroups: the same
// value as threadIdx.x): the output pixel's coordinates and index come from it
// instead of staying live across trender, where both table kernels spilled them
// to scratch (5 VGPRs, round 5).  Volatile so that LLVM cannot fold it back onto
// the prologue's threadIdx.x.
__device__ __forceinline__ int out_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// Index in the launch's [rows][width] image of pixel (tx, ty) of tile (bx, by)
// of `edge` x `edge` pixels.
__device__ __forceinline__ size_t out_index(const Frame& F, int tx, int ty, int edge, int bx, int by) {
  return (size_t)(by * edge + ty) * (size_t)F.width + (size_t)(bx * edge + tx);
}

// main glsl:291-344 without AA: one lane per pixel, 8x8 pixels per wave.
template <bool COUNT, int KL, int SL>
__device__ __forceinline__ void table_pixel_body(const Frame& F, float* lds, int rowslot) {
  const Table S = stage(F, lds);
  const int lane = threadIdx.x;
  const int by = tile_row(rowslot, gridDim.y);
  const int bx = tile_col(blockIdx.x, gridDim.x, 4);
  const int px = bx * 8 + (lane & 7);
  const int lrow = by * 8 + (lane >> 3);
  if (px >= F.width || lrow >= F.rows) return;
  const size_t idx = (size_t)lrow * (size_t)F.width + (size_t)px;
  const int py = global_row(F, lrow);
  TCnt c = {0, 0, 0, 0, 0, 0};
  if (py < 0) {
    store_pixel(F, idx, 0.0f, 0.0f, 0.0f, 0.0f);
    return;
  }
  f3 ro, rd;
  cast_ray(F, lane_uv(F, 0, px, -1), lane_uv(F, 1, py, -1), ro, rd);
  if (COUNT) c.rays++;
  const f3 col = trender<COUNT, KL, SL>(F, S, ro, rd, c);
  const size_t at = out_index(F, out_lane() & 7, out_lane() >> 3, 8, bx, by);
  store_pixel(F, at, col.x, col.y, col.z, 1.0f);
  if (COUNT) {
    F.sdf_counts[at] = c.march + c.reflect + c.shadow + 4u * c.normals;
    flush_counts(F, c);
  }
}

// main glsl:291-344 with 4x supersampling: one lane per (pixel, sample), the 4
// samples of a pixel in adjacent lanes, summed in the reference's order
// ((c0 + c1) + c2) + c3 before the / 4 (glsl:315-335).
template <bool COUNT, int KL, int SL>
__device__ __forceinline__ void table_sample_body(const Frame& F, float* lds, int rowslot) {
  const Table S = stage(F, lds);
  const int lane = threadIdx.x, s = lane & 3, q = lane >> 2;
  const int by = tile_row(rowslot, gridDim.y);
  const int bx = tile_col(blockIdx.x, gridDim.x, 8);
  const int px = bx * 4 + (q & 3);
  const int lrow = by * 4 + (q >> 2);
  if (px >= F.width || lrow >= F.rows) return;  // the 4 lanes of a pixel leave together
  const int py = global_row(F, lrow);
  TCnt c = {0, 0, 0, 0, 0, 0};
  f3 col = mk(0.0f, 0.0f, 0.0f);
  if (py >= 0) {
    f3 ro, rd;
    cast_ray(F, lane_uv(F, 0, px, s), lane_uv(F, 1, py, s), ro, rd);
    if (COUNT) c.rays++;
    col = trender<COUNT, KL, SL>(F, S, ro, rd, c);
  }
  const float r1 = __shfl(col.x, lane + 1), g1 = __shfl(col.y, lane + 1), b1 = __shfl(col.z, lane + 1);
  const float r2 = __shfl(col.x, lane + 2), g2 = __shfl(col.y, lane + 2), b2 = __shfl(col.z, lane + 2);
  const float r3 = __shfl(col.x, lane + 3), g3 = __shfl(col.y, lane + 3), b3 = __shfl(col.z, lane + 3);
  uint32_t cnt = 0;
  if (COUNT) {
    const uint32_t mine = c.march + c.reflect + c.shadow + 4u * c.normals;
    cnt = mine + __shfl(mine, lane + 1) + __shfl(mine, lane + 2) + __shfl(mine, lane + 3);
    flush_counts(F, c);
  }
  // the pixel's coordinates and index re-formed from the lane id (not kept
  // across the march: see out_lane)
  const int ol = out_lane();
  if ((ol & 3) != 0) return;
  const size_t at = out_index(F, (ol >> 2) & 3, ol >> 4, 4, bx, by);
  if (global_row(F, by * 4 + (ol >> 4)) >= 0) {
    const float o0 = ((col.x + r1) + r2) + r3, o1 = ((col.y + g1) + g2) + g3,
                o2 = ((col.z + b1) + b2) + b3;
    store_pixel(F, at, o0 / 4.0f, o1 / 4.0f, o2 / 4.0f, 1.0f);
  } else {
    store_pixel(F, at, 0.0f, 0.0f, 0.0f, 0.0f);
  }
  if (COUNT) F.sdf_counts[at] = cnt;
}

template <bool COUNT, int KL = rm::EX_MAX_SLOTS, int SL = 0>
__global__ __launch_bounds__(64, SL ? RM_TABLE_SL_WAVES : RM_TABLE_MIN_WAVES) void k_table_pixel(Frame F) {
  extern __shared__ float lds[];
  table_pixel_body<COUNT, KL, SL>(F, lds, blockIdx.y);
}
template <bool COUNT, int KL = rm::EX_MAX_SLOTS, int SL = 0>
__global__ __launch_bounds__(64, SL ? RM_TABLE_SL_WAVES : RM_TABLE_MIN_WAVES) void k_table_sample(Frame F) {
  extern __shared__ float lds[];
  table_sample_body<COUNT, KL, SL>(F, lds, blockIdx.y);
}

// Frame batches (rm_dispatch_frames): n frames of one table,
// size and AA setting in one launch, each workgroup reading its frame's
// constants from the batch in the kernel arguments.  The (y, z) workgroup slots
// are read row-major over the frames, as k_sample_frames reads them
// (rm_kernels.hip batch_slot: every frame's slowest rows first).  The bodies are
// the kernels' above, so every frame is the image of its own dispatch.
// Production kernels only (a batch collects no counters).
__device__ __forceinline__ void table_batch_slot(int& frame, int& rowslot) {
  const int L = blockIdx.z * gridDim.y + blockIdx.y, n = gridDim.z;
  // uniform: kept in SGPRs (the division is VALU code)
  rowslot = __builtin_amdgcn_readfirstlane(L / n);
  frame = __builtin_amdgcn_readfirstlane(L - rowslot * n);
}
template <int KL = rm::EX_MAX_SLOTS, int SL = 0>
__global__ __launch_bounds__(64, SL ? RM_TABLE_SL_WAVES : RM_TABLE_MIN_WAVES) void k_table_pixel_frames(
    FrameBatch B) {
  extern __shared__ float lds[];
  int f, r;
  table_batch_slot(f, r);
  table_pixel_body<false, KL, SL>(B.f[f], lds, r);
}
template <int KL = rm::EX_MAX_SLOTS, int SL = 0>
__global__ __launch_bounds__(64, SL ? RM_TABLE_SL_WAVES : RM_TABLE_MIN_WAVES) void k_table_sample_frames(
    FrameBatch B) {
  extern __shared__ float lds[];
  int f, r;
  table_batch_slot(f, r);
  table_sample_body<false, KL, SL>(B.f[f], lds, r);
}

}  // namespace rmd

#ifndef RM_TABLE_STATIC
namespace rm {

namespace {
template <int KL, int SL>
void launch_table_frames_kl(const rmd::FrameBatch& B, int n, hipStream_t s);
// A production frame renders with the batch kernel, as a batch of one (round 6,
// as the specialised kernels: rm_jit.hip): the single-frame production kernel,
// whose Frame lives in scalar registers from the prologue on, was 1.0 % slower
// per cfg3 frame (profiles/r06_ab_b1_single.txt) and is no longer compiled.  The
// counting kernels keep their single-frame form.
template <int KL, int SL>
void launch_table_kl(const rmd::Frame& F, bool counters, hipStream_t s) {
  if (!counters) {
    static thread_local rmd::FrameBatch B;
    B.f[0] = F;
    launch_table_frames_kl<KL, SL>(B, 1, s);
    return;
  }
  // the table, then the lazy slots' balls (Table::sb)
  const size_t lds = (((rm::scene_words(F.nprims) + 3) & ~(size_t)3) + 4 * (size_t)rm::EX_MAX_SLOTS) * sizeof(float);
  if (F.aa)
    hipLaunchKernelGGL((rmd::k_table_sample<true, KL>), dim3((F.width + 3) / 4, (F.rows + 3) / 4), dim3(64), lds, s, F);
  else
    hipLaunchKernelGGL((rmd::k_table_pixel<true, KL>), dim3((F.width + 7) / 8, (F.rows + 7) / 8), dim3(64), lds, s, F);
}

template <int KL, int SL>
void launch_table_frames_kl(const rmd::FrameBatch& B, int n, hipStream_t s) {
  const rmd::Frame& F = B.f[0];
  const size_t lds = (((rm::scene_words(F.nprims) + 3) & ~(size_t)3) + 4 * (size_t)rm::EX_MAX_SLOTS) * sizeof(float);
  if (F.aa)
    hipLaunchKernelGGL((rmd::k_table_sample_frames<KL, SL>), dim3((F.width + 3) / 4, (F.rows + 3) / 4, n), dim3(64),
                       lds, s, B);
  else
    hipLaunchKernelGGL((rmd::k_table_pixel_frames<KL, SL>), dim3((F.width + 7) / 8, (F.rows + 7) / 8, n), dim3(64),
                       lds, s, B);
}

// The generic kernel's instance for a table: KL = TABLE_FEW_SLOTS or
// EX_MAX_SLOTS slots (the table's lazy slots, EX_NSLOTS, fit), and the march
// shape (rm::table_shape).
template <class L>
void with_instance(int nslots, int shape, L&& launch) {
  auto sh = [&](auto kl) {
    if (shape == 1) launch(kl, std::integral_constant<int, 1>());
    else if (shape == 2) launch(kl, std::integral_constant<int, 2>());
    else launch(kl, std::integral_constant<int, 0>());
  };
  if (nslots <= TABLE_FEW_SLOTS) sh(std::integral_constant<int, TABLE_FEW_SLOTS>());
  else sh(std::integral_constant<int, rm::EX_MAX_SLOTS>());
}
}  // namespace

// The frames B.f[0..n) of one table, size and AA setting in one launch.
hipError_t launch_table_frames(const rmd::FrameBatch& B, int n, hipStream_t s, int nslots, int shape) {
  if (n < 1 || n > rmd::kMaxBatch) return hipErrorInvalidValue;
  with_instance(nslots, shape, [&](auto kl, auto sh) { launch_table_frames_kl<decltype(kl)::value, decltype(sh)::value>(B, n, s); });
  return hipGetLastError();
}

// nslots: the table's lazy slots (EX_NSLOTS of its compiled words).  Tables with
// at most TABLE_FEW_SLOTS of them (the reference scene has 5) take an instance
// holding that many: 3 fewer live expiries in the march loops, 15 -> 8 spilled
// VGPRs at the 7-wave bound, -2.4 % per cfg3 frame.
// shape: the production kernels' march (rm::table_shape): 1 the built-in march
// shape (smarch, reference-shaped tables), 2 the block shape of any
// plane-bounded table (gmarch), 0 TLazy; the counting kernels keep TLazy.
hipError_t launch_table(const rmd::Frame& F, bool counters, hipStream_t s, int nslots, int shape) {
  with_instance(nslots, shape, [&](auto kl, auto sh) { launch_table_kl<decltype(kl)::value, decltype(sh)::value>(F, counters, s); });
  return hipGetLastError();
}

// smarch's conditions on a compiled table (slazy_table, device): valid exit
// bounds; exactly one plane, the last entry, unswizzled, normal (0, n_y, 0);
// every other entry in a lazy slot, slot j holding entry j.
bool table_slazy(const uint32_t* words, int32_t n);
// The production march of a compiled table: 1 smarch, 2 gmarch (valid exit
// bounds and a plane: glazy_table, device), 0 TLazy.
int table_shape(const uint32_t* words, int32_t n) {
  if (table_slazy(words, n)) return 1;
  const float* ex = reinterpret_cast<const float*>(words) + (size_t)n * TABLE_WORDS;
  return ex[EX_VALID] != 0.0f && ex[EX_NPLANES] >= 1.0f ? 2 : 0;
}
bool table_slazy(const uint32_t* words, int32_t n) {
  const float* t = reinterpret_cast<const float*>(words);
  const float* ex = t + (size_t)n * TABLE_WORDS;
  const float* P = t + (size_t)(n - 1) * TABLE_WORDS;
  int type, swz;
  std::memcpy(&type, P + TW_TYPE, sizeof type);
  std::memcpy(&swz, P + TW_SWIZZLE, sizeof swz);
  if (ex[EX_VALID] == 0.0f || ex[EX_NPLANES] != 1.0f || type != RM_PRIM_PLANE || swz != RM_SWIZZLE_XYZ) return false;
  if (!(P[TW_P] == 0.0f && P[TW_P + 2] == 0.0f) || (int)ex[EX_NSLOTS] != n - 1) return false;
  for (int j = 0; j < n - 1; ++j)
    if ((int)ex[EX_SLOTS + j] != j) return false;
  return true;
}

}  // namespace rm
#endif
