// rm_kernels.hip — the hot path: per-pixel SDF sphere tracing on gfx950.
//
// Reference: shaders/computeShader.glsl:68-344 (dispatched by main.cpp:123).
// Two kernels compute the same pure function of (pixel, uniforms), with the
// GLSL call tree (render -> bounce -> softshadow) as their control flow:
//   * k_sample — 4x supersampled frames: one lane per (pixel, sample), a wave
//                covers 4x4 pixels x 4 samples;
//   * k_pixel  — frames without supersampling: one lane per pixel, 8x8 pixels
//                per wave.
// Each is built twice: COUNT = false is the production kernel (every
// proof-based early exit taken), COUNT = true the counting build of the tests.
// See DESIGN.md §4 for the kernel designs and their rooflines.
//
// Diagnostic builds only (tools/build_variant.sh; tests/test_abi.py compiles
// them): RM_STATS (wave / lane counters, tools/stats_probe.py), RM_WAVE_TIMES
// (per-wave lifetimes, tools/wave_timeline.hip), RM_DBL_<PHASE> (a phase run
// twice: its marginal cost, tools/ab_kernel.py).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rm_scene.hpp"

namespace rmd {

// Marches run in segments ending at these scalar step indices, where the lanes
// still marching take the step-cap miss check (rm_scene.hpp cap_miss).
constexpr int kCapI0 = 16, kCapI1 = 64;

#ifdef RM_WAVE_TIMES
__device__ unsigned long long* g_wave_times;
#endif

struct Cnt {
  uint32_t rays, march, reflect, shadow, normals, lights;
};

// Keeps the compiler from hoisting a value (and its registers) across a loop,
// and feeds the RM_DBL_<PHASE> cost probes an opaque copy of their inputs.
__device__ __forceinline__ float opaque(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ f3 opaque(f3 v) { return mk(opaque(v.x), opaque(v.y), opaque(v.z)); }

// RayMarch glsl:125-142 / reflectedRay glsl:144-161.  Returns t or -1.
// UNIT: a primary ray of a frame whose rays all have |rd| within 2^-20 of 1
// (Frame::unit_rd, checked on the host): |rd| = 1 serves every bound that
// needs |rd| from below or above, with the bounds' own 2^-12 / 2^-16 margins
// (it stood for a v_sqrt within 1.5 ulp), so |rd|, its reciprocal and the
// slack slope become constants and the miss exit's object bound is uniform.
// PPROJ: primary rays take the projection bound of the miss exit too (k_pixel;
// see miss_T).
template <bool COUNT, bool UNIT = false, bool PPROJ = false>
__device__ float march(const Frame& F, f3 ro, f3 rd, bool reflected, int& id, f3& col, Cnt& c,
                       float& dlast) {
  float t = 0.0f, dl = 0.0f;
  const float tmax = reflected ? 200.0f : 400.0f;
  const int nmax = reflected ? 256 : 512;
  bool hit = false;
  // per-ray constants; the ro-dependent ones of primary rays come from the host
  // (rm_api.hip prep_host: every primary ray starts at the camera)
  const bool prep = !reflected && F.prepv[PREP_VALID] != 0.0f;
  const float rdl = UNIT ? 1.0f : ray_rdl(rd), s1 = ray_s1(rdl);
  const float s0 = prep ? F.prepv[PREP_SLACK] : ray_s0(ro);
  // ro in VGPRs: a primary ray's ro is the camera, uniform, and an SGPR operand
  // keeps an f32 add / mul from dual issue (4 instead of 2 cycles per wave64
  // instruction on gfx950, tools/valu_peak.hip), once per march step here.
  ro = opaque(ro);
  LazyCull lc;
  if (UNIT) lazy_init_unit(lc, rd, s0, s1);
  else lazy_init(lc, rd, rdl, s0, s1);
  // the provable-miss threshold mx (rm_scene.hpp "early exits"), formed where it
  // is used: its ro-dependent terms b1, b2 with it (a downward ray has mx = +inf,
  // so waves of downward rays never form either)
  auto miss_T = [&]() {
    float b1, b2;
    if (prep) {
      b1 = F.prepv[PREP_B1];
      b2 = F.prepv[PREP_B2];
    } else {
      lin_exit_b(ro, s0, 0.0f, b1, b2);
    }
    // the objects' ball seen along the ray: reflected rays, and the primary rays
    // of frames without supersampling.  A primary ray from the camera mostly heads
    // into the scene, where the projection is close to |ro - C|: in 4x-supersampled
    // frames the bound costs more than it saves (cfg3 +0.4 %), in k_pixel's frames
    // it saves (cfg2 -3.5 %, profiles/r05_ab_exits2.txt)
    if (!prep || PPROJ)
      b1 = __builtin_fminf(b1, lin_exit_b1p(ro, rd, UNIT ? 1.0f : __builtin_amdgcn_rcpf(rdl), s0, 0.0f));
    const float b3 = prep ? F.prepv[PREP_B3] : lin_exit_b3(ro.y, s0, 0.0f);
    return lin_exit_T(MISS_C, rdl, rd.y, s1, b1, b2, b3);
  };
  // lin_exit's object bound T1 for the step-cap check, re-formed there from the
  // ray (rare) rather than kept live through the loop
  auto cap_T1 = [&](f3 o, f3 r) {
    float b1c, b2c;
    if (prep) b1c = F.prepv[PREP_B1];
    else lin_exit_b(o, lc.s0, 0.0f, b1c, b2c);
    return lin_exit_T1(MISS_C, UNIT ? 1.0f : ray_rdl(r), lc.s1, b1c);
  };
  // provable miss: production stops there; the counting build runs on to the
  // reference's step count and poisons the colour with NaN should the ray hit
  // after all (parity tests compare NaN masks)
  bool proven_miss = false;
  int i0 = 1;
  // Primary rays: step 0 is at the camera for every pixel; the host evaluated it
  // once (its distance is exact, its gaps as the block's re-test would form
  // them with U = d0).  Each lane only turns the gaps into expiries with its own
  // |rd|: te = max(g / 2|rd|, plane gap / (|rd| + rd.y), 0) at t = 0, where a
  // gap the host found <= 0 is -inf (te = 0: re-test at the next step).
  if (prep) {
    const float d0 = F.prepv[PREP_D0];
#pragma unroll
    for (int k = 0; k < 5; ++k)
      lc.te[k] = vmax3(F.prepv[PREP_G + k] * lc.inv2v, F.prepv[PREP_H + k] * lc.invp, 0.0f);
    lc.tegrp = vmin(vmin3(lc.te[0], lc.te[1], lc.te[2]), lc.te[4]);
    lc.temin = vmin(lc.tegrp, lc.te[3]);
    if (COUNT) c.march++;
    dl = d0;
    t = d0;
    i0 = 2;
  }
#ifndef RM_STATS
  if (!COUNT) {
    // Production loop.  A lane leaves on hit | escape | proven miss; the 512 /
    // 256 step cap is the same step for every lane of the wave (all start at
    // i0), so it is a scalar loop bound.  t advances on every step and the
    // step's own t is kept in tp, so the loop has a single exit at its latch
    // (hit | escape | t + d past mx, a NaN failing the compare | segment end)
    // and at the exit (t, dl) is the last step's pair: `dl < 1e-6 t` re-forms
    // its hit test exactly.  A NaN distance (degenerate scenes) leaves at once:
    // the reference marches on with t = NaN to the cap, also a miss.
    //
    // The escape test d > tmax is implied, for a lane, by either of
    //   mx <= tmax:  d > tmax  =>  t + d >= d > tmax >= mx (t >= 0, rounding is
    //                monotone): the proven-miss compare already fires, also a miss;
    //   rd.y <= 0 and ro.y + 5.5 <= tmax:  d <= plane(t) = (ro.y + rd.y t) + 5.5
    //                <= ro.y + 5.5 <= tmax: no step ever escapes.
    // Only waves with a lane outside both cases run the loop with the test.
    // Waves of downward rays only (rd.y <= 0 gives mx = +inf) also drop the mx
    // compare: the hit is their only lane exit.
    const float QNAN = __builtin_nanf("");
    auto run = [&](auto esc, auto usemx, const float mx) {
      // A march runs in segments ending at kCapI0 and kCapI1: the step
      // loop itself is the plain one, with the segment end as its scalar bound.
      // Between segments a lane's exit test is re-formed from its last (t, dl)
      // (same operations, same result), the lanes still marching take the
      // step-cap check, and those that go on take the step.
      // Reflected marches take the step-cap check too (round 6, VERDICT r05 #5:
      // no scratch since round 5's register changes; cfg3 -0.4 %, cfg4 -0.6 % per
      // frame at the bench's throughput, profiles/r06_ab_reflcap.txt).
      int ib = i0, iend = kCapI0;
      bool live = true;
#pragma unroll 1
      for (;;) {
        if (live && !decltype(usemx)::value && !decltype(esc)::value) {
          // Waves of downward rays (the hit is the only lane exit): t advances at
          // the top of the step, t + the last step's d, so the loop carries only
          // (t, d) -- the step's own pair at the exit -- and needs no copy of t
          // (round 6: one VALU per step fewer, cfg3 -0.5 %, cfg2 -0.5 % per frame,
          // profiles/r06_ab_hadd_cfg*.txt).  At a segment's start d = 0: t + 0 = t.
          float dp = 0.0f;
          for (int i = ib;; ++i) {
            t = t + dp;
            const float d = scene_lazy(ro, rd, t, lc, F.blend, F.omblend);
            dp = d;
            if ((d < 0.000001f * t) | (i >= iend)) break;
          }
          dl = dp;
        } else if (live) {
          float tp = t;
          for (int i = ib;; ++i) {
#ifdef RM_WAVE_STATS
            RM_STAT(reflected ? 6 : 15);
#endif
            const float d = scene_lazy(ro, rd, t, lc, F.blend, F.omblend);
            bool ex = d < 0.000001f * t;
            dl = d;
            tp = t;
            t = t + d;
            if (decltype(usemx)::value) ex = ex | !(t <= mx);
            if (decltype(esc)::value) ex = ex | (d > tmax);
            if (ex | (i >= iend)) break;
          }
          t = tp;
        }
        if (iend >= nmax) break;
        {
          float probe = (dl < 0.000001f * t) ? QNAN : t + dl;
          if (decltype(esc)::value) probe = (dl > tmax) ? QNAN : probe;
          live = live && (probe <= mx);
          // step-cap miss exit (rm_scene.hpp) for waves holding a grazing downward
          // ray; K = nmax - iend evaluations would remain
          if (__any(live && rd.y < 0.0f && rd.y > -0.05f)) {
            const f3 o = opaque(ro), r = opaque(rd);
            live = live && !cap_miss(t, dl, nmax - iend, o.y, r.y, cap_T1(o, r));
          }
          if (live) t = probe;
        }
        ib = iend + 1;
        iend = iend < kCapI1 ? kCapI1 : nmax;  // segments end at I0 < I1 < nmax
      }
    };
    // rd.y <= 0: lin_exit_T's plane slope a2 = (rd.y - s1 - c) LO - .. is < 0, so
    // mx = +inf, and with ro.y + 5.5 <= tmax no step escapes (above)
    const bool down = rd.y <= 0.0f && ro.y + 5.5f <= tmax;
    if (__all(down)) {
      run(std::false_type(), std::false_type(), __builtin_huge_valf());
    } else {
      const float mx = miss_T();
      const bool need_esc = (mx > tmax) && !down;
      if (__any(need_esc)) run(std::true_type(), std::true_type(), mx);
      else run(std::false_type(), std::true_type(), mx);
    }
    asm volatile("" : "+v"(t), "+v"(dl));  // re-form the test, not a lane mask kept per step
    if (dl < 0.000001f * t) {
      const f3 q = add(ro, muls(rd, t));
      id = lazy_id(lc, t, dl, ro.y, rd.y);
      col = hit_color(id, q);
      dlast = dl;
      return t;
    }
    id = -1;
    col = mk(0.0f, 0.0f, 0.0f);
    return -1.0f;
  }
#endif
  // Counting build (and RM_STATS): one exit per step (hit | escape | step cap
  // | proven miss); the proofs are only checked.
  const float mx = miss_T();
#ifdef RM_STATS
  int nst = 0;  // this lane's steps (diagnostic builds)
#endif
  for (int i = i0;; ++i) {
#ifdef RM_STATS
    ++nst;
    {
      const unsigned long long m = __ballot(1);
      if (__lane_id() == __builtin_ffsll(m) - 1) {
        atomicAdd(&g_stats[reflected ? 6 : 15], 1ull);
        atomicAdd(&g_stats[7], (unsigned long long)__popcll(m));
        atomicAdd(&g_stats[32 + (reflected ? 6 : 15)], (unsigned long long)__popcll(m));
      }
    }
#endif
    const float d = scene_lazy(ro, rd, t, lc, F.blend, F.omblend);
    if (COUNT) {
      if (reflected) c.reflect++;
      else c.march++;
    }
    hit = d < 0.000001f * t;
    dl = d;
    bool stop = hit | (d > tmax) | (i >= nmax);
    if (i == kCapI0 || i == kCapI1) {  // same check as the production loop
      const bool cm = !stop && cap_miss(t, d, nmax - i, ro.y, rd.y, cap_T1(ro, rd));
      if (COUNT) proven_miss |= cm;
      else stop |= cm;
    }
    t += stop ? 0.0f : d;  // t >= +0: t + 0 == t
    const bool gone = !stop && lin_exit(mx, t);
    if (COUNT) proven_miss |= gone;
    else stop |= gone;
    if (stop) break;
  }
#ifdef RM_STATS
  // lane sums of steps: [4] primary miss, [5] primary hit, [24] reflected miss,
  // [25] reflected hit; [3] / [23] count the primary miss / hit lanes
  atomicAdd(&g_stats[(reflected ? 24 : 4) + (hit ? 1 : 0)], (unsigned long long)nst);
  if (!reflected) atomicAdd(&g_stats[hit ? 23 : 3], 1ull);
#endif
  if (hit) {
    // the opU id (and colour) of the hit: from the last step's sdf (same point)
    const f3 q = add(ro, muls(rd, t));
    id = lazy_id(lc, t, dl, ro.y, rd.y);
    col = hit_color(id, q);
    if (COUNT && proven_miss) col = mk(__builtin_nanf(""), 0.0f, 0.0f);
    dlast = dl;
    return t;
  }
  id = -1;
  col = mk(0.0f, 0.0f, 0.0f);
  return -1.0f;
}

// GetNormal glsl:278-288, samples with shared culling (rm_scene.hpp).  HAVE_C0:
// the centre sample sdf(pos) is the primary march's last distance (same point).
template <bool COUNT, bool HAVE_C0>
__device__ f3 get_normal(const Frame& F, f3 pos, Cnt& c, float c0 = 0.0f) {
  if (COUNT) c.normals++;
  RM_STAT(27);
  float vx, vy, vz;
  normal_samples<HAVE_C0>(pos, F.blend, F.omblend, c0, vx, vy, vz);
#ifdef RM_DBL_NORMAL
  if (!COUNT) {
    float c0b = c0, wx, wy, wz;
    normal_samples<HAVE_C0>(opaque(pos), F.blend, F.omblend, c0b, wx, wy, wz);
    vx = vmin(vx, wx); vy = vmin(vy, wy); vz = vmin(vz, wz); c0 = vmin(c0, c0b);
  }
#endif
  return normalize(subs(mk(vx, vy, vz), c0));
}

// softshadow glsl:201-216
template <bool COUNT>
__device__ float softshadow_impl(const Frame& F, f3 ro, f3 rd, float rdl, Cnt& c);
// rdl: |rd| (the light term's exact distance, shadow_exit_init)
template <bool COUNT>
__device__ __forceinline__ float softshadow(const Frame& F, f3 ro, f3 rd, float rdl, Cnt& c) {
#ifdef RM_DBL_SHADOW
  if (!COUNT) return vmin(softshadow_impl<COUNT>(F, ro, rd, rdl, c), softshadow_impl<COUNT>(F, opaque(ro), rd, rdl, c));
#endif
  return softshadow_impl<COUNT>(F, ro, rd, rdl, c);
}
template <bool COUNT>
__device__ __forceinline__ float softshadow_impl(const Frame& F, f3 ro, f3 rd, float rdl, Cnt& c) {
  float res = 1.0f, t = 0.0f;
  int dummy;
  RM_STAT(29);
  const float ex = shadow_exit_init(F.shc, ro, rd, rdl, light_in_ball(F));
  for (int i = 0; i < 16; ++i) {
    if (lin_exit(ex, t)) {  // the remaining steps are no-ops
      if (COUNT) c.shadow += 16 - i;
      return res;
    }
    float h = scene_cull<false, true>(add(ro, muls(rd, t)), F.blend, F.omblend, dummy);
    RM_STAT(2);
    if (COUNT) c.shadow++;
    if (h < 0.001f) return 0.05f;
    res = shadow_min(res, F.k, h, t);
    t += h;
  }
  return res;
}

// bounce glsl:163-199 (dead tail skipped; see rm_oracle.h "live" counters)
template <bool COUNT>
__device__ f3 bounce(const Frame& F, f3 rayDir, f3 pos, f3 normal, f3 color, f3 primColor,
                     Cnt& c) {
  bool prevMatte = false;  // the primary object is never MATTE here (glsl:232-240)
  f3 prevColor = primColor;
  f3 lpos = mk(F.lpos[0], F.lpos[1], F.lpos[2]);
  for (int i = 1; i <= F.bounces; ++i) {
    // After a MATTE prevObject every remaining iteration is a colour no-op
    // (glsl:181,189-190): stop instead of running the dead marches.
    if (prevMatte) break;
    RM_STAT(26);
    rayDir = reflect(rayDir, normal);
    int id;
    f3 tcol;
    float dl;
    float ldist;  // set with the light term; read only after a hit on the floor (id 7)
    float th = march<COUNT>(F, add(pos, muls(normal, 0.001f)), rayDir, true, id, tcol, c, dl);
#ifdef RM_DBL_BMARCH
    if (!COUNT) {
      int id2; f3 tc2; float dl2;
      const float th2 = march<COUNT>(F, opaque(add(pos, muls(normal, 0.001f))), rayDir, true, id2, tc2, c, dl2);
      th = (th2 == th) ? th : __builtin_nanf("");
    }
#endif
    pos = add(pos, muls(rayDir, th));
    // The normal of a miss on the last bounce is never read: skip it.
    // (the hit point is pos + rayDir t, not the march's ro + rd t: no centre reuse)
    if (th != -1.0f || i < F.bounces) normal = get_normal<COUNT, false>(F, pos, c);
    if (th == -1.0f) {
      tcol = subs(mk(0.36f, 0.36f, 0.60f), rayDir.y * 0.2f);
    } else {
      if (COUNT) c.lights++;
      tcol = point_light(F, tcol, normal, pos, &ldist);
    }
    // The weights x / i (glsl:186-187).  For i = 1, 2, 4 the quotient is the
    // real number x * 2^-k, exactly representable unless it underflows, and
    // where it does the correctly rounded quotient and the correctly rounded
    // product x * 2^-k round that same real number: x * (1, 0.5, 0.25) equals
    // the IEEE division bit for bit.  i is wave-uniform, so this is a scalar
    // branch, and 2 of cfg3's 3 bounce iterations skip four IEEE divisions
    // (~10 VALU each) per lane.
    const bool pow2 = (i & (i - 1)) == 0;
    const float w = i == 1 ? 1.0f : (i == 2 ? 0.5f : 0.25f);
    if (id == 7 && !prevMatte && i < 3) {
      float sh = softshadow<COUNT>(F, add(pos, muls(normal, 0.02f)), sub(lpos, pos), ldist, c);
      color = muls(color, pow2 ? sh * w : div_small(sh, i));
    }
    const f3 tw = mul(tcol, prevColor);
    if (pow2) color = add(color, muls(tw, w));
    else color = add(color, divi(tw, i));
    prevColor = tcol;
    prevMatte = (id == 7);  // material of the hit: MATTE only for the floor; dummy is 1.0
  }
  return color;
}

// render glsl:218-251
template <bool COUNT, bool PPROJ = false>
__device__ __forceinline__ f3 render(const Frame& F, f3 ro, f3 rd, Cnt& c) {
  f3 color = subs(mk(0.30f, 0.36f, 0.60f), rd.y * 0.2f);
  int id;
  f3 hcol;
  float dl;
  // (F.unit_rd is uniform: one march or the other for the whole wave)
  float th = F.unit_rd ? march<COUNT, true, PPROJ>(F, ro, rd, false, id, hcol, c, dl)
                       : march<COUNT, false, PPROJ>(F, ro, rd, false, id, hcol, c, dl);
#ifdef RM_DBL_MARCH
  if (!COUNT) {
    int id2; f3 hc2; float dl2;
    const float th2 = march<COUNT>(F, opaque(ro), rd, false, id2, hc2, c, dl2);
    th = (th2 == th) ? th : __builtin_nanf("");
  }
#endif
  RM_STAT(30);
  if (th != -1.0f) {
    RM_STAT(31);
    f3 pos = add(ro, muls(rd, th));
    f3 normal = get_normal<COUNT, true>(F, pos, c, dl);
    if (COUNT) c.lights++;
    float ldist;
    color = point_light(F, hcol, normal, pos, &ldist);
#ifdef RM_DBL_LIGHT
    if (!COUNT) {
      const f3 c2 = point_light(F, hcol, normal, opaque(pos));
      color = mk(vmin(color.x, c2.x), vmin(color.y, c2.y), vmin(color.z, c2.z));
    }
#endif
    if (id == 7) {
      f3 lpos = mk(F.lpos[0], F.lpos[1], F.lpos[2]);
      float sh = softshadow<COUNT>(F, add(pos, muls(normal, 0.02f)), sub(lpos, pos), ldist, c);
      color = muls(color, sh);
      return gamma(color);
    }
    if (F.bounces > 0) color = bounce<COUNT>(F, rd, pos, normal, color, hcol, c);
  }
#ifdef RM_DBL_GAMMA
  if (!COUNT) {
    const f3 g1 = gamma(color), g2 = gamma(opaque(color));
    return mk(vmin(g1.x, g2.x), vmin(g1.y, g2.y), vmin(g1.z, g2.z));
  }
#endif
  return gamma(color);
}

// tile_row / tile_col (dispatch order): rm_scene.hpp

// main glsl:291-344, one thread per pixel, frames without supersampling (AA
// frames go to k_sample).  One-wave workgroups of an 8x8 pixel tile: the 64
// rays of a wave are spatially coherent (similar step counts, same culled
// primitives), and a finished wave's slot is refilled at once instead of
// waiting for its workgroup's slowest wave.  This replaces the reference's
// 39x39 tiles; its W/wg truncation band (main.cpp:123) is not reproduced.
constexpr int kTileW = 8, kTileH = 8;
template <bool COUNT>
__device__ __forceinline__ void pixel_body(const Frame& F, int rowslot) {
  const int lane = threadIdx.x & 63;
  const int by = tile_row(rowslot, F.grid_y);
  const int bx = tile_col(blockIdx.x, F.grid_x, 128 / (kTileW * 4));
  const int px = bx * kTileW + (lane & 7);
  const int lrow = by * kTileH + (lane >> 3);
  if (px >= F.width || lrow >= F.rows) return;
  const size_t idx = (size_t)lrow * (size_t)F.width + (size_t)px;
  const int py = global_row(F, lrow);
  Cnt c = {0, 0, 0, 0, 0, 0};
  float o0 = 0.0f, o1 = 0.0f, o2 = 0.0f, o3 = 0.0f;
  if (py >= 0) {
    f3 ro, rd;
    cast_ray(F, lane_uv(F, 0, px, -1), lane_uv(F, 1, py, -1), ro, rd);
    if (COUNT) c.rays++;
    f3 col = render<COUNT, true>(F, ro, rd, c);
    o0 = col.x;
    o1 = col.y;
    o2 = col.z;
    o3 = 1.0f;
  }
  store_pixel(F, idx, o0, o1, o2, o3);
  if (COUNT) {
    F.sdf_counts[idx] = c.march + c.reflect + c.shadow + 4u * c.normals;
    atomicAdd(&F.counters[0], (unsigned long long)c.rays);
    atomicAdd(&F.counters[1], (unsigned long long)c.march);
    atomicAdd(&F.counters[2], (unsigned long long)c.reflect);
    atomicAdd(&F.counters[3], (unsigned long long)c.shadow);
    atomicAdd(&F.counters[4], (unsigned long long)c.normals);
    atomicAdd(&F.counters[5], (unsigned long long)c.lights);
  }
}

// main glsl:291-344 with 4x supersampling, one thread per (pixel, sample).
// The 4 samples of a pixel sit in 4 adjacent lanes, so a one-wave workgroup
// covers a 4x4 pixel tile with all its samples (the most coherent 64 rays
// available: the sample rays of one pixel are sub-pixel apart; 8x2 and 16x1
// tiles measured 3 % and 17 % slower).  Lane s reads the cumulative uv of
// glsl:311-332 from the host tables (the same sequential float adds), and lane
// s == 0 sums the samples in the reference's fixed order ((c0+c1)+c2)+c3 via
// lane shuffles before the /4 (glsl:315-335).
constexpr int kSampleTileW = 4, kSampleTileH = 4;
template <bool COUNT>
__device__ __forceinline__ void sample_body(const Frame& F, int rowslot) {
  const int lane = threadIdx.x & 63;
  const int s = lane & 3, q = lane >> 2;
  const int by = tile_row(rowslot, F.grid_y);
  const int bx = tile_col(blockIdx.x, F.grid_x, 128 / (kSampleTileW * 4));
  const int px = bx * kSampleTileW + q % kSampleTileW;
  const int lrow = by * kSampleTileH + q / kSampleTileW;
  if (px >= F.width || lrow >= F.rows) return;  // all 4 lanes of a pixel leave together
  const size_t idx = (size_t)lrow * (size_t)F.width + (size_t)px;
  const int py = global_row(F, lrow);
  Cnt c = {0, 0, 0, 0, 0, 0};
  f3 col = mk(0.0f, 0.0f, 0.0f);
#ifdef RM_WAVE_TIMES
  const unsigned long long wt0 = wall_clock64();
#endif
  if (py >= 0) {
    f3 ro, rd;
    cast_ray(F, lane_uv(F, 0, px, s), lane_uv(F, 1, py, s), ro, rd);
    if (COUNT) c.rays++;
    col = render<COUNT>(F, ro, rd, c);
  }
#ifdef RM_DPP_AA
  // the quad's other samples by DPP quad permutes (lane s = 0 reads lanes 1, 2, 3
  // of its quad): VALU moves instead of LDS permutes
  auto q1 = [](float v) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x39, 0xf, 0xf, false)); };
  auto q2 = [](float v) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4e, 0xf, 0xf, false)); };
  auto q3 = [](float v) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x93, 0xf, 0xf, false)); };
  const float r1 = q1(col.x), g1 = q1(col.y), b1 = q1(col.z);
  const float r2 = q2(col.x), g2 = q2(col.y), b2 = q2(col.z);
  const float r3 = q3(col.x), g3 = q3(col.y), b3 = q3(col.z);
#else
  const float r1 = __shfl(col.x, lane + 1), g1 = __shfl(col.y, lane + 1), b1 = __shfl(col.z, lane + 1);
  const float r2 = __shfl(col.x, lane + 2), g2 = __shfl(col.y, lane + 2), b2 = __shfl(col.z, lane + 2);
  const float r3 = __shfl(col.x, lane + 3), g3 = __shfl(col.y, lane + 3), b3 = __shfl(col.z, lane + 3);
#endif
  uint32_t cnt = 0;
  if (COUNT) {
    const uint32_t mine = c.march + c.reflect + c.shadow + 4u * c.normals;
    cnt = mine + __shfl(mine, lane + 1) + __shfl(mine, lane + 2) + __shfl(mine, lane + 3);
    atomicAdd(&F.counters[0], (unsigned long long)c.rays);
    atomicAdd(&F.counters[1], (unsigned long long)c.march);
    atomicAdd(&F.counters[2], (unsigned long long)c.reflect);
    atomicAdd(&F.counters[3], (unsigned long long)c.shadow);
    atomicAdd(&F.counters[4], (unsigned long long)c.normals);
    atomicAdd(&F.counters[5], (unsigned long long)c.lights);
  }
#ifdef RM_WAVE_TIMES
  // diagnostic (tools/wave_timeline.hip): per-wave start/end and hardware slot
  if (lane == 0) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const size_t w = (size_t)by * F.grid_x + bx;
    g_wave_times[3 * w] = wt0;
    g_wave_times[3 * w + 1] = wall_clock64();
    g_wave_times[3 * w + 2] = hw;
  }
#endif
  if (s != 0) return;
  if (py >= 0) {
    const float o0 = ((col.x + r1) + r2) + r3, o1 = ((col.y + g1) + g2) + g3,
                o2 = ((col.z + b1) + b2) + b3;
    store_pixel(F, idx, o0 / 4.0f, o1 / 4.0f, o2 / 4.0f, 1.0f);
  } else {
    store_pixel(F, idx, 0.0f, 0.0f, 0.0f, 0.0f);
  }
  if (COUNT) F.sdf_counts[idx] = cnt;
}

// Entry points: the frame constants by value (kernel arguments in SGPRs).
// 64 VGPRs: 8 waves per SIMD, the most a SIMD holds (the kernels are latency
// bound; 7 and 6 waves measured slower).
#ifndef RM_KERNELS_AA_ONLY
template <bool COUNT>
__global__ __launch_bounds__(64, 8) void k_pixel(Frame F) {
  pixel_body<COUNT>(F, blockIdx.y);
}
#endif
#ifndef RM_KERNELS_PIXEL_ONLY
// Built in its own object without SLP vectorisation (Makefile): pairing
// independent f32 adds / muls into v_pk_add_f32 / v_pk_mul_f32 costs register
// moves to form the pairs and measured 3.5 % slower per cfg3 frame (round 3,
// profiles/r03_compiler_ab.txt); k_pixel keeps it (1-2 % faster with it, cfg2).
template <bool COUNT>
__global__ __launch_bounds__(64, 8) void k_sample(Frame F) {
  sample_body<COUNT>(F, blockIdx.y);
}
#endif

// Frame batches (rm_dispatch_frames): n frames in one grid of gridDim.y x n tile
// rows.  The hardware dispatches workgroups in x, y, z order; (y, z) is read
// row-major over the frames: dispatch slot L = z gridDim.y + y renders tile-row
// slot L / n (inside-out order, tile_row) of frame L % n, so the slowest rows of
// every frame of the batch start first and the launch ends on the cheap rows of
// all its frames (round 5; frame-major order ended each launch on its last
// frame's cheap rows but started every frame's slow rows only after the previous
// frame's whole grid).  Production builds only.
__device__ __forceinline__ void batch_slot(int& frame, int& rowslot) {
  const int L = blockIdx.z * gridDim.y + blockIdx.y, n = gridDim.z;
  // uniform: kept in SGPRs (the division is VALU code)
  rowslot = __builtin_amdgcn_readfirstlane(L / n);
  frame = __builtin_amdgcn_readfirstlane(L - rowslot * n);
}
#ifndef RM_KERNELS_AA_ONLY
__global__ __launch_bounds__(64, 8) void k_pixel_frames(FrameBatch B) {
  int f, r;
  batch_slot(f, r);
  pixel_body<false>(B.f[f], r);
}
#endif
#ifndef RM_KERNELS_PIXEL_ONLY
__global__ __launch_bounds__(64, 8) void k_sample_frames(FrameBatch B) {
  int f, r;
  batch_slot(f, r);
  sample_body<false>(B.f[f], r);
}
#endif

// Reassemble packed shard images into the frame: shard r's rows start at row
// r * rank_stride of `gathered` (rank_stride = rows_cap for [nshards][rows_cap]
// [width]; n * rows_cap for one frame of a batch gathered as [nshards][n]
// [rows_cap][width]).  One grid row per frame row: the source row (shard, local
// row; rm_shard.hpp's weighted interleave) is computed once per workgroup in
// scalar registers; lanes copy 16 B (4 pixels) each when rows are 16-B aligned
// (width % 4 == 0 and both images 16-B aligned), one pixel otherwise.
// RGB3: the shards are packed RGB (3 B per pixel, rm_config.shard_format): a
// lane reads a group of 4 pixels as 3 dwords (rows of 3 width bytes are 4-B
// aligned when width % 4 == 0) and writes them as RGBA with alpha 255, the
// reference's constant alpha 1.0 quantised.
template <bool VEC, bool RGB3>
__global__ __launch_bounds__(256) void k_unshard(const uint32_t* __restrict__ gathered,
                                                 uint32_t* __restrict__ frame, int width,
                                                 int height, rm::ShardMap map,
                                                 size_t rank_stride) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int y = blockIdx.y; y < height; y += gridDim.y) {  // gridDim.y <= 65535
    int r, lrow;
    rm::shard_owner(map, y, &r, &lrow);
    const size_t srow = (size_t)r * rank_stride + lrow;
    uint32_t* dst = frame + (size_t)y * (size_t)width;
    if (RGB3) {
      const uint8_t* src = reinterpret_cast<const uint8_t*>(gathered) + srow * (size_t)width * 3;
      if (VEC) {
        const int nw = width / 4, lanes = (int)(gridDim.x * blockDim.x);
        for (int j = i; j < nw && j < i + 2 * lanes; j += lanes) {
          const uint32_t* s3 = reinterpret_cast<const uint32_t*>(src) + 3 * (size_t)j;
          const uint32_t a = s3[0], b = s3[1], c = s3[2];
          reinterpret_cast<uint4*>(dst)[j] =
              make_uint4(a | 0xff000000u, (a >> 24) | (b << 8) | 0xff000000u,
                         (b >> 16) | (c << 16) | 0xff000000u, (c >> 8) | 0xff000000u);
        }
      } else if (i < width) {
        const uint8_t* p = src + 3 * (size_t)i;
        dst[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | 0xff000000u;
      }
      continue;
    }
    const uint32_t* src = gathered + srow * (size_t)width;
    if (VEC) {
      // two 16-byte words per lane, the lanes of a row strided (round 4,
      // tools/probe_unshard.py: 10.4 against 11.0 us per 4K frame, 6.4 TB/s;
      // four words or non-temporal loads and stores measured slower)
      const int nw = width / 4, lanes = (int)(gridDim.x * blockDim.x);
      if (i < nw) reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
      if (i + lanes < nw)
        reinterpret_cast<uint4*>(dst)[i + lanes] = reinterpret_cast<const uint4*>(src)[i + lanes];
    } else if (i < width) {
      dst[i] = src[i];
    }
  }
}

}  // namespace rmd

// ---- launch wrappers used by rm_api.hip --------------------------------------
namespace rm {

#ifndef RM_KERNELS_AA_ONLY
void pixel_grid(int width, int rows, bool aa, int32_t* gx, int32_t* gy) {
  *gx = aa ? (width + rmd::kSampleTileW - 1) / rmd::kSampleTileW : (width + rmd::kTileW - 1) / rmd::kTileW;
  *gy = aa ? (rows + rmd::kSampleTileH - 1) / rmd::kSampleTileH : (rows + rmd::kTileH - 1) / rmd::kTileH;
}
#endif

// F.grid_x / grid_y must be pixel_grid(F.width, F.rows, F.aa) (make_frame): the
// kernels read the grid from their arguments, not from the hidden dispatch
// arguments, so the prologue's tile arithmetic waits for one round of loads.
#ifndef RM_KERNELS_PIXEL_ONLY
// k_sample lives in its own code object (this file built with RM_KERNELS_AA_ONLY
// and -fno-slp-vectorize, Makefile): see the note at k_sample.
hipError_t launch_sample(const rmd::Frame& F, bool counters, hipStream_t s) {
  const dim3 grid(F.grid_x, F.grid_y);
  if (counters)
    hipLaunchKernelGGL(rmd::k_sample<true>, grid, dim3(64), 0, s, F);
  else
    hipLaunchKernelGGL(rmd::k_sample<false>, grid, dim3(64), 0, s, F);
  return hipGetLastError();
}
#endif
#ifndef RM_KERNELS_PIXEL_ONLY
// n frames of one size and AA setting (rm_dispatch_frames): B.f[0..n) are set,
// every frame's grid_x / grid_y equal to the first's
hipError_t launch_sample_frames(const rmd::FrameBatch& B, int n, hipStream_t s) {
  const dim3 grid(B.f[0].grid_x, B.f[0].grid_y, n);
  hipLaunchKernelGGL(rmd::k_sample_frames, grid, dim3(64), 0, s, B);
  return hipGetLastError();
}
#endif
#ifndef RM_KERNELS_AA_ONLY
hipError_t launch_sample_frames(const rmd::FrameBatch& B, int n, hipStream_t s);
hipError_t launch_frames(const rmd::FrameBatch& B, int n, hipStream_t s) {
  if (n < 1 || n > rmd::kMaxBatch) return hipErrorInvalidValue;
  if (B.f[0].aa) return launch_sample_frames(B, n, s);
  const dim3 grid(B.f[0].grid_x, B.f[0].grid_y, n);
  hipLaunchKernelGGL(rmd::k_pixel_frames, grid, dim3(64), 0, s, B);
  return hipGetLastError();
}

hipError_t launch_sample(const rmd::Frame& F, bool counters, hipStream_t s);
hipError_t launch_pixel(const rmd::Frame& F, bool counters, hipStream_t s) {
  if (F.aa) return launch_sample(F, counters, s);
  const dim3 grid(F.grid_x, F.grid_y);
  if (counters)
    hipLaunchKernelGGL(rmd::k_pixel<true>, grid, dim3(64), 0, s, F);
  else
    hipLaunchKernelGGL(rmd::k_pixel<false>, grid, dim3(64), 0, s, F);
  return hipGetLastError();
}
#endif

#if defined(RM_STATS) && !defined(RM_KERNELS_AA_ONLY)
// Diagnostic builds: rm_debug_stats() (rm_api.hip) reads and clears g_stats.
hipError_t debug_stats(unsigned long long* out, bool clear) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(rmd::g_stats), 64 * sizeof(unsigned long long));
  if (e == hipSuccess && clear) {
    static const unsigned long long z[64] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(rmd::g_stats), z, sizeof z);
  }
  return e;
}
#endif

#ifndef RM_KERNELS_AA_ONLY
hipError_t launch_unshard(const void* gathered, void* frame, int width, int height, int row_block,
                          int row_block0, int nshards, int rows_cap, hipStream_t s, size_t rank_stride_rows,
                          bool rgb3) {
  if (nshards < 1 || row_block < 1 || row_block0 < 1) return hipErrorInvalidValue;
  const rm::ShardMap map{row_block, row_block0, nshards};
  const size_t stride = rank_stride_rows ? rank_stride_rows : (size_t)rows_cap;
  // 16-B copies need 16-B rows (width % 4 == 0) and 16-B aligned images: the
  // C-ABI takes caller pointers, which may be offset (packed RGB sources: 4-B)
  const uintptr_t ga = reinterpret_cast<uintptr_t>(gathered), fa = reinterpret_cast<uintptr_t>(frame);
  const bool vec = width % 4 == 0 && fa % 16 == 0 && ga % (rgb3 ? 4 : 16) == 0;
  const unsigned per_row = (unsigned)(vec ? (width / 4 + 1) / 2 : width);  // lanes per row
  const dim3 grid((per_row + 255) / 256, (unsigned)(height < 65535 ? height : 65535));
  const uint32_t* g = static_cast<const uint32_t*>(gathered);
  uint32_t* f = static_cast<uint32_t*>(frame);
  if (rgb3) {
    if (vec)
      hipLaunchKernelGGL((rmd::k_unshard<true, true>), grid, dim3(256), 0, s, g, f, width, height, map, stride);
    else
      hipLaunchKernelGGL((rmd::k_unshard<false, true>), grid, dim3(256), 0, s, g, f, width, height, map, stride);
  } else if (vec) {
    hipLaunchKernelGGL((rmd::k_unshard<true, false>), grid, dim3(256), 0, s, g, f, width, height, map, stride);
  } else {
    hipLaunchKernelGGL((rmd::k_unshard<false, false>), grid, dim3(256), 0, s, g, f, width, height, map, stride);
  }
  return hipGetLastError();
}
#endif

}  // namespace rm
