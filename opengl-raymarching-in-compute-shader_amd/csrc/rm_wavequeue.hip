// rm_wavequeue.hip — the performance kernel for the per-pixel sphere tracer.
//
// Same pure function of (pixel, uniforms) as computeShader.glsl:291-344 and
// k_pixel, restructured for a 64-lane CDNA4 wave:
//
//  * Persistent waves pull 64-pixel chunks from a global counter (one
//    atomicAdd per chunk) and hand pixels to idle lanes with a ballot +
//    popcount (mbcnt), so a lane whose pixel is done takes a new one instead
//    of idling until the slowest lane of the wave finishes.
//  * Each lane runs its samples as a phase machine.  The hot loop body is ONE
//    scene sdf per iteration for every lane that is marching, whatever it is
//    marching for: the 512-step primary march (RayMarch glsl:125-142), the
//    256-step reflection marches (glsl:144-161), the GetNormal probes
//    (glsl:278-288) and the 16-step shadow march (glsl:201-216).
//  * Shading (normalize, getPointLight, pow gamma, castRay, the bounce
//    bookkeeping) is batched: a lane that reaches such an event parks, and the
//    wave runs the shading code for all parked lanes together once at least
//    `batch` lanes are parked or idle (or none is marching).  Without the
//    batching nearly every iteration has some lane with an event, and the
//    whole wave would pay for shading on every step.
//
// Every lane performs the reference's float operations in the reference's
// order, so results are bit-identical to k_pixel and the oracle (scheduling
// changes nothing).  Value-preserving shortcuts:
//  * the primary-hit GetNormal reuses the last march sdf as its centre sample
//    (the march point and `pos` are the same float expression, glsl:132/226);
//  * the GetNormal of a miss on the last bounce is skipped (never read);
//  * after a MATTE (floor) hit inside bounce() the remaining iterations are
//    colour no-ops (glsl:189-190): the sample finishes there.
// Counters are kept in the reference's units (live work, see rm_oracle.h).
#include <hip/hip_runtime.h>

#include "rm_scene.hpp"

#ifndef RM_SHADOW_EXIT
#define RM_SHADOW_EXIT 1
#endif
#ifndef RM_MISS_EXIT
#define RM_MISS_EXIT 1
#endif

namespace rmd {

enum : int { PH_IDLE = 0, PH_PEND = 1, PH_MARCH = 2, PH_NORMAL = 3, PH_SHADOW = 4 };
// parked events
enum : int { E_PMISS = 1, E_NDONE = 2, E_RESOLVE = 3, E_SDONE = 4 };

constexpr int kChunk = 64;   // pixels per queue pull
constexpr int kBlock = 256;  // threads per workgroup (4 waves)

struct WQFrame {
  Frame F;
  float offx[4], offy[4];  // 0.25/W, 0.75/W ... (glsl:311-332), host-divided
  uint32_t total;          // pixels in this launch = rows * width
  int32_t batch;           // shading runs when >= batch lanes are not marching
};

__device__ __forceinline__ f3 sky_primary(f3 rd) { return subs(mk(0.30f, 0.36f, 0.60f), rd.y * 0.2f); }
__device__ __forceinline__ f3 sky_bounce(f3 rd) { return subs(mk(0.36f, 0.36f, 0.60f), rd.y * 0.2f); }

template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_wavequeue(WQFrame W) {
  const Frame& F = W.F;
  const int lane = threadIdx.x & 63;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int nsamp = F.aa ? 4 : 1;
  const f3 lpos = mk(F.lpos[0], F.lpos[1], F.lpos[2]);

  // ---- lane state --------------------------------------------------------
  int pix = -1;                        // launch-local pixel index, -1 = none
  int s = 0;                           // sample index
  float ux = 0.f, uy = 0.f;            // cumulative uv (glsl:302-332)
  float ar = 0.f, ag = 0.f, ab = 0.f;  // fixed-order sample accumulator (glsl:315-335)
  int phase = PH_IDLE;
  int pend = 0;                        // parked event (phase == PH_PEND)
  f3 ro = mk(0.f, 0.f, 0.f), rd = mk(0.f, 0.f, 0.f);
  float t = 0.f;
  int i = 0;                           // step counter (MARCH, SHADOW) or probe index (NORMAL)
  f3 pos = mk(0.f, 0.f, 0.f);
  float c0 = 0.f, nx = 0.f, ny = 0.f, nz = 0.f;  // GetNormal probes
  f3 col = mk(0.f, 0.f, 0.f);          // render()/bounce() `color`
  f3 pcol = mk(0.f, 0.f, 0.f);         // bounce prevColor (or the stashed term after a shadow)
  int bi = 0;                          // 0 = primary ray, 1..bounceVar = bounce()
  int hid = -1;                        // id of the current hit (-1 = miss)
  float hchk = 0.f;                    // checkers() at the current hit point
  float res = 1.f;                     // softshadow running minimum
  float sx = 0.f;                          // early-exit bounds of the current march / shadow
  uint32_t c_pix = 0;
  uint32_t c_rays = 0, c_march = 0, c_refl = 0, c_shadow = 0, c_norm = 0, c_light = 0;
  uint32_t c_iters = 0;

  // ---- per-wave job pool (wave-uniform) ---------------------------------------
  uint32_t pool_next = 0, pool_end = 0;
  bool exhausted = false;

  // Begin sample `s` of the lane's pixel: castRay (glsl:68-74, 311-332).
  auto start_sample = [&]() {
    if (F.aa) {
      ux += W.offx[s];
      uy += W.offy[s];
    }
    cast_ray(F, ux, uy, ro, rd);
    col = sky_primary(rd);
    t = 0.f;
    i = 0;
    bi = 0;
    sx = miss_exit_init(ro, rd);
    phase = PH_MARCH;
    if (COUNT) c_rays++;
  };
  auto add_sample = [&](f3 c) {  // pow gamma (glsl:238/247) + accumulate
    f3 g = gamma(c);
    ar += g.x;
    ag += g.y;
    ab += g.z;
  };

  while (true) {
    const unsigned long long act =
        __ballot(phase == PH_MARCH || phase == PH_NORMAL || phase == PH_SHADOW);
    const unsigned long long waiting = __ballot(phase == PH_PEND || (phase == PH_IDLE && !exhausted));
    if (waiting != 0ull && (act == 0ull || __popcll(act) <= 64 - W.batch)) {
      // ================= batched shading for parked lanes ==================
      if (phase == PH_PEND) {
        int ev = pend;
        bool sample_done = false;
        f3 nrm = mk(0.f, 0.f, 0.f);
        if (ev == E_NDONE) {
          nrm = normalize(subs(mk(nx, ny, nz), c0));  // glsl:284-286
          if (bi == 0) {
            f3 hc = id_color(hid, hchk);
            if (COUNT) c_light++;
            col = point_light(F, hc, nrm, pos);  // glsl:230
            if (hid == 7) {
              // floor: soft shadow, then return (glsl:232-240)
              ro = add(pos, muls(nrm, 0.02f));
              rd = sub(lpos, pos);
              t = 0.f;
              i = 0;
              res = 1.f;
              sx = shadow_exit_init(F.k, ro, rd);
              phase = PH_SHADOW;
            } else if (F.bounces > 0) {
              pcol = hc;  // prevColor = primaryObject.color (glsl:167)
              bi = 1;
              rd = reflect(rd, nrm);  // glsl:171-172
              ro = add(pos, muls(nrm, 0.001f));
              t = 0.f;
              i = 0;
              sx = miss_exit_init(ro, rd);
              phase = PH_MARCH;
            } else {
              add_sample(col);
              sample_done = true;
            }
          } else {
            ev = E_RESOLVE;
          }
        }
        if (ev == E_RESOLVE) {  // bounce bi (glsl:176-195); prevObject is not MATTE here
          f3 tc;
          if (hid == -1) {
            tc = sky_bounce(rd);
          } else {
            if (COUNT) c_light++;
            tc = point_light(F, id_color(hid, hchk), nrm, pos);
          }
          const f3 term = divi(mul(tc, pcol), bi);
          if (hid == 7 && bi < 3) {
            pcol = term;  // stash: added after the shadow scales `color`
            ro = add(pos, muls(nrm, 0.02f));
            rd = sub(lpos, pos);
            t = 0.f;
            i = 0;
            res = 1.f;
            sx = shadow_exit_init(F.k, ro, rd);
            phase = PH_SHADOW;
          } else {
            col = add(col, term);
            pcol = tc;
            if (hid == 7 || bi >= F.bounces) {
              add_sample(col);  // a floor hit ends the useful bounces (glsl:189-190)
              sample_done = true;
            } else {
              ++bi;
              rd = reflect(rd, nrm);
              ro = add(pos, muls(nrm, 0.001f));
              t = 0.f;
              i = 0;
              sx = miss_exit_init(ro, rd);
              phase = PH_MARCH;
            }
          }
        } else if (ev == E_PMISS) {
          add_sample(col);  // render(): a miss keeps the sky colour (glsl:220,247)
          sample_done = true;
        } else if (ev == E_SDONE) {
          if (bi == 0) {
            col = muls(col, res);  // glsl:237
          } else {
            col = muls(col, div_small(res, bi));  // glsl:186
            col = add(col, pcol);              // t.color * prevColor / i (glsl:192)
          }
          add_sample(col);
          sample_done = true;
        }
        if (sample_done) {
          ++s;
          if (s < nsamp) {
            start_sample();
          } else {
            if (F.aa) store_pixel(F, (size_t)pix, ar / 4.0f, ag / 4.0f, ab / 4.0f, 1.0f);
            else store_pixel(F, (size_t)pix, ar, ag, ab, 1.0f);
            if (COUNT) F.sdf_counts[pix] = c_pix;
            pix = -1;
            phase = PH_IDLE;
          }
        }
      }
      // ---------------- refill idle lanes and start their first sample ----------------
      unsigned long long need = __ballot(phase == PH_IDLE);
      while (need != 0ull && !exhausted) {
        if (pool_next >= pool_end) {
          uint32_t base = 0;
          if (lane == 0) base = atomicAdd(F.queue, (uint32_t)kChunk);
          base = __builtin_amdgcn_readfirstlane(base);
          if (base >= W.total) {
            exhausted = true;
            break;
          }
          pool_next = base;
          pool_end = min(base + (uint32_t)kChunk, W.total);
        }
        const uint32_t avail = pool_end - pool_next;
        const uint32_t rank = (uint32_t)__popcll(need & lt_mask);
        if (phase == PH_IDLE && rank < avail) {
          pix = (int)(pool_next + rank);
          const int lrow = pix / F.width;
          const int px = pix - lrow * F.width;
          const int py = global_row(F, lrow);
          if (py < 0) {  // padding row of a shard image
            store_pixel(F, (size_t)pix, 0.f, 0.f, 0.f, 0.f);
            if (COUNT) F.sdf_counts[pix] = 0;
            pix = -1;
          } else {
            s = 0;
            ar = ag = ab = 0.f;
            c_pix = 0;
            ux = (float)(px * 2 - F.width) / (float)F.width;   // glsl:302
            uy = (float)(py * 2 - F.height) / (float)F.height; // glsl:303
            start_sample();
          }
        }
        pool_next += min((uint32_t)__popcll(need), avail);
        need = __ballot(phase == PH_IDLE);
      }
      if (exhausted && __ballot(phase != PH_IDLE) == 0ull) break;
      continue;
    }

    // ===================== the one sdf evaluation of this iteration =====================
    if (COUNT) c_iters++;
    const bool isn = (phase == PH_NORMAL);
    const f3 base = isn ? pos : ro;
    const f3 dir =
        isn ? mk(i == 1 ? 0.001f : 0.f, i == 2 ? 0.001f : 0.f, i == 3 ? 0.001f : 0.f) : rd;
    const float tq = isn ? 1.0f : t;
    const f3 q = add(base, muls(dir, tq));  // ro + rd*t, or pos + eps_k (glsl:132,151,207,284)
    int qid;
    const float d = scene<true>(q, F.blend, F.omblend, qid);

    if (phase == PH_MARCH) {
      if (COUNT) {
        if (bi == 0) c_march++;
        else c_refl++;
        c_pix++;
      }
      const bool hit = d < 0.000001f * t;  // glsl:133
      bool miss = false;
      if (!hit) {
        if (d > (bi == 0 ? 400.0f : 200.0f)) {  // glsl:136
          miss = true;
        } else {
          t += d;
          ++i;
          miss = (i >= (bi == 0 ? 512 : 256));
          // provable miss (rm_scene.hpp "early exits"); counting runs the full march
          if (!COUNT && RM_MISS_EXIT && lin_exit(sx, t)) miss = true;
        }
      }
      if (hit) {
        hid = qid;
        hchk = (qid == 7) ? checkers(q) : 0.f;
        if (COUNT) {
          c_norm++;
          c_pix += 4;
        }
        if (bi == 0) {
          pos = q;  // == ro + rd * t, the same float expression (glsl:226)
          c0 = d;   // GetNormal's centre sample sdf(pos) is this very sdf
          i = 1;
        } else {
          pos = add(pos, muls(rd, t));  // glsl:173
          i = 0;
        }
        phase = PH_NORMAL;
      } else if (miss) {
        if (bi == 0) {
          phase = PH_PEND;
          pend = E_PMISS;
        } else {
          pos = add(pos, muls(rd, -1.0f));  // t.hitpoint == -1 (glsl:173)
          hid = -1;
          if (bi < F.bounces) {  // the normal feeds the next reflect
            if (COUNT) {
              c_norm++;
              c_pix += 4;
            }
            i = 0;
            phase = PH_NORMAL;
          } else {
            phase = PH_PEND;
            pend = E_RESOLVE;
          }
        }
      }
    } else if (phase == PH_SHADOW) {
      if (COUNT) {
        c_shadow++;
        c_pix++;
      }
      bool done;
      if (d < 0.001f) {  // glsl:208-209
        res = 0.05f;
        done = true;
      } else {
        res = shadow_min(res, F.k, d, t);  // glsl:211
        t += d;
        ++i;
        done = (i >= 16);
        if (!done && RM_SHADOW_EXIT && lin_exit(sx, t)) {  // the remaining steps are no-ops
          if (COUNT) {
            c_shadow += 16 - i;
            c_pix += 16 - i;
          }
          done = true;
        }
      }
      if (done) {
        phase = PH_PEND;
        pend = E_SDONE;
      }
    } else if (phase == PH_NORMAL) {
      if (i == 0) c0 = d;
      else if (i == 1) nx = d;
      else if (i == 2) ny = d;
      else {
        nz = d;
        phase = PH_PEND;
        pend = E_NDONE;
      }
      ++i;
    }
  }

  if (COUNT) {
    atomicAdd(&F.counters[0], (unsigned long long)c_rays);
    atomicAdd(&F.counters[1], (unsigned long long)c_march);
    atomicAdd(&F.counters[2], (unsigned long long)c_refl);
    atomicAdd(&F.counters[3], (unsigned long long)c_shadow);
    atomicAdd(&F.counters[4], (unsigned long long)c_norm);
    atomicAdd(&F.counters[5], (unsigned long long)c_light);
    if (lane == 0) atomicAdd(&F.counters[6], (unsigned long long)c_iters);
  }
}

}  // namespace rmd

namespace rm {

int g_wq_batch = 24;          // tunable via RM_WQ_BATCH (read at rm_create)
int g_wq_blocks_per_cu = 8;   // tunable via RM_WQ_BLOCKS_PER_CU

hipError_t launch_wavequeue(const rmd::Frame& F, bool counters, hipStream_t s, int num_cus) {
  rmd::WQFrame W;
  W.F = F;
  const float ox[4] = {0.25f, 0.75f, 0.25f, 0.75f};
  const float oy[4] = {0.25f, 0.25f, 0.75f, 0.75f};
  for (int k = 0; k < 4; ++k) {
    W.offx[k] = ox[k] / (float)F.width;  // glsl:311-332: 0.25 / dims.x ...
    W.offy[k] = oy[k] / (float)F.height;
  }
  W.total = (uint32_t)((size_t)F.rows * (size_t)F.width);
  W.batch = g_wq_batch < 1 ? 1 : (g_wq_batch > 64 ? 64 : g_wq_batch);
  const uint32_t chunks = (W.total + rmd::kChunk - 1) / rmd::kChunk;
  const uint32_t waves_per_block = rmd::kBlock / 64;
  uint32_t blocks = (uint32_t)num_cus * (uint32_t)(g_wq_blocks_per_cu > 0 ? g_wq_blocks_per_cu : 8);
  const uint32_t max_useful = (chunks + waves_per_block - 1) / waves_per_block;
  if (blocks > max_useful) blocks = max_useful;
  if (blocks == 0) blocks = 1;
  if (counters)
    hipLaunchKernelGGL(rmd::k_wavequeue<true>, dim3(blocks), dim3(rmd::kBlock), 0, s, W);
  else
    hipLaunchKernelGGL(rmd::k_wavequeue<false>, dim3(blocks), dim3(rmd::kBlock), 0, s, W);
  return hipGetLastError();
}

}  // namespace rm
