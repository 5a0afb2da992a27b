// rm_wavequeue.hip — the performance kernel for the per-pixel sphere tracer.
//
// Same pure function of (pixel, uniforms) as computeShader.glsl:291-344 and
// k_pixel, restructured for a 64-lane CDNA4 wave:
//
//  * Persistent waves pull 64-pixel chunks from a global counter (one
//    atomicAdd per chunk), then hand pixels to idle lanes with a ballot +
//    popcount (mbcnt) — a lane whose pixel is done gets a new one at the next
//    iteration instead of idling until the slowest lane of the wave finishes.
//  * Each lane runs its pixel's samples as a phase machine (MARCH, NORMAL,
//    SHADOW) so that every loop iteration evaluates exactly ONE scene sdf for
//    all live lanes, whatever phase each is in: the 512-step primary march,
//    the 256-step reflection marches, the 4 GetNormal probes and the 16-step
//    shadow march all share the one hot sdf body (the ~95 % cost).
//  * Phase transitions (hit/miss/normal done/shadow done/sample done) are the
//    rare, divergent part; shading (getPointLight, gamma pow) runs there.
//
// Every lane performs the reference's float operations in the reference's
// order, so results are bit-identical to k_pixel (the order in which lanes
// take pixels changes nothing).  Value-preserving shortcuts:
//  * the primary-hit GetNormal reuses the last march sdf as its centre sample
//    (the march point and `pos` are the same float expression);
//  * the GetNormal of a bounce that missed on the LAST bounce is skipped
//    (its result is never read: reflect happens only on a following bounce);
//  * after a MATTE (floor) hit inside bounce(), the remaining iterations are
//    no-ops for colour (glsl:189-190) and the sample finishes early.
// Counters are kept in the reference's units (calls as written in the GLSL).
#include <hip/hip_runtime.h>

#include "rm_scene.hpp"

namespace rmd {

enum : int { PH_IDLE = 0, PH_MARCH = 1, PH_NORMAL = 2, PH_SHADOW = 3 };

constexpr int kChunk = 64;      // pixels per queue pull
constexpr int kBlock = 256;     // threads per workgroup (4 waves)

struct WQFrame {
  Frame F;
  float offx[4], offy[4];  // 0.25/W, 0.75/W ... (glsl:311-332), host-divided
  uint32_t total;          // pixels in this launch = rows * width
};

__device__ __forceinline__ f3 sky_primary(f3 rd) { return subs(mk(0.30f, 0.36f, 0.60f), rd.y * 0.2f); }
__device__ __forceinline__ f3 sky_bounce(f3 rd) { return subs(mk(0.36f, 0.36f, 0.60f), rd.y * 0.2f); }

template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_wavequeue(WQFrame W) {
  const Frame& F = W.F;
  const int lane = threadIdx.x & 63;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int nsamp = F.aa ? 4 : 1;

  // ---- lane state --------------------------------------------------------
  int pix = -1;          // launch-local pixel index, -1 = none
  int s = 0;             // sample index
  float ux = 0.f, uy = 0.f;        // cumulative uv (glsl:305-332)
  float ar = 0.f, ag = 0.f, ab = 0.f;  // fixed-order sample accumulator
  int phase = PH_IDLE;
  f3 ro = mk(0.f, 0.f, 0.f), rd = mk(0.f, 0.f, 0.f);
  float t = 0.f;
  int i = 0;             // step counter (MARCH, SHADOW) or probe index (NORMAL)
  f3 pos = mk(0.f, 0.f, 0.f);
  float c0 = 0.f, nx = 0.f, ny = 0.f;  // GetNormal probes
  f3 nrm = mk(0.f, 0.f, 0.f);
  f3 col = mk(0.f, 0.f, 0.f);      // colour being built (render/bounce `color`)
  f3 pcol = mk(0.f, 0.f, 0.f);     // bounce prevColor (or the stashed term, see below)
  int bi = 0;            // bounce index: 0 = primary ray, 1..bounceVar = bounce()
  int hid = -1;          // id of the current hit (-1 = dummy/miss)
  float hchk = 0.f;      // checkers() value at the current hit point (floor only)
  float res = 1.f;       // softshadow running minimum
  // counters (reference units)
  uint32_t c_pix = 0;
  uint32_t c_rays = 0, c_march = 0, c_refl = 0, c_shadow = 0, c_norm = 0, c_light = 0;

  // ---- per-wave job pool ----------------------------------------------------
  uint32_t pool_next = 0, pool_end = 0;  // wave-uniform
  bool exhausted = false;                 // wave-uniform

  const f3 lpos = mk(F.lpos[0], F.lpos[1], F.lpos[2]);

  while (true) {
    // ---- refill idle lanes -------------------------------------------------
    unsigned long long need = __ballot(pix < 0);
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
      if (pix < 0 && rank < avail) {
        pix = (int)(pool_next + rank);
        // start the pixel (glsl:296-305)
        const int lrow = pix / F.width;
        const int px = pix - lrow * F.width;
        const int py = global_row(F, lrow);
        s = 0;
        ar = ag = ab = 0.f;
        c_pix = 0;
        if (py < 0) {
          // padding row of a shard image: nothing to render
          store_pixel(F, (size_t)pix, 0.f, 0.f, 0.f, 0.f);
          if (COUNT) F.sdf_counts[pix] = 0;
          pix = -1;
        } else {
          ux = (float)(px * 2 - F.width) / (float)F.width;
          uy = (float)(py * 2 - F.height) / (float)F.height;
          phase = PH_IDLE;  // the sample is started below
        }
      }
      const uint32_t nneed = (uint32_t)__popcll(need);
      pool_next += min(nneed, avail);
      need = __ballot(pix < 0);
    }
    if (exhausted && __ballot(pix >= 0) == 0ull) break;

    // ---- start a sample for lanes that have a pixel but no phase ------------
    if (pix >= 0 && phase == PH_IDLE) {
      if (F.aa) {
        ux += W.offx[s];
        uy += W.offy[s];
      }
      cast_ray(F, ux, uy, ro, rd);
      col = sky_primary(rd);
      t = 0.f;
      i = 0;
      bi = 0;
      phase = PH_MARCH;
      if (COUNT) c_rays++;
    }

    // ---- the one sdf evaluation of this iteration -------------------------------
    const bool isn = (phase == PH_NORMAL);
    f3 base = isn ? pos : ro;
    f3 dir = isn ? mk(i == 1 ? 0.001f : 0.f, i == 2 ? 0.001f : 0.f, i == 3 ? 0.001f : 0.f) : rd;
    float tq = isn ? 1.0f : t;
    f3 q = add(base, muls(dir, tq));
    int qid;
    float d = scene<true>(q, F.blend, F.omblend, qid);
    if (phase == PH_IDLE) continue;  // lane has no work (tail of the queue)

    // ---- phase update (cheap, common) -------------------------------------------
    int ev = 0;  // 1 hit, 2 miss, 3 normal done, 4 shadow done
    if (phase == PH_MARCH) {
      if (COUNT) {
        if (bi == 0) c_march++;
        else c_refl++;
        c_pix++;
      }
      if (d < 0.000001f * t) {
        ev = 1;
      } else if (d > (bi == 0 ? 400.0f : 200.0f)) {
        ev = 2;
      } else {
        t += d;
        ++i;
        if (i >= (bi == 0 ? 512 : 256)) ev = 2;
      }
    } else if (phase == PH_SHADOW) {
      if (COUNT) {
        c_shadow++;
        c_pix++;
      }
      if (d < 0.001f) {
        res = 0.05f;
        ev = 4;
      } else {
        res = gmin(res, F.k * d / t);
        t += d;
        ++i;
        if (i >= 16) ev = 4;
      }
    } else {  // PH_NORMAL
      if (i == 0) c0 = d;
      else if (i == 1) nx = d;
      else if (i == 2) ny = d;
      if (i == 3) {
        nrm = normalize(subs(mk(nx, ny, d), c0));
        ev = 3;
      }
      ++i;
    }

    // ---- transitions (divergent, rare) ---------------------------------------------
    while (ev != 0) {
      int next = 0;
      if (ev == 1) {  // march hit
        hid = qid;
        hchk = (qid == 7) ? checkers(q) : 0.f;
        if (COUNT) {
          c_norm++;
          c_pix += 4;
        }
        if (bi == 0) {
          pos = q;        // == ro + rd * t, the same float expression (glsl:226)
          c0 = d;         // GetNormal's centre sample sdf(pos) == this sdf
          i = 1;
        } else {
          pos = add(pos, muls(rd, t));  // glsl:173
          i = 0;
        }
        phase = PH_NORMAL;
      } else if (ev == 2) {  // march miss
        if (bi == 0) {
          // render(): miss keeps the sky colour (glsl:220,247)
          f3 g = gamma(col);
          ar += g.x;
          ag += g.y;
          ab += g.z;
          next = 5;
        } else {
          pos = add(pos, muls(rd, -1.0f));  // t.hitpoint == -1 (glsl:173)
          hid = -1;
          if (bi < F.bounces) {
            if (COUNT) {
              c_norm++;
              c_pix += 4;
            }
            i = 0;
            phase = PH_NORMAL;
          } else {
            next = 6;  // last bounce: normal unused
          }
        }
      } else if (ev == 3) {  // GetNormal done
        if (bi == 0) {
          f3 hc = id_color(hid, hchk);
          if (COUNT) c_light++;
          col = point_light(F, hc, nrm, pos);  // glsl:230
          if (hid == 7) {
            // floor: soft shadow then return (glsl:232-240)
            ro = add(pos, muls(nrm, 0.02f));
            rd = sub(lpos, pos);
            t = 0.f;
            i = 0;
            res = 1.f;
            phase = PH_SHADOW;
          } else if (F.bounces > 0) {
            pcol = hc;  // prevColor = primaryObject.color (glsl:167)
            bi = 1;
            next = 7;   // start bounce 1
          } else {
            f3 g = gamma(col);
            ar += g.x;
            ag += g.y;
            ab += g.z;
            next = 5;
          }
        } else {
          next = 6;
        }
      } else if (ev == 4) {  // shadow done
        if (bi == 0) {
          col = muls(col, res);  // glsl:237
        } else {
          col = muls(col, res / (float)bi);  // glsl:186
          col = add(col, pcol);              // stashed t.color*prevColor/i (glsl:192)
        }
        f3 g = gamma(col);
        ar += g.x;
        ag += g.y;
        ab += g.z;
        next = 5;
      } else if (ev == 6) {  // resolve bounce bi (glsl:176-195); prevObject is not MATTE here
        f3 tc;
        if (hid == -1) {
          tc = sky_bounce(rd);
        } else {
          f3 hc = id_color(hid, hchk);
          if (COUNT) c_light++;
          tc = point_light(F, hc, nrm, pos);
        }
        f3 term = divs(mul(tc, pcol), (float)bi);
        if (hid == 7 && bi < 3) {
          pcol = term;  // stash; added after the shadow scales `color`
          ro = add(pos, muls(nrm, 0.02f));
          rd = sub(lpos, pos);
          t = 0.f;
          i = 0;
          res = 1.f;
          phase = PH_SHADOW;
        } else {
          col = add(col, term);
          pcol = tc;
          if (hid == 7 || bi >= F.bounces) {
            // floor hit: every later iteration is a no-op (glsl:189-190)
            f3 g = gamma(col);
            ar += g.x;
            ag += g.y;
            ab += g.z;
            next = 5;
          } else {
            ++bi;
            next = 7;
          }
        }
      } else if (ev == 7) {  // start reflected march of bounce bi (glsl:171-172)
        rd = reflect(rd, nrm);
        ro = add(pos, muls(nrm, 0.001f));
        t = 0.f;
        i = 0;
        phase = PH_MARCH;
      } else if (ev == 5) {  // sample done
        ++s;
        if (s < nsamp) {
          phase = PH_IDLE;  // next sample starts at the top of the loop
        } else {
          if (F.aa) store_pixel(F, (size_t)pix, ar / 4.0f, ag / 4.0f, ab / 4.0f, 1.0f);
          else store_pixel(F, (size_t)pix, ar, ag, ab, 1.0f);
          if (COUNT) F.sdf_counts[pix] = c_pix;
          pix = -1;
          phase = PH_IDLE;
        }
      }
      ev = next;
    }
  }

  if (COUNT) {
    atomicAdd(&F.counters[0], (unsigned long long)c_rays);
    atomicAdd(&F.counters[1], (unsigned long long)c_march);
    atomicAdd(&F.counters[2], (unsigned long long)c_refl);
    atomicAdd(&F.counters[3], (unsigned long long)c_shadow);
    atomicAdd(&F.counters[4], (unsigned long long)c_norm);
    atomicAdd(&F.counters[5], (unsigned long long)c_light);
  }
}

}  // namespace rmd

namespace rm {

hipError_t launch_wavequeue(const rmd::Frame& F, bool counters, hipStream_t s, int num_cus) {
  rmd::WQFrame W;
  W.F = F;
  const float ox[4] = {0.25f, 0.75f, 0.25f, 0.75f};
  const float oy[4] = {0.25f, 0.25f, 0.75f, 0.75f};
  for (int k = 0; k < 4; ++k) {
    W.offx[k] = ox[k] / (float)F.width;   // glsl:311-332: 0.25 / dims.x ...
    W.offy[k] = oy[k] / (float)F.height;
  }
  W.total = (uint32_t)((size_t)F.rows * (size_t)F.width);
  const uint32_t chunks = (W.total + rmd::kChunk - 1) / rmd::kChunk;
  const uint32_t waves_per_block = rmd::kBlock / 64;
  uint32_t blocks = (uint32_t)num_cus * 8u;  // 32 waves / CU resident at most
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
