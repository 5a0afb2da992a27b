"""Diagnostic: wave / lane counters of the RM_STAT points (rm_scene.hpp, rm_kernels.hip).

  tools/build_variant.sh stats -DRM_STATS=1
  RM_LIBRM=tools/variants/librm_stats.so python tools/stats_probe.py [cfg] [frame]

g_stats[k] = waves reaching point k, g_stats[32 + k] = active lanes there.
"""
import ctypes as C
import sys

sys.path.insert(0, "opengl-raymarching-in-compute-shader_amd")
import rmarch as rm  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
frame = int(sys.argv[2]) if len(sys.argv) > 2 else 30
W, H, b, aa, sm = {3: (3840, 2160, 3, True, 0), 2: (1920, 1080, 1, False, 0),
                   1: (512, 512, 0, False, 1), 4: (3840, 2160, 5, True, 0)}[cfg]
L = rm.lib()
L.rm_debug_stats.argtypes = [C.POINTER(C.c_ulonglong)]
h = (C.c_ulonglong * 64)()
with rm.Renderer(W, H) as r:
    r.dispatch(rm.sweep_uniforms(frame, 120, b, aa, sm))
    r.synchronize()
    L.rm_debug_stats(h)  # clears the first (warm-up) frame's counts
    r.dispatch(rm.sweep_uniforms(frame, 120, b, aa, sm))
    r.synchronize()
    assert L.rm_debug_stats(h) == 0
h = list(h)
nm = {0: "cull-sdf(shadow)", 1: "lazy-retests", 2: "shadow-steps", 6: "refl-iters",
      8: "lazy-sdf", 9: "lazy-block", 10: "eval-sph0", 11: "eval-sph1", 12: "eval-blend",
      13: "eval-torus", 14: "eval-capsule", 15: "prim-iters", 16: "retest-sph0",
      17: "retest-sph1", 18: "retest-blend", 19: "retest-torus", 20: "retest-capsule",
      26: "bounce-iters", 27: "normals", 29: "shadows", 30: "render-after-march",
      31: "primary-hit-shade"}
waves = (W * H * (4 if aa else 1) + 63) // 64
print(f"cfg {cfg} frame {frame}: {waves} waves")
print("%-20s %12s %14s %8s %8s" % ("point", "waves", "lanes", "lanes/w", "per wave"))
for k, n in nm.items():
    print("%-20s %12d %14d %8.1f %8.2f" % (n, h[k], h[32 + k], h[32 + k] / h[k] if h[k] else 0.0,
                                           h[k] / waves))
print("march lane utilisation %.3f (primary %.3f, reflected %.3f)"
      % (h[7] / (64.0 * (h[6] + h[15])), h[47] / (64.0 * h[15]), h[38] / (64.0 * max(h[6], 1))))
print("lazy block rate: waves %.3f lanes %.3f" % (h[9] / h[8], h[41] / h[40]))
print("primary rays: %d misses, %.1f steps each; %d hits, %.1f steps each"
      % (h[3], h[4] / max(h[3], 1), h[23], h[5] / max(h[23], 1)))
print("reflected: lane steps of misses %d, of hits %d" % (h[24], h[25]))
