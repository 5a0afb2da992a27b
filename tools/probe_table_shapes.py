"""Kernel time per cfg3 frame of tables that are not reference-shaped:
the generic and the specialised table kernels against the built-in scene's kernel
(rm_enable_timing, one frame at a time, the bench's sweep frames).

  python tools/probe_table_shapes.py [frames] [shape ...]

Shapes (the reference scene, rm_default_scene, reshaped):
  reference  the scene itself (smarch)
  planes2    plus a ceiling plane after the floor: two planes, the floor not last
  plane_mid  the floor moved to the middle of the table
  tilted     the floor's normal tilted by 0.05 in x (not axis-aligned)
  many       plus four spheres: 9 bounded entries, one more than the slots
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd"))
import rmarch as rm  # noqa: E402


def clone(p):
    q = rm.rm_primitive()
    C.memmove(C.byref(q), C.byref(p), C.sizeof(q))
    return q


def shape_table(name):
    sc = rm.default_scene()
    floor = sc[-1]
    if name == "reference":
        return sc
    if name == "planes2":
        ceil = clone(floor)
        ceil.param[:] = [0.0, -1.0, 0.0, 40.0, 0.0, 0.0, 0.0]
        ceil.id = 8
        return sc + [ceil]
    if name == "plane_mid":
        return sc[:2] + [floor] + sc[2:-1]
    if name == "tilted":
        f = clone(floor)
        n = (0.05, 1.0, 0.0)
        ln = (n[0] ** 2 + n[1] ** 2) ** 0.5
        f.param[:] = [n[0] / ln, n[1] / ln, 0.0, 5.5, 0.0, 0.0, 0.0]
        return sc[:-1] + [f]
    if name == "many":
        extra = []
        for i, (x, z) in enumerate(((30.0, -20.0), (-40.0, -25.0), (8.0, -40.0), (-15.0, 20.0))):
            s = clone(sc[0])
            s.center[:] = [x, 1.0, z]
            s.param[0] = 2.0 + 0.5 * i
            s.id = 10 + i
            extra.append(s)
        return sc[:-1] + extra + [floor]
    raise ValueError(name)


SHAPES = ["reference", "planes2", "plane_mid", "tilted", "many"]


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    shapes = sys.argv[2:] or SHAPES
    W, H = 3840, 2160
    us = [rm.sweep_uniforms((k * 120) // frames, 120, 3, True, 0) for k in range(frames)]

    def time_it(scene, spec):
        with rm.Renderer(W, H) as r:
            if spec:
                r.specialize_scene(True)
            if scene is not None:
                r.set_scene(scene)
            for u in us[:2]:
                r.dispatch(u)
            r.synchronize()
            r.enable_timing(True)
            r.kernel_time_ms(reset=True)
            for u in us:
                r.dispatch(u)
            ms, n = r.kernel_time_ms(reset=True)
            waves = r.scene_kernel_waves() if spec else 0
            return ms / n, waves

    base, _ = time_it(None, False)
    print(json.dumps({"shape": "builtin", "ms_per_frame": round(base, 4)}), flush=True)
    for name in shapes:
        sc = shape_table(name)
        words = rm.scene_words(sc)
        nslots = int(words[len(sc) * 24 + 25].view("float32"))
        g, _ = time_it(sc, False)
        s, w = time_it(sc, True)
        print(json.dumps({"shape": name, "entries": len(sc), "slots": nslots,
                          "generic_ms": round(g, 4), "generic_x": round(g / base, 3),
                          "specialised_ms": round(s, 4), "specialised_x": round(s / base, 3),
                          "specialised_waves": w}), flush=True)


if __name__ == "__main__":
    main()
