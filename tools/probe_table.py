"""Kernel time of the scene-table path (generic and specialised) vs the built-in scene's kernel (rm_enable_timing).

usage: python tools/probe_table.py [W H bounces aa reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "opengl-raymarching-in-compute-shader_amd"))
import rmarch as rm  # noqa: E402

W, H, B, AA, REPS = (int(a) for a in (sys.argv[1:6] + ["3840", "2160", "3", "1", "20"][len(sys.argv[1:6]):]))
u = rm.sweep_uniforms(45, 120, B, bool(AA), 0)
import time  # noqa: E402

for label, scene, spec in (("builtin", None, False), ("table", rm.default_scene(), False),
                           ("table-spec", rm.default_scene(), True)):
    with rm.Renderer(W, H) as r:
        if spec:
            t0 = time.time()
            r.specialize_scene(True)
            r.set_scene(scene)
            print(f"specialise (hiprtc compile + load): {time.time() - t0:.2f} s", flush=True)
        elif scene is not None:
            r.set_scene(scene)
        for _ in range(3):
            r.dispatch(u)
        r.synchronize()
        r.enable_timing(True)
        r.kernel_time_ms(reset=True)
        for _ in range(REPS):
            r.dispatch(u)
        ms, n = r.kernel_time_ms(reset=True)
        print(f"{label:8s} {W}x{H} b{B} aa{AA}: {ms / n:.3f} ms/frame ({n} launches)", flush=True)
