"""Render a few cfg frames with one kernel variant (driver for rocprofv3 --pmc)."""
import sys
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd')
import rmarch as rm
kname = sys.argv[1] if len(sys.argv) > 1 else "wavequeue"
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 3
nfr = int(sys.argv[3]) if len(sys.argv) > 3 else 3
W, H, b, aa, sm = {3: (3840, 2160, 3, True, 0), 2: (1920, 1080, 1, False, 0),
                   1: (512, 512, 0, False, 1), 4: (3840, 2160, 5, True, 0)}[cfg]
k = rm.RM_KERNEL_WAVEQUEUE if kname == "wavequeue" else rm.RM_KERNEL_PIXEL
with rm.Renderer(W, H, kernel=k) as r:
    if kname == "table-spec":  # the same, with kernels compiled for the table (hiprtc)
        r.specialize_scene(True)
    if kname in ("table", "table-spec"):  # the reference scene as a runtime table (k_table_* kernels)
        r.set_scene(rm.default_scene())
    for f in range(nfr):
        r.dispatch(rm.sweep_uniforms(10 + f, 120, b, aa, sm))
    r.synchronize()
print("done", kname, cfg)
