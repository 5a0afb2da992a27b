"""Debug: production (no counters) vs counting build vs oracle for one uniform set."""
import sys, os
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd'); sys.path.insert(0, 'oracle')
import numpy as np
import rmarch as rm
import oracle as O
W, H = 80, 48
b, aa = int(sys.argv[1]), bool(int(sys.argv[2]))
light = [float(v) for v in sys.argv[3].split(',')] if len(sys.argv) > 3 else None
u = rm.sweep_uniforms(20, 120, b, aa, 0)
if light:
    for i in range(3): u.light.position[i] = light[i]
ref = O.render(u, W, H)["rgba32f"]
out = {}
for cnt in (True, False):
    with rm.Renderer(W, H, outputs=3, kernel=rm.RM_KERNEL_PIXEL, counters=cnt) as r:
        r.dispatch(u); out[cnt] = r.read_rgba32f()
d = np.abs(out[False] - out[True]).max(-1)
ys, xs = np.nonzero(d > 1e-6)
print("differing px", len(ys))
for y, x in list(zip(ys, xs))[:12]:
    print(y, x, "prod", out[False][y, x, :3], "count", out[True][y, x, :3], "oracle", ref[y, x, :3])
