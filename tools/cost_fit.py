"""Attribute k_sample/k_pixel time to work types: time ~ sum_j coef_j * units_j (least squares)."""
import sys, json, itertools
import numpy as np
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd')
import rmarch as rm
rows = []
for b, aa, f, sm in itertools.product([0, 1, 3, 5], [True, False], [0, 40, 80, 119], [0]):
    W, H = 3840, 2160
    u = rm.sweep_uniforms(f, 120, b, aa, sm)
    with rm.Renderer(W, H) as r:
        r.enable_timing(True)
        r.dispatch(u); r.dispatch(u)
        r.kernel_time_ms(reset=True)
        for _ in range(3): r.dispatch(u)
        ms, n = r.kernel_time_ms(reset=True)
    with rm.Renderer(W, H, counters=True) as r:
        r.dispatch(u); c = r.counters()
    rows.append((ms / n, c, b, aa, f))
    print(json.dumps({"b": b, "aa": aa, "f": f, "ms": round(ms / n, 3), **c}), flush=True)
keys = ["march_steps", "reflect_steps", "shadow_steps", "normals", "lights", "rays"]
A = np.array([[r[1][k] for k in keys] for r in rows], float)
y = np.array([r[0] for r in rows])
coef, *_ = np.linalg.lstsq(A, y, rcond=None)
print("ns per unit:", {k: round(c * 1e6, 4) for k, c in zip(keys, coef)})
pred = A @ coef
print("fit rel err max", float(np.max(np.abs(pred - y) / y)))
for r, p in zip(rows, pred):
    if r[2] == 3 and r[3]:
        share = {k: round(float(coef[i] * r[1][k] / r[0]), 3) for i, k in enumerate(keys)}
        print("cfg3-like share", r[4], share)
