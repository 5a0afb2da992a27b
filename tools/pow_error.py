"""Max ulp / abs error of the GPU gamma chain vs the oracle across golden frames."""
import sys, json
import numpy as np
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd'); sys.path.insert(0, 'oracle')
import rmarch as rm, oracle as O
worst = {}
for f, b, aa in [(0, 3, True), (60, 3, True), (119, 5, True), (30, 1, False), (-1, 0, True)]:
    u = rm.sweep_uniforms(f, 120, b, aa, 0)
    W, H = 192, 108
    ref = O.render(u, W, H)
    with rm.Renderer(W, H, outputs=3) as r:
        r.dispatch(u); g32 = r.read_rgba32f(); g8 = r.read_rgba8()
    d = np.abs(g32 - ref["rgba32f"])
    ulp = np.abs(g32.view(np.int32).astype(np.int64) - ref["rgba32f"].view(np.int32).astype(np.int64))
    d8 = np.abs(g8.astype(int) - ref["rgba8"].astype(int))
    print(json.dumps({"f": f, "b": b, "aa": aa, "max_abs": float(d.max()), "max_ulp": int(ulp.max()),
                      "mean_ulp": float(ulp.mean()), "rgba8_max": int(d8.max()),
                      "rgba8_diff_px": int((d8 > 0).any(-1).sum())}))
