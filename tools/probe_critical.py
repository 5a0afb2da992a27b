"""Critical path of rank 0's shard at N = 1, 2, 4, 8 (cfg 3) with one frame in flight:
ms per frame rendered one at a time (the strong-scaling latency of SURVEY 8(e)), for
the librm given by RM_LIBRM.  Diagnostic tool."""
import json
import sys
import time

sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd')
import torch  # noqa: E402
import rmarch as rm  # noqa: E402

W, H, K = 3840, 2160, 24
out = {}
for N in (1, 8):
    kw = dict(row_block=8, shard=0, nshards=N) if N > 1 else {}
    with rm.Renderer(W, H, **kw) as r:
        for f in range(6):
            r.dispatch(rm.sweep_uniforms(f, 120, 3, True, 0))
        r.synchronize()
        r.enable_timing(True)
        r.kernel_time_ms(reset=True)
        t0 = time.perf_counter()
        for f in range(K):
            r.dispatch(rm.sweep_uniforms((f * 120) // K, 120, 3, True, 0))
            r.synchronize()
        dt = (time.perf_counter() - t0) / K * 1e3
        ms, n = r.kernel_time_ms(reset=True)
    out[N] = {"wall_ms": round(dt, 4), "kernel_ms": round(ms / n, 4)}
print(json.dumps(out), flush=True)
