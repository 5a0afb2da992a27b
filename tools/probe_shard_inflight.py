"""Render-only throughput of rank 0's shard at N = 1, 2, 4, 8 (cfg 3) with
1..4 frames in flight (separate contexts and streams): what the multi-GPU step
can reach before the gather."""
import json, os, sys, time
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd')
import torch
import rmarch as rm
W, H, K = 3840, 2160, 24
NS = [int(x) for x in os.environ.get("PROBE_N", "1,2,4,8").split(",")]
NFL = [int(x) for x in os.environ.get("PROBE_NFL", "1,2,3,4").split(",")]
for N in NS:
    for nfl in NFL:
        streams = [torch.cuda.Stream() for _ in range(nfl)]
        kw = dict(row_block=8, shard=0, nshards=N) if N > 1 else {}
        rs = [rm.Renderer(W, H, **kw) for _ in range(nfl)]
        for j, r in enumerate(rs):
            r.set_stream(streams[j].cuda_stream)
        for f in range(6):
            rs[f % nfl].dispatch(rm.sweep_uniforms(f, 120, 3, True, 0))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(K):
            rs[f % nfl].dispatch(rm.sweep_uniforms(6 + f, 120, 3, True, 0))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K * 1e3
        for r in rs:
            r.close()
        print(json.dumps({"N": N, "inflight": nfl, "ms_per_frame": round(dt, 4)}), flush=True)
