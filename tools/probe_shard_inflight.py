"""Render-only throughput of rank 0's shard at N = 1, 2, 4, 8 (cfg 3) with
1..4 contexts in flight (separate contexts and streams) and B frames per launch
(rm_dispatch_frames): what the multi-GPU step can reach before the gather.

  PROBE_N=1,2,4,8 PROBE_NFL=1,2,3,4 PROBE_BATCH=1,4,8 python tools/probe_shard_inflight.py
"""
import json, os, sys, time
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd')
import torch
import rmarch as rm
W, H, K = 3840, 2160, 24
NS = [int(x) for x in os.environ.get("PROBE_N", "1,2,4,8").split(",")]
NFL = [int(x) for x in os.environ.get("PROBE_NFL", "1,2,3,4").split(",")]
BS = [int(x) for x in os.environ.get("PROBE_BATCH", "1").split(",")]
for N in NS:
    for nfl in NFL:
        for B in BS:
            streams = [torch.cuda.Stream() for _ in range(nfl)]
            kw = dict(row_block=8, shard=0, nshards=N) if N > 1 else {}
            rs = [rm.Renderer(W, H, **kw) for _ in range(nfl)]
            for j, r in enumerate(rs):
                r.set_stream(streams[j].cuda_stream)
            us = [rm.sweep_uniforms(6 + f, 120, 3, True, 0) for f in range(K)]

            def run():
                if B == 1:
                    for f in range(K):
                        rs[f % nfl].dispatch(us[f])
                else:
                    for j, i in enumerate(range(0, K, B)):
                        rs[j % nfl].dispatch_frames(us[i:i + B])
                torch.cuda.synchronize()
            run()  # warm: buffers, rings
            t0 = time.perf_counter()
            run()
            dt = (time.perf_counter() - t0) / K * 1e3
            for r in rs:
                r.close()
            print(json.dumps({"N": N, "inflight": nfl, "batch": B, "ms_per_frame": round(dt, 4)}), flush=True)
