"""Per-shard render time of cfg 3 at N = 2, 4, 8 (row-block sharding), one GPU:
the render part of the multi-GPU step, shard by shard (no gather)."""
import json, sys
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd')
import rmarch as rm
W, H = 3840, 2160
for N in (1, 2, 4, 8):
    times = []
    for s in range(N):
        with rm.Renderer(W, H, row_block=8 if N > 1 else 0, shard=s, nshards=N) as r:
            r.enable_timing(True)
            for f in range(3): r.dispatch(rm.sweep_uniforms(f, 120, 3, True, 0))
            r.kernel_time_ms(reset=True)
            for f in range(10): r.dispatch(rm.sweep_uniforms(f, 120, 3, True, 0))
            ms, n = r.kernel_time_ms(reset=True)
            times.append(ms / n)
    print(json.dumps({"N": N, "max_ms": round(max(times), 4), "mean_ms": round(sum(times) / N, 4),
                      "ideal_ms": round(times[0] if N == 1 else 0, 4), "shards": [round(t, 3) for t in times]}),
          flush=True)
