"""Rank balance of the weighted interleave, on one MI355X.

For each N and rank-0 rows per round R0, every shard s of the frame is rendered as
its rank would render it in bench.py's N > 1 step (--comms 0: 4 contexts in flight,
one frame per context in turn):
  * s = 0: render into slot 0 of a gather buffer, then assemble the frame from it
    (k_unshard, rm_unshard_rgba8) on the same stream: rank 0's render + assembly;
  * s >= 1: render only.
The gather itself is not included (one GPU).  Prints one JSON line per (config, N,
R0): ms per frame of every shard, rank 0's total and the largest other shard.

  PROBE_CFG=3 PROBE_N=8 PROBE_R0=8,7,6 python tools/probe_shard_weighted.py
"""
import json
import os
import sys
import time

sys.path.insert(0, "opengl-raymarching-in-compute-shader_amd")
import torch  # noqa: E402
import rmarch as rm  # noqa: E402

CFGS = {2: (1920, 1080, 1, False), 3: (3840, 2160, 3, True), 5: (7680, 4320, 3, True)}
CF = [int(x) for x in os.environ.get("PROBE_CFG", "3").split(",")]
NS = [int(x) for x in os.environ.get("PROBE_N", "8").split(",")]
R0S = [int(x) for x in os.environ.get("PROBE_R0", "8,7,6").split(",")]
R, NFL = 8, int(os.environ.get("PROBE_NFL", "4"))
REPS = int(os.environ.get("PROBE_REPS", "3"))

for cfg in CF:
    W, H, B, AA = CFGS[cfg]
    K = 24 if cfg != 5 else 12
    us = [rm.sweep_uniforms(6 + 4 * f, 120, B, AA, 0) for f in range(K)]
    for N in NS:
        for R0 in R0S:
            cap = rm.shard_rows_cap(H, R, N, R0)
            per = []
            for s in range(N):
                rs = [rm.Renderer(W, H, row_block=R, shard=s, nshards=N, rank0_rows=R0) for _ in range(NFL)]
                gbuf = frame = None
                if s == 0:
                    gbuf = [torch.zeros((N, cap, W, 4), dtype=torch.uint8, device="cuda") for _ in range(NFL)]
                    frame = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(NFL)]
                    for j, r in enumerate(rs):
                        r.set_output_rgba8(gbuf[j][0].data_ptr())

                def run():
                    for f in range(K):
                        j = f % NFL
                        rs[j].dispatch(us[f])
                        if s == 0:
                            rs[j].unshard_rgba8(gbuf[j].data_ptr(), frame[j].data_ptr())
                    for r in rs:
                        r.synchronize()
                    torch.cuda.synchronize()

                run()  # warm
                best = None
                for _ in range(REPS):
                    t0 = time.perf_counter()
                    run()
                    dt = (time.perf_counter() - t0) / K * 1e3
                    best = dt if best is None else min(best, dt)
                per.append(round(best, 4))
                for r in rs:
                    r.close()
            rows = [rm.shard_rows(H, R, N, s, R0)[0] for s in range(N)]
            print(json.dumps({"cfg": cfg, "N": N, "rank0_rows": R0, "rows_per_shard": rows,
                              "ms_per_frame": per, "rank0_render_plus_assemble": per[0],
                              "max_other": max(per[1:]) if N > 1 else None,
                              "balanced": per[0] <= max(per[1:]) if N > 1 else None,
                              "inflight": NFL}), flush=True)
