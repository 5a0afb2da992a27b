"""Diagnostic: where the fixed overhead of a short bench run goes.  Renders K sweep
frames of cfg3 with 3 frames in flight, as bench.py does, on torch streams handed to
librm (rm_set_stream), and records a torch event after every frame: prints the
completion time of each frame relative to the start of the timed region.

  python tools/probe_ramp.py [K] [inflight] [idle_ms]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import rmarch as rm  # noqa: E402
from bench import CONFIGS, bench_frames  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
nfl = int(sys.argv[2]) if len(sys.argv) > 2 else 3
idle = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
cfg = CONFIGS[3]
W, H = cfg["width"], cfg["height"]
streams = [torch.cuda.Stream() for _ in range(nfl)]
rs = [rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8) for _ in range(nfl)]
for r, s in zip(rs, streams):
    r.set_stream(s.cuda_stream)
us = {f: rm.sweep_uniforms(f, 120, cfg["bounces"], cfg["aa"], cfg["shadow"]) for f in range(120)}
frames = bench_frames(K)
for k in range(5):
    rs[k % nfl].dispatch(us[frames[k % K]])
torch.cuda.synchronize()
if idle:
    time.sleep(idle / 1e3)
start = torch.cuda.Event(enable_timing=True)
evs = []
with torch.cuda.stream(streams[0]):
    start.record()
for s in streams[1:]:
    s.wait_event(start)
t0 = time.perf_counter()
for k, f in enumerate(frames):
    j = k % nfl
    rs[j].dispatch(us[f])
    e = torch.cuda.Event(enable_timing=True)
    e.record(streams[j])
    evs.append(e)
torch.cuda.synchronize()
t1 = time.perf_counter()
ends = [start.elapsed_time(e) for e in evs]
print(f"K {K} inflight {nfl} idle {idle} ms: wall {1e3 * (t1 - t0):.3f} ms = {1e3 * (t1 - t0) / K:.4f} ms/frame; "
      f"last event {max(ends):.3f} ms")
print("frame ends (ms):", " ".join(f"{x:.2f}" for x in ends))
for r in rs:
    r.close()
