"""Render the bench's sweep frames with one kernel variant (driver for rocprofv3 --pmc).

  python tools/prof_kernels.py KIND CFG STEPS [BATCH]
KIND: pixel | table | table-spec.  The frames are bench.py's own
(bench_frames(STEPS): step k renders sweep frame floor(k * 120 / STEPS)), one
launch each, so the per-launch PMC means describe the benched workload.  BATCH >
1: the same frames once more as rm_dispatch_frames batches of BATCH frames
(k_pixel_frames / k_sample_frames, or a table's k_table_*_frames: the kernels
bench.py times for that configuration); tools/summarize_profiles.py divides
their per-launch counters by BATCH.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'opengl-raymarching-in-compute-shader_amd'))
import rmarch as rm  # noqa: E402
from bench import CONFIGS, bench_frames  # noqa: E402

kname = sys.argv[1] if len(sys.argv) > 1 else "pixel"
cfg = CONFIGS[int(sys.argv[2]) if len(sys.argv) > 2 else 3]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 1
k = rm.RM_KERNEL_PIXEL
with rm.Renderer(cfg["width"], cfg["height"], kernel=k) as r:
    if kname == "table-spec":  # the same, with kernels compiled for the table (hiprtc)
        r.specialize_scene(True)
    if kname in ("table", "table-spec"):  # the reference scene as a runtime table (k_table_* kernels)
        r.set_scene(rm.default_scene())
    us = [rm.sweep_uniforms(f, 120, cfg["bounces"], cfg["aa"], cfg["shadow"]) for f in bench_frames(steps)]
    # (a table renders single frames with its batch kernel too, as a batch of
    # one: with BATCH > 1 only the batches run, so the batch kernel's per-launch
    # counters are all launches of BATCH frames)
    if not (kname in ("table", "table-spec") and batch > 1):
        for u in us:
            r.dispatch(u)
    r.synchronize()
    if batch > 1:
        for i in range(0, len(us), batch):
            r.dispatch_frames(us[i:i + batch])
        r.synchronize()
print("done", kname, sys.argv[2:])
