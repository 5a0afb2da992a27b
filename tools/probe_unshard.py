"""Diagnostic: k_unshard time per frame at N = 2, 4, 8 (row blocks of 8, plain and
weighted interleave) for the BASELINE frame sizes, HIP events on the assembling
context's stream.  RM_LIBRM selects the library.  The per-config assembly ratio of
bench.py (ASSEMBLE_RATIO) is this time over one GPU's frame time.
PROBE_FMT=rgb8 (default) / rgba8: the shards' format (rm_config.shard_format; a
communicator context gathers RGB8, 3 B per pixel)."""
import os
import sys

sys.path.insert(0, "opengl-raymarching-in-compute-shader_amd")
import torch  # noqa: E402
import rmarch as rm  # noqa: E402

R, K = 8, 50
FMT = os.environ.get("PROBE_FMT", "rgb8")
BPP = 3 if FMT == "rgb8" else 4
SF = rm.RM_SHARD_RGB8 if FMT == "rgb8" else rm.RM_SHARD_RGBA8
s = torch.cuda.Stream()
for W, H in ((512, 512), (1920, 1080), (3840, 2160), (7680, 4320)):
    for N, R0 in ((2, 8), (4, 8), (8, 8), (8, 7), (8, 5)):
        cap = rm.shard_rows_cap(H, R, N, R0)
        g = torch.randint(0, 255, (N, cap, W, BPP), dtype=torch.uint8, device="cuda")
        fr = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        with rm.Renderer(W, H, row_block=R, shard=0, nshards=N, rank0_rows=R0, shard_format=SF) as r:
            r.set_stream(s.cuda_stream)
            for _ in range(5):
                r.unshard_rgba8(g.data_ptr(), fr.data_ptr())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(K):
                r.unshard_rgba8(g.data_ptr(), fr.data_ptr())
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / K * 1000
            print(f"{W}x{H} N={N} R0={R0} {FMT} unshard {us:.1f} us/frame  "
                  f"({H * W * (BPP + 4) / us / 1e3:.0f} GB/s)", flush=True)
