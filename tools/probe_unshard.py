"""Diagnostic: k_unshard time for a 3840x2160 frame at N = 2, 4, 8 (row blocks of 8),
HIP events on the assembling context's stream.  RM_LIBRM selects the library."""
import sys

sys.path.insert(0, "opengl-raymarching-in-compute-shader_amd")
import torch  # noqa: E402
import rmarch as rm  # noqa: E402

W, H, R, K = 3840, 2160, 8, 50
s = torch.cuda.Stream()
for N in (2, 4, 8):
    cap = rm.shard_rows_cap(H, R, N)
    g = torch.randint(0, 255, (N, cap, W, 4), dtype=torch.uint8, device="cuda")
    fr = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    with rm.Renderer(W, H, row_block=R, shard=0, nshards=N) as r:
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
        print(f"N={N} unshard {us:.1f} us/frame  ({2 * H * W * 4 / us / 1e3:.0f} GB/s)")
