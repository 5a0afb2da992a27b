"""The multi-GPU step of bench.py, rehearsed on one GPU: N virtual ranks render
their row-block shards of consecutive frames with several frames in flight
(one context and stream per in-flight frame), a `comm` stream gathers the
shards (device copies standing in for the RCCL gather) and assembles each frame
(rm_unshard_rgba8), all ordered only by events.  Every assembled frame must
equal a plain full-frame render."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,nfl", [(2, 2), (4, 3), (8, 4)])
def test_inflight_sharded_frames_assemble(rm, gpu, N, nfl):
    import torch
    W, H, R, F = 160, 90, 8, 7
    us = [rm.sweep_uniforms(9 * f, 120, 3, True, 0) for f in range(F)]
    cap = rm.shard_rows_cap(H, R, N)
    streams = [[torch.cuda.Stream() for _ in range(nfl)] for _ in range(N)]
    rs = [[rm.Renderer(W, H, row_block=R, shard=k, nshards=N) for _ in range(nfl)]
          for k in range(N)]
    outs = [[torch.zeros((cap, W, 4), dtype=torch.uint8, device="cuda") for _ in range(nfl)]
            for _ in range(N)]
    for k in range(N):
        for j in range(nfl):
            rs[k][j].set_stream(streams[k][j].cuda_stream)
            rs[k][j].set_output_rgba8(outs[k][j].data_ptr())
    comm = torch.cuda.Stream()
    ru = rm.Renderer(W, H, row_block=R, shard=0, nshards=N)
    ru.set_stream(comm.cuda_stream)
    gathered = torch.zeros((N, cap, W, 4), dtype=torch.uint8, device="cuda")
    frames = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(F)]
    render_done = [[torch.cuda.Event() for _ in range(nfl)] for _ in range(N)]
    gather_done = [torch.cuda.Event() for _ in range(nfl)]
    for ev in gather_done:
        ev.record(comm)
    for f in range(F):
        j = f % nfl
        for k in range(N):
            streams[k][j].wait_event(gather_done[j])
            rs[k][j].dispatch(us[f])
            render_done[k][j].record(streams[k][j])
        with torch.cuda.stream(comm):
            for k in range(N):
                comm.wait_event(render_done[k][j])
                gathered[k].copy_(outs[k][j])
            ru.unshard_rgba8(gathered.data_ptr(), frames[f].data_ptr())
            gather_done[j].record(comm)
    torch.cuda.synchronize()
    with rm.Renderer(W, H) as full:
        for f in range(F):
            full.dispatch(us[f])
            np.testing.assert_array_equal(frames[f].cpu().numpy(), full.read_rgba8(), err_msg=f"frame {f}")
    for row in rs:
        for r in row:
            r.close()
    ru.close()
