"""bench.py's N > 1 step with frames in flight, through the product path.

Each in-flight frame has its own context, stream and RCCL communicator
(rm_comm_init); rm_dispatch renders the shard, gathers it to rank 0 (ncclGather)
and assembles the frame (k_unshard), all inside librm on the context's stream, and
consecutive frames overlap on the contexts' streams exactly as in bench.py.  This
box has one GPU, so the communicators have one rank (RCCL refuses two ranks on one
device); the N-rank row-block geometry of the assembly is covered by
tests/test_gpu_api.py (N in {2, 3, 8}) and tests/test_shard.py (gloo, world size 2).
Every assembled frame must equal a plain one-GPU render byte for byte.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nfl,graph", [(2, False), (4, False), (4, True)])
def test_inflight_comm_contexts_assemble(rm, gpu, nfl, graph):
    W, H, R, F = 160, 90, 8, 9
    us = [rm.sweep_uniforms(13 * f, 120, 3, True, 0) for f in range(F)]
    rs = [rm.Renderer(W, H, row_block=R, shard=0, nshards=1) for _ in range(nfl)]
    for r in rs:
        r.comm_init(rm.comm_unique_id(), 1, 0)
        if graph:
            r.graph_enable(True)
    got = {}
    for f in range(F):
        r = rs[f % nfl]
        if f >= nfl:  # the context's previous frame is complete before its buffers are reused
            got[f - nfl] = r.read_rgba8()
        (r.graph_dispatch if graph else r.dispatch)(us[f])
    for f in range(F - nfl, F):
        got[f] = rs[f % nfl].read_rgba8()
    with rm.Renderer(W, H) as full:
        for f in range(F):
            full.dispatch(us[f])
            np.testing.assert_array_equal(got[f], full.read_rgba8(), err_msg=f"frame {f}")
    for r in rs:
        r.close()
