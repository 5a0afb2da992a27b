"""Multi-GPU frames behind the C-ABI: RCCL inside librm.

Two forms, both replacing one reference dispatch (main.cpp:123-125) per frame:
  * rm_config.ngpus: one process drives N devices (ncclCommInitAll), the frame is
    assembled on the first;
  * rm_comm_init: one rank per process (ncclCommInitRank), rank 0 assembles.
This box has one GPU, so both run with a one-rank communicator: the render,
the ncclGather (in place on rank 0), the k_unshard assembly and the captured
hipGraph of all three run for real; only the number of peers is 1.  The
N-rank shard geometry is covered by tests/test_gpu_api.py (shard assembly on
one GPU, N in {2, 3, 8}) and tests/test_shard.py (gloo, world size 2).
Every frame must equal a plain one-GPU render byte for byte.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _frames(rm, n, b=3, aa=True):
    return [rm.sweep_uniforms(f, 120, b, aa, rm.RM_SHADOW_SOFT) for f in np.linspace(0, 119, n).astype(int)]


def _reference(rm, W, H, us):
    with rm.Renderer(W, H) as r:
        out = []
        for u in us:
            r.dispatch(u)
            out.append(r.read_rgba8())
        return out


@pytest.mark.parametrize("W,H,R", [(160, 90, 8), (37, 23, 4), (640, 360, 8)])
def test_multi_gpu_context_one_device(rm, gpu, W, H, R):
    us = _frames(rm, 4)
    ref = _reference(rm, W, H, us)
    with rm.Renderer(W, H, ngpus=1, row_block=R) as m:
        assert m.comm_info() == (0, 1, 1)
        for u, want in zip(us, ref):
            m.dispatch(u)
            np.testing.assert_array_equal(m.read_rgba8(), want)
        # readback flip and graph replay work as on a one-GPU context
        np.testing.assert_array_equal(m.read_rgba8(flip_y=True), ref[-1][::-1])
        m.graph_enable(True)
        for u, want in zip(us, ref):
            m.graph_dispatch(u)
            np.testing.assert_array_equal(m.read_rgba8(), want)


def test_multi_gpu_context_explicit_device_list(rm, gpu):
    us = _frames(rm, 2, b=1, aa=False)
    ref = _reference(rm, 96, 64, us)
    with rm.Renderer(96, 64, devices=[0]) as m:
        for u, want in zip(us, ref):
            m.dispatch(u)
            np.testing.assert_array_equal(m.read_rgba8(), want)
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(96, 64, devices=[0, 0])
    assert e.value.code == rm.RM_ERR_INVALID
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(96, 64, devices=[gpu])  # out of range
    assert e.value.code == rm.RM_ERR_INVALID


def test_multi_gpu_context_scene_table_and_external_output(rm, gpu):
    import torch
    W, H = 128, 72
    u = _frames(rm, 1)[0]
    ref = _reference(rm, W, H, [u])[0]
    with rm.Renderer(W, H, ngpus=1) as m:
        m.set_scene(rm.default_scene())  # the reference scene as a table: same image
        assert len(m.get_scene()) == 6
        m.dispatch(u)
        np.testing.assert_array_equal(m.read_rgba8(), ref)
        m.set_scene(None)
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        m.set_output_rgba8(out.data_ptr())
        assert m.output_rgba8_ptr() == out.data_ptr()
        m.dispatch(u)
        m.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
        with pytest.raises(rm.RMError):
            m.set_stream(None)  # one stream per device, the context's own


@pytest.mark.parametrize("W,H,R", [(160, 90, 8), (65, 3, 1)])
def test_comm_rank_renders_gathers_and_assembles(rm, gpu, W, H, R):
    us = _frames(rm, 4)
    ref = _reference(rm, W, H, us)
    with rm.Renderer(W, H, row_block=R, shard=0, nshards=1) as r:
        r.comm_init(rm.comm_unique_id(), 1, 0)
        assert r.comm_info() == (0, 1, 1)
        for u, want in zip(us, ref):
            r.dispatch(u)
            np.testing.assert_array_equal(r.read_rgba8(), want)


def test_comm_graph_captures_render_gather_and_assembly(rm, gpu):
    """cfg 5's per-rank graph: render + ncclGather + k_unshard captured once and
    replayed with new frame constants; a new output buffer re-captures."""
    import torch
    W, H = 192, 108
    us = _frames(rm, 6)
    ref = _reference(rm, W, H, us)
    with rm.Renderer(W, H, row_block=8, shard=0, nshards=1) as r:
        r.comm_init(rm.comm_unique_id(), 1, 0)
        r.graph_enable(True)
        for u, want in zip(us[:3], ref[:3]):  # the first runs eagerly (RCCL set-up), then replays
            r.graph_dispatch(u)
            np.testing.assert_array_equal(r.read_rgba8(), want)
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        r.set_output_rgba8(out.data_ptr())
        for u, want in zip(us[3:], ref[3:]):
            r.graph_dispatch(u)
            r.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_comm_init_validation(rm, gpu):
    cid = rm.comm_unique_id()
    with rm.Renderer(32, 32, counters=True) as r:
        with pytest.raises(rm.RMError) as e:  # no counters on gathered frames
            r.comm_init(cid, 1, 0)
        assert e.value.code == rm.RM_ERR_INVALID
    with rm.Renderer(32, 32, row_block=8, shard=1, nshards=2) as r:
        with pytest.raises(rm.RMError) as e:  # the shard must be the rank
            r.comm_init(cid, 2, 0)
        assert e.value.code == rm.RM_ERR_INVALID
    with rm.Renderer(32, 32) as r:
        r.comm_check()  # no communicator: healthy
        with pytest.raises(rm.RMError) as e:
            r.comm_set_timeout(-1)
        assert e.value.code == rm.RM_ERR_INVALID
        r.comm_init(cid, 1, 0)
        r.comm_check()
        with pytest.raises(rm.RMError) as e:
            r.comm_init(cid, 1, 0)
        assert e.value.code == rm.RM_ERR_STATE


def test_frameloop_on_a_multi_gpu_context(rm, gpu, tmp_path):
    """The C++ host (rm_frameloop, the main.cpp:92-147 replacement) renders with
    --gpus 1 (rm_config.ngpus, RCCL in librm, no torch) and with its graph, and
    dumps the same last frame as a plain run."""
    exe = os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd", "rm_frameloop")
    base = [exe, "--width", "160", "--height", "96", "--frames", "5", "--bounces", "2"]
    outs = {}
    for name, extra in (("plain", []), ("gpus", ["--gpus", "1"]), ("graph", ["--gpus", "1", "--graph"])):
        ppm = tmp_path / f"{name}.ppm"
        p = subprocess.run(base + extra + ["--dump", str(ppm)], capture_output=True, text=True, timeout=60)
        assert p.returncode == 0, p.stderr
        outs[name] = ppm.read_bytes()
    assert outs["gpus"] == outs["plain"] and outs["graph"] == outs["plain"]


def _reference32(rm, W, H, us):
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F) as r:
        out = []
        for u in us:
            r.dispatch(u)
            out.append((r.read_rgba8(), r.read_rgba32f()))
        return out


@pytest.mark.parametrize("form", ["comm_init", "ngpus", "comm_init-graph"])
def test_gathered_rgba32f_equals_one_gpu_render(rm, gpu, form):
    """the reference texture's true storage (RGBA32F, texture.cpp:19)
    on RCCL-gathered frames: 16 B/px shards gathered as ncclFloat32 and assembled by
    k_unshard (a row of 4 x width words); bit-identical to a one-GPU render."""
    W, H, R = 160, 90, 8
    us = _frames(rm, 3)
    ref = _reference32(rm, W, H, us)
    outs = rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F
    if form == "ngpus":
        r = rm.Renderer(W, H, outputs=outs, ngpus=1, row_block=R)
    else:
        r = rm.Renderer(W, H, outputs=outs, row_block=R, shard=0, nshards=1)
        r.comm_init(rm.comm_unique_id(), 1, 0)
    with r:
        if form.endswith("graph"):
            r.graph_enable(True)
        for u, (want8, want32) in zip(us, ref):
            (r.graph_dispatch if form.endswith("graph") else r.dispatch)(u)
            np.testing.assert_array_equal(r.read_rgba8(), want8)
            np.testing.assert_array_equal(r.read_rgba32f().view(np.uint32), want32.view(np.uint32))
    # RGBA32F alone (no RGBA8) gathers too
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA32F, row_block=R, shard=0, nshards=1) as r:
        r.comm_init(rm.comm_unique_id(), 1, 0)
        r.dispatch(us[0])
        np.testing.assert_array_equal(r.read_rgba32f().view(np.uint32), ref[0][1].view(np.uint32))


def test_output_set_before_comm_init_is_dropped_on_rank0(rm, gpu):
    """a caller RGBA8 buffer set before rm_comm_init is shard-sized;
    rank 0's image becomes the full frame, so the buffer is dropped (no
    out-of-bounds assembly into it) and the output pointer is re-queried."""
    import torch
    W, H = 96, 64
    u = _frames(rm, 1)[0]
    want = _reference(rm, W, H, [u])[0]
    with rm.Renderer(W, H, row_block=8, shard=0, nshards=1) as r:
        small = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        r.set_output_rgba8(small.data_ptr())
        r.comm_init(rm.comm_unique_id(), 1, 0)
        p = r.output_rgba8_ptr()
        assert p and p != small.data_ptr()
        r.dispatch(u)
        np.testing.assert_array_equal(r.read_rgba8(), want)
        r.synchronize()
        assert int(small.sum().item()) == 0  # never written
        big = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        r.set_output_rgba8(big.data_ptr())  # set after rm_comm_init: the frame's destination
        r.dispatch(u)
        r.synchronize()
        np.testing.assert_array_equal(big.cpu().numpy(), want)


def test_comm_init_never_joined_rank_times_out(rm, gpu):
    """rm_comm_init of rank 0 of 2 whose peer never joins returns
    RM_ERR_COMM within the deadline (non-blocking init, ncclCommAbort), and the
    process stays usable: the same context joins a one-rank communicator and
    renders, and a fresh context renders."""
    import time
    W, H = 64, 48
    u = _frames(rm, 1)[0]
    want = _reference(rm, W, H, [u])[0]
    with rm.Renderer(W, H, row_block=8, shard=0, nshards=2) as r:
        r.comm_set_timeout(3000)
        t0 = time.monotonic()
        with pytest.raises(rm.RMError) as e:
            r.comm_init(rm.comm_unique_id(), 2, 0)
        dt = time.monotonic() - t0
        assert e.value.code == rm.RM_ERR_COMM, e.value
        assert "never joined" in str(e.value)
        assert 2.5 < dt < 30.0, dt
        assert r.comm_info() == (0, 1, 1)  # no communicator attached
    with rm.Renderer(W, H, row_block=8, shard=0, nshards=1) as r:
        r.comm_init(rm.comm_unique_id(), 1, 0)
        r.comm_check()
        r.dispatch(u)
        np.testing.assert_array_equal(r.read_rgba8(), want)


def test_stalled_frame_hits_the_deadline_and_aborts(rm, gpu):
    """The bounded wait of rm_synchronize on a communicator context: a stream that
    does not drain within the deadline (here a spin kernel queued behind the
    gathered frame stands in for a peer that never sends) aborts the
    communicator and returns RM_ERR_COMM; later calls report it; the context is
    destroyed cleanly once the stream drains."""
    import time
    import torch
    W, H = 64, 48
    u = _frames(rm, 1)[0]
    want = _reference(rm, W, H, [u])[0]
    s = torch.cuda.Stream()
    r = rm.Renderer(W, H, row_block=8, shard=0, nshards=1)
    r.set_stream(s.cuda_stream)
    r.comm_init(rm.comm_unique_id(), 1, 0)
    r.dispatch(u)
    np.testing.assert_array_equal(r.read_rgba8(), want)
    r.comm_set_timeout(300)
    with torch.cuda.stream(s):
        torch.cuda._sleep(int(6e9))  # ~2-3 s of spinning on the context's stream
    t0 = time.monotonic()
    with pytest.raises(rm.RMError) as e:
        r.synchronize()
    assert e.value.code == rm.RM_ERR_COMM and "did not complete within 300 ms" in str(e.value)
    # the deadline fires at 300 ms; ncclCommAbort then waits for the device work
    # already queued to quiesce (here the spin kernel, ~2-3 s), so no hang, no more
    assert time.monotonic() - t0 < 30.0
    with pytest.raises(rm.RMError) as e:
        r.dispatch(u)
    assert e.value.code == rm.RM_ERR_COMM and "aborted" in str(e.value)
    with pytest.raises(rm.RMError) as e:
        r.comm_check()
    assert e.value.code == rm.RM_ERR_COMM
    s.synchronize()
    r.close()
    with rm.Renderer(W, H) as q:  # the process and the device stay usable
        q.dispatch(u)
        np.testing.assert_array_equal(q.read_rgba8(), want)


def test_frame_phases_split_render_gather_assembly(rm, gpu):
    """The per-phase times bench.py's N > 1 line reports (render, gather,
    assembly), from HIP events on the context's stream."""
    W, H = 640, 360
    u = _frames(rm, 1)[0]
    with rm.Renderer(W, H, row_block=8, shard=0, nshards=1) as r:
        r.comm_init(rm.comm_unique_id(), 1, 0)
        with pytest.raises(rm.RMError):
            r.frame_phases()  # no timed dispatch yet
        r.enable_timing(True)
        r.dispatch(u)
        ph = r.frame_phases()
        assert ph["render_ms"] > 0 and ph["gather_ms"] >= 0 and ph["assemble_ms"] > 0, ph
    with rm.Renderer(W, H) as r:
        r.enable_timing(True)
        r.dispatch(u)
        ph = r.frame_phases()
        assert ph["render_ms"] > 0 and ph["gather_ms"] == 0 and ph["assemble_ms"] == 0


@pytest.mark.parametrize("N", [2, 3, 8])
def test_rgba32f_assembly_geometry_at_n_shards(rm, gpu, N):
    """The RGBA32F frame of an N-rank gather is assembled by k_unshard as an
    image of 4 x width 32-bit words (rm_api.hip comm_assemble).  With one GPU the
    N-rank geometry is rehearsed directly: N sharded contexts render RGBA32F
    shards, the shards are laid out as ncclGather leaves them on rank 0
    ([N][rows_cap][W] float4), and the same unshard over a 4W-wide context
    reassembles them; the frame equals a one-GPU RGBA32F render bit for bit."""
    import torch
    W, H, R = 160, 90, 8
    u = _frames(rm, 1)[0]
    cap = rm.shard_rows_cap(H, R, N)
    shards = []
    for k in range(N):
        with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA32F, row_block=R, shard=k, nshards=N) as r:
            r.dispatch(u)
            shards.append(r.read_rgba32f())
    gathered = torch.from_numpy(np.stack(shards)).cuda().contiguous()  # [N][cap][W][4]
    frame = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()  # torch's stream is not ordered with the context's
    with rm.Renderer(4 * W, H, row_block=R, shard=0, nshards=N) as asm:
        asm.unshard_rgba8(gathered.data_ptr(), frame.data_ptr())
        asm.synchronize()
    want = _reference32(rm, W, H, [u])[0][1]
    assert gathered.shape[1] == cap
    np.testing.assert_array_equal(frame.cpu().numpy().view(np.uint32), want.view(np.uint32))
