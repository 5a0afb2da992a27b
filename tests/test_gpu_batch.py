"""Frame batches (rm_dispatch_frames, API version 4): n frames in one launch.

A batch must produce, for every frame k, exactly the image that
rm_set_uniforms(frames[k]) + rm_dispatch (glDispatchCompute, main.cpp:123)
produces: the batched kernels (k_pixel_frames / k_sample_frames, grid.z = the
frame) are separate code objects from k_pixel / k_sample, so every test here
compares them byte for byte (RGBA8) and bit for bit (RGBA32F) with the
per-frame kernels, whose parity with the oracle the other suites pin, and the
small-frame test also checks a batch against the oracle directly.  Afterwards
the context must read as after n rm_dispatch calls (its image = the last frame,
its uniforms = the last frame's).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(rm, n, b=3, aa=True, shadow=0):
    return [rm.sweep_uniforms(int(f), 120, b, aa, shadow) for f in np.linspace(0, 119, n).astype(int)]


def _per_frame(rm, W, H, us, outputs=None, **kw):
    outputs = outputs or (rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F)
    with rm.Renderer(W, H, outputs=outputs, **kw) as r:
        out = []
        for u in us:
            r.dispatch(u)
            out.append((r.read_rgba8() if outputs & rm.RM_OUT_RGBA8 else None,
                        r.read_rgba32f() if outputs & rm.RM_OUT_RGBA32F else None))
        return out


def _check_batch(rm, r, us, ref):
    for k, (w8, w32) in enumerate(ref):
        if w8 is not None:
            np.testing.assert_array_equal(r.read_frame_rgba8(k), w8, err_msg=f"frame {k}")
        if w32 is not None:
            np.testing.assert_array_equal(r.read_frame_rgba32f(k).view(np.uint32), w32.view(np.uint32),
                                          err_msg=f"frame {k} (RGBA32F)")
    # the context reads as after len(us) dispatches
    if ref[-1][0] is not None:
        np.testing.assert_array_equal(r.read_rgba8(), ref[-1][0])
    u = r.get_uniforms()
    assert bytes(u) == bytes(us[-1])


@pytest.mark.parametrize("W,H,b,aa,shadow,n", [
    (160, 90, 3, True, 0, 7),     # cfg3-like, supersampled
    (192, 108, 1, False, 0, 12),  # cfg2-like
    (64, 64, 0, False, 1, 32),    # cfg1-like (hard shadows), the largest batch
    (37, 23, 5, True, 0, 3),      # ragged tiles, 5 bounces
    (1, 1, 2, False, 0, 2),
])
def test_batch_equals_per_frame_dispatch(rm, gpu, W, H, b, aa, shadow, n):
    us = _frames(rm, n, b, aa, shadow)
    ref = _per_frame(rm, W, H, us)
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F) as r:
        r.dispatch_frames(us)
        _check_batch(rm, r, us, ref)
        # a second, shorter batch and a plain dispatch reuse the ring
        r.dispatch_frames(us[:2])
        _check_batch(rm, r, us[:2], ref[:2])
        r.dispatch(us[-1])
        np.testing.assert_array_equal(r.read_frame_rgba8(0), ref[-1][0])
        with pytest.raises(rm.RMError):
            r.read_frame_rgba8(1)  # a plain dispatch holds one frame


def test_batch_matches_oracle(rm, gpu, oracle):
    """The batched kernels against the CPU oracle directly (geometry exact, RGBA8 <= 1 LSB)."""
    W, H = 96, 54
    us = _frames(rm, 4, 3, True) + _frames(rm, 3, 1, False)  # two AA runs: two launches
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8) as r:
        r.dispatch_frames(us)
        for k, u in enumerate(us):
            ref = oracle.render(u, W, H)
            d = np.abs(r.read_frame_rgba8(k).astype(np.int16) - ref["rgba8"].astype(np.int16))
            assert d.max() <= 1, (k, int(d.max()))


def test_batch_mixed_uniforms(rm, gpu):
    """Every uniform may change inside a batch (bounces, AA, shadow mode, light)."""
    W, H = 128, 72
    us = [rm.sweep_uniforms(f, 120, f % 6, f % 3 == 0, f % 2) for f in range(0, 120, 7)]
    us[3].light.position[1] = -3.0
    us[5].iTime = 123.0
    ref = _per_frame(rm, W, H, us)
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F) as r:
        r.dispatch_frames(us)
        _check_batch(rm, r, us, ref)


def test_batch_sharded_and_external_output(rm, gpu):
    import torch
    W, H = 160, 90
    us = _frames(rm, 5)
    ref = _per_frame(rm, W, H, us, outputs=rm.RM_OUT_RGBA8, row_block=8, shard=1, nshards=3)
    with rm.Renderer(W, H, row_block=8, shard=1, nshards=3) as r:
        r.dispatch_frames(us)
        _check_batch(rm, r, us, ref)
        out = torch.zeros((r.rows, W, 4), dtype=torch.uint8, device="cuda")
        r.set_output_rgba8(out.data_ptr())
        r.dispatch_frames(us)
        r.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ref[-1][0])  # the last frame lands there
        np.testing.assert_array_equal(r.read_frame_rgba8(1), ref[1][0])


def _tables(rm):
    from test_gpu_scene import floor_last_scene, random_scene
    return {"reference": rm.default_scene(), "floor": floor_last_scene(rm, 3),
            "random": random_scene(rm, 5)}


@pytest.mark.parametrize("spec", [False, True], ids=["generic", "specialised"])
@pytest.mark.parametrize("table", ["reference", "floor", "random"])
@pytest.mark.parametrize("n,aa", [(1, True), (5, True), (32, False), (13, False)])
def test_batch_scene_table(rm, gpu, spec, table, n, aa):
    """a runtime scene table renders a batch in one launch
    (k_table_*_frames, grid.z = the frame; the hiprtc-specialised ones too): every
    frame byte-equal to its own rm_dispatch (RGBA32F bit-equal)."""
    W, H = 96, 54
    sc = _tables(rm)[table]
    us = _frames(rm, n, b=2 if aa else 1, aa=aa)
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F) as one:
        if spec:
            one.specialize_scene(True)
        one.set_scene(sc)
        ref = []
        for u in us:
            one.dispatch(u)
            ref.append((one.read_rgba8(), one.read_rgba32f()))
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F) as r:
        if spec:
            r.specialize_scene(True)
        r.set_scene(sc)
        r.enable_timing(True)
        r.kernel_time_ms(reset=True)
        r.dispatch_frames(us)
        _, launches = r.kernel_time_ms(reset=True)
        assert launches == n  # one timed launch counting its n frames
        _check_batch(rm, r, us, ref)


def test_batch_scene_table_mixed_kernels(rm, gpu):
    """A specialised table's batch whose frames need different kernels (a camera
    beyond 1e15 renders with the generic kernel, rm_api.hip frame_jit) and both AA
    settings: runs of one kernel each, every frame equal to its own dispatch."""
    W, H = 64, 40
    us = _frames(rm, 6)
    far = _frames(rm, 1)[0]
    far.camera.pos[0] = 3e15
    us = us[:2] + [far] + us[2:4] + _frames(rm, 2, b=1, aa=False)
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F) as one:
        one.specialize_scene(True)
        one.set_scene(rm.default_scene())
        ref = []
        for u in us:
            one.dispatch(u)
            ref.append((one.read_rgba8(), one.read_rgba32f()))
        one.dispatch_frames(us)
        _check_batch(rm, one, us, ref)


def test_batch_scene_table_matches_oracle(rm, oracle, gpu):
    """A table batch (generic kernel, reference-shaped and random tables) against the
    oracle's table mode: every frame within 1 LSB."""
    W, H = 64, 40
    for name, sc in _tables(rm).items():
        us = _frames(rm, 3, b=2)
        with rm.Renderer(W, H) as r:
            r.set_scene(sc)
            r.dispatch_frames(us)
            for k, u in enumerate(us):
                ref = oracle.render(u, W, H, scene=sc, want_counts=False)["rgba8"]
                d = np.abs(r.read_frame_rgba8(k).astype(int) - ref.astype(int))
                assert d.max() <= 1, (name, k, d.max())


@pytest.mark.parametrize("form", ["comm_init", "ngpus"])
def test_batch_on_communicator_contexts(rm, gpu, form):
    """One rank (rm_comm_init) / one device (rm_config.ngpus): the batch's shards move
    in one ncclGather on the gather stream and rank 0 assembles every frame; plain
    dispatches and graph replays interleave with batches in order."""
    W, H, R = 160, 90, 8
    us = _frames(rm, 9)
    ref = _per_frame(rm, W, H, us)
    outs = rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F
    if form == "ngpus":
        r = rm.Renderer(W, H, outputs=outs, ngpus=1, row_block=R)
    else:
        r = rm.Renderer(W, H, outputs=outs, row_block=R, shard=0, nshards=1)
        r.comm_init(rm.comm_unique_id(), 1, 0)
    with r:
        for rep in range(3):  # both slots, then the first again
            r.dispatch_frames(us)
            _check_batch(rm, r, us, ref)
        # batches back to back without a read between them (slot reuse ordering)
        r.dispatch_frames(us[:4])
        r.dispatch_frames(us[4:])
        _check_batch(rm, r, us[4:], ref[4:])
        r.dispatch(us[2])
        np.testing.assert_array_equal(r.read_rgba8(), ref[2][0])
        r.dispatch_frames(us[:3])
        r.dispatch(us[7])  # ordered after the batch's gather
        np.testing.assert_array_equal(r.read_rgba8(), ref[7][0])
        r.graph_enable(True)
        r.graph_dispatch(us[5])
        r.graph_dispatch(us[6])
        np.testing.assert_array_equal(r.read_rgba8(), ref[6][0])
        r.dispatch_frames(us[:2])
        _check_batch(rm, r, us[:2], ref[:2])


@pytest.mark.parametrize("form", ["comm_init", "ngpus"])
def test_wait_output_orders_a_caller_stream(rm, gpu, form):
    """on a communicator context a batch's frame n-1 is assembled into
    the caller's output buffer on the context's gather stream.  rm_wait_output
    orders the caller's stream after it: a copy enqueued there afterwards (no host
    sync in between) reads the finished frame."""
    import torch
    W, H = 160, 90
    us = _frames(rm, 6)
    ref = _per_frame(rm, W, H, us, outputs=rm.RM_OUT_RGBA8)
    s = torch.cuda.Stream()
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    if form == "ngpus":
        r = rm.Renderer(W, H, ngpus=1, row_block=8)
    else:
        r = rm.Renderer(W, H, row_block=8, shard=0, nshards=1)
        r.set_stream(s.cuda_stream)
        r.comm_init(rm.comm_unique_id(), 1, 0)
    with r:
        r.set_output_rgba8(out.data_ptr())
        for rep in range(3):
            r.dispatch_frames(us[2 * rep:2 * rep + 2] + us[:3])
            r.wait_output(s.cuda_stream)
            with torch.cuda.stream(s):
                got = out.clone()
            s.synchronize()
            np.testing.assert_array_equal(got.cpu().numpy(), ref[2][0], err_msg=f"rep {rep}")
        r.dispatch(us[5])
        r.wait_output(s.cuda_stream)
        with torch.cuda.stream(s):
            got = out.clone()
        s.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy(), ref[5][0])


def test_stalled_batch_slot_wait_is_bounded(rm, gpu):
    """a batch longer than its slot re-allocates the slot after its
    last gather; on a communicator context that wait is the bounded poll, so a
    stream that does not drain (a spin kernel standing in for a stalled peer) is
    RM_ERR_COMM at the deadline, not a hang; the failed batch leaves the
    uniforms of the last good dispatch."""
    import time
    import torch
    W, H = 64, 48
    us = _frames(rm, 8)
    s = torch.cuda.Stream()
    r = rm.Renderer(W, H, row_block=8, shard=0, nshards=1)
    r.set_stream(s.cuda_stream)
    r.comm_init(rm.comm_unique_id(), 1, 0)
    r.dispatch_frames(us[:2])
    r.synchronize()
    before = bytes(r.get_uniforms())
    r.comm_set_timeout(300)
    with torch.cuda.stream(s):
        torch.cuda._sleep(int(6e9))  # ~2-3 s of spinning on the context's stream
    t0 = time.monotonic()
    with pytest.raises(rm.RMError) as e:
        r.dispatch_frames(us)  # 8 frames: the next slot holds none yet
    assert e.value.code == rm.RM_ERR_COMM and "did not complete within 300 ms" in str(e.value)
    assert time.monotonic() - t0 < 30.0
    assert bytes(r.get_uniforms()) == before
    s.synchronize()
    r.close()


def test_batch_timing_and_phases(rm, gpu):
    W, H = 160, 90
    us = _frames(rm, 6)
    with rm.Renderer(W, H, row_block=8, shard=0, nshards=1) as r:
        r.comm_init(rm.comm_unique_id(), 1, 0)
        r.enable_timing(True)
        r.kernel_time_ms(reset=True)
        r.dispatch_frames(us)
        ms, n = r.kernel_time_ms(reset=True)
        assert n == 6 and ms > 0  # a batch counts its frames
        ph = r.frame_phases()
        assert ph["render_ms"] > 0 and ph["gather_ms"] >= 0 and ph["assemble_ms"] > 0


def test_batch_validation(rm, gpu):
    us = _frames(rm, 2)
    with rm.Renderer(32, 32) as r:
        for bad in ([], us * 17):  # n = 0, n = 34 > RM_MAX_BATCH
            with pytest.raises(rm.RMError) as e:
                if bad:
                    r.dispatch_frames(bad)
                else:
                    import ctypes as C
                    rm._check(rm.lib().rm_dispatch_frames(r.handle, (rm.rm_uniforms * 1)(), 0), r.handle)
            assert e.value.code == rm.RM_ERR_INVALID
        bad = _frames(rm, 2)
        bad[1].bounceVar = 6
        with pytest.raises(rm.RMError) as e:
            r.dispatch_frames(bad)
        assert e.value.code == rm.RM_ERR_INVALID
        with pytest.raises(rm.RMError) as e:
            r.read_frame_rgba8(0)  # nothing dispatched yet
        assert e.value.code == rm.RM_ERR_STATE
        r.dispatch_frames(us)
        for k in (-1, 2):
            with pytest.raises(rm.RMError) as e:
                r.read_frame_rgba8(k)
            assert e.value.code == rm.RM_ERR_INVALID
    with rm.Renderer(32, 32, counters=True) as r:
        with pytest.raises(rm.RMError) as e:
            r.dispatch_frames(us)
        assert e.value.code == rm.RM_ERR_STATE


@pytest.mark.parametrize("cfg", [2, 3])
def test_batch_full_size(rm, gpu, cfg):
    """BASELINE cfg2 / cfg3 at full size: a 20-frame batch of the bench's sweep frames
    equals the per-frame production kernel on every pixel of every frame."""
    W, H, b, aa = {2: (1920, 1080, 1, False), 3: (3840, 2160, 3, True)}[cfg]
    frames = [(k * 120) // 20 for k in range(20)]
    us = [rm.sweep_uniforms(f, 120, b, aa, 0) for f in frames]
    with rm.Renderer(W, H) as r, rm.Renderer(W, H) as one:
        r.dispatch_frames(us)
        r.synchronize()
        for k, u in enumerate(us):
            one.dispatch(u)
            np.testing.assert_array_equal(r.read_frame_rgba8(k), one.read_rgba8(), err_msg=f"frame {frames[k]}")


@pytest.mark.parametrize("N,R,R0,n", [(2, 8, 8, 5), (3, 4, 4, 3), (8, 8, 8, 4), (8, 8, 7, 4), (4, 8, 6, 3)])
@pytest.mark.parametrize("fmt", ["rgba8", "rgb8"])
def test_batch_gather_layout_assembles(rm, gpu, N, R, R0, n, fmt):
    """The N-rank layout of a gathered batch, rehearsed with N virtual ranks on one GPU
    (RCCL refuses two ranks on one device): rank r's n shards rendered by
    rm_dispatch_frames, placed as ncclGather places them on rank 0 ([N][n][rows_cap]
    [width]: each rank's n shards back to back), and every frame k assembled by
    rm_unshard_batch_rgba8 (the k_unshard launch rm_dispatch_frames uses on rank 0,
    rank stride n x rows_cap) equals a full render.  fmt rgb8: the shards are packed
    RGB (rm_config.shard_format, API version 6), as a communicator context gathers
    them: rendered packed, read back expanded, packed again for the gather buffer."""
    import torch
    W, H = 160, 90
    us = _frames(rm, n)
    cap = rm.shard_rows_cap(H, R, N, R0)
    sf = rm.RM_SHARD_RGB8 if fmt == "rgb8" else rm.RM_SHARD_RGBA8
    bpp = 3 if fmt == "rgb8" else 4
    gathered = torch.zeros((N, n, cap, W, bpp), dtype=torch.uint8, device="cuda")
    for r in range(N):
        with rm.Renderer(W, H, row_block=R, shard=r, nshards=N, rank0_rows=R0, shard_format=sf) as s:
            s.dispatch_frames(us)
            for k in range(n):
                gathered[r, k] = torch.from_numpy(s.read_frame_rgba8(k)[..., :bpp].copy()).cuda()
    ref = _per_frame(rm, W, H, us, outputs=rm.RM_OUT_RGBA8)
    with rm.Renderer(W, H, row_block=R, shard=0, nshards=N, rank0_rows=R0, shard_format=sf) as a:
        for k in range(n):
            frame = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            a.unshard_batch_rgba8(gathered.data_ptr(), k, n, frame.data_ptr())
            a.synchronize()
            np.testing.assert_array_equal(frame.cpu().numpy(), ref[k][0], err_msg=f"frame {k}")
        with pytest.raises(rm.RMError):
            a.unshard_batch_rgba8(gathered.data_ptr(), n, n, frame.data_ptr())


def _two_gpus(rm):
    if rm.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")


@pytest.mark.parametrize("R0", [8, 5])
def test_batch_on_two_gpus_ngpus(rm, gpu, R0):
    """a real two-device gather of a batch (rm_config.ngpus = 2, one
    process): every frame of the batch on device 0 equals its one-GPU render."""
    _two_gpus(rm)
    W, H = 160, 90
    us = _frames(rm, 5)
    ref = _per_frame(rm, W, H, us)
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F, ngpus=2, row_block=8,
                     rank0_rows=R0) as r:
        for rep in range(2):
            r.dispatch_frames(us)
            _check_batch(rm, r, us, ref)


def test_batch_on_two_ranks_comm_init(rm, gpu):
    """two rm_comm_init ranks on two devices (one thread each, the
    calls are collective): rank 0 reads every assembled frame of the batch, rank 1
    (the non-root branch of batch_finish and read_frame) its shard of every frame."""
    import threading
    _two_gpus(rm)
    W, H, R, R0 = 160, 90, 8, 6
    us = _frames(rm, 4)
    ref = _per_frame(rm, W, H, us, outputs=rm.RM_OUT_RGBA8)
    cid = rm.comm_unique_id()
    got, errs = {}, []

    def rank(r):
        try:
            with rm.Renderer(W, H, row_block=R, shard=r, nshards=2, rank0_rows=R0, device=r) as c:
                c.comm_init(cid, 2, r)
                for rep in range(2):
                    c.dispatch_frames(us)
                    got[(r, rep)] = [c.read_frame_rgba8(k) for k in range(len(us))]
                    got[(r, rep, "last")] = c.read_rgba8()
        except Exception as e:  # reported by the main thread
            errs.append(e)

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    rows1 = rm.shard_global_rows(H, R, 1, 2, R0)
    real1 = rows1[rows1 >= 0]
    for rep in range(2):
        for k in range(len(us)):
            np.testing.assert_array_equal(got[(0, rep)][k], ref[k][0], err_msg=f"rank 0 frame {k}")
            np.testing.assert_array_equal(got[(1, rep)][k][: len(real1)], ref[k][0][real1],
                                          err_msg=f"rank 1 shard of frame {k}")
        np.testing.assert_array_equal(got[(0, rep, "last")], ref[-1][0])
        np.testing.assert_array_equal(got[(1, rep, "last")][: len(real1)], ref[-1][0][real1])
