"""Strong-scaling projection of the sharded frame on ONE MI355X.

Every shard s of an N-rank cfg3 frame is rendered exactly as its rank renders it in
bench.py's N > 1 step, and N = 1 (the whole frame) is rendered with the SAME frames
and the SAME issue method, so T1 / max-rank is a like-for-like projection:

  mode "frames": NFL contexts, one frame per rm_dispatch, contexts in turn
                 (bench --comms 0; N = 1: the same on the whole frame);
  mode "bB"    : NFL contexts, B frames per rm_dispatch_frames, contexts in turn
                 (bench --comms 1 uses one context; N = 1 with B = 2 on 4 contexts is
                 the one-GPU headline).
Rank 0 (s = 0) also assembles every frame from an [N][B][rows_cap][W] gather buffer
(rm_unshard_rgba8 / rm_unshard_batch_rgba8) on its render stream, as it does after
the gather.  The gather itself is not included (one GPU).

Frames: bench.py's timed frames for --steps K (sweep frame floor(k*120/K)).  Per run:
  steady_ms : REPS x K frames back to back, ms per frame (best of TRIES);
  k_ms      : exactly K frames from an idle GPU to drained streams (the driver's
              timed region: fill and drain included), best of TRIES;
  issue_ms  : host time to issue one frame (no waiting).

  PROBE_N=1,2,4,8 PROBE_MODES=frames,b2,b4,b8 PROBE_NFL=4 python tools/probe_scale.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd"))
import torch  # noqa: E402
import rmarch as rm  # noqa: E402

CFGS = {2: (1920, 1080, 1, False, rm.RM_SHADOW_SOFT), 3: (3840, 2160, 3, True, rm.RM_SHADOW_SOFT),
        4: (3840, 2160, 5, True, rm.RM_SHADOW_SOFT), 5: (7680, 4320, 3, True, rm.RM_SHADOW_SOFT)}
CFG = int(os.environ.get("PROBE_CFG", "3"))
NS = [int(x) for x in os.environ.get("PROBE_N", "1,2,4,8").split(",")]
MODES = os.environ.get("PROBE_MODES", "frames,b2,b4,b8").split(",")
NFLS = [int(x) for x in os.environ.get("PROBE_NFL", "4").split(",")]
K = int(os.environ.get("PROBE_K", "20"))
REPS = int(os.environ.get("PROBE_REPS", "4"))
TRIES = int(os.environ.get("PROBE_TRIES", "3"))
R = int(os.environ.get("PROBE_ROW_BLOCK", "8"))
R0 = os.environ.get("PROBE_R0", "auto")  # rank 0 rows per round: auto (bench's), or an int
SHARDS = os.environ.get("PROBE_SHARDS", "all")  # all, or a list
# the contexts' streams: "hip" = non-blocking streams made here as librm makes its own
# (hipStreamCreateWithFlags), so completion events can be recorded on them; "torch" =
# torch.cuda.Stream(); "own" = librm's own streams (no completion profile)
STREAMS = os.environ.get("PROBE_STREAMS", "hip")
# the shards' RGBA8 format: rgb8 (3 B per pixel, what a communicator context gathers,
# rm_config.shard_format AUTO) or rgba8
FMT = os.environ.get("PROBE_FMT", "rgb8")

W, H, B3, AA, SH = CFGS[CFG]
ASSEMBLE_RATIO = {2: 0.082, 3: 0.0132, 4: 0.0122, 5: 0.0139}  # bench.py
frames = [(k * 120 // K) % 120 for k in range(K)]
U = {f: rm.sweep_uniforms(f, 120, B3, AA, SH) for f in set(frames)}


_hip = None


def hip_stream():
    global _hip
    import ctypes
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    if _hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) != 0:  # hipStreamNonBlocking
        raise RuntimeError("hipStreamCreateWithFlags")
    return st.value


def run_shard(N, s, mode, nfl, r0):
    B = 1 if mode == "frames" else int(mode[1:])
    kw = (dict(row_block=R, shard=s, nshards=N, rank0_rows=r0,
               shard_format=rm.RM_SHARD_RGB8 if FMT == "rgb8" else rm.RM_SHARD_RGBA8) if N > 1 else {})
    rs = [rm.Renderer(W, H, **kw) for _ in range(nfl)]
    streams = [None] * nfl
    if STREAMS == "torch":
        streams = [torch.cuda.Stream() for _ in range(nfl)]
    elif STREAMS == "hip":
        streams = [torch.cuda.ExternalStream(hip_stream()) for _ in range(nfl)]
    for r, st in zip(rs, streams):
        if st is not None:
            r.set_stream(st.cuda_stream)
    cap = rm.shard_rows_cap(H, R, N, r0) if N > 1 else H
    gbuf = frame = None
    if N > 1 and s == 0:
        bpp = 3 if FMT == "rgb8" else 4
        gbuf = [torch.zeros((N, B, cap, W, bpp), dtype=torch.uint8, device="cuda") for _ in range(nfl)]
        frame = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(nfl)]
        if B == 1:
            for j, r in enumerate(rs):
                r.set_output_rgba8(gbuf[j][0, 0].data_ptr())
    seq = frames * REPS
    batches = [[U[f] for f in seq[i:i + B]] for i in range(0, len(seq), B)]
    kb = [[U[f] for f in frames[i:i + B]] for i in range(0, K, B)]

    def issue(bl, evs=None):
        for n_, fr in enumerate(bl):
            j = n_ % nfl
            if B == 1:
                rs[j].dispatch(fr[0])
                if gbuf is not None:
                    rs[j].unshard_rgba8(gbuf[j].data_ptr(), frame[j].data_ptr())
            else:
                rs[j].dispatch_frames(fr)
                if gbuf is not None:
                    for k in range(len(fr)):
                        rs[j].unshard_batch_rgba8(gbuf[j].data_ptr(), k, len(fr), frame[j].data_ptr())
            if evs is not None and streams[j] is not None:
                e = torch.cuda.Event(enable_timing=True)
                e.record(streams[j])
                evs.append((len(fr), e))

    def drain():
        for r in rs:
            r.synchronize()
        torch.cuda.synchronize()

    issue(batches)  # warm: buffers, rings, clocks
    drain()
    steady = kk = iss = None
    done = None
    for _ in range(TRIES):
        t0 = time.perf_counter()
        issue(batches)
        ti = time.perf_counter()
        drain()
        dt = (time.perf_counter() - t0) / len(seq) * 1e3
        steady = dt if steady is None else min(steady, dt)
        di = (ti - t0) / len(seq) * 1e3
        iss = di if iss is None else min(iss, di)
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        evs = []
        t0 = time.perf_counter()
        issue(kb, evs)
        drain()
        dk = (time.perf_counter() - t0) / K * 1e3
        if kk is None or dk < kk:
            kk = dk
            # completion time (ms after the start) of every launch, in issue order
            done = [(n_, round(start.elapsed_time(e), 4)) for n_, e in evs] or None
    for r in rs:
        r.close()
    if STREAMS == "hip":
        import ctypes
        for st in streams:
            _hip.hipStreamDestroy(ctypes.c_void_p(st.cuda_stream))
    return round(steady, 4), round(kk, 4), round(iss, 4), done


def gather_model(done, N, gbw):
    """Modelled end of the K frames when every launch's shards then move to rank 0
    (one gather per launch, in completion order, serialised on rank 0's links at gbw
    GB/s of received bytes): returns ms per frame."""
    if N <= 1:
        return max(t for _, t in done) / K
    per_frame = (N - 1) / N * W * H * (3 if FMT == "rgb8" else 4) / (gbw * 1e9) * 1e3  # ms to receive one frame
    end = 0.0
    for n_, t in sorted(done, key=lambda x: x[1]):
        end = max(end, t) + n_ * per_frame
    return end / K


def main():
    t1 = {}
    for N in NS:
        for mode in MODES:
            for nfl in NFLS:
                if R0 == "auto":
                    r0 = rm.best_rank0_rows(R, N, ASSEMBLE_RATIO[CFG]) if N > 1 else 0
                else:
                    r0 = int(R0) if N > 1 else 0
                shards = range(N) if SHARDS == "all" else [int(x) for x in SHARDS.split(",") if int(x) < N]
                res = {s: run_shard(N, s, mode, nfl, r0) for s in shards}
                worst = max(v[0] for v in res.values())
                worst_k = max(v[1] for v in res.values())
                slow = max(res, key=lambda s_: res[s_][1])
                model = ({str(g): round(gather_model(res[slow][3], N, g), 4) for g in (150, 300, 600)}
                         if res[slow][3] else None)
                line = {"cfg": CFG, "N": N, "mode": mode, "contexts": nfl, "K": K, "streams": STREAMS,
                        "shard_format": FMT,
                        "rank0_rows": (r0 or R) if N > 1 else None,
                        "rows": [rm.shard_rows(H, R, N, s, r0)[0] if N > 1 else H for s in shards],
                        "steady_ms": [res[s][0] for s in shards],
                        "k_ms": [res[s][1] for s in shards],
                        "issue_ms": [res[s][2] for s in shards],
                        "max_steady_ms": worst, "max_k_ms": worst_k,
                        "slowest_done_ms": res[slow][3], "k_ms_with_gather_model": model}
                if N == 1:
                    t1[(mode, nfl)] = (worst, worst_k)
                ref = t1.get((mode, nfl))
                best1 = min(t1.values()) if t1 else None
                if ref:
                    line["speedup_same_mode"] = round(ref[0] / worst, 3)
                    line["speedup_same_mode_k"] = round(ref[1] / worst_k, 3)
                if best1:
                    line["speedup_vs_best_1gpu"] = round(best1[0] / worst, 3)
                    line["speedup_vs_best_1gpu_k"] = round(best1[1] / worst_k, 3)
                print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
