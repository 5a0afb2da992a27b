#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X SDF ray marcher (librm).

Metric (BASELINE.json): Mpixels/s = frames/s x W x H of the per-pixel sphere
tracer (reference hot path shaders/computeShader.glsl, dispatched by
main.cpp:123), on synthetic frames of the fixed camera sweep S(120) of SURVEY
8(d).  One "step" = one frame of the sweep rendered by the HIP kernel (for
N > 1: every rank renders its interleaved row blocks, then an RCCL gather to
rank 0 and an on-device un-shard assemble the frame).

Default workload = BASELINE config 3: 3840x2160, 3 reflection bounces, soft
shadows, 4x supersampling, 1 MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1..5]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

--gpus N > 1 without a launcher (no WORLD_SIZE in the environment) runs the same
sharded, RCCL-gathered step in this one process over N devices (librm's
rm_config.ngpus contexts: one shard per device, a single-process communicator,
the gather and rank 0's assembly inside librm); with fewer than N visible devices
it exits with status 2.

Step k of K renders sweep frame floor(k * 120 / K): every run samples the whole
sweep evenly, so `value` is the sweep mean.

Timing: barrier + device synchronise, t0, the K steps, each rank's streams drained
+ device synchronise, t1, barrier; `value` uses the max over ranks of t1 - t0 (the
host barrier's own round trip is outside the interval, the slowest rank's end is in).

Rank 0 prints ONE JSON line.  Extra objects:
  roofline        : FP32-VALU issue roofline of the dominant kernel (k_sample /
                    k_pixel): achieved = SQ_INSTS_VALU per launch (committed
                    rocprofv3 PMC pass over the same sweep frames, profiles/) x 64
                    lanes / the mean kernel time measured here with HIP events on
                    the launch stream, against 78.65 T lane-instructions/s.
  algorithmic_rate: the reference's brute-force op count per kernel
                    second; the kernel skips most of it by proof, so it is not a
                    utilisation.
  cpu_baseline    : the CPU oracle (a C restatement of the reference shader) on
                    this host's cores, -O3 and -O3 -march=native builds, over the
                    last timed frame; its rows are also compared with the GPU frame
                    (parity).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd")
sys.path.insert(0, PKG)

import rmarch as rm  # noqa: E402

METRIC = "Mpixels/s (frames/s × W×H) at 1/2/4/8 MI355X; max-|Δ| vs GLSL ref"

# BASELINE.json configs (index 1-based as in SURVEY 8(d)).
CONFIGS = {
    1: dict(width=512, height=512, bounces=0, aa=False, shadow=rm.RM_SHADOW_HARD,
            desc="512x512, 0 reflections, hard shadows, no MSAA"),
    2: dict(width=1920, height=1080, bounces=1, aa=False, shadow=rm.RM_SHADOW_SOFT,
            desc="1920x1080, 1 reflection, soft shadows, no MSAA"),
    3: dict(width=3840, height=2160, bounces=3, aa=True, shadow=rm.RM_SHADOW_SOFT,
            desc="3840x2160, 3 reflections, soft shadows, 4xMSAA"),
    4: dict(width=3840, height=2160, bounces=5, aa=True, shadow=rm.RM_SHADOW_SOFT,
            desc="3840x2160, 5 reflections, soft shadows, 4xMSAA"),
    5: dict(width=7680, height=4320, bounces=3, aa=True, shadow=rm.RM_SHADOW_SOFT,
            desc="7680x4320, 3 reflections, soft shadows, 4xMSAA"),
}
SWEEP_FRAMES = 120

# Rank 0 also assembles every gathered frame (k_unshard, HBM-bound: the RGB8 shards
# read and the RGBA8 frame written at ~6.3 TB/s).  Its time over one GPU's render
# time of the whole frame, per config, measured on one MI355X (tools/probe_unshard.py,
# profiles/r06_unshard_rgb8.txt: 3.6 / 3.8 / 9.3 / 9.3 / 36.0 us; frame times of
# DESIGN §9): --rank0-share -1 gives rank 0 the rows per round that balance its
# render + assembly against the other ranks' render (rm.best_rank0_rows).
ASSEMBLE_RATIO = {1: 0.58, 2: 0.082, 3: 0.0132, 4: 0.0122, 5: 0.0139}  # round 6


def bench_frames(steps: int) -> list:
    """Sweep frames of the K timed steps: step k renders frame floor(k * 120 / K), so
    every run samples the whole sweep S(120) evenly (K = 120: every frame once) and
    `value` is the sweep mean, not the cost of one stretch of it."""
    return [(k * SWEEP_FRAMES // steps) % SWEEP_FRAMES for k in range(steps)]

# Algorithmic FP32 ops per unit of work, SURVEY 8(d) (counted as written in the
# GLSL; uniform-only subexpressions excluded).  See DESIGN.md §6.
OPS = dict(march=116, reflect=116, shadow=117, normal=446, light=90, ray=33)
VALU_PEAK_TFLOPS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md), FMA = 2 ops
VALU_LANE_PEAK_T = VALU_PEAK_TFLOPS / 2  # VALU lane-instructions/s
# VALU issue slots: each SIMD issues one VALU slot per quad-cycle (4 cycles), in
# which either one instruction issues, or two dual-issuable ones of different
# waves (f32 add / mul / fma / mov with VGPR, literal or inline operands); an
# SGPR operand, compares, selects, min / max take a whole slot, transcendentals
# two (measured: tools/valu_peak.hip, profiles/r03_valu_peak.txt).
VALU_ISSUE_PEAK_G = 256 * 4 * 2.4 / 4  # G quad-cycle slots/s: 256 CUs x 4 SIMDs at 2.4 GHz
HBM_PEAK_GBS = 8000.0      # HBM3E spec


def algorithmic_ops(c: dict) -> int:
    return (OPS["march"] * c["march_steps"] + OPS["reflect"] * c["reflect_steps"]
            + OPS["shadow"] * c["shadow_steps"] + OPS["normal"] * c["normals"]
            + OPS["light"] * c["lights"] + OPS["ray"] * c["rays"])


def pmc_entry(kernel_name: str, workload: str):
    """Per-launch PMC values of `kernel_name` from the newest committed summary
    (profiles/rNN_pmc.json, separate rocprofv3 passes of tools/profile_round.sh:
    FETCH_SIZE / WRITE_SIZE -> HBM bytes, SQ_INSTS_VALU -> executed VALU)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("_meta", {}).get("workload") != workload:
            continue
        # "k_table_sample<false>" also names its slot instances "k_table_sample<false, 5>"
        stem = kernel_name[:-1] if kernel_name.endswith(">") else kernel_name
        for k, v in d.items():
            if (kernel_name in k or stem + "," in k) and "hbm_bytes_per_launch" in v:
                # a batch kernel's counters are per frame only when the summary divided
                # them by the frames of a launch (tools/summarize_profiles.py records
                # frames_per_launch); an entry without it is per launch: not used
                if "_frames" in k and "frames_per_launch" not in v:
                    continue
                return v, os.path.basename(path)
    return None, None


def cpu_share() -> dict:
    """Logical CPUs of this host (nproc) and those this process may run on: the
    affinity mask, capped by a cgroup CPU quota (cpu.max) when there is one."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(period)))
    except (OSError, ValueError):
        pass
    share = min(aff, quota) if quota else aff
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "share": share, "model": model}


def cpu_baseline(args, cfg, u, f):
    """The reference's path on this host's cores: the CPU oracle (a C restatement of
    computeShader.glsl, test/baseline infrastructure) in both BASELINE.md builds,
    -O3 -ffp-contract=off and the same plus -march=native (compiled here, for this
    CPU), OpenMP schedule(dynamic,1) over rows.  Returns (cpu_baseline, the default
    build's rows, the rows rendered)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import tempfile
    import oracle as O  # test/baseline infrastructure only
    W, H = cfg["width"], cfg["height"]
    # the whole frame for every BASELINE config (cfg5, the largest: ~7 s per build
    # on the box's 16 CPUs); every 4th row only beyond that
    stride = args.cpu_row_stride or (1 if W * H * (4 if cfg["aa"] else 1) * max(cfg["bounces"], 1)
                                     <= 7680 * 4320 * 4 * 5 else 4)
    rows = list(range(0, H, stride))
    sh = cpu_share()
    threads = args.cpu_threads or sh["share"]
    variants, ref = {}, None
    for name in ("O3", "O3 -march=native"):
        try:
            L = O.lib() if name == "O3" else O.load(O.build_native(tempfile.mkdtemp(prefix="rmo_")))
        except Exception as e:  # no compiler on this host: report the default build only
            variants[name] = {"error": str(e)[:200]}
            continue
        c0 = time.perf_counter()
        res = O.render(u, W, H, rows=rows, nthreads=threads, want_f32=False, want_counts=False, L=L)
        dt = time.perf_counter() - c0
        if ref is None:
            ref = res
        variants[name] = {"Mpixels_per_s": round(len(rows) * W / dt / 1e6, 4), "wall_s": round(dt, 3)}
    best = max((v["Mpixels_per_s"] for v in variants.values() if "Mpixels_per_s" in v))
    sample = (f"sweep frame {f} of {cfg['desc']}: "
              + ("the whole frame" if stride == 1 else f"every {stride}th row ({len(rows)} rows)")
              + f", {len(rows) * W} px, one process, {threads} OpenMP threads")
    cpu = {"value": best, "unit": "Mpixels/s", "cores": sh["share"], "threads": threads,
           "kind": "port", "sample": sample, "variants": variants,
           "host": {"nproc_logical": sh["nproc"], "affinity": sh["affinity"],
                    "cgroup_cpu_quota": sh["cgroup_quota"], "cpu_model": sh["model"]},
           "note": "cores = logical CPUs this process may use (affinity mask, cgroup quota); "
                   "value = the faster build"}
    return cpu, ref, rows


def pmc_frames(name):
    if not name:
        return None
    try:
        return json.load(open(os.path.join(ROOT, "profiles", name)))["_meta"].get("frames")
    except (OSError, ValueError, KeyError):
        return None


def comm_ids(n: int, rank: int) -> list:
    """n RCCL unique ids for rm_comm_init, made on rank 0 (rm_comm_unique_id) and
    broadcast over the torch.distributed host channel (gloo)."""
    import torch.distributed as dist
    ids = [rm.comm_unique_id() for _ in range(n)] if rank == 0 else [None] * n
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast_object_list(ids, src=0)
    return ids


def default_batch(config: int, sharded: bool, one_comm: bool, steps: int, table: bool = False) -> int:
    """Frames per launch when --batch is not given (measured).

    One GPU: cfg1 / cfg2 frames (4K / 32K one-wave workgroups) are shorter than their
    longest waves and cannot fill 256 CUs alone.  Over the whole 120-frame sweep, 20
    frames per launch on 3 contexts render at 0.0090 / 0.0575 ms per frame against
    0.0124 / 0.0594 for 10 on 2 (round 4, tools/probe_batch.py --steps 120,
    profiles/r04_probe_batch120.txt); fewer steps cap the batch so that the launches
    still spread over the 3 contexts.  The 4K supersampled frames fill the chip by
    themselves: single frames on 3 contexts (k_sample) measure 1.4 % (cfg3) and 1.3 %
    (cfg4) faster than pairs on 4 (k_sample_frames: the same VALU instructions per
    frame, 7 % more SALU) since round 5's kernel (round 6, tools/ab_issue.sh, 5
    interleaved rounds: 0.7041 against 0.7139 ms, profiles/r06_ab_issue.txt; round 4
    had measured pairs 0.8 % ahead); the 8K graph-replayed frames (cfg5) stay single,
    3 in flight.  A runtime scene table's 4K frames keep pairs on 4 contexts: its
    kernels gain from them (generic -2.5 %, specialised -0.7 % per cfg3 frame against
    single frames on 3, profiles/r06_ab_tables.txt).

    N > 1: pairs of frames per launch on 2 contexts (round 6, tools/probe_scale.py,
    profiles/r06_scale.txt): a rank's 1/N share of a frame is shorter than its
    longest waves, so single-frame launches left the SIMDs idle behind them (N = 8:
    4.4x one GPU on 4 contexts); pairs on 2 contexts give ~6.9x at N = 8 in the
    probe with either stream placement, and a launch's gather starts as soon as its
    two frames are done (larger batches gather more bytes after the last render)."""
    if one_comm:
        return 4  # N > 1, one communicator: gather batch j while batch j + 1 renders
    if sharded:
        return 2
    if config in (1, 2):
        return max(1, min(20, -(-steps // 3)))
    return 2 if table and config in (3, 4) else 1


def _gather_objects(mine, ws):
    """Every rank's `mine` (torch.distributed over gloo), or [mine] in one process."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [mine]
    allp = [None] * ws
    dist.all_gather_object(allp, mine)
    return allp


def frame_phase_stats(r, frames, uniforms, batch, rank, ws):
    """Per-rank render / gather / assembly split (rm_frame_phases: HIP events around the
    render kernel, the ncclGather and rank 0's assembly) over EVERY timed frame, re-rendered
    eagerly after the timed region (one frame, or one batch, at a time), so a scaling
    shortfall can be attributed to render imbalance or to the gather."""
    vals = {"render_ms": [], "gather_ms": [], "assemble_ms": []}
    r.enable_timing(True)
    for i in range(0, len(frames), batch):
        chunk = frames[i:i + batch]
        if batch > 1:
            r.dispatch_frames([uniforms(f) for f in chunk])
        else:
            r.dispatch(uniforms(chunk[0]))
        ph = r.frame_phases()  # synchronizes
        for k in vals:
            vals[k].append(ph[k] / len(chunk))
    r.enable_timing(False)
    r.kernel_time_ms(reset=True)
    vals["render_plus_assemble_ms"] = [a + b for a, b in zip(vals["render_ms"], vals["assemble_ms"])]
    mine = {"rank": rank}
    for k, v in vals.items():
        mine[k.replace("_ms", "_mean_ms")] = round(float(np.mean(v)), 4)
        mine[k.replace("_ms", "_max_ms")] = round(float(np.max(v)), 4)
    allp = _gather_objects(mine, ws)
    return {"per_rank": allp,
            "frames": len(frames), "frames_per_sample": batch,
            "max_render_mean_ms": max(p["render_mean_ms"] for p in allp),
            "max_render_max_ms": max(p["render_max_ms"] for p in allp),
            "max_gather_mean_ms": max(p["gather_mean_ms"] for p in allp),
            "max_gather_max_ms": max(p["gather_max_ms"] for p in allp),
            "assemble_mean_ms": allp[0]["assemble_mean_ms"],
            # rank 0 renders its (smaller, --rank0-share) shard and assembles; the others
            # render: balanced when rank 0's sum is at most the largest other render
            "rank0_render_plus_assemble_mean_ms": allp[0]["render_plus_assemble_mean_ms"],
            "max_other_render_mean_ms": max((p["render_mean_ms"] for p in allp[1:]), default=None),
            "note": "every timed frame re-rendered eagerly after the timed region, one "
                    + ("frame" if batch == 1 else f"batch of {batch} frames (values per frame)")
                    + " at a time; gather_ms runs from this rank's render end to its gather end, "
                      "so it includes waiting for the slowest peer's shard"}


def rccl_report(rs, rank, ws):
    """What RCCL itself reports for every communicator of every rank (ncclCommCount,
    ncclCommUserRank, ncclCommCuDevice, ncclGetVersion via rm_comm_rccl_info): the line
    proves how many ranks RCCL formed, not only torch's WORLD_SIZE."""
    mine = {"rank": rank, "comms": [rj.rccl_info() for rj in rs]}
    allr = _gather_objects(mine, ws)
    counts = sorted({c["count"] for p in allr for c in p["comms"]})
    # (one process over N devices: rm_comm_rccl_info checks every device's member
    # communicator against its user rank and device, and reports device 0's)
    ok = all(c["count"] == ws and c["user_rank"] == p["rank"] for p in allr for c in p["comms"])
    return {"version": allr[0]["comms"][0]["version"] if allr[0]["comms"] else None,
            "nranks_seen": counts, "world_size": ws, "all_communicators_match": ok,
            "per_rank": allr}


def run_mode(gpus: int, launched: bool, ws: int, single_process: bool):
    """How bench.py runs --gpus N: ("launcher", None) under torch.distributed.run
    (one process per GPU, WORLD_SIZE set); ("single_process", None) without a
    launcher when N > 1 or --single-process (every device in this process, librm's
    rm_config.ngpus contexts); ("single_gpu", None) for N = 1; ("error", why) for a
    launcher whose world size is not N, or N < 1."""
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    if launched:
        if ws != gpus:
            return "error", f"launched with WORLD_SIZE={ws} but --gpus {gpus}"
        if single_process:
            return "error", "--single-process runs without a launcher"
        return "launcher", None
    if gpus > 1 or single_process:
        return "single_process", None
    return "single_gpu", None


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--row-block", type=int, default=8,
                    help="rows per interleaved block when sharding over ranks")
    ap.add_argument("--single-process", action="store_true",
                    help="the sharded, RCCL-gathered step over --gpus devices in this one process "
                         "(rm_config.ngpus), also at --gpus 1; the default when --gpus N > 1 runs "
                         "without a launcher")
    ap.add_argument("--rank0-share", type=float, default=-1.0,
                    help="N > 1: rank 0's rows per round as a share of --row-block (rank 0 also "
                         "assembles every frame, so it renders fewer rows: rm_config.rank0_rows = "
                         "round(share x row_block)); -1 = the share that balances rank 0's render + "
                         "assembly against the other ranks' render for this config (ASSEMBLE_RATIO)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="1: replay the frame from a captured hipGraph (rm_graph_dispatch); "
                         "default: on for config 5 (BASELINE 'hipGraph-captured frame')")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight: consecutive frames render from separate contexts on "
                         "separate streams, so frame f+1's waves fill the SIMDs that frame f's "
                         "last long waves leave idle (1 = one context, frames in turn; "
                         "0 = 3 on one GPU, 2 on a sharded frame, each launch two frames)")
    ap.add_argument("--batch", type=int, default=-1,
                    help="frames per launch (rm_dispatch_frames: one grid over B frames, so frame "
                         "k+1's waves fill the SIMDs frame k's longest waves leave idle); 1 = one "
                         "rm_dispatch per frame; -1 = the measured default for the configuration")
    ap.add_argument("--comms", type=int, default=0,
                    help="N > 1: communicators per rank.  0 = one per in-flight context (frames in "
                         "flight on separate streams, each gathering behind its own render); 1 = one "
                         "context and one communicator per rank: batches of --batch frames render in "
                         "one launch and move in one ncclGather on the context's gather stream, "
                         "ordered by events, while the next batch renders")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="N > 1: gather frame f on a second stream while frame f+1 renders "
                         "(double-buffered shard images); 0 = render, gather, assemble in turn")
    ap.add_argument("--scene", default="builtin", choices=["builtin", "table", "table-spec"],
                    help="table = the reference scene as a runtime scene table (rm_set_scene with "
                         "rm_default_scene: the k_table_* kernels, SURVEY 8(f) row 4); table-spec = "
                         "the same with kernels compiled for the table (rm_scene_specialize, hiprtc, "
                         "before the timed region); the image is the built-in scene's")
    ap.add_argument("--spinup-ms", type=float, default=200.0,
                    help="before the warmup steps, render sweep frames (untimed) for this long so "
                         "the GPU reaches its sustained clocks: with the 5-step warmup alone the "
                         "first timed frames run ~6%% slower (tools/probe_ramp.py)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-row-stride", type=int, default=0,
                    help="cpu_baseline renders every k-th row of one frame (0: the whole "
                         "frame for every BASELINE config)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = nproc, capped at the CPUs this process may run on")
    args = ap.parse_args()

    # stdout carries exactly the one JSON line: library banners written to fd 1
    # (gloo's connection notice, RCCL's version block) go to stderr until then
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    ws, rank, local = dist_env()
    # RM_BENCH_FORCE_DIST=1 (tests/test_gpu_bench_dist.py): the sharded, RCCL-gathered
    # step even at world size 1, so one GPU runs the driver's N > 1 code path and its
    # RCCL calls (communicator, gather, assembly inside librm) on hardware
    dist_on = ws > 1 or os.environ.get("RM_BENCH_FORCE_DIST") == "1"
    # --gpus N without a launcher: every device in this process (rm_config.ngpus)
    mode, why = run_mode(args.gpus, "WORLD_SIZE" in os.environ, ws, args.single_process)
    if mode == "error":
        print(f"bench.py: {why}", file=sys.stderr)
        return 2
    single = mode == "single_process"
    if single:
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} in one process needs {args.gpus} visible devices, "
                  f"this host shows {ndev}", file=sys.stderr)
            return 2
    sharded = dist_on or single
    nsh = ws if dist_on else (args.gpus if single else 1)  # shards of every frame
    torch.cuda.set_device(local)
    if dist_on:
        # host-side control only (RCCL ids, barriers, the max over ranks of the time):
        # the frame data moves inside librm, over its own RCCL communicators
        import datetime
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))

    cfg = CONFIGS[args.config]
    W, H = cfg["width"], cfg["height"]
    kernel = rm.RM_KERNEL_PIXEL
    use_graph = (args.graph == 1) or (args.graph < 0 and args.config == 5)
    # Frames in flight: consecutive frames go to separate contexts, each with its own
    # stream, image and (N > 1) RCCL communicator, so frame f+1's waves fill the SIMDs
    # that frame f's last long waves leave idle, and frame f gathers while f+1 renders.
    one_comm = sharded and args.comms == 1
    batch = (args.batch if args.batch > 0
             else default_batch(args.config, sharded, one_comm, args.steps, args.scene != "builtin"))
    batch = max(1, min(batch, rm.RM_MAX_BATCH, args.steps))
    if use_graph:
        batch = 1  # a graph replays one frame
    # contexts in flight: 3 frames or batches on one GPU (4 for the 4K pairs), 2
    # batches of a sharded step (default_batch)
    nfl = args.inflight if args.inflight > 0 else (2 if sharded else (4 if batch == 2 and args.config in (3, 4)
                                                                    else 3))
    nfl = nfl if (not sharded or args.pipeline) else 1
    if one_comm:
        nfl = 1  # one context, one communicator; batches overlap through its gather stream

    ucache = {}

    def uniforms(f):
        # host camera per sweep frame (rm_sweep_uniforms), built once: at N = 8 a
        # frame takes ~0.15 ms of GPU time and the host must keep ahead of it
        f %= SWEEP_FRAMES
        if f not in ucache:
            ucache[f] = rm.sweep_uniforms(f, SWEEP_FRAMES, cfg["bounces"], cfg["aa"], cfg["shadow"])
        return ucache[f]

    scene = rm.default_scene() if args.scene in ("table", "table-spec") else None
    spec = args.scene == "table-spec"
    # the weighted interleave (rm_config.rank0_rows, rm_shard.hpp): rank 0's rows per round
    if args.rank0_share > 0:
        rank0_rows = max(1, int(round(args.rank0_share * args.row_block)))
        rank0_src = f"--rank0-share {args.rank0_share}"
    elif nsh > 1 and scene is None:
        rank0_rows = rm.best_rank0_rows(args.row_block, nsh, ASSEMBLE_RATIO[args.config])
        rank0_src = (f"rm.best_rank0_rows(row_block, N, ASSEMBLE_RATIO[{args.config}] = "
                     f"{ASSEMBLE_RATIO[args.config]}): k_unshard time over the built-in scene's one-GPU "
                     "frame time, tools/probe_unshard.py")
    else:
        #  the assembly ratio was measured for the built-in scene's frame
        # time: a runtime table renders slower, so it keeps the plain interleave
        rank0_rows = 0
        rank0_src = "plain interleave" + (" (scene table)" if nsh > 1 else "")
    if dist_on:
        shard_args = dict(row_block=args.row_block, shard=rank, nshards=ws, rank0_rows=rank0_rows)
    elif single:
        shard_args = dict(row_block=args.row_block, ngpus=nsh, rank0_rows=rank0_rows)
    else:
        shard_args = {}
    rs = [rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8, kernel=kernel, device=local, **shard_args)
          for _ in range(nfl)]
    if dist_on:
        # one communicator per in-flight context (rm_comm_init): rank 0 makes the
        # ids, the host channel carries them; every rank joins in the same order
        for rj, cid in zip(rs, comm_ids(nfl, rank)):
            rj.comm_init(cid, ws, rank)

    def use_scene(rj):
        if spec:
            rj.specialize_scene(True)
        rj.set_scene(scene)

    if scene is not None:
        for rj in rs:
            use_scene(rj)
    r = rs[0]
    for rj in rs:
        if use_graph:
            rj.graph_enable(True)

    def render(j, f):
        # one frame on context j: render; for N > 1 also the gather on rank 0 and
        # rank 0's assembly, all inside librm on the context's stream
        if use_graph:
            rs[j].graph_dispatch(uniforms(f))
        else:
            rs[j].dispatch(uniforms(f))

    nstep = [0]  # steps issued so far: step n renders on context n % nfl

    def step(f):
        j = nstep[0] % nfl
        nstep[0] += 1
        render(j, f)

    barr = {}  # rm_uniforms arrays of the batches, built before the timed region

    def issue(frames):
        # the frames of a run of steps: one rm_dispatch per frame, or rm_dispatch_frames
        # per `batch` consecutive frames (the contexts take the batches in turn)
        if batch <= 1 or use_graph:
            for f in frames:
                step(f)
            return
        for i in range(0, len(frames), batch):
            key = tuple(frames[i:i + batch])
            if key not in barr:
                barr[key] = [uniforms(f) for f in key]
            j = nstep[0] % nfl
            nstep[0] += 1
            rs[j].dispatch_frames(barr[key])

    devs = list(range(local, local + nsh)) if single else [local]

    def sync_devices():
        for d in devs:  # the device(s): every librm stream
            torch.cuda.synchronize(d)

    def barrier():
        # librm's own wait first: on a communicator context it is bounded
        # (rm_comm_set_timeout) and turns a hung gather into RM_ERR_COMM
        for rj in rs:
            rj.synchronize()
        sync_devices()
        if dist_on:
            dist.barrier()
        sync_devices()

    frames_timed = bench_frames(args.steps)
    # ---- spin-up (untimed): sustained load until the GPU's clocks have ramped ----
    # (rounds of nfl frames; with N > 1 every rank runs the same rounds, as each
    # frame's gather is a collective: rank 0's clock decides, over the host group)
    if args.spinup_ms > 0:
        s0, k = time.perf_counter(), 0
        while True:
            for _ in range(nfl):
                n = max(batch, 1) if not use_graph else 1
                issue([frames_timed[(k + i) % args.steps] for i in range(n)])
                k += n
            for rj in rs:
                rj.synchronize()
            sync_devices()
            more = (time.perf_counter() - s0) * 1e3 < args.spinup_ms
            if dist_on:
                flag = torch.tensor([1 if more else 0], dtype=torch.int32)
                dist.broadcast(flag, src=0)
                more = bool(flag.item())
            if not more:
                break
        nstep[0] = 0
    # ---- warmup (untimed): the first W frames of the same list ----
    issue([frames_timed[k % args.steps] for k in range(args.warmup)])
    barrier()

    # ---- timed region: exactly K steps ----
    # (with frames in flight the kernel time comes from a one-at-a-time re-render
    # below, so no per-launch timing events are recorded in the timed region)
    for f in frames_timed:
        uniforms(f)
    for i in range(0, len(frames_timed), batch):
        key = tuple(frames_timed[i:i + batch])
        barr.setdefault(key, [uniforms(f) for f in key])
    for rj in rs:
        rj.enable_timing(nfl == 1)
        rj.kernel_time_ms(reset=True)
    barrier()
    t0 = time.perf_counter()
    issue(frames_timed)
    t_issue = time.perf_counter()
    # the end of the K steps on this rank: every librm stream drained (bounded on a
    # communicator context) and the device synchronised; then the host barrier,
    # whose own latency (a gloo round trip, ~0.1-1 ms) is not frame work.  The max
    # over ranks below takes the slowest rank's end.
    for rj in rs:
        rj.synchronize()
    sync_devices()
    t1 = time.perf_counter()
    barrier()
    kernel_ms, launches = 0.0, 0
    for rj in rs:
        ms_j, n_j = rj.kernel_time_ms(reset=True)
        kernel_ms += ms_j
        launches += n_j
        rj.enable_timing(False)
    kernel_time_basis = "HIP events on the launch stream over the timed region"
    batched = batch > 1 and not use_graph
    mean_launch_ms = None
    if nfl > 1 or batch > 1 or (use_graph and sharded):
        # Overlapping frames stretch each launch's event interval (and on a
        # communicator context a graph launch holds the gather and the assembly
        # too), so the roofline takes its kernel time from the same frames rendered
        # one at a time on one context through rm_dispatch, whose HIP events
        # bracket the render kernel alone (untimed for `value`).
        # A batched run re-renders the same batches one at a time: the events
        # bracket each batch's launch, which counts its frames.
        barrier()
        r.enable_timing(True)
        r.kernel_time_ms(reset=True)
        nlaunch = 0
        if batched:
            for i in range(0, len(frames_timed), batch):
                r.dispatch_frames(barr[tuple(frames_timed[i:i + batch])])
                nlaunch += 1
        else:
            for f in frames_timed:
                r.dispatch(uniforms(f))
                nlaunch += 1
        barrier()
        kernel_ms, launches = r.kernel_time_ms(reset=True)
        r.enable_timing(False)
        kernel_time_basis = ("HIP events around the render kernel, the timed frames re-rendered "
                             + (f"in their batches of {batch}, one launch at a time through "
                                "rm_dispatch_frames" if batched else "one at a time through rm_dispatch")
                             + " (the timed region overlaps frames)")
        mean_launch_ms = kernel_ms / max(nlaunch, 1)
    elapsed = t1 - t0
    phases = None
    rccl = None
    if sharded:
        phases = frame_phase_stats(r, frames_timed, uniforms, batch if batched else 1, rank, ws)
        if single:
            phases["note"] += ("; one process over N devices: rm_frame_phases reports device 0 "
                               "(rank 0's render, the grouped gather, the assembly)")
        barrier()
        rccl = rccl_report(rs, rank, nsh if single else ws)
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    frames = args.steps
    value = frames * W * H / elapsed / 1e6  # whole-job Mpixels/s

    # ---- work counters of exactly the frames timed (untimed pass) ----
    ops_total = 0
    cnt_total = None
    # (the timed kernel's share of the frame: this rank's shard, device 0's in one process)
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8, kernel=kernel, counters=True, device=local,
                     row_block=args.row_block if sharded else 0, shard=rank if dist_on else 0,
                     nshards=nsh, rank0_rows=rank0_rows if sharded else 0) as rc:
        if scene is not None:
            use_scene(rc)
        seen = {}
        for f in frames_timed:
            if f not in seen:
                rc.dispatch(uniforms(f))
                seen[f] = rc.counters()
            c = seen[f]
            ops_total += algorithmic_ops(c)
            cnt_total = dict(c) if cnt_total is None else {x: cnt_total[x] + c[x] for x in c}
    mean_kernel_ms = kernel_ms / max(launches, 1)
    kname = "k_sample" if cfg["aa"] else "k_pixel"
    if scene is not None:
        kname = "k_table_sample" if cfg["aa"] else "k_table_pixel"
    if batched:
        kname += "_frames"  # the batched kernels (grid.z = frame); PMC values per frame
    pmc, traffic_src = pmc_entry(kname if kname.endswith("_frames") else kname + "<false>",
                                 f"cfg{args.config}" + ("-spec" if spec else ""))
    traffic = int(pmc["hbm_bytes_per_launch"]) if pmc else None
    # Roofline of the dominant kernel: the FP32 VALU issue rate.  SQ_INSTS_VALU
    # (wave64 VALU instructions per launch, committed PMC pass over the bench's own
    # sweep frames, tools/profile_round.sh) x 64 lanes / the kernel time measured
    # here, against the lane-instruction peak: 256 CUs x 4 SIMD x 16 lanes x 2.4 GHz
    # x 2 (dual issue) = 157.3 T FP32 ops/s counting an FMA as 2 -> 78.65 T
    # lane-instructions/s.  frac = SQ_INSTS_VALU x 64 / kernel time / 78.65 T.
    valu_frame = pmc.get("SQ_INSTS_VALU") if pmc else None  # the whole frame's, per frame
    # the timed kernel renders this rank's shard (device 0's in one process): the
    # frame's instructions in proportion to its rows (an estimate; PMC passes are
    # one-GPU whole frames)
    share = (rm.shard_rows(H, args.row_block, nsh, 0 if single else rank, rank0_rows)[0] / H
             if sharded and nsh > 1 else 1.0)
    valu_insts = valu_frame * share if valu_frame else None
    valu_issue = (valu_insts * 64 / (mean_kernel_ms * 1e-3) / 1e12) if valu_insts else None
    # the same instructions per frame of the timed region's throughput over the whole
    # job's GPUs: frames overlap on several contexts, so this is
    # the utilisation the measured value implies
    valu_tput = (valu_frame * 64 / (elapsed / frames) / 1e12 / max(nsh, 1)) if valu_frame else None
    # The same kernel against the SIMDs' VALU issue slots: its busy slots per launch
    # (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2, committed PMC pass) per second of
    # the kernel time measured here, over 614.4 G slots/s.
    busy_frame = pmc.get("valu_busy_quads") if pmc else None
    busy_quads = busy_frame * share if busy_frame else None
    issue_rate = (busy_quads / (mean_kernel_ms * 1e-3) / 1e9) if busy_quads else None
    # ... and per frame of the timed region's throughput (frames in flight / batched)
    issue_tput = (busy_frame / (elapsed / frames) / 1e9 / max(nsh, 1)) if busy_frame else None
    ms_step = elapsed / frames * 1e3
    overlap_note = None
    if mean_kernel_ms > ms_step:
        overlap_note = (f"the kernel's own time per frame ({mean_kernel_ms:.4f} ms, launches timed one at a "
                        f"time) exceeds ms_per_step ({ms_step:.4f} ms): in the timed region {nfl} contexts "
                        "overlap their launches, so the next launch's waves fill the SIMDs a launch's last "
                        "long waves leave idle and a frame's share of the wall clock is shorter than one "
                        "launch's duration; frac_throughput is the utilisation at the measured value")
    # The reference's brute-force work (SURVEY 8(d) op weights x the exact counters of
    # the frames timed): the kernel skips most of it by proof, so this rate is not
    # hardware utilisation and can exceed the peak.
    achieved_tflops = ops_total / max(launches, 1) / (mean_kernel_ms * 1e-3) / 1e12
    # algorithmic bytes of the timed kernel's image: RGBA8, or a gathered shard's packed
    # RGB (rm_config.shard_format AUTO on a communicator context)
    bytes_per_launch = (rm.shard_rows_cap(H, args.row_block, nsh, rank0_rows) * W * 3 if sharded
                        else H * W * 4)
    hbm_gbs = bytes_per_launch / (mean_kernel_ms * 1e-3) / 1e9

    # ---- CPU baseline + parity sample (rank 0, N = 1 only) ----
    cpu = None
    parity = None
    if rank == 0 and not sharded and not args.no_cpu_baseline:
        cpu, ref, rows = cpu_baseline(args, cfg, uniforms(frames_timed[-1]), frames_timed[-1])
        # GPU frame of the same sweep frame: the last step rendered it into its context's buffer.
        torch.cuda.synchronize()
        g = rs[(nstep[0] - 1) % nfl].read_rgba8()[rows]
        d = np.abs(g.astype(np.int16) - ref["rgba8"].astype(np.int16))
        parity = {"max_abs_delta_rgba8": int(d.max()), "pixels_over_2": int((d.max(-1) > 2).sum()),
                  "pixels_checked": int(d.shape[0] * d.shape[1]), "reference": "CPU oracle"}

    # ---- N > 1: the assembled frame of the last step against a single-GPU render ----
    if sharded and rank == 0:
        sync_devices()
        last = frames_timed[-1]
        with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8, kernel=kernel, device=local) as rf:
            if scene is not None:
                use_scene(rf)
            rf.dispatch(uniforms(last))
            full = rf.read_rgba8()
        frame = rs[(nstep[0] - 1) % nfl].read_rgba8()  # rank 0: the assembled frame
        d = np.abs(frame.astype(np.int16) - full.astype(np.int16))
        parity = {"assembled_equals_single_gpu": bool(d.max() == 0),
                  "max_abs_delta_rgba8": int(d.max()), "pixels_checked": int(W * H),
                  "reference": f"single-GPU render of sweep frame {last % SWEEP_FRAMES}"}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mpixels/s",
            "n_gpus": nsh if sharded else ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / frames * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (camera sweep S(120), SURVEY 8(d))",
            "config": {"workload": f"cfg{args.config}: {cfg['desc']}"
                                   + (" (scene table)" if scene is not None and not spec else "")
                                   + (" (scene table, specialised)" if spec else ""), "width": W, "height": H,
                       "bounces": cfg["bounces"], "aa": cfg["aa"],
                       "shadow": "hard" if cfg["shadow"] == rm.RM_SHADOW_HARD else "soft",
                       "kernel": kname, "hipgraph": bool(use_graph),
                       "contexts_in_flight": nfl,
                       "frames_per_launch": batch if batched else 1,
                       "frames_in_flight": nfl * (batch if batched else 1),
                       "communicators_per_rank": (1 if one_comm else nfl) if sharded else 0,
                       "parallelism": (f"row-blocks of {args.row_block} x {nsh} GPUs + RCCL gather"
                                       + (" (pipelined)" if args.pipeline else "")
                                       + (", one process (rm_config.ngpus)" if single
                                          else ", one process per GPU (rm_comm_init)")
                                       if sharded else "single GPU"),
                       "rank0_rows_per_round": (rank0_rows or args.row_block) if sharded else None,
                       "rank0_rows_source": rank0_src if sharded else None,
                       "shard_format": ("RGB8: 3 B per pixel gathered, alpha 255 restored by k_unshard "
                                        "(rm_config.shard_format AUTO)") if sharded else None,
                       "rows_per_rank": ([rm.shard_rows(H, args.row_block, nsh, s_, rank0_rows)[0]
                                          for s_ in range(nsh)] if sharded else None)},
            "fps": round(frames / elapsed, 3),
            # host time to issue the K steps (rank 0): well below ms_per_step = GPU-bound
            "host_issue_ms_per_step": round((t_issue - t0) / args.steps * 1e3, 4),
            "spinup_ms": args.spinup_ms,
            "roofline": {"bound": "valu",
                         "achieved": round(valu_issue, 3) if valu_issue else None,
                         "peak": VALU_LANE_PEAK_T, "unit": "T VALU lane-instructions/s",
                         "frac": round(valu_issue / VALU_LANE_PEAK_T, 4) if valu_issue else None,
                         "frac_throughput": round(valu_tput / VALU_LANE_PEAK_T, 4) if valu_tput else None,
                         "achieved_throughput": round(valu_tput, 3) if valu_tput else None,
                         "frac_note": ("frac: executed VALU lane-instructions per frame (PMC) over the "
                                       "kernel's own time per frame; frac_throughput: the same "
                                       "instructions over ms_per_step" + (" and the N GPUs; at N > 1 "
                                       "the shard's instructions are the frame's in proportion to its "
                                       "rows" if sharded and nsh > 1 else "")),
                         "kernel_time_vs_step": overlap_note,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "valu_insts_per_launch": valu_insts, "valu_insts_per_frame": valu_frame,
                         "pmc_frames": pmc_frames(traffic_src),
                         "kernel": kname, "mean_kernel_ms": round(mean_kernel_ms, 4),
                         "mean_launch_ms": round(mean_launch_ms, 4) if mean_launch_ms else None,
                         "per": "frame" + (f" (launches of {batch} frames: PMC values, kernel time and "
                                           "traffic divided by the frames of a launch)" if batched else ""),
                         "kernel_time_basis": kernel_time_basis,
                         "hbm_write_GBs": round(hbm_gbs, 2),
                         "hbm_frac": round(hbm_gbs / HBM_PEAK_GBS, 6),
                         "issue": {"achieved": round(issue_rate, 2) if issue_rate else None,
                                   "peak": VALU_ISSUE_PEAK_G, "unit": "G VALU issue slots/s (quad-cycles)",
                                   "frac": round(issue_rate / VALU_ISSUE_PEAK_G, 4) if issue_rate else None,
                                   "busy_slots_per_launch": busy_quads,
                                   "throughput_frac": (round(issue_tput / VALU_ISSUE_PEAK_G, 4)
                                                       if issue_tput else None),
                                   "dual_issued_slots_per_launch": pmc.get("SQ_ACTIVE_INST_VALU2") if pmc else None,
                                   "note": "frac above counts executed VALU lane-instructions at the FP32 "
                                           "vector peak (157.3 TFLOP/s = every instruction dual-issued); "
                                           "this one counts the SIMDs' VALU issue slots the kernel keeps "
                                           "busy (a slot issues one instruction, or two dual-issuable "
                                           "ones; streams that saturate it reach 0.92-0.96, "
                                           "tools/valu_peak.hip); throughput_frac divides the same "
                                           "busy slots per frame by ms_per_step instead"}},
            "algorithmic_rate": {"ops_per_launch": int(ops_total / max(launches, 1)),
                                 "TFLOPs": round(achieved_tflops, 3),
                                 "vs_fp32_peak": round(achieved_tflops / VALU_PEAK_TFLOPS, 4),
                                 "note": "the reference's brute-force op count (SURVEY 8(d)) per "
                                         "kernel second; the kernel skips most of that work by "
                                         "proof, so this is not a utilisation"},
            "work": cnt_total,
            "phases": phases,
            "rccl": rccl,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        sys.stdout.flush()
        os.dup2(json_fd, 1)
        print(json.dumps(out), flush=True)
    for rj in rs:
        rj.close()
    if dist_on:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    try:
        sys.exit(main())
    except rm.RMError as e:
        # a communicator failure (RM_ERR_COMM: RCCL error, a peer that died or
        # stalled past the deadline) ends this rank with a diagnosis, non-zero
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(3 if e.code == rm.RM_ERR_COMM else 4)
