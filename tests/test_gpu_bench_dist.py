"""Rehearsal of bench.py's multi-GPU step on ONE GPU.

The driver runs `torch.distributed.run --nproc-per-node N bench.py --gpus N` on
an 8-GPU node with RCCL.  Here N ranks share cuda:0 (RM_BENCH_DEVICE=0) and
gather through host memory with gloo (RM_BENCH_BACKEND=gloo); everything else --
interleaved row-block shards, frames in flight on separate streams, the
event-ordered comm stream, rank 0's on-device un-shard, the max-over-ranks
timing, the JSON line -- is bench.py's own code.  Rank 0 checks the assembled
frame of the last step against a single-GPU render and reports it as `parity`.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(n, *args):
    env = dict(os.environ, RM_BENCH_BACKEND="gloo", RM_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(n), *args]
    out = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("n,args", [
    (2, ("--config", "2", "--steps", "4", "--warmup", "2")),
    (3, ("--config", "3", "--steps", "3", "--warmup", "1")),
    (2, ("--config", "2", "--steps", "3", "--warmup", "1", "--pipeline", "0")),
])
def test_bench_ranks_share_one_gpu(n, args):
    d = _run(n, *args)
    assert d["n_gpus"] == n and d["steps"] == int(args[args.index("--steps") + 1])
    assert d["value"] > 0 and d["scaling"] == "strong"
    assert "RCCL gather" in d["config"]["parallelism"]
    p = d["parity"]
    assert p["assembled_equals_single_gpu"] and p["max_abs_delta_rgba8"] == 0, p
    assert p["pixels_checked"] == d["config"]["width"] * d["config"]["height"]


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ("--config", "2", "--steps", "4", "--warmup", "2"),
    ("--config", "3", "--steps", "3", "--warmup", "1", "--pipeline", "0"),
])
def test_bench_rccl_path_at_world_size_one(args):
    """bench.py's N > 1 step with its real RCCL calls (backend "nccl": init with
    device_id, gather on the comm stream, barrier, all-reduce of the time) at
    world size 1 (RM_BENCH_FORCE_DIST=1): RCCL refuses two ranks on one GPU, so
    this is the one-GPU run of the driver's multi-GPU code path."""
    env = dict(os.environ, RM_BENCH_FORCE_DIST="1", RANK="0", LOCAL_RANK="0", WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.pop("RM_BENCH_BACKEND", None)
    env.pop("RM_BENCH_DEVICE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                         cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and "RCCL gather" in d["config"]["parallelism"]
    p = d["parity"]
    assert p["assembled_equals_single_gpu"] and p["max_abs_delta_rgba8"] == 0, p
