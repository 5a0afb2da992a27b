"""bench.py's multi-GPU step on ONE GPU.

The driver runs `torch.distributed.run --nproc-per-node N bench.py --gpus N` on
an 8-GPU node: every rank joins its in-flight shard contexts to RCCL
communicators inside librm (rm_comm_init; the ids travel over a gloo host
group), and each step renders, gathers (ncclGather) and assembles (rank 0)
inside librm.  RCCL refuses two ranks on one GPU, so RM_BENCH_FORCE_DIST=1 runs
that exact code path at world size 1; rank 0 checks its assembled last frame
against a plain one-GPU render and reports it as `parity`.
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


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ("--config", "2", "--steps", "4", "--warmup", "2"),
    ("--config", "3", "--steps", "3", "--warmup", "1", "--pipeline", "0"),
    ("--config", "2", "--steps", "5", "--warmup", "2", "--graph", "1"),
    # one communicator per rank: batches of frames gathered on the context's gather stream
    ("--config", "2", "--steps", "9", "--warmup", "2", "--comms", "1", "--batch", "4"),
    ("--config", "3", "--steps", "4", "--warmup", "1", "--comms", "1", "--batch", "2"),
])
def test_bench_rccl_path_at_world_size_one(args):
    """bench.py's N > 1 step with its real RCCL calls (librm communicators, gather
    and assembly; gloo host group for the ids, barriers and the max of the time)
    at world size 1, plainly and from the captured per-rank graph."""
    env = dict(os.environ, RM_BENCH_FORCE_DIST="1", RANK="0", LOCAL_RANK="0", WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                         cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = out.stdout.strip().splitlines()  # stdout is the JSON line alone (banners: stderr)
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and "RCCL gather" in d["config"]["parallelism"]
    p = d["parity"]
    assert p["assembled_equals_single_gpu"] and p["max_abs_delta_rgba8"] == 0, p
    # per-rank render / gather / assembly split over every timed frame
    ph = d["phases"]
    steps = int(args[args.index("--steps") + 1])
    assert len(ph["per_rank"]) == 1 and ph["frames"] == steps, ph
    assert ph["max_render_mean_ms"] > 0 and ph["max_render_max_ms"] >= ph["max_render_mean_ms"], ph
    assert ph["assemble_mean_ms"] > 0 and ph["max_gather_max_ms"] >= ph["max_gather_mean_ms"] >= 0, ph
    # what RCCL itself formed: every communicator of every rank is rank r of WORLD_SIZE
    rc = d["rccl"]
    assert rc["nranks_seen"] == [1] and rc["all_communicators_match"] and rc["version"] > 0, rc
    ncomm = d["config"]["communicators_per_rank"]
    one = "--comms" in args or ("--pipeline" in args and args[args.index("--pipeline") + 1] == "0")
    assert len(rc["per_rank"][0]["comms"]) == ncomm == (1 if one else 2), rc
    assert "render kernel" in d["roofline"]["kernel_time_basis"] or args[-1] == "0"
    assert d["config"]["shard_format"].startswith("RGB8") and d["config"]["rank0_rows_source"]


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ("--config", "2", "--steps", "6", "--warmup", "2"),
    ("--config", "3", "--steps", "4", "--warmup", "2", "--batch", "1"),
])
def test_bench_single_process_ngpus_path(args):
    """`python bench.py --gpus N` without a launcher runs the sharded,
    RCCL-gathered step in one process over N devices (rm_config.ngpus contexts: one
    shard per device, a single-process communicator, grouped gather, assembly on
    device 0).  --single-process forces that path at N = 1, so one GPU runs it: the
    same JSON line, RCCL's own view of every communicator, per-phase times and the
    assembled frame equal to a plain one-GPU render."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                             "RM_BENCH_FORCE_DIST")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--single-process",
                          *args], env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = out.stdout.strip().splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and "one process (rm_config.ngpus)" in d["config"]["parallelism"]
    assert d["parity"]["assembled_equals_single_gpu"] and d["parity"]["max_abs_delta_rgba8"] == 0
    rc = d["rccl"]
    assert rc["nranks_seen"] == [1] and rc["all_communicators_match"] and rc["version"] > 0, rc
    ph = d["phases"]
    assert ph["frames"] == int(args[args.index("--steps") + 1]) and ph["max_render_mean_ms"] > 0, ph
    assert d["value"] > 0 and d["cpu_baseline"] is None


@pytest.mark.gpu
def test_bench_exits_nonzero_on_a_communicator_failure():
    """A gather that misses the communicator deadline ends bench.py with a
    diagnosis and a non-zero status (RM_ERR_COMM -> exit 3), never a hang: a
    1 ms deadline (RM_COMM_TIMEOUT_MS) cannot be met by a 4K frame."""
    env = dict(os.environ, RM_BENCH_FORCE_DIST="1", RANK="0", LOCAL_RANK="0", WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RM_COMM_TIMEOUT_MS="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "3",
                          "--steps", "3", "--warmup", "1", "--no-cpu-baseline"], env=env,
                         cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 3, (out.returncode, out.stderr[-3000:])
    assert "librm error -6" in out.stderr and out.stdout.strip() == ""
