"""bench.py's issue configuration per BASELINE config (no GPU): frames per launch
and the steps they are capped by (profiles/r04_probe_batch120.txt,
profiles/r04_inflight.txt)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_cfg", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_default_batches():
    b = _bench()
    # cfg1 / cfg2: 20 frames per launch over the whole sweep, a third of the steps
    # below that, so the launches still spread over the 3 contexts
    assert b.default_batch(1, False, False, 120) == 20
    assert b.default_batch(2, False, False, 120) == 20
    assert b.default_batch(2, False, False, 20) == 7
    assert b.default_batch(1, False, False, 1) == 1
    # cfg3 / cfg4: single frames since round 6 (tools/ab_issue.sh); cfg5 (graph-
    # replayed 8K frames): single frames
    assert b.default_batch(3, False, False, 30) == 1
    assert b.default_batch(4, False, False, 20) == 1
    # a scene table's 4K frames keep pairs (profiles/r06_ab_tables.txt)
    assert b.default_batch(3, False, False, 20, table=True) == 2
    assert b.default_batch(5, False, False, 20) == 1
    # N > 1: pairs of frames per launch (round 6, tools/probe_scale.py), or batches
    # of 4 on one communicator
    assert b.default_batch(3, True, False, 30) == 2
    assert b.default_batch(3, True, True, 30) == 4


def test_run_mode_selection():
    """--gpus N > 1 without a launcher runs in this one process over
    N devices (rm_config.ngpus); a launcher's world size must equal N."""
    b = _bench()
    assert b.run_mode(1, False, 1, False) == ("single_gpu", None)
    assert b.run_mode(8, False, 1, False) == ("single_process", None)
    assert b.run_mode(1, False, 1, True) == ("single_process", None)
    assert b.run_mode(8, True, 8, False) == ("launcher", None)
    assert b.run_mode(1, True, 1, False) == ("launcher", None)
    mode, why = b.run_mode(8, True, 4, False)
    assert mode == "error" and "WORLD_SIZE=4" in why
    assert b.run_mode(2, True, 2, True)[0] == "error"
    assert b.run_mode(0, False, 1, False)[0] == "error"


def test_gpus_beyond_the_visible_devices_exits_2():
    """--gpus N in one process with fewer than N visible devices: a clear message
    and status 2, before any context is created (here: no GPU at all)."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = env.get("HIP_VISIBLE_DEVICES", "")  # (no change on a box)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--steps", "2"],
                         env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 2, (out.returncode, out.stderr[-2000:])
    assert "--gpus 64 in one process needs 64 visible devices" in out.stderr
    assert out.stdout.strip() == ""


def test_committed_pmc_entries_are_per_frame():
    """The roofline reads per-frame PMC values from profiles/ (bench.pmc_entry): every batch
    kernel it would use carries the frames per launch its summary divided by (the batched
    configurations' launches of 20 and 2 frames), and the single-frame kernels none."""
    b = _bench()
    for kernel, workload, frames in (("k_pixel_frames", "cfg1", 20), ("k_pixel_frames", "cfg2", 20),
                                     ("k_table_sample_frames", "cfg3", 2),
                                     ("k_table_sample_frames", "cfg3-spec", 2),
                                     ("k_sample<false>", "cfg3", None), ("k_sample<false>", "cfg4", None)):
        v, src = b.pmc_entry(kernel, workload)
        assert v is not None, (kernel, workload)
        assert v.get("frames_per_launch") == frames, (kernel, workload, src, v.get("frames_per_launch"))
