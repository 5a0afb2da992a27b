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
    # cfg3 / cfg4: pairs; cfg5 (graph-replayed 8K frames): single frames
    assert b.default_batch(3, False, False, 30) == 2
    assert b.default_batch(4, False, False, 20) == 2
    assert b.default_batch(5, False, False, 20) == 1
    # N > 1: single frames in flight, or batches of 4 on one communicator
    assert b.default_batch(3, True, False, 30) == 1
    assert b.default_batch(3, True, True, 30) == 4
