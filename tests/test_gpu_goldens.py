"""librm (HIP, through the C-ABI) against the committed golden fixtures — no
oracle at test time.  Geometry bit-exact, colour within the parity bar."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(__file__), "golden")
META = json.load(open(os.path.join(HERE, "oracle_goldens.json")))


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(HERE, "oracle_goldens.npz"))


@pytest.mark.parametrize("name", sorted(META))
def test_gpu_matches_golden(rm, gpu, gold, name):
    m = META[name]
    u = rm.sweep_uniforms(m["frame"], 120, m["bounces"], m["aa"], m["shadow"])
    with rm.Renderer(m["W"], m["H"], outputs=3, counters=True) as r:
        r.dispatch(u)
        f = r.read_rgba32f()
        q = r.read_rgba8()
        cnt = r.counters()
        sc = r.sdf_counts()
    np.testing.assert_array_equal(sc, gold[name + "_counts"])
    assert cnt == m["counters"]
    assert np.abs(q.astype(int) - gold[name + "_rgba8"].astype(int)).max() <= 1
    assert np.abs(f - gold[name + "_rgba32f"]).max() <= 2e-6
