"""The oracle reproduces the committed golden fixtures bit-for-bit
(tests/golden/make_goldens.py)."""
import json
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(__file__), "golden")
META = json.load(open(os.path.join(HERE, "oracle_goldens.json")))


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(HERE, "oracle_goldens.npz"))


@pytest.mark.parametrize("name", sorted(META))
def test_oracle_reproduces_golden(rm, oracle, gold, name):
    m = META[name]
    u = rm.sweep_uniforms(m["frame"], 120, m["bounces"], m["aa"], m["shadow"])
    r = oracle.render(u, m["W"], m["H"])
    np.testing.assert_array_equal(r["rgba32f"], gold[name + "_rgba32f"])
    np.testing.assert_array_equal(r["rgba8"], gold[name + "_rgba8"])
    np.testing.assert_array_equal(r["sdf_counts"], gold[name + "_counts"])
    assert r["counters"] == m["counters"]
    assert r["full_counters"] == m["full_counters"]
