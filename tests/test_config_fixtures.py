"""The full-size config fixtures (tests/golden/configs/, made by tests/golden/make_config_fixtures.py with the oracle in
the build container) are present and well-formed, and the cheapest one reproduces: C1 (10^6 ticks) rerun through the
oracle here hashes to the committed digest. The GPU side of these fixtures is tests/test_gpu_configs.py."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_config_fixtures as mcf  # noqa: E402

NAMES = ["c1", "c1_adv", "c2", "c3_15", "c3_25", "c4_1e5", "c4_1e6"]


@pytest.mark.parametrize("name", NAMES)
def test_fixture_is_well_formed(name):
    fx = mcf.load_fixture(name)
    assert fx["name"] == name and len(fx["sha256"]) == 64
    assert fx["rows"] >= 0 and len(fx["head"]) == min(8, fx["rows"]) and len(fx["tail"]) == min(8, fx["rows"])
    if name != "c3_25":  # the literal C3 query never matches
        assert fx["rows"] > 10_000
    else:
        assert fx["rows"] == 0


def test_digest_is_order_sensitive():
    ts = np.arange(5, dtype=np.int64)
    vals = np.arange(10, dtype=np.int64).reshape(5, 2)
    nulls = np.zeros((5, 2), np.uint8)
    d = mcf.digest_rows(ts, vals, nulls)
    assert d == mcf.digest_rows(ts.copy(), vals.copy(), nulls.copy())
    assert d != mcf.digest_rows(ts[::-1].copy(), vals[::-1].copy(), nulls)
    nulls[2, 1] = 1
    assert d != mcf.digest_rows(ts, vals, nulls)
    assert mcf.digest_rows(ts[:0], vals[:0], nulls[:0]) != d


def test_c1_fixture_reproduces(oracle_built):
    ts, vals, nulls = mcf.c1(False)
    fx = mcf.load_fixture("c1")
    assert len(ts) == fx["rows"] and mcf.digest_rows(ts, vals, nulls) == fx["sha256"]
