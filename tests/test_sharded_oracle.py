"""The key-sharded oracle (tests/sharded_oracle.py, used for full-size GPU parity) equals the single oracle run on
the same trace: C3 and C2 generators at small sizes."""
import numpy as np

from sharded_oracle import sharded_rows
from siddhi_amd import workloads as w
from test_gpu_parity import oracle_batch_rows


def test_sharded_c3_equals_single(oracle_built):
    c = w.c3_columns(3_000)
    app = w.C3_APP.replace("<2:5>", "<1:5>")
    cols = [c["id"], c["key"], c["price"], c["volume"]]
    ref = oracle_batch_rows(app, "S", c["ts"], [c["id"], c["key"], c["price"].view(np.int64), c["volume"]], 4)
    got = sharded_rows(app, "S", c["ts"], cols, 4, c["key"], threads=5, order=(3,))
    assert len(ref[0]) > 1000
    assert all(np.array_equal(a, b) for a, b in zip(ref, got))


def test_sharded_c2_equals_single(oracle_built):
    keys = 500
    cols = w.c2_columns(300_000, keys=keys, per_ms=20)
    syms = w.symbols(keys)
    ref = oracle_batch_rows(w.C2_APP, "StockStream", cols["ts"],
                            [cols["id"], None, cols["price"].view(np.int64), cols["volume"]], 2,
                            str_col=(1, cols["key"], syms))
    got = sharded_rows(w.C2_APP, "StockStream", cols["ts"], [cols["id"], None, cols["price"], cols["volume"]], 2,
                       cols["key"], threads=7, order=(1, 0), str_col=(1, cols["key"], syms))
    assert len(ref[0]) > 10_000
    assert all(np.array_equal(a, b) for a, b in zip(ref, got))
