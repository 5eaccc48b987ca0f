"""Parity at the configs' full sizes against the key-sharded oracle (tests/sharded_oracle.py): every match row of
C3 (10^6 keys x 100 events, the register sequence kernel) and C2 (10^8 events over 10^4 keys, the fused bucket
matcher -- the bench's own step) equal to the oracle's, in delivery order."""
import numpy as np
import pytest

import siddhi_amd as sa
from sharded_oracle import sharded_rows
from siddhi_amd import workloads as w

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("query", ["<1:5>", "<2:5>"])
def test_c3_full_config_vs_sharded_oracle(query, oracle_built):
    """C3 at its config size: 10^6 long keys x 100 events = 10^8 events in one flush"""
    c = w.c3_columns(1_000_000)
    app = w.C3_APP.replace("<2:5>", query)
    rt = sa.SiddhiAppRuntime(app, batch_capacity=len(c["ts"]) + 1)  # one flush (an auto-flush would deliver to
    try:                                                              # callbacks, of which there are none here)
        assert rt.query_paths() == [2]
        rt.getInputHandler("S").send_columns(c["ts"], [c["id"], c["key"], c["price"], c["volume"]])
        rt.flush(deliver=False)
        gts, gvals, gnulls, _ = rt.poll_arrays(0)
    finally:
        rt.shutdown()
    # at most one match per event: the emitting event's id (e3id, its position) orders delivery
    ots, ovals, onulls = sharded_rows(app, "S", c["ts"], [c["id"], c["key"], c["price"], c["volume"]], 4,
                                      c["key"], order=(3,))
    if query == "<1:5>":
        assert len(ots) > 10_000_000
    else:
        assert len(ots) == 0
    assert np.array_equal(gts, ots) and np.array_equal(gvals.T, ovals) and np.array_equal(gnulls.T, onulls)


def test_c2_full_step_vs_sharded_oracle(oracle_built):
    """C2's full bench step: 10^8 device-resident events over 10^4 string keys in one flush on the fused matcher"""
    import torch
    n, keys = 100_000_000, 10_000
    cols = w.c2_columns(n, keys=keys)
    syms = w.symbols(keys)
    rt = sa.SiddhiAppRuntime(w.C2_APP)
    try:
        sym_ids = np.array([rt.intern(s) for s in syms], dtype=np.uint32)
        dev = [torch.from_numpy(np.ascontiguousarray(v)).cuda() for v in
               (cols["ts"], cols["id"], sym_ids[cols["key"]].astype(np.int32), cols["price"], cols["volume"])]
        rt.push_device("StockStream", n, dev[0].data_ptr(), [d.data_ptr() for d in dev[1:]])
        rt.flush(deliver=False)
        assert rt.stats().fused == 1
        gts, gvals, gnulls, _ = rt.poll_arrays(0)
        del dev
    finally:
        rt.shutdown()
    # delivery order: by emitting event (e2id = its position), then e1 arrival (e1id)
    ots, ovals, onulls = sharded_rows(w.C2_APP, "StockStream", cols["ts"],
                                      [cols["id"], None, cols["price"], cols["volume"]], 2, cols["key"],
                                      order=(1, 0), str_col=(1, cols["key"], syms))
    assert len(ots) > 30_000_000
    assert np.array_equal(gts, ots) and np.array_equal(gvals.T, ovals) and not gnulls.any() and not onulls.any()
