"""Engine robustness on the GPU: a flush that fails part-way through, and a restore of a corrupt snapshot.

* A flush consumes its batch even when a query fails (include/siddhi_amd.h). The queries that committed before the
  failing one hold state stamped with the batch's positions and clock, so the next flush must continue after them:
  event_seq stays monotone and `within` keeps its meaning across the failed batch.
* sdg_restore validates the whole blob before touching any state (the reference deserialises the snapshot before
  restoring, SiddhiAppRuntimeImpl.java:677-737): a truncated blob or one with trailing bytes fails with
  CannotRestoreSiddhiAppStateException and leaves the engine exactly as it was.
"""
import numpy as np
import pytest

import siddhi_amd as sa
import synth
from oracle_rt import Oracle
from product_rt import ProductAdapter

pytestmark = pytest.mark.gpu

DEF = "@app:playback define stream S (id long, sym string, price double, volume int); "
Q_WITHIN = ("@info(name='q1') from every e1=S[price>20] -> e2=S[price>e1.price] within 30 milliseconds "
            "select e1.id as a, e2.id as b insert into O1; ")
# never completes within the batch (the absent state waits 100 s): every event opens a partial with a queued timer, so a
# long enough batch overflows the 4096-slot cap of the generic NFA -- queries with timers do not spill to the host
# (tests/test_gpu_spill.py covers the ones that do), so this flush fails with SDG_ERR_CAPACITY
Q_OVERFLOW = ("define stream T2 (p double); @info(name='q2') from every e1=S[price>0] -> not T2[p>e1.price] for "
              "100000 milliseconds select e1.id as a insert into O2; ")


def _cols(n, seed, id0=0, t0=0):
    rng = np.random.default_rng(seed)
    ts = 1_000 + t0 + np.arange(n, dtype=np.int64) // 4
    price = np.round(rng.uniform(10, 30, n), 2)
    return {"ts": ts, "id": np.arange(id0, id0 + n, dtype=np.int64), "price": price,
            "volume": np.zeros(n, dtype=np.int32)}


def test_failed_flush_keeps_positions_and_clock(oracle_built):
    rt = sa.SiddhiAppRuntime(DEF + Q_WITHIN + Q_OVERFLOW)
    sym = rt.intern("IBM")
    h = rt.getInputHandler("S")
    a = _cols(6000, 1)                     # > 4096 open partials in q2: this flush fails in q2, after q1 committed
    b = _cols(400, 2, id0=6000, t0=int(a["ts"][-1] - 1000 + 1))
    for c in (a, b):
        c["sym"] = np.full(len(c["ts"]), sym, dtype=np.uint32)
    h.send_columns(a["ts"], [a["id"], a["sym"], a["price"], a["volume"]])
    with pytest.raises(sa.CapacityError):
        rt.flush(deliver=False)
    assert rt._L.sdg_pending(rt._h) == 0  # the failed batch was consumed
    h.send_columns(b["ts"], [b["id"], b["sym"], b["price"], b["volume"]])
    rt.flush(deliver=False)
    ts, vals, nulls, seq = rt.poll_arrays(0)
    rt.shutdown()
    # q1 processed both batches: its output equals the oracle's single run over all events
    o = Oracle(DEF + Q_WITHIN)
    try:
        for c in (a, b):
            for i in range(len(c["ts"])):
                o.send("S", int(c["ts"][i]), [int(c["id"][i]), "IBM", float(c["price"][i]), 0])
        ref = [(r["ts"], r["values"][0][1], r["values"][1][1]) for r in o.outputs() if r["kind"] == "query"]
    finally:
        o.close()
    got = list(zip(ts.tolist(), vals[0].tolist(), vals[1].tolist()))
    assert len(ref) > 100 and got == ref
    # positions: the second batch's records carry positions after the failed batch's 6000
    assert np.all(np.diff(seq) >= 0)
    sec = seq[vals[1] >= 6000]
    assert len(sec) > 0 and sec.min() >= 6000


@pytest.mark.parametrize("corrupt", ["truncated", "trailing"])
def test_corrupt_snapshot_leaves_engine_intact(corrupt, oracle_built):
    app = synth.APPS["c3_sequence_min1"]
    tr = synth.trace(3000, keys=7, seed=31, null_rate=0.02)
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    cut = len(tr) // 2
    a = ProductAdapter(app)
    for s, ts, row in tr[:cut]:
        a.send(s, ts, row)
    a.flush()
    blob = a.rt.snapshot()
    first = [(r["name"], r["ts"], tuple(r["values"])) for r in a.outputs() if r["kind"] == "query"]
    # feed the engine on: its state must survive the failed restore of the (now stale) blob untouched
    for s, ts, row in tr[cut: cut + 200]:
        a.send(s, ts, row)
    a.flush()
    bad = blob[: len(blob) * 2 // 3] if corrupt == "truncated" else blob + b"\x00" * 8
    with pytest.raises(sa.CannotRestoreSiddhiAppStateException):
        a.rt.restore(bad)
    for s, ts, row in tr[cut + 200:]:
        a.send(s, ts, row)
    a.flush()
    rest = [(r["name"], r["ts"], tuple(r["values"])) for r in a.outputs() if r["kind"] == "query"]
    a.close()
    assert len(ref) > 20
    assert rest[: len(first)] == first and rest == ref
