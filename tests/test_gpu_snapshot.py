"""Snapshot / restore of the device state (SiddhiAppRuntime.snapshot/restore,
core/SiddhiAppRuntimeImpl.java:677-737). Behavioural parity: a run interrupted by snapshot -> new engine -> restore
produces exactly the oracle's uninterrupted output. Covers every kind of state that outlives a flush: chain-path
carries, generic-NFA arenas (count / sequence / logical), absent-state timers (scheduler model), selector aggregators,
numeric partition-key dictionaries."""
import zlib

import pytest

import siddhi_amd as sa
import synth
from oracle_rt import Oracle
from product_rt import ProductAdapter

pytestmark = pytest.mark.gpu

CASES = {
    "chain_c2": synth.CHAIN_APPS["gt"][0],
    "count_pattern": synth.APPS["count_pattern"],
    "c3_sequence_min1": synth.APPS["c3_sequence_min1"],
    "logical_and": synth.APPS["logical_and"],
    "sequence_plus": synth.APPS["sequence_plus"],
    "absent_every_20": synth.ABSENT_APPS["absent_every_20"],
    "absent_start": synth.ABSENT_APPS["absent_start"],
    "agg_all": synth.SELECT_APPS["agg_all"],
    "numeric_keys": synth.DEFS_NUM + "partition with (k of S, k of T) begin @info(name='q') from every e1=S[price>40] "
                    "-> e2=T[price>e1.price] within 25 milliseconds select e1.id as a, e2.id as b insert into O; end;",
}


def _run(adapter, tr):
    for s, ts, row in tr:
        adapter.send(s, ts, row)
    adapter.flush()


@pytest.mark.parametrize("name", sorted(CASES))
def test_snapshot_restore_matches_uninterrupted_run(name, oracle_built):
    app = CASES[name]
    tr = synth.trace(4000, keys=7, seed=zlib.crc32(name.encode()) % 1000, null_rate=0.03)
    if name == "numeric_keys":
        tr = [(s, ts, row[:1] + [int(row[1][1:]) * 1000003] + row[2:]) for s, ts, row in tr]
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    cut = len(tr) // 2 + 17
    a = ProductAdapter(app)
    _run(a, tr[: cut // 2])  # two flushes before the snapshot
    _run(a, tr[cut // 2: cut])
    blob = a.rt.snapshot()
    first = [(r["name"], r["ts"], tuple(r["values"])) for r in a.outputs() if r["kind"] == "query"]
    a.close()
    b = ProductAdapter(app)
    try:
        b.rt.restore(blob)
        _run(b, tr[cut:])
        second = [(r["name"], r["ts"], tuple(r["values"])) for r in b.outputs() if r["kind"] == "query"]
    finally:
        b.close()
    assert len(ref) > 20
    assert first + second == ref


def test_persistence_restore_mid_pattern():
    """PersistenceTestCase.persistenceTest2 (:150-230): restore mid-pattern through a persistence store"""
    app = ("@app:name('Test') define stream Stream1 (symbol string, price float, volume int); "
           "define stream Stream2 (symbol string, price float, volume int); "
           "@info(name = 'query1') from e1=Stream1[price>20] <2:5> -> e2=Stream2[price>20] "
           "select e1[0].price as price1_0, e1[1].price as price1_1, e1[2].price as price1_2, "
           "e1[3].price as price1_3, e2.price as price2 insert into OutputStream ;")
    got = []

    class CB(sa.QueryCallback):
        def receive(self, timestamp, inEvents, removeEvents):
            got.extend(ev.data for ev in inEvents)

    store = sa.InMemoryPersistenceStore()
    m = sa.SiddhiManager()
    m.setPersistenceStore(store)
    rt = m.createSiddhiAppRuntime(app)
    rt.addCallback("query1", CB())
    s1 = rt.getInputHandler("Stream1")
    rt.start()
    s1.send(["WSO2", 25.6, 100])
    s1.send(["GOOG", 47.6, 100])
    s1.send(["GOOG", 13.7, 100])
    rt.persist()
    rt.shutdown()
    assert got == []
    rt = m.createSiddhiAppRuntime(app)
    rt.addCallback("query1", CB())
    s1, s2 = rt.getInputHandler("Stream1"), rt.getInputHandler("Stream2")
    rt.start()
    rt.restoreLastRevision()
    s2.send(["IBM", 45.7, 100])
    s1.send(["GOOG", 47.8, 100])
    s2.send(["IBM", 55.7, 100])
    rt.shutdown()
    assert len(got) == 1
    assert [None if v is None else round(v, 1) for v in got[0]] == [25.6, 47.6, None, None, 45.7]


def test_restore_rejects_a_different_app():
    a = sa.SiddhiAppRuntime(synth.APPS["count_pattern"])
    blob = a.snapshot()
    a.shutdown()
    b = sa.SiddhiAppRuntime(synth.APPS["logical_and"])
    with pytest.raises(sa.CannotRestoreSiddhiAppStateException):
        b.restore(blob)
    b.shutdown()
