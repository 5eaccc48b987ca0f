"""Snapshot state maps on the GPU engine (VERDICT r3 missing item 7): a snapshot taken between flushes, decoded by
sdg_snapshot_states into the reference's StreamPreState.snapshot() maps (StreamPreStateProcessor.java:450-469),
equals the oracle's maps after the same history (orc_state_dump) -- per query, partition key and processor: the
Pending and NewAndEvery lists with every StateEvent's timestamp, type and bound events (the attributes the query
reads), Initialized / Started, and the Count / Absent / AbsentLogical fields. Generic-NFA queries ("arena" form)
match exactly; chain queries ("chain" form) after the merge the next event's updateState() performs (both sides
normalised the same way, see DESIGN.md "Snapshot state maps")."""
import pytest

import synth
from oracle_rt import Oracle
from product_rt import ProductAdapter
from state_maps_util import check_maps, merge_lists as _merge_lists

pytestmark = pytest.mark.gpu


def _compare(app, tr, cut_batches, total_batches=None, force_generic=True, expect_form="arena", **kw):
    o = Oracle(app)
    p = ProductAdapter(app, force_generic=force_generic, **kw)
    try:
        synth.run(o, tr, cut_batches)
        synth.run(p, tr, cut_batches)
        ref = {q["name"]: q["states"] for q in o.state_dump()["queries"]}
        got = p.rt.snapshot_states()
    finally:
        p.close()
        o.close()
    return check_maps(ref, got, expect_form)


GENERIC = ["c3_sequence", "three_state_within", "non_every", "every_group", "count_pattern", "count_zero_min",
           "logical_and", "logical_or", "sequence_plus", "sequence_star_within", "arith_nulls"]


@pytest.mark.parametrize("name", GENERIC)
def test_generic_state_maps_equal_oracle(name):
    tr = synth.trace(900, keys=5, seed=3, null_rate=0.03 if name == "arith_nulls" else 0.0)
    if name == "count_zero_min":
        tr = tr[:60]  # without `every` a key's pattern is spent after its first match: snapshot before that
    elif name == "non_every":  # one partial waiting for e2 (T 10.0 does not beat e1's 60.0)
        tr = [("S", 1000, [0, "k0", 60.0, 1]), ("T", 1001, [1, "k0", 10.0, 2]), ("S", 1002, [2, "k1", 70.0, 3])]
    n = _compare(synth.APPS[name], tr, 3)
    assert n > 0


@pytest.mark.parametrize("name", ["absent_every_20", "absent_and", "absent_mid", "absent_start"])
def test_absent_state_maps_equal_oracle(name):
    tr = synth.trace(700, keys=3, seed=4)
    assert _compare(synth.ABSENT_APPS[name], tr, 2) > 0


def test_state_maps_without_reclaim(monkeypatch):
    monkeypatch.setenv("SDG_NO_RECLAIM", "1")
    assert _compare(synth.APPS["count_pattern"], synth.trace(900, keys=5, seed=5), 2) > 0


def test_state_maps_unpartitioned():
    app = synth.flat("@info(name='q') from every e1=S[price>60] -> e2=T[price>e1.price] -> e3=S[price<e1.price] "
                     "select e1.id as a, e2.id as b, e3.id as c insert into O;")
    assert _compare(app, synth.trace(600, keys=5, seed=6), 2) > 0


@pytest.mark.parametrize("name", ["gt", "lt", "int_gt_nowithin", "const"])
def test_chain_state_maps_equal_oracle(name):
    app, _ = synth.CHAIN_APPS[name]
    tr = synth.descending_trace(1200, keys=4, seed=7, run=40)
    assert _compare(app, tr, 2, force_generic=False, expect_form="chain") > 0


def test_chain_and_arena_forms_agree():
    """the same history on the fused path and on the arenas: the chain form is the arena form merged"""
    app, _ = synth.CHAIN_APPS["int_gt_nowithin"]
    tr = synth.descending_trace(800, keys=3, seed=8, run=30)
    pa = ProductAdapter(app, force_generic=True)
    pc = ProductAdapter(app)
    try:
        synth.run(pa, tr, 2)
        synth.run(pc, tr, 2)
        a = pa.rt.snapshot_states()["q"]
        c = pc.rt.snapshot_states()["q"]
    finally:
        pa.close()
        pc.close()
    assert a["form"] == "arena" and c["form"] == "chain"
    assert _merge_lists(a["states"]) == _merge_lists(c["states"])


def test_restored_engine_decodes_the_same_maps():
    app = synth.APPS["logical_and"]
    tr = synth.trace(600, keys=4, seed=9)
    p = ProductAdapter(app, force_generic=True)
    try:
        synth.run(p, tr, 2)
        blob = p.rt.snapshot()
        first = p.rt.snapshot_states(blob)
    finally:
        p.close()
    q = ProductAdapter(app, force_generic=True)
    try:
        q.rt.restore(blob)
        again = q.rt.snapshot_states()
    finally:
        q.close()
    assert first == again and first["q"]["states"]


def test_spilled_key_state_maps():
    """a key past the device arena's 4096 partials lives in a host arena with 32-bit indices: decoded the same"""
    from test_fallbacks import DEEP, spill_trace
    tr = spill_trace(depth=4600, keys=("k0",), seed=8)
    tr = tr[:int(len(tr) * 0.85)]  # k0 holds 4374 pending partials here (past the 4096 of the device arena)
    o = Oracle(DEEP)
    p = ProductAdapter(DEEP, force_generic=True, max_partials=4096)
    try:
        synth.run(o, tr, 1)
        synth.run(p, tr, 1)
        assert sum(s.spilled_keys for s in p.stats) == 1
        ref = {q["name"]: q["states"] for q in o.state_dump()["queries"]}
        got = p.rt.snapshot_states()
    finally:
        p.close()
        o.close()
    assert check_maps(ref, got, "arena") > 4000


def test_seq3_query_state_maps_are_refused_not_guessed():
    """the register sequence kernel keeps e2[0] / e2[last] of a count chain only, so its state cannot be
    decoded into CountPreStateProcessor's maps (CountPreStateProcessor.java:206-219): sdg_snapshot_states refuses
    with OperationNotSupportedException; the same app on the arenas (seq3=False) decodes"""
    import numpy as np
    import siddhi_amd as sa
    from siddhi_amd import workloads as w
    cols = w.c3_columns(50, per_key=20)
    for seq3 in (True, False):
        rt = sa.SiddhiAppRuntime(w.C3_APP, seq3=seq3)
        try:
            rt.getInputHandler("S").send_columns(cols["ts"], [cols["id"], cols["key"], cols["price"],
                                                              cols["volume"]])
            rt.flush(deliver=False)
            if seq3:
                assert rt.stats().path == 2  # the register kernel ran
                with pytest.raises(sa.OperationNotSupportedException, match="register sequence kernel"):
                    rt.snapshot_states()
            else:
                maps = rt.snapshot_states()
                assert maps["query1"]["form"] == "arena" and len(maps["query1"]["states"]) > 0
        finally:
            rt.shutdown()
    assert np.all(np.diff(cols["ts"]) >= 0)
