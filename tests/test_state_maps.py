"""Snapshot state maps, CPU side: the oracle's StreamPreState dump (orc_state_dump) pinned on a hand-checked history;
the engine's decoder (sdg_snapshot_states) refusing what is not a snapshot of its app; and snapshots the GPU engine
wrote (tests/golden/state_maps/) decoded here without a device, equal to the oracle's maps. The live engine-vs-oracle
comparison runs on the GPU (test_gpu_state_maps.py)."""
import os

import pytest

import siddhi_amd as sa
import state_fixture_cases
import synth
from oracle_rt import Oracle
from state_maps_util import check_maps

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "state_maps")

CHAIN = synth.part_s("@info(name='q') from every e1=S[price>20] -> e2=S[price>e1.price] "
                     "select e1.id as a, e2.id as b insert into O;")
# prices per event: ids 0..6, keys MSFT (even ids) / IBM (odd ids)
PRICES = [25.0, 21.0, 30.0, 10.0, 22.0, 21.5, 25.0]


def _history():
    return [("S", 1000 + i, [i, "IBM" if i % 2 else "MSFT", PRICES[i], 0]) for i in range(7)]


def test_oracle_state_dump_pins_the_reference_lists(oracle_built):
    """StreamPreStateProcessor: a partial enters the next processor's NewAndEvery list (addState) and moves to
    Pending at the start of that key's next event (updateState); `every` re-seeds the start state with the
    timestamp of the event that matched it; a completed partial leaves both lists."""
    o = Oracle(CHAIN)
    try:
        synth.run(o, _history(), 1)
        doc = o.state_dump()
    finally:
        o.close()
    (q,) = doc["queries"]
    assert q["name"] == "q"
    st = q["states"]
    assert sorted(st) == ["IBM", "MSFT"]
    msft = st["MSFT"]
    # MSFT: 25 (e1) -> 30 completes it and starts a partial -> 22 (e1, no completion: 22 < 30) -> 25 completes
    # the 22 partial (25 > 22) and starts a new one; the 30 partial stays pending
    assert msft["0"]["Initialized"] is True and msft["0"]["PendingStateEventList"] == []
    assert [s["ts"] for s in msft["0"]["NewAndEveryStateEventList"]] == [1006]
    assert [s["events"][0][0]["data"][0] for s in msft["1"]["PendingStateEventList"]] == [2]
    assert [s["events"][0][0]["data"][0] for s in msft["1"]["NewAndEveryStateEventList"]] == [6]
    assert msft["1"]["Initialized"] is False and msft["1"]["FirstEvent"] is None
    ibm = st["IBM"]
    assert [s["events"][0][0]["data"] for s in ibm["1"]["NewAndEveryStateEventList"]] == [[5, "IBM", 21.5, 0]]
    assert ibm["1"]["PendingStateEventList"] == []


def test_oracle_state_dump_count_and_absent_fields(oracle_built):
    o = Oracle(synth.APPS["count_pattern"])
    try:
        synth.run(o, synth.trace(200, keys=3, seed=1), 1)
        doc = o.state_dump()
    finally:
        o.close()
    states = doc["queries"][0]["states"]
    assert states and all("SuccessCondition" in m["0"] and "StartStateReset" in m["0"] for m in states.values())
    o = Oracle(synth.ABSENT_APPS["absent_every_20"])
    try:
        synth.run(o, synth.trace(200, keys=3, seed=1), 1)
        doc = o.state_dump()
    finally:
        o.close()
    absent = [m["1"] for m in doc["queries"][0]["states"].values() if "1" in m]
    assert absent and all("LastScheduledTime" in m and "IsActive" in m for m in absent)


def test_engine_decoder_refuses_foreign_bytes():
    rt = sa.SiddhiAppRuntime(CHAIN, compile_only=True)
    with pytest.raises(Exception, match="not an engine snapshot"):
        rt.snapshot_states(b"\0" * 64)
    with pytest.raises(Exception, match="truncated|not an engine snapshot"):
        rt.snapshot_states(b"")


def test_engine_decoder_refuses_format_1_snapshots():
    """blobs of the earlier layout (magic SSDGSNP1, no spilled-key / partition-order sections) get a version error,
    not a misleading truncation error"""
    rt = sa.SiddhiAppRuntime(CHAIN, compile_only=True)
    with open(os.path.join(GOLD, "chain_gt.snap"), "rb") as f:
        blob = bytearray(f.read())
    assert bytes(blob[:8]) == b"SSDGSNP2"
    blob[:8] = b"SSDGSNP1"
    with pytest.raises(Exception, match="format 1"):
        rt.snapshot_states(bytes(blob))


@pytest.mark.parametrize("name", sorted(state_fixture_cases.CASES))
def test_committed_snapshot_decodes_to_the_oracle_maps(name, oracle_built):
    """snapshots the GPU engine wrote (scripts/make_state_fixtures.py), decoded here by a compile-only engine of
    the same app -- no device -- equal the oracle's maps after the same seeded history"""
    app, tr, batches, generic = state_fixture_cases.CASES[name]
    with open(os.path.join(GOLD, name + ".snap"), "rb") as f:
        blob = f.read()
    got = sa.SiddhiAppRuntime(app, compile_only=True, force_generic=generic).snapshot_states(blob)
    o = Oracle(app)
    try:
        state_fixture_cases.feed(o, tr, batches)
        ref = {q["name"]: q["states"] for q in o.state_dump()["queries"]}
    finally:
        o.close()
    assert check_maps(ref, got, "arena" if generic else "chain") > 0
