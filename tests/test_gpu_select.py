"""The selector beyond plain attributes (QuerySelector.processNoGroupBy :161-205): core
functions, attribute aggregators running per partition key in delivery order, having, select *. GPU against the
oracle, bit-exact, over one and several flushes (the aggregators' per-key state persists across flushes)."""
import zlib

import pytest

import synth
from oracle_rt import Oracle
from product_rt import ProductAdapter

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(synth.SELECT_APPS))
@pytest.mark.parametrize("batches", [1, 3])
def test_selector_on_gpu(name, batches, oracle_built):
    app = synth.SELECT_APPS[name]
    tr = synth.trace(3000, keys=6, seed=zlib.crc32(name.encode()) % 1000, null_rate=0.05)
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    p = ProductAdapter(app)
    try:
        got = synth.run(p, tr, batches)
    finally:
        p.close()
    assert len(ref) > 10, "workload too small"
    assert got == ref


def test_aggregators_many_keys_on_gpu(oracle_built):
    """per-key aggregator state over 2000 keys (the key-sorted post pass, state growth across flushes)"""
    app = synth.SELECT_APPS["agg_all"]
    tr = synth.trace(30_000, keys=2000, seed=3)
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    p = ProductAdapter(app)
    try:
        got = synth.run(p, tr, 4)
    finally:
        p.close()
    assert len(ref) > 1000 and got == ref


@pytest.mark.parametrize("name", sorted(synth.ABSENT_APPS))
@pytest.mark.parametrize("seed", [100, 104])
def test_absent_collisions_on_gpu(name, seed, oracle_built):
    """few keys, many equal due times: collapse, multi-pop fires, re-arms after a destroyed state"""
    app = synth.ABSENT_APPS[name]
    tr = synth.trace(3000, keys=6, seed=seed, null_rate=0.05)
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    for batches in (1, 3):
        p = ProductAdapter(app)
        try:
            got = synth.run(p, tr, batches)
        finally:
            p.close()
        assert got == ref, batches


@pytest.mark.parametrize("name", ["absent_every_20", "absent_start", "absent_mid"])
@pytest.mark.parametrize("chunk", [3, 11])
def test_send_event_arrays_on_gpu(name, chunk, oracle_built):
    """InputHandler.send(Event[]): the clock moves to the array's last timestamp before its first event"""
    app = synth.ABSENT_APPS[name]
    tr = synth.trace(2000, keys=5, seed=7, null_rate=0.02)
    o = Oracle(app)
    try:
        ref = synth.run_events(o, tr, chunk)
        per_event = synth.run(Oracle(app), tr)
    finally:
        o.close()
    assert ref != per_event, "the workload does not tell Event[] from per-event sends"
    p = ProductAdapter(app)
    try:
        got = synth.run_events(p, tr, chunk, batches=2)
    finally:
        p.close()
    assert got == ref


@pytest.mark.parametrize("name", sorted(synth.PURGE_APPS))
@pytest.mark.parametrize("batches", [1, 4])
def test_purge_on_gpu(name, batches, oracle_built):
    """@purge: idle keys' states destroyed, initPartition again at their next event (the oracle's model of the
    purge task); non-vacuous: the output differs from the same app without @purge"""
    import re
    app = synth.PURGE_APPS[name]
    tr = synth.purge_trace(6000, seed=3)
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    o2 = Oracle(re.sub(r"@purge\([^)]*\)", "", app))
    try:
        assert synth.run(o2, tr) != ref
    finally:
        o2.close()
    p = ProductAdapter(app)
    try:
        got = synth.run(p, tr, batches)
    finally:
        p.close()
    assert got == ref


@pytest.mark.parametrize("name", sorted(synth.RANGE_APPS))
@pytest.mark.parametrize("batches", [1, 3])
def test_range_partitions_on_gpu(name, batches, oracle_built):
    """range partitions: one view row per range that holds, processed in range order within the event"""
    app = synth.RANGE_APPS[name]
    tr = synth.trace(3000, keys=1, seed=21, null_rate=0.03)
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    p = ProductAdapter(app)
    try:
        got = synth.run(p, tr, batches)
    finally:
        p.close()
    assert len(ref) > 50 and got == ref
