"""A stream without a partition key inside a partition, on the GPU: the engine expands each
of its events into one view row per initialised key, ranked in getPartitionKeys() order (keyorder.h), and the
generic keyed NFA runs them. Bit-exact against the oracle (whose key order tests/test_broadcast_order.py pins against
a transliteration of the JDK 8 classes), over >= 1000 keys, in one and several flushes."""
import pytest

import synth
from oracle_rt import Oracle
from product_rt import ProductAdapter
from test_broadcast_order import APP, keysets

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(synth.BCAST_APPS))
@pytest.mark.parametrize("batches", [1, 3])
def test_broadcast_apps_vs_oracle(name, batches, oracle_built):
    app = synth.BCAST_APPS[name]
    tr = synth.trace(6000, keys=1000, seed=41, two_streams=True)
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    p = ProductAdapter(app)
    try:
        assert p.rt.query_paths() == [1]
        got = synth.run(p, tr, batches)
    finally:
        p.close()
    assert len(ref) > 100, (name, len(ref))
    assert got == ref, name


def test_broadcast_key_order_through_resizes(oracle_built):
    """the order test's trace (9 colliding keys first, then 4500 keys, re-puts, a broadcast at 11 key-set sizes)"""
    import numpy as np
    keys = keysets(0)
    rng = np.random.default_rng(10)
    rows, eid, ts, sent = [], 0, 1000, []
    stops = {5, 9, 11, 12, 13, 40, 100, 700, 1500, 3000, len(keys)}
    for i, k in enumerate(keys):
        rows.append(("S", ts, [eid, k, -1.0])); eid += 1; sent.append(k)
        if rng.random() < 0.3:
            rows.append(("S", ts, [eid, sent[int(rng.integers(0, len(sent)))], -1.0])); eid += 1
        if i + 1 in stops:
            for k2 in sent:
                rows.append(("S", ts, [eid, k2, 2.0])); eid += 1
            rows.append(("T", ts, [eid, "ignored", 0.0])); eid += 1
        ts += 1
    o = Oracle(APP)
    try:
        ref = synth.run(o, rows)
    finally:
        o.close()
    for batches in (1, 4):
        p = ProductAdapter(APP)
        try:
            got = synth.run(p, rows, batches)
        finally:
            p.close()
        assert len(ref) > 9_000 and got == ref, batches


@pytest.mark.parametrize("batches", [1, 3])
def test_broadcast_100k_keys_device_expansion(batches, oracle_built):
    """10^5 initialised keys, each broadcast event expanded into 10^5 view rows ON THE DEVICE
    (engine bcast_expand: one host placeholder per event plus each distinct key order once), bit-exact vs the oracle.
    Three T events start a partial in every key; the S events that follow complete them key by key."""
    import numpy as np
    keys = ["k%06d" % i for i in range(100_000)]
    rng = np.random.default_rng(17)
    rows, eid, ts = [], 0, 1000
    for k in keys:  # initPartition of every key (price 0: no partial of its own)
        rows.append(("S", ts, [eid, k, 0.0, 1])); eid += 1
    ts += 1
    for p in (95.0, 91.5, 93.0):
        rows.append(("T", ts, [eid, "ignored", p, 1])); eid += 1
        ts += 1
    for i in rng.permutation(len(keys))[:60_000]:
        rows.append(("S", ts, [eid, keys[i], float(np.round(rng.uniform(85, 100), 2)), 1])); eid += 1
        if eid % 1000 == 0:
            ts += 1
    app = synth.BCAST_APPS["bc_only_t"]
    o = Oracle(app)
    try:
        ref = synth.run(o, rows)
    finally:
        o.close()
    p = ProductAdapter(app)
    try:
        got = synth.run(p, rows, batches)
    finally:
        p.close()
    assert len(ref) > 50_000 and got == ref
