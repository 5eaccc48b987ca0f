"""The register sequence kernel (seq3.hip) against the oracle: SEQUENCE `every e1=S[f1], e2=S[f2]<m:n>, e3=S[f3]` with
several quantifier ranges and filter shapes, batch splits (per-key partials carried across flushes), null scan
values, one key (unpartitioned), device-resident long keys, and against the generic keyed NFA on the same input."""
import numpy as np
import pytest

import siddhi_amd as sa
import synth
from oracle_rt import Oracle
from product_rt import ProductAdapter
from test_seq3_model import F2, F3, app as seq_app

pytestmark = pytest.mark.gpu


def run_both(app, tr, batches, seq3=True, path=None):
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    p = ProductAdapter(app, seq3=seq3)
    try:
        assert p.rt.query_paths() == [path if path is not None else 2 if seq3 else 1]
        got = synth.run(p, tr, batches)
    finally:
        p.close()
    return ref, got


def price_trace(n, keys, seed, dom, null_rate=0.0):
    rng = np.random.default_rng(seed)
    ts = 1000 + np.cumsum(rng.integers(0, 3, size=n))
    out = []
    for i in range(n):
        price = float(rng.choice(dom))
        row = [i, "k%d" % rng.integers(0, keys), None if (null_rate and rng.random() < null_rate) else price, 0]
        out.append(("S", int(ts[i]), row))
    return out


@pytest.mark.parametrize("lo,hi", [(1, 5), (2, 5), (1, 1), (1, 2), (3, 3), (1, -1)])
@pytest.mark.parametrize("f2kind,f3kind", [("e1", "last"), ("first", "last"), ("e1", "e1")])
def test_seq3_shapes_vs_oracle(lo, hi, f2kind, f3kind, oracle_built):
    app = seq_app(lo, hi, F3[f3kind], F2[f2kind])
    dom = [15, 21, 22, 23, 25, 30]
    tr = price_trace(6000, keys=11, seed=lo * 31 + hi, dom=dom)
    ref, got = run_both(app, tr, 4)
    assert got == ref
    if lo == 1:
        assert len(ref) > 50


@pytest.mark.parametrize("within", [0, 3, 8])
@pytest.mark.parametrize("lo,hi", [(1, 5), (1, -1)])
def test_seq3_within_vs_oracle(lo, hi, within, oracle_built):
    """`within T`: partials whose e1 is more than T away are expired before the event (also across flushes)"""
    app = seq_app(lo, hi, within=within)
    tr = price_trace(6000, keys=13, seed=within * 7 + lo, dom=[15, 21, 22, 23, 25, 30])
    ref, got = run_both(app, tr, 5)
    assert got == ref
    if within >= 3:
        assert len(ref) > 10


def test_seq3_ineligible_filter_runs_generic(oracle_built):
    """an arithmetic e2 filter is not a FastPred: the same shape stays on the generic keyed NFA"""
    app = seq_app(1, 5, F3["last"], "price>=e2[0].price - 5")
    tr = price_trace(4000, keys=9, seed=2, dom=[15, 21, 22, 23, 25, 30])
    ref, got = run_both(app, tr, 3, path=1)
    assert len(ref) > 20 and got == ref


@pytest.mark.parametrize("batches", [1, 3, 17])
def test_seq3_c3_min1_batches_nulls(batches, oracle_built):
    """C3 <1:5> with null prices (a null compares false), split into batches: partials live across flushes"""
    app = synth.APPS["c3_sequence_min1"]
    tr = price_trace(20_000, keys=300, seed=batches, dom=list(np.round(np.linspace(10, 30, 21), 1)), null_rate=0.05)
    ref, got = run_both(app, tr, batches)
    assert len(ref) > 200 and got == ref


def test_seq3_unpartitioned(oracle_built):
    app = ("@app:playback define stream S (id long, key string, price double, volume int); @info(name='q') "
           "from every e1=S[price>20], e2=S[price>e1.price]<1:3>, e3=S[price<e2[last].price] "
           "select e1.id as a, e2[0].id as b, e2[last].id as c, e3.id as d, e3.price as p insert into O;")
    tr = price_trace(8000, keys=1, seed=5, dom=[15, 21, 22, 23, 25, 30])
    ref, got = run_both(app, tr, 3)
    assert len(ref) > 100 and got == ref


def test_seq3_matches_generic_nfa(oracle_built):
    """the same trace through both device kernels and the oracle"""
    app = synth.APPS["c3_sequence_min1"]
    tr = synth.trace(30_000, keys=500, seed=3, two_streams=False, null_rate=0.02)
    ref, got3 = run_both(app, tr, 5, seq3=True)
    _, gotg = run_both(app, tr, 5, seq3=False)
    assert len(ref) > 100 and got3 == ref and gotg == ref


def test_seq3_device_resident_long_keys(oracle_built):
    """C3 generator columns pushed from HBM (device key table), two flushes, vs the oracle"""
    import torch
    from siddhi_amd import workloads as w
    from test_gpu_parity import oracle_batch_rows

    app = w.C3_APP.replace("<2:5>", "<1:5>")
    c = w.c3_columns(20_000)
    n = len(c["ts"])
    dev = torch.device("cuda", 0)
    rt = sa.SiddhiAppRuntime(app)
    try:
        assert rt.query_paths() == [2]
        half = n // 2
        outs = []
        for lo, hi in ((0, half), (half, n)):
            d = [torch.from_numpy(np.ascontiguousarray(c[k][lo:hi])).to(dev) for k in ("id", "key", "price", "volume")]
            d_ts = torch.from_numpy(np.ascontiguousarray(c["ts"][lo:hi])).to(dev)
            rt.push_device("S", hi - lo, d_ts.data_ptr(), [x.data_ptr() for x in d])
            rt.flush(deliver=False)
            outs.append(rt.poll_arrays(0))
            assert rt.stats().path == 2
        gts = np.concatenate([o[0] for o in outs])
        gvals = np.concatenate([o[1] for o in outs], axis=1)
    finally:
        rt.shutdown()
    ots, ovals, _ = oracle_batch_rows(app, "S", c["ts"], [c["id"], c["key"], c["price"].view(np.int64), c["volume"]], 4)
    assert len(ots) > 10_000
    assert np.array_equal(gts, ots) and np.array_equal(gvals.T, ovals)


@pytest.mark.parametrize("seq3", [True, False])
def test_event_seq_counts_other_streams(seq3):
    """event_seq of a partitioned sequence's matches is the global position of the emitting event: stream A's 100
    events pushed before B's in the same flush come first (view rows of B map to positions 100..)"""
    app = ("@app:playback define stream A (id long, key string, price double, volume int); "
           "define stream B (id long, key string, price double, volume int); "
           "partition with (key of A, key of B) begin "
           "@info(name='qa') from every e1=A[price>20] -> e2=A[price>e1.price] within 1 sec "
           "select e1.id as a, e2.id as b insert into OA; "
           "@info(name='qb') from every e1=B[price>20], e2=B[price>e1.price]<1:5>, e3=B[price<e2[last].price] "
           "select e1.id as a, e3.id as d insert into OB; end;")
    rt = sa.SiddhiAppRuntime(app, seq3=seq3)
    try:
        assert rt.query_paths() == [0, 2 if seq3 else 1]
        n = 100
        rng = np.random.default_rng(1)
        k = [rt.intern("k%d" % (i % 3)) for i in range(n)]
        for sid in ("A", "B"):
            ts = 1000 + np.arange(n, dtype=np.int64)
            rt.getInputHandler(sid).send_columns(ts, [np.arange(n, dtype=np.int64), np.array(k, np.uint32),
                                                      rng.choice([15.0, 22.0, 25.0, 28.0], n), np.zeros(n, np.int32)])
        rt.flush(deliver=False)
        _, vals, _, seq = rt.poll_arrays(1)
    finally:
        rt.shutdown()
    assert len(seq) > 5
    # the emitting event is e3 (attribute d = its id = its index within B): position = 100 + d
    assert np.array_equal(seq, n + vals[1])
