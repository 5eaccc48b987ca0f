"""Spilled keys on the GPU engine: a partition key that outgrows the device arena's largest
layout (4096 partial matches) goes on on the host in a 32-bit arena (engine.cpp spill_keys, nfa.h
make_layout<int32_t>), the device skips it from then on (reclaiming queries: slot_of -3; others: KH_HOST in the key's
arena head), and its records merge with the device's in delivery order. Results must equal the oracle's; the CPU
twin of these cases is tests/test_fallbacks.py (host NFA build)."""
import numpy as np
import pytest

import synth
from oracle_rt import Oracle
from product_rt import ProductAdapter
from test_fallbacks import DEEP, oracle_rows, spill_trace

pytestmark = pytest.mark.gpu

# the same pattern without a partition (one key: the non-reclaiming arena path)
DEEP_UNPART = ("@app:playback " + synth.DEFS +
               "@info(name='q') from every e1=S[price>0] -> e2=S[price>e1.price] select e1.id as a, e2.id as b "
               "insert into O;")


def _flush_all(p, tr, batches):
    bounds = np.linspace(0, len(tr), batches + 1).astype(int)
    for b in range(batches):
        for s, ts, row in tr[bounds[b]:bounds[b + 1]]:
            p.send(s, ts, row)
        p.flush()


def _rows(p):
    return [(o["name"], o["ts"], tuple(o["values"])) for o in p.outputs() if o["kind"] == "query" and not o["expired"]]


# (each case runs a key with thousands of open partials on one GPU lane until it spills: ~40 s)
@pytest.mark.parametrize("app_name,batches", [("partitioned", 1), ("partitioned", 4), ("unpartitioned", 1),
                                              ("no_reclaim", 4)])
def test_spilled_key_vs_oracle(app_name, batches, oracle_built, monkeypatch):
    app = DEEP_UNPART if app_name == "unpartitioned" else DEEP
    if app_name == "no_reclaim":
        monkeypatch.setenv("SDG_NO_RECLAIM", "1")
    # (unpartitioned: one descending run, no noise key -- its rows would complete the run's partials)
    tr = (spill_trace(depth=4600, keys=("k0",), noise=False) if app_name == "unpartitioned"
          else spill_trace(depth=4600, keys=("k0", "k1")))
    ref = oracle_rows(app, tr, batches)
    p = ProductAdapter(app, force_generic=True, max_partials=1024)
    try:
        _flush_all(p, tr, batches)
        got = _rows(p)
        spilled = sum(s.spilled_keys for s in p.stats)
        growths = sum(s.arena_growths for s in p.stats)
    finally:
        p.close()
    assert len(ref) > 4000 and got == ref
    assert spilled == (1 if app_name == "unpartitioned" else 2)  # k0 and k1 each once (then resident on the host)
    assert growths >= 2  # 1024 -> 4096 on the device first


def test_spilled_key_doubles_host_arena(oracle_built):
    tr = spill_trace(depth=9000, tail=300, seed=6, step=0.008)  # 8192 host slots -> 16384
    ref = oracle_rows(DEEP, tr, 2)
    p = ProductAdapter(DEEP, force_generic=True, max_partials=4096)
    try:
        _flush_all(p, tr, 2)
        got = _rows(p)
    finally:
        p.close()
    assert len(ref) > 9000 and got == ref


def test_spilled_key_survives_snapshot(oracle_built):
    """snapshot after the key spilled, restore into a fresh runtime, continue: the host arena travels in the
    snapshot and the restored device still skips the key"""
    tr = spill_trace(depth=4600, keys=("k0",), seed=8)
    ref = oracle_rows(DEEP, tr, 1)
    cut = int(len(tr) * 0.9)  # inside the tail: k0 has spilled with thousands of partials pending
    a = ProductAdapter(DEEP, force_generic=True, max_partials=4096)
    try:
        _flush_all(a, tr[:cut], 1)
        assert sum(s.spilled_keys for s in a.stats) == 1
        snap = a.rt.snapshot()
        first = _rows(a)
    finally:
        a.close()
    b = ProductAdapter(DEEP, force_generic=True, max_partials=4096)
    try:
        b.rt.restore(snap)
        _flush_all(b, tr[cut:], 2)
        second = _rows(b)
    finally:
        b.close()
    assert len(ref) > 4000 and first + second == ref


def test_never_completing_partials_spill_instead_of_failing(oracle_built):
    """the old capacity failure case (test_gpu_robust's Q_OVERFLOW: > 4096 open partials): now it spills"""
    app = ("@app:playback " + synth.DEFS + "@info(name='q') from every e1=S[price>0] -> e2=S[price<0] -> "
           "e3=S[price<0] select e1.id as a insert into O; @info(name='q1') from every e1=S[price>20] -> "
           "e2=S[price>e1.price] within 30 milliseconds select e1.id as a, e2.id as b insert into O1;")
    rng = np.random.default_rng(1)
    tr = [("S", 1000 + i // 4, [i, "IBM", float(np.round(rng.uniform(10, 30), 2)), 0]) for i in range(4400)]
    o = Oracle(app)
    try:
        ref = synth.run(o, tr, 2)
    finally:
        o.close()
    p = ProductAdapter(app, force_generic=True)
    try:
        got = synth.run(p, tr, 2)
        spilled = sum(s.spilled_keys for s in p.stats)
    finally:
        p.close()
    assert len(ref) > 100 and got == ref
    assert spilled == 1
