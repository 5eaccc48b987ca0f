"""Spilled keys on the GPU engine: a partition key that outgrows the device arena's largest
layout (4096 partial matches) goes on on the host in a 32-bit arena (engine.cpp spill_keys, nfa.h
make_layout<int32_t>), the device skips it from then on (reclaiming queries: slot_of -3; others: KH_HOST in the key's
arena head), and its records merge with the device's in delivery order. Results must equal the oracle's; the CPU
twin of these cases is tests/test_fallbacks.py (host NFA build)."""
import numpy as np
import pytest

import synth
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


# Device-side cases (a key with thousands of open partials runs on one GPU lane until it spills: ~40 s each): one and
# four flushes (the device skipping a spilled key in later flushes), and a snapshot / restore across a spilled key
# (mark_spilled, the restored device's skip and the device arena growth before the spill run only here).
# The other shapes -- the unpartitioned and non-reclaiming arenas, host-arena doubling, the never-completing-partials
# case -- run on the CPU through the host build of the same nfa.h code (tests/test_fallbacks.py), which shares
# spill_keys' arena migration and KeyRunT.
@pytest.mark.parametrize("batches", [1, 4])
def test_spilled_key_vs_oracle(batches, oracle_built):
    tr = spill_trace(depth=4600, keys=("k0", "k1"))
    ref = oracle_rows(DEEP, tr, batches)
    p = ProductAdapter(DEEP, force_generic=True, max_partials=1024)
    try:
        _flush_all(p, tr, batches)
        got = _rows(p)
        spilled = sum(s.spilled_keys for s in p.stats)
        growths = sum(s.arena_growths for s in p.stats)
        host_rows = sum(s.host_rows for s in p.stats)
    finally:
        p.close()
    assert len(ref) > 4000 and got == ref
    assert spilled == 2  # k0 and k1 each once (then resident on the host)
    assert growths >= 2  # 1024 -> 4096 on the device first
    assert host_rows >= (2 * 4600 if batches == 1 else 1)  # the keys' rows ran on the host (sdg_stats.host_rows)


def test_spilled_key_survives_snapshot(oracle_built):
    """snapshot after the key spilled, restore into a fresh runtime, continue over two more flushes: the host arena
    travels in the snapshot and the restored device still skips the key"""
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
