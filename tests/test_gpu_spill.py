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


# One device-side case (a key with thousands of open partials runs on one GPU lane until it spills: ~40 s). The other
# spill shapes -- 4 batches, the unpartitioned and non-reclaiming arenas, host-arena doubling, snapshot across a
# spilled key, the never-completing-partials case -- run on the CPU through the host build of the same nfa.h code
# (tests/test_fallbacks.py), which shares spill_keys' arena migration and KeyRunT.
def test_spilled_key_vs_oracle(oracle_built):
    tr = spill_trace(depth=4600, keys=("k0", "k1"))
    ref = oracle_rows(DEEP, tr, 1)
    p = ProductAdapter(DEEP, force_generic=True, max_partials=1024)
    try:
        _flush_all(p, tr, 1)
        got = _rows(p)
        spilled = sum(s.spilled_keys for s in p.stats)
        growths = sum(s.arena_growths for s in p.stats)
        host_rows = sum(s.host_rows for s in p.stats)
    finally:
        p.close()
    assert len(ref) > 4000 and got == ref
    assert spilled == 2  # k0 and k1 each once (then resident on the host)
    assert growths >= 2  # 1024 -> 4096 on the device first
    assert host_rows >= 2 * 4600  # both keys' rows of the flush ran on the host (sdg_stats.host_rows)
