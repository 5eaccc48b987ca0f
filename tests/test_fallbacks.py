"""Fallbacks instead of failed flushes:
- a key that runs out of partial-match slots doubles the arenas (nfa.h migrate_key, from the batch-start state)
  and the batch reruns -- host NFA build on CPU, the engine on the GPU;
- a chain-path query that meets decreasing per-key timestamps (inside a batch or across the batch boundary) moves
  to the generic NFA, its carried partials replayed into the arenas first.
Reference semantics for out-of-order time: StreamPreStateProcessor.isExpired uses |start.ts - now| (:118-129)."""
import numpy as np
import pytest

import golden_util
import synth
from emu_rt import EmuAdapter, EmuError, lib as emu_lib, run_emu_fixture
from oracle_rt import Oracle, OracleError, run_oracle_fixture

DEEP = synth.chain_app("price>0", "price>e1.price", within="")  # no window: a descending run stays pending


def deep_trace(depth=600, tail=300, seed=3):
    """one key: `depth` strictly descending prices (every partial stays pending: `depth` deep), then a noisy tail
    that completes them from the top"""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(depth):
        out.append(("S", 1000 + i // 3, [i, "k0", float(100.0 - 0.125 * i), int(rng.integers(0, 100))]))
    for j in range(tail):
        i = depth + j
        out.append(("S", 1000 + i // 3, [i, "k0", float(np.round(rng.uniform(20, 110), 2)), int(rng.integers(0, 100))]))
    return out


def query_rows(outs):
    return [(o["name"], o["ts"], tuple(o["values"])) for o in outs if o["kind"] == "query" and not o["expired"]]


def oracle_rows(app, tr, batches=1):
    o = Oracle(app)
    try:
        return synth.run(o, tr, batches)
    finally:
        o.close()


def test_host_nfa_grows_arenas_through_every_fixture(oracle_built, emu_built):
    """every device-path fixture with 4 starting slots per key: growth (migration of lists, pools, timer queues)
    must be invisible in the results"""
    L = emu_lib()
    g0 = L.emu_sched_stat(5)
    bad, ran = [], 0
    for path in golden_util.fixture_paths():
        fx = golden_util.load(path)
        try:
            got = run_emu_fixture(fx, max_partials=4)
        except EmuError:
            continue  # not on the device path
        try:
            ref = run_oracle_fixture(fx)
        except OracleError:
            continue
        ran += 1
        if query_rows(got) != query_rows(ref):
            bad.append(fx["source"])
    assert ran > 400 and not bad, bad[:10]
    assert L.emu_sched_stat(5) > g0  # some fixtures did outgrow 4 slots


@pytest.mark.parametrize("batches", [1, 3])
def test_host_nfa_500_deep_descending_run(batches, oracle_built, emu_built):
    tr = deep_trace()
    ref = oracle_rows(DEEP, tr, batches)
    L = emu_lib()
    g0 = L.emu_sched_stat(5)
    e = EmuAdapter(DEEP, max_partials=16)
    try:
        got = synth.run(e, tr, batches)
    finally:
        e.close()
    assert len(ref) > 100 and got == ref
    assert L.emu_sched_stat(5) - g0 >= 5  # 16 -> 512 slots at least


def spill_trace(depth=6000, tail=600, seed=5, keys=("k0",), step=0.01, noise=True):
    """`depth` slowly descending prices on each key of `keys` (every partial stays pending: more than the device's
    4096 partial matches per key), a lighter key k9 alongside, then a noisy tail that completes them"""
    rng = np.random.default_rng(seed)
    out, i = [], 0
    for d in range(depth):
        for k in keys:
            out.append(("S", 1000 + i // 8, [i, k, float(100.0 - step * d), int(rng.integers(0, 100))]))
            i += 1
        if noise and d % 10 == 0:
            out.append(("S", 1000 + i // 8, [i, "k9", float(np.round(rng.uniform(20, 110), 2)), 1]))
            i += 1
    for _ in range(tail):
        k = keys[int(rng.integers(0, len(keys)))] if rng.random() < 0.8 or not noise else "k9"
        out.append(("S", 1000 + i // 8, [i, k, float(np.round(rng.uniform(20, 110), 2)), int(rng.integers(0, 100))]))
        i += 1
    return out


@pytest.mark.parametrize("batches", [1, 4])
def test_host_nfa_spills_key_past_4096_partials(batches, oracle_built, emu_built):
    """a key with 6000 pending partials outgrows the device layout's 4096: it moves to a 32-bit host arena (nfa.h
    migrate_key<int16_t> into make_layout<int32_t>) and goes on there, oracle-equal"""
    tr = spill_trace()
    ref = oracle_rows(DEEP, tr, batches)
    L = emu_lib()
    s0 = L.emu_sched_stat(7)
    e = EmuAdapter(DEEP, max_partials=1024)
    try:
        got = synth.run(e, tr, batches)
    finally:
        e.close()
    assert len(ref) > 5000 and got == ref
    assert L.emu_sched_stat(7) - s0 == 1  # k0 spilled once (and stayed on the host)


def test_host_nfa_spilled_key_doubles_its_host_arena(oracle_built, emu_built):
    """20000 pending partials: the spilled key's 32-bit arena doubles (8192 -> 16384 -> 32768 slots)"""
    tr = spill_trace(depth=20000, tail=300, seed=6, step=0.004)
    ref = oracle_rows(DEEP, tr, 2)
    e = EmuAdapter(DEEP, max_partials=4096)
    try:
        got = synth.run(e, tr, 2)
    finally:
        e.close()
    assert len(ref) > 20000 and got == ref


def out_of_order(tr, seed, start, jitter=6):
    """the rows from `start` on get their timestamps jittered: per-key decreases inside the batch and across the
    boundary with the rows before"""
    rng = np.random.default_rng(seed)
    out = list(tr[:start])
    for s, ts, row in tr[start:]:
        out.append((s, int(ts + rng.integers(-jitter, jitter + 1)), row))
    return out


@pytest.mark.gpu
def test_device_arena_growth_500_deep(oracle_built):
    from product_rt import ProductAdapter
    tr = deep_trace()
    ref = oracle_rows(DEEP, tr, 3)
    p = ProductAdapter(DEEP, force_generic=True, max_partials=16)
    try:
        bounds = np.linspace(0, len(tr), 4).astype(int)
        growths = 0
        for b in range(3):
            for s, ts, row in tr[bounds[b]:bounds[b + 1]]:
                p.send(s, ts, row)
            p.flush()
            growths += p.rt.stats().arena_growths
        got = query_rows(p.outputs())
    finally:
        p.close()
    assert len(ref) > 100 and got == ref
    assert growths >= 5


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gt", "const", "cross_col"])
@pytest.mark.parametrize("partitioned", [True, False])
def test_chain_query_falls_back_on_decreasing_timestamps(name, partitioned, oracle_built):
    from product_rt import ProductAdapter
    app = synth.CHAIN_APPS[name][0]
    if not partitioned:
        app = synth.flat(app.split("begin ", 1)[1].rsplit(" end;", 1)[0])
    tr = synth.trace(3000, keys=6, seed=17, two_streams=False)
    tr = out_of_order(tr, seed=5, start=1600)
    ref = oracle_rows(app, tr, 3)
    p = ProductAdapter(app)
    try:
        assert p.rt.query_paths() == [0]  # starts on the chain path
        bounds = np.linspace(0, len(tr), 4).astype(int)
        paths = []
        for b in range(3):
            for s, ts, row in tr[bounds[b]:bounds[b + 1]]:
                p.send(s, ts, row)
            p.flush()
            paths.append(p.rt.stats().path)
        got = query_rows(p.outputs())
    finally:
        p.close()
    assert paths[0] == 0 and paths[-1] == 1  # ordered batch on the chain path, then the generic NFA
    assert len(ref) > 50 and got == ref
