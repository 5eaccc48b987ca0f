"""Generic keyed NFA (host build of nfa.h) vs the oracle on seeded synthetic traces of every NFA construct, with
several flush batches (partials carried in the per-key arenas) and nulls."""
import zlib

import pytest

import synth
from emu_rt import EmuAdapter
from oracle_rt import Oracle


def oracle_rows(app, tr):
    o = Oracle(app)
    try:
        return synth.run(o, tr)
    finally:
        o.close()


@pytest.mark.parametrize("name", sorted(synth.APPS))
@pytest.mark.parametrize("batches", [1, 4, 40])
def test_synthetic_trace(name, batches, oracle_built, emu_built):
    """40 batches with idle records: keys go idle between batches and are rebuilt from their records"""
    import emu_rt
    app = synth.APPS[name]
    tr = synth.trace(1500, keys=4, seed=zlib.crc32(name.encode()) % 1000, null_rate=0.05 if name == "arith_nulls" else 0.0)
    ref = oracle_rows(app, tr)
    emu_rt.lib().emu_set_reclaim(1 if batches == 40 else 0)
    e = EmuAdapter(app, max_partials=256)
    try:
        got = synth.run(e, tr, batches)
    finally:
        e.close()
        emu_rt.lib().emu_set_reclaim(0)
    if name != "c3_sequence":  # the literal C3 (<2:5> in a sequence) never matches under the reference semantics
        assert len(ref) > 0, "trace produces no matches; test is vacuous"
    assert got == ref


@pytest.mark.parametrize("name", sorted(synth.BCAST_APPS))
@pytest.mark.parametrize("batches", [1, 3])
def test_broadcast_apps_on_host_nfa(name, batches, oracle_built, emu_built):
    """a stream without a partition key (synth.BCAST_APPS): the host build of nfa.h with the engine's key order
    (keyorder.h) against the oracle, as tests/test_gpu_broadcast.py runs it on the GPU"""
    from emu_rt import EmuAdapter
    from oracle_rt import Oracle
    app = synth.BCAST_APPS[name]
    tr = synth.trace(3000, keys=300, seed=41, two_streams=True)
    o = Oracle(app)
    try:
        ref = synth.run(o, tr)
    finally:
        o.close()
    e = EmuAdapter(app)
    try:
        got = synth.run(e, tr, batches)
    finally:
        e.close()
    assert len(ref) > 50 and got == ref, name
