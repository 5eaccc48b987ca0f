"""C4 (absent + logical, partitioned, playback) at 10^4 keys through the host build of the device NFA code and
the host scheduler simulation (the engine's own code, tests/native), against the oracle. Many keys share a timer
due time, so Scheduler.onTimeChange's TreeMultimap collapse (one key per due time per clock advance, in JDK
HashMap order) delays fires and the per-key fixpoint has to reproduce it. The GPU run of the same trace is
test_gpu_parity.py::test_c4_vs_oracle."""
import numpy as np
import pytest

from siddhi_amd import workloads as w


def c4_slots(c):
    n = len(c["ts"])
    slots = np.empty((n, 3), dtype=np.int64)
    slots[:, 0] = c["id"]
    slots[:, 1] = c["key"]
    slots[:, 2] = c["v"].view(np.int64)
    return slots


def oracle_c4(c, end):
    from oracle_rt import Oracle, lib
    o = Oracle(w.C4_APP)
    try:
        L = lib()
        n = len(c["ts"])
        sidx = np.array([o.stream(s) for s in w.C4_STREAMS], dtype=np.int32)[c["stream"]]
        slots = c4_slots(c)
        offs = np.arange(n, dtype=np.int64) * 3
        tsa = np.ascontiguousarray(c["ts"])
        assert L.orc_send_batch(o.h, n, sidx.ctypes.data, tsa.ctypes.data, offs.ctypes.data, slots.ctypes.data,
                                None) == 0
        o.advance(end)
        return o.query_arrays(3)
    finally:
        o.close()


def emu_c4(c, end, batches=1):
    from emu_rt import EmuAdapter
    e = EmuAdapter(w.C4_APP)
    try:
        n = len(c["ts"])
        sidx = np.array([e.L.emu_stream_index(e.h, s.encode()) for s in w.C4_STREAMS], dtype=np.int32)[c["stream"]]
        slots = c4_slots(c)
        offs = np.arange(n, dtype=np.int64) * 3
        tsa = np.ascontiguousarray(c["ts"])
        bounds = np.linspace(0, n, batches + 1).astype(np.int64)
        for b in range(batches):
            lo, hi = bounds[b], bounds[b + 1]
            o2 = offs[lo:] - offs[lo]  # named: a temporary's buffer is freed before the call
            e.L.emu_send_batch(e.h, hi - lo, sidx[lo:].ctypes.data, tsa[lo:].ctypes.data, o2.ctypes.data,
                               slots[lo:].ctypes.data, None)
            e.flush()
        e.advance(end)
        e.flush()
        outs = [r for r in e.outputs() if r["kind"] == "query"]
        ts = np.array([r["ts"] for r in outs], dtype=np.int64)
        vals = np.array([[v[1] for v in r["values"]] for r in outs], dtype=np.int64).reshape(-1, 3)
        return ts, vals
    finally:
        e.close()


def test_c4_host_nfa_matches_oracle(oracle_built, emu_built):
    c = w.c4_columns(10_000, per_tick=100)  # 2000 ticks of 10 ms, as at 10^6 keys: timers fall due mid-run
    end = int(c["ts"][-1]) + 5000
    ots, ovals, onulls = oracle_c4(c, end)
    assert len(ots) > 1000 and not onulls.any()
    gts, gvals = emu_c4(c, end, batches=3)
    assert np.array_equal(gts, ots) and np.array_equal(gvals, ovals)


# ---- timer collisions on few keys: the host build of the device path (nfa.h + the scheduler simulation) ----
import synth as _synth  # noqa: E402


@pytest.mark.parametrize("name", sorted(_synth.ABSENT_APPS))
@pytest.mark.parametrize("seed", [100, 102, 104, 106])
def test_absent_collisions_host(name, seed, oracle_built, emu_built):
    from emu_rt import EmuAdapter
    from oracle_rt import Oracle
    app = _synth.ABSENT_APPS[name]
    tr = _synth.trace(3000, keys=6, seed=seed, null_rate=0.05)
    o = Oracle(app)
    try:
        ref = _synth.run(o, tr)
    finally:
        o.close()
    for batches in (1, 3):
        e = EmuAdapter(app)
        try:
            got = _synth.run(e, tr, batches)
        finally:
            e.close()
        assert got == ref, (name, seed, batches)
