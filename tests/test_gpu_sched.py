"""The scheduler's exact pass and host replay against the oracle.

The default flush skips the exact pass whenever the device reruns reproduce the optimistic pass (SchedSim::confirm),
so at test sizes neither the exact pass nor the host replay (KeyRun) would run. Two test flags force them:
SDG_SCHED_EXACT runs the exact pass after every rerun; SDG_SCHED_HOST skips the optimistic pass and the device
rerun, so the exact pass sees the ideal-order device run and every key the collapse reorders is replayed on the
host from its batch-start state. Either way the rows must equal the oracle's (Scheduler.java:71-103, 171-209)."""
import numpy as np
import pytest

import synth
from oracle_rt import Oracle
from product_rt import ProductAdapter
from siddhi_amd import workloads as w
from test_c4_host import oracle_c4
from test_gpu_parity import product_c4

pytestmark = pytest.mark.gpu


# (10^5 keys through both branches: tests/test_gpu_configs.py, against the container-made C4 fixture)
@pytest.mark.parametrize("keys,mode", [(10_000, "exact"), (10_000, "host"), (30_000, "host")])
def test_c4_forced_scheduler_branch_vs_oracle(keys, mode, oracle_built):
    c = w.c4_columns(keys, per_tick=keys // 100)
    end = int(c["ts"][-1]) + 5000
    ots, ovals, onulls = oracle_c4(c, end)
    kw = {"sched_exact": True} if mode == "exact" else {"sched_host": True}
    gts, gvals, gnulls, stats = product_c4(c, end, **kw)
    exact = sum(s.sched_exact_passes for s in stats)
    host = sum(s.sched_host_keys for s in stats)
    rerun = sum(s.sched_rerun_keys for s in stats)
    print("C4 %d keys, %s: exact passes %d, host replays %d, device reruns %d" % (keys, mode, exact, host, rerun))
    assert len(ots) > 1000
    assert exact > 0
    if mode == "host":
        assert host > 100 and rerun == 0  # every reordered key went through KeyRun
    assert np.array_equal(gts, ots) and np.array_equal(gvals.T, ovals) and not gnulls.any()


@pytest.mark.parametrize("mode", ["exact", "host"])
def test_absent_collisions_forced_scheduler_branch(mode, oracle_built):
    """few keys, many equal due times (synth.ABSENT_APPS), every app x {1, 3} batches through the forced branch"""
    kw = {"sched_exact": True} if mode == "exact" else {"sched_host": True}
    exact = host = 0
    for name in sorted(synth.ABSENT_APPS):
        app = synth.ABSENT_APPS[name]
        tr = synth.trace(3000, keys=6, seed=100, null_rate=0.05)
        o = Oracle(app)
        try:
            ref = synth.run(o, tr)
        finally:
            o.close()
        for batches in (1, 3):
            p = ProductAdapter(app, **kw)
            try:
                got = synth.run(p, tr, batches)
                exact += sum(s.sched_exact_passes for s in p.stats)
                host += sum(s.sched_host_keys for s in p.stats)
            finally:
                p.close()
            assert got == ref, (name, batches)
    print("%s: exact passes %d, host replays %d" % (mode, exact, host))
    assert exact > 0
    if mode == "host":
        assert host > 0
