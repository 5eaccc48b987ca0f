"""CPU check of the product's generic keyed-NFA state machine (nfa.h, host build via tests/native) against the
oracle on every golden fixture the device path accepts: same rows, same delivery order. The GPU parity tests
(test_gpu_parity.py) then run the identical code as the gfx950 kernel."""
import pytest

import golden_util
from emu_rt import EmuError, run_emu_fixture
from oracle_rt import OracleError, check_fixture, run_oracle_fixture

PATHS = golden_util.fixture_paths()


def query_rows(outs, kind="query"):
    return [(o["name"], o["ts"], tuple(o["values"])) for o in outs if o["kind"] == kind and not o["expired"]]


@pytest.fixture(params=[0, 1], ids=["arenas", "idle_records"])
def reclaim(request, emu_built):
    """1: every key that ends a run idle goes through its idle record (nfa.h to_idle / from_idle), as the engine's
    reclaiming queries do when a key's state shrinks to what the reference keeps (canDestroy)"""
    import emu_rt
    emu_rt.lib().emu_set_reclaim(request.param)
    yield request.param
    emu_rt.lib().emu_set_reclaim(0)


@pytest.mark.parametrize("path", PATHS, ids=golden_util.fixture_ids())
def test_golden_fixture_on_host_nfa(path, reclaim, oracle_built, emu_built):
    fx = golden_util.load(path)
    try:
        got = run_emu_fixture(fx)
    except EmuError as e:
        msg = str(e)
        if "arena overflow" in msg:
            raise
        pytest.skip("not on the device path: " + msg[:100])
    try:
        ref = run_oracle_fixture(fx)
    except OracleError as e:
        pytest.skip("oracle does not restate this app: " + str(e)[:100])
    assert query_rows(got) == query_rows(ref), fx["source"]
    assert not check_fixture(fx, got), fx["source"]
