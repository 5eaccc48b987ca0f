"""SiddhiQL front end + lowering checks through the compile-only C-ABI (no GPU needed)."""
import pytest

import siddhi_amd as sa
import synth
from siddhi_amd import workloads as w


def compile_only(app):
    return sa.SiddhiAppRuntime(app, compile_only=True)


def test_c1_c2_lower_to_chain_kernel():
    for app in (w.C1_APP, w.C2_APP):
        rt = compile_only(app)
        assert rt.query_paths() == [0]
        name, target, types, names = rt._queries[0]
        assert (name, target, names) == ("query1", "M", ["e1id", "e2id"])
        assert types == [sa.LONG, sa.LONG]


def test_output_types_follow_java_promotion():
    app = ("define stream S (a int, b long, f float, d double, s string); "
           "from every e1=S[a > 1] -> e2=S[f > e1.b] select e1.a + e2.b as x, e1.f * 2 as y, e2.d / e1.a as z, "
           "e1.a % 2 as m insert into O;")
    rt = compile_only(app)
    assert rt._queries[0][2] == [sa.LONG, sa.FLOAT, sa.DOUBLE, sa.INT]


@pytest.mark.parametrize("app,exc", [
    ("define stream S (a int); from every e1=S[a > 'x'] -> e2=S[a > 1] select e1.a as a insert into O;",
     sa.OperationNotSupportedException),
    ("define stream S (a int); from every e1=T[a > 1] -> e2=S[a > 1] select e1.a as a insert into O;",
     sa.SiddhiAppCreationException),
    ("define stream S (a int); from every e1=S[b > 1] -> e2=S[a > 1] select e1.a as a insert into O;",
     sa.SiddhiAppCreationException),
    ("define stream S (a int); from every e1=S[a > 1] -> e2=S[a > 1 select e1.a insert into O;",
     sa.SiddhiParserException),
])
def test_errors_map_to_reference_exceptions(app, exc):
    with pytest.raises(exc):
        compile_only(app)


def test_sequence_lowers_to_seq3_or_generic_nfa():
    """the C3 shape runs on the register sequence kernel (path 2); SDG_NO_SEQ3 / other sequences: generic NFA"""
    assert compile_only(w.C3_APP).query_paths() == [2]
    rt = sa.SiddhiAppRuntime(w.C3_APP, compile_only=True, seq3=False)
    assert rt.query_paths() == [1]
    for a in ("c3_sequence", "c3_sequence_min1"):
        assert compile_only(synth.APPS[a]).query_paths() == [2]
    for a in ("sequence_plus", "sequence_star_within", "count_pattern"):  # two streams / within / pattern: generic
        assert compile_only(synth.APPS[a]).query_paths() == [1]


def test_absent_states_lower_to_schedulers():
    """absent states (plain and inside logical) compile onto the device path: one Scheduler per absent processor,
    element 1's before element 2's (StateInputStreamParser :289-378)"""
    app = ("define stream S1 (symbol string, price float); define stream S2 (symbol string, price float); "
           "from e1=S1[price>10] -> not S2[price>e1.price] for 1 sec select e1.symbol as s insert into O;")
    assert compile_only(app).query_paths() == [1]
    app2 = ("define stream A (x int); define stream B (x int); define stream C (x int); "
            "from not A[x>1] for 1 sec and not B[x>2] for 2 sec -> e3=C select e3.x as x insert into O;")
    assert compile_only(app2).query_paths() == [1]


def test_push_needs_a_device():
    rt = compile_only(w.C1_APP)
    with pytest.raises(sa.DeviceError):
        rt.flush()


# ---- the selector: every synthetic selector app compiles for the device and runs in the oracle
import synth as _synth  # noqa: E402


@pytest.mark.parametrize("name", sorted(_synth.SELECT_APPS))
def test_selector_apps_compile_and_run_in_oracle(name, oracle_built):
    from oracle_rt import Oracle
    app = _synth.SELECT_APPS[name]
    sa.SiddhiAppRuntime(app, compile_only=True)
    o = Oracle(app)
    try:
        rows = _synth.run(o, _synth.trace(800, keys=3, seed=1, null_rate=0.05))
    finally:
        o.close()
    assert rows, name


@pytest.mark.parametrize("sel,err", [
    ("count(e1.price) as n", "count"),            # count() takes no arguments
    ("ifThenElse(e1.price, 1, 2) as x", "bool"),  # condition must be bool
    ("coalesce(e1.price, e1.id) as x", "same type"),
    ("sum(e1.key) as x", "numeric"),
])
def test_selector_validation_errors(sel, err):
    app = _synth.part("@info(name='q') from every e1=S[price>30] -> e2=T[price>e1.price] select %s insert into O;" % sel)
    with pytest.raises(Exception) as ei:
        sa.SiddhiAppRuntime(app, compile_only=True)
    assert err in str(ei.value)
