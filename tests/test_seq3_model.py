"""Pins the seq3 register model (tests/seq3_model.py, the semantics of the seq3 kernel) against the oracle: random
traces over few keys and a small price domain (ties), several quantifier ranges, filters on e1 / e2[0] / e2[last]."""
import itertools

import numpy as np
import pytest

from oracle_rt import Oracle
from seq3_model import run_key

DEFS = "@app:playback define stream S (id long, key string, price double, volume int); "


def app(lo, hi, f3="price<e2[last].price", f2="price>e1.price", within=None):
    q = "<%d:%d>" % (lo, hi) if hi >= 0 else ("+" if lo == 1 else "<%d:>" % lo)
    w = " within %d milliseconds" % within if within is not None else ""
    return (DEFS + "partition with (key of S) begin @info(name='q') from every e1=S[price>20], e2=S[%s]%s, e3=S[%s]%s "
            "select e1.id as a, e2[0].id as b, e2[last].id as c, e3.id as d insert into O; end;" % (f2, q, f3, w))


def model(tr, lo, hi, f2kind, f3kind, within=None):
    keys = {}
    tsof = {row[0]: ts for ts, row in tr}
    for i, (ts, row) in enumerate(tr):
        keys.setdefault(row[1], []).append((i, row))
    f1 = lambda y: y[2] > 20
    f2 = {"e1": lambda y, e1, l: y[2] > e1[2], "first": lambda y, e1, l: y[2] >= l[0][2]}[f2kind]
    f3 = {"last": lambda y, e1, l: y[2] < l[-1][2], "e1": lambda y, e1, l: y[2] < e1[2]}[f3kind]
    out = []
    for k, evs in keys.items():
        for pos, (e1, l2, y) in run_key(evs, f1, f2, f3, lo, hi, within, lambda r: tsof[r[0]]):
            out.append((pos, (e1[0], l2[0][0], l2[-1][0], y[0])))
    out.sort()
    return [(tr[p][0], v) for p, v in out]


def oracle(tr, text):
    o = Oracle(text)
    for ts, row in tr:
        o.send("S", ts, row)
    got = [(r["ts"], tuple(v[1] for v in r["values"])) for r in o.outputs() if r["kind"] == "query"]
    o.close()
    return got


def trace(n, keys, seed, dom):
    rng = np.random.default_rng(seed)
    ts = 1000 + np.cumsum(rng.integers(0, 3, size=n))
    return [(int(ts[i]), [i, "k%d" % rng.integers(0, keys), float(rng.choice(dom)), 0]) for i in range(n)]


F2 = {"e1": "price>e1.price", "first": "price>=e2[0].price"}
F3 = {"last": "price<e2[last].price", "e1": "price<e1.price"}


@pytest.mark.parametrize("lo,hi", [(1, 5), (2, 5), (1, 1), (1, 2), (3, 3), (1, -1), (2, -1)])
@pytest.mark.parametrize("f2kind,f3kind", [("e1", "last"), ("first", "last"), ("e1", "e1")])
def test_model_vs_oracle(lo, hi, f2kind, f3kind):
    text = app(lo, hi, F3[f3kind], F2[f2kind])
    total = 0
    for seed in range(6):
        dom = [15, 21, 22, 23, 25, 30] if seed % 2 else list(np.round(np.linspace(10, 30, 41), 1))
        tr = trace(600, keys=3 + seed, seed=seed * 7 + lo * 3 + (hi % 7), dom=dom)
        want = oracle(tr, text)
        assert model(tr, lo, hi, f2kind, f3kind) == want, (lo, hi, seed)
        total += len(want)
    if lo == 1:
        assert total > 0


@pytest.mark.parametrize("within", [0, 2, 5, 9])
@pytest.mark.parametrize("lo,hi", [(1, 5), (1, -1), (2, 3)])
def test_model_within_vs_oracle(lo, hi, within):
    text = app(lo, hi, within=within)
    total = 0
    for seed in range(5):
        tr = trace(800, keys=3 + seed, seed=seed * 11 + within, dom=[15, 21, 22, 23, 25, 30])
        want = oracle(tr, text)
        assert model(tr, lo, hi, "e1", "last", within) == want, (lo, hi, within, seed)
        total += len(want)
    if lo == 1 and within >= 2:
        assert total > 0


def test_model_exhaustive_small():
    """every price sequence of length 7 over 3 values, one key, <1:2>"""
    text = app(1, 2)
    dom = [19, 21, 23]
    rows = []
    for seq in itertools.product(dom, repeat=7):
        rows.append(seq)
    # one key per sequence: keys never interact
    tr = []
    for k, seq in enumerate(rows[:700]):
        for j, p in enumerate(seq):
            tr.append((1000 + j, [len(tr), "k%d" % k, float(p), 0]))
    tr.sort(key=lambda r: r[0])
    tr = [(ts, [i] + row[1:]) for i, (ts, row) in enumerate(tr)]
    assert model(tr, 1, 2, "e1", "last") == oracle(tr, text)
