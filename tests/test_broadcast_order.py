"""A stream without a partition key inside a partition (PartitionStreamReceiver.send(ComplexEvent)
:274-283): each of its events reaches every key the partition initialised, in getPartitionKeys() order. The oracle's
key order (oracle.cpp JavaCHM) against an independent transliteration of the JDK 8 classes (tests/jdk_order.py),
over key sets that grow through several resizes, re-puts of existing keys, and a bin of 9 colliding keys in a
small table (treeifyBin -> tryPresize)."""
import numpy as np
import pytest

import jdk_order
from oracle_rt import Oracle

APP = ("@app:playback define stream S (id long, key string, price double); "
       "define stream T (id long, key string, price double); "
       "partition with (key of S) begin @info(name='q') from every e1=S[price > 0] -> e2=T "
       "select e1.key as k, e2.id as t insert into O; end;")


def colliding(n, bucket_bits=4):
    """n strings whose ConcurrentHashMap bin in a 16-bin table is the same"""
    out, i = [], 0
    while len(out) < n:
        s = "c%d" % i
        if jdk_order.chm_spread(jdk_order.string_hash(s)) & ((1 << bucket_bits) - 1) == 5:
            out.append(s)
        i += 1
    return out


def keysets(seed):
    rng = np.random.default_rng(seed)
    first = colliding(9)  # the 9th put walks 8 nodes of its bin: a 16-bin table presizes
    rest = ["k%d" % i for i in rng.permutation(3000)] + ["x%05d" % i for i in range(1500)]
    return first + rest


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_broadcast_order_matches_jdk_model(seed, oracle_built):
    keys = keysets(seed)
    rng = np.random.default_rng(seed + 10)
    o = Oracle(APP)
    model = jdk_order.CHM()
    ts, eid = 1000, 0
    checks = 0
    try:
        sent, seen = [], set()
        stops = {5, 9, 11, 12, 13, 40, 100, 700, 1500, 3000, len(keys)}
        for i, k in enumerate(keys):
            o.send("S", ts, [eid, k, -1.0]); eid += 1; model.put(k); sent.append(k)
            if rng.random() < 0.3:  # a re-put of an earlier key (initPartition of a known key: walks its bin)
                k2 = sent[int(rng.integers(0, len(sent)))]
                o.send("S", ts, [eid, k2, -1.0]); eid += 1; model.put(k2)
            if i + 1 in stops:
                for k2 in sent:  # a fresh partial for every key (each a re-put, in sending order)
                    o.send("S", ts, [eid, k2, 2.0]); eid += 1; model.put(k2)
                o.send("T", ts, [eid, "ignored", 0.0])
                outs = [r for r in o.outputs() if r["kind"] == "query"]
                got = [r["values"][0][1] for r in outs if r["values"][1][1] == eid]
                want = [k for k in jdk_order.hashset_order(model)]
                # every key holds exactly one partial (its fresh S event): each key once, in the set's order
                assert got == want, (seed, i + 1)
                eid += 1
                checks += 1
            ts += 1
    finally:
        o.close()
    assert checks == len({5, 9, 11, 12, 13, 40, 100, 700, 1500, 3000, len(keys)})


def test_jdk_model_presizes_small_table():
    m = jdk_order.CHM()
    for k in colliding(9):
        m.put(k)
    assert len(m.table) == 128  # tryPresize(32): tableSizeFor(49) = 64 > sizeCtl until the table is 128


def same_hash(n):
    """n distinct strings with one String.hashCode ("Aa" and "BB" hash alike): one bin at every table size"""
    out = []
    for i in range(1 << 12):
        out.append("".join("Aa" if (i >> b) & 1 else "BB" for b in range(12)))
        if len(out) == n:
            return out
    raise AssertionError


def test_tree_bin_is_refused_not_misordered(oracle_built, emu_built):
    """a key set whose map bin the JDK turns into a tree bin (a put walking 8 nodes of a bin in a table of
    >= 64) has an iteration order neither side models; the oracle and the engine's host code (keyorder.h, through
    the emulation harness) both refuse the broadcast instead of delivering some order"""
    from emu_rt import EmuAdapter
    keys = same_hash(10)  # the 9th put presizes the 16-bin table to 128; the 10th walks 9 nodes there: a TreeBin
    tr = [("S", 1000 + i, [i, k, 2.0]) for i, k in enumerate(keys)] + [("T", 2000, [99, "x", 0.0])]
    o = Oracle(APP)
    try:
        with pytest.raises(Exception, match="tree bin"):
            for s, ts, row in tr:
                o.send(s, ts, row)
            o.outputs()
    finally:
        o.close()
    e = EmuAdapter(APP)
    try:
        with pytest.raises(Exception, match="tree bin"):
            for s, ts, row in tr:
                e.send(s, ts, row)
            e.flush()
    finally:
        e.close()
    # one key fewer (+ a few others): the presized map has no tree bin, the HashSet copy's table (16 or 32 bins)
    # doubles ONCE when the colliding bin reaches 9, and both sides deliver the same order
    for extra in range(4):
        _same_order(keys[:9] + ["z%d" % i for i in range(extra)])


def _same_order(keys):
    from emu_rt import EmuAdapter
    tr9 = [("S", 1000 + i, [i, k, 2.0]) for i, k in enumerate(keys)] + [("T", 2000, [99, "x", 0.0])]
    o = Oracle(APP)
    e = EmuAdapter(APP)
    try:
        for s, ts, row in tr9:
            o.send(s, ts, row)
            e.send(s, ts, row)
        e.flush()
        ref = [r["values"][0][1] for r in o.outputs() if r["kind"] == "query"]
        got = [r["values"][0][1] for r in e.outputs() if r["kind"] == "query"]
    finally:
        o.close()
        e.close()
    assert len(ref) == len(keys) and got == ref
