"""Device key table (keytab.hip): device-resident batches partitioned by an int / long attribute map their key
values to dense key ids on the GPU. The same events pushed from host columns (host dictionary, itself oracle-checked
in test_gpu_parity / the golden fixtures) and from device columns must give identical results, whatever the order in
which keys first appear, across batches, with host and device pushes interleaved, and with table growth. One small
case is checked against the oracle directly. MI355X only (-m gpu)."""
import numpy as np
import pytest
import torch

import siddhi_amd as sa
from oracle_rt import Oracle
from siddhi_amd import workloads as w

pytestmark = pytest.mark.gpu

CHAIN_LONG = ("@app:playback define stream S (id long, key long, price double, volume int); "
              "partition with (key of S) begin @info(name = 'query1') "
              "from every e1=S[price>20] -> e2=S[price>e1.price] within 1 sec "
              "select e1.id as e1id, e2.id as e2id, e2.key as k insert into M; end;")
CHAIN_INT = CHAIN_LONG.replace("key long", "key int")
SEQ_LONG = ("@app:playback define stream S (id long, key long, price double, volume int); "
            "partition with (key of S) begin @info(name = 'query1') "
            "from every e1=S[price>20], e2=S[price>e1.price]<1:5>, e3=S[price<e2[last].price] "
            "select e1.id as e1id, e2[0].id as e2f, e2[last].id as e2l, e3.id as e3id insert into M; end;")


def key_values(n_keys, seed, int32=False):
    """distinct key values: large, negative, 0, and (long) Long.MIN_VALUE / MAX_VALUE"""
    rng = np.random.default_rng(seed)
    lo, hi = (-2**31, 2**31 - 1) if int32 else (-2**62, 2**62)
    v = np.unique(rng.integers(lo, hi, size=n_keys * 2, dtype=np.int64))[:n_keys - 3]
    extra = [0, -2**31, 2**31 - 1] if int32 else [0, -2**63, 2**63 - 1]
    v = np.concatenate([np.array(extra, dtype=np.int64), v])
    rng.shuffle(v)
    return v


def columns(n, n_keys, seed=3, int32=False, per_ms=4):
    c = w.c2_columns(n, keys=n_keys, seed=seed, per_ms=per_ms)
    kv = key_values(n_keys, seed, int32)
    key = kv[c["key"]]
    return {"ts": c["ts"], "id": c["id"], "key": key.astype(np.int32) if int32 else key, "price": c["price"],
            "volume": c["volume"]}


def run(app, cols, batches, sources, fused=True):
    """sources[b]: 'host' (send_columns) or 'dev' (push_device) for batch b; rows of all batches in delivery order"""
    rt = sa.SiddhiAppRuntime(app, fused=fused)
    dev = torch.device("cuda", 0)
    rows = []
    try:
        n = len(cols["ts"])
        bounds = np.linspace(0, n, batches + 1).astype(int)
        for b in range(batches):
            s, e = bounds[b], bounds[b + 1]
            part = [cols[k][s:e] for k in ("id", "key", "price", "volume")]
            if sources[b] == "host":
                rt.getInputHandler("S").send_columns(cols["ts"][s:e], part)
                rt.flush(deliver=False)
            else:
                d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in part]
                d_ts = torch.from_numpy(np.ascontiguousarray(cols["ts"][s:e])).to(dev)
                rt.push_device("S", e - s, d_ts.data_ptr(), [x.data_ptr() for x in d])
                rt.flush(deliver=False)
                torch.cuda.synchronize()
            types, ts, vals, nulls = rt.raw_outputs(0)
            rows += [(ts[i],) + tuple(v[i] for v in vals) for i in range(len(ts))]
        return rows
    finally:
        rt.shutdown()


@pytest.mark.parametrize("int32", [False, True])
@pytest.mark.parametrize("fused", [True, False])
def test_chain_device_keys_match_host_keys(int32, fused):
    cols = columns(120_000, 3_000, int32=int32)
    app = CHAIN_INT if int32 else CHAIN_LONG
    ref = run(app, cols, 4, ["host"] * 4, fused)
    got = run(app, cols, 4, ["dev"] * 4, fused)
    assert len(ref) > 1000
    assert got == ref


def test_interleaved_host_and_device_pushes():
    """keys first seen in a host batch, then in a device batch, and the other way round: one dictionary"""
    cols = columns(90_000, 5_000, seed=9)
    ref = run(CHAIN_LONG, cols, 6, ["host"] * 6)
    got = run(CHAIN_LONG, cols, 6, ["dev", "host", "dev", "dev", "host", "dev"])
    assert got == ref


def test_table_growth_many_keys():
    """300k keys: the first device batch outgrows the initial table (rebuilt and probed again)"""
    cols = columns(900_000, 300_000, seed=5, per_ms=50)
    ref = run(CHAIN_LONG, cols, 2, ["host", "host"])
    got = run(CHAIN_LONG, cols, 2, ["dev", "dev"])
    assert len(ref) > 1000
    assert got == ref


def test_generic_nfa_device_keys():
    cols = columns(60_000, 2_000, seed=13)
    ref = run(SEQ_LONG, cols, 3, ["host"] * 3)
    got = run(SEQ_LONG, cols, 3, ["dev"] * 3)
    assert len(ref) > 100
    assert got == ref


def test_device_keys_match_oracle(oracle_built):
    cols = columns(6_000, 200, seed=21)
    o = Oracle(CHAIN_LONG)
    try:
        for i in range(len(cols["ts"])):
            o.send("S", int(cols["ts"][i]), [int(cols["id"][i]), int(cols["key"][i]), float(cols["price"][i]),
                                             int(cols["volume"][i])])
        ref = [(r["ts"],) + tuple(v[1] for v in r["values"]) for r in o.outputs() if r["kind"] == "query"]
    finally:
        o.close()
    got = run(CHAIN_LONG, cols, 2, ["dev", "dev"])
    assert len(ref) > 100
    assert got == ref


# ---- float / double / bool partition keys (toString identity: -0.0 and 0.0 are two keys, every NaN one key) ----
def real_key_values(n_keys, seed, f32):
    rng = np.random.default_rng(seed)
    dt = np.float32 if f32 else np.float64
    special = np.array([0.0, -0.0, np.inf, -np.inf, 1e-40 if f32 else 5e-324, 3.4e38 if f32 else 1e300], dtype=dt)
    v = np.unique(rng.normal(0, 1e6, size=n_keys * 2).astype(dt))[: n_keys - len(special) - 2]
    v = np.concatenate([special, v]).astype(dt)
    bits = v.view(np.uint32 if f32 else np.uint64).copy()
    # two NaNs with different bit patterns: one key ("NaN") in the reference
    nan_a, nan_b = (0x7FC00000, 0xFFC00001) if f32 else (0x7FF8000000000000, 0xFFF0000000000001)
    bits = np.concatenate([bits, np.array([nan_a, nan_b], dtype=bits.dtype)])
    rng.shuffle(bits)
    return bits.view(dt)


REAL_APP = ("@app:playback define stream S (id long, key %s, price double, volume int); "
            "partition with (key of S) begin @info(name = 'query1') "
            "from every e1=S[price>20] -> e2=S[price>e1.price] within 1 sec "
            "select e1.id as e1id, e2.id as e2id insert into M; end;")


def real_columns(n, n_keys, f32, seed=17):
    c = w.c2_columns(n, keys=n_keys, seed=seed, per_ms=4)
    kv = real_key_values(n_keys, seed, f32)
    return {"ts": c["ts"], "id": c["id"], "key": kv[c["key"] % len(kv)], "price": c["price"], "volume": c["volume"]}


@pytest.mark.parametrize("kind", ["double", "float"])
@pytest.mark.parametrize("fused", [True, False])
def test_real_device_keys_match_host_keys(kind, fused):
    cols = real_columns(80_000, 2_000, kind == "float")
    app = REAL_APP % kind
    ref = run(app, cols, 3, ["host"] * 3, fused)
    got = run(app, cols, 3, ["dev", "host", "dev"], fused)
    assert len(ref) > 1000
    assert got == ref


def test_bool_device_keys_match_host_keys():
    cols = columns(40_000, 2, seed=4)
    cols["key"] = (cols["key"] != cols["key"][0]).astype(np.uint8)
    app = REAL_APP % "bool"
    ref = run(app, cols, 2, ["host"] * 2)
    got = run(app, cols, 2, ["dev"] * 2)
    assert len(ref) > 100
    assert got == ref


@pytest.mark.parametrize("kind", ["double", "float"])
def test_real_device_keys_match_oracle(kind, oracle_built):
    f32 = kind == "float"
    cols = real_columns(6_000, 60, f32, seed=23)
    app = REAL_APP % kind
    o = Oracle(app)
    try:
        for i in range(len(cols["ts"])):
            o.send("S", int(cols["ts"][i]), [int(cols["id"][i]), float(cols["key"][i]), float(cols["price"][i]),
                                             int(cols["volume"][i])])
        ref = [(r["ts"],) + tuple(v[1] for v in r["values"]) for r in o.outputs() if r["kind"] == "query"]
    finally:
        o.close()
    got = run(app, cols, 2, ["dev", "dev"])
    assert len(ref) > 100
    assert got == ref


def test_string_keys_bulk_interned_device_resident(oracle_built):
    """string partition keys through sdg_intern_many (one bulk dictionary fill per batch) and device-resident
    columns end to end: the C3 <1:5> shape with "K%d" keys vs the oracle"""
    keys = 3_000
    c = w.c3_columns(keys, per_key=40)
    app = SEQ_LONG.replace("key long", "key string")
    names = np.array(["K%d" % k for k in range(keys)])
    rt = sa.SiddhiAppRuntime(app)
    dev = torch.device("cuda", 0)
    try:
        n = len(c["ts"])
        rows = []
        for lo, hi in ((0, n // 2), (n // 2, n)):
            uniq, inv = np.unique(c["key"][lo:hi], return_inverse=True)
            enc = [s.encode() for s in names[uniq]]
            offs = np.cumsum([0] + [len(x) for x in enc]).astype(np.int64)
            ids = rt.intern_many(b"".join(enc), offs)
            d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in
                 (c["id"][lo:hi], ids[inv].view(np.int32), c["price"][lo:hi], c["volume"][lo:hi])]
            d_ts = torch.from_numpy(np.ascontiguousarray(c["ts"][lo:hi])).to(dev)
            rt.push_device("S", hi - lo, d_ts.data_ptr(), [x.data_ptr() for x in d])
            rt.flush(deliver=False)
            torch.cuda.synchronize()
            types, ts, vals, nulls = rt.raw_outputs(0)
            rows += [(ts[i],) + tuple(v[i] for v in vals) for i in range(len(ts))]
    finally:
        rt.shutdown()
    o = Oracle(app)
    try:
        for i in range(len(c["ts"])):
            o.send("S", int(c["ts"][i]), [int(c["id"][i]), str(names[c["key"][i]]), float(c["price"][i]),
                                         int(c["volume"][i])])
        ref = [(r["ts"],) + tuple(v[1] for v in r["values"]) for r in o.outputs() if r["kind"] == "query"]
    finally:
        o.close()
    assert len(ref) > 100
    assert rows == ref
