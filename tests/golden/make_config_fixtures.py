#!/usr/bin/env python3
"""Full-size config fixtures (test infrastructure, run in the build container, never on the GPU box).

The oracle (oracle/, the C++ restatement of the reference) runs each BASELINE.json config at its full size here and
the result is committed as DATA under tests/golden/configs/: the row count, a SHA-256 digest of the rows in
delivery order, and the first / last rows for diagnostics. The -m gpu tests regenerate the same synthetic inputs
(siddhi_amd/workloads.py, deterministic splitmix64) on the box, run the product, and compare the digest of its rows
-- a row-for-row comparison without running the oracle on the GPU box.

Digest (`digest_rows`): sha256 over  b"SDGROWS1" | int64 m | int64 nv | ts int64[m] | vals int64[m][nv] (row-major,
the query's output slots: ints as int64, doubles as their IEEE bits) | nulls uint8[m][nv], little-endian.

Configs:
  c1, c1_adv   C1: 10^6 ticks, one stream, no partition (random prices seed 42 / the descending adversarial variant)
  c2           C2: the bench's full step, 10^8 events over 10^4 string keys (key-sharded oracle, 8 threads)
  c3_15, c3_25 C3: 10^6 long keys x 100 events, `<1:5>` and the literal `<2:5>` (key-sharded)
  c4_1e5       C4 at 10^5 keys x 20 events (per_tick = keys / 100), final advance_time(T_end + 5000)
  c4_1e6       C4 at its config size, 10^6 keys (single oracle: the scheduler's collapse couples every key)

Run:  python tests/golden/make_config_fixtures.py c1 c1_adv c2 c3_15 c3_25 c4_1e5 c4_1e6
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "configs")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from siddhi_amd import workloads as w  # noqa: E402


def digest_rows(ts, vals, nulls):
    """the fixtures' row digest (module docstring); vals / nulls are [m][nv]"""
    ts = np.ascontiguousarray(ts, dtype="<i8")
    vals = np.ascontiguousarray(vals, dtype="<i8")
    nulls = np.ascontiguousarray(nulls, dtype=np.uint8)
    m = len(ts)
    nv = vals.shape[1] if vals.ndim == 2 else 0
    assert vals.shape == (m, nv) and nulls.shape == (m, nv)
    h = hashlib.sha256()
    h.update(b"SDGROWS1")
    h.update(np.array([m, nv], dtype="<i8").tobytes())
    for a in (ts, vals, nulls):
        if a.size == 0:
            continue
        mv = memoryview(a.reshape(-1)).cast("B")
        step = 1 << 26
        for i in range(0, len(mv), step):
            h.update(mv[i:i + step])
    return h.hexdigest()


def fixture_path(name):
    return os.path.join(OUT, name + ".json")


def load_fixture(name):
    with open(fixture_path(name)) as f:
        return json.load(f)


def _rows_json(ts, vals, nulls, lo, hi):
    return [[int(ts[i]), [int(x) for x in vals[i]], [int(x) for x in nulls[i]]] for i in range(lo, hi)]


def write_fixture(name, config, ts, vals, nulls, seconds, extra=None):
    m = len(ts)
    d = {"name": name, "config": config, "rows": m, "sha256": digest_rows(ts, vals, nulls),
         "head": _rows_json(ts, vals, nulls, 0, min(m, 8)), "tail": _rows_json(ts, vals, nulls, max(0, m - 8), m),
         "oracle_seconds": round(seconds, 1),
         "generator": "tests/golden/make_config_fixtures.py (oracle/oracle.cpp in the build container)"}
    if extra:
        d.update(extra)
    os.makedirs(OUT, exist_ok=True)
    with open(fixture_path(name), "w") as f:
        json.dump(d, f, indent=1)
        f.write("\n")
    print("%s: %d rows, %.1f s, %s" % (name, m, seconds, d["sha256"][:16]), flush=True)


def c1(adversarial):
    from oracle_rt import Oracle, lib
    c = w.c1_columns(1_000_000, adversarial=adversarial)
    L = lib()
    o = Oracle(w.C1_APP)
    try:
        n = len(c["ts"])
        sym = L.orc_intern(o.h, b"IBM")
        slots = np.empty((n, 4), dtype=np.int64)
        slots[:, 0] = c["id"]
        slots[:, 1] = sym
        slots[:, 2] = c["price"].view(np.int64)
        slots[:, 3] = c["volume"]
        offs = np.arange(n, dtype=np.int64) * 4
        strm = np.full(n, o.stream("StockStream"), dtype=np.int32)
        tsa = np.ascontiguousarray(c["ts"])
        assert L.orc_send_batch(o.h, n, strm.ctypes.data, tsa.ctypes.data, offs.ctypes.data, slots.ctypes.data,
                                None) == 0
        return o.query_arrays(2)
    finally:
        o.close()


def c2():
    from sharded_oracle import sharded_rows
    n, keys = 100_000_000, 10_000
    cols = w.c2_columns(n, keys=keys)
    syms = w.symbols(keys)
    return sharded_rows(w.C2_APP, "StockStream", cols["ts"], [cols["id"], None, cols["price"], cols["volume"]], 2,
                        cols["key"], threads=8, order=(1, 0), str_col=(1, cols["key"], syms))


def c3(query):
    from sharded_oracle import sharded_rows
    c = w.c3_columns(1_000_000)
    app = w.C3_APP.replace("<2:5>", query)
    return sharded_rows(app, "S", c["ts"], [c["id"], c["key"], c["price"], c["volume"]], 4, c["key"], threads=8,
                        order=(3,))


def c4(keys):
    from test_c4_host import oracle_c4
    c = w.c4_columns(keys, per_tick=keys // 100)
    end = int(c["ts"][-1]) + 5000
    return oracle_c4(c, end)


JOBS = {
    "c1": ("C1 1e6 ticks, seed 42", lambda: c1(False)),
    "c1_adv": ("C1 1e6 ticks, adversarial descending prices", lambda: c1(True)),
    "c2": ("C2 full step: 1e8 events, 1e4 keys 'S%05d', seed 7, per_ms 100", c2),
    "c3_15": ("C3 1e6 long keys x 100 events, <1:5>", lambda: c3("<1:5>")),
    "c3_25": ("C3 1e6 long keys x 100 events, literal <2:5>", lambda: c3("<2:5>")),
    "c4_1e5": ("C4 1e5 keys x 20 events, per_tick 1000, advance_time(T_end + 5000)", lambda: c4(100_000)),
    "c4_1e6": ("C4 1e6 keys x 20 events, per_tick 10000, advance_time(T_end + 5000)", lambda: c4(1_000_000)),
}


def main(names):
    for name in names:
        desc, fn = JOBS[name]
        t = time.time()
        ts, vals, nulls = fn()
        write_fixture(name, desc, ts, vals, nulls, time.time() - t)


if __name__ == "__main__":
    main(sys.argv[1:] or list(JOBS))
