"""CPU baselines for BASELINE.md §2 (C1, C2, C3, C4): the oracle -- the reference-semantics C++ restatement, not the
JVM engine (no JVM here) -- timed on bounded samples of each config's generator, on one host core
and key-sharded over N threads (one oracle instance per shard, keys are independent; ctypes releases the GIL in
orc_send_batch). Data generation and interning are outside the timed region. One JSON line per (config, threads).

    python scripts/cpu_baselines.py [--threads 16] [--only c1,c2,c3,c4]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

from oracle_rt import Oracle, lib  # noqa: E402  (test infrastructure: the oracle is only ever the baseline here)
from siddhi_amd import workloads as w  # noqa: E402


def run_shards(app, streams, ts, stream_of_row, slots, key, threads, advance=None, strings=None):
    """rows (stream name per row, ts, [n, nattr] int64 slots) through `threads` oracles, rows of key k on shard
    k % threads; returns (events/s, matches, seconds)"""
    L = lib()
    n = len(ts)
    jobs = []
    for sh in range(threads):
        idx = np.nonzero(key % threads == sh)[0] if threads > 1 else np.arange(n)
        o = Oracle(app)
        L.orc_count_only(o.h, 1)
        sl = slots[idx].copy()
        if strings is not None:  # string attribute: dictionary ids of this oracle instance
            col, names = strings
            ids = np.array([L.orc_intern(o.h, s.encode()) for s in names], dtype=np.int64)
            sl[:, col] = ids[sl[:, col]]
        sidx = np.array([o.stream(s) for s in streams], dtype=np.int32)
        m = len(idx)
        jobs.append({"o": o, "m": m, "slots": np.ascontiguousarray(sl),
                     "offs": np.arange(m, dtype=np.int64) * slots.shape[1],
                     "strm": np.ascontiguousarray(sidx[stream_of_row[idx]]),
                     "ts": np.ascontiguousarray(ts[idx]), "rc": -1})

    def work(j):
        j["rc"] = L.orc_send_batch(j["o"].h, j["m"], j["strm"].ctypes.data, j["ts"].ctypes.data, j["offs"].ctypes.data,
                                   j["slots"].ctypes.data, None)
        if advance is not None and j["rc"] == 0:
            j["rc"] = L.orc_advance_time(j["o"].h, advance)

    ths = [threading.Thread(target=work, args=(j,)) for j in jobs]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t
    matches = sum(L.orc_output_count(j["o"].h) for j in jobs)
    for j in jobs:
        j["o"].close()
    if any(j["rc"] != 0 for j in jobs):
        raise RuntimeError("oracle failed")
    return n / dt, int(matches), dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--only", default="c1,c2,c3,c4")
    args = ap.parse_args()
    only = args.only.split(",")
    cfgs = []
    if "c1" in only:
        n = 1_000_000
        c = w.c1_columns(n)
        slots = np.stack([c["id"], np.zeros(n, np.int64), c["price"].view(np.int64), c["volume"].astype(np.int64)], 1)
        cfgs.append(("C1", "1M events (the full config), one key", w.C1_APP, ["StockStream"], c["ts"], np.zeros(n, np.int64),
                     slots, np.zeros(n, np.int64), None, (1, ["IBM"]), [1]))
    if "c2" in only:
        n = 3_000_000
        c = w.c2_columns(n)
        syms = w.symbols(10_000)
        slots = np.stack([c["id"], c["key"], c["price"].view(np.int64), c["volume"].astype(np.int64)], 1)
        cfgs.append(("C2", "first 3M of the 100M-event stream, 10k keys", w.C2_APP, ["StockStream"], c["ts"],
                     np.zeros(n, np.int64), slots, c["key"], None, (1, syms), [1, args.threads]))
    if "c3" in only:
        keys = 50_000
        c = w.c3_columns(keys)
        n = len(c["ts"])
        app = w.C3_APP.replace("<2:5>", "<1:5>")
        slots = np.stack([c["id"], c["key"], c["price"].view(np.int64), c["volume"].astype(np.int64)], 1)
        cfgs.append(("C3 <1:5>", "50k keys x 100 events (per-key stream as in the 1M-key config)", app, ["S"], c["ts"],
                     np.zeros(n, np.int64), slots, c["key"], None, None, [1, args.threads]))
    if "c4" in only:
        keys = 20_000  # the oracle's global scheduler is quadratic in the keys with queued timers on one core
        c = w.c4_columns(keys, per_tick=keys // 100)
        n = len(c["ts"])
        slots = np.stack([c["id"], c["key"], c["v"].view(np.int64)], 1)
        end = int(c["ts"][-1]) + 5000
        cfgs.append(("C4", "20k keys x 20 events, 4 streams (per-key timing as in the 1M-key config), "
                           "advance_time(T_end + 5000)", w.C4_APP, list(w.C4_STREAMS), c["ts"],
                     c["stream"].astype(np.int64), slots, c["key"], end, None, [1, args.threads]))
    for name, sample, app, streams, ts, srow, slots, key, adv, strings, thr in cfgs:
        for t in thr:
            rate, matches, dt = run_shards(app, streams, ts, srow, slots, key, t, adv, strings)
            print(json.dumps({"config": name, "sample": sample, "threads": t, "events": int(len(ts)),
                              "events_per_s": rate, "matches": matches, "seconds": dt,
                              "kind": "port (reference-semantics C++ restatement, not the JVM engine)"}), flush=True)


if __name__ == "__main__":
    main()
