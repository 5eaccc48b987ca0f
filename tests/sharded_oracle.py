"""The oracle key-sharded over host threads, for parity at full config sizes (test infrastructure).

Partition keys are independent (PartitionStreamReceiver.java:262-272: each key's events reach only its own
PartitionInstance), so the reference's output restricted to a set of keys is the output of the same app fed only
those keys' events. Each thread runs one Oracle over the rows of its keys (ctypes drops the GIL inside
orc_send_batch); the shards' rows are merged back into one delivery order by a caller-given order key (for the
configs' queries: the id of the emitting event, which is its global position, then the ordinal's id)."""
import threading

import numpy as np

from oracle_rt import Oracle, lib


def sharded_rows(app, stream, ts, slot_cols, nv, shard_key, threads=16, order=(), str_col=None):
    """ts / slot_cols: the whole trace (one stream); shard_key: int64[n] partition key index per row; nv: output
    values per row; order: output value indices, most significant first, giving the global delivery order.
    str_col = (attribute index, key index column, symbol list) as in test_gpu_parity.oracle_batch_rows.
    Returns (ts[m], vals[m][nv], nulls[m][nv]) in delivery order."""
    L = lib()
    n = len(ts)
    shard_of = (np.asarray(shard_key) % threads).astype(np.int64)
    perm = np.argsort(shard_of, kind="stable")
    bounds = np.searchsorted(shard_of[perm], np.arange(threads + 1))
    jobs = []
    for sh in range(threads):
        idx = perm[bounds[sh]:bounds[sh + 1]]
        o = Oracle(app)
        cols = list(slot_cols)
        if str_col is not None:
            ai, kidx, syms = str_col
            ids = np.array([L.orc_intern(o.h, s.encode()) for s in syms], dtype=np.int64)
            cols[ai] = ids[np.asarray(kidx)]
        m = len(idx)
        slots = np.empty((m, len(cols)), dtype=np.int64)
        for a, c in enumerate(cols):
            slots[:, a] = np.asarray(c)[idx].astype(np.int64) if np.asarray(c).dtype != np.float64 \
                else np.asarray(c)[idx].view(np.int64)
        jobs.append({"o": o, "m": m, "slots": slots, "offs": np.arange(m, dtype=np.int64) * len(cols),
                     "strm": np.full(m, o.stream(stream), dtype=np.int32),
                     "ts": np.ascontiguousarray(np.asarray(ts)[idx]), "rc": -1})
    del perm

    def work(j):
        j["rc"] = L.orc_send_batch(j["o"].h, j["m"], j["strm"].ctypes.data, j["ts"].ctypes.data,
                                   j["offs"].ctypes.data, j["slots"].ctypes.data, None)
        j["slots"] = None

    ths = [threading.Thread(target=work, args=(j,)) for j in jobs]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    try:
        if any(j["rc"] != 0 for j in jobs):
            raise RuntimeError("oracle failed on a shard")
        parts = [j["o"].query_arrays(nv) for j in jobs]
    finally:
        for j in jobs:
            j["o"].close()
    ots = np.concatenate([p[0] for p in parts])
    ovals = np.concatenate([p[1] for p in parts])
    onulls = np.concatenate([p[2] for p in parts])
    if order:
        o = np.lexsort(tuple(ovals[:, c] for c in reversed(order)))
        ots, ovals, onulls = ots[o], ovals[o], onulls[o]
    return ots, ovals, onulls
