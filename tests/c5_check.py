"""C5 parity helpers (test infrastructure, also used by bench.py's C5 parity leg): the oracle restatement on a sample
of one rank's partition keys (keys are independent, so the reference's output restricted to those keys is the
oracle's output over their events alone; SURVEY.md 8(d): "Parity for C5 uses the restatement on a seeded sample of
10^4 keys"), against the GPU's match records of the same keys."""
import numpy as np

from oracle_rt import Oracle, lib
from siddhi_amd import c5
from siddhi_amd import workloads as w


def oracle_sample_rows(shard, skeys, smap, g_end):
    """(ts, e1id, e2id) of the oracle's matches over the sample keys' events of global indices [0, g_end), in the
    reference's delivery order"""
    ev = shard.sample_events(smap, len(skeys), 0, g_end)
    o = Oracle(w.C2_APP)
    try:
        L = lib()
        oid = np.array([L.orc_intern(o.h, ("S%08d" % k).encode()) for k in skeys], dtype=np.int64)
        n = len(ev["ts"])
        slots = np.empty((n, 4), dtype=np.int64)
        slots[:, 0] = ev["id"]
        slots[:, 1] = oid[ev["sym"]]
        slots[:, 2] = ev["price"].view(np.int64)
        slots[:, 3] = ev["volume"]
        strm = np.full(n, o.stream("StockStream"), dtype=np.int32)
        ts = np.ascontiguousarray(ev["ts"])
        offs = np.arange(n, dtype=np.int64) * 4
        if L.orc_send_batch(o.h, n, strm.ctypes.data, ts.ctypes.data, offs.ctypes.data, slots.ctypes.data, None) != 0:
            raise RuntimeError("oracle failed")
        ots, ovals, _ = o.query_arrays(2)
    finally:
        o.close()
    return n, np.stack([ots, ovals[:, 0], ovals[:, 1]], axis=1) if len(ots) else np.zeros((0, 3), np.int64)


def sample_records(shard, smap, ts, e1, e2):
    """the GPU records (device tensors) whose key is in the sample, as host (ts, e1id, e2id) rows"""
    sel = shard.key_of(e2, smap) >= 0
    return np.stack([ts[sel].cpu().numpy(), e1[sel].cpu().numpy(), e2[sel].cpu().numpy()], axis=1)


def delivery_order(rows):
    """rows (ts, e1id, e2id) in single-engine delivery order: by emitting event (e2 = global position), then the
    partial's pending-list position (e1 arrival)"""
    if len(rows) == 0:
        return rows
    return rows[np.lexsort((rows[:, 1], rows[:, 2]))]


__all__ = ["oracle_sample_rows", "sample_records", "delivery_order", "c5"]
