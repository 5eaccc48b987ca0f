"""Key-hash sharding of a partitioned query across GPUs.

One process per GPU. Rank r owns the partition keys whose hash is r mod N; keys are independent in the NFA step
(no cross-key state, PartitionRuntimeImpl.java:346-366), so each rank runs the whole query on its shard with no
data-path collective. The reference's single delivery order is recovered by merging the ranks' match streams on
(global sequence number of the emitting event, emission ordinal).
"""
import heapq

import numpy as np

_FNV_OFF = 0xcbf29ce484222325
_FNV_PRIME = 0x100000001b3


def key_hash(key):
    """64-bit FNV-1a of the key's toString (ValuePartitionExecutor.java:34-40 uses the toString as the key)"""
    h = _FNV_OFF
    for b in str(key).encode():
        h = ((h ^ b) * _FNV_PRIME) & 0xFFFFFFFFFFFFFFFF
    return h


def owner(key, world):
    return key_hash(key) % world


def route(keys, world):
    """rank of each event, for an array/list of partition key values"""
    cache = {}
    out = np.empty(len(keys), dtype=np.int32)
    for i, k in enumerate(keys):
        r = cache.get(k)
        if r is None:
            r = cache[k] = owner(k, world)
        out[i] = r
    return out


def merge(parts):
    """parts: per rank, lists of (global_seq, ordinal, record) already in local order -> one ordered list"""
    return [rec for _, _, rec in heapq.merge(*parts, key=lambda t: (t[0], t[1]))]


def lexsort(keys):
    """permutation ordering records by `keys` (torch tensors, most significant first), stable"""
    import torch
    order = torch.arange(keys[0].numel(), device=keys[0].device)
    for k in reversed(keys):
        order = order[torch.argsort(k[order], stable=True)]
    return order


def merge_runs(runs, key):
    """G-way merge of sorted runs (dicts of torch tensors, records along the last dim) by their 1-D `key` column:
    record i of run r lands at  i + sum_{r' < r} #{x in run r' : x <= v} + sum_{r' > r} #{x in run r' : x < v}
    (binary searches into the other runs), so equal keys keep run order, then their order inside the run. Linear
    in the records (times log of a run), no re-sort of the concatenation."""
    import torch
    runs = [r for r in runs if r[key].numel() > 0]
    if not runs:
        return None
    if len(runs) == 1:
        return runs[0]
    dev = runs[0][key].device
    total = sum(int(r[key].numel()) for r in runs)
    out = {k: torch.empty(list(v.shape[:-1]) + [total], dtype=v.dtype, device=dev) for k, v in runs[0].items()}
    for r, run in enumerate(runs):
        v = run[key]
        pos = torch.arange(v.numel(), device=dev, dtype=torch.int64)
        for r2, other in enumerate(runs):
            if r2 != r:
                pos += torch.searchsorted(other[key], v, right=r2 < r)
        for k, col in run.items():
            out[k][..., pos] = col
    return out


def ordered_gather(dist, rank, world, cols, key_names):
    """Ordered result gather: `cols` maps names to this rank's record tensors (1-D [n], or 2-D
    [m, n] with records along the last dim) on the communication device. Every rank sorts its records by
    `key_names` on its device, the run lengths are all-gathered, and each rank's sorted run goes to rank 0
    point-to-point (send/recv: RCCL over xGMI with the nccl backend, gloo on CPU), where the G runs are merged on the
    first key (merge_runs: records of different ranks with equal first keys keep rank order, which is the
    tie-break every caller's key implies -- either the first key is unique across ranks, e.g. the global position of
    the emitting event, or the rank is the next key). Returns the merged dict on rank 0, None elsewhere."""
    import torch
    names = sorted(cols)
    ref = cols[key_names[0]]
    order = lexsort([cols[k] for k in key_names])
    mine = {k: cols[k][..., order].contiguous() for k in names}
    n = torch.tensor([ref.numel()], dtype=torch.int64, device=ref.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    if rank != 0:
        if counts[rank] > 0:
            for k in names:
                dist.send(mine[k], dst=0)
        return None
    runs = [mine]
    for r in range(1, world):
        if counts[r] == 0:
            continue
        run = {}
        for k in names:
            shape = list(cols[k].shape[:-1]) + [counts[r]]
            run[k] = torch.empty(shape, dtype=cols[k].dtype, device=ref.device)
            dist.recv(run[k], src=r)
        runs.append(run)
    merged = merge_runs(runs, key_names[0])
    if merged is None:
        return {k: mine[k] for k in names}
    return merged


Q_PARTITIONED, Q_TIMERS = 1, 2


class ShardedAppRuntime:
    """One rank's share of a Siddhi app on an N-GPU node: partitioned queries are key-hash sharded
    (rank r processes the events whose partition key hashes to r, `owner`), unpartitioned queries run as replicas
    on rank 0. N > 1 is refused with OperationNotSupportedException for queries with absent states: the reference's
    Scheduler collapses the due timers of ALL partition keys into one TreeMultimap per clock advance
    (Scheduler.java:75-98, only the first state per due time fires), so which fires it delays depends on keys that
    would live on other GPUs -- sharding them would silently change the matches (7,857 vs 9,790).
    Such an app runs on one GPU (world 1), where the engine reproduces the collapse exactly."""

    def __init__(self, app_text, rank, world, device=0, key_attr=None, **kw):
        import siddhi_amd as sa
        self.rank, self.world = rank, world
        self.rt = sa.SiddhiAppRuntime(app_text, device=device, **kw)
        flags = self.rt.query_flags()
        if world > 1 and any(f & Q_TIMERS for f in flags):
            names = [q[0] for q, f in zip(self.rt._queries, flags) if f & Q_TIMERS]
            self.rt.shutdown()
            raise sa.OperationNotSupportedException(
                "queries %s have absent states: the reference's scheduler orders timers across all partition keys "
                "(Scheduler.java:75-98), so they cannot be key-sharded over %d GPUs; run the app on one GPU" % (names, world))
        self.sharded = all(f & Q_PARTITIONED for f in flags)
        self.replica = not self.sharded  # an unpartitioned query: every event, on rank 0 only
        self.key_attr = key_attr or {}    # stream id -> index of its partition attribute

    def mine(self, stream_id, row):
        """whether this rank processes the event"""
        if self.world == 1:
            return True
        if self.replica:
            return self.rank == 0
        return owner(row[self.key_attr[stream_id]], self.world) == self.rank

    def send(self, stream_id, ts, row):
        if self.mine(stream_id, row):
            self.rt.getInputHandler(stream_id).send(ts, row)

    def shutdown(self):
        self.rt.shutdown()
