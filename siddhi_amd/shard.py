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


def route(keys, world, cache=None):
    """rank of each event, for an array/list of partition key values (PartitionStreamReceiver.receive(Event[])
    :176-216 routes a batch key by key; here the batch is split by owner at once): each distinct key's toString is
    hashed once (np.unique + a per-router cache keyed by that string), then the ranks are gathered back to the rows.
    The distinct keys are hashed as the numpy scalars of the column (str(np.float32(0.1)) == '0.1', as a per-row
    send() of the same float32 value hashes it), never as Python floats widened from another width."""
    if world == 1:
        return np.zeros(len(keys), dtype=np.int32)
    cache = {} if cache is None else cache

    def rank_of(k):
        sk = str(k)
        r = cache.get(sk)
        if r is None:
            r = cache[sk] = key_hash(sk) % world
        return r
    arr = np.asarray(keys)
    if arr.dtype == object or arr.ndim != 1:
        return np.fromiter((rank_of(k) for k in keys), dtype=np.int32, count=len(keys))
    uniq, inv = np.unique(arr, return_inverse=True)
    ranks = np.fromiter((rank_of(k) for k in uniq), dtype=np.int32, count=len(uniq))
    return ranks[inv]


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
    """G-way merge of sorted runs (dicts of torch tensors, records along the last dim) by their 1-D `key` column;
    equal keys keep run order, then their order inside the run. Runs on the GPU go through the device merge
    (sdg_merge_runs, merge.hip: regular-sampling splitters, one workgroup per bucket merging in LDS, every record
    read and written once; int64 keys). Runs in host memory (the gloo rehearsals on CPU) are merged on the host: the
    runs concatenated in run order and one stable sort of the key, or binary searches of each record into the other
    runs for small inputs."""
    import torch
    runs = [r for r in runs if r[key].numel() > 0]
    if not runs:
        return None
    if len(runs) == 1:
        return runs[0]
    if runs[0][key].is_cuda and runs[0][key].dtype == torch.int64 and len(runs) <= 32:
        return _merge_runs_device(runs, key)
    total = sum(int(r[key].numel()) for r in runs)
    if total >= (1 << 20):
        cat = {k: torch.cat([r[k] for r in runs], dim=-1) for k in runs[0]}
        kv = cat[key]
        lo = kv.min()
        span = int((kv.max() - lo).item())
        rel = (kv - lo).to(torch.int32) if span < (1 << 31) else kv - lo
        perm = torch.sort(rel, stable=True).indices
        return {k: v[..., perm] for k, v in cat.items()}
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


def _merge_runs_device(runs, key):
    """merge_runs on the GPU (sdg_merge_runs): each 2-D column [m, n] travels as its m rows"""
    import torch
    from siddhi_amd import merge_runs_device
    names = [k for k in runs[0] if k != key]
    total = sum(int(r[key].numel()) for r in runs)
    dev = runs[0][key].device
    out = {key: torch.empty(total, dtype=torch.int64, device=dev)}
    out_cols, src = [], [[] for _ in runs]
    for k in names:
        v = runs[0][k]
        out[k] = torch.empty(list(v.shape[:-1]) + [total], dtype=v.dtype, device=dev)
        rows = [out[k]] if v.dim() == 1 else list(out[k].reshape(-1, total))
        out_cols += rows
        for i, r in enumerate(runs):
            c = r[k].contiguous()
            src[i] += [c] if c.dim() == 1 else list(c.reshape(-1, c.shape[-1]))
    if len(out_cols) > 16:
        raise ValueError("merge_runs: more than 16 payload columns")
    merge_runs_device([r[key].contiguous() for r in runs], src, out[key], out_cols)
    return out


def ordered_gather(dist, rank, world, cols, key_names, presorted=False, first_key_unique=False, timings=None):
    """Ordered result gather: `cols` maps names to this rank's record tensors (1-D [n], or 2-D
    [m, n] with records along the last dim) on the communication device. Every rank sorts its records by
    `key_names` on its device, the run lengths are all-gathered, and each rank's sorted run goes to rank 0
    point-to-point (send/recv: RCCL over xGMI with the nccl backend, gloo on CPU), where the G runs are merged on the
    first key (merge_runs: records of different ranks with equal first keys keep rank order, which is the
    tie-break every caller's key implies -- either the first key is unique across ranks, e.g. the global position of
    the emitting event, or the rank is the next key). presorted: the records already are in `key_names` order (an
    sdg_export_ordered run), no local sort. timings: a dict whose "transfer" / "merge" entries get this call's seconds
    added (device-synchronised). Returns the merged dict on rank 0, None elsewhere."""
    import torch
    # the merge orders by key_names[0], then rank, then each run's own order: that equals key_names order only if
    # the first key is unique across ranks or the rank is the next key
    if not (len(key_names) == 1 or key_names[1] == "rank" or first_key_unique):
        raise ValueError("ordered_gather merges on %r then rank: pass first_key_unique=True or put 'rank' second"
                         % key_names[0])
    names = sorted(cols)
    ref = cols[key_names[0]]
    if presorted:
        mine = {k: cols[k].contiguous() for k in names}
    else:
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
    import time
    torch.cuda.synchronize() if ref.is_cuda else None
    t0 = time.perf_counter()
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
    torch.cuda.synchronize() if ref.is_cuda else None
    t1 = time.perf_counter()
    merged = merge_runs(runs, key_names[0])
    torch.cuda.synchronize() if ref.is_cuda else None
    if timings is not None:
        timings["transfer"] = timings.get("transfer", 0.0) + t1 - t0
        timings["merge"] = timings.get("merge", 0.0) + time.perf_counter() - t1
    if merged is None:
        return {k: mine[k] for k in names}
    return merged


Q_PARTITIONED, Q_TIMERS, Q_BROADCAST = 1, 2, 4


class ShardedAppRuntime:
    """One rank's share of a Siddhi app on an N-GPU node: partitioned queries are key-hash sharded
    (rank r processes the events whose partition key hashes to r, `owner`), unpartitioned queries run as replicas
    on rank 0 (the streams only they read go to rank 0 whole; a stream read by both kinds makes the whole app run on
    rank 0, with a RuntimeWarning). Each stream is routed by the partition attribute the ENGINE compiled for it
    (sdg_query_key_attr), so the router and the queries cannot disagree. At N > 1 these partitioned queries cannot be
    key-sharded and run whole on rank 0 instead (RuntimeWarning; the same rule as unpartitioned ones, so a stream they
    share with sharded queries sends the whole app to rank 0):
      * absent states: the reference's Scheduler collapses the due timers of ALL partition keys into one TreeMultimap
        per clock advance (Scheduler.java:75-98, only the first state per due time fires), so which fires it delays
        depends on keys that would live on other GPUs (7,857 vs 9,790);
      * a stream without a partition key (PartitionStreamReceiver.send(ComplexEvent) :274-283): its events go to
        every key of the partition in ONE global key order that interleaves the ranks' keys;
      * range partitions: an event may belong to several ranges (keys), so it has no single owner;
      * a stream that two partitions key by different attributes: no single owner either.
    Rank 0 then runs them exactly as one GPU does. A caller's key_attr that disagrees with the engine is refused
    (OperationNotSupportedException)."""

    def __init__(self, app_text, rank, world, device=0, key_attr=None, **kw):
        import siddhi_amd as sa
        self.rank, self.world = rank, world
        self.rt = sa.SiddhiAppRuntime(app_text, device=device, **kw)
        flags = self.rt.query_flags()
        names = [q[0] for q in self.rt._queries]

        def refuse(msg):
            self.rt.shutdown()
            raise sa.OperationNotSupportedException(msg)
        streams = self.rt.app_stream_ids()
        reads = {s: [q for q in range(len(names)) if self.rt.query_reads(q, s)] for s in streams}
        # partitioned queries that cannot be key-sharded at N > 1 run whole on rank 0 (class docstring)
        whole = {}
        if world > 1:
            for q, f in enumerate(flags):
                if not f & Q_PARTITIONED:
                    continue
                if f & Q_TIMERS:
                    whole[q] = "absent states (one global timer order, Scheduler.java:75-98)"
                elif f & Q_BROADCAST:
                    whole[q] = "a stream without a partition key (one global key order, PartitionStreamReceiver.java:274-283)"
                elif any(self.rt.query_key_attr(q, s) == -2 for s in streams if q in reads[s]):
                    whole[q] = "range partitions (an event may belong to several keys)"
            for s in streams:
                qs = [q for q in reads[s] if flags[q] & Q_PARTITIONED and q not in whole]
                if len({self.rt.query_key_attr(q, s) for q in qs} - {-1}) > 1:
                    for q in qs:
                        whole[q] = "stream '%s' keyed by different attributes in different partitions" % s
        part = [bool(f & Q_PARTITIONED) and q not in whole for q, f in enumerate(flags)]
        # a stream that an unpartitioned (or rank-0-only) query reads must reach ONE rank whole (rank 0); if a sharded
        # query reads it too, that query's keys would be split between the sharded streams and this one, so at N > 1
        # the whole app goes to rank 0 -- said out loud (warning), never silently
        mixed = sorted(s for s, qs in reads.items() if any(part[q] for q in qs) and not all(part[q] for q in qs))
        self.sharded = all(part)
        self.replica = bool(mixed)  # every event, on rank 0 only
        self.whole_streams = {s for s, qs in reads.items() if qs and not any(part[q] for q in qs)}  # rank 0 only
        self.whole_queries = {names[q]: why for q, why in whole.items()}
        if world > 1 and (mixed or whole):
            import warnings
            for q, why in sorted(whole.items()):
                warnings.warn("query '%s' has %s: it runs whole on rank 0 of %d, not key-sharded" % (names[q], why, world),
                              RuntimeWarning, stacklevel=2)
            if mixed:
                warnings.warn("streams %s are read by key-sharded and rank-0-only queries: the app cannot be key-sharded "
                              "and runs whole on rank 0 of %d" % (mixed, world), RuntimeWarning, stacklevel=2)
        # stream id -> the partition attribute every partitioned query reading it keys it by
        self.key_attr = {}
        for s in streams:
            attrs = {self.rt.query_key_attr(q, s) for q in range(len(names)) if part[q]} - {-1}
            if not attrs:
                continue
            if world > 1 and (len(attrs) > 1 or min(attrs) < 0):
                refuse("stream '%s' is keyed by %s in different partitions (or by ranges): its events have no single "
                       "owner GPU" % (s, sorted(attrs)))
            self.key_attr[s] = attrs.pop()
        for s, a in (key_attr or {}).items():  # a caller's statement of the keys must agree with the engine's
            if self.key_attr.get(s, a) != a:
                refuse("key_attr[%r] = %d, but the app partitions it by attribute %d" % (s, a, self.key_attr[s]))
        self._cache = {}

    def mine(self, stream_id, row):
        """whether this rank processes the event"""
        if self.world == 1:
            return True
        if self.replica:
            return self.rank == 0
        ai = self.key_attr.get(stream_id)
        if ai is None:  # no partitioned query reads the stream: whole, on rank 0
            return self.rank == 0
        return route([row[ai]], self.world, self._cache)[0] == self.rank

    def send(self, stream_id, ts, row):
        if self.mine(stream_id, row):
            self.rt.getInputHandler(stream_id).send(ts, row)

    def send_columns(self, stream_id, ts, columns, key_values=None):
        """a columnar batch (InputHandler.send per row, in order): this rank's rows, routed at once. key_values:
        the key attribute's values as the app sees them (e.g. strings when `columns` hold sdg_intern ids); default
        the key column itself"""
        ts = np.asarray(ts)
        if self.world == 1:
            mask = slice(None)
        elif self.replica or stream_id not in self.key_attr:
            if self.rank != 0:
                return 0
            mask = slice(None)
        else:
            kv = columns[self.key_attr[stream_id]] if key_values is None else key_values
            mask = route(kv, self.world, self._cache) == self.rank
        cols = [np.ascontiguousarray(np.asarray(c)[mask]) for c in columns]
        sel = np.ascontiguousarray(ts[mask])
        if len(sel):
            self.rt.getInputHandler(stream_id).send_columns(sel, cols)
        return len(sel)

    def shutdown(self):
        self.rt.shutdown()
