"""C5 (BASELINE.json configs[4]): the C2 query over 10^10 events and 10^8 partition keys, key-hash
sharded over the GPUs of one node, each rank generating its own shard on its GPU in batches of 2^28 events.

    partition with (symbol of StockStream) begin
      from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec
      select e1.id as e1id, e2.id as e2id insert into M; end;

Global event i: key k_i = splitmix64(17, i) mod 10^8 (symbol "S%08d" % k_i), price from splitmix64(18, i) as C2,
ts_i = T0 + floor(i / 10^6), id_i = i (so a match's e2id is the global position of the event that emitted it, and
(e2id, e1id) is the single-engine delivery order of PartitionStreamReceiver -> StateMultiProcessStreamReceiver).
Rank r of N owns the keys whose "S%08d" string hashes to r (siddhi_amd/shard.py owner, PartitionRuntimeImpl's
per-key independence, PartitionRuntimeImpl.java:346-366); it interns exactly those strings, in key order, and
generates only their events: global batch j = indices [j 2^28 N, (j + 1) 2^28 N), so every rank's flush j holds
~2^28 events and the ranks' flushes cover the same span of event time.

The generator is siddhi_amd/csrc/synth/synth.hip (libsdg_synth.so), benchmark / test infrastructure beside the
engine: its columns enter the engine through sdg_push_device like any application's device-resident batch.
"""
import ctypes
import os

import numpy as np

SEED = 17
KEYS = 100_000_000
EVENTS = 10_000_000_000
PER_MS = 1_000_000
BATCH = 1 << 28
T0 = 1_700_000_000_000

_HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH_PATH = os.path.join(_HERE, "_lib", "libsdg_synth.so")
_lib = None


def synth_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SYNTH_PATH):
            raise RuntimeError("libsdg_synth.so missing at %s (make -C siddhi_amd)" % SYNTH_PATH)
        L = ctypes.CDLL(SYNTH_PATH)
        P, I32, I64, U64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
        L.sdg_synth_owner.argtypes = [I64, I32, P, P]
        L.sdg_synth_workspace.restype = I64
        L.sdg_synth_workspace.argtypes = [I64, I64]
        L.sdg_synth_batch.argtypes = [U64, I64, P, I64, I64, I64, I64, P, I64, P, P, P, P, P, P, P, P]
        L.sdg_synth_key_of.argtypes = [U64, I64, P, I64, P, P, P]
        L.sdg_synth_price_of.argtypes = [U64, P, I64, P, P]
        _lib = L
    return _lib


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError("C5 generator: %s failed" % what)


def key_strings(keys):
    """'S%08d' % k for an int64 array of keys < 10^8, as one uint8 buffer of 9-byte strings"""
    keys = np.asarray(keys, dtype=np.int64)
    b = np.empty((len(keys), 9), dtype=np.uint8)
    b[:, 0] = ord("S")
    for d in range(8):
        b[:, 1 + d] = (keys // 10 ** (7 - d)) % 10 + ord("0")
    return b.reshape(-1)


def _sync():
    import torch
    torch.cuda.synchronize()


class C5Shard:
    """Rank `rank` of `world`: its keys interned into the runtime `rt` (in key order), the key -> id map on the GPU,
    and the generator of its flushes."""

    def __init__(self, rt, rank, world, device, nkeys=KEYS, events=EVENTS, batch=BATCH, seed=SEED, per_ms=PER_MS):
        import torch
        self.rank, self.world, self.device = rank, world, device
        self.nkeys, self.events, self.batch, self.seed, self.per_ms = nkeys, events, batch, seed, per_ms
        L = synth_lib()
        owner = torch.empty(nkeys, dtype=torch.uint8, device=device)
        _sync()
        _ok(L.sdg_synth_owner(nkeys, world, owner.data_ptr(), None), "owner")
        owned = torch.nonzero(owner == rank).flatten()  # ascending key indices
        del owner
        self.keys = owned.cpu().numpy()
        ids = rt.intern_many(key_strings(self.keys), np.arange(len(self.keys) + 1, dtype=np.int64) * 9)
        self.map = torch.full((nkeys,), -1, dtype=torch.int32, device=device)
        self.map[owned] = torch.from_numpy(ids.view(np.int32)).to(device)
        _sync()
        self.n_keys = len(self.keys)

    def n_batches(self):
        return -(-self.events // (self.batch * self.world))

    def global_range(self, j):
        g0 = j * self.batch * self.world
        return g0, min(g0 + self.batch * self.world, self.events)

    def _gen(self, kmap, g0, g1, expect):
        """the events of [g0, g1) whose key has kmap[key] >= 0, as torch columns on the device (sym = kmap value)"""
        import torch
        L = synth_lib()
        dev = self.device
        work = torch.empty(max(8, L.sdg_synth_workspace(g0, g1)), dtype=torch.uint8, device=dev)
        cnt_d = torch.zeros(1, dtype=torch.int64, device=dev)
        cap = int(expect * 1.02) + 65536
        for _ in range(2):
            cols = {"ts": torch.empty(cap, dtype=torch.int64, device=dev),
                    "id": torch.empty(cap, dtype=torch.int64, device=dev),
                    "sym": torch.empty(cap, dtype=torch.int32, device=dev),
                    "price": torch.empty(cap, dtype=torch.float64, device=dev),
                    "volume": torch.empty(cap, dtype=torch.int32, device=dev)}
            n = ctypes.c_int64()
            _sync()
            _ok(L.sdg_synth_batch(self.seed, self.nkeys, kmap.data_ptr(), g0, g1, T0, self.per_ms, work.data_ptr(), cap,
                                  cols["ts"].data_ptr(), cols["id"].data_ptr(), cols["sym"].data_ptr(),
                                  cols["price"].data_ptr(), cols["volume"].data_ptr(), cnt_d.data_ptr(),
                                  ctypes.byref(n), None), "batch")
            if n.value <= cap:
                return {k: v[: n.value] for k, v in cols.items()}, n.value
            cap = n.value
        raise RuntimeError("C5 generator: capacity")

    def generate(self, j):
        """this rank's flush j: (columns, n)"""
        g0, g1 = self.global_range(j)
        return self._gen(self.map, g0, g1, (g1 - g0) / self.world)

    def sample(self, nsample):
        """`nsample` of this rank's keys, evenly spread over them: (key indices, map key -> sample index)"""
        import torch
        step = max(1, self.n_keys // nsample)
        keys = self.keys[::step][:nsample]
        smap = torch.full((self.nkeys,), -1, dtype=torch.int32, device=self.device)
        smap[torch.from_numpy(keys).to(self.device)] = torch.arange(len(keys), dtype=torch.int32, device=self.device)
        _sync()
        return keys, smap

    def sample_events(self, smap, nsample, g0, g1):
        """the sample keys' events of [g0, g1) (host numpy columns; sym = sample index)"""
        cols, n = self._gen(smap, g0, g1, (g1 - g0) * nsample / self.nkeys)
        return {k: v.cpu().numpy() for k, v in cols.items()}

    def key_of(self, ids, kmap=None):
        """per event id (int64 device tensor): kmap[key] (default: this rank's id map)"""
        import torch
        out = torch.empty_like(ids)
        m = self.map if kmap is None else kmap
        _sync()
        _ok(synth_lib().sdg_synth_key_of(self.seed, self.nkeys, ids.data_ptr(), ids.numel(), m.data_ptr(),
                                         out.data_ptr(), None), "key_of")
        _sync()
        return out

    def price_of(self, ids):
        import torch
        out = torch.empty(ids.numel(), dtype=torch.float64, device=ids.device)
        _sync()
        _ok(synth_lib().sdg_synth_price_of(self.seed, ids.data_ptr(), ids.numel(), out.data_ptr(), None), "price_of")
        _sync()
        return out


def check_matches(shard, e1, e2, ts, within_ms=1000):
    """Size-independent properties of C5 match records (device tensors e1id, e2id, ts): both events of a match are
    of one key owned by this rank, e1 came first, e2 lies in e1's window, e1 passed price > 20, e2's price beats
    e1's, and the record's timestamp is e2's. Returns a dict of violation counts (all 0 when the records hold)."""
    import torch
    k1, k2 = shard.key_of(e1), shard.key_of(e2)
    p1, p2 = shard.price_of(e1), shard.price_of(e2)
    t1 = T0 + torch.div(e1, shard.per_ms, rounding_mode="floor")
    t2 = T0 + torch.div(e2, shard.per_ms, rounding_mode="floor")
    bad = {"key": int(((k1 != k2) | (k1 < 0)).sum().item()),
           "order": int((e1 >= e2).sum().item()),
           "window": int(((t2 - t1) > within_ms).sum().item()),
           "e1_filter": int((~(p1 > 20.0)).sum().item()),
           "e2_filter": int((~(p2 > p1)).sum().item()),
           "ts": int((ts != t2).sum().item())}
    return bad
