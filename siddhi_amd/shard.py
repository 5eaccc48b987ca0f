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
