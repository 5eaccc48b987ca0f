"""JDK 8 iteration orders, transliterated from java.util.concurrent.ConcurrentHashMap (putVal / addCount /
treeifyBin -> tryPresize / transfer) and java.util.HashSet(Collection) -> HashMap.putVal, for a third, independent
statement of the partition-key order a broadcast follows (PartitionRuntimeImpl.getPartitionKeys :404-407). Used by
tests/test_broadcast_order.py to pin the oracle's and the engine's restatements (oracle.cpp JavaCHM, keyorder.h)."""


def string_hash(s):
    """String.hashCode over UTF-16 code units, as an unsigned 32-bit value"""
    b = s.encode("utf-16-le")
    h = 0
    for i in range(0, len(b), 2):
        h = (31 * h + (b[i] | (b[i + 1] << 8))) & 0xFFFFFFFF
    return h


def chm_spread(h):
    return (h ^ (h >> 16)) & 0x7FFFFFFF


def table_size_for(c):
    n = 1
    while n < c:
        n <<= 1
    return n


class CHM:
    """ConcurrentHashMap<String, Long>, one thread; bins are Python lists of (hash, key) in list order"""

    def __init__(self):
        self.table = None
        self.size_ctl = 0
        self.count = 0

    def _transfer(self):
        tab = self.table
        n = len(tab)
        nxt = [None] * (2 * n)
        for i in range(n - 1, -1, -1):  # transfer walks the bins from the top
            f = tab[i]
            if not f:
                nxt[i], nxt[i + n] = [], []
                continue
            run_bit = f[0][0] & n
            last_run = 0
            for p in range(1, len(f)):
                b = f[p][0] & n
                if b != run_bit:
                    run_bit, last_run = b, p
            ln, hn = (f[last_run:], []) if run_bit == 0 else ([], f[last_run:])
            for p in range(last_run):
                if f[p][0] & n == 0:
                    ln = [f[p]] + ln
                else:
                    hn = [f[p]] + hn
            nxt[i], nxt[i + n] = ln, hn
        self.table = nxt
        self.size_ctl = (n << 1) - (n >> 1)

    def _try_presize(self, size):
        c = table_size_for(size + (size >> 1) + 1)
        while True:
            n = len(self.table)
            if c <= self.size_ctl:
                break
            self._transfer()

    def put(self, key):
        h = chm_spread(string_hash(key))
        if self.table is None:
            self.table = [[] for _ in range(16)]
            self.size_ctl = 12
        n = len(self.table)
        f = self.table[(n - 1) & h]
        bin_count = 0
        found = False
        if not f:
            f.append((h, key))
        else:
            bin_count = 1
            p = 0
            while True:
                if f[p][0] == h and f[p][1] == key:
                    found = True
                    break
                if p + 1 == len(f):
                    f.append((h, key))
                    break
                p += 1
                bin_count += 1
        if bin_count != 0 and bin_count >= 8:  # treeifyBin
            if n < 64:
                self._try_presize(n << 1)
            else:
                raise NotImplementedError("tree bin")
        if found:
            return
        self.count += 1
        if self.count >= self.size_ctl:
            self._transfer()

    def keys(self):
        return [k for b in self.table or [] for _, k in b]


def hashset_order(chm):
    """new HashSet<>(chm.keySet()) iterated"""
    keys = chm.keys()
    import numpy as np
    cap = table_size_for(max(int(np.float32(len(keys)) / np.float32(0.75)) + 1, 16))  # (int)(size / .75f)
    tab = [[] for _ in range(cap)]
    for k in keys:
        h = string_hash(k)
        h ^= h >> 16
        b = tab[h & (cap - 1)]
        b.append((h, k))
        if len(b) - 1 >= 8:  # binCount >= TREEIFY_THRESHOLD - 1 with binCount = nodes before the new one
            if cap >= 64:
                raise NotImplementedError("tree bin")
            cap *= 2  # HashMap.resize: lo / hi split keeps the relative order
            new = [[] for _ in range(cap)]
            for ob in tab:
                for x in ob:
                    new[x[0] & (cap - 1)].append(x)
            tab = new
    return [k for b in tab for _, k in b]
