"""Per-key state lifetime on the GPU (PartitionStateHolder.returnState :51-70 destroys a
key's processor states once StreamPreState.canDestroy :443-448 holds). 10^7 distinct partition keys pass through
over time, at most 10^5 of them live in any flush: every key gets 10 events inside one block of 1,000 events, the
last of them closing its partial matches (strict sequence), so its state shrinks to the start processor's seed --
what the reference keeps -- and the engine keeps an idle record instead of a partial-match arena. The arena pool
must stay sized by the live keys, and the matches of a sample of keys must equal the oracle's."""
import numpy as np
import pytest

import siddhi_amd as sa
from oracle_rt import Oracle
from siddhi_amd import workloads as w

pytestmark = pytest.mark.gpu

APP = ("@app:playback define stream S (id long, key long, price double, volume int); "
       "partition with (key of S) begin @info(name = 'query1') "
       "from every e1=S[price>20], e2=S[price>e1.price] "
       "select e1.id as e1id, e2.id as e2id insert into M; end;")
BLOCK, KEYS_PER_BLOCK = 1000, 100


def churn_columns(lo, hi):
    i = np.arange(lo, hi, dtype=np.int64)
    key_idx = (i // BLOCK) * KEYS_PER_BLOCK + (i % KEYS_PER_BLOCK)
    price = w.prices(29, hi - lo, lo)
    price[(i % BLOCK) >= BLOCK - KEYS_PER_BLOCK] = 5.0  # each key's last event: e1 fails, open partials dropped
    return {"ts": w.T0 + i // 100, "id": i, "key": key_idx * 7919 + 13, "price": price,
            "volume": (i % 1000).astype(np.int32)}


def test_churn_ten_million_keys_arena_bounded(oracle_built):
    import torch
    dev = torch.device("cuda", 0)
    n_total, per_flush = 100_000_000, 1_000_000   # 10^7 keys over time, 10^5 per flush
    sample_blocks = [0, 1, 3, 17, 50_000, 99_998, 99_999]  # keys of these blocks go to the oracle
    rt = sa.SiddhiAppRuntime(APP)
    got, max_slots = [], 0
    try:
        assert rt.query_paths() == [1]
        for lo in range(0, n_total, per_flush):
            c = churn_columns(lo, lo + per_flush)
            d = [torch.from_numpy(c[k]).to(dev) for k in ("id", "key", "price", "volume")]
            d_ts = torch.from_numpy(c["ts"]).to(dev)
            rt.push_device("S", per_flush, d_ts.data_ptr(), [x.data_ptr() for x in d])
            rt.flush(deliver=False)
            max_slots = max(max_slots, rt.stats().arena_slots)
            ts, vals, nulls, seq = rt.poll_arrays(0)
            blk = vals[0] // BLOCK
            sel = np.isin(blk, sample_blocks)
            got.append(np.stack([ts[sel], vals[0][sel], vals[1][sel]], axis=1))
    finally:
        rt.shutdown()
    # the pool holds the live keys (10^5 per flush, with the pool's growth headroom), not the 10^7 seen
    assert max_slots <= 400_000, max_slots
    got = np.concatenate(got)
    o = Oracle(APP)
    try:
        for b in sample_blocks:
            c = churn_columns(b * BLOCK, (b + 1) * BLOCK)
            for r in range(BLOCK):
                o.send("S", int(c["ts"][r]), [int(c["id"][r]), int(c["key"][r]), float(c["price"][r]),
                                              int(c["volume"][r])])
        ref = np.array([(r["ts"], r["values"][0][1], r["values"][1][1]) for r in o.outputs() if r["kind"] == "query"],
                       dtype=np.int64)
    finally:
        o.close()
    assert len(ref) > 100
    assert got.shape == ref.shape and np.array_equal(got, ref)
