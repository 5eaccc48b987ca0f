"""C5 on one GPU (BASELINE.json configs[4]): one rank's key-hash shard of the 8-GPU C5 stream
(10^8 keys / 8 = 12.5M partition keys on this GPU, the radix key-sort path), generated on the device
(siddhi_amd/c5.py), pushed device-resident over several flushes so partials are carried across batch boundaries.

* a 10^4-key sample of the shard against the oracle, bit-exact and in delivery order ("Parity for
  C5 uses the restatement on a seeded sample of 10^4 keys");
* every other match record by size-independent properties (same owned key, order, window, both filters, the
  record timestamp), and every e1 matched at most once across the flushes;
* the generator itself against the numpy C2 generator of siddhi_amd/workloads.py and shard.owner.
"""
import numpy as np
import pytest

import siddhi_amd as sa
from siddhi_amd import c5, shard
from siddhi_amd import workloads as w

pytestmark = pytest.mark.gpu

WORLD, RANK = 8, 0
BATCH = 1 << 27          # rank events per flush (the bench uses 2^28)
FLUSHES = 3
SAMPLE = 10_000


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    return torch.device("cuda", 0)


def test_generator_matches_numpy_and_shard_owner(torch_dev):
    import torch
    rt = sa.SiddhiAppRuntime(w.C2_APP)
    try:
        nkeys = 1_000_000
        sh = c5.C5Shard(rt, 1, 4, torch_dev, nkeys=nkeys, events=10 ** 9, batch=1 << 16)
        # ownership: fnv1a64 of the key string, as shard.owner
        ks = np.random.default_rng(3).integers(0, nkeys, 2000)
        own = set(sh.keys.tolist())
        assert all((shard.owner("S%08d" % k, 4) == 1) == (k in own) for k in ks)
        cols, n = sh.generate(3)
        g0, g1 = sh.global_range(3)
        ref = w.c2_columns(g1 - g0, keys=nkeys, seed=c5.SEED, per_ms=c5.PER_MS, offset=g0)
        keep = np.isin(ref["key"], sh.keys)
        assert n == keep.sum() and n > 0
        assert np.array_equal(cols["id"].cpu().numpy(), ref["id"][keep])
        assert np.array_equal(cols["ts"].cpu().numpy(), ref["ts"][keep])
        assert np.array_equal(cols["price"].cpu().numpy().view(np.int64), ref["price"][keep].view(np.int64))
        assert np.array_equal(cols["volume"].cpu().numpy(), ref["volume"][keep])
        names = [rt.string(int(i)) for i in cols["sym"][:50].cpu().numpy()]
        assert names == ["S%08d" % k for k in ref["key"][keep][:50]]
        ids = cols["id"][:1000]
        assert np.array_equal(sh.key_of(ids, sh.map).cpu().numpy(), cols["sym"][:1000].cpu().numpy())
        assert np.array_equal(sh.price_of(ids).cpu().numpy(), cols["price"][:1000].cpu().numpy())
        del cols
        torch.cuda.empty_cache()
    finally:
        rt.shutdown()


def test_c5_rank_shard_radix_path_vs_oracle_sample(torch_dev, oracle_built):
    import torch
    from c5_check import delivery_order, oracle_sample_rows, sample_records
    rt = sa.SiddhiAppRuntime(w.C2_APP)
    sh = c5.C5Shard(rt, RANK, WORLD, torch_dev, batch=BATCH)
    assert sh.n_keys >= 10 ** 7
    skeys, smap = sh.sample(SAMPLE)
    gpu_rows, e1_all, n_matches, pushed = [], [], 0, 0
    try:
        for j in range(FLUSHES):
            cols, n = sh.generate(j)
            pushed += n
            rt.push_device("StockStream", n, cols["ts"].data_ptr(),
                           [cols["id"].data_ptr(), cols["sym"].data_ptr(), cols["price"].data_ptr(),
                            cols["volume"].data_ptr()])
            rt.flush(deliver=False)
            st = rt.stats()
            assert st.fused == 0 and st.path == 0  # > 2^16 keys: radix key sort + chain kernels
            m = int(st.matches)
            t_ts = torch.empty(max(m, 1), dtype=torch.int64, device=torch_dev)
            t_seq, t_sub = torch.empty_like(t_ts), torch.empty_like(t_ts)
            t_vals = torch.empty((2, max(m, 1)), dtype=torch.int64, device=torch_dev)
            got = rt.export_device(0, max(m, 1), t_ts.data_ptr(), t_seq.data_ptr(), t_sub.data_ptr(),
                                   t_vals.data_ptr())
            assert got == m
            e1, e2, ts = t_vals[0, :m], t_vals[1, :m], t_ts[:m]
            bad = c5.check_matches(sh, e1, e2, ts)
            assert not any(bad.values()), bad
            gpu_rows.append(sample_records(sh, smap, ts, e1, e2))
            e1_all.append(e1.clone())
            n_matches += m
            del cols, t_ts, t_seq, t_sub, t_vals
            torch.cuda.empty_cache()
        assert n_matches > pushed // 4
        allk = torch.sort(torch.cat(e1_all)).values
        assert allk.numel() == n_matches and bool((allk[1:] > allk[:-1]).all())  # each e1 matched at most once
        del allk, e1_all
        _, g_end = sh.global_range(FLUSHES - 1)
        n_s, ref = oracle_sample_rows(sh, skeys, smap, g_end)
        got = delivery_order(np.concatenate(gpu_rows))
        assert n_s > 100 * len(skeys) // 4 and len(ref) > 1000
        assert got.shape == ref.shape and np.array_equal(got, ref)
    finally:
        rt.shutdown()
