"""The ordered result gather's device merge (sdg_merge_runs, merge.hip) against a stable sort of the concatenated
runs by (key, run, index): ties inside and across runs, empty and one-record runs, 1 to 32 runs, negative keys and a
full 64-bit key span, payload columns of every width, 2-D columns (shard.merge_runs). Runs on an MI355X (-m gpu)."""
import numpy as np
import pytest
import torch

from siddhi_amd import shard

pytestmark = pytest.mark.gpu


def _runs(G, seed, n_max, key_range, lo=0, dev="cuda"):
    g = torch.Generator().manual_seed(seed)
    runs = []
    for r in range(G):
        n = int(torch.randint(0, n_max + 1, (1,), generator=g))
        if r == 1:
            n = 1 if n_max > 0 else 0
        k = torch.sort(torch.randint(lo, lo + key_range, (n,), generator=g, dtype=torch.int64)).values
        runs.append({"k": k.to(dev), "run": torch.full((n,), r, dtype=torch.int32, device=dev),
                     "i": torch.arange(n, dtype=torch.int64, device=dev),
                     "b": (k % 251).to(torch.uint8).to(dev), "h": (k % 30011).to(torch.int16).to(dev),
                     "f": (k.to(torch.float64) * 0.5).to(dev), "v": torch.stack([k * 3, k * 5]).to(dev)})
    return runs


def _expect(runs):
    cat = {c: torch.cat([r[c].cpu() for r in runs], dim=-1) for c in runs[0]}
    order = shard.lexsort([cat["k"], cat["run"].to(torch.int64), cat["i"]])
    return {c: v[..., order] for c, v in cat.items()}


@pytest.mark.parametrize("G,n_max,key_range,lo", [(2, 3000, 50, 0), (5, 4000, 300, -1000), (8, 20000, 10 ** 6, 0),
                                                  (8, 5000, 3, 0), (32, 2000, 700, -5), (17, 9000, 2 ** 40, -2 ** 39),
                                                  (6, 20000, 2 ** 40, 0), (4, 20000, 2 ** 33, -2 ** 60)])
@pytest.mark.parametrize("pairwise", ["1", "0"])
def test_device_merge_is_a_stable_g_way_merge(G, n_max, key_range, lo, pairwise, monkeypatch):
    """pairwise=1: buckets whose keys span < 2^32 take the pairwise LDS merge paths, the others the rank search;
    pairwise=0: every bucket ranks (SDG_MG_PAIR)"""
    monkeypatch.setenv("SDG_MG_PAIR", pairwise)
    runs = _runs(G, seed=G * 7 + n_max, n_max=n_max, key_range=key_range, lo=lo)
    m = shard.merge_runs(runs, "k")
    exp = _expect([r for r in runs if r["k"].numel() > 0])
    for c in exp:
        assert torch.equal(m[c].cpu(), exp[c]), c


@pytest.mark.parametrize("pairwise", ["1", "0"])
def test_device_merge_mixed_bucket_spans(pairwise, monkeypatch):
    """dense keys (buckets spanning < 2^32: pairwise merge) and sparse keys up to 2^62 (wide buckets: rank search)
    in one merge, with ties between the two populations' runs"""
    monkeypatch.setenv("SDG_MG_PAIR", pairwise)
    g = torch.Generator().manual_seed(11)
    runs = []
    for r in range(7):
        dense = torch.randint(0, 5000, (30000,), generator=g, dtype=torch.int64)
        sparse = torch.randint(0, 2 ** 62, (int(torch.randint(0, 20000, (1,), generator=g)),), generator=g,
                               dtype=torch.int64)
        k = torch.sort(torch.cat([dense, sparse, torch.tensor([2 ** 40] * r, dtype=torch.int64)])).values
        runs.append({"k": k.cuda(), "run": torch.full((len(k),), r, dtype=torch.int32).cuda(),
                     "i": torch.arange(len(k)).cuda()})
    m = shard.merge_runs(runs, "k")
    exp = _expect(runs)
    for c in exp:
        assert torch.equal(m[c].cpu(), exp[c]), c


def test_device_merge_full_key_span():
    """keys at both ends of int64 (the sample sort works on key - min over 64 bits)"""
    vals = [np.iinfo(np.int64).min, -1, 0, 1, np.iinfo(np.int64).max]
    runs = []
    for r in range(4):
        k = torch.tensor(sorted(vals[r:] + vals[:2]), dtype=torch.int64)
        runs.append({"k": k.cuda(), "run": torch.full((len(k),), r, dtype=torch.int32).cuda(),
                     "i": torch.arange(len(k)).cuda()})
    m = shard.merge_runs(runs, "k")
    exp = _expect(runs)
    for c in exp:
        assert torch.equal(m[c].cpu(), exp[c]), c


def test_device_merge_large_uniform_runs():
    """8 runs x 2M records of interleaved global positions (the C5 gather's shape: unique keys across ranks)"""
    G, n = 8, 2_000_000
    perm = torch.randperm(G * n, generator=torch.Generator().manual_seed(3))
    owner = perm % G
    runs = []
    for r in range(G):
        k = torch.nonzero(owner == r).flatten().to(torch.int64)
        runs.append({"k": k.cuda(), "e1": (k * 7).cuda(), "ts": (k // 100).cuda()})
    m = shard.merge_runs(runs, "k")
    total = sum(int(r["k"].numel()) for r in runs)
    assert torch.equal(m["k"].cpu(), torch.arange(total, dtype=torch.int64))
    assert torch.equal(m["e1"], m["k"] * 7) and torch.equal(m["ts"], m["k"] // 100)


def test_device_merge_rejects_bad_arguments():
    import siddhi_amd as sa
    k = torch.zeros(4, dtype=torch.int64, device="cuda")
    with pytest.raises(Exception):
        sa.merge_runs_device([k] * 33, [[]] * 33, torch.empty(132, dtype=torch.int64, device="cuda"), [])
