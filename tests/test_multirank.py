"""N>1 path on CPU: world-size-2 gloo run of the key-hash sharding (siddhi_amd/shard.py). Each rank runs its shard
of the trace through the generic keyed-NFA code (host build, tests/native) -- the GPU run of bench.py does the same
with the device kernel -- then the ranks' match streams are gathered and merged in global delivery order, and the
result must equal the oracle's single-process run of the whole trace. The batch-boundary match-count all-gather
of bench.py is exercised too."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import synth
from siddhi_amd import shard

APPS = ["c3_sequence_min1", "logical_and", "three_state_within"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emu_rt import EmuAdapter
        for name in APPS:
            tr = synth.trace(3000, keys=40, seed=21)
            owners = shard.route([row[1] for _, _, row in tr], world)
            mine = [i for i in range(len(tr)) if owners[i] == rank]
            e = EmuAdapter(synth.APPS[name], max_partials=256)
            recs = []
            try:
                for b in range(3):  # three batches, partials carried across
                    lo, hi = b * len(mine) // 3, (b + 1) * len(mine) // 3
                    for i in mine[lo:hi]:
                        s, ts, row = tr[i]
                        e.send(s, ts, row)
                    before = len(recs)
                    e.flush()
                    cur = [r for r in e.outputs() if r["kind"] == "query"]
                    recs = cur
                    cnt = torch.tensor([len(recs) - before], dtype=torch.int64)
                    allc = [torch.empty_like(cnt) for _ in range(world)]
                    dist.all_gather(allc, cnt)  # global output offsets of this batch
            finally:
                e.close()
            # local sequence number (position among this rank's sends, all streams) -> global position in the trace
            part = [(mine[r["seq"]], r["ordinal"], (r["name"], r["ts"], tuple(r["values"]))) for r in recs]
            parts = [None] * world
            dist.all_gather_object(parts, part)
            # the tensor path bench.py takes on the GPUs: per-rank sort, send/recv to rank 0, merge on the key
            g = shard.ordered_gather(dist, rank, world, {
                "gseq": torch.tensor([p[0] for p in part], dtype=torch.int64),
                "ord": torch.tensor([p[1] for p in part], dtype=torch.int64),
                "rank": torch.full((len(part),), rank, dtype=torch.int64),
                "idx": torch.arange(len(part), dtype=torch.int64)}, ["gseq", "ord"], first_key_unique=True)
            if rank == 0:
                merged = shard.merge(parts)
                tensor_merged = [parts[r][i][2] for r, i in zip(g["rank"].tolist(), g["idx"].tolist())]
                assert tensor_merged == merged
                with open(os.path.join(out_dir, name + ".txt"), "w") as f:
                    f.write(repr(merged))
    finally:
        dist.destroy_process_group()


def test_two_rank_key_sharding_matches_single_process(tmp_path, oracle_built, emu_built):
    from oracle_rt import Oracle
    mp.spawn(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for name in APPS:
        tr = synth.trace(3000, keys=40, seed=21)
        o = Oracle(synth.APPS[name])
        try:
            ref = synth.run(o, tr)
        finally:
            o.close()
        got = eval((tmp_path / (name + ".txt")).read_text())
        assert len(ref) > 0
        assert got == ref, name


def test_route_is_balanced_and_stable():
    keys = ["S%07d" % k for k in range(10_000)]
    r = shard.route(keys, 8)
    counts = [(r == i).sum() for i in range(8)]
    assert min(counts) > 1100 and max(counts) < 1400
    assert (shard.route(keys, 8) == r).all()


def test_merge_runs_is_a_stable_g_way_merge():
    """shard.merge_runs == a stable sort of the concatenation by (key, run), for G sorted runs with ties inside and
    across runs"""
    g = torch.Generator().manual_seed(5)
    runs = []
    for r in range(5):
        n = int(torch.randint(0, 400, (1,), generator=g))
        k = torch.sort(torch.randint(0, 300, (n,), generator=g)).values
        runs.append({"k": k, "run": torch.full((n,), r, dtype=torch.int64), "i": torch.arange(n),
                     "v": torch.stack([k * 3, k * 5])})
    m = shard.merge_runs(runs, "k")
    cat = {c: torch.cat([r[c] for r in runs], dim=-1) for c in runs[0]}
    order = shard.lexsort([cat["k"], cat["run"], cat["i"]])
    for c in cat:
        assert torch.equal(m[c], cat[c][..., order]), c


def test_sharded_runtime_runs_absent_states_whole_on_rank_0():
    """N > 1 semantics for absent queries: the reference's scheduler collapse is global across keys,
    so such a query is not key-sharded -- its streams go whole to rank 0 (with a warning); on one GPU it is a plain
    partitioned query"""
    import siddhi_amd as sa
    from siddhi_amd import workloads as w
    flags = sa.SiddhiAppRuntime(w.C4_APP, compile_only=True).query_flags()
    assert flags == [shard.Q_PARTITIONED | shard.Q_TIMERS]
    assert sa.SiddhiAppRuntime(w.C2_APP, compile_only=True).query_flags() == [shard.Q_PARTITIONED]
    assert sa.SiddhiAppRuntime(w.C1_APP, compile_only=True).query_flags() == [0]
    with pytest.warns(RuntimeWarning, match="absent states"):
        r1 = shard.ShardedAppRuntime(w.C4_APP, 1, 2, compile_only=True)
    with pytest.warns(RuntimeWarning, match="absent states"):
        r0 = shard.ShardedAppRuntime(w.C4_APP, 0, 2, compile_only=True)
    assert r1.whole_streams == set(w.C4_STREAMS) and not r1.key_attr
    assert all(r0.mine(s, [0, k, 1.0]) and not r1.mine(s, [0, k, 1.0]) for s in w.C4_STREAMS for k in range(50))
    rt = shard.ShardedAppRuntime(w.C4_APP, 0, 1, compile_only=True)
    assert rt.sharded
    s2 = shard.ShardedAppRuntime(w.C2_APP, 1, 4, compile_only=True, key_attr={"StockStream": 1})
    keys = ["S%05d" % k for k in range(2000)]
    mine = [k for k in keys if s2.mine("StockStream", [0, k, 1.0, 1])]
    assert mine == [k for k in keys if shard.owner(k, 4) == 1]
    r1 = shard.ShardedAppRuntime(w.C1_APP, 1, 2, compile_only=True)
    assert "StockStream" in r1.whole_streams and not r1.mine("StockStream", [0, "IBM", 1.0, 1])


def test_sharded_runtime_mixed_partitioned_and_unpartitioned_queries():
    """a stream read by both a partitioned and an unpartitioned query cannot be key-sharded; the
    app then runs whole on rank 0 WITH a warning. Streams only unpartitioned queries read go to rank 0 whole while
    the partitioned queries' streams stay sharded."""
    import warnings
    defs = "define stream S (id long, k string, p double); define stream T (id long, k string, p double); "
    part = "partition with (k of S) begin @info(name='qp') from every e1=S -> e2=S select e1.id as a insert into O1; end; "
    mixed = defs + part + "@info(name='qu') from every e1=S -> e2=S select e1.id as a insert into O2;"
    with pytest.warns(RuntimeWarning, match="cannot be key-sharded"):
        m = shard.ShardedAppRuntime(mixed, 1, 2, compile_only=True)
    assert m.replica and not m.mine("S", [0, "a", 1.0]) and not m.mine("S", [0, "b", 1.0])
    sep = defs + part + "@info(name='qu') from every e1=T -> e2=T select e1.id as a insert into O2;"
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        s0 = shard.ShardedAppRuntime(sep, 0, 2, compile_only=True)
        s1 = shard.ShardedAppRuntime(sep, 1, 2, compile_only=True)
    assert not s1.replica and s1.whole_streams == {"T"} and s1.key_attr == {"S": 1}
    keys = ["x%d" % i for i in range(200)]
    assert all(s0.mine("S", [0, k, 1.0]) != s1.mine("S", [0, k, 1.0]) for k in keys)  # S sharded
    assert all(s0.mine("T", [0, k, 1.0]) and not s1.mine("T", [0, k, 1.0]) for k in keys)  # T whole on rank 0


def test_route_float32_keys_like_per_row_send():
    """send() and send_columns() must route a float32 key alike -- the columnar path hashes the numpy
    scalars (str(np.float32(0.1)) == '0.1'), not Python floats widened to double ('0.10000000149011612')"""
    import numpy as np
    defs = "define stream S (id long, k float, p double); "
    app = defs + "partition with (k of S) begin @info(name='q') from every e1=S -> e2=S select e1.id as a insert into O; end;"
    r = shard.ShardedAppRuntime(app, 1, 3, compile_only=True)
    ks = np.round(np.random.default_rng(5).uniform(0, 10, 3000), 2).astype(np.float32)
    cols = shard.route(ks, 3, {})
    rows = [1 if r.mine("S", [0, k, 0.0]) else 0 for k in ks]
    assert [int(x == 1) for x in cols] == rows
    assert cols.tolist() == [shard.owner(str(k), 3) for k in ks]
    assert any(shard.owner(str(k), 3) != shard.owner(str(float(k)), 3) for k in ks)  # the old bug would show


def test_sharded_runtime_routes_by_the_engines_partition_attribute():
    """the router takes each stream's key attribute from the engine (sdg_query_key_attr), refuses a
    caller's key_attr that disagrees, runs a stream keyed by two attributes and broadcast streams whole on rank 0 at
    N > 1 (warned), and routes columnar batches at once (route over the distinct keys)"""
    import numpy as np
    import siddhi_amd as sa
    import synth
    from siddhi_amd import workloads as w
    s = shard.ShardedAppRuntime(w.C2_APP, 1, 4, compile_only=True)
    assert s.key_attr == {"StockStream": 1}
    assert s.rt.query_key_attr(0, "StockStream") == 1
    with pytest.raises(sa.OperationNotSupportedException):
        shard.ShardedAppRuntime(w.C2_APP, 1, 4, compile_only=True, key_attr={"StockStream": 0})
    two = ("define stream S (id long, a string, b string); partition with (a of S) begin @info(name='q1') "
           "from every e1=S -> e2=S select e1.id as x insert into O1; end; partition with (b of S) begin "
           "@info(name='q2') from every e1=S -> e2=S select e1.id as x insert into O2; end;")
    assert shard.ShardedAppRuntime(two, 0, 1, compile_only=True).key_attr  # one GPU: fine
    # N > 1: no single owner GPU for S's events -> both queries run whole on rank 0 (warned), never refused
    for rank in (0, 1):
        with pytest.warns(RuntimeWarning, match="keyed by different attributes"):
            t = shard.ShardedAppRuntime(two, rank, 2, compile_only=True)
        assert t.whole_streams == {"S"} and not t.key_attr and set(t.whole_queries) == {"q1", "q2"}
        assert all(t.mine("S", [0, "a%d" % i, "b%d" % i]) == (rank == 0) for i in range(100))
    bc = synth.BCAST_APPS["bc_pattern"]
    assert sa.SiddhiAppRuntime(bc, compile_only=True).query_flags() == [shard.Q_PARTITIONED | shard.Q_BROADCAST]
    assert sa.SiddhiAppRuntime(bc, compile_only=True).query_key_attr(0, "T") == -3
    for rank in (0, 1):
        with pytest.warns(RuntimeWarning, match="without a partition key"):
            b = shard.ShardedAppRuntime(bc, rank, 2, compile_only=True)
        assert not b.key_attr and b.whole_streams and all(b.mine(st, [0, 1, 1.0]) == (rank == 0)
                                                          for st in b.whole_streams)
    rg = synth.RANGE_APPS["range_overlap"]
    for rank in (0, 1):
        with pytest.warns(RuntimeWarning, match="range partitions"):
            g = shard.ShardedAppRuntime(rg, rank, 2, compile_only=True)
        assert g.whole_streams == {"S", "T"} and not g.key_attr
        assert all(g.mine(st, [0, "k", 50.0, 90]) == (rank == 0) for st in ("S", "T"))
    keys = np.array(["S%05d" % k for k in np.random.default_rng(3).integers(0, 5000, 20000)])
    r = shard.route(keys, 4)
    assert r.tolist() == [shard.owner(k, 4) for k in keys.tolist()]
    ints = np.random.default_rng(4).integers(-10**12, 10**12, 5000)
    assert shard.route(ints, 3).tolist() == [shard.owner(int(k), 3) for k in ints.tolist()]


def test_ordered_gather_checks_its_merge_precondition():
    import torch
    with pytest.raises(ValueError):
        shard.ordered_gather(None, 0, 1, {"a": torch.zeros(3), "b": torch.zeros(3)}, ["a", "b"])


def _c4_rank_main(rank, world, port, out_dir, keys):
    import warnings
    import numpy as np
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from siddhi_amd import workloads as w
        from test_c4_host import c4_slots
        from emu_rt import EmuAdapter
        c = w.c4_columns(keys, per_tick=keys // 100)
        end = int(c["ts"][-1]) + 5000
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            router = shard.ShardedAppRuntime(w.C4_APP, rank, world, compile_only=True)
        streams = np.array(w.C4_STREAMS)[c["stream"]]
        mine = np.array([router.mine(s, [0, int(k), 0.0]) for s, k in zip(streams, c["key"])])
        idx = np.nonzero(mine)[0]
        e = EmuAdapter(w.C4_APP)
        try:
            sidx = np.array([e.L.emu_stream_index(e.h, s.encode()) for s in w.C4_STREAMS], dtype=np.int32)[c["stream"][idx]]
            slots = np.ascontiguousarray(c4_slots(c)[idx])
            offs = np.arange(len(idx), dtype=np.int64) * 3
            tsa = np.ascontiguousarray(c["ts"][idx])
            if len(idx):
                e.L.emu_send_batch(e.h, len(idx), sidx.ctypes.data, tsa.ctypes.data, offs.ctypes.data, slots.ctypes.data,
                                   None)
            e.flush()
            e.advance(end)  # every rank's clock reaches the end (the batch-boundary watermark)
            e.flush()
            recs = [(r["ts"], tuple(v[1] for v in r["values"])) for r in e.outputs() if r["kind"] == "query"]
        finally:
            e.close()
        parts = [None] * world
        dist.all_gather_object(parts, (int(mine.sum()), recs))
        if rank == 0:
            assert parts[1][0] == 0 and not parts[1][1]  # the timer query's streams are not sharded
            with open(os.path.join(out_dir, "c4.txt"), "w") as f:
                f.write(repr(parts[0][1]))
    finally:
        dist.destroy_process_group()


def test_two_rank_absent_app_equals_single_process(tmp_path, oracle_built, emu_built):
    """the C4 app at 2*10^4 keys on a world-2 run is no longer refused; its streams go
    whole to rank 0 (shard.ShardedAppRuntime), so the merged output equals the single-process oracle -- the case where
    a naive key split changes the result (7,857 vs 9,790 matches)"""
    from siddhi_amd import workloads as w
    from test_c4_host import oracle_c4
    keys = 20_000
    mp.spawn(_c4_rank_main, args=(2, _free_port(), str(tmp_path), keys), nprocs=2, join=True)
    c = w.c4_columns(keys, per_tick=keys // 100)
    ots, ovals, _ = oracle_c4(c, int(c["ts"][-1]) + 5000)
    ref = [(int(t), tuple(int(x) for x in v)) for t, v in zip(ots, ovals)]
    got = eval((tmp_path / "c4.txt").read_text())
    assert len(ref) > 1000 and got == ref
