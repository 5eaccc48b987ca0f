"""N = 2 key-hash sharding through the GPU engine itself (the CPU gloo test runs
the host emulator). Two processes on one GPU (gloo for the collectives, CPU tensors), each running its shard of a
trace through the product kernels -- fused chain matcher, register sequence kernel, generic keyed NFA -- in three
flushes; the ranks' records go through shard.ordered_gather and must equal the single-process GPU run of the whole
trace and the oracle's single-process run of it, record by record and in delivery order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import synth
from siddhi_amd import shard

pytestmark = pytest.mark.gpu

APPS = ["c3_sequence_min1", "logical_and", "chain_gt"]


def _app(name):
    return synth.CHAIN_APPS["gt"][0] if name == "chain_gt" else synth.APPS[name]


def _trace():
    return synth.trace(6000, keys=60, seed=23, two_streams=True)


def _run(app, rows, batches=3):
    """rows: [(stream, ts, values)] -> [(local position, ts, value tuple)] in delivery order"""
    import siddhi_amd as sa
    rt = sa.SiddhiAppRuntime(app, device=0)
    out = []
    try:
        hs = {}
        bounds = np.linspace(0, len(rows), batches + 1).astype(int)
        for b in range(batches):
            for s, ts, vals in rows[bounds[b]:bounds[b + 1]]:
                if s not in hs:
                    hs[s] = rt.getInputHandler(s)
                hs[s].send(ts, vals)
            rt.flush(deliver=False)
            ts, v, nl, seq = rt.poll_arrays(0)
            for i in range(len(ts)):
                out.append((int(seq[i]), int(ts[i]), tuple(None if nl[j][i] else int(v[j][i]) for j in range(len(v)))))
    finally:
        rt.shutdown()
    return out


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.init()  # torch's HIP runtime first, then the engine's
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = _trace()
        owners = shard.route([row[1] for _, _, row in tr], world)
        mine = [i for i in range(len(tr)) if owners[i] == rank]
        for name in APPS:
            recs = _run(_app(name), [tr[i] for i in mine])
            g = shard.ordered_gather(dist, rank, world, {
                "gseq": torch.tensor([mine[r[0]] for r in recs], dtype=torch.int64),
                "rank": torch.full((len(recs),), rank, dtype=torch.int64),
                "idx": torch.arange(len(recs), dtype=torch.int64)}, ["gseq", "rank", "idx"])
            parts = [None] * world
            dist.all_gather_object(parts, [(mine[r[0]],) + r[1:] for r in recs])
            if rank == 0:
                merged = [parts[r][i] for r, i in zip(g["rank"].tolist(), g["idx"].tolist())]
                with open(os.path.join(out_dir, name + ".txt"), "w") as f:
                    f.write(repr(merged))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gpu_sharding_matches_single_gpu_run(tmp_path, oracle_built):
    from oracle_rt import Oracle
    mp.spawn(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    tr = _trace()
    for name in APPS:
        single = _run(_app(name), tr)
        o = Oracle(_app(name))
        try:
            ref = synth.run(o, tr)
        finally:
            o.close()
        got = eval((tmp_path / (name + ".txt")).read_text())
        # the oracle's rows as (ts, payloads): every select item of these apps is a long id
        want = [(ts, tuple(None if v is None else v[1] for v in vals)) for _, ts, vals in ref]
        assert len(ref) > 50, name
        assert [r[1:] for r in single] == want, name
        assert [r[1:] for r in got] == want, name
        assert got == single, name
