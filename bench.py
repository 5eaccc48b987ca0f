#!/usr/bin/env python3
"""Headline benchmark: input events/s through the pattern NFA path on MI355X (BASELINE.json metric).

Workload (the 1-GPU config the metric is quoted on):
    partition with (symbol of StockStream) begin
      from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec
      select e1.id as e1id, e2.id as e2id insert into M; end;
    100,000,000 events per GPU per step, 10,000 keys per GPU, ts = T0 + floor(i/100) (splitmix64, synthetic).
A step = one flush of one 100M-event batch, inputs already resident in HBM (sdg_push_device); consecutive steps
are consecutive batches of one stream (timestamps continue), so partials crossing a batch boundary are carried.

Multi-GPU (torchrun, one process per GPU): key-hash sharding (siddhi_amd/shard.py), each rank generates the events
of the keys it owns; no data-path
collective — only the batch-boundary all-gather of per-rank match counts (RCCL over xGMI). scaling = weak.

Roofline: algorithmic bytes per step B = N_in*28 + N_match*28 (ts 8 + key 4 + price 8 + id 8 in,
ts 8 + key 4 + two ids out). The dominant kernel is launched once per step and covers the whole batch, so its
algorithmic bytes per launch are B; achieved = B / its average launch duration (HIP events recorded on the engine
stream around that launch). traffic = HBM bytes per launch of that kernel from the committed rocprofv3 --pmc passes
(profiles/pmc_traffic.json: FETCH_SIZE doubled per the gfx950 note of the MI355X guide, plus WRITE_SIZE).
CPU baseline: the oracle (C++ restatement of the reference engine, one core) on a bounded sample of the same
workload.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

B_IN = 28
B_OUT = 28
HBM_PEAK_GBS = 8000.0


T_START = time.time()


def log(msg):
    """progress on stderr (the JSON line is the only stdout output)"""
    print("[bench %6.1fs] %s" % (time.time() - T_START, msg), file=sys.stderr, flush=True)


def gen_shard(n, keys, rank, world, seed=7):
    """C2 columns of this rank's shard (numpy, chunked to bound host memory)."""
    from siddhi_amd import workloads as w
    out = {k: [] for k in ("ts", "id", "key", "price", "volume")}
    chunk = 10_000_000
    for off in range(0, n, chunk):
        m = min(chunk, n - off)
        c = w.c2_columns(m, keys=keys, seed=seed + 1000 * rank, offset=off)
        for k in out:
            out[k].append(c[k])
    return {k: np.concatenate(v) for k, v in out.items()}


def end_to_end(cols, syms, n, steps, device):
    """host SoA push -> flush -> poll of every match to host memory, per step (PCIe both ways, host assembly and
    the delivery-order sort included): the rate a host application sees, beside the device-resident value"""
    import siddhi_amd as sa
    from siddhi_amd import workloads as w
    rt = sa.SiddhiAppRuntime(w.C2_APP, device=device, batch_capacity=n + 1)
    sym_ids = np.array([rt.intern(s) for s in syms], dtype=np.uint32)
    h = rt.getInputHandler("StockStream")
    symcol = sym_ids[cols["key"][:n]]
    span = int(cols["ts"][n - 1] - cols["ts"][0]) + 1
    data = [cols["id"][:n], symcol, cols["price"][:n], cols["volume"][:n]]
    # the application's timestamps of each step (made before the clock starts: producing input is not the engine's)
    warm = 2  # first-use allocations (staging, output, pinned buffers; the two poll buffers that alternate)
    tss = [cols["ts"][:n] + s * span for s in range(steps + warm)]
    for s in range(warm):
        h.send_columns(tss[s], data)
        rt.flush(deliver=False)
        rt.poll_arrays(0, copy=False)
    rows, ph = 0, [0.0, 0.0, 0.0]
    t = time.perf_counter()
    for s in range(warm, steps + warm):
        t0 = time.perf_counter()
        h.send_columns(tss[s], data)
        t1 = time.perf_counter()
        rt.flush(deliver=False)
        t2 = time.perf_counter()
        ts, vals, nulls, seq = rt.poll_arrays(0, copy=False)  # the delivered columns, in place until the next poll
        t3 = time.perf_counter()
        ph[0] += t1 - t0
        ph[1] += t2 - t1
        ph[2] += t3 - t2
        rows += len(ts)
    dt = time.perf_counter() - t
    rt.shutdown()
    return {"value": n * steps / dt, "unit": "events/s", "ms_per_step": dt * 1000 / steps, "events_per_step": n,
            "matches_delivered_per_step": rows / steps, "warmup_steps": warm,
            "ms_push": ph[0] * 1000 / steps, "ms_flush": ph[1] * 1000 / steps, "ms_poll": ph[2] * 1000 / steps,
            "path": "host columns (sdg_push) -> device flush -> sdg_poll into host arrays, delivery order"}


def cpu_baseline(cols, syms, sample):
    """Oracle (reference-semantics C++ restatement, single thread) on the first `sample` events."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_rt import Oracle, lib
    from siddhi_amd import workloads as w
    o = Oracle(w.C2_APP)
    L = lib()
    L.orc_count_only(o.h, 1)
    ids = np.array([L.orc_intern(o.h, s.encode()) for s in syms], dtype=np.int64)
    si = o.stream("StockStream")
    n = sample
    slots = np.empty((n, 4), dtype=np.int64)
    slots[:, 0] = cols["id"][:n]
    slots[:, 1] = ids[cols["key"][:n]]
    slots[:, 2] = cols["price"][:n].view(np.int64)
    slots[:, 3] = cols["volume"][:n]
    offs = np.arange(n, dtype=np.int64) * 4
    strm = np.full(n, si, dtype=np.int32)
    ts = np.ascontiguousarray(cols["ts"][:n])
    t = time.perf_counter()
    rc = L.orc_send_batch(o.h, n, strm.ctypes.data, ts.ctypes.data, offs.ctypes.data, slots.ctypes.data, None)
    dt = time.perf_counter() - t
    matches = L.orc_output_count(o.h)
    o.close()
    if rc != 0:
        raise RuntimeError("oracle failed")
    return n / dt, matches, dt


def parity_check(cols, syms, sample, dev_cols, device, flushes=3):
    """Outside the timed region: the first `sample` events of this rank's bench stream through a fresh runtime on
    the GPU (device-resident, the bench's own path, in `flushes` consecutive batches like the timed steps, so
    partials are carried across batch boundaries at the bench's ~10 events per key-window) and through the oracle;
    the match rows (ts, e1id, e2id) must be identical and in the same delivery order, or the bench fails."""
    import siddhi_amd as sa
    from siddhi_amd import workloads as w
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_rt import Oracle, lib
    n = sample
    rt = sa.SiddhiAppRuntime(w.C2_APP, device=device)
    sym_ids = np.array([rt.intern(s) for s in syms], dtype=np.uint32)
    d_id, d_sym, d_price, d_vol, d_ts = dev_cols
    assert int(sym_ids[cols["key"][0]]) == int(d_sym[0].item())  # same dictionary ids as the bench runtime
    parts, carried = [], 0
    bounds = np.linspace(0, n, flushes + 1).astype(np.int64)
    for f in range(flushes):
        lo, hi = int(bounds[f]), int(bounds[f + 1])
        rt.push_device("StockStream", hi - lo, d_ts[lo:].data_ptr(), [d_id[lo:].data_ptr(), d_sym[lo:].data_ptr(),
                                                                      d_price[lo:].data_ptr(), d_vol[lo:].data_ptr()])
        rt.flush(deliver=False)
        carried += rt.stats().carry_in
        parts.append(rt.poll_arrays(0))
    rt.shutdown()
    gts = np.concatenate([p[0] for p in parts])
    gvals = np.concatenate([p[1] for p in parts], axis=1)
    gnulls = np.concatenate([p[2] for p in parts], axis=1)
    o = Oracle(w.C2_APP)
    L = lib()
    ids = np.array([L.orc_intern(o.h, s.encode()) for s in syms], dtype=np.int64)
    slots = np.empty((n, 4), dtype=np.int64)
    slots[:, 0] = cols["id"][:n]
    slots[:, 1] = ids[cols["key"][:n]]
    slots[:, 2] = cols["price"][:n].view(np.int64)
    slots[:, 3] = cols["volume"][:n]
    strm = np.full(n, o.stream("StockStream"), dtype=np.int32)  # named: temporaries die before the call
    tsa = np.ascontiguousarray(cols["ts"][:n])
    offs = np.arange(n, dtype=np.int64) * 4
    rc = L.orc_send_batch(o.h, n, strm.ctypes.data, tsa.ctypes.data, offs.ctypes.data, slots.ctypes.data, None)
    if rc != 0:
        raise RuntimeError("oracle failed")
    ots, ovals, onulls = o.query_arrays(2)
    o.close()
    ok = (len(gts) == len(ots) and np.array_equal(gts, ots) and np.array_equal(gvals.T, ovals)
          and not gnulls.any() and not onulls.any())
    if not ok:
        raise RuntimeError("GPU match rows differ from the oracle on the first %d bench events (%d vs %d rows)"
                           % (n, len(gts), len(ots)))
    return {"events": n, "matches": int(len(ots)), "bit_exact": True, "flushes": flushes,
            "partials_carried_across_flushes": int(carried)}


def cpu_baseline_sharded(cols, syms, sample, threads):
    """The same oracle, key-sharded over `threads` host threads (one Oracle instance per shard; keys are
    independent). ctypes drops the GIL inside orc_send_batch, so the shards run in parallel."""
    import threading
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_rt import Oracle, lib
    from siddhi_amd import workloads as w
    L = lib()
    n = sample
    key = cols["key"][:n]
    jobs = []
    for sh in range(threads):
        idx = np.nonzero(key % threads == sh)[0]
        o = Oracle(w.C2_APP)
        L.orc_count_only(o.h, 1)
        ids = np.array([L.orc_intern(o.h, s.encode()) for s in syms], dtype=np.int64)
        m = len(idx)
        slots = np.empty((m, 4), dtype=np.int64)
        slots[:, 0] = cols["id"][idx]
        slots[:, 1] = ids[key[idx]]
        slots[:, 2] = cols["price"][idx].view(np.int64)
        slots[:, 3] = cols["volume"][idx]
        jobs.append({"o": o, "m": m, "slots": slots, "offs": np.arange(m, dtype=np.int64) * 4,
                     "strm": np.full(m, o.stream("StockStream"), dtype=np.int32),
                     "ts": np.ascontiguousarray(cols["ts"][idx]), "rc": -1})

    def work(j):
        j["rc"] = L.orc_send_batch(j["o"].h, j["m"], j["strm"].ctypes.data, j["ts"].ctypes.data,
                                   j["offs"].ctypes.data, j["slots"].ctypes.data, None)

    ths = [threading.Thread(target=work, args=(j,)) for j in jobs]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t
    matches = sum(L.orc_output_count(j["o"].h) for j in jobs)
    for j in jobs:
        j["o"].close()
    if any(j["rc"] != 0 for j in jobs):
        raise RuntimeError("oracle failed")
    return n / dt, matches, dt


def ordered_gather_leg(rt, step_push, n, dev, dist, rank, world):
    """The ordered result gather of one batch: each rank's match records exported device-to-device already in its
    delivery order (sdg_export_ordered: the engine's device ordering pass), sent to rank 0 over RCCL (send/recv) and
    merged there into the single delivery order of the combined stream: (event time, rank, position of the emitting
    event in its rank's stream, ordinal) -- a rank's delivery order is already sorted by event time, so the merge is
    a G-way merge of the runs by time (shard.merge_runs: the device merge sdg_merge_runs, no re-sort). Rank 0 checks
    the merged order."""
    import torch
    from siddhi_amd import shard
    cap = n + n // 4 + 4096
    t_ts = torch.empty(cap, dtype=torch.int64, device=dev)
    t_seq = torch.empty(cap, dtype=torch.int64, device=dev)
    t_sub = torch.empty(cap, dtype=torch.int64, device=dev)
    t_vals = torch.empty((2, cap), dtype=torch.int64, device=dev)
    t_rank = torch.full((cap,), rank, dtype=torch.int64, device=dev)  # the merge key's rank column
    # one untimed export first: the ordering pass sizes its workspaces on first use (device allocations)
    step_push()
    rt.flush(deliver=False)
    rt.export_ordered(0, cap, t_ts.data_ptr(), t_seq.data_ptr(), t_sub.data_ptr(), t_vals.data_ptr())
    step_push()
    rt.flush(deliver=False)
    key = ["ts", "rank", "seq", "sub"]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cnt = rt.export_ordered(0, cap, t_ts.data_ptr(), t_seq.data_ptr(), t_sub.data_ptr(), t_vals.data_ptr())
    recs = {"ts": t_ts[:cnt], "seq": t_seq[:cnt], "sub": t_sub[:cnt],
            "rank": t_rank[:cnt], "vals": t_vals[:, :cnt]}
    gph = {"export": time.perf_counter() - t0, "transfer": 0.0, "merge": 0.0}
    if dist is None:
        merged = recs
    else:
        merged = shard.ordered_gather(dist, rank, world, recs, key, presorted=True, timings=gph)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank != 0:
        return None
    total = int(merged["ts"].numel())
    ok = True
    if total > 1:  # lexicographic non-decreasing on the key (strictly increasing: records are distinct)
        less = torch.zeros(total - 1, dtype=torch.bool, device=dev)
        eq = torch.ones(total - 1, dtype=torch.bool, device=dev)
        for k in key:
            a, b = merged[k][:-1], merged[k][1:]
            less |= eq & (a < b)
            eq &= a == b
        ok = bool(less.all().item())
    if not ok:
        raise RuntimeError("ordered gather: merged records are not in delivery order")
    return {"records": total, "ms": dt * 1000.0, "rank0_ms": {k: v * 1000.0 for k, v in gph.items()},
            "bytes_to_rank0": int((total - cnt) * 8 * 6),
            "key": "(event ts, rank, event position in its rank's stream, ordinal)", "ordered": True,
            "path": "sdg_export_ordered (per-rank device ordering) -> RCCL send/recv to rank 0 -> device G-way "
                    "merge of the sorted runs by time (shard.merge_runs, sdg_merge_runs)"}


def c5_cpu_baseline(sh, nkeys=100_000):
    """The oracle (one core, count-only) on a bounded sample of this rank's C5 shard: the events of `nkeys` of its keys
    in the first global batch (keys are independent: the same per-key streams the GPU processes)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_rt import Oracle, lib
    from siddhi_amd import workloads as w
    skeys, smap = sh.sample(nkeys)
    g0, g1 = sh.global_range(0)
    ev = sh.sample_events(smap, len(skeys), g0, g1)
    o = Oracle(w.C2_APP)
    L = lib()
    L.orc_count_only(o.h, 1)
    oid = np.array([L.orc_intern(o.h, ("S%08d" % k).encode()) for k in skeys], dtype=np.int64)
    n = len(ev["ts"])
    slots = np.empty((n, 4), dtype=np.int64)
    slots[:, 0] = ev["id"]
    slots[:, 1] = oid[ev["sym"]]
    slots[:, 2] = ev["price"].view(np.int64)
    slots[:, 3] = ev["volume"]
    strm = np.full(n, o.stream("StockStream"), dtype=np.int32)
    ts = np.ascontiguousarray(ev["ts"])
    offs = np.arange(n, dtype=np.int64) * 4
    t = time.perf_counter()
    rc = L.orc_send_batch(o.h, n, strm.ctypes.data, ts.ctypes.data, offs.ctypes.data, slots.ctypes.data, None)
    dt = time.perf_counter() - t
    m = L.orc_output_count(o.h)
    o.close()
    if rc != 0:
        raise RuntimeError("oracle failed")
    return {"value": n / dt, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": "%d events of %d of this rank's keys in global batch 0 (%.2f s, %d matches), oracle restatement"
                      % (n, len(skeys), dt, m)}


def run_c5(args, rank, world, local, dist):
    """C5 (BASELINE.json configs[4]): the C2 query over the 10^10-event / 10^8-key stream, key-hash sharded, every rank
    generating its shard on its GPU (siddhi_amd/c5.py) in batches of 2^28 of its own events. A step = one rank flush
    of one batch, inputs resident in HBM (all batches of the run are generated before the timed region). value =
    events of every rank's timed flushes / max-over-ranks time. Outside the timed region: the ordered result gather
    of one more batch to rank 0 (RCCL send/recv, G-way merge on the global position of the emitting event) and a
    10^4-key oracle sample of this rank's shard (tests/c5_check.py)."""
    import torch
    import siddhi_amd as sa
    from siddhi_amd import c5, shard
    from siddhi_amd import workloads as w
    dev = torch.device("cuda", local)
    srank, sworld = rank, world
    if args.c5_shard:  # one rank's shard of a larger run, measured on this one GPU
        if world > 1:
            raise SystemExit("--c5-shard is for a single process")
        srank, sworld = (int(x) for x in args.c5_shard.split("/"))
    rt = sa.SiddhiAppRuntime(w.C2_APP, device=local)
    log("C5: interning this rank's keys (shard %d/%d)" % (srank, sworld))
    sh = c5.C5Shard(rt, srank, sworld, dev, events=args.c5_events, batch=args.c5_batch)
    nb = sh.n_batches()
    nsteps = args.warmup + args.steps
    if nsteps > nb:
        raise SystemExit("C5: %d batches in the stream at this world size, %d requested" % (nb, nsteps))
    log("C5: %d keys on this rank; generating %d batches of ~%d events" % (sh.n_keys, nsteps, args.c5_batch))
    batches = [sh.generate(j) for j in range(nsteps)]
    torch.cuda.synchronize()

    def push(j):
        cols, n = batches[j]
        rt.push_device("StockStream", n, cols["ts"].data_ptr(), [cols["id"].data_ptr(), cols["sym"].data_ptr(),
                                                                cols["price"].data_ptr(), cols["volume"].data_ptr()])
        return n

    # the ordered result gather is part of the C5 step: the flush's records leave the engine already in delivery
    # order (sdg_export_ordered), go to rank 0 over RCCL (send/recv) and are merged there on e2id (the global position
    # of the emitting event: unique across ranks; shard.merge_runs)
    gcap = args.c5_batch // 2 + (1 << 20)
    g_ts = torch.empty(gcap, dtype=torch.int64, device=dev)
    g_vals = torch.empty((2, gcap), dtype=torch.int64, device=dev)
    last_merged = [None]

    gph = {"export": 0.0, "transfer": 0.0, "merge": 0.0}

    def gather():
        t = time.perf_counter()
        # (the merge key is (e2id, e1id): the engine's own position columns are not exported)
        cnt = rt.export_ordered(0, gcap, g_ts.data_ptr(), 0, 0, g_vals.data_ptr())
        recs = {"e2": g_vals[1, :cnt], "e1": g_vals[0, :cnt], "ts": g_ts[:cnt]}
        gph["export"] += time.perf_counter() - t
        if dist is None:
            merged = recs
        else:
            merged = shard.ordered_gather(dist, rank, world, recs, ["e2", "e1"], presorted=True, first_key_unique=True,
                                          timings=gph)
        last_merged[0] = merged
        return cnt

    def step(j):
        """one flush (its records stay on the device for the gather that follows)"""
        n = push(j)
        rt.flush(deliver=False)
        st = rt.stats()
        if dist is not None:  # batch-boundary match-count all-gather (global output offsets)
            cnt = torch.tensor([st.matches], dtype=torch.int64, device=dev)
            allc = [torch.empty_like(cnt) for _ in range(world)]
            dist.all_gather(allc, cnt)
        if args.no_gather:
            rt.discard()
        return n, st

    log("C5: warm-up (%d flushes)" % args.warmup)
    for j in range(args.warmup):
        step(j)
        if not args.no_gather:
            gather()
    for k in gph:
        gph[k] = 0.0
    keys_k = ["ms_kg_hist", "ms_kg_prefix", "ms_kg_scatter", "ms_chain_carry", "ms_chain_match", "ms_chain_emit"]
    acc = {k: 0.0 for k in keys_k}
    events = matches = carries = 0
    t_flush = 0.0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(args.warmup, nsteps):
        tf = time.perf_counter()
        n, st = step(j)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t_flush += time.perf_counter() - tf  # (the flush phase; then the gather of the same batch)
        if not args.no_gather:
            gather()
        events += n
        matches += st.matches
        carries += st.carry_in
        for k in keys_k:
            acc[k] += getattr(st, k)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tot_events, tot_matches = events, matches
    if dist is not None:
        t = torch.tensor([elapsed, t_flush], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, t_flush = float(t[0].item()), float(t[1].item())
        v = torch.tensor([events, matches], dtype=torch.int64, device=dev)
        dist.all_reduce(v)
        tot_events, tot_matches = int(v[0].item()), int(v[1].item())
    K = args.steps
    per_kernel = {k: acc[k] / K for k in keys_k}
    dom = max(per_kernel, key=per_kernel.get)
    step_bytes = (events * B_IN + matches * B_OUT) / K  # this rank's algorithmic bytes per flush
    achieved = step_bytes / (per_kernel[dom] / 1000.0) / 1e9
    names = {"ms_kg_scatter": "rx_scatter (all radix passes of the flush)", "ms_chain_match": "chain_deque_k",
             "ms_chain_emit": "chain_match_k (emission)", "ms_chain_carry": "chain_carry_wave_k", "ms_kg_hist": "rx_hist",
             "ms_kg_prefix": "rx_p1/p2/p3"}
    out = {
        "metric": "input events/sec matched (node) at 1/2/4/8 MI355X; % HBM roofline",
        "value": tot_events / elapsed, "unit": "events/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
        "ms_per_step": elapsed * 1000.0 / K, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (splitmix64 C5 generator on the GPU, siddhi_amd/c5.py), device-resident",
        "config": {"workload": "C5: C2 query, %d events / 10^8 keys key-hash sharded over %d GPU(s)%s, batches of "
                               "%d rank events; a step = flush + ordered result gather to rank 0" % (
                                   args.c5_events, sworld, "" if sworld == world else
                                   " (shard %d of %d measured on this GPU)" % (srank, sworld), args.c5_batch),
                   "keys_this_rank": sh.n_keys, "events_per_rank_step": events / K, "matches_per_step": tot_matches / K,
                   "carried_partials_per_rank_step": carries / K,
                   "parallelism": "key-hash shards x%d" % sworld, "path": "radix key sort + chain kernels"},
        "without_gather": {"value": tot_events / t_flush, "ms_per_step": t_flush * 1000.0 / K},
        "gather": None if args.no_gather else {
            "ms_per_step": (elapsed - t_flush) * 1000.0 / K, "inside_step": True,
            "records_per_rank_step": matches / K,
            "rank0_ms_per_step": {k: v * 1000.0 / K for k, v in gph.items()},
            "key": "(e2id = global position of the emitting event, e1id)",
            "path": "sdg_export_ordered (device ordering) -> RCCL send/recv to rank 0 -> device G-way merge of the "
                    "sorted runs on e2id (shard.merge_runs, sdg_merge_runs)"},
        "roofline": {"bound": "hbm", "kernel": names.get(dom, dom), "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_launch": step_bytes,
                     "step_frac": step_bytes / (t_flush / K) / 1e9 / HBM_PEAK_GBS, "kernel_ms": per_kernel},
        "cpu_baseline": None,
    }
    tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):  # PMC HBM bytes per launch of the dominant kernel at this batch size, if measured
        ent = json.load(open(tpath)).get("c5", {}).get(names.get(dom, dom).split(" ")[0])
        if ent and ent.get("events_per_launch") == args.c5_batch:
            out["roofline"]["traffic"] = ent["fetch_bytes"] + ent["write_bytes"]
    if rank == 0 and last_merged[0] is not None:  # the last step's merged records are in delivery order
        e2, e1 = last_merged[0]["e2"], last_merged[0]["e1"]
        ok = bool(((e2[1:] > e2[:-1]) | ((e2[1:] == e2[:-1]) & (e1[1:] > e1[:-1]))).all().item()) \
            if e2.numel() > 1 else True
        if not ok:
            raise RuntimeError("C5 ordered gather: merged records are not in delivery order")
        out["gather"]["ordered"] = True
        out["gather"]["records_merged_last_step"] = int(e2.numel())
    last_merged[0] = None
    del batches, g_ts, g_vals
    torch.cuda.empty_cache()
    if rank == 0 and not args.no_cpu:
        out["cpu_baseline"] = c5_cpu_baseline(sh)
    if not args.no_parity:
        log("C5: oracle sample of this rank's shard (%d keys)" % args.c5_sample)
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from c5_check import delivery_order, oracle_sample_rows, sample_records
        rt.shutdown()
        rt = sa.SiddhiAppRuntime(w.C2_APP, device=local)  # a fresh run of the same stream prefix
        sh2 = c5.C5Shard(rt, srank, sworld, dev, events=args.c5_events, batch=args.c5_batch)
        skeys, smap = sh2.sample(args.c5_sample)
        rows, bad_all = [], {}
        nf = min(2, nb)
        for j in range(nf):
            cols, n = sh2.generate(j)
            rt.push_device("StockStream", n, cols["ts"].data_ptr(), [cols["id"].data_ptr(), cols["sym"].data_ptr(),
                                                                    cols["price"].data_ptr(), cols["volume"].data_ptr()])
            rt.flush(deliver=False)
            del cols
            m = int(rt.stats().matches)
            t_ts = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
            t_seq, t_sub = torch.empty_like(t_ts), torch.empty_like(t_ts)
            t_vals = torch.empty((2, max(m, 1)), dtype=torch.int64, device=dev)
            rt.export_device(0, max(m, 1), t_ts.data_ptr(), t_seq.data_ptr(), t_sub.data_ptr(), t_vals.data_ptr())
            bad = c5.check_matches(sh2, t_vals[0, :m], t_vals[1, :m], t_ts[:m])
            for k, v in bad.items():
                bad_all[k] = bad_all.get(k, 0) + v
            rows.append(sample_records(sh2, smap, t_ts[:m], t_vals[0, :m], t_vals[1, :m]))
            del t_ts, t_seq, t_sub, t_vals
            torch.cuda.empty_cache()
        _, g_end = sh2.global_range(nf - 1)
        n_s, ref = oracle_sample_rows(sh2, skeys, smap, g_end)
        got = delivery_order(np.concatenate(rows))
        ok = got.shape == ref.shape and np.array_equal(got, ref) and not any(bad_all.values())
        if not ok:
            raise RuntimeError("C5: GPU match rows differ from the oracle on the %d-key sample (%d vs %d rows; %s)"
                               % (len(skeys), len(got), len(ref), bad_all))
        out["parity"] = {"sample_keys": len(skeys), "sample_events": int(n_s), "sample_matches": int(len(ref)),
                         "flushes": nf, "bit_exact": True, "property_violations": bad_all}
        if dist is not None:
            okt = torch.tensor([1], dtype=torch.int64, device=dev)
            dist.all_reduce(okt)
            out["parity"]["ranks_checked"] = int(okt.item())
    rt.shutdown()
    log("done")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


class _HostStagedDist:
    """torch.distributed over gloo with CUDA tensors staged through host memory: a rehearsal of the N > 1 path
    (SDG_BENCH_BACKEND=gloo, every rank on one GPU with SDG_BENCH_SHARE_GPU=1) on a one-GPU box. The measured
    multi-GPU runs use the nccl backend (RCCL over xGMI) directly."""

    def __init__(self, d):
        self.d = d
        self.ReduceOp = d.ReduceOp

    def barrier(self):
        self.d.barrier()

    def all_gather(self, out, t):
        host = [x.cpu() for x in out]
        self.d.all_gather(host, t.cpu())
        for x, y in zip(out, host):
            x.copy_(y)

    def all_reduce(self, t, op=None):
        c = t.cpu()
        self.d.all_reduce(c, op=op if op is not None else self.d.ReduceOp.SUM)
        t.copy_(c)

    def send(self, t, dst):
        self.d.send(t.contiguous().cpu(), dst=dst)

    def recv(self, t, src):
        import torch
        c = torch.empty(t.shape, dtype=t.dtype)
        self.d.recv(c, src=src)
        t.copy_(c)

    def destroy_process_group(self):
        self.d.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--events", type=int, default=100_000_000, help="events per GPU per step")
    ap.add_argument("--keys", type=int, default=10_000, help="keys per GPU")
    ap.add_argument("--cpu-sample", type=int, default=3_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--parity-sample", type=int, default=3_000_000,
                    help="events of the bench stream re-run through a fresh runtime and the oracle (bit-exact check)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--e2e-steps", type=int, default=2, help="end-to-end (host push -> poll) steps, 0 = skip")
    ap.add_argument("--no-gather", action="store_true", help="skip the ordered result gather leg")
    ap.add_argument("--no-ordered", action="store_true", help="skip the timed flush + delivery-order export steps")
    ap.add_argument("--config", choices=["c2", "c5"], default="c2",
                    help="c2 (default, the metric's 1-GPU config) or c5 (10^10 events / 10^8 keys, key-hash sharded)")
    ap.add_argument("--c5-events", type=int, default=10 ** 10, help="C5: events of the whole stream")
    ap.add_argument("--c5-batch", type=int, default=1 << 28, help="C5: rank events per flush")
    ap.add_argument("--c5-sample", type=int, default=10_000, help="C5: partition keys in the oracle sample")
    ap.add_argument("--c5-shard", default=None,
                    help="C5 on one process: run shard R/W (rank R of a W-GPU run) instead of this process's rank")
    args = ap.parse_args()

    # --gpus N is honoured: without a launcher (no WORLD_SIZE in the environment) this process starts the N ranks
    # itself -- torch.distributed.run as a CHILD process, before anything here touches the GPU -- and exits with its
    # status; under a launcher the world size must agree with --gpus
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        log("starting %d ranks: %s" % (args.gpus, " ".join(cmd)))
        raise SystemExit(subprocess.call(cmd))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s" % (args.gpus, os.environ.get("WORLD_SIZE")))

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SDG_BENCH_SHARE_GPU"):  # rehearsal: every rank on GPU 0 (see _HostStagedDist)
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as tdist
        if os.environ.get("SDG_BENCH_BACKEND", "nccl") == "gloo":
            tdist.init_process_group("gloo")
            dist = _HostStagedDist(tdist)
        else:
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dist = tdist

    if args.config == "c5":
        return run_c5(args, rank, world, local, dist)
    import siddhi_amd as sa
    from siddhi_amd import workloads as w

    n, keys = args.events, args.keys
    log("generating %d events x %d keys (rank %d/%d)" % (n, keys, rank, world))
    cols = gen_shard(n, keys, rank, world)
    from siddhi_amd import shard
    syms = []  # this rank's keys: the first `keys` global key names that hash to this rank (shard.py)
    g = 0
    while len(syms) < keys:
        name = "S%07d" % g
        if world == 1 or shard.owner(name, world) == rank:
            syms.append(name)
        g += 1
    rt = sa.SiddhiAppRuntime(w.C2_APP, device=local)
    sym_ids = np.array([rt.intern(s) for s in syms], dtype=np.uint32)
    dev = torch.device("cuda", local)
    d_id = torch.from_numpy(cols["id"]).to(dev)
    d_sym = torch.from_numpy(sym_ids[cols["key"]].view(np.int32)).to(dev)
    d_price = torch.from_numpy(cols["price"]).to(dev)
    d_vol = torch.from_numpy(cols["volume"]).to(dev)
    d_ts0 = torch.from_numpy(cols["ts"]).to(dev)
    span = int(cols["ts"][-1] - cols["ts"][0]) + 1
    nsteps = args.warmup + args.steps
    ts_steps = [d_ts0 + s * span for s in range(nsteps)]  # consecutive batches of one stream (the ordered steps and
                                                          # the gather leg continue its time after them)
    torch.cuda.synchronize()

    def step(s):
        rt.push_device("StockStream", n, ts_steps[s].data_ptr(),
                       [d_id.data_ptr(), d_sym.data_ptr(), d_price.data_ptr(), d_vol.data_ptr()])
        rt.flush(deliver=False)
        rt.discard()  # matches stay in HBM (device-resident measurement)
        st = rt.stats()
        if dist is not None:  # batch-boundary match-count all-gather (global output offsets)
            cnt = torch.tensor([st.matches], dtype=torch.int64, device=dev)
            allc = [torch.empty_like(cnt) for _ in range(world)]
            dist.all_gather(allc, cnt)
        return st

    log("warm-up (%d steps)" % args.warmup)
    for s in range(args.warmup):
        step(s)
    log("timed steps (%d)" % args.steps)
    keys_k = ["ms_kg_hist", "ms_kg_prefix", "ms_kg_scatter", "ms_chain_carry", "ms_chain_match"]
    acc = {k: 0.0 for k in keys_k}
    matches = 0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, nsteps):
        st = step(s)
        matches += st.matches
        for k in keys_k:
            acc[k] += getattr(st, k)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        m = torch.tensor([matches], dtype=torch.int64, device=dev)
        dist.all_reduce(m)
        total_matches = int(m.item())
    else:
        total_matches = matches
    K = args.steps
    ms_per_step = elapsed * 1000.0 / K
    value = n * world * K / elapsed

    per_kernel = {k: acc[k] / K for k in keys_k}
    dom = max(per_kernel, key=per_kernel.get)
    step_bytes = n * B_IN + (matches / K) * B_OUT
    # fused time sub-batches (SDG_FU_SUB): the matcher runs once per sub-batch; per launch = the step's bytes and
    # time divided by the launches (the same ratio)
    launches = max(1, int(st.sub_batches)) if dom in ("ms_chain_match", "ms_kg_scatter") else 1
    achieved = step_bytes / (per_kernel[dom] / 1000.0) / 1e9
    kernel_names = {"ms_chain_match": "chain_fused_k" if st.fused == 1 else "chain_deque_k",
                    "ms_kg_scatter": "rx_scatter", "ms_kg_hist": "rx_hist", "ms_chain_carry": "chain_carry_k"}
    traffic = None
    tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        ent = tj.get("kernels", {}).get(kernel_names.get(dom, ""))
        if ent and tj.get("events_per_launch") == n and tj.get("launches_per_step", 1) == launches:
            traffic = ent["fetch_bytes"] + ent["write_bytes"]
    out = {
        "metric": "input events/sec matched (node) at 1/2/4/8 MI355X; % HBM roofline",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (splitmix64 C2 generator, BASELINE.md), device-resident",
        "config": {"workload": "C2: partition with (symbol of StockStream) every e1=StockStream[price>20] -> "
                               "e2=StockStream[price>e1.price] within 1 sec",
                   "events_per_gpu_per_step": n, "keys_per_gpu": keys, "parallelism": "key-hash shards x%d" % world,
                   "matches_per_step": total_matches / K, "overflow_scans_last_step": st.fused_ovf, "path": "fused bucket matcher" if st.fused == 1 else
                   "radix key sort + chain kernels"},
        "roofline": {"bound": "hbm", "kernel": kernel_names.get(dom, dom), "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 --pmc, profiles/pmc_traffic.json)",
                     "algorithmic_bytes_per_launch": step_bytes / launches, "launches_per_step": launches,
                     "step_frac": step_bytes / (ms_per_step / 1000.0) / 1e9 / HBM_PEAK_GBS,
                     "kernel_ms": per_kernel},
    }
    if not args.no_ordered:
        # the same steps with the reference's observable order inside the timed region: flush, then the flush's
        # records exported in delivery order (sdg_export_ordered: ts, emitting position, e1id, e2id into device buffers)
        log("timed ordered steps (%d): flush + delivery-order export" % K)
        cap = n + n // 4 + 4096
        o_ts = torch.empty(cap, dtype=torch.int64, device=dev)
        o_seq = torch.empty(cap, dtype=torch.int64, device=dev)
        o_vals = torch.empty((2, cap), dtype=torch.int64, device=dev)
        ots = [d_ts0 + (nsteps + 2 + s) * span for s in range(K + 1)]  # (the stream's time continues)

        def ostep(s):
            rt.push_device("StockStream", n, ots[s].data_ptr(),
                           [d_id.data_ptr(), d_sym.data_ptr(), d_price.data_ptr(), d_vol.data_ptr()])
            rt.flush(deliver=False)
            return rt.export_ordered(0, cap, o_ts.data_ptr(), o_seq.data_ptr(), 0, o_vals.data_ptr())
        ostep(0)  # (warm-up: the ordering pass sizes its workspaces on first use)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        orecs = 0
        for s in range(1, K + 1):
            orecs += ostep(s)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        oel = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([oel], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            oel = float(t.item())
        if orecs > 1:  # the last step's export is in delivery order: (emitting position, e1 position) increasing;
            m = orecs // K  # ids restart every step, so a partial carried from the step before (e1id > e2id: its e1
            seq, e1, e2 = o_seq[:m], o_vals[0, :m], o_vals[1, :m]  # lies at the end of the previous batch) ranks first
            e1k = e1 + (e1 < e2).to(torch.int64) * (1 << 40)
            okd = bool(((seq[1:] > seq[:-1]) | ((seq[1:] == seq[:-1]) & (e1k[1:] > e1k[:-1]))).all().item())
            if not okd:
                raise RuntimeError("ordered steps: the export is not in delivery order")
        out["value_ordered"] = n * world * K / oel
        out["ordered"] = {"ms_per_step": oel * 1000.0 / K, "records_per_step": orecs / K,
                          "ms_export_per_step": oel * 1000.0 / K - ms_per_step,
                          "path": "flush + sdg_export_ordered (device radix sort by emitting position, run ranks by "
                                  "e1 position, one row gather) per step, inside the timed region",
                          "step_frac": step_bytes / (oel / K) / 1e9 / HBM_PEAK_GBS}
    if rank == 0 and not args.no_cpu:  # (at N > 1: rank 0's shard, a third of the sample, after the timed region)
        cs = min(args.cpu_sample if world == 1 else args.cpu_sample // 3, n)
        log("cpu baseline (oracle, 1 thread, %d events)" % cs)
        rate, cm, dt = cpu_baseline(cols, syms, cs)
        out["cpu_baseline"] = {"value": rate, "unit": "events/s", "cores": 1, "kind": "port",
                               "sample": "first %d events of %s C2 stream (%.1f s, %d matches), oracle restatement"
                                         % (cs, "the" if world == 1 else "rank 0's", dt, cm),
                               "note": "box-to-box variance: this 1-core figure measured 4.4e5 to 1.05e6 events/s "
                                       "for the same sample on different pooled boxes (BASELINE.md); compare it "
                                       "with the GPU figure of the same run only"}
        thr = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
        log("cpu baseline, key-sharded over %d threads" % thr)
        srate, scm, sdt = cpu_baseline_sharded(cols, syms, cs, thr)
        if scm != cm:
            raise RuntimeError("key-sharded CPU baseline disagrees with the single-thread run: %d vs %d" % (scm, cm))
        out["cpu_baseline_sharded"] = {"value": srate, "unit": "events/s", "cores": thr, "kind": "port",
                                       "sample": "same events, key-sharded over %d threads (%.2f s, %d matches)"
                                                 % (thr, sdt, scm)}
    else:
        out["cpu_baseline"] = None
    if not args.no_gather:
        log("ordered result gather (one more batch, outside the timed region)")
        # the leg's two batches (a warm-up export, then the timed one) continue the stream's time after the ordered
        # steps (a batch earlier than the last one sends time backwards: the chain query then falls back to the generic
        # NFA, whose carry replay overflowed at N = 2)
        t_first = nsteps if args.no_ordered else nsteps + 2 + K + 1
        leg_ts = [d_ts0 + (t_first + j) * span for j in range(2)]
        nxt = [0]

        def leg_push():
            rt.push_device("StockStream", n, leg_ts[nxt[0]].data_ptr(),
                           [d_id.data_ptr(), d_sym.data_ptr(), d_price.data_ptr(), d_vol.data_ptr()])
            nxt[0] += 1
        out["ordered_gather"] = ordered_gather_leg(rt, step_push=leg_push, n=n, dev=dev, dist=dist, rank=rank,
                                                   world=world)
    rt.shutdown()
    if args.e2e_steps > 0 and world == 1:
        log("end-to-end (host push -> poll), %d step(s)" % args.e2e_steps)
        out["end_to_end"] = end_to_end(cols, syms, n, args.e2e_steps, local)
    if not args.no_parity:
        log("parity leg (GPU vs oracle on the bench stream's first events)")
        ps = min(args.parity_sample if world == 1 else args.parity_sample // 3, n)
        out["parity"] = parity_check(cols, syms, ps, (d_id[:ps], d_sym[:ps], d_price[:ps], d_vol[:ps], d_ts0[:ps]),
                                     local)
        if dist is not None:  # every rank checked its own shard
            okt = torch.tensor([1], dtype=torch.int64, device=dev)
            dist.all_reduce(okt)
            out["parity"]["ranks_checked"] = int(okt.item())
    log("done")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
