#!/usr/bin/env python3
"""Secondary throughput lines for the other BASELINE.json configs (bench.py measures C2 only).

C1: unpartitioned chain query on 1M ticks, one flush per step, consecutive batches of one stream.
C3: the count-quantifier SEQUENCE on `--c3-keys` keys x 100 events (generic keyed NFA, nfa_k); the literal query
    never matches under the reference semantics, so the `<1:5>` form is timed too.
Inputs are device-resident; one JSON line per config. Timing brackets K flushes with torch.cuda.synchronize().
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(rt, stream, n, ts, cols, steps, warmup):
    span = int(ts[-1].item() - ts[0].item()) + 1
    tss = [ts + s * span for s in range(steps + warmup)]
    torch.cuda.synchronize()

    def step(s):
        rt.push_device(stream, n, tss[s].data_ptr(), [c.data_ptr() for c in cols])
        rt.flush(deliver=False)
        rt.discard()  # matches stay in HBM (device-resident measurement)
        return rt.stats()

    for s in range(warmup):
        step(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = 0
    for s in range(warmup, warmup + steps):
        m += step(s).matches
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return n * steps / dt, dt * 1000 / steps, m / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--c1-events", type=int, default=1_000_000)
    ap.add_argument("--c3-keys", type=int, default=1_000_000)
    ap.add_argument("--only", default="c1,c3,c3m,c4")
    ap.add_argument("--c4-keys", type=int, default=1_000_000)
    ap.add_argument("--c3-steps", type=int, default=2)
    ap.add_argument("--max-partials", type=int, default=0)
    ap.add_argument("--c2-events", type=int, default=100_000_000)
    args = ap.parse_args()
    torch.cuda.init()
    import siddhi_amd as sa
    from siddhi_amd import workloads as w
    dev = torch.device("cuda", 0)
    only = args.only.split(",")
    if "c1" in only:
        n = args.c1_events
        c = w.c1_columns(n)
        rt = sa.SiddhiAppRuntime(w.C1_APP, device=0)
        sym = np.full(n, rt.intern("IBM"), dtype=np.int32)
        cols = [torch.from_numpy(c["id"]).to(dev), torch.from_numpy(sym).to(dev),
                torch.from_numpy(c["price"]).to(dev), torch.from_numpy(c["volume"]).to(dev)]
        # >= 4 warm-up flushes: the first flushes with carried partials still grow buffers (one-time hipMalloc),
        # which at 0.3 ms per flush is most of a short timed run
        ev, ms, m = run(rt, "StockStream", n, torch.from_numpy(c["ts"]).to(dev), cols, args.steps, max(args.warmup, 4))
        print(json.dumps({"config": "C1 unpartitioned, %d events/step" % n, "events_per_s": ev, "ms_per_step": ms,
                          "matches_per_step": m}), flush=True)
    # C2 on the paths a query that just misses the fused envelope takes: the radix key sort + chain matcher, and the
    # generic keyed NFA (one lane per key) -- the cost of falling outside each kernel's shape
    for tag, kw, n in (("c2radix", {"fused": False}, args.c2_events), ("c2generic", {"force_generic": True}, args.c2_events // 10)):
        if tag not in only:
            continue
        c = w.c2_columns(n)
        rt = sa.SiddhiAppRuntime(w.C2_APP, device=0, **kw)
        syms = w.symbols(10_000)
        sym_ids = np.array([rt.intern(x) for x in syms], dtype=np.uint32)
        cols = [torch.from_numpy(c["id"]).to(dev), torch.from_numpy(sym_ids[c["key"]].view(np.int32)).to(dev),
                torch.from_numpy(c["price"]).to(dev), torch.from_numpy(c["volume"]).to(dev)]
        ev, ms, m = run(rt, "StockStream", n, torch.from_numpy(c["ts"]).to(dev), cols, args.steps, args.warmup)
        st = rt.stats()
        print(json.dumps({"config": "C2 on the %s path, %d events/step, 10k keys" % (tag[2:], n), "events_per_s": ev,
                          "ms_per_step": ms, "matches_per_step": m, "path": st.path, "fused": st.fused,
                          "ms_keygroup": st.ms_keygroup, "ms_match": st.ms_match}), flush=True)
    for tag in ("c3", "c3m"):
        if tag not in only:
            continue
        keys = args.c3_keys
        c = w.c3_columns(keys)
        n = len(c["ts"])
        app = w.C3_APP if tag == "c3" else w.C3_APP.replace("<2:5>", "<1:5>")
        rt = sa.SiddhiAppRuntime(app, device=0, batch_capacity=n + 1,  # one flush per step (no auto-flush)
                                 max_partials=args.max_partials)
        ih = rt.getInputHandler("S")
        cols = [c["id"], c["key"], c["price"], c["volume"]]
        span = int(c["ts"][-1] - c["ts"][0]) + 1
        # long partition keys: host push (the key's toString dictionary is built on the host), so this rate
        # includes the host key mapping and the H2D copy
        for s in range(args.warmup):
            ih.send_columns(c["ts"] + s * span, cols)
            rt.flush(deliver=False)
            rt.discard()  # matches stay in HBM (device-resident measurement)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = 0
        dev_ms = 0.0
        for s in range(args.warmup, args.warmup + args.c3_steps):
            ih.send_columns(c["ts"] + s * span, cols)
            rt.flush(deliver=False)
            rt.discard()  # matches stay in HBM (device-resident measurement)
            st = rt.stats()
            m += st.matches
            dev_ms += st.ms_keygroup + st.ms_match
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        form = ("literal BASELINE form every e1, e2<2:5>, e3 (0 matches by the reference's semantics, DESIGN.md 5)"
                if tag == "c3" else "survey form every e1, e2<1:5>, e3 (the throughput figure)")
        print(json.dumps({"config": "C3 %s, %d keys x 100 events/step (host push)" % ("<2:5>" if tag == "c3" else "<1:5>", keys),
                          "c3_form_timed": form,
                          "max_partials": args.max_partials or 8,
                          "events_per_s_end_to_end": n * args.c3_steps / dt, "ms_per_step": dt * 1000 / args.c3_steps,
                          "device_ms_per_step": dev_ms / args.c3_steps, "events_per_s_device": n * args.c3_steps / (dev_ms / 1000),
                          "matches_per_step": m / args.c3_steps, "events_per_flush": st.events}), flush=True)
    if "c3md" in only:  # C3 <1:5> device-resident: long keys through the device key table (keytab.hip)
        keys = args.c3_keys
        c = w.c3_columns(keys)
        n = len(c["ts"])
        rt = sa.SiddhiAppRuntime(w.C3_APP.replace("<2:5>", "<1:5>"), device=0, batch_capacity=n + 1,
                                 max_partials=args.max_partials)
        d = [torch.from_numpy(c[k]).to(dev) for k in ("id", "key", "price", "volume")]
        d_ts0 = torch.from_numpy(c["ts"]).to(dev)
        span = int(c["ts"][-1] - c["ts"][0]) + 1
        ts_steps = [d_ts0 + s * span for s in range(args.warmup + args.c3_steps)]
        torch.cuda.synchronize()

        def step(s):
            rt.push_device("S", n, ts_steps[s].data_ptr(), [x.data_ptr() for x in d])
            rt.flush(deliver=False)
            rt.discard()
            return rt.stats()
        for s in range(args.warmup):
            step(s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = 0
        for s in range(args.warmup, args.warmup + args.c3_steps):
            m += step(s).matches
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"config": "C3 <1:5>, %d keys x 100 events/step, device-resident (device key table)" % keys,
                          "c3_form_timed": "survey form every e1, e2<1:5>, e3 (the literal <2:5> form has 0 matches)",
                          "events_per_s": n * args.c3_steps / dt, "ms_per_step": dt * 1000 / args.c3_steps,
                          "matches_per_step": m / args.c3_steps}), flush=True)
    if "c4" in only:
        run_c4(args.c4_keys)


def run_c4(keys):
    """C4: e1=A[v>10] -> (e2=B[v>20] and e3=C[v>30]) -> not D[v>40] for 5 sec over `keys` keys x 20 events, the 4
    streams interleaved (sdg_push_mixed, host columns), then advance_time(T_end + 5000). One flush + the final
    timer flush; device ms from sdg_stats (NFA + key grouping), end to end includes the host mixed-batch
    assembly, the scheduler simulation and the host replays."""
    import siddhi_amd as sa
    from siddhi_amd import workloads as w
    c = w.c4_columns(keys)
    n = len(c["ts"])
    end = int(c["ts"][-1]) + 5000
    rt = sa.SiddhiAppRuntime(w.C4_APP, device=0, batch_capacity=n + 1)
    idx = np.array([rt._L.sdg_stream_index(rt._h, s.encode()) for s in w.C4_STREAMS], dtype=np.int32)[c["stream"]]
    t0 = time.perf_counter()
    rt.push_mixed(idx, c["ts"], [c["id"], c["key"], c["v"]])
    rt.flush(deliver=False)
    s1 = rt.stats()
    rt.advance_time(end)
    rt.flush(deliver=False)
    s2 = rt.stats()
    ts, vals, nulls, seq = rt.poll_arrays(0)
    dt = time.perf_counter() - t0
    rt.shutdown()
    dev_ms = s1.ms_keygroup + s1.ms_match + s2.ms_keygroup + s2.ms_match
    print(json.dumps({"config": "C4 %d keys x 20 events (4 streams interleaved, host push)" % keys,
                      "events": n, "matches": int(len(ts)), "events_per_s_end_to_end": n / dt,
                      "device_ms": dev_ms, "ms_nfa": s1.ms_nfa + s2.ms_nfa, "events_per_s_device": n / (dev_ms / 1000),
                      "timer_fires": s1.sched_fires + s2.sched_fires,
                      "fires_shifted_by_collapse": s1.sched_shifted + s2.sched_shifted,
                      "ms_nfa_kernel": s1.ms_nfa_kernel + s2.ms_nfa_kernel,
                      "ms_sched_host": s1.ms_sched_host + s2.ms_sched_host,
                      "keys_rerun_in_scheduler_order": s1.sched_rerun_keys + s2.sched_rerun_keys,
                      "keys_replayed_on_host": s1.sched_host_keys + s2.sched_host_keys,
                      "end_to_end_s": dt}), flush=True)


if __name__ == "__main__":
    main()
