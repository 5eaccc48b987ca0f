#!/usr/bin/env python3
"""Time the ordered gather's device merge (sdg_merge_runs) on one GPU: G sorted runs of R records each, 24-B
records (int64 key + two int64 payload columns, the C5 gather's ts / e1id / e2id shape), against the round-5 merge
(concatenate + one stable torch.sort of the key). Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--records", type=int, default=100_000_000, help="records per run")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-sort-baseline", action="store_true")
    a = ap.parse_args()
    torch.cuda.init()
    from siddhi_amd import merge_runs_device
    G, R = a.runs, a.records
    g = torch.Generator(device="cuda").manual_seed(1)
    keys, cols = [], []
    for r in range(G):
        k = torch.sort(torch.randint(0, 10 * G * R, (R,), device="cuda", generator=g)).values
        keys.append(k)
        cols.append([k // 100, k * 3])
    N = G * R
    out_k = torch.empty(N, dtype=torch.int64, device="cuda")
    out_c = [torch.empty(N, dtype=torch.int64, device="cuda") for _ in range(2)]
    merge_runs_device(keys, cols, out_k, out_c)  # warm-up (workspace)
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        merge_runs_device(keys, cols, out_k, out_c)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ok = bool(torch.all(out_k[1:] >= out_k[:-1]).item()) and torch.equal(out_c[0], out_k // 100) and \
        torch.equal(out_c[1], out_k * 3)
    ms = sorted(ts)[len(ts) // 2] * 1e3
    res = {"what": "device G-way merge (sdg_merge_runs)", "runs": G, "records_per_run": R, "record_bytes": 24,
           "ms_median": ms, "ms_all": [t * 1e3 for t in ts], "sorted_and_payload_ok": ok,
           "hbm_bytes": N * 24 * 2, "achieved_GBps": N * 24 * 2 / (ms * 1e-3) / 1e9}
    if not a.no_sort_baseline and N <= 400_000_000:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cat = torch.cat(keys)
        perm = torch.sort(cat, stable=True).indices
        _ = [torch.cat([c[j] for c in cols])[perm] for j in range(2)]
        torch.cuda.synchronize()
        res["ms_round5_sort_merge"] = (time.perf_counter() - t0) * 1e3
    print(json.dumps(res))


if __name__ == "__main__":
    main()
