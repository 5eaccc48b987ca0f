#!/usr/bin/env python3
"""Host profile of the product's keyed-NFA and scheduler-simulation code (nfa.h, sched.cpp) through the test
emulator (tests/native/libnfa_emu.so, the same sources built for the CPU): one flush of C3 or C4 at a given key
count, SIGPROF samples mapped to functions with addr2line. A proxy for where the device NFA spends instructions,
and the direct profile of the host scheduler simulation. Test infrastructure, CPU only.

  python3 scripts/emu_prof.py c4 --keys 100000
  python3 scripts/emu_prof.py c3 --keys 20000
"""
import argparse
import collections
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
from emu_rt import EMU_SO, lib  # noqa: E402
from siddhi_amd import workloads as w  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["c3", "c4"])
    ap.add_argument("--keys", type=int, default=100_000)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--out", default="/tmp/emu_prof.txt")
    args = ap.parse_args()
    L = lib()
    L.emu_prof_start.argtypes = []
    L.emu_prof_stop.argtypes = [ctypes.c_char_p]
    if args.config == "c4":
        app = w.C4_APP
        c = w.c4_columns(args.keys)
    else:
        app = w.C3_APP
        c = w.c3_columns(args.keys)
    h = L.emu_create(app.encode(), 0)
    if not h:
        raise SystemExit(L.emu_error().decode())
    n = len(c["ts"])
    if args.config == "c4":
        sidx = np.array([L.emu_stream_index(h, s.encode()) for s in w.C4_STREAMS], dtype=np.int32)
        strm = sidx[c["stream"]]
        slots = np.stack([c["id"], c["key"], c["v"].view(np.int64)], axis=1).astype(np.int64)
    else:
        strm = np.full(n, L.emu_stream_index(h, b"S"), dtype=np.int32)
        slots = np.stack([c["id"], c["key"], c["price"].view(np.int64), c["volume"].astype(np.int64)], axis=1)
    slots = np.ascontiguousarray(slots)
    na = slots.shape[1]
    offs = np.arange(n, dtype=np.int64) * na
    ts = np.ascontiguousarray(c["ts"], dtype=np.int64)
    L.emu_send_batch(h, n, strm.ctypes.data, ts.ctypes.data, offs.ctypes.data, slots.ctypes.data, None)
    if args.config == "c4":
        L.emu_advance(h, int(ts[-1]) + 5000)
    t = time.perf_counter()
    L.emu_prof_start()
    rc = L.emu_flush(h)
    L.emu_prof_stop(args.out.encode())
    dt = time.perf_counter() - t
    if rc:
        raise SystemExit(L.emu_error().decode())
    print("%s %d keys, %d events: flush %.2f s, %d matches; scheduler passes (us): optimistic %d rerun %d exact %d,"
          " reordered %d taken %d exact passes %d" % (args.config, args.keys, n, dt, L.emu_num_out(h, 0), L.emu_sched_stat(2),
                                       L.emu_sched_stat(3), L.emu_sched_stat(4), L.emu_sched_stat(0),
                                       L.emu_sched_stat(1), L.emu_sched_stat(6)))
    L.emu_destroy(h)
    # samples -> functions
    cnt = collections.Counter()
    for line in open(args.out):
        obj, off = line.split()
        if obj.endswith("libnfa_emu.so"):
            cnt[off] += 1
        else:
            cnt[os.path.basename(obj)] += 1
    total = sum(cnt.values())
    addrs = [a for a in cnt if a.startswith("0x")]
    names = {}
    if addrs:
        # the innermost (possibly inlined) function of each address: two lines (function, file:line) per address
        out = subprocess.run(["addr2line", "-f", "-C", "-e", EMU_SO] + addrs, capture_output=True, text=True).stdout
        lines = out.splitlines()
        for j, a in enumerate(addrs):
            names[a] = lines[2 * j] if 2 * j < len(lines) else "?"
    fn = collections.Counter()
    for a, k in cnt.items():
        nm = names.get(a, a)
        fn[nm.split("(")[0][:110]] += k
    print("%d samples" % total)
    for nm, k in fn.most_common(args.top):
        print("%6.2f%%  %s" % (100.0 * k / total, nm))


if __name__ == "__main__":
    main()
