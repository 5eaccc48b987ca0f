"""debug: C3 host push at 10^6 keys, with and without an auto-flush inside the push"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (torch's HIP runtime first)
torch.cuda.init()
import siddhi_amd as sa
from siddhi_amd import workloads as w

for keys, cap in ((200_000, 0), (1_000_000, 100_000_001), (1_000_000, 0)):
    c = w.c3_columns(keys)
    app = w.C3_APP.replace("<2:5>", "<1:5>")
    rt = sa.SiddhiAppRuntime(app, batch_capacity=cap)
    h = rt.getInputHandler("S")
    h.send_columns(c["ts"], [c["id"], c["key"], c["price"], c["volume"]])
    s1 = rt.stats()
    rt.flush(deliver=False)
    s2 = rt.stats()
    ts, vals, nulls, seq = rt.poll_arrays(0)
    print("keys %d cap %d: after push events %d matches %d path %d; after flush events %d matches %d; polled %d"
          % (keys, cap, s1.events, s1.matches, s1.path, s2.events, s2.matches, len(ts)), flush=True)
    rt.shutdown()
