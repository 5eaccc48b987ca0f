"""Host-side time per C1 flush (push_device / flush / discard / stats) beside the device time: where a small,
launch-bound flush spends its wall clock."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import siddhi_amd as sa  # noqa: E402
from siddhi_amd import workloads as w  # noqa: E402

n = 1_000_000
torch.cuda.init()
c = w.c1_columns(n)
rt = sa.SiddhiAppRuntime(w.C1_APP, device=0)
dev = torch.device("cuda", 0)
sym = np.full(n, rt.intern("IBM"), dtype=np.int32)
cols = [torch.from_numpy(c["id"]).to(dev), torch.from_numpy(sym).to(dev), torch.from_numpy(c["price"]).to(dev),
        torch.from_numpy(c["volume"]).to(dev)]
span = n
tss = [torch.from_numpy(c["ts"]).to(dev) + s * span for s in range(24)]
torch.cuda.synchronize()
tt = {"push": 0.0, "flush": 0.0, "discard": 0.0, "stats": 0.0}
for s in range(24):
    t0 = time.perf_counter()
    rt.push_device("StockStream", n, tss[s].data_ptr(), [x.data_ptr() for x in cols])
    t1 = time.perf_counter()
    rt.flush(deliver=False)
    t2 = time.perf_counter()
    rt.discard()
    t3 = time.perf_counter()
    st = rt.stats()
    t4 = time.perf_counter()
    if s >= 4:
        for k, v in zip(tt, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            tt[k] += v
print({k: round(v / 20 * 1e3, 4) for k, v in tt.items()}, "device ms", round(st.ms_total, 4), flush=True)
