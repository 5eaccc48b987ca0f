"""Host-side time per bench step (push_device / flush / discard / stats) next to the device time, to find the
inter-step gap the kernel trace shows."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import siddhi_amd as sa  # noqa: E402
from siddhi_amd import workloads as w  # noqa: E402

n, keys = 100_000_000, 10_000
torch.cuda.init()
cols = w.c2_columns(n, keys=keys)
rt = sa.SiddhiAppRuntime(w.C2_APP, device=0)
syms = w.symbols(keys)
sym_ids = np.array([rt.intern(s) for s in syms], dtype=np.uint32)
dev = torch.device("cuda", 0)
d_id = torch.from_numpy(cols["id"]).to(dev)
d_sym = torch.from_numpy(sym_ids[cols["key"]].view(np.int32)).to(dev)
d_price = torch.from_numpy(cols["price"]).to(dev)
d_vol = torch.from_numpy(cols["volume"]).to(dev)
d_ts0 = torch.from_numpy(cols["ts"]).to(dev)
span = int(cols["ts"][-1] - cols["ts"][0]) + 1
torch.cuda.synchronize()
tt = {"push": 0.0, "flush": 0.0, "discard": 0.0, "stats": 0.0}
steps = 8
for s in range(steps):
    ts = d_ts0 + s * span
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rt.push_device("StockStream", n, ts.data_ptr(), [d_id.data_ptr(), d_sym.data_ptr(), d_price.data_ptr(),
                                                     d_vol.data_ptr()])
    t1 = time.perf_counter()
    rt.flush(deliver=False)
    t2 = time.perf_counter()
    rt.discard()
    t3 = time.perf_counter()
    st = rt.stats()
    t4 = time.perf_counter()
    if s >= 2:
        for k, v in zip(tt, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            tt[k] += v
    print("step %d flush %.3f ms (device total %.3f ms: keygroup %.3f match %.3f)" %
          (s, (t2 - t1) * 1e3, st.ms_total, st.ms_keygroup, st.ms_match), flush=True)
print({k: round(v / (steps - 2) * 1e3, 4) for k, v in tt.items()}, flush=True)
