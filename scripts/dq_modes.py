import sys; sys.path.insert(0,'.'); sys.path.insert(0,'tests')
import numpy as np, siddhi_amd as sa
from siddhi_amd import workloads as w
from test_gpu_parity import DQ_APPS
cols = w.c1_columns(5000)
for a in DQ_APPS:
    app = "@app:playback " + w.STOCK_STREAM + " @info(name = 'query1') from " + a + " select e1.id as e1id, e2.id as e2id insert into M;"
    rt = sa.SiddhiAppRuntime(app)
    h = rt.getInputHandler("StockStream")
    h.send_columns(cols["ts"], [cols["id"], np.full(5000, rt.intern("IBM"), np.uint32), cols["price"], cols["volume"]])
    rt.flush(deliver=False)
    st = rt.stats()
    print("deque", st.deque, "path", st.path, "matches", st.matches, a, flush=True)
    rt.shutdown()
