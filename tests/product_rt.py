"""Replays golden-fixture traces through the product (GPU engine via the C-ABI) in the oracle's output format."""
import ctypes
import struct

import siddhi_amd as sa

TAG = {sa.INT: "i", sa.LONG: "l", sa.FLOAT: "f", sa.DOUBLE: "d", sa.BOOL: "b", sa.STRING: "s"}


class ProductAdapter:
    def __init__(self, app, force_generic=False, fused=True, max_partials=0, seq3=True, **kw):
        self.rt = sa.SiddhiAppRuntime(app, force_generic=force_generic, fused=fused, max_partials=max_partials,
                                      seq3=seq3, **kw)
        self.stats = []  # sdg_stats of every flush
        self.handlers = {}
        self.records = []

    def start(self, ts):
        self.rt.start(ts)

    def handler(self, sid):
        if sid not in self.handlers:
            self.handlers[sid] = self.rt.getInputHandler(sid)
        return self.handlers[sid]

    def send(self, sid, ts, values, now=None, mode=0):
        if not self.rt.playback and now is not None:
            self.rt.advance_time(now)  # the wall clock at this send: timers due by then fire before the event
        h = self.handler(sid)
        if mode == 1 and self.rt.playback:
            h.send(values)
        else:
            h.send(ts, values)

    def send_events(self, sid, rows):
        """InputHandler.send(Event[]) with rows [(ts, values), ...]"""
        self.handler(sid).send([sa.Event(ts, values) for ts, values in rows])

    def advance(self, ts):
        self.rt.advance_time(ts)

    def flush(self):
        self.rt.flush(deliver=False)
        self.stats.append(self.rt.stats())
        for q, (name, target, types, names) in enumerate(self.rt._queries):
            types, ts, vals, nulls = self.rt.raw_outputs(q)
            def dec(t, v):
                if v is None:
                    return None
                if t == sa.INT:
                    return ("i", ctypes.c_int32(v).value)
                if t == sa.FLOAT:
                    return ("f", v & 0xffffffff)
                if t == sa.BOOL:
                    return ("b", bool(v))
                if t == sa.STRING:
                    return ("s", self.rt.string(v))
                return (TAG[t], v)
            for i in range(len(ts)):
                row = []
                for j, t in enumerate(types):
                    if isinstance(vals[j][i], list):  # multi-value selection
                        row.append(("list", tuple(dec(t, x) for x in vals[j][i])))
                    elif nulls[j][i]:
                        row.append(None)
                    elif t == sa.INT:
                        row.append(("i", ctypes.c_int32(vals[j][i]).value))
                    elif t == sa.FLOAT:
                        row.append(("f", vals[j][i] & 0xffffffff))
                    elif t == sa.BOOL:
                        row.append(("b", bool(vals[j][i])))
                    elif t == sa.STRING:
                        row.append(("s", self.rt.string(vals[j][i])))
                    else:
                        row.append((TAG[t], vals[j][i]))
                for kind, nm in (("query", name), ("stream", target)):
                    self.records.append({"kind": kind, "name": nm, "ts": ts[i], "expired": False, "values": row})

    def outputs(self):
        return self.records

    def close(self):
        self.rt.shutdown()


def run_product_fixture(fx):
    from oracle_rt import Driver, callback_events
    p = ProductAdapter(fx["app"])
    try:
        def count_fn(ci):
            p.flush()
            return len(callback_events(p.outputs(), fx["callbacks"][ci])[0])
        Driver(fx, p).run(count_fn)
        p.flush()
        return p.outputs()
    finally:
        p.close()
