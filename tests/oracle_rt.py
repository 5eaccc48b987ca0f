"""ctypes wrapper around the parity oracle (oracle/_build/liboracle.so) + the golden-fixture runner.

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import math
import os
import struct

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "_build", "liboracle.so")

# sql::Type codes
INT, LONG, FLOAT, DOUBLE, BOOL, STRING, OBJECT, LIST = range(8)
TAG_TYPE = {"i": INT, "l": LONG, "f": FLOAT, "d": DOUBLE, "b": BOOL, "s": STRING}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError("oracle not built: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(ORACLE_SO)
        P, I64, I32, U32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
        L.orc_create.restype = P
        L.orc_create.argtypes = [ctypes.c_char_p, ctypes.c_char_p, I32]
        L.orc_destroy.argtypes = [P]
        L.orc_stream_index.argtypes = [P, ctypes.c_char_p]
        L.orc_num_attrs.argtypes = [P, I32]
        L.orc_attr_type.argtypes = [P, I32, I32]
        L.orc_intern.restype = U32
        L.orc_intern.argtypes = [P, ctypes.c_char_p]
        L.orc_string.restype = ctypes.c_char_p
        L.orc_string.argtypes = [P, U32]
        L.orc_start.argtypes = [P, I64]
        L.orc_send_ex.argtypes = [P, I32, I64, I64, I32, ctypes.POINTER(I64), ctypes.POINTER(ctypes.c_uint8)]
        L.orc_send_batch.argtypes = [P, I64, P, P, P, P, P]
        L.orc_advance_time.argtypes = [P, I64]
        L.orc_num_outputs.restype = I64
        L.orc_num_outputs.argtypes = [P]
        L.orc_output.argtypes = [P, I64, ctypes.POINTER(I32), ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(I64),
                                 ctypes.POINTER(I32), ctypes.POINTER(I32)]
        L.orc_output_value.argtypes = [P, I64, I32, ctypes.POINTER(I64), ctypes.POINTER(I32)]
        L.orc_output_list_len.argtypes = [P, I64, I32]
        L.orc_output_list_item.argtypes = [P, I64, I32, I32, ctypes.POINTER(I64), ctypes.POINTER(I32)]
        L.orc_clear_outputs.argtypes = [P]
        L.orc_count_only.argtypes = [P, I32]
        L.orc_output_count.restype = I64
        L.orc_output_count.argtypes = [P]
        L.orc_export_query_outputs.restype = I64
        L.orc_export_query_outputs.argtypes = [P, I64, I32, P, P, P]
        L.orc_last_error.restype = ctypes.c_char_p
        L.orc_state_dump.restype = ctypes.c_char_p
        L.orc_state_dump.argtypes = [P]
        _lib = L
    return _lib


class OracleError(Exception):
    pass


def f32_bits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def f64_bits(x):
    return struct.unpack("<q", struct.pack("<d", x))[0]


def bits_f32(u):
    return struct.unpack("<f", struct.pack("<I", u & 0xffffffff))[0]


def bits_f64(u):
    return struct.unpack("<d", struct.pack("<q", u))[0]


class Oracle:
    def __init__(self, app_text):
        self.playback = "@app:playback" in app_text.replace(" ", "").lower()
        L = lib()
        err = ctypes.create_string_buffer(2048)
        self.h = L.orc_create(app_text.encode(), err, 2048)
        if not self.h:
            raise OracleError(err.value.decode())
        self.L = L

    def close(self):
        if self.h:
            self.L.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self, sid):
        i = self.L.orc_stream_index(self.h, sid.encode())
        if i < 0:
            raise OracleError("unknown stream " + sid)
        return i

    def types(self, si):
        return [self.L.orc_attr_type(self.h, si, a) for a in range(self.L.orc_num_attrs(self.h, si))]

    def encode(self, t, v):
        """python value -> slot for attribute type t"""
        if v is None:
            return 0
        if t in (INT, LONG):
            return int(v)
        if t == FLOAT:
            return f32_bits(float(v))
        if t == DOUBLE:
            return f64_bits(float(v))
        if t == BOOL:
            return 1 if v else 0
        if t == STRING:
            return self.L.orc_intern(self.h, str(v).encode())
        raise OracleError("unsupported attribute type %d" % t)

    def start(self, ts):
        if self.L.orc_start(self.h, ts) != 0:
            raise OracleError(self.L.orc_last_error().decode())

    def send(self, sid, ts, values, now=None, mode=0):
        si = self.stream(sid)
        ts_ = self.types(si)
        if len(values) != len(ts_):
            raise OracleError("arity mismatch for %s" % sid)
        slots = (ctypes.c_int64 * max(1, len(values)))(*[self.encode(t, v) for t, v in zip(ts_, values)])
        nulls = (ctypes.c_uint8 * max(1, len(values)))(*[1 if v is None else 0 for v in values])
        rc = self.L.orc_send_ex(self.h, si, ts, ts if now is None else now, mode, slots, nulls)
        if rc != 0:
            raise OracleError(self.L.orc_last_error().decode())

    def send_events(self, sid, rows):
        """InputHandler.send(Event[]) with rows [(ts, values), ...]: the clock moves to the last event's timestamp,
        then each event is processed without moving it (InputHandler.java:85-95)"""
        if rows and self.playback:
            self.advance(rows[-1][0])
        for ts, values in rows:
            self.send(sid, ts, values, mode=2)

    def advance(self, ts):
        if self.L.orc_advance_time(self.h, ts) != 0:
            raise OracleError(self.L.orc_last_error().decode())

    def decode(self, t, slot, isnull):
        if isnull:
            return None
        if t == INT:
            return ("i", ctypes.c_int32(slot).value)
        if t == LONG:
            return ("l", slot)
        if t == FLOAT:
            return ("f", f32_bits(bits_f32(slot)))
        if t == DOUBLE:
            return ("d", slot)
        if t == BOOL:
            return ("b", bool(slot))
        if t == STRING:
            return ("s", self.L.orc_string(self.h, slot).decode())
        return ("?", slot)

    def state_dump(self):
        """every pattern processor's StreamPreState.snapshot() map per partition key (orc_state_dump)"""
        import json
        r = self.L.orc_state_dump(self.h)
        if r is None:
            raise OracleError(self.L.orc_last_error().decode())
        return json.loads(r.decode())

    def query_arrays(self, nv):
        """query-callback rows as numpy arrays (ts[n], vals[n][nv] slots, nulls[n][nv]) in delivery order"""
        import numpy as np
        cap = self.L.orc_num_outputs(self.h)
        ts = np.zeros(cap, np.int64)
        vals = np.zeros((cap, nv), np.int64)
        nulls = np.zeros((cap, nv), np.uint8)
        k = self.L.orc_export_query_outputs(self.h, cap, nv, ts.ctypes.data, vals.ctypes.data, nulls.ctypes.data)
        return ts[:k], vals[:k], nulls[:k]

    def outputs(self):
        L = self.L
        out = []
        n = L.orc_num_outputs(self.h)
        kind, nv, exp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        name = ctypes.c_char_p()
        ts = ctypes.c_int64()
        slot, isn = ctypes.c_int64(), ctypes.c_int()
        for i in range(n):
            L.orc_output(self.h, i, ctypes.byref(kind), ctypes.byref(name), ctypes.byref(ts), ctypes.byref(exp),
                         ctypes.byref(nv))
            vals = []
            for j in range(nv.value):
                t = L.orc_output_value(self.h, i, j, ctypes.byref(slot), ctypes.byref(isn))
                if t == LIST:
                    items = []
                    for k in range(L.orc_output_list_len(self.h, i, j)):
                        tt = L.orc_output_list_item(self.h, i, j, k, ctypes.byref(slot), ctypes.byref(isn))
                        items.append(self.decode(tt, slot.value, isn.value))
                    vals.append(("list", tuple(items)))
                else:
                    vals.append(self.decode(t, slot.value, isn.value))
            out.append({"kind": "query" if kind.value == 0 else "stream", "name": name.value.decode(),
                        "ts": ts.value, "expired": bool(exp.value), "values": vals})
        return out


# ---------------------------------------------------------------------------------------------------
# fixtures
def tagged_to_py(v):
    if v is None:
        return None
    tag, txt = v.split(":", 1)
    if tag in ("i", "l"):
        return int(txt)
    if tag in ("f", "d"):
        return float(txt)
    if tag == "b":
        return txt == "true"
    return txt


def tagged_expect(v):
    """expected literal -> comparable (tag, canonical)"""
    if v is None:
        return None
    tag, txt = v.split(":", 1)
    if tag == "i":
        return ("i", int(txt))
    if tag == "l":
        return ("l", int(txt))
    if tag == "f":
        # Java float literal: nearest float (strtof), compare bit patterns like Float.equals
        return ("f", f32_bits(float(txt)) if "e" not in txt.lower() else f32_bits(float(txt)))
    if tag == "d":
        return ("d", f64_bits(float(txt)))
    if tag == "b":
        return ("b", txt == "true")
    return ("s", txt)


class Driver:
    """Replays a fixture trace against an engine exposing send/advance/count(callback)."""

    def __init__(self, fx, engine):
        self.fx = fx
        self.e = engine
        self.clock = fx["start_ts"]
        self.playback = fx["playback"]

    def sleep(self, ms):
        self.clock += ms
        if not self.playback:
            self.e.advance(self.clock)

    def run(self, count_fn):
        fx = self.fx
        self.e.start(fx["start_ts"])
        for op in fx["trace"]:
            o = op["op"]
            if o == "send":
                vals = [tagged_to_py(v) for v in op["data"]]
                if self.playback:
                    self.e.send(op["stream"], op["ts"], vals, mode=0 if op["explicit_ts"] else 1)
                else:
                    if op["explicit_ts"]:
                        self.e.send(op["stream"], op["ts"], vals, now=self.clock, mode=0)
                    else:
                        self.e.send(op["stream"], self.clock, vals, now=self.clock, mode=1)
            elif o == "sleep":
                self.sleep(op["ms"])
            elif o == "wait_in_events":
                c = 0
                while True:
                    self.sleep(op["sleep"])
                    c += 1
                    if count_fn(op["callback"]) == 1 or c == op["retry"]:
                        break
            elif o == "wait_events":
                snapshot = count_fn(op["callback"])
                elapsed = 0
                while True:
                    cur = snapshot if op["by_value"] else count_fn(op["callback"])
                    if not (cur < op["count"] and elapsed <= op["timeout"]):
                        break
                    self.sleep(op["sleep"])
                    elapsed += op["sleep"]
            else:
                raise ValueError(o)


def callback_events(outputs, cb):
    ins, rms = [], []
    for o in outputs:
        if o["kind"] == cb["kind"] and o["name"] == cb["name"]:
            if cb["kind"] == "query" and o["expired"]:
                rms.append(o)
            else:
                ins.append(o)
    return ins, rms


def check_fixture(fx, outputs):
    """returns a list of problems (empty == pass)"""
    problems = []
    cbs = fx["callbacks"]
    per_cb = [callback_events(outputs, cb) for cb in cbs]
    exp = fx["expected"]
    if exp.get("count") is not None:
        ci, v = exp["count"]["callback"], exp["count"]["value"]
        got = len(per_cb[ci][0])
        if got != v:
            problems.append("in-event count: expected %d got %d" % (v, got))
    if exp.get("remove_count") is not None:
        ci, v = exp["remove_count"]["callback"], exp["remove_count"]["value"]
        got = len(per_cb[ci][1])
        if got != v:
            problems.append("remove-event count: expected %d got %d" % (v, got))
    if exp.get("arrived") is not None:  # assertEquals(.., true / false, eventArrived) over every callback
        n_any = sum(len(a) + len(r) for a, r in per_cb)
        if exp["arrived"] and n_any == 0:
            problems.append("expected at least one event, got none")
        if not exp["arrived"] and n_any:
            problems.append("expected no event, got %d" % n_any)
    for ci, cb in enumerate(cbs):
        rows = cb["rows"]
        if not rows:
            continue
        actual = [tuple(e["values"]) for e in per_cb[ci][0]]
        want = [tuple(tagged_expect(v) for v in r["values"]) for r in rows]
        if cb["ordered_rows"]:
            for k, w in enumerate(want):
                if k < len(actual) and actual[k] != w:
                    problems.append("row %d: expected %s got %s" % (k, w, actual[k]))
        elif any(r["case"] is not None for r in rows):
            for r, w in zip(rows, want):
                k = (r["case"] or 1) - 1
                if k < len(actual) and actual[k] != w:
                    problems.append("case %s: expected %s got %s" % (r["case"], w, actual[k]))
        else:
            if len(want) == len(actual):
                if sorted(map(repr, want)) != sorted(map(repr, actual)):
                    problems.append("rows: expected %s got %s" % (want, actual))
            else:
                for a in actual:
                    if a not in want:
                        problems.append("unexpected row %s (allowed %s)" % (a, want))
                        break
    return problems


def run_oracle_fixture(fx):
    o = Oracle(fx["app"])
    try:
        def count_fn(ci):
            cb = fx["callbacks"][ci]
            return len(callback_events(o.outputs(), cb)[0])
        Driver(fx, o).run(count_fn)
        return o.outputs()
    finally:
        o.close()
