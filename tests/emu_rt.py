"""TEST-ONLY: the host build of the product's keyed-NFA code (tests/native/libnfa_emu.so) driven like the
oracle, so the NFA state machine is checked against the oracle on CPU. See tests/native/nfa_emu.cpp."""
import ctypes
import os

from oracle_rt import BOOL, DOUBLE, FLOAT, INT, LONG, STRING, f32_bits, f64_bits

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_SO = os.path.join(REPO, "tests", "native", "_build", "libnfa_emu.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(EMU_SO):
            raise RuntimeError("emulation harness not built: run `make -C tests/native`")
        L = ctypes.CDLL(EMU_SO)
        P, I64, I32, U32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
        L.emu_error.restype = ctypes.c_char_p
        L.emu_create.restype = P
        L.emu_create.argtypes = [ctypes.c_char_p, I32]
        L.emu_destroy.argtypes = [P]
        L.emu_stream_index.argtypes = [P, ctypes.c_char_p]
        L.emu_stream_nattrs.argtypes = [P, I32]
        L.emu_stream_attr_type.argtypes = [P, I32, I32]
        L.emu_intern.restype = U32
        L.emu_intern.argtypes = [P, ctypes.c_char_p]
        L.emu_string.restype = ctypes.c_char_p
        L.emu_string.argtypes = [P, U32]
        L.emu_send.argtypes = [P, I32, I64, ctypes.POINTER(I64), ctypes.POINTER(ctypes.c_uint8)]
        L.emu_flush.argtypes = [P]
        L.emu_advance.argtypes = [P, I64]
        L.emu_send_batch.argtypes = [P, I64, P, P, P, P, P]
        L.emu_sched_stat.restype = I64
        L.emu_sched_stat.argtypes = [I32]
        L.emu_start.argtypes = [P, I64]
        L.emu_set_reclaim.argtypes = [I32]
        L.emu_idles.restype = I64
        L.emu_num_queries.argtypes = [P]
        for f in ("emu_query_name", "emu_query_target"):
            getattr(L, f).restype = ctypes.c_char_p
            getattr(L, f).argtypes = [P, I32]
        L.emu_query_nout.argtypes = [P, I32]
        L.emu_query_out_type.argtypes = [P, I32, I32]
        L.emu_query_chain.argtypes = [P, I32]
        L.emu_num_out.restype = I64
        L.emu_num_out.argtypes = [P, I32]
        L.emu_out.argtypes = [P, I32, I64, ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(U32), ctypes.POINTER(I64)]
        _lib = L
    return _lib


class EmuError(Exception):
    pass


class EmuAdapter:
    def __init__(self, app, max_partials=0):
        self.L = lib()
        self.h = self.L.emu_create(app.encode(), max_partials)
        if not self.h:
            raise EmuError(self.L.emu_error().decode())
        self.playback = "@app:playback" in app.replace(" ", "").lower()
        self.last_ts = 0
        self.nq = self.L.emu_num_queries(self.h)
        self.meta = []
        for q in range(self.nq):
            types = [self.L.emu_query_out_type(self.h, q, j) for j in range(self.L.emu_query_nout(self.h, q))]
            self.meta.append((self.L.emu_query_name(self.h, q).decode(), self.L.emu_query_target(self.h, q).decode(),
                              types))
        self.delivered = [0] * self.nq
        self.records = []

    def start(self, ts):
        self.L.emu_start(self.h, ts)

    def send(self, sid, ts, values, now=None, mode=0):
        if not self.playback and now is not None:
            self.L.emu_advance(self.h, now)  # the wall clock at this send (timers due by then fire first)
        si = self.L.emu_stream_index(self.h, sid.encode())
        if si < 0:
            raise EmuError("unknown stream " + sid)
        types = [self.L.emu_stream_attr_type(self.h, si, a) for a in range(self.L.emu_stream_nattrs(self.h, si))]
        if mode == 1 and self.playback:
            ts = self.last_ts
        self.last_ts = max(self.last_ts, ts)
        enc = []
        for t, v in zip(types, values):
            if v is None:
                enc.append(0)
            elif t in (INT, LONG):
                enc.append(int(v))
            elif t == FLOAT:
                enc.append(f32_bits(float(v)))
            elif t == DOUBLE:
                enc.append(f64_bits(float(v)))
            elif t == BOOL:
                enc.append(1 if v else 0)
            elif t == STRING:
                enc.append(self.L.emu_intern(self.h, str(v).encode()))
            else:
                raise EmuError("attribute type %d" % t)
        vals = (ctypes.c_int64 * max(1, len(enc)))(*enc)
        nulls = (ctypes.c_uint8 * max(1, len(enc)))(*[1 if v is None else 0 for v in values])
        self.L.emu_send(self.h, si, ts, vals, nulls)

    def advance(self, ts):
        self.L.emu_advance(self.h, ts)

    def flush(self):
        if self.L.emu_flush(self.h) != 0:
            raise EmuError(self.L.emu_error().decode())
        ts, nl = ctypes.c_int64(), ctypes.c_uint32()
        vals = (ctypes.c_int64 * 64)()
        seq = (ctypes.c_int64 * 2)()
        for q in range(self.nq):
            name, target, types = self.meta[q]
            n = self.L.emu_num_out(self.h, q)
            for i in range(self.delivered[q], n):
                self.L.emu_out(self.h, q, i, ctypes.byref(ts), vals, ctypes.byref(nl), seq)
                row = []
                for j, t in enumerate(types):
                    v = vals[j]
                    if (nl.value >> j) & 1:
                        row.append(None)
                    elif t == INT:
                        row.append(("i", ctypes.c_int32(v).value))
                    elif t == LONG:
                        row.append(("l", v))
                    elif t == FLOAT:
                        row.append(("f", v & 0xffffffff))
                    elif t == DOUBLE:
                        row.append(("d", v))
                    elif t == BOOL:
                        row.append(("b", bool(v)))
                    elif t == STRING:
                        row.append(("s", self.L.emu_string(self.h, v).decode()))
                    else:
                        row.append(("?", v))
                for kind, nm in (("query", name), ("stream", target)):
                    self.records.append({"kind": kind, "name": nm, "ts": ts.value, "expired": False, "values": row,
                                         "seq": seq[0], "ordinal": seq[1]})
            self.delivered[q] = n

    def outputs(self):
        return self.records

    def close(self):
        if self.h:
            self.L.emu_destroy(self.h)
            self.h = None


def run_emu_fixture(fx, max_partials=0):
    from oracle_rt import Driver, callback_events
    p = EmuAdapter(fx["app"], max_partials)
    try:
        def count_fn(ci):
            p.flush()
            return len(callback_events(p.outputs(), fx["callbacks"][ci])[0])
        Driver(fx, p).run(count_fn)
        p.flush()
        return p.outputs()
    finally:
        p.close()
