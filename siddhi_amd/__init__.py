"""siddhi_amd — MI355X-native engine for Siddhi's pattern/sequence NFA path.

Host-side mirror of the reference API the path sits behind (modules/siddhi-core/src/main/java/io/siddhi/core/):

    SiddhiManager.createSiddhiAppRuntime(String)           SiddhiManager.java:93-96
    SiddhiAppRuntime.getInputHandler / addCallback / start / shutdown   SiddhiAppRuntimeImpl.java:260-440
    InputHandler.send(Object[]) / send(long, Object[]) / send(Event) / send(Event[])   stream/input/InputHandler.java:50-95
    QueryCallback.receive(long, Event[], Event[])            query/output/callback/QueryCallback.java:106
    StreamCallback.receive(Event[])                          stream/output/StreamCallback.java:129

Every call goes through the C-ABI in include/siddhi_amd.h (siddhi_amd/_lib/libsiddhi_amd.so). There is no CPU
fallback: importing works anywhere, but creating a runtime needs the gfx950 library and a GPU, and fails loudly
otherwise. Events are processed in batches on the GPU: callbacks fire when a batch is flushed
(SiddhiAppRuntime.flush(), shutdown(), or when the ingestion buffer fills), in the reference's delivery order.
"""
import ctypes
import os
import struct
import time

__all__ = ["SiddhiManager", "SiddhiAppRuntime", "InputHandler", "Event", "QueryCallback", "StreamCallback",
           "SiddhiAppCreationException", "OperationNotSupportedException", "SiddhiParserException",
           "DeviceError", "library_path", "load_library"]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libsiddhi_amd.so")

INT, LONG, FLOAT, DOUBLE, BOOL, STRING = range(6)
_CT = {INT: ctypes.c_int32, LONG: ctypes.c_int64, FLOAT: ctypes.c_float, DOUBLE: ctypes.c_double,
       BOOL: ctypes.c_uint8, STRING: ctypes.c_uint32}


class SiddhiAppCreationException(Exception):
    pass


class SiddhiParserException(SiddhiAppCreationException):
    pass


class OperationNotSupportedException(SiddhiAppCreationException):
    pass


class DeviceError(RuntimeError):
    pass


class CapacityError(RuntimeError):
    pass


_ERRS = {1: SiddhiParserException, 2: SiddhiAppCreationException, 3: OperationNotSupportedException,
         4: ValueError, 5: DeviceError, 6: CapacityError}


class _Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("batch_capacity", ctypes.c_int64), ("max_partials", ctypes.c_int32),
                ("flags", ctypes.c_int32)]


class _Out(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("ts", ctypes.POINTER(ctypes.c_int64)),
                ("expired", ctypes.POINTER(ctypes.c_uint8)), ("n_attrs", ctypes.c_int32),
                ("types", ctypes.POINTER(ctypes.c_int32)),
                ("values", ctypes.POINTER(ctypes.POINTER(ctypes.c_int64))),
                ("nulls", ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))),
                ("event_seq", ctypes.POINTER(ctypes.c_int64))]


class Stats(ctypes.Structure):
    _fields_ = [("events", ctypes.c_int64), ("matches", ctypes.c_int64), ("ms_keygroup", ctypes.c_double),
                ("ms_match", ctypes.c_double), ("ms_total", ctypes.c_double),
                ("keygroup_launches", ctypes.c_int64), ("match_launches", ctypes.c_int64),
                ("path", ctypes.c_int32), ("overflow", ctypes.c_int32),
                ("ms_kg_hist", ctypes.c_double), ("ms_kg_prefix", ctypes.c_double),
                ("ms_kg_scatter", ctypes.c_double), ("ms_chain_carry", ctypes.c_double),
                ("ms_chain_match", ctypes.c_double),
                ("ms_nfa", ctypes.c_double),
                ("ms_chain_emit", ctypes.c_double),
                ("deque", ctypes.c_int32),
                ("fused", ctypes.c_int32),
                ("fused_ovf", ctypes.c_int64),
                ("sched_fires", ctypes.c_int64),
                ("sched_shifted", ctypes.c_int64),
                ("sched_host_keys", ctypes.c_int64), ("sched_rerun_keys", ctypes.c_int64),
                ("ms_nfa_kernel", ctypes.c_double), ("ms_sched_host", ctypes.c_double),
                ("arena_growths", ctypes.c_int64), ("carry_in", ctypes.c_int64), ("carry_out", ctypes.c_int64),
                ("arena_slots", ctypes.c_int64), ("sched_exact_passes", ctypes.c_int64),
                ("sorted_view", ctypes.c_int32), ("spilled_keys", ctypes.c_int32),
                ("host_rows", ctypes.c_int64), ("sub_batches", ctypes.c_int32)]


_lib = None


def library_path():
    return LIB_PATH


def load_library():
    """Load the gfx950 engine library (raises if it was not built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("SDG_LIB", LIB_PATH)  # an alternative build of the same library (A/B measurements)
    if not os.path.exists(path):
        raise DeviceError("siddhi_amd native library missing at %s — run __graft_entry__.build() "
                          "(make -C siddhi_amd); there is no CPU fallback" % LIB_PATH)
    L = ctypes.CDLL(path)
    P, I32, I64, U32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32
    L.sdg_compile.argtypes = [ctypes.c_char_p, ctypes.POINTER(_Opts), ctypes.POINTER(P)]
    L.sdg_destroy.argtypes = [P]
    L.sdg_last_error.restype = ctypes.c_char_p
    L.sdg_stream_index.argtypes = [P, ctypes.c_char_p]
    L.sdg_stream_schema.argtypes = [P, I32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.POINTER(ctypes.c_int32))]
    L.sdg_num_queries.argtypes = [P]
    L.sdg_query_path.argtypes = [P, I32]
    L.sdg_query_flags.argtypes = [P, I32]
    L.sdg_query_name.restype = ctypes.c_char_p
    L.sdg_query_name.argtypes = [P, I32]
    L.sdg_query_target.restype = ctypes.c_char_p
    L.sdg_query_target.argtypes = [P, I32]
    L.sdg_query_output_schema.argtypes = [P, I32, ctypes.POINTER(ctypes.c_int32),
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_int32)),
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_char_p))]
    L.sdg_intern.restype = U32
    L.sdg_intern.argtypes = [P, ctypes.c_char_p, ctypes.c_size_t]
    L.sdg_intern_many.argtypes = [P, I64, P, P, P]
    L.sdg_string.restype = ctypes.c_char_p
    L.sdg_string.argtypes = [P, U32]
    L.sdg_push.argtypes = [P, I32, I64, P, P, P]
    L.sdg_push_events.argtypes = [P, I32, I64, P, P, P]
    L.sdg_push_device.argtypes = [P, I32, I64, P, P, P]
    L.sdg_push_mixed.argtypes = [P, I64, P, P, I32, P, P]
    L.sdg_advance_time.argtypes = [P, I64]
    L.sdg_start.argtypes = [P, I64]
    L.sdg_pending.restype = I64
    L.sdg_pending.argtypes = [P]
    L.sdg_flush.argtypes = [P]
    L.sdg_sync.argtypes = [P]
    L.sdg_poll.argtypes = [P, I32, ctypes.POINTER(_Out)]
    L.sdg_discard.argtypes = [P]
    L.sdg_poll_list.argtypes = [P, I32, I32, ctypes.POINTER(I32), ctypes.POINTER(I32),
                                ctypes.POINTER(ctypes.POINTER(ctypes.POINTER(I64))),
                                ctypes.POINTER(ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)))]
    L.sdg_snapshot.argtypes = [P, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(I64)]
    L.sdg_restore.argtypes = [P, ctypes.c_char_p, I64]
    L.sdg_snapshot_states.argtypes = [P, ctypes.c_char_p, I64, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(I64)]
    L.sdg_export_device.argtypes = [P, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), P, P, P, P]
    L.sdg_export_ordered.argtypes = [P, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), P, P, P, P]
    L.sdg_query_key_attr.argtypes = [P, I32, I32]
    L.sdg_query_reads.argtypes = [P, I32, I32]
    L.sdg_last_stats.argtypes = [P, ctypes.POINTER(Stats)]
    L.sdg_merge_runs.argtypes = [I32, I32, P, P, I32, P, P, P, P]
    _lib = L
    return L


def merge_runs_device(keys, cols, out_keys, out_cols):
    """sdg_merge_runs (merge.hip): stable G-way merge of sorted runs on the GPU. keys: per run a contiguous int64
    CUDA tensor (non-decreasing); cols: per run a list of contiguous CUDA tensors (1 / 2 / 4 / 8-byte elements, one
    per record); out_keys / out_cols: preallocated outputs of the total length. Synchronises torch's stream first
    (the library runs on its own stream and returns when the outputs are written)."""
    import torch
    L = load_library()
    G = len(keys)
    nc = len(out_cols)
    torch.cuda.synchronize()
    kp = (ctypes.c_void_p * G)(*[k.data_ptr() for k in keys])
    ln = (ctypes.c_int64 * G)(*[k.numel() for k in keys])
    cp = (ctypes.c_void_p * max(G * nc, 1))(*[c.data_ptr() for r in cols for c in r])
    wd = (ctypes.c_uint8 * max(nc, 1))(*[c.element_size() for c in out_cols])
    op = (ctypes.c_void_p * max(nc, 1))(*[c.data_ptr() for c in out_cols])
    dev = out_keys.device.index if out_keys.device.index is not None else torch.cuda.current_device()
    _check(L.sdg_merge_runs(dev, G, kp, ln, nc, cp, wd, out_keys.data_ptr(), op))


def _check(rc):
    if rc != 0:
        msg = load_library().sdg_last_error().decode()
        raise _ERRS.get(rc, RuntimeError)(msg)


class Event:
    """io.siddhi.core.event.Event: (timestamp, data, isExpired)"""
    __slots__ = ("timestamp", "data", "expired")

    def __init__(self, timestamp=-1, data=None, expired=False):
        self.timestamp = timestamp
        self.data = list(data) if data is not None else []
        self.expired = expired

    def getData(self, i=None):
        return self.data if i is None else self.data[i]

    def getTimestamp(self):
        return self.timestamp

    def isExpired(self):
        return self.expired

    def __repr__(self):
        return "Event{timestamp=%d, data=%r, isExpired=%s}" % (self.timestamp, self.data, self.expired)


class QueryCallback:
    def receive(self, timestamp, inEvents, removeEvents):  # noqa: N802 (reference API names)
        raise NotImplementedError


class StreamCallback:
    def receive(self, events):
        raise NotImplementedError


class InputHandler:
    def __init__(self, rt, stream_id, index, types):
        self._rt = rt
        self.stream_id = stream_id
        self._idx = index
        self._types = types

    def getStreamId(self):  # noqa: N802
        return self.stream_id

    def send(self, *args):
        """send(data) | send(timestamp, data) | send(Event) | send([Event, ...])"""
        if len(args) == 2:
            self._rt._send(self._idx, self._types, [(int(args[0]), list(args[1]))])
        elif isinstance(args[0], Event):
            self._rt._send(self._idx, self._types, [(args[0].timestamp, args[0].data)])
        elif args and isinstance(args[0], (list, tuple)) and args[0] and isinstance(args[0][0], Event):
            # send(Event[]): the clock moves to the last event's timestamp first (InputHandler.java:85-95)
            self._rt._send(self._idx, self._types, [(ev.timestamp, ev.data) for ev in args[0]], events=True)
        else:
            self._rt._send(self._idx, self._types, [(None, list(args[0]))])

    def send_columns(self, ts, columns, nulls=None):
        """Columnar fast path: ts int64[n], one array per attribute (numpy or ctypes-compatible)."""
        self._rt._push_columns(self._idx, self._types, ts, columns, nulls)


class SiddhiAppRuntime:
    def __init__(self, app_text, device=0, batch_capacity=0, compile_only=False, force_generic=False, fused=True,
                 max_partials=0, seq3=True, sched_exact=False, sched_host=False, sorted_view=True):
        L = load_library()
        self._L = L
        h = ctypes.c_void_p()
        opts = _Opts(device, batch_capacity, max_partials,
                     (1 if compile_only else 0) | (2 if force_generic else 0) | (0 if fused else 4) |
                     (0 if seq3 else 8) | (16 if sched_exact else 0) | (32 if sched_host else 0) |
                     (0 if sorted_view else 64))
        _check(L.sdg_compile(app_text.encode(), ctypes.byref(opts), ctypes.byref(h)))
        self._h = h
        self._compile_only = compile_only
        self._app_text = app_text
        self.playback = "@app:playback" in app_text.replace(" ", "").lower()
        import re as _re
        m = _re.search(r"@app:name\(\s*['\"]([^'\"]*)['\"]", app_text)
        self.name = m.group(1) if m else "siddhi_app"
        self._store = None
        self._last_ts = 0
        self._callbacks = {}  # name -> [callback]
        self._queries = []
        for q in range(L.sdg_num_queries(h)):
            name = L.sdg_query_name(h, q).decode()
            target = L.sdg_query_target(h, q).decode()
            n = ctypes.c_int32()
            types = ctypes.POINTER(ctypes.c_int32)()
            names = ctypes.POINTER(ctypes.c_char_p)()
            _check(L.sdg_query_output_schema(h, q, ctypes.byref(n), ctypes.byref(types), ctypes.byref(names)))
            self._queries.append((name, target, [types[i] for i in range(n.value)],
                                  [names[i].decode() for i in range(n.value)]))
        self._started = False

    # --- reference API ---------------------------------------------------------------------------------
    def getInputHandler(self, stream_id):  # noqa: N802
        idx = self._L.sdg_stream_index(self._h, stream_id.encode())
        if idx < 0:
            raise SiddhiAppCreationException("Stream with id '%s' is not defined" % stream_id)
        n = ctypes.c_int32()
        types = ctypes.POINTER(ctypes.c_int32)()
        _check(self._L.sdg_stream_schema(self._h, idx, ctypes.byref(n), ctypes.byref(types)))
        return InputHandler(self, stream_id, idx, [types[i] for i in range(n.value)])

    def addCallback(self, name, callback):  # noqa: N802
        self._callbacks.setdefault(name, []).append(callback)

    def start(self, timestamp=None):
        """SiddhiAppRuntime.start(); a live (non-playback) app's clock starts at `timestamp` (default: now, ms)"""
        self._started = True
        if timestamp is None:
            timestamp = int(time.time() * 1000)
        _check(self._L.sdg_start(self._h, int(timestamp)))

    def shutdown(self):
        if self._h:
            try:
                if not self._compile_only:
                    self.flush()
            finally:
                self._L.sdg_destroy(self._h)
                self._h = None

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                self._L.sdg_destroy(self._h)
                self._h = None
        except Exception:
            pass

    # --- engine ----------------------------------------------------------------------------------------
    def query_flags(self):
        """per query: SDG_Q_PARTITIONED (1) | SDG_Q_TIMERS (2) | SDG_Q_BROADCAST (4)"""
        return [self._L.sdg_query_flags(self._h, q) for q in range(len(self._queries))]

    def app_stream_ids(self):
        """the app's defined stream ids, in definition order"""
        import re as _re
        return [s for s in _re.findall(r"define\s+stream\s+([A-Za-z_]\w*)", self._app_text, flags=_re.I)
                if self._L.sdg_stream_index(self._h, s.encode()) >= 0]

    def query_key_attr(self, q, stream_id):
        """how query q keys stream_id: attribute index of its value partition, -2 ranges, -3 no key (broadcast), -1
        not read / not partitioned (sdg_query_key_attr)"""
        return self._L.sdg_query_key_attr(self._h, q, self._L.sdg_stream_index(self._h, stream_id.encode()))

    def query_reads(self, q, stream_id):
        """whether query q reads stream_id (sdg_query_reads)"""
        return bool(self._L.sdg_query_reads(self._h, q, self._L.sdg_stream_index(self._h, stream_id.encode())))

    def query_paths(self):
        """device path per query: 0 chain kernel, 1 generic keyed NFA, 2 register sequence kernel (seq3)"""
        return [self._L.sdg_query_path(self._h, q) for q in range(len(self._queries))]

    def intern(self, s):
        b = s.encode()
        return self._L.sdg_intern(self._h, b, len(b))

    def intern_many(self, data, offsets):
        """bulk intern: string i = data[offsets[i]:offsets[i + 1]] (bytes / uint8 array, int64 offsets[n + 1]);
        returns the ids (uint32 numpy array)"""
        import numpy as np
        buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else \
            np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        n = len(off) - 1
        ids = np.empty(max(n, 0), dtype=np.uint32)
        _check(self._L.sdg_intern_many(self._h, n, buf.ctypes.data, off.ctypes.data, ids.ctypes.data))
        return ids

    def string(self, i):
        r = self._L.sdg_string(self._h, i)
        return None if r is None else r.decode()

    def _encode(self, t, v):
        if v is None:
            return 0
        if t == STRING:
            return self.intern(str(v))
        if t == BOOL:
            return 1 if v else 0
        if t in (INT, LONG):
            return int(v)
        return float(v)

    def _send(self, idx, types, rows, events=False):
        n = len(rows)
        ts = (ctypes.c_int64 * n)()
        for i, (t, _) in enumerate(rows):
            if t is None:
                t = self._last_ts if self.playback else int(time.time() * 1000)
            ts[i] = t
            self._last_ts = max(self._last_ts, t)
        cols = (ctypes.c_void_p * max(1, len(types)))()
        nulls = (ctypes.c_void_p * max(1, len(types)))()
        keep = []
        for a, t in enumerate(types):
            arr = (_CT[t] * n)(*[self._encode(t, r[1][a]) for r in rows])
            nl = (ctypes.c_uint8 * n)(*[1 if r[1][a] is None else 0 for r in rows])
            keep += [arr, nl]
            cols[a] = ctypes.cast(arr, ctypes.c_void_p)
            nulls[a] = ctypes.cast(nl, ctypes.c_void_p) if any(r[1][a] is None for r in rows) else None
        self._push(idx, n, ts, cols, nulls, events)

    def _push(self, idx, n, ts, cols, nulls, events=False):
        before = self._L.sdg_pending(self._h)
        push = self._L.sdg_push_events if events else self._L.sdg_push
        _check(push(self._h, idx, n, ts, cols, nulls))
        if self._L.sdg_pending(self._h) < before + n:  # the push filled the batch and flushed it
            self._deliver()

    def _push_columns(self, idx, types, ts, columns, nulls=None):
        import numpy as np
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        n = len(ts)
        cols = (ctypes.c_void_p * max(1, len(types)))()
        nl = (ctypes.c_void_p * max(1, len(types)))()
        keep = [ts]
        dt = {INT: np.int32, LONG: np.int64, FLOAT: np.float32, DOUBLE: np.float64, BOOL: np.uint8, STRING: np.uint32}
        for a, t in enumerate(types):
            c = np.ascontiguousarray(columns[a], dtype=dt[t])
            keep.append(c)
            cols[a] = c.ctypes.data
            if nulls is not None and nulls[a] is not None:
                m = np.ascontiguousarray(nulls[a], dtype=np.uint8)
                keep.append(m)
                nl[a] = m.ctypes.data
        self._push(idx, n, ts.ctypes.data, cols, nl)

    def push_mixed(self, stream_ids, ts, slot_columns, nulls=None):
        """Rows of several streams interleaved in one batch (in send order): stream_ids[i] names row i's stream
        (a sequence of ids, or an int array of sdg stream indices); slot_columns[a][i] = attribute a of row i as an
        int64 slot (int/long value, float/double bit pattern, bool 0/1, string id from intern())."""
        import numpy as np
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        n = len(ts)
        if len(stream_ids) and isinstance(stream_ids[0], str):
            idx = {s: self._L.sdg_stream_index(self._h, s.encode()) for s in set(stream_ids)}
            streams = np.array([idx[s] for s in stream_ids], dtype=np.int32)
        else:
            streams = np.ascontiguousarray(stream_ids, dtype=np.int32)
        cols = [np.ascontiguousarray(c).view(np.int64) if np.asarray(c).dtype.itemsize == 8 else
                np.ascontiguousarray(c, dtype=np.int64) for c in slot_columns]
        cp = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        keep = list(cols)
        nl = None
        if nulls is not None:
            ns = [None if m is None else np.ascontiguousarray(m, dtype=np.uint8) for m in nulls]
            keep += [m for m in ns if m is not None]
            nl = (ctypes.c_void_p * len(ns))(*[None if m is None else m.ctypes.data for m in ns])
        before = self._L.sdg_pending(self._h)
        _check(self._L.sdg_push_mixed(self._h, n, streams.ctypes.data, ts.ctypes.data, len(cols), cp, nl))
        if self._L.sdg_pending(self._h) < before + n:
            self._deliver()

    def push_device(self, stream_id, n, ts_ptr, col_ptrs):
        """Device-resident columns (e.g. torch CUDA tensors' data_ptr()); kept alive by the caller."""
        idx = self._L.sdg_stream_index(self._h, stream_id.encode())
        cols = (ctypes.c_void_p * len(col_ptrs))(*col_ptrs)
        _check(self._L.sdg_push_device(self._h, idx, n, ctypes.c_void_p(ts_ptr), cols, None))

    def advance_time(self, ts):
        """the clock reached ts (playback: event time; live: the wall clock): due absent-state timers fire at the
        next flush, in this position of the input"""
        if self.playback:
            self._last_ts = max(self._last_ts, int(ts))
        _check(self._L.sdg_advance_time(self._h, int(ts)))

    # --- persistence (core/SiddhiAppRuntimeImpl.java:677-737) ------------------------------------------------
    def snapshot(self):
        """every partial match / timer / aggregator state, after processing what was sent; results produced by
        then are delivered to the callbacks"""
        data = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_int64()
        _check(self._L.sdg_snapshot(self._h, ctypes.byref(data), ctypes.byref(n)))
        blob = ctypes.string_at(data, n.value)
        self._deliver()
        return blob

    def restore(self, snapshot):
        try:
            _check(self._L.sdg_restore(self._h, bytes(snapshot), len(snapshot)))
        except (SiddhiAppCreationException, ValueError) as ex:
            raise CannotRestoreSiddhiAppStateException(str(ex))

    def snapshot_states(self, snapshot=None):
        """a snapshot (default: a new one) decoded into the reference's state maps: {query: {"form": ..,
        "states": {partition key: {stateId: StreamPreState.snapshot() map}}}} (StreamPreStateProcessor.java:450-459;
        layout: DESIGN.md "Snapshot state maps")"""
        import json
        blob = self.snapshot() if snapshot is None else bytes(snapshot)
        out = ctypes.c_char_p()
        n = ctypes.c_int64()
        _check(self._L.sdg_snapshot_states(self._h, blob, len(blob), ctypes.byref(out), ctypes.byref(n)))
        doc = json.loads(ctypes.string_at(out, n.value).decode())
        return {q["name"]: {"form": q["form"], "states": q["states"]} for q in doc["queries"]}

    def persist(self):
        """snapshot into the manager's persistence store; returns the revision"""
        if getattr(self, "_store", None) is None:
            raise SiddhiAppCreationException("NoPersistenceStoreException: no persistence store assigned")
        rev = "%d_%s" % (int(time.time() * 1e6), self.name)
        self._store.save(self.name, rev, self.snapshot())
        return rev

    def restoreRevision(self, revision):  # noqa: N802
        blob = self._store.load(self.name, revision) if getattr(self, "_store", None) else None
        if blob is None:
            raise CannotRestoreSiddhiAppStateException("no revision %s of %s" % (revision, self.name))
        self.restore(blob)

    def restoreLastRevision(self):  # noqa: N802
        if getattr(self, "_store", None) is None:
            raise SiddhiAppCreationException("NoPersistenceStoreException: no persistence store assigned")
        rev = self._store.getLastRevision(self.name)
        if rev is not None:
            self.restoreRevision(rev)
        return rev

    def flush(self, deliver=True):
        _check(self._L.sdg_flush(self._h))
        if deliver:
            self._deliver()

    def discard(self):
        """drop the unpolled results of every query (device-resident measurement only)"""
        _check(self._L.sdg_discard(self._h))

    def export_device(self, q, cap, d_ts, d_seq, d_sub, d_vals):
        """copy query q's records of the last flush into device buffers (raw pointers, `cap` records each,
        d_vals: [n_out][cap]); unordered -- delivery order is (seq, sub). Returns the record count."""
        n = ctypes.c_int64()
        _check(self._L.sdg_export_device(self._h, q, cap, ctypes.byref(n), d_ts, d_seq, d_sub, d_vals))
        return n.value

    def export_ordered(self, q, cap, d_ts, d_seq, d_sub, d_vals):
        """export_device with the records already in delivery order ((seq, sub) ascending, ordered on the device):
        a rank's sorted run for the multi-GPU merge. Returns the record count."""
        n = ctypes.c_int64()
        _check(self._L.sdg_export_ordered(self._h, q, cap, ctypes.byref(n), d_ts, d_seq, d_sub, d_vals))
        return n.value

    def stats(self):
        s = Stats()
        _check(self._L.sdg_last_stats(self._h, ctypes.byref(s)))
        return s

    def _lists(self, q, n_attrs):
        """multi-value selections of the last poll: {attr: (cap, items, item_nulls)}"""
        res = {}
        for j in range(n_attrs):
            cap, et = ctypes.c_int32(), ctypes.c_int32()
            items = ctypes.POINTER(ctypes.POINTER(ctypes.c_int64))()
            nls = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))()
            _check(self._L.sdg_poll_list(self._h, q, j, ctypes.byref(cap), ctypes.byref(et), ctypes.byref(items),
                                         ctypes.byref(nls)))
            if cap.value:
                res[j] = (cap.value, items, nls)
        return res

    def _decode(self, t, v):
        if t == INT:
            return ctypes.c_int32(v).value
        if t == LONG:
            return v
        if t == FLOAT:
            return struct.unpack("<f", struct.pack("<I", v & 0xffffffff))[0]
        if t == DOUBLE:
            return struct.unpack("<d", struct.pack("<q", v))[0]
        if t == BOOL:
            return bool(v)
        return self.string(v)

    def poll(self, q):
        out = _Out()
        _check(self._L.sdg_poll(self._h, q, ctypes.byref(out)))
        name, target, types, names = self._queries[q]
        lists = self._lists(q, len(types))
        evs = []
        for i in range(out.n):
            data = []
            for j, t in enumerate(types):
                if j in lists:  # a multi-value selection: the list of the count state's values
                    _, items, nls = lists[j]
                    data.append([None if nls[e][i] else self._decode(t, items[e][i]) for e in range(out.values[j][i])])
                    continue
                if out.nulls[j][i]:
                    data.append(None)
                    continue
                v = out.values[j][i]
                if t == INT:
                    data.append(ctypes.c_int32(v).value)
                elif t == LONG:
                    data.append(v)
                elif t == FLOAT:
                    data.append(struct.unpack("<f", struct.pack("<I", v & 0xffffffff))[0])
                elif t == DOUBLE:
                    data.append(struct.unpack("<d", struct.pack("<q", v))[0])
                elif t == BOOL:
                    data.append(bool(v))
                else:
                    data.append(self.string(v))
            evs.append(Event(out.ts[i], data, bool(out.expired[i])))
        return evs

    def _deliver(self):
        # one callback invocation per match, in delivery order: the receivers hand every returned StateEvent to
        # QuerySelector.process as its own chunk (SingleProcessStreamReceiver.processAndClear :66-71,
        # StateMultiProcessStreamReceiver.processAndClear :58-66), so QueryCallback.receiveStreamEvent and
        # StreamCallback.receive(ComplexEvent) each see a one-event Event[] stamped with that event's timestamp
        for q, (name, target, types, names) in enumerate(self._queries):
            evs = self.poll(q)
            for ev in evs:
                for cb in self._callbacks.get(name, []):
                    cb.receive(ev.timestamp, [ev], None)
                for cb in self._callbacks.get(target, []):
                    cb.receive([ev])

    def poll_arrays(self, q, copy=True):
        """numpy arrays of one poll: (ts[n], values[n_attrs][n] int64 payloads, nulls[n_attrs][n], event_seq[n]);
        copy=True: copies, valid after the next poll; copy=False: views of the engine's poll buffers (sdg_poll's
        contract: valid until the next sdg_poll of this query), values / nulls as lists of per-attribute arrays"""
        import numpy as np
        out = _Out()
        _check(self._L.sdg_poll(self._h, q, ctypes.byref(out)))
        n, na = out.n, out.n_attrs
        if n == 0:
            z = np.zeros(0, np.int64)
            return z, np.zeros((na, 0), np.int64), np.zeros((na, 0), np.uint8), z
        if not copy:
            return (np.ctypeslib.as_array(out.ts, (n,)),
                    [np.ctypeslib.as_array(out.values[j], (n,)) for j in range(na)],
                    [np.ctypeslib.as_array(out.nulls[j], (n,)) for j in range(na)],
                    np.ctypeslib.as_array(out.event_seq, (n,)))
        ts = np.ctypeslib.as_array(out.ts, (n,)).copy()
        seq = np.ctypeslib.as_array(out.event_seq, (n,)).copy()
        vals = np.stack([np.ctypeslib.as_array(out.values[j], (n,)).copy() for j in range(na)]) if na else \
            np.zeros((0, n), np.int64)
        nulls = np.stack([np.ctypeslib.as_array(out.nulls[j], (n,)).copy() for j in range(na)]) if na else \
            np.zeros((0, n), np.uint8)
        return ts, vals, nulls, seq

    def raw_outputs(self, q):
        """(types, ts[n], values[attr][n] payload ints, nulls[attr][n]) straight from sdg_poll"""
        out = _Out()
        _check(self._L.sdg_poll(self._h, q, ctypes.byref(out)))
        n = out.n
        types = self._queries[q][2]
        lists = self._lists(q, len(types))
        vals = []
        for j in range(len(types)):
            if j in lists:  # multi-value selection: a list of payloads (None = null element) per record
                _, items, nls = lists[j]
                vals.append([[None if nls[e][i] else items[e][i] for e in range(out.values[j][i])] for i in range(n)])
            else:
                vals.append([out.values[j][i] for i in range(n)])
        return types, [out.ts[i] for i in range(n)], vals, \
            [[0 if j in lists else out.nulls[j][i] for i in range(n)] for j in range(len(types))]


class InMemoryPersistenceStore:
    """PersistenceStore (core/util/persistence/PersistenceStore.java) kept in memory: revisions per app"""

    def __init__(self):
        self._revs = {}

    def save(self, app_name, revision, snapshot):
        self._revs.setdefault(app_name, []).append((revision, bytes(snapshot)))

    def load(self, app_name, revision):
        for r, b in self._revs.get(app_name, []):
            if r == revision:
                return b
        return None

    def getLastRevision(self, app_name):  # noqa: N802
        revs = self._revs.get(app_name, [])
        return revs[-1][0] if revs else None

    def clearAllRevisions(self, app_name):  # noqa: N802
        self._revs.pop(app_name, None)


class CannotRestoreSiddhiAppStateException(SiddhiAppCreationException):
    pass


class SiddhiManager:
    def __init__(self, device=0):
        self.device = device
        self._store = None

    def setPersistenceStore(self, store):  # noqa: N802
        self._store = store

    def createSiddhiAppRuntime(self, app, batch_capacity=0):  # noqa: N802
        rt = SiddhiAppRuntime(app, device=self.device, batch_capacity=batch_capacity)
        rt._store = self._store
        return rt

    def shutdown(self):
        pass
