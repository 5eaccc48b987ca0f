#!/usr/bin/env python3
"""Generate golden fixtures from the reference's own pattern/sequence known-answer tests.

Reads the reference TestNG sources as TEXT (study only — nothing from the reference is executed or
imported) and writes one JSON fixture per test method: the SiddhiQL app, the input trace and the
expectations the test asserts (expected rows and/or expected counts). Fixtures are data; the reference
sources are not copied.

Modelling assumptions, recorded in every fixture's "model" field:
  * Wall-clock tests (no @app:playback): each `Thread.sleep(d)` advances a modelled clock by d ms;
    `send(Object[])` gets the modelled clock as its timestamp; scheduler timers fire in notify-time
    order whenever the modelled clock passes them (SURVEY.md 8(c) "sleep -> ts delta").
  * Playback tests keep their explicit timestamps.
Run:  python tests/golden/gen_golden.py  [--ref /root/reference]   (needs the reference checkout; the
generated fixtures under tests/golden/fixtures/ are committed and are what the tests read.)
"""
import argparse
import json
import os
import re
import sys

TEST_ROOT = "modules/siddhi-core/src/test/java/io/siddhi/core/query"
FILES = [
    "pattern/WithinPatternTestCase.java",
    "pattern/EveryPatternTestCase.java",
    "pattern/CountPatternTestCase.java",
    "pattern/LogicalPatternTestCase.java",
    "pattern/ComplexPatternTestCase.java",
    "sequence/SequenceTestCase.java",
    "partition/PatternPartitionTestCase.java",
    "partition/SequencePartitionTestCase.java",
    "pattern/absent/AbsentPatternTestCase.java",
    "pattern/absent/EveryAbsentPatternTestCase.java",
    "pattern/absent/AbsentWithEveryPatternTestCase.java",
    "pattern/absent/LogicalAbsentPatternTestCase.java",
    "sequence/absent/AbsentSequenceTestCase.java",
    "sequence/absent/EveryAbsentSequenceTestCase.java",
    "sequence/absent/AbsentWithEverySequenceTestCase.java",
    "sequence/absent/LogicalAbsentSequenceTestCase.java",
]
LIVE_T0 = 1_000_000  # modelled wall clock at siddhiAppRuntime.start()

TOKEN_RE = re.compile(r'''
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/)
  | (?P<str>"(?:\\.|[^"\\])*")
  | (?P<chr>'(?:\\.|[^'\\])')
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[fFdDlL]?)
  | (?P<id>[A-Za-z_$][A-Za-z_$0-9]*)
  | (?P<sym>==|!=|<=|>=|&&|\|\||\+\+|--|\+=|->|[{}()\[\];,.=<>+\-*/%!?:&|@^~])
''', re.S | re.X)


def tokenize(src):
    out = []
    pos = 0
    while pos < len(src):
        m = TOKEN_RE.match(src, pos)
        if not m:
            raise ValueError("cannot tokenize at %d: %r" % (pos, src[pos:pos + 20]))
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        out.append((kind, m.group(kind), m.start()))
    return out


def unescape(s):
    body = s[1:-1]
    return bytes(body, "utf-8").decode("unicode_escape")


class Skip(Exception):
    pass


def find_methods(toks, src):
    """yield (name, line, body_tokens) for each @Test method"""
    i = 0
    while i < len(toks):
        if toks[i][1] == "@" and i + 1 < len(toks) and toks[i + 1][1] == "Test":
            j = i + 2
            while j < len(toks) and toks[j][1] != "void":
                j += 1
            name = toks[j + 1][1]
            line = src.count("\n", 0, toks[j + 1][2]) + 1
            k = j
            while toks[k][1] != "{":
                k += 1
            depth, start = 0, k
            while True:
                if toks[k][1] == "{":
                    depth += 1
                elif toks[k][1] == "}":
                    depth -= 1
                    if depth == 0:
                        break
                k += 1
            yield name, line, toks[start + 1:k]
            i = k
        else:
            i += 1


def eval_string_expr(toks, i, env, stop=(";",)):
    """evaluate `"a" + x + "b"` starting at i; returns (value, next index)"""
    parts = []
    depth = 0
    while i < len(toks) and not (depth == 0 and toks[i][1] in stop):
        kind, text, _ = toks[i]
        if text == "(":
            depth += 1
        elif text == ")":
            if depth == 0:
                break
            depth -= 1
        elif kind == "str":
            parts.append(unescape(text))
        elif kind == "id":
            if text not in env:
                raise Skip("unknown string variable " + text)
            parts.append(env[text])
        elif text == "+":
            pass
        else:
            raise Skip("unsupported string expression token " + text)
        i += 1
    return "".join(parts), i


def eval_int_expr(toks, i, stop, longs=None):
    """constant / `now`-style long expression (supports ++x, x++, x + c); mutates longs"""
    longs = {} if longs is None else longs
    expr = []
    depth = 0
    while not (depth == 0 and toks[i][1] in stop):
        t = toks[i][1]
        if t == "(":
            depth += 1
        elif t == ")":
            depth -= 1
        if t in ("++", "--") and toks[i + 1][1] in longs:  # pre-increment
            v = toks[i + 1][1]
            longs[v] += 1 if t == "++" else -1
            expr.append(str(longs[v]))
            i += 2
            continue
        if toks[i][0] == "id" and t in longs:
            if toks[i + 1][1] in ("++", "--"):  # post-increment
                expr.append(str(longs[t]))
                longs[t] += 1 if toks[i + 1][1] == "++" else -1
                i += 2
                continue
            expr.append(str(longs[t]))
            i += 1
            continue
        expr.append(t)
        i += 1
    s = "".join(expr)
    if not re.fullmatch(r"[0-9+\-*/ ()L]+", s):
        raise Skip("non-constant int expression " + s)
    return int(eval(s.replace("L", ""))), i


def literal(toks, i):
    """parse one Java literal value -> (tagged value, next index)"""
    kind, text, _ = toks[i]
    neg = False
    if text in ("-", "+"):
        neg = text == "-"
        i += 1
        kind, text, _ = toks[i]
    if kind == "str":
        return "s:" + unescape(text), i + 1
    if kind == "num":
        t = text
        sign = "-" if neg else ""
        if t[-1] in "fF":
            return "f:" + sign + t[:-1], i + 1
        if t[-1] in "lL":
            return "l:" + sign + t[:-1], i + 1
        if t[-1] in "dD":
            return "d:" + sign + t[:-1], i + 1
        if "." in t or "e" in t or "E" in t:
            return "d:" + sign + t, i + 1
        return "i:" + sign + t, i + 1
    if text in ("true", "false"):
        return "b:" + text, i + 1
    if text == "null":
        return None, i + 1
    raise Skip("non-literal value " + text)


def object_array(toks, i, longs=None, now=None):
    """`new Object[]{...}` starting at `new` -> (values, next index); `now`-style long expressions (++now) are
    evaluated against `longs` (mutating it, in Java's left-to-right order)"""
    if [t[1] for t in toks[i:i + 5]] != ["new", "Object", "[", "]", "{"]:
        raise Skip("expected new Object[]{...}")
    i += 5
    vals = []
    while toks[i][1] != "}":
        if now is not None and [t[1] for t in toks[i:i + 5]] == ["System", ".", "currentTimeMillis", "(", ")"]:
            vals.append("l:%d" % now)  # the modelled wall clock at the send
            i += 5
            if toks[i][1] == ",":
                i += 1
            continue
        if longs is not None and (toks[i][1] in ("++", "--") or (toks[i][0] == "id" and toks[i][1] in longs)):
            n, i = eval_int_expr(toks, i, (",", "}"), longs)
            v = "l:%d" % n
        else:
            v, i = literal(toks, i)
        vals.append(v)
        if toks[i][1] == ",":
            i += 1
    return vals, i + 1


def skip_balanced(toks, i):
    """toks[i] is an opening bracket; return index after its match"""
    pairs = {"(": ")", "{": "}", "[": "]"}
    o = toks[i][1]
    c = pairs[o]
    depth = 0
    while True:
        if toks[i][1] == o:
            depth += 1
        elif toks[i][1] == c:
            depth -= 1
            if depth == 0:
                return i + 1
        i += 1


def parse_callback_body(toks, a, b):
    """expected rows inside a callback anonymous class [a, b)"""
    rows = []
    case = None
    i = a
    while i < b:
        t = toks[i][1]
        if t == "case" and toks[i + 1][0] == "num":
            case = int(toks[i + 1][1])
        if t == "assertArrayEquals" and toks[i + 1][1] == "(":
            try:
                vals, j = object_array(toks, i + 2)
            except Skip:
                i += 1
                continue
            rows.append((case, vals))
            case = None
        i += 1
    return rows


def unroll_loops(body, limit=200_000):
    """`for (int X = A; X < B; X++) { ... }` with literal bounds -> the body B - A times, X replaced by its value
    (the input traces of e.g. CountPatternTestCase.testQuery16 are such loops)"""
    out = []
    i = 0
    n = len(body)
    while i < n:
        t = [x[1] for x in body[i:i + 13]]
        if (len(t) == 13 and t[0] == "for" and t[1] == "(" and t[2] == "int" and t[4] == "=" and t[6] == ";" and
                t[7] == t[3] and t[8] in ("<", "<=") and t[10] == ";" and
                ((t[11] == t[3] and t[12] == "++") or (t[11] == "++" and t[12] == t[3])) and
                body[i + 5][0] == "num" and body[i + 9][0] == "num" and body[i + 13][1] == ")" and
                body[i + 14][1] == "{"):
            var = t[3]
            lo, hi = int(t[5]), int(t[9]) + (1 if t[8] == "<=" else 0)
            end = skip_balanced(body, i + 14)
            inner = unroll_loops(body[i + 15:end - 1], limit)
            if (hi - lo) * len(inner) + len(out) > limit:
                raise Skip("loop too long to unroll")
            for v in range(lo, hi):
                out.extend(("num", str(v), x[2]) if x[0] == "id" and x[1] == var else x for x in inner)
            i = end
            continue
        out.append(body[i])
        i += 1
    return out


def extract(name, line, body, relpath, class_src):
    body = unroll_loops(body)
    env = {}
    longs = {}
    app = None
    handlers = {}
    callbacks = []
    cb_vars = {}
    trace = []
    started = False
    expected_count = None
    remove_count = None
    arrived = None  # True / False: the test asserts that some / no event arrived
    clock = LIVE_T0
    i = 0
    n = len(body)

    def counter_callback(argtoks):
        """which callback a counter expression refers to (index) -> int"""
        txt = "".join(t[1] for t in argtoks)
        for v, idx in cb_vars.items():
            if txt.startswith(v + "."):
                return idx
        return 0

    while i < n:
        kind, text, _ = body[i]
        # String x = ... ;
        if text == "String" and body[i + 1][0] == "id" and body[i + 2][1] == "=":
            var = body[i + 1][1]
            try:
                val, j = eval_string_expr(body, i + 3, env)
                env[var] = val
                i = j
            except Skip:
                i += 3
            continue
        if text == "long" and body[i + 1][0] == "id" and body[i + 2][1] == "=":
            var = body[i + 1][1]
            if body[i + 3][1] == "System" and body[i + 5][1] == "currentTimeMillis":
                longs[var] = LIVE_T0
                i += 8
            else:
                longs[var], i = eval_int_expr(body, i + 3, (";",), longs)
            continue
        if kind == "id" and text in longs and body[i + 1][1] in ("+=", "-=", "="):
            op = body[i + 1][1]
            v, j = eval_int_expr(body, i + 2, (";",), longs)
            longs[text] = longs[text] + v if op == "+=" else longs[text] - v if op == "-=" else v
            i = j
            continue
        if kind == "id" and body[i + 1][1] == "+=" and text in env:
            val, j = eval_string_expr(body, i + 2, env)
            env[text] += val
            i = j
            continue
        if text == "createSiddhiAppRuntime" and body[i + 1][1] == "(":
            app, j = eval_string_expr(body, i + 2, env, stop=(")",))
            i = j
            continue
        if text == "getInputHandler" and body[i + 1][1] == "(":
            sid = unescape(body[i + 2][1])
            k = i
            while body[k][1] != "=":
                k -= 1
            handlers[body[k - 1][1]] = sid
            i += 3
            continue
        if text in ("addQueryCallback", "addStreamCallback") and body[i - 2][1] == "TestUtil":
            # TestUtil.addXCallback(runtime, "name", new Object[]{...}, ...)  (expected rows in order)
            k = i
            while body[k][1] != "=":
                k -= 1
            var = body[k - 1][1]
            end = skip_balanced(body, i + 1)
            j = i + 2
            while body[j][1] != ",":
                j += 1
            cbname = unescape(body[j + 1][1])
            j += 2
            rows = []
            while j < end - 1:
                if body[j][1] == ",":
                    j += 1
                    continue
                vals, j = object_array(body, j)
                rows.append((None, vals))
            cb_vars[var] = len(callbacks)
            callbacks.append({"kind": "query" if text == "addQueryCallback" else "stream", "name": cbname,
                              "rows": rows, "ordered": True})
            i = end
            continue
        if text == "addCallback" and body[i + 1][1] == "(" and body[i + 2][0] == "str":
            cbname = unescape(body[i + 2][1])
            ctype = body[i + 5][1] if body[i + 4][1] == "new" else None
            if ctype not in ("QueryCallback", "StreamCallback"):
                raise Skip("unsupported callback " + str(ctype))
            k = i + 6
            while body[k][1] != "{":
                k += 1
            end = skip_balanced(body, k)
            callbacks.append({"kind": "query" if ctype == "QueryCallback" else "stream", "name": cbname,
                              "rows": parse_callback_body(body, k, end), "ordered": False})
            i = end
            continue
        if text == "start" and body[i - 1][1] == "." and body[i + 1][1] == "(":
            started = True
            i += 1
            continue
        if started and text == "shutdown" and body[i - 1][1] == ".":
            started = False  # the runtime is gone: later sleeps/sends do not reach it
            i += 1
            continue
        if started and text in ("for", "while") and body[i + 1][1] == "(":
            raise Skip("loop in the input trace")
        if started and text == "send" and body[i - 1][1] == "." and body[i - 2][1] in handlers:
            sid = handlers[body[i - 2][1]]
            j = i + 2
            if body[j][1] == "new" and body[j + 1][1] == "Object":
                vals, j = object_array(body, j, longs, clock)
                trace.append({"op": "send", "stream": sid, "ts": clock, "data": vals, "explicit_ts": False})
            elif body[j][1] == "new" and body[j + 1][1] == "Event":
                if body[j + 2][1] == "[":
                    raise Skip("Event[] batch send")
                ts, j2 = eval_int_expr(body, j + 3, (",",), longs)
                vals, j = object_array(body, j2 + 1, longs)
                trace.append({"op": "send", "stream": sid, "ts": ts, "data": vals, "explicit_ts": True})
            else:
                ts, j2 = eval_int_expr(body, j, (",",), longs)
                vals, j = object_array(body, j2 + 1, longs)
                trace.append({"op": "send", "stream": sid, "ts": ts, "data": vals, "explicit_ts": True})
            i = j
            continue
        if started and text == "sleep" and body[i - 1][1] == "." and body[i - 2][1] == "Thread":
            d, j = eval_int_expr(body, i + 2, (")",), longs)
            clock += d
            trace.append({"op": "sleep", "ms": d})
            i = j
            continue
        if started and text == "waitForInEvents" and body[i + 1][1] == "(":
            end = skip_balanced(body, i + 1)
            args = [t[1] for t in body[i + 2:end - 1]]
            parts = "".join(args).split(",")
            trace.append({"op": "wait_in_events", "sleep": int(parts[0]), "callback": cb_vars.get(parts[1], 0),
                          "retry": int(parts[2])})
            i = end
            continue
        if started and text == "waitForEvents" and body[i + 1][1] == "(":
            end = skip_balanced(body, i + 1)
            argt = body[i + 2:end - 1]
            pieces, cur, depth = [], [], 0
            for t in argt:
                if t[1] in "([{":
                    depth += 1
                elif t[1] in ")]}":
                    depth -= 1
                if t[1] == "," and depth == 0:
                    pieces.append(cur)
                    cur = []
                else:
                    cur.append(t)
            pieces.append(cur)
            if len(pieces) == 4:
                sleep_ms = int("".join(t[1] for t in pieces[0]).replace("L", ""))
                cnt = int(eval("".join(t[1] for t in pieces[1])))
                ctr = pieces[2]
                ctr_name = ctr[0][1]
                atomic = re.search(r"AtomicInteger\s+" + re.escape(ctr_name) + r"\b", class_src) is not None \
                    or ".get" in "".join(t[1] for t in ctr)
                timeout = int("".join(t[1] for t in pieces[3]).replace("L", ""))
                trace.append({"op": "wait_events", "sleep": sleep_ms, "count": cnt, "timeout": timeout,
                              "callback": counter_callback(ctr), "by_value": not atomic})
            else:
                trace.append({"op": "sleep", "ms": int("".join(t[1] for t in pieces[0]).replace("L", ""))})
            i = end
            continue
        if started and text in ("assertEquals",) and body[i + 1][1] == "(":
            end = skip_balanced(body, i + 1)
            args = body[i + 2:end - 1]
            joined = " ".join(t[1] for t in args).lower()
            m_in = "ineventcount" in joined
            m_rm = "removeeventcount" in joined
            if re.search(r"\btrue\s*,\s*eventarrived\b", joined) or re.search(r"\beventarrived\s*,\s*true\b", joined):
                arrived = True  # assertEquals("Event arrived", true, eventArrived): at least one event delivered
            elif re.search(r"\bfalse\s*,\s*eventarrived\b", joined) or re.search(r"\beventarrived\s*,\s*false\b", joined):
                arrived = False  # ... false, eventArrived: nothing delivered
            if (m_in or m_rm) and "getdata" not in joined:
                pieces, depth, cur = [], 0, []
                for t in args:
                    if t[1] in "([{":
                        depth += 1
                    elif t[1] in ")]}":
                        depth -= 1
                    if t[1] == "," and depth == 0:
                        pieces.append(cur)
                        cur = []
                    else:
                        cur.append(t)
                pieces.append(cur)
                val = None
                ctr_cb = 0
                for p in pieces:
                    s2 = "".join(t[1] for t in p)
                    if re.fullmatch(r"[0-9+\-*/ ()]+", s2):
                        val = int(eval(s2))
                    elif "count" in s2.lower():
                        ctr_cb = counter_callback(p)
                if val is not None:
                    if m_in and not m_rm:
                        expected_count = (ctr_cb, val)
                    elif m_rm:
                        remove_count = (ctr_cb, val)
            i = end
            continue
        i += 1
    if app is None:
        raise Skip("no app")
    if not callbacks:
        raise Skip("no callback")
    playback = "@app:playback" in app.replace(" ", "")
    return {
        "source": "%s/%s:%d" % (TEST_ROOT, relpath, line),
        "test": name,
        "app": app,
        "playback": playback,
        "start_ts": LIVE_T0,
        "trace": trace,
        "callbacks": [{"kind": c["kind"], "name": c["name"], "ordered_rows": c["ordered"],
                       "rows": [{"case": r[0], "values": r[1]} for r in c["rows"]]} for c in callbacks],
        "expected": {
            "count": None if expected_count is None else {"callback": expected_count[0], "value": expected_count[1]},
            "remove_count": None if remove_count is None else {"callback": remove_count[0], "value": remove_count[1]},
            "arrived": arrived,
        },
        "model": "playback timestamps (sleeps do not move the engine clock)" if playback else
                 "wall-clock test: Thread.sleep(d) -> modelled clock += d; timers fire as the clock passes them",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    stats = {"written": 0, "skipped": 0}
    skipped = []
    for rel in FILES:
        path = os.path.join(a.ref, TEST_ROOT, rel)
        src = open(path, encoding="utf-8").read()
        toks = tokenize(src)
        for name, line, body in find_methods(toks, src):
            try:
                fx = extract(name, line, body, rel, src)
            except Skip as e:
                stats["skipped"] += 1
                skipped.append("%s:%d %s: %s" % (rel, line, name, e))
                continue
            base = os.path.splitext(os.path.basename(rel))[0]
            fn = os.path.join(a.out, "%s__%s.json" % (base, name))
            with open(fn, "w") as f:
                json.dump(fx, f, indent=1)
            stats["written"] += 1
    with open(os.path.join(a.out, "_skipped.txt"), "w") as f:
        f.write("\n".join(skipped) + "\n")
    print(json.dumps(stats))


if __name__ == "__main__":
    sys.exit(main())
