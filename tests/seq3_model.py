"""Register model of the SEQUENCE shape `every e1=S[f1], e2=S[f2]<m:n>, e3=S[f3]` (one stream, per partition key),
the semantics the seq3 kernel (siddhi_amd/csrc/kernels/seq3.hip) implements. Derived from the processors
(reference paths under modules/siddhi-core/src/main/java/io/siddhi/core/query/input/stream/state/):

* SequenceMultiProcessStreamReceiver: per event, stabilizeStates -> resetState of every state (pending lists cleared,
  StreamPreStateProcessor.java:288-305) -> updateState (newAndEvery -> pending, :308-323); then the states in reverse
  order e3, e2, e1 (PatternMultiProcessStreamReceiver.java:33-39).
* SEQUENCE addState keeps at most one state event per newAndEvery list (StreamPreStateProcessor.java:214-227,
  CountPreStateProcessor.java:97-125), so per key there is at most one partial waiting at e2 (Q) and one at e3 (P);
  they are the same object when the count state forwarded and re-added it (CountPostStateProcessor.java:49-58: both
  only when n >= min; re-added to e2 only while n != max).
* e3 matching P sets P's e3 slot, so e2 drops the same object (CountPreStateProcessor.java:58-62 nextProcessed).
* e1 (every) always holds one seed; a passing event adds a new partial to e2's newAndEvery only if that list is
  still empty, i.e. when Q did not stay at e2 in this event.

Test infrastructure only (tests/test_seq3_model.py pins it against the oracle on random traces)."""


def run_key(events, f1, f2, f3, m, n, within=None, ts=None):
    """events: list of (pos, row) of ONE key in order; f1(y), f2(y, e1, e2_list_with_y), f3(y, e1, e2_list).
    within: `within T` (ts(row) gives an event's timestamp): before each event, stabilizeStates expires a partial
    whose e1 is more than T away (StreamPreStateProcessor.isExpired :118-129; the every-start's extra seed from
    withinEveryPreStateProcessor changes no output: e2 keeps one partial). Returns [(pos, (e1, e2_list, y))]."""
    out = []
    P = None      # partial at e3: (e1, e2 list)
    Q = None      # partial at e2: (e1, e2 list)
    same = False  # P is Q (one object)
    for pos, y in events:
        if within is not None:
            if P is not None and abs(ts(P[0]) - ts(y)) > within:
                P, same = None, False
            if Q is not None and abs(ts(Q[0]) - ts(y)) > within:
                Q, same = None, False
        consumed = False
        if P is not None:
            if f3(y, P[0], P[1]):
                out.append((pos, (P[0], list(P[1]), y)))
                consumed = same
        nP, nQ, nsame = None, None, False
        if Q is not None and not consumed:
            lst = Q[1] + [y]
            if f2(y, Q[0], lst):
                if len(lst) >= m:
                    nP = (Q[0], lst)
                    if len(lst) != n:
                        nQ = nP
                        nsame = True
        if f1(y) and nQ is None:
            nQ = (y, [])
            nsame = False
        P, Q, same = nP, nQ, nsame
    return out
