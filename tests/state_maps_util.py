"""Comparison of the engine's decoded snapshot state maps (sdg_snapshot_states) with the oracle's (orc_state_dump);
used by tests/test_gpu_state_maps.py and tests/test_state_maps.py."""


def project(o, e):
    """oracle events carry every attribute of their stream; keep those the engine's event names"""
    if isinstance(o, dict) and isinstance(e, dict):
        if isinstance(o.get("data"), list) and isinstance(e.get("data"), dict):
            d = o["data"]
            return {"ts": o["ts"], "data": {k: d[int(k)] if int(k) < len(d) else "<missing>" for k in e["data"]}}
        return {k: (project(v, e[k]) if k in e else v) for k, v in o.items()}
    if isinstance(o, list) and isinstance(e, list) and len(o) == len(e):
        return [project(a, b) for a, b in zip(o, e)]
    return o


def merge_lists(states):
    """what the next event's updateState() sees: NewAndEvery appended to Pending; the start state's seed (no
    bound event) without its timestamp; keys whose only state is that seed (equal to a fresh key) left out"""
    out = {}
    for key, procs in states.items():
        ms = {}
        for sid, m in procs.items():
            m = dict(m)
            lst = m["PendingStateEventList"] + m["NewAndEveryStateEventList"]
            m["PendingStateEventList"] = [dict(s, ts=-1) if all(x is None for x in s["events"]) else s for s in lst]
            m["NewAndEveryStateEventList"] = []
            ms[sid] = m
        seed_only = list(ms) == ["0"] and all(all(x is None for x in s["events"])
                                              for s in ms["0"]["PendingStateEventList"])
        if not seed_only:
            out[key] = ms
    return out


def check_maps(ref, got, expect_form):
    """ref: {query: states} from the oracle; got: SiddhiAppRuntime.snapshot_states(); returns the number of
    StateEvents compared"""
    assert set(got) == set(ref)
    n = 0
    for name, g in got.items():
        assert g["form"] == expect_form, name
        r = ref[name]
        for procs in r.values():
            for m in procs.values():
                assert m["FirstEvent"] is None  # between events the processing chunk is empty
        if g["form"] == "chain":
            r, gs = merge_lists(r), merge_lists(g["states"])
        else:
            gs = g["states"]
        assert project(r, gs) == gs, name
        n += sum(len(m["PendingStateEventList"]) + len(m["NewAndEveryStateEventList"])
                 for procs in gs.values() for m in procs.values())
    return n
