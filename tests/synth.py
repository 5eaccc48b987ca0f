"""Seeded synthetic traces for the pattern shapes of SURVEY.md 8 (C1-C3 and the generic-NFA constructs:
sequences, count quantifiers, logical and/or, non-every and >= 3-state chains, within), run through any adapter
with send/flush/outputs (oracle, host NFA build, GPU engine)."""
import numpy as np

DEFS = ("define stream S (id long, key string, price double, volume int); "
        "define stream T (id long, key string, price double, volume int); ")


DEFS_NUM = ("@app:playback define stream S (id long, k long, price double, volume int); "
            "define stream T (id long, k long, price double, volume int); ")


def part(q):
    return "@app:playback " + DEFS + "partition with (key of S, key of T) begin " + q + " end;"


def part_s(q):
    """a partition keyed on S only: T has no partition key, so each T event goes to every key (broadcast)"""
    return "@app:playback " + DEFS + "partition with (key of S) begin " + q + " end;"


def flat(q):
    return "@app:playback " + DEFS + q


APPS = {
    "c3_sequence": part("@info(name='q') from every e1=S[price>20], e2=S[price>e1.price]<2:5>, "
                        "e3=S[price<e2[last].price] select e1.id as a, e2[0].id as b, e2[last].id as c, e3.id as d "
                        "insert into O;"),
    "c3_sequence_min1": part("@info(name='q') from every e1=S[price>20], e2=S[price>e1.price]<1:5>, "
                             "e3=S[price<e2[last].price] select e1.id as a, e2[0].id as b, e2[last].id as c, "
                             "e3.id as d insert into O;"),
    "three_state_within": part("@info(name='q') from every e1=S[price>30] -> e2=S[price>e1.price] -> "
                               "e3=T[price<e2.price] within 40 milliseconds "
                               "select e1.id as a, e2.id as b, e3.id as c insert into O;"),
    "non_every": flat("@info(name='q') from e1=S[price>50] -> e2=T[price>e1.price] "
                      "select e1.id as a, e2.id as b insert into O;"),
    "every_group": part("@info(name='q') from every (e1=S[price>40] -> e2=T[price>e1.price]) -> e3=S[volume>50] "
                        "select e1.id as a, e2.id as b, e3.id as c insert into O;"),
    "count_pattern": part("@info(name='q') from every e1=S[price>20]<2:4> -> e2=T[price>e1[0].price] "
                          "select e1[0].id as a, e1[1].id as b, e1[last].id as c, e2.id as d insert into O;"),
    "count_zero_min": part("@info(name='q') from e1=S[price>60] -> e2=T[price>e1.price]<0:3> -> e3=S[volume<20] "
                           "select e1.id as a, e2[0].id as b, e3.id as c insert into O;"),
    "logical_and": part("@info(name='q') from every (e1=S[price>30] and e2=T[price>40]) -> e3=S[price>e1.price] "
                        "select e1.id as a, e2.id as b, e3.id as c insert into O;"),
    "logical_or": part("@info(name='q') from every e1=S[price>70] -> (e2=S[price>e1.price] or e3=T[volume>90]) "
                       "select e1.id as a, e2.id as b, e3.id as c insert into O;"),
    "sequence_plus": part("@info(name='q') from every e1=S[price>20], e2=T[price>e1.price]+, e3=S[price>e2[0].price] "
                          "select e1.id as a, e2[0].id as b, e3.id as c insert into O;"),
    "sequence_star_within": part("@info(name='q') from every e1=S[price>20], e2=S[volume>30]*, e3=T[price>e1.price] "
                                 "within 30 milliseconds select e1.id as a, e2[last].id as b, e3.id as c "
                                 "insert into O;"),
    "arith_nulls": part("@info(name='q') from every e1=S[price>20] -> e2=T[(price - e1.price) / volume > 0.5 "
                        "or e1.volume % volume == 0] select e1.id as a, e2.id as b, e1.price * e2.volume as c "
                        "insert into O;"),
}


def trace(n, keys=5, seed=0, two_streams=True, null_rate=0.0):
    """list of (stream, ts, [id, key, price, volume]) with non-decreasing ts (some equal)"""
    rng = np.random.default_rng(seed)
    ts = 1000 + np.cumsum(rng.integers(0, 4, size=n))
    out = []
    for i in range(n):
        s = "T" if two_streams and rng.random() < 0.4 else "S"
        price = float(np.round(rng.uniform(0, 100), 1))
        vol = int(rng.integers(0, 100))
        row = [i, "k%d" % rng.integers(0, keys), price, vol]
        if null_rate and rng.random() < null_rate:
            row[2 + int(rng.integers(0, 2))] = None
        out.append((s, int(ts[i]), row))
    return out


def run(adapter, tr, batches=1):
    bounds = np.linspace(0, len(tr), batches + 1).astype(int)
    for b in range(batches):
        for s, ts, row in tr[bounds[b]:bounds[b + 1]]:
            adapter.send(s, ts, row)
        if hasattr(adapter, "flush"):
            adapter.flush()
    return [(o["name"], o["ts"], tuple(o["values"])) for o in adapter.outputs()
            if o["kind"] == "query" and not o["expired"]]


# ---- chain-path shapes (every e1=S[c0] -> e2=S[c1], one stream): deque (stack / complete-all) and scan ----
def chain_app(c0, c1, within="within 30 milliseconds", sel="e1.id as a, e2.id as b"):
    return part("@info(name='q') from every e1=S[%s] -> e2=S%s %s select %s insert into O;"
                % (c0, "[%s]" % c1 if c1 else "", within, sel))


CHAIN_APPS = {  # name -> (app, expected sdg_stats.deque: 1 stack, 2 complete-all, 0 forward scan)
    "gt": (chain_app("price>20", "price>e1.price"), 1),
    "ge": (chain_app("price>20", "price>=e1.price"), 1),
    "lt": (chain_app("price<80", "price<e1.price"), 1),
    "le_flipped": (chain_app("price<80", "e1.price>=price"), 1),
    "int_gt_nowithin": (chain_app("volume>10", "volume>e1.volume", within=""), 1),
    "const": (chain_app("price>20", "price>90"), 2),
    "no_filter": (chain_app("volume<50", ""), 2),
    "ne_const": (chain_app("price>20", "price!=e1.price"), 0),
    "cross_col": (chain_app("price>20", "volume>e1.price"), 0),
    "e1_const_e2": (chain_app("price>20", "e1.volume>50"), 0),
    "arith_sel": (chain_app("price>20", "price>e1.price", sel="e1.id as a, e2.price - e1.price as d"), 0),
}


def descending_trace(n, keys=3, seed=0, run=200):
    """long descending price runs per key (deque overflow: every pending partial stays pending)"""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = int(rng.integers(0, keys))
        price = float(100.0 - (i % run) * 0.25) if rng.random() < 0.97 else float(np.round(rng.uniform(0, 100), 1))
        out.append(("S", 1000 + i // 4, [i, "k%d" % k, price, int(rng.integers(0, 100))]))
    return out


def nan_trace(n, keys=4, seed=0, nan_rate=0.05, null_rate=0.05):
    rng = np.random.default_rng(seed)
    out = []
    ts = 1000 + np.cumsum(rng.integers(0, 3, size=n))
    for i in range(n):
        price = float(np.round(rng.uniform(0, 100), 1))
        u = rng.random()
        if u < nan_rate:
            price = float("nan")
        elif u < nan_rate + null_rate:
            price = None
        out.append(("S", int(ts[i]), [i, "k%d" % rng.integers(0, keys), price, int(rng.integers(0, 100))]))
    return out


# ---- the selector: functions, attribute aggregators per partition key, having, select * ----
SELECT_APPS = {
    "agg_all": part("@info(name='q') from every e1=S[price>30] -> e2=T[price>e1.price] select e1.id as a, "
                    "count() as n, sum(e2.volume) as sv, sum(e2.price) as sp, avg(e1.price) as ap, "
                    "min(e2.price) as mn, max(e1.volume) as mx, minForever(e2.volume) as mf insert into O;"),
    "agg_expr": part("@info(name='q') from every e1=S[price>30] -> e2=T[price>e1.price] select e2.id as b, "
                     "sum(e2.price) / count() as mean, count() + 1 as n1, maxForever(e1.price) - min(e2.price) as r "
                     "insert into O;"),
    "agg_flat": flat("@info(name='q') from every e1=S[price>20] -> e2=T[price>e1.price] select count() as n, "
                     "avg(e2.price) as a, sum(e1.volume) as s insert into O;"),
    "having_count": part("@info(name='q') from every e1=S[price>20] -> e2=T[price>e1.price] "
                         "select e1.id as a, e2.id as b, count() as n having n % 3 == 0 insert into O;"),
    "having_inputs": part("@info(name='q') from every e1=S[price>20]<1:3> -> e2=T[price>e1[0].price] "
                          "select e1[0].id as a, e2.id as b having instanceOfDouble(e1[1].price) and "
                          "not (e1[2] is null) and e2.volume > 10 insert into O;"),
    "having_agg": part("@info(name='q') from every e1=S[price>40] -> e2=T[price>e1.price] "
                       "select e1.id as a, e2.price as p having avg(e2.price) > 70.0 or count() < 3 insert into O;"),
    "functions": part("@info(name='q') from every e1=S[price>20] -> e2=T[price>e1.price] "
                      "select ifThenElse(e2.volume > 50, e1.id, e2.id) as a, coalesce(e1.price, e2.price) as b, "
                      "maximum(e1.price, e2.price, 55.0) as c, minimum(e1.volume, e2.volume) as d, "
                      "instanceOfLong(e1.id) as e, default(e2.price, -1.0) as f, instanceOfString(e1.price) as g "
                      "insert into O;"),
    "select_star": part("@info(name='q') from every e1=S[price>90] select * insert into O;"),
    "agg_absent": part("@info(name='q') from every e1=S[price>60] -> not T[price>e1.price] for 20 milliseconds "
                       "select e1.id as a, count() as n, max(e1.price) as m insert into O;"),
}


# ---- absent states under heavy timer collisions (few keys, many equal due times): the scheduler's
# TreeMultimap collapse, multi-pop fires and destroyed-state re-arms (Scheduler.java:71-127,
# AbsentStreamPreStateProcessor.process :150-227) ----
ABSENT_APPS = {
    "absent_every_20": part("@info(name='q') from every e1=S[price>60] -> not T[price>e1.price] for 20 milliseconds "
                            "select e1.id as a, e1.key as k insert into O;"),
    "absent_every_7": part("@info(name='q') from every e1=S[price>60] -> not T[price>e1.price] for 7 milliseconds "
                           "select e1.id as a, e1.key as k insert into O;"),
    "absent_once": part("@info(name='q') from e1=S[price>30] -> not T[price>e1.price] for 15 milliseconds "
                        "select e1.id as a, e1.key as k insert into O;"),
    "absent_start": part("@info(name='q') from every not S[price>90] for 10 milliseconds -> e2=T[price>50] "
                         "select e2.id as a insert into O;"),
    "absent_and": part("@info(name='q') from every e1=S[price>50] -> (not T[price>e1.price] for 12 milliseconds "
                       "and e3=S[price>80]) select e1.id as a, e3.id as b insert into O;"),
    "absent_mid": part("@info(name='q') from every e1=S[price>50] -> not T[price>e1.price] for 9 milliseconds -> "
                       "e3=S[price>e1.price] select e1.id as a, e3.id as b insert into O;"),
}


def run_events(adapter, tr, chunk=7, batches=1):
    """the trace through InputHandler.send(Event[]): consecutive rows of one stream in arrays of <= chunk events
    (InputHandler.java:85-95 -- the playback clock moves to each array's last timestamp first)"""
    groups, cur = [], []
    for s, ts, row in tr:
        if cur and (cur[0][0] != s or len(cur) == chunk):
            groups.append(cur)
            cur = []
        cur.append((s, ts, row))
    if cur:
        groups.append(cur)
    bounds = np.linspace(0, len(groups), batches + 1).astype(int)
    for b in range(batches):
        for g in groups[bounds[b]:bounds[b + 1]]:
            adapter.send_events(g[0][0], [(ts, row) for _, ts, row in g])
        if hasattr(adapter, "flush"):
            adapter.flush()
    return [(o["name"], o["ts"], tuple(o["values"])) for o in adapter.outputs()
            if o["kind"] == "query" and not o["expired"]]


# ---- @purge: keys active in bursts, idle in between (PartitionRuntimeImpl.java:368-401) ----
def purge_part(q, idle="1 sec", interval="1 sec"):
    return ("@app:playback " + DEFS + "@purge(enable='true', interval='%s', idle.period='%s') "
            "partition with (key of S, key of T) begin %s end;" % (interval, idle, q))


PURGE_APPS = {
    "purge_pattern": purge_part("@info(name='q') from every e1=S[price>60] -> e2=T[price>e1.price] "
                                "select e1.id as a, e2.id as b insert into O;"),
    "purge_count": purge_part("@info(name='q') from every e1=S[price>40]<2:4> -> e2=T[price>e1[0].price] "
                              "select e1[0].id as a, e1[last].id as b, e2.id as c insert into O;"),
    "purge_non_every": purge_part("@info(name='q') from e1=S[price>80] -> e2=T[price>e1.price] "
                                  "select e1.id as a, e2.id as b insert into O;", idle="2 sec"),
    "purge_sequence": purge_part("@info(name='q') from every e1=S[price>30], e2=T[price>e1.price]+, "
                                 "e3=S[price>e2[0].price] select e1.id as a, e2[0].id as b, e3.id as c insert into O;"),
    # absent states: the purge destroys the key's pending absence candidates and its SchedulerState (timer queue)
    "purge_absent": purge_part("@info(name='q') from every e1=S[price>70] -> not T[price>e1.price] for 3 sec "
                               "select e1.id as a insert into O;"),
    "purge_absent_logical": purge_part("@info(name='q') from every e1=S[price>60] -> "
                                       "(not T[price>e1.price] for 2 sec and e3=S[price<20]) "
                                       "select e1.id as a, e3.id as c insert into O;"),
    # aggregators: the purge restarts the key's aggregator states (cleanGroupByStates of the selector's holders)
    "purge_agg": purge_part("@info(name='q') from every e1=S[price>60] -> e2=T[price>e1.price] "
                            "select e1.id as a, count() as n, sum(e2.price) as s, max(e1.volume) as m insert into O;"),
}


def purge_trace(n, keys=8, burst=120, seed=0):
    """every key is active for `burst` consecutive events, then idle while the other keys take their turns;
    ts steps of 0-24 ms, so a key's idle gaps span seconds"""
    rng = np.random.default_rng(seed)
    ts = 1000 + np.cumsum(rng.integers(0, 25, size=n))
    out = []
    for i in range(n):
        s = "T" if rng.random() < 0.4 else "S"
        k = (i // burst) % keys if rng.random() < 0.9 else int(rng.integers(0, keys))
        out.append((s, int(ts[i]), [i, "k%d" % k, float(np.round(rng.uniform(0, 100), 1)), int(rng.integers(0, 100))]))
    return out


# ---- range partitions (RangePartitionExecutor): overlapping ranges send one event to several keys ----
RANGE_APPS = {
    "range_disjoint": flat("partition with (price < 30 as 'low' or price >= 30 and price < 70 as 'mid' or "
                           "price >= 70 as 'high' of S, volume < 50 as 'low' or volume >= 50 as 'high' of T) begin "
                           "@info(name='q') from every e1=S[volume>40] -> e2=T[price>e1.price] "
                           "select e1.id as a, e2.id as b insert into O; end;"),
    "range_overlap": flat("partition with (price < 60 as 'a' or price > 40 as 'b' or volume > 80 as 'c' of S, "
                          "price < 60 as 'a' or price > 40 as 'b' of T) begin "
                          "@info(name='q') from every e1=S[volume>30] -> e2=T[volume>e1.volume] "
                          "select e1.id as a, e2.id as b insert into O; end;"),
    "range_sequence": flat("partition with (price < 50 as 'lo' or price >= 50 as 'hi' of S, "
                           "price < 50 as 'lo' or price >= 50 as 'hi' of T) begin "
                           "@info(name='q') from every e1=S[volume>20], e2=T[volume>e1.volume]+, e3=S[volume<e2[0].volume] "
                           "select e1.id as a, e2[0].id as b, e3.id as c insert into O; end;"),
}

SELECT_APPS["multi_value"] = part(
    "@info(name='q') from every e1=S[price>40]<1:4> -> e2=T[price>e1[0].price] "
    "select e1.id as ids, e1.price as prices, e2.id as b, e1[0].volume as v0 insert into O;")
SELECT_APPS["multi_value_seq"] = part(
    "@info(name='q') from every e1=S[price>20], e2=T[price>e1.price]+, e3=S[price<e2[last].price] "
    "select e1.id as a, e2.volume as vols, e3.id as c insert into O;")


# ---- a stream without a partition key inside a partition (PartitionStreamReceiver.send(ComplexEvent) :274-283):
# T events reach every key S initialised, in getPartitionKeys() order ----
BCAST_APPS = {
    "bc_pattern": part_s("@info(name='q') from every e1=S[price>20] -> e2=T[price>e1.price] within 50 milliseconds "
                         "select e1.id as a, e2.id as b insert into O;"),
    "bc_count": part_s("@info(name='q') from every e1=S[price>50 and volume>10] -> e2=T[price<40]<1:> -> "
                       "e3=T[volume<=70] select e3.id as a, e2[0].id as b, e1.id as c insert into O;"),
    "bc_sequence": part_s("@info(name='q') from every e1=S[price>20], e2=T[price>e1.price] "
                          "select e1.id as a, e2.id as b insert into O;"),
    "bc_absent": part_s("@info(name='q') from every e1=S[price>60] -> not T[price>e1.price] for 20 milliseconds "
                        "select e1.id as a insert into O;"),
    "bc_logical": part_s("@info(name='q') from every (e1=S[price>30] and e2=T[price>40]) -> e3=S[price>e1.price] "
                         "select e1.id as a, e2.id as b, e3.id as c insert into O;"),
    "bc_only_t": part_s("@info(name='q') from every e1=T[price>90] -> e2=S[price>e1.price] "
                        "select e1.id as a, e2.id as b insert into O;"),
}
