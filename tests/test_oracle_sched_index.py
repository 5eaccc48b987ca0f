"""The oracle's scheduler due index (oracle.cpp Scheduler::heads) against the oracle's own literal walk of every
state per clock advance (Scheduler.java:71-103, ORACLE_SCHED_WALK=1): identical outputs on C4 (10^4 keys, the
TreeMultimap collapse delaying most fires) and on every timer-collision app of tests/synth.py. The index is what lets
the oracle run C4 at 10^6 keys (tests/golden/make_config_fixtures.py); the walk is the restatement it must equal."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

SCRIPT = r"""
import hashlib, json, sys
sys.path.insert(0, %(repo)r); sys.path.insert(0, %(tests)r)
import synth
from siddhi_amd import workloads as w
from test_c4_host import oracle_c4
from oracle_rt import Oracle
out = {}
c = w.c4_columns(10_000, per_tick=100)
ts, vals, nulls = oracle_c4(c, int(c["ts"][-1]) + 5000)
out["c4"] = [len(ts), hashlib.sha256(ts.tobytes() + vals.tobytes() + nulls.tobytes()).hexdigest()]
for name in sorted(synth.ABSENT_APPS):
    for seed in (100, 102, 104):
        o = Oracle(synth.ABSENT_APPS[name])
        try:
            rows = synth.run(o, synth.trace(3000, keys=6, seed=seed, null_rate=0.05), 1)
        finally:
            o.close()
        out["%%s/%%d" %% (name, seed)] = hashlib.sha256(repr(rows).encode()).hexdigest()
print(json.dumps(out))
"""


def run(walk):
    env = dict(os.environ)
    env.pop("ORACLE_SCHED_WALK", None)
    if walk:
        env["ORACLE_SCHED_WALK"] = "1"
    src = SCRIPT % {"repo": os.path.dirname(HERE), "tests": HERE}
    res = subprocess.run([sys.executable, "-c", src], env=env, capture_output=True, text=True, timeout=900)
    assert res.returncode == 0, res.stderr[-2000:]
    return json.loads(res.stdout.strip().splitlines()[-1])


def test_due_index_equals_the_walk(oracle_built):
    fast, walk = run(False), run(True)
    assert fast["c4"][0] > 1000
    assert fast == walk
