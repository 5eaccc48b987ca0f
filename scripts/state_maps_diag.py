"""Writes the oracle's and the engine's state maps for a few histories under gpurun_out/maps/ (debug aid for
tests/test_gpu_state_maps.py)."""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402
from oracle_rt import Oracle  # noqa: E402
from product_rt import ProductAdapter  # noqa: E402

out = os.path.join("gpurun_out", "maps")
os.makedirs(out, exist_ok=True)
cases = {
    "count_pattern": (synth.APPS["count_pattern"], synth.trace(900, keys=5, seed=3), True),
    "sequence_star_within": (synth.APPS["sequence_star_within"], synth.trace(900, keys=5, seed=3), True),
    "absent_and": (synth.ABSENT_APPS["absent_and"], synth.trace(700, keys=3, seed=4), True),
    "absent_mid": (synth.ABSENT_APPS["absent_mid"], synth.trace(700, keys=3, seed=4), True),
    "absent_every_20": (synth.ABSENT_APPS["absent_every_20"], synth.trace(700, keys=3, seed=4), True),
}
for name, (app, tr, gen) in cases.items():
    o = Oracle(app)
    p = ProductAdapter(app, force_generic=gen)
    nb = 3 if name == "sequence_star_within" else 2
    synth.run(o, tr, nb)
    synth.run(p, tr, nb)
    with open(os.path.join(out, name + "_oracle.json"), "w") as f:
        json.dump(o.state_dump(), f, indent=1, sort_keys=True)
    with open(os.path.join(out, name + "_engine.json"), "w") as f:
        json.dump(p.rt.snapshot_states(), f, indent=1, sort_keys=True)
    p.close()
    o.close()
    print("wrote", name, flush=True)
