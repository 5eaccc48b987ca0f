"""Writes engine snapshots of a few seeded histories to gpurun_out/state_fixtures/ (run on the GPU box; the blobs
are committed under tests/golden/state_maps/ and decoded on the CPU by tests/test_state_maps.py)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import state_fixture_cases as cases  # noqa: E402
from product_rt import ProductAdapter  # noqa: E402

out = os.path.join("gpurun_out", "state_fixtures")
os.makedirs(out, exist_ok=True)
for name, (app, tr, batches, generic) in cases.CASES.items():
    p = ProductAdapter(app, force_generic=generic)
    try:
        cases.feed(p, tr, batches)
        blob = p.rt.snapshot()
    finally:
        p.close()
    with open(os.path.join(out, name + ".snap"), "wb") as f:
        f.write(blob)
    print("wrote", name, len(blob), flush=True)
