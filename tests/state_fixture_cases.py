"""Seeded histories whose engine snapshots are committed under tests/golden/state_maps/ (made on the GPU by
scripts/make_state_fixtures.py) and decoded on the CPU by tests/test_state_maps.py."""
import synth

CASES = {  # name -> (app, trace, batches, force_generic)
    "absent_mid": (synth.ABSENT_APPS["absent_mid"], synth.trace(300, keys=3, seed=13), 2, True),
    "chain_gt": (synth.CHAIN_APPS["gt"][0], synth.descending_trace(400, keys=3, seed=14, run=30), 2, False),
}


def feed(adapter, tr, batches):
    synth.run(adapter, tr, batches)
