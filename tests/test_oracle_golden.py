"""Pin the oracle: every golden fixture (the reference's own known-answer tests, converted to traces) must
reproduce the asserted rows and counts. Fixtures needing a feature the oracle does not restate yet are
reported as xfail with the missing feature."""
import pytest

import golden_util
from oracle_rt import OracleError, check_fixture, run_oracle_fixture

PATHS = golden_util.fixture_paths()


@pytest.mark.parametrize("path", PATHS, ids=golden_util.fixture_ids())
def test_oracle_matches_reference_test(path, oracle_built):
    fx = golden_util.load(path)
    try:
        outs = run_oracle_fixture(fx)
    except OracleError as e:
        msg = str(e)
        if "unsupported" in msg.lower() or "OperationNotSupported" in msg or "out of scope" in msg \
                or "not supported" in msg or "not on the accelerated path" in msg:
            pytest.xfail("oracle does not restate: " + msg[:120])
        raise
    problems = check_fixture(fx, outs)
    assert not problems, "%s (%s): %s" % (fx["test"], fx["source"], problems)


def test_fixture_inventory():
    # the generator must keep producing the full set (458 @Test methods in the 16 files, 2 skipped: loops)
    assert len(PATHS) >= 450
