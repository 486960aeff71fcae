"""Pins the CPU oracle against the reference's own golden event scripts (tests/golden)."""
import pytest

from fixture_runner import OracleAdapter, load_fixtures, replay

FIXTURES = load_fixtures()


def test_fixture_count():
    assert len(FIXTURES) >= 10


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_oracle_reproduces_reference_golden(fx):
    replay(fx, OracleAdapter(fx))
