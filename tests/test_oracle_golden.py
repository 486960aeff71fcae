"""Pins the CPU oracle against the reference's own golden event scripts (tests/golden): the
one-phase operator on every fixture, the two-phase plan (LOCAL + GLOBAL restatement) on the
WindowAggregateTestPrograms / WindowAggregateITCase fixtures that the reference runs with both
agg-phase strategies, and the slice assigners' known-answer tests."""
import pytest

from fixture_runner import OracleAdapter, TwoPhaseOracleAdapter, load_fixtures, load_kats, replay

FIXTURES = load_fixtures()
TWO_PHASE = [f for f in FIXTURES if f.get("two_phase")]


def test_fixture_count():
    assert len(FIXTURES) >= 19 and len(TWO_PHASE) >= 9


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_oracle_reproduces_reference_golden(fx):
    replay(fx, OracleAdapter(fx))


@pytest.mark.parametrize("fx", TWO_PHASE, ids=[f["name"] for f in TWO_PHASE])
def test_oracle_two_phase_reproduces_reference_golden(fx):
    replay(fx, TwoPhaseOracleAdapter(fx), check_late=False)
