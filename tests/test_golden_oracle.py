"""The parity oracle against the reference's own unit-test vectors (CPU)."""
import pytest

from golden_runner import load_cases, run_case
from oracle_binding import oracle

CASES = load_cases()


@pytest.mark.parametrize("name,case", CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_reference_vectors(name, case):
    errs = run_case(oracle, case)
    assert not errs, f"{case['src']}: {errs}"
