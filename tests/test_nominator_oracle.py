"""The nominator boundary on the oracle (tests/nominator_scenario.py; the device side: test_gpu_nominated.py)."""
from nominator_scenario import run
from oracle_binding import oracle


def test_nominator_refusals_on_the_oracle():
    log = run(oracle({}))
    got = {tag: out for tag, out, _ in log}
    assert got == {
        "no nominations": "ok",
        "lower priority pod, a priority-100 nomination on n1: refused": "refused",
        "equal priority: refused": "refused",
        "higher priority pod: the nomination is not added": "ok",
        "the nominated pod itself (own uid)": "ok",
        "after the nominated pod was assumed": "ok",
        "nominated to a node outside the snapshot": "ok",
        "priority-50 nomination on n2: refused": "refused",
        "re-added without a node": "ok",
        "batch with one pod under a nomination: refused whole": "refused",
        "batch after the nomination was deleted": "ok",
        "preemption under a nomination: refused": "refused",
    }
    # every accepted single pod was placed (four empty 4-CPU nodes)
    assert all(v[0] == 0 for tag, out, v in log if out == "ok" and isinstance(v, tuple))
